// heads.hip — AlphaZeroNet's policy and value heads in one kernel, writing the engine's
// prior and value buffers directly (the computation: heads_az.h).
//
// One wavefront per board, four boards per workgroup; every global load up front (one
// round trip): the lane's activation row, then the wave's share of the FC weights.
// (Round 2: each wave read the full FC weights for its own board -- 97 KB of L2 reads per
// board; staging the weights in LDS per workgroup measured slower still.)  Replaces a MIOpen
// 1x1 conv, its epilogue, two hipBLASLt GEMMs, softmax, ReLU/tanh kernels and two device
// copies per step.  The last trunk conv can run the same heads in its epilogue instead
// (az_conv3x3_wino4_heads_gpu, conv_wino4.hip).
#include "common.h"
#include "heads_az.h"

namespace {

constexpr int kWaves = azh::kBoards;

template <int C>
__global__ __launch_bounds__(64 * kWaves) void k_heads_az(const float* __restrict__ h,
                                                          azh::Weights W,
                                                          float* __restrict__ priors,
                                                          float* __restrict__ values,
                                                          int n_boards) {
  __shared__ float s_p[kWaves][128];
  __shared__ float s_v[kWaves][64];
  __shared__ float s_lp[kWaves][kWaves][65];
  __shared__ __align__(16) float4 s_hv[kWaves][kWaves][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x * kWaves + w;
  const bool live = b < n_boards;
  float4 x[C / 4];
  const float4* hp = reinterpret_cast<const float4*>(h + ((size_t)(live ? b : 0) * 64 + lane) * C);
#pragma unroll
  for (int c = 0; c < C / 4; ++c) x[c] = hp[c];
  const azh::Scratch L{s_p, s_v, s_lp, s_hv};
  azh::heads_four<C>([&](int c) { return x[c]; }, lane, w, b, live, true, W, L, priors, values);
}

}  // namespace

extern "C" int az_heads_az_gpu(const float* h, const float* wpv, const float* bpv,
                               const float* wpolT, const float* bpol, const float* w1T,
                               const float* b1, const float* w2, const float* b2,
                               float* priors, float* values, int32_t n_boards,
                               int32_t channels, void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_heads_az_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(h && wpv && bpv && wpolT && bpol && w1T && b1 && w2 && b2 && priors && values,
             AZ_ERR_ARG, "az_heads_az_gpu: null buffer");
  AZ_REQUIRE(((uintptr_t)h | (uintptr_t)wpv | (uintptr_t)w1T | (uintptr_t)b1 | (uintptr_t)w2) %
                     16 == 0,
             AZ_ERR_ARG, "az_heads_az_gpu: buffers must be 16-byte aligned");
  hipStream_t s = azc::as_stream(stream);
  const unsigned grid = (unsigned)((n_boards + kWaves - 1) / kWaves);
  const azh::Weights W{wpv, bpv, wpolT, bpol, w1T, b1, w2, b2};
  if (channels == 128)
    hipLaunchKernelGGL((k_heads_az<128>), dim3(grid), dim3(64 * kWaves), 0, s, h, W, priors,
                       values, n_boards);
  else if (channels == 64)
    hipLaunchKernelGGL((k_heads_az<64>), dim3(grid), dim3(64 * kWaves), 0, s, h, W, priors,
                       values, n_boards);
  else
    return azc::set_error(AZ_ERR_ARG, "az_heads_az_gpu: channels must be 64 or 128, got %d",
                          channels);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

// FastOthelloNet's heads after their two input GEMMs (reference Models.py:106-112 + the
// softmax of MCTS_model.py:319): the host runs ONE GEMM of the flattened tail output against
// [fc_policy; fc_value1], split over `parts` slices of the reduction (part p: logits partial
// sums [n][ld] at p * part_stride; columns 0..64 the policy logits, 65..128 the value hidden
// layer before its ReLU); this kernel adds the parts in order and the bias, then finishes both
// heads per board -- softmax over the 65 logits into priors, tanh(b2 + sum_j w2[j]
// relu(hidden_j)) into values.  One wavefront per board, lane j holds logit j (lane 0 also
// logit 64) and hidden unit j.
namespace {
__global__ __launch_bounds__(256) void k_heads_fast_finish(const float* __restrict__ logits,
                                                           int ld, int parts,
                                                           long long part_stride,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ w2,
                                                           const float* __restrict__ b2,
                                                           float* __restrict__ priors,
                                                           float* __restrict__ values,
                                                           int n_boards) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= n_boards) return;  // wave-uniform
  const float* row = logits + (size_t)b * ld;
  float l0 = row[lane], l64 = row[64], hid = row[65 + lane];
  for (int p = 1; p < parts; ++p) {
    const float* r = row + p * part_stride;
    l0 += r[lane];
    l64 += r[64];
    hid += r[65 + lane];
  }
  l0 += bias[lane];
  l64 += bias[64];
  hid += bias[65 + lane];
  float m = fmaxf(l0, l64);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  const float e0 = expf(l0 - m), e64 = expf(l64 - m);
  float s = e0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  s += e64;
  float* pr = priors + (size_t)b * 65;
  pr[lane] = e0 / s;
  if (lane == 0) pr[64] = e64 / s;
  float v = fmaxf(hid, 0.0f) * w2[lane];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane == 0) values[b] = tanhf(v + b2[0]);
}
}  // namespace

extern "C" int az_heads_fast_finish_gpu(const float* logits, int32_t ld, int32_t parts,
                                        const float* bias, const float* w2, const float* b2,
                                        float* priors, float* values, int32_t n_boards,
                                        void* stream) {
  AZ_REQUIRE(n_boards >= 0 && ld >= 129 && parts >= 1, AZ_ERR_ARG,
             "az_heads_fast_finish_gpu: n_boards %d < 0, ld %d < 129 or parts %d < 1", n_boards,
             ld, parts);
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(logits && bias && w2 && b2 && priors && values, AZ_ERR_ARG,
             "az_heads_fast_finish_gpu: null buffer");
  const unsigned grid = (unsigned)((n_boards + 3) / 4);
  hipLaunchKernelGGL(k_heads_fast_finish, dim3(grid), dim3(256), 0, azc::as_stream(stream),
                     logits, (int)ld, (int)parts, (long long)n_boards * ld, bias, w2, b2, priors,
                     values, (int)n_boards);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
