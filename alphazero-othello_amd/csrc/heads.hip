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
