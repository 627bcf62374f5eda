// heads.hip — AlphaZeroNet's policy and value heads in one kernel, writing the engine's
// prior and value buffers directly.
//
// Reference Models.py:164-221 (inference copy, BatchNorm folded into the 1x1 convs):
//   p = relu(conv1x1_{C->2}(h) + b)            flattened NCHW: p[c*64 + pos]
//   logits = pol_fc(p)  (128 -> 65)            priors = softmax(logits)  (MCTS_model.py:319)
//   v = relu(conv1x1_{C->1}(h) + b)            v[pos]
//   value = tanh(val_fc2(relu(val_fc1(v))))   (64 -> 256 -> 1)
// One wavefront per board, four boards per workgroup: lane = board square for the 1x1
// convs.  The FCs are split by INPUT range over the workgroup's waves, each wave computing
// its quarter for all four boards (pol_fc^T [128][65]: inputs 32w..32w+31; val_fc1^T
// [64][256]: inputs 16w..16w+15), so every FC weight is read from L2 once per workgroup
// instead of once per board; the partial sums meet in LDS and wave b adds them in order for
// board b.  (Round 2: each wave read the full FC weights for its own board -- 97 KB of L2
// reads per board; staging the weights in LDS per workgroup measured slower still.)
// Replaces a MIOpen 1x1 conv, its epilogue, two hipBLASLt GEMMs, softmax, ReLU/tanh kernels
// and two device copies per step.
#include "common.h"

namespace {

constexpr int kWaves = 4;  // boards per workgroup

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
  return x;
}

template <int C>
__global__ __launch_bounds__(64 * kWaves) void k_heads_az(
    const float* __restrict__ h, const float* __restrict__ wpv, const float* __restrict__ bpv,
    const float* __restrict__ wpolT, const float* __restrict__ bpol,
    const float* __restrict__ w1T, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, float* __restrict__ priors, float* __restrict__ values,
    int n_boards) {
  static_assert(kWaves == 4, "input quarters");
  constexpr int KP = 128 / kWaves, KV = 64 / kWaves;  // FC inputs per wave
  __shared__ float s_p[kWaves][128];
  __shared__ float s_v[kWaves][64];
  __shared__ float s_lp[kWaves][kWaves][65];               // [wave][board][logit] partials
  __shared__ __align__(16) float4 s_hv[kWaves][kWaves][64];  // [wave][board][lane] hidden
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x * kWaves + w;
  const bool live = b < n_boards;

  // every global load up front (one round trip): this lane's activation row (square `lane`)
  // and its share of the FC weights for the wave's input quarter
  float4 x[C / 4];
  const float4* hp = reinterpret_cast<const float4*>(h + ((size_t)(live ? b : 0) * 64 + lane) * C);
#pragma unroll
  for (int c = 0; c < C / 4; ++c) x[c] = hp[c];
  float wpl[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) wpl[k] = wpolT[(KP * w + k) * 65 + lane];
  const float w64 = lane < KP ? wpolT[(KP * w + lane) * 65 + 64] : 0.f;
  float4 wq[KV];
#pragma unroll
  for (int i = 0; i < KV; ++i) wq[i] = reinterpret_cast<const float4*>(w1T + (KV * w + i) * 256)[lane];

  // 1x1 convs (policy 2 channels, value 1 channel) at square `lane`
  float d0 = 0.f, d1 = 0.f, d2 = 0.f;
  const float4* w0 = reinterpret_cast<const float4*>(wpv);
  const float4* w1 = reinterpret_cast<const float4*>(wpv + C);
  const float4* w2v = reinterpret_cast<const float4*>(wpv + 2 * C);
#pragma unroll
  for (int c = 0; c < C / 4; ++c) {
    const float4 a = w0[c], q = w1[c], r = w2v[c];
    d0 += x[c].x * a.x + x[c].y * a.y + x[c].z * a.z + x[c].w * a.w;
    d1 += x[c].x * q.x + x[c].y * q.y + x[c].z * q.z + x[c].w * q.w;
    d2 += x[c].x * r.x + x[c].y * r.y + x[c].z * r.z + x[c].w * r.w;
  }
  s_p[w][lane] = fmaxf(d0 + bpv[0], 0.f);
  s_p[w][64 + lane] = fmaxf(d1 + bpv[1], 0.f);
  s_v[w][lane] = fmaxf(d2 + bpv[2], 0.f);
  __syncthreads();

  // this wave's input quarter of both FCs, for every board of the workgroup
#pragma unroll
  for (int bd = 0; bd < kWaves; ++bd) {
    float la = 0.f;
#pragma unroll
    for (int k = 0; k < KP; ++k) la += wpl[k] * s_p[bd][KP * w + k];
    s_lp[w][bd][lane] = la;
    const float l64 = wave_sum(lane < KP ? w64 * s_p[bd][KP * w + lane] : 0.f);
    if (lane == 0) s_lp[w][bd][64] = l64;
    float4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < KV; ++i) {
      const float vi = s_v[bd][KV * w + i];
      acc.x += wq[i].x * vi;
      acc.y += wq[i].y * vi;
      acc.z += wq[i].z * vi;
      acc.w += wq[i].w * vi;
    }
    s_hv[w][bd][lane] = acc;
  }
  __syncthreads();
  if (!live) return;  // whole wave (b is uniform per wave); no barrier follows

  // board w: the quarters added in order, softmax over the 65 logits
  float la = bpol[lane], l64 = bpol[64];
#pragma unroll
  for (int q = 0; q < kWaves; ++q) {
    la += s_lp[q][w][lane];
    l64 += s_lp[q][w][64];
  }
  const float m = fmaxf(wave_max(la), l64);
  const float e = __expf(la - m), e64 = __expf(l64 - m);
  const float inv = 1.f / (wave_sum(e) + e64);
  priors[(size_t)b * 65 + lane] = e * inv;
  if (lane == 0) priors[(size_t)b * 65 + 64] = e64 * inv;

  // value: lane j -> hidden units 4j..4j+3 of val_fc1, then val_fc2 reduced over the wave
  float4 acc = reinterpret_cast<const float4*>(b1)[lane];
#pragma unroll
  for (int q = 0; q < kWaves; ++q) {
    const float4 a = s_hv[q][w][lane];
    acc.x += a.x;
    acc.y += a.y;
    acc.z += a.z;
    acc.w += a.w;
  }
  const float4 o = reinterpret_cast<const float4*>(w2)[lane];
  const float part = fmaxf(acc.x, 0.f) * o.x + fmaxf(acc.y, 0.f) * o.y +
                     fmaxf(acc.z, 0.f) * o.z + fmaxf(acc.w, 0.f) * o.w;
  const float val = wave_sum(part) + b2[0];
  if (lane == 0) values[b] = tanhf(val);
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
  if (channels == 128)
    hipLaunchKernelGGL((k_heads_az<128>), dim3(grid), dim3(64 * kWaves), 0, s, h, wpv,
                       bpv, wpolT, bpol, w1T, b1, w2, b2, priors, values, n_boards);
  else if (channels == 64)
    hipLaunchKernelGGL((k_heads_az<64>), dim3(grid), dim3(64 * kWaves), 0, s, h, wpv,
                       bpv, wpolT, bpol, w1T, b1, w2, b2, priors, values, n_boards);
  else
    return azc::set_error(AZ_ERR_ARG, "az_heads_az_gpu: channels must be 64 or 128, got %d",
                          channels);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
