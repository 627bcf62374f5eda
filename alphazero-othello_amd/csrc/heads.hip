// heads.hip — AlphaZeroNet's policy and value heads in one kernel, writing the engine's
// prior and value buffers directly.
//
// Reference Models.py:164-221 (inference copy, BatchNorm folded into the 1x1 convs):
//   p = relu(conv1x1_{C->2}(h) + b)            flattened NCHW: p[c*64 + pos]
//   logits = pol_fc(p)  (128 -> 65)            priors = softmax(logits)  (MCTS_model.py:319)
//   v = relu(conv1x1_{C->1}(h) + b)            v[pos]
//   value = tanh(val_fc2(relu(val_fc1(v))))   (64 -> 256 -> 1)
// One wavefront per board, four boards per workgroup: lane = board square for the 1x1
// convs, lane = output for the FCs, whose weights are pre-transposed (pol_fc as [128][65],
// val_fc1 as [64][256]) and read from L2, where every workgroup finds them (STAGE = true
// stages them in LDS per workgroup instead: measured slower); the per-board vectors pass
// through LDS.  Replaces a MIOpen 1x1 conv, its epilogue, two hipBLASLt GEMMs, softmax,
// ReLU/tanh kernels and two device copies per step.
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

template <int C, bool STAGE = true>
__global__ __launch_bounds__(64 * kWaves) void k_heads_az(
    const float* __restrict__ h, const float* __restrict__ wpv, const float* __restrict__ bpv,
    const float* __restrict__ wpolT, const float* __restrict__ bpol,
    const float* __restrict__ w1T, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, float* __restrict__ priors, float* __restrict__ values,
    int n_boards) {
  constexpr int kThreads = 64 * kWaves;
  constexpr int kPol = 128 * 65, kVal = 64 * 256;   // FC weight floats
  __shared__ __align__(16) float s_wpol[STAGE ? kPol : 4];  // pol_fc^T  [128][65]
  __shared__ __align__(16) float s_w1[STAGE ? kVal : 4];    // val_fc1^T [64][256]
  const float* wpol = STAGE ? s_wpol : wpolT;  // !STAGE: straight from L2 (shared by all)
  const float* w1s = STAGE ? s_w1 : w1T;
  __shared__ float s_p[kWaves][128];
  __shared__ float s_v[kWaves][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x * kWaves + w;
  const bool live = b < n_boards;

  // Every global load of the kernel is issued up front (one round trip, not one per loop
  // batch): the workgroup's FC weights (shared by its boards, staged to LDS) and this
  // lane's activation row (square `lane`: C floats).
  constexpr int NP = STAGE ? (kPol / 4 + kThreads - 1) / kThreads : 1;
  constexpr int NV = STAGE ? kVal / 4 / kThreads : 1;
  float4 wp[NP], wv[NV];
  if (STAGE) {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int q = i * kThreads + tid;
      wp[i] = q < kPol / 4 ? reinterpret_cast<const float4*>(wpolT)[q] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) wv[i] = reinterpret_cast<const float4*>(w1T)[i * kThreads + tid];
  }
  float4 x[C / 4];
  const float4* hp = reinterpret_cast<const float4*>(h + ((size_t)(live ? b : 0) * 64 + lane) * C);
#pragma unroll
  for (int c = 0; c < C / 4; ++c) x[c] = hp[c];
  // the lane's policy-FC weights (L2) in the same round trip as its activation row
  float wpl[128];
  float wl0 = 0.f, wl1 = 0.f;
  if (!STAGE) {
#pragma unroll
    for (int k = 0; k < 128; ++k) wpl[k] = wpolT[k * 65 + lane];
    wl0 = wpolT[lane * 65 + 64];
    wl1 = wpolT[(lane + 64) * 65 + 64];
  }
  if (STAGE) {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int q = i * kThreads + tid;
      if (q < kPol / 4) reinterpret_cast<float4*>(s_wpol)[q] = wp[i];
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) reinterpret_cast<float4*>(s_w1)[i * kThreads + tid] = wv[i];
  }

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
  if (!live) return;  // whole wave (b is uniform per wave); no barrier follows

  // policy FC: lane a -> logit a; logit 64 split over the lanes and reduced.  The FC weights
  // come from L2 (shared by every workgroup): a lane's 128 policy weights were requested with
  // its activation row, its 64 value-weight quads are requested here before any FMA (one round
  // trip each instead of one per 16-iteration batch; one wave per SIMD, so the registers are
  // there)
  float4 wq[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) wq[i] = reinterpret_cast<const float4*>(w1s + i * 256)[lane];
  if (STAGE) {
#pragma unroll
    for (int k = 0; k < 128; ++k) wpl[k] = wpol[k * 65 + lane];
    wl0 = wpol[lane * 65 + 64];
    wl1 = wpol[(lane + 64) * 65 + 64];
  }
  float la = bpol[lane];
#pragma unroll
  for (int k = 0; k < 128; ++k) la += wpl[k] * s_p[w][k];
  float l64 = wl0 * s_p[w][lane] + wl1 * s_p[w][lane + 64];
  l64 = wave_sum(l64) + bpol[64];
  const float m = fmaxf(wave_max(la), l64);
  const float e = __expf(la - m), e64 = __expf(l64 - m);
  const float inv = 1.f / (wave_sum(e) + e64);
  priors[(size_t)b * 65 + lane] = e * inv;
  if (lane == 0) priors[(size_t)b * 65 + 64] = e64 * inv;

  // value: lane j -> hidden units 4j..4j+3 of val_fc1, then val_fc2 reduced over the wave
  float4 acc = reinterpret_cast<const float4*>(b1)[lane];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const float vi = s_v[w][i];
    acc.x += wq[i].x * vi;
    acc.y += wq[i].y * vi;
    acc.z += wq[i].z * vi;
    acc.w += wq[i].w * vi;
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
  // FC weights read straight from L2 (shared by every workgroup): measured 15.3-15.6 us
  // against 16.8-17.8 us staging them in LDS per workgroup (scripts/exp/heads_ab.py)
  if (channels == 128)
    hipLaunchKernelGGL((k_heads_az<128, false>), dim3(grid), dim3(64 * kWaves), 0, s, h, wpv,
                       bpv, wpolT, bpol, w1T, b1, w2, b2, priors, values, n_boards);
  else if (channels == 64)
    hipLaunchKernelGGL((k_heads_az<64, false>), dim3(grid), dim3(64 * kWaves), 0, s, h, wpv,
                       bpv, wpolT, bpol, w1T, b1, w2, b2, priors, values, n_boards);
  else
    return azc::set_error(AZ_ERR_ARG, "az_heads_az_gpu: channels must be 64 or 128, got %d",
                          channels);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
