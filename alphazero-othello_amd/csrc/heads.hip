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

#ifndef AZ_HG_PD
#define AZ_HG_PD 3
#endif
#ifndef AZ_FINISH_UNROLLED
#define AZ_FINISH_UNROLLED 1
#endif

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
// logit 64) and hidden unit j.  P > 0: the part count at compile time, every part's three words
// requested before the first add (one memory round trip instead of P dependent ones; the adds
// keep the part order, so the sums are the same bits); P = 0: any count, one part at a time.
namespace {
template <int P>
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
  float l0, l64, hid;
  if constexpr (P > 0) {
    float a[P], c[P], d[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const float* r = row + p * part_stride;
      a[p] = r[lane];
      c[p] = r[64];
      d[p] = r[65 + lane];
    }
    l0 = a[0], l64 = c[0], hid = d[0];
#pragma unroll
    for (int p = 1; p < P; ++p) {
      l0 += a[p];
      l64 += c[p];
      hid += d[p];
    }
  } else {
    l0 = row[lane], l64 = row[64], hid = row[65 + lane];
    for (int p = 1; p < parts; ++p) {
      const float* r = row + p * part_stride;
      l0 += r[lane];
      l64 += r[64];
      hid += r[65 + lane];
    }
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
  // AZ_FINISH_UNROLLED=0 (A/B builds): every part count on the one-part-at-a-time loop
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, azc::as_stream(stream), logits, (int)ld,
                       (int)parts, (long long)n_boards * ld, bias, w2, b2, priors, values,
                       (int)n_boards);
  };
  if (AZ_FINISH_UNROLLED && parts == 1) go(k_heads_fast_finish<1>);
  else if (AZ_FINISH_UNROLLED && parts == 4) go(k_heads_fast_finish<4>);
  else if (AZ_FINISH_UNROLLED && parts == 8) go(k_heads_fast_finish<8>);
  else if (AZ_FINISH_UNROLLED && parts == 16) go(k_heads_fast_finish<16>);
  else go(k_heads_fast_finish<0>);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

// FastOthelloNet's heads GEMM (the host's torch.bmm before az_heads_fast_finish_gpu) on the
// 16-bit MFMA pipe, fp32-accurate: logits partials part[s][b][0..128] = sum over the s-th
// slice of the K = 4,096 flattened tail features (NHWC order, the permuted FC weights' rows)
// of x[b][k] * W[k][n], for n = [fc_policy; fc_value1] (129 columns).
//   * Workgroup = 32 R boards (R MFMA row tiles) x one K slice of 4,096 / S; four waves, wave w
//     the columns 32w .. 32w+31 (v_mfma_f32_32x32x16_f16) of every row tile, so each weight
//     fragment a wave requests feeds R tiles: the weight bytes streamed per board fall as 1 / R
//     (R = 1: 8 KiB per board, four times the board's own slice bytes).
//   * FP16X2 numerics as the trunk's: the weights scaled once by 2^wshift (the host prepares
//     wq = [K/16][hi, lo][128][16] fp16 words), each board's slice scaled by 2^(15 - e) with
//     max |x| < 2^e over the slice (reduced in the workgroup while the slice is staged), three
//     products lo*hi + hi*lo + hi*hi accumulated in fp32, both scales removed exactly in the
//     epilogue.  A partial's scale is its own slice's: the partials are unscaled fp32 sums,
//     which the finish kernel adds in slice order as before.
//   * Column 128 (fc_value1's last unit, the one column past four MFMA tiles) as fp32 FMAs
//     on the staged slice: eight lanes per row, reduced in a fixed order (deterministic; the
//     same bits for every R at one S).
namespace {
template <int S, int R>
struct HG {
  static constexpr int K = 4096, KS = K / S, STEPS = KS / 16, ITER = KS / 32;
  static constexpr int ROWS = 32 * R;
  static constexpr int SLAB = ROWS * 32 + 16;  // one (step, plane): rows x 32 B, + 16 B (banks)
  static constexpr int LDS_BYTES = STEPS * 2 * SLAB;
  static constexpr int PD = AZ_HG_PD;  // weight fragments requested this many steps ahead
  static constexpr int RING = PD < 4 ? 4 : 8;
  static_assert(STEPS % RING == 0 && ITER >= 1 && PD < RING, "slice");
  static_assert(R * ITER <= 32 && LDS_BYTES <= 160 * 1024, "staging registers / LDS");
};

typedef _Float16 hf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 hf16x4 __attribute__((ext_vector_type(4)));
typedef float hf32x16 __attribute__((ext_vector_type(16)));
typedef float hf32x4 __attribute__((ext_vector_type(4)));

template <int S, int R>
__global__ __launch_bounds__(256) void k_heads_fast_gemm(const float* __restrict__ x,
                                                         const char* __restrict__ wq,
                                                         const float* __restrict__ w128,
                                                         int wshift, float* __restrict__ part,
                                                         int ld, int n_boards) {
  using G = HG<S, R>;
  extern __shared__ float4 lds4[];
  char* lds = reinterpret_cast<char*>(lds4);
  __shared__ unsigned s_max[G::ROWS];
  __shared__ float s_c[G::ROWS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int b0 = blockIdx.x * G::ROWS, sl = blockIdx.y, k0 = sl * G::KS;

  // the wave's first weight fragments in flight while the slice is staged
  const int wlane = (32 * wave + r) * 32 + h * 16;
  auto load_b = [&](hf16x8 (&f)[2], int j) {
    const char* p = wq + (size_t)(k0 / 16 + j) * 2 * 128 * 32 + wlane;
    f[0] = *reinterpret_cast<const hf16x8*>(p);
    f[1] = *reinterpret_cast<const hf16x8*>(p + 128 * 32);
  };
  hf16x8 bf[G::RING][2];
#pragma unroll
  for (int j = 0; j < G::PD; ++j) load_b(bf[j], j);

  // ---- the slice: thread t owns rows t / 8 + 32 j (j < R) and the float4 columns k4 = t % 8
  // + 8 i (eight lanes per row read 128 contiguous bytes per iteration), so a row's max |x| and
  // its column-128 dot are per-thread sums reduced over eight lanes in a fixed order
  constexpr int Q = G::KS / 4;  // float4s per row
  static_assert(Q == 8 * G::ITER, "eight lanes per row");
  const int row0 = tid >> 3, q0 = tid & 7;
  float4 a[R][G::ITER];
  {
    const float4* wr = reinterpret_cast<const float4*>(w128 + k0);
    unsigned m[R];
    float c[R];
    const float4* xr[R];
    bool live[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      live[j] = b0 + row0 + 32 * j < n_boards;
      xr[j] = reinterpret_cast<const float4*>(
          x + (size_t)(live[j] ? b0 + row0 + 32 * j : 0) * G::K + k0);
      m[j] = 0u;
      c[j] = 0.0f;
    }
#pragma unroll
    for (int i = 0; i < G::ITER; ++i) {
      const float4 wv = wr[q0 + 8 * i];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const float4 v = live[j] ? xr[j][q0 + 8 * i] : make_float4(0.f, 0.f, 0.f, 0.f);
        a[j][i] = v;
        m[j] = max(m[j], max(max(__float_as_uint(fabsf(v.x)), __float_as_uint(fabsf(v.y))),
                             max(__float_as_uint(fabsf(v.z)), __float_as_uint(fabsf(v.w)))));
        c[j] = fmaf(v.w, wv.w, fmaf(v.z, wv.z, fmaf(v.y, wv.y, fmaf(v.x, wv.x, c[j]))));
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
#pragma unroll
      for (int off = 4; off > 0; off >>= 1) {  // the row's eight lanes (aligned groups of 8)
        m[j] = max(m[j], (unsigned)__shfl_xor((int)m[j], off, 64));
        c[j] += __shfl_xor(c[j], off, 64);
      }
      if (q0 == 0) {
        s_max[row0 + 32 * j] = m[j];
        s_c[row0 + 32 * j] = c[j];
      }
    }
  }
  __syncthreads();
  // split into the LDS image [step][plane][row][16] (fp16 hi, lo of x * 2^(15 - e_row))
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int row = row0 + 32 * j;
    const unsigned mb = s_max[row];
    const int be = (int)((mb >> 23) & 0xff), e = be == 0 ? 0 : be - 126;  // max < 2^e
    const float sc = ldexpf(1.0f, 15 - e);
#pragma unroll
    for (int i = 0; i < G::ITER; ++i) {
      const int kl = (q0 + 8 * i) * 4;
      const hf32x4 v = {a[j][i].x * sc, a[j][i].y * sc, a[j][i].z * sc, a[j][i].w * sc};  // exact
      const hf16x4 hi = __builtin_convertvector(v, hf16x4);
      const hf16x4 lo = __builtin_convertvector(v - __builtin_convertvector(hi, hf32x4), hf16x4);
      char* dst = lds + ((kl >> 4) * 2) * G::SLAB + row * 32 + (kl & 15) * 2;
      *reinterpret_cast<hf16x4*>(dst) = hi;
      *reinterpret_cast<hf16x4*>(dst + G::SLAB) = lo;
    }
  }
  __syncthreads();

  // ---- K loop: per step, A fragments (every row tile) from LDS, B from the weight ring
  hf32x16 acc[R];
#pragma unroll
  for (int t = 0; t < R; ++t) acc[t] = hf32x16{};
  const int aoff = r * 32 + h * 16;
#pragma unroll G::RING
  for (int j = 0; j < G::STEPS; ++j) {
    const int jn = j + G::PD < G::STEPS ? j + G::PD : G::STEPS - 1;
    load_b(bf[(j + G::PD) & (G::RING - 1)], jn);
    const hf16x8(&b)[2] = bf[j & (G::RING - 1)];
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const char* ap = lds + (j * 2) * G::SLAB + t * 32 * 32 + aoff;
      const hf16x8 ahi = *reinterpret_cast<const hf16x8*>(ap);
      const hf16x8 alo = *reinterpret_cast<const hf16x8*>(ap + G::SLAB);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, b[0], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, b[1], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, b[0], acc[t], 0, 0, 0);
    }
  }

  // ---- epilogue: D[row][col], col = lane & 31, row = 32 t + (k & 3) + 8 (k >> 2) + 4 h
  float* out = part + (size_t)sl * n_boards * ld;
  const int col = 32 * wave + r;
#pragma unroll
  for (int t = 0; t < R; ++t)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int row = 32 * t + (k & 3) + 8 * (k >> 2) + 4 * h, b = b0 + row;
      const unsigned mb = s_max[row];
      const int be = (int)((mb >> 23) & 0xff), e = be == 0 ? 0 : be - 126;
      if (b < n_boards) out[(size_t)b * ld + col] = acc[t][k] * ldexpf(1.0f, -(15 - e) - wshift);
    }
  if (tid < G::ROWS && b0 + tid < n_boards) {  // column 128 (fp32 FMAs), columns past it zero
    float* o = out + (size_t)(b0 + tid) * ld;
    o[128] = s_c[tid];
    for (int n = 129; n < ld; ++n) o[n] = 0.0f;
  }
}

template <int S, int R>
int launch_heads_fast_gemm(const float* x, const void* wq, const float* w128, int wshift,
                           float* part, int ld, int n_boards, hipStream_t s) {
  using G = HG<S, R>;
  static bool attr_set = false;  // > 64 KiB of dynamic LDS needs the opt-in once
  if (!attr_set) {
    AZ_HIP(hipFuncSetAttribute((const void*)k_heads_fast_gemm<S, R>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES));
    attr_set = true;
  }
  const dim3 grid((unsigned)((n_boards + G::ROWS - 1) / G::ROWS), S);
  hipLaunchKernelGGL((k_heads_fast_gemm<S, R>), grid, dim3(256), G::LDS_BYTES, s, x,
                     static_cast<const char*>(wq), w128, wshift, part, ld, n_boards);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
}  // namespace

extern "C" int az_heads_fast_gemm_gpu(const float* x, const void* wq, const float* w128,
                                      int32_t wshift, float* part, int32_t ld, int32_t splits,
                                      int32_t board_tile, int32_t n_boards, void* stream) {
  AZ_REQUIRE(n_boards >= 0 && ld >= 129, AZ_ERR_ARG,
             "az_heads_fast_gemm_gpu: n_boards %d < 0 or ld %d < 129", n_boards, ld);
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && wq && w128 && part, AZ_ERR_ARG, "az_heads_fast_gemm_gpu: null buffer");
  AZ_REQUIRE(((uintptr_t)x | (uintptr_t)wq | (uintptr_t)w128) % 16 == 0, AZ_ERR_ARG,
             "az_heads_fast_gemm_gpu: buffers must be 16-byte aligned");
  AZ_REQUIRE(wshift > -126 && wshift < 126, AZ_ERR_ARG, "az_heads_fast_gemm_gpu: wshift %d",
             wshift);
  hipStream_t s = azc::as_stream(stream);
  if (board_tile == 32 && splits == 4)
    return launch_heads_fast_gemm<4, 1>(x, wq, w128, wshift, part, ld, n_boards, s);
  if (board_tile == 32 && splits == 8)
    return launch_heads_fast_gemm<8, 1>(x, wq, w128, wshift, part, ld, n_boards, s);
  if (board_tile == 64 && splits == 8)
    return launch_heads_fast_gemm<8, 2>(x, wq, w128, wshift, part, ld, n_boards, s);
  if (board_tile == 64 && splits == 16)
    return launch_heads_fast_gemm<16, 2>(x, wq, w128, wshift, part, ld, n_boards, s);
  if (board_tile == 128 && splits == 16)
    return launch_heads_fast_gemm<16, 4>(x, wq, w128, wshift, part, ld, n_boards, s);
  return azc::set_error(AZ_ERR_ARG,
                        "az_heads_fast_gemm_gpu: (board_tile, splits) must be (32, 4), (32, 8), "
                        "(64, 8), (64, 16) or (128, 16), got (%d, %d)",
                        board_tile, splits);
}
