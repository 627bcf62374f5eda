// conv16.hip — 16-bit-operand MFMA 3x3 convolution for 8x8 boards, epilogue fused.
//
// Same op as conv.hip (conv + bias (+ residual) + ReLU over NHWC fp32 activations,
// Ci = Co = C), on the 16x-denser 16-bit MFMA pipe (v_mfma_f32_32x32x16_{bf16,f16}),
// in two numerics modes:
//
//   AZ_CONV_SPLIT3 (fp32-accurate): every fp32 operand x is split into three bf16 words
//     x = x0 + x1 + x2 (x0 = RN(x), x1 = RN(x - x0), x2 = RN(x - x0 - x1): 3 x 8 mantissa
//     bits = fp32's 24) and the product is accumulated in fp32 from the six partial
//     products whose order is at most 2^-16 below the leading one:
//       x0y0 + x0y1 + x1y0 + x0y2 + x1y1 + x2y0
//     (dropped: x1y2, x2y1, x2y2 ~ 2^-24 relative — fp32's own rounding unit).  Six bf16
//     MFMAs cost 6/16 of one fp32 MFMA of the same shape.
//   AZ_CONV_FP16: one fp16 product (BASELINE configs[4]'s fp16 inference).
//
// GEMM view: M = B*64 output positions, N = C, K = 9 taps x C.  Workgroup = 2 boards
// (M = 128) x all C columns, waves 2 (M) x C/64 (N), each wave 64 x 64 (2 x 2 tiles of
// 32x32).  The two input boards sit in LDS as fp32 for the whole kernel (positions padded
// to C + 4 floats: conflict-free ds_read_b128 row gathers; one all-zero position for the
// off-board taps); A fragments are split into bf16 words in registers.  Weights arrive
// pre-split from az_conv3x3_mx_prep_gpu as [tap][ci/16][plane][co][16] 16-bit words: each
// (tap, 16-channel chunk) step is one contiguous PLANES*C*32-byte block, loaded by the
// workgroup two steps ahead into registers and stored into a double-buffered LDS stage
// (rows padded to 48 B: conflict-free ds_read_b128), one barrier per step.
#include <type_traits>

#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int C_, int MODE_>
struct Mx {
  static constexpr int C = C_, MODE = MODE_;
  static constexpr int PLANES = MODE == AZ_CONV_SPLIT3 ? 3 : 1;
  static constexpr int BOARDS = 2;
  static constexpr int WAVES_N = C / 64, WAVES = 2 * WAVES_N, THREADS = 64 * WAVES;
  static constexpr int TM = 2, TN = 2;
  static constexpr int APOS = PLANES * C * 2 + 16;  // bytes per staged position (padded)
  static constexpr int A_BYTES = (BOARDS * 64 + 1) * APOS;
  static constexpr int BROW = 48;                   // bytes per (plane, co) row of a stage
  static constexpr int BSTAGE = PLANES * C * BROW;  // bytes per LDS stage
  static constexpr int CHUNKS = C / 16, STEPS = 9 * CHUNKS;
  static constexpr int STEP_BYTES = PLANES * C * 32;  // global bytes per step
  static constexpr int LOADS = STEP_BYTES / (THREADS * 16);
  static constexpr size_t LDS_BYTES = (size_t)A_BYTES + 2 * BSTAGE;
  static_assert(LOADS == PLANES, "one 16-byte load per plane per thread per step");
};


// MFMA operands of one step: PLANES 16-bit words per element for A and for B
template <class G>
struct Frags {
  using T = typename std::conditional<G::MODE == AZ_CONV_SPLIT3, bf16x8, f16x8>::type;
  T a[G::PLANES][G::TM];
  T b[G::PLANES][G::TN];
};

// one step's A fragments: lane (r, h) of tile mi reads, per plane, the 8 words of channels
// ci0+8h.. of its row's tapped position (or of the all-zero position)
template <class G>
__device__ __forceinline__ void mx_read_a(Frags<G>& f, const char* lds_a, int s,
                                          const int (&pos0)[G::TM], const int (&ok9)[G::TM],
                                          int h) {
  using T = typename Frags<G>::T;
  const int tap = s / G::CHUNKS, ci0 = (s % G::CHUNKS) * 16;
  const int d = (tap / 3 - 1) * 8 + (tap % 3 - 1);
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi) {
    const int pos = (ok9[mi] >> tap) & 1 ? pos0[mi] + d : G::BOARDS * 64;
    const char* p = lds_a + pos * G::APOS + (ci0 + 8 * h) * 2;
#pragma unroll
    for (int pl = 0; pl < G::PLANES; ++pl)
      f.a[pl][mi] = *reinterpret_cast<const T*>(p + pl * G::C * 2);
  }
}

template <class G>
__device__ __forceinline__ void mx_read_b(Frags<G>& f, const char* stage, const int (&boff)[G::TN]) {
  using T = typename Frags<G>::T;
#pragma unroll
  for (int p = 0; p < G::PLANES; ++p)
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni)
      f.b[p][ni] = *reinterpret_cast<const T*>(stage + p * G::C * G::BROW + boff[ni]);
}

template <class G>
__device__ __forceinline__ void mx_mma(f32x16 (&acc)[G::TM][G::TN], const Frags<G>& f) {
  if constexpr (G::MODE == AZ_CONV_SPLIT3) {
    // smallest partial products first (x2y0, x1y1, x0y2, x1y0, x0y1, x0y0); consecutive
    // MFMAs write different accumulators
    constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < G::TN; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[PA[t]][mi], f.b[PB[t]][ni],
                                                                acc[mi][ni], 0, 0, 0);
  } else {
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < G::TN; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.a[0][mi], f.b[0][ni], acc[mi][ni],
                                                             0, 0, 0);
  }
}

template <class G>
__device__ __forceinline__ void mx_load_w(u32x4 (&wr)[G::LOADS], const u32x4* wsrc, int s) {
#pragma unroll
  for (int k = 0; k < G::LOADS; ++k)
    wr[k] = wsrc[(size_t)s * (G::STEP_BYTES / 16) + k * G::THREADS];
}
template <class G>
__device__ __forceinline__ void mx_store_w(const u32x4 (&wr)[G::LOADS], char* stage,
                                           const int (&bdst)[G::LOADS]) {
#pragma unroll
  for (int k = 0; k < G::LOADS; ++k) *reinterpret_cast<u32x4*>(stage + bdst[k]) = wr[k];
}

template <class G, bool RES, bool RELU>
__global__ __launch_bounds__(G::THREADS) void k_conv3x3_mx(const float* __restrict__ x,
                                                           const u32x4* __restrict__ wq,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ res,
                                                           float* __restrict__ y,
                                                           int n_boards) {
  constexpr int C = G::C, kBoards = G::BOARDS, kThreads = G::THREADS;
  extern __shared__ float4 lds4[];
  char* lds_a = reinterpret_cast<char*>(lds4);
  char* lds_b = lds_a + G::A_BYTES;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int b0 = blockIdx.x * kBoards;
  const int nb = n_boards - b0 < kBoards ? n_boards - b0 : kBoards;

  // ---- weights: this thread's share of one step (LOADS x 16 B) and its LDS slots
  const u32x4* wsrc = wq + tid;
  int bdst[G::LOADS];
#pragma unroll
  for (int k = 0; k < G::LOADS; ++k) {
    const int idx = k * kThreads + tid;  // 16-byte unit within the step block
    const int plane = idx / (2 * C), rem = idx % (2 * C);
    bdst[k] = plane * C * G::BROW + (rem >> 1) * G::BROW + (rem & 1) * 16;
  }
  u32x4 wx[G::LOADS], wy[G::LOADS];
  mx_load_w<G>(wx, wsrc, 0);
  mx_load_w<G>(wy, wsrc, 1);

  // ---- stage the input boards (NHWC) into LDS as PLANES 16-bit words per element (the
  // split of every activation done once here, not once per tap); zero-fill a missing tail
  // board and the all-zero position (index kBoards*64) that off-board taps read
  {
    constexpr int V = (kBoards * 64 + 1) * C / 4;
    const float4* src = reinterpret_cast<const float4*>(x + (size_t)b0 * 64 * C);
    for (int v = tid; v < V; v += kThreads) {
      const int pos = v / (C / 4), c4 = v % (C / 4);
      float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
      if (pos < nb * 64) val = src[v];
      char* dst = lds_a + pos * G::APOS + c4 * 8;
      const f32x4 a = {val.x, val.y, val.z, val.w};
      if constexpr (G::MODE == AZ_CONV_SPLIT3) {
        const bf16x4 x0 = __builtin_convertvector(a, bf16x4);
        const f32x4 r1 = a - __builtin_convertvector(x0, f32x4);
        const bf16x4 x1 = __builtin_convertvector(r1, bf16x4);
        const bf16x4 x2 = __builtin_convertvector(r1 - __builtin_convertvector(x1, f32x4), bf16x4);
        *reinterpret_cast<bf16x4*>(dst) = x0;
        *reinterpret_cast<bf16x4*>(dst + C * 2) = x1;
        *reinterpret_cast<bf16x4*>(dst + C * 4) = x2;
      } else {
        *reinterpret_cast<f16x4*>(dst) = __builtin_convertvector(a, f16x4);
      }
    }
  }
  mx_store_w<G>(wx, lds_b, bdst);
  mx_load_w<G>(wx, wsrc, 2);
  __syncthreads();

  const int wm = wave / G::WAVES_N, wn = wave % G::WAVES_N;
  const int row0 = wm * 64, col0 = wn * 64;
  const int r = lane & 31, h = lane >> 5;
  // per A tile: this lane's output position and which of the 9 taps land on the board
  int pos0[G::TM], ok9[G::TM];
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi) {
    const int m = row0 + 32 * mi + r;
    const int py = (m >> 3) & 7, px = m & 7;
    pos0[mi] = m;
    int ok = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
      ok |= ((unsigned)yy < 8u && (unsigned)xx < 8u) << t;
    }
    ok9[mi] = ok;
  }
  int boff[G::TN];
#pragma unroll
  for (int ni = 0; ni < G::TN; ++ni) boff[ni] = (col0 + 32 * ni + r) * G::BROW + h * 16;

  f32x16 acc[G::TM][G::TN];
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[mi][ni][k] = 0.0f;

  // Two LDS weight stages, one barrier per step; the next step's A fragments are read
  // from the resident boards before this step's MFMAs; weights are loaded two steps ahead
  // into registers.  Every load and store is unconditional (indices clamped to the last
  // step; surplus stores land in a stage nobody reads again), which keeps the compiler's
  // vmcnt bookkeeping exact.
  static_assert(G::STEPS % 2 == 0 && G::STEPS >= 4, "step pairs");
  constexpr int last = G::STEPS - 1;
  Frags<G> f0, f1;
  mx_read_a<G>(f0, lds_a, 0, pos0, ok9, h);
  for (int s = 0; s < G::STEPS; s += 2) {
    mx_read_a<G>(f1, lds_a, s + 1, pos0, ok9, h);
    mx_read_b<G>(f0, lds_b, boff);
    mx_mma<G>(acc, f0);
    mx_store_w<G>(wy, lds_b + G::BSTAGE, bdst);
    mx_load_w<G>(wy, wsrc, s + 3 < last ? s + 3 : last);
    __syncthreads();
    mx_read_a<G>(f0, lds_a, s + 2 < last ? s + 2 : last, pos0, ok9, h);
    mx_read_b<G>(f1, lds_b + G::BSTAGE, boff);
    mx_mma<G>(acc, f1);
    mx_store_w<G>(wx, lds_b, bdst);
    mx_load_w<G>(wx, wsrc, s + 4 < last ? s + 4 : last);
    __syncthreads();
  }

  // ---- epilogue: D[row][col], col = lane&31, row = (k&3) + 8*(k>>2) + 4*(lane>>5); a
  // 32-row tile lies inside one board, so the tail-board test is uniform per tile
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi) {
    if (((row0 + 32 * mi) >> 6) >= nb) continue;
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni) {
      const int co = col0 + 32 * ni + r;
      const float bv = bias[co];
      const size_t o0 = ((size_t)b0 * 64 + row0 + 32 * mi + 4 * h) * C + co;
      float rv[16];
      if (RES) {
#pragma unroll
        for (int k = 0; k < 16; ++k) rv[k] = res[o0 + (size_t)((k & 3) + 8 * (k >> 2)) * C];
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        float v = acc[mi][ni][k] + bv;
        if (RES) v += rv[k];
        if (RELU) v = fmaxf(v, 0.0f);
        y[o0 + (size_t)((k & 3) + 8 * (k >> 2)) * C] = v;
      }
    }
  }
}

// w9 [9][Co][Ci] fp32 -> wq [9][Ci/16][PLANES][Co][16] 16-bit words
template <int MODE>
__global__ void k_conv_mx_prep(const float* __restrict__ w9, uint16_t* __restrict__ wq, int C) {
  constexpr int P = MODE == AZ_CONV_SPLIT3 ? 3 : 1;
  const int n = 9 * C * C;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int tap = i / (C * C), co = (i / C) % C, ci = i % C;
    const float v = w9[i];
    const size_t base = ((((size_t)tap * (C / 16) + ci / 16) * P) * C + co) * 16 + (ci & 15);
    const size_t pstride = (size_t)C * 16;
    if constexpr (MODE == AZ_CONV_SPLIT3) {
      const __bf16 x0 = (__bf16)v;
      const float r1 = v - (float)x0;
      const __bf16 x1 = (__bf16)r1;
      const __bf16 x2 = (__bf16)(r1 - (float)x1);
      wq[base] = __builtin_bit_cast(uint16_t, x0);
      wq[base + pstride] = __builtin_bit_cast(uint16_t, x1);
      wq[base + 2 * pstride] = __builtin_bit_cast(uint16_t, x2);
    } else {
      wq[base] = __builtin_bit_cast(uint16_t, (_Float16)v);
    }
  }
}

template <class G>
int launch_mx(const float* x, const void* wq, const float* bias, const float* res, float* y,
              int n_boards, int relu, hipStream_t s) {
  const unsigned grid = (unsigned)((n_boards + G::BOARDS - 1) / G::BOARDS);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS needs the opt-in once per kernel
  if (!attr_set) {
    const void* ks[] = {(const void*)k_conv3x3_mx<G, true, true>,
                        (const void*)k_conv3x3_mx<G, true, false>,
                        (const void*)k_conv3x3_mx<G, false, true>,
                        (const void*)k_conv3x3_mx<G, false, false>};
    for (const void* k : ks)
      AZ_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)G::LDS_BYTES));
    attr_set = true;
  }
  const u32x4* w = static_cast<const u32x4*>(wq);
  const dim3 blk(G::THREADS);
  const size_t lds = G::LDS_BYTES;
  if (res && relu)
    hipLaunchKernelGGL((k_conv3x3_mx<G, true, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else if (res)
    hipLaunchKernelGGL((k_conv3x3_mx<G, true, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else if (relu)
    hipLaunchKernelGGL((k_conv3x3_mx<G, false, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else
    hipLaunchKernelGGL((k_conv3x3_mx<G, false, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

}  // namespace

extern "C" int az_conv3x3_mx_prep_gpu(const float* w9, void* wq, int32_t channels, int32_t mode,
                                      void* stream) {
  AZ_REQUIRE(w9 && wq, AZ_ERR_ARG, "az_conv3x3_mx_prep_gpu: null buffer");
  AZ_REQUIRE(channels == 64 || channels == 128, AZ_ERR_ARG,
             "az_conv3x3_mx_prep_gpu: channels must be 64 or 128, got %d", channels);
  hipStream_t s = azc::as_stream(stream);
  const unsigned grid = (unsigned)((9 * channels * channels + 255) / 256);
  uint16_t* out = static_cast<uint16_t*>(wq);
  if (mode == AZ_CONV_SPLIT3)
    hipLaunchKernelGGL(k_conv_mx_prep<AZ_CONV_SPLIT3>, dim3(grid), dim3(256), 0, s, w9, out, channels);
  else if (mode == AZ_CONV_FP16)
    hipLaunchKernelGGL(k_conv_mx_prep<AZ_CONV_FP16>, dim3(grid), dim3(256), 0, s, w9, out, channels);
  else
    return azc::set_error(AZ_ERR_ARG, "az_conv3x3_mx_prep_gpu: unknown mode %d", mode);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

extern "C" int az_conv3x3_mx_gpu(const float* x, const void* wq, const float* bias,
                                 const float* res, float* y, int32_t n_boards,
                                 int32_t channels, int32_t relu, int32_t mode, void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_conv3x3_mx_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && wq && bias && y && x != y, AZ_ERR_ARG,
             "az_conv3x3_mx_gpu: null buffer or in-place call");
  AZ_REQUIRE(((uintptr_t)x | (uintptr_t)wq | (uintptr_t)bias) % 16 == 0, AZ_ERR_ARG,
             "az_conv3x3_mx_gpu: buffers must be 16-byte aligned");
  hipStream_t s = azc::as_stream(stream);
  if (channels == 128 && mode == AZ_CONV_SPLIT3)
    return launch_mx<Mx<128, AZ_CONV_SPLIT3>>(x, wq, bias, res, y, n_boards, relu, s);
  if (channels == 64 && mode == AZ_CONV_SPLIT3)
    return launch_mx<Mx<64, AZ_CONV_SPLIT3>>(x, wq, bias, res, y, n_boards, relu, s);
  if (channels == 128 && mode == AZ_CONV_FP16)
    return launch_mx<Mx<128, AZ_CONV_FP16>>(x, wq, bias, res, y, n_boards, relu, s);
  if (channels == 64 && mode == AZ_CONV_FP16)
    return launch_mx<Mx<64, AZ_CONV_FP16>>(x, wq, bias, res, y, n_boards, relu, s);
  return azc::set_error(AZ_ERR_ARG, "az_conv3x3_mx_gpu: channels %d / mode %d unsupported",
                        channels, mode);
}
