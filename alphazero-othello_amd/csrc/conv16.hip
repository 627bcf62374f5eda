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
//   AZ_CONV_FP16X2 (fp32-accurate, half of SPLIT3's products): both operands as an fp16
//     pair hi + lo (22 significant bits) after exact power-of-two scaling -- the weights per
//     layer (az_conv3x3_mx_prep_gpu's header), the inputs per board from the board's max |x|,
//     reduced in the workgroup while it stages the board (no range buffer) -- and the three
//     leading products lo*hi + hi*lo + hi*hi accumulated in fp32; the epilogue removes both
//     scales exactly (a power of two).  FastOthelloNet's 64-channel convs (configs[1]).
//
// GEMM view: M = B*64 output positions, N = C, K = 9 taps x C.  Workgroup = 1 board
// (M = 64 rows; 51 KB of LDS: 3 workgroups per CU, so one workgroup's staging and
// epilogue overlap another's MFMAs) or 2 boards (cfg 0: 101 KB, one per CU) x all C
// columns; wave w owns all the rows x columns 32w..32w+31, so each weight fragment feeds
// two (four) MFMAs.
//   * A: the two boards are split into PLANES 16-bit words per element ONCE, while being
//     staged into LDS as [position][plane][C] (+16 B per position: conflict-free
//     ds_read_b128 row gathers; one all-zero position for the off-board taps), and stay
//     resident for all 9 taps.
//   * B: weights pre-split by az_conv3x3_mx_prep_gpu into [tap][ci/16][plane][Co][16]
//     words; every wave streams its own 32 columns straight from L2 into registers, three
//     (tap, 16-channel) steps ahead.  No LDS stage, so the main loop has no barrier.
//   * A fragments of the next step are read from LDS during this step's MFMAs.
//   * Epilogue straight from the accumulators: + bias, + residual, ReLU, NHWC store.
#include <stdlib.h>

#include <type_traits>

#include "common.h"

// experiment hooks (scripts/exp/conv16_exp.py builds copies with bits set): 1 = no A reads
// in the main loop, 2 = no weight loads in the main loop, 4 = no board staging, 8 = no
// epilogue stores, 16 = workgroup 0 stamps s_memtime / s_memrealtime around its main loop
// into y[0..3] (shader clock).  The product build leaves it 0.
#ifndef AZ_MX_EXP
#define AZ_MX_EXP 0
#endif

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

template <int C_, int MODE_, int BOARDS_ = 2>
struct Mx {
  static constexpr int C = C_, MODE = MODE_;
  static constexpr int PLANES = MODE == AZ_CONV_SPLIT3 ? 3 : (MODE == AZ_CONV_FP16X2 ? 2 : 1);
  static constexpr bool SCALED = MODE == AZ_CONV_FP16X2;  // power-of-two operand scaling
  // MFMA products per (A, B) fragment pair
  static constexpr int PRODUCTS = MODE == AZ_CONV_SPLIT3 ? 6 : (MODE == AZ_CONV_FP16X2 ? 3 : 1);
  static constexpr int BOARDS = BOARDS_;
  static constexpr int TM = 2 * BOARDS;             // 32-row tiles per wave (= all rows)
  static constexpr int WAVES = C / 32, THREADS = 64 * WAVES;
  static constexpr int APOS = PLANES * C * 2 + 16;  // LDS bytes per staged position
  static constexpr int A_BYTES = (BOARDS * 64 + 1) * APOS;
  static constexpr int CHUNKS = C / 16, STEPS = 9 * CHUNKS;
  static constexpr int STEP_BYTES = PLANES * C * 32;  // weight bytes per (tap, chunk) step
  static constexpr int W_BYTES = STEPS * STEP_BYTES;  // the weight words (FP16X2: header after)
  static constexpr size_t LDS_BYTES = A_BYTES;
  static_assert(CHUNKS % 4 == 0, "the chunk loop is unrolled by 4");
};

template <class G>
using Word8 = typename std::conditional<G::MODE == AZ_CONV_SPLIT3, bf16x8, f16x8>::type;

template <class G>
struct AFrag {
  Word8<G> v[G::PLANES][G::TM];
};
template <class G>
struct BFrag {
  Word8<G> v[G::PLANES];
};

// LDS byte offset of the A row each tile's lane reads at `tap` (its tapped position, or
// the all-zero position), with the lane's k-half folded in
template <class G>
__device__ __forceinline__ void mx_tap_base(int (&base)[G::TM], int tap,
                                            const int (&pos0)[G::TM], const int (&ok9)[G::TM],
                                            int h) {
  const int d = (tap / 3 - 1) * 8 + (tap % 3 - 1);
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi) {
    const int pos = (ok9[mi] >> tap) & 1 ? pos0[mi] + d : G::BOARDS * 64;
    base[mi] = pos * G::APOS + 16 * h;
  }
}

// A fragments of (tap, chunk ch): per plane, the 8 words of channels 16ch+8h.. (the chunk
// and plane offsets are ds_read immediates); issued in the order mx_mma consumes them
template <class G>
__device__ __forceinline__ void mx_read_a(AFrag<G>& f, const char* lds_a,
                                          const int (&base)[G::TM], int ch) {
#pragma unroll
  for (int pl = G::PLANES - 1; pl >= 0; --pl)
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi)
      f.v[pl][mi] = *reinterpret_cast<const Word8<G>*>(lds_a + base[mi] + ch * 32 + pl * G::C * 2);
}

// B fragments of step s: this lane's 16 bytes of each plane (column col0 + r, k = 8h..)
template <class G>
__device__ __forceinline__ void mx_load_b(BFrag<G>& f, const char* wq, int lane_off, int s) {
  const char* step = wq + (size_t)s * G::STEP_BYTES;  // uniform base: saddr + lane offset
#pragma unroll
  for (int pl = 0; pl < G::PLANES; ++pl)
    f.v[pl] = *reinterpret_cast<const Word8<G>*>(step + lane_off + pl * G::C * 32);
}

template <class G>
__device__ __forceinline__ void mx_mma(f32x16 (&acc)[G::TM], const AFrag<G>& a,
                                       const BFrag<G>& b) {
  if constexpr (G::MODE == AZ_CONV_SPLIT3) {
    // smallest partial products first (x2y0, x1y1, x0y2, x1y0, x0y1, x0y0); consecutive
    // MFMAs write different accumulators
    constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi)
        acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[PA[t]][mi], b.v[PB[t]], acc[mi],
                                                          0, 0, 0);
  } else if constexpr (G::MODE == AZ_CONV_FP16X2) {
    // lo * hi, hi * lo, hi * hi (the lo * lo term is below fp32's rounding unit); consecutive
    // MFMAs write different accumulators
    constexpr int PA[3] = {1, 0, 0}, PB[3] = {0, 1, 0};
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi)
        acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[PA[t]][mi], b.v[PB[t]], acc[mi],
                                                         0, 0, 0);
  } else {
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi)
      acc[mi] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[0][mi], b.v[0], acc[mi], 0, 0, 0);
  }
}

// issue pattern of one main-loop step (see AZ_MX_STEP)
template <class G>
__device__ __forceinline__ void mx_sched() {
  constexpr int kMfma = G::PRODUCTS * G::TM;
  constexpr int kDs = G::PLANES * G::TM;
  constexpr int kPer = kMfma / kDs > 0 ? kMfma / kDs : 1;
#pragma unroll
  for (int i = 0; i < kDs; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, kPer, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);     // DS read
  }
  __builtin_amdgcn_sched_group_barrier(0x008, kMfma, 0);   // remaining MFMAs
  __builtin_amdgcn_sched_group_barrier(0x020, G::PLANES, 0);  // VMEM read
  __builtin_amdgcn_sched_barrier(0);
}

// The stem (1 -> C 3x3 conv + bias + ReLU on the canonical planes, k_conv_stem's exact
// fmaf chain) evaluated where its output is consumed, so it is never written to HBM:
// STEM = 1: this conv's input is stem(planes) (the first residual block's conv1);
// STEM = 2: this conv's residual is stem(planes) (that block's conv2).
struct StemArgs {
  const float* planes;  // [n_boards][64] float, canonical boards
  const float* w;       // [9][C]
  const float* b;       // [C]
};

// stem output for 4 channels c..c+3 at square p of the staged plane grid `pl` (10 x 10,
// zero border): same tap order and fmaf chain as k_conv_stem
// (sw / sb: the four channels' weights and bias, loaded once by the caller)
__device__ __forceinline__ float4 stem4(const float* pl, int p, const float4 (&sw)[9], float4 sb) {
  const int py = p >> 3, px = p & 7;
  float4 acc = sb;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
    if ((unsigned)yy < 8u && (unsigned)xx < 8u) {
      const float v = pl[(yy + 1) * 10 + xx + 1];
      const float4 wv = sw[t];
      acc.x = fmaf(v, wv.x, acc.x);
      acc.y = fmaf(v, wv.y, acc.y);
      acc.z = fmaf(v, wv.z, acc.z);
      acc.w = fmaf(v, wv.w, acc.w);
    }
  }
  return make_float4(fmaxf(acc.x, 0.f), fmaxf(acc.y, 0.f), fmaxf(acc.z, 0.f), fmaxf(acc.w, 0.f));
}

// The main loop of one conv: 9 taps x C/16 chunks of 16 input channels, A fragments from the
// staged image lds_a, B (weights) streamed three steps ahead through the ring b0f..b3f (the
// first three requested by the caller: steps 0, 1, 2); acc is zeroed here.
template <class G>
__device__ __forceinline__ void mx_kloop(f32x16 (&acc)[G::TM], const char* lds_a, const char* wq,
                                         int wlane, const int (&pos0)[G::TM],
                                         const int (&ok9)[G::TM], int h, BFrag<G>& b0f,
                                         BFrag<G>& b1f, BFrag<G>& b2f, BFrag<G>& b3f) {
  constexpr int last = G::STEPS - 1;
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[mi][k] = 0.0f;

  // Step s = (tap, chunk): MFMAs on A set s%2 and B set s%4; the A set of step s+1 is read
  // meanwhile (next tap's row offsets precomputed at the tap's start) and B set (s+3)%4 —
  // consumed by step s-1 — reloaded with step s+3.  Indices are clamped to the last step
  // so every load is unconditional (exact vmcnt bookkeeping); surplus loads are unused.
  // The machine scheduler would put a step's loads in one burst ahead of its MFMAs (the
  // MFMA pipe then idles while they issue) or sink them behind; mx_sched pins the issue
  // pattern: each LDS read in the shadow of two MFMAs, the weight loads behind the MFMAs.
  static_assert(G::CHUNKS % 4 == 0, "B ring of 4 and A ring of 2 within a tap");
  AFrag<G> a0f, a1f;
  int bcur[G::TM], bnxt[G::TM];
  mx_tap_base<G>(bcur, 0, pos0, ok9, h);
  mx_read_a<G>(a0f, lds_a, bcur, 0);
#define AZ_MX_STEP(CH, AC, AN, BC, BL)                                              \
  {                                                                                 \
    const int s_ = tap * G::CHUNKS + (CH);                                          \
    if (!(AZ_MX_EXP & 1)) {                                                         \
      if ((CH) + 1 < G::CHUNKS)                                                     \
        mx_read_a<G>(AN, lds_a, bcur, (CH) + 1);                                    \
      else                                                                          \
        mx_read_a<G>(AN, lds_a, bnxt, 0);                                           \
    }                                                                               \
    mx_mma<G>(acc, AC, BC);                                                         \
    if (!(AZ_MX_EXP & 2)) mx_load_b<G>(BL, wq, wlane, s_ + 3 < last ? s_ + 3 : last); \
    mx_sched<G>();                                                                  \
  }
  for (int tap = 0; tap < 9; ++tap) {
    mx_tap_base<G>(bnxt, tap + 1 < 9 ? tap + 1 : 8, pos0, ok9, h);
#pragma unroll
    for (int c4 = 0; c4 < G::CHUNKS; c4 += 4) {
      AZ_MX_STEP(c4 + 0, a0f, a1f, b0f, b3f)
      AZ_MX_STEP(c4 + 1, a1f, a0f, b1f, b0f)
      AZ_MX_STEP(c4 + 2, a0f, a1f, b2f, b1f)
      AZ_MX_STEP(c4 + 3, a1f, a0f, b3f, b2f)
    }
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi) bcur[mi] = bnxt[mi];
  }
#undef AZ_MX_STEP
}

template <class G, bool RES, bool RELU, int STEM>
__global__ __launch_bounds__(G::THREADS) void k_conv3x3_mx(const float* __restrict__ x,
                                                           const char* __restrict__ wq,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ res,
                                                           float* __restrict__ y,
                                                           int n_boards, StemArgs st) {
  constexpr int C = G::C, kBoards = G::BOARDS, kThreads = G::THREADS;
  extern __shared__ float4 lds4[];
  __shared__ float s_plane[kBoards][100];  // STEM: the boards' planes with a zero border
  char* lds_a = reinterpret_cast<char*>(lds4);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int col0 = wave * 32;
  const int b0 = blockIdx.x * kBoards;
  const int nb = n_boards - b0 < kBoards ? n_boards - b0 : kBoards;
  // FP16X2: each staged board's max |x| (float bits: non-negative floats order as unsigned)
  __shared__ unsigned s_amax[kBoards];
  if (G::SCALED) {
    if (tid < kBoards) s_amax[tid] = 0u;
    __syncthreads();
  }

  // weights of the first three steps are in flight while the boards are staged
  const int wlane = (col0 + r) * 32 + h * 16;
  BFrag<G> b0f, b1f, b2f, b3f;
  mx_load_b<G>(b0f, wq, wlane, 0);
  mx_load_b<G>(b1f, wq, wlane, 1);
  mx_load_b<G>(b2f, wq, wlane, 2);

  // ---- stage the input boards (NHWC) into LDS as PLANES 16-bit words per element (the
  // split of every activation done once here, not once per tap); zero-fill a missing tail
  // board and the all-zero position (index kBoards*64) that off-board taps read
  {
    // every load issued before the first conversion (one HBM round trip, not one per
    // iteration)
    constexpr int V = (kBoards * 64 + 1) * C / 4;
    constexpr int ITER = (V + kThreads - 1) / kThreads;
    if (STEM) {
      for (int i = tid; i < kBoards * 100; i += kThreads) {
        const int bb = i / 100, q = i % 100, yy = q / 10 - 1, xx = q % 10 - 1;
        const bool in = bb < nb && (unsigned)yy < 8u && (unsigned)xx < 8u;
        s_plane[bb][q] = in ? st.planes[(size_t)(b0 + bb) * 64 + yy * 8 + xx] : 0.f;
      }
      __syncthreads();
    }
    const float4* src = reinterpret_cast<const float4*>(x + (size_t)b0 * 64 * C);
    // STEM = 1: a thread's channel quad is the same in every iteration (kThreads is a multiple
    // of C / 4), so its stem weights and bias are loaded once
    static_assert(kThreads % (C / 4) == 0, "one channel quad per thread");
    float4 stw[9], stb = make_float4(0.f, 0.f, 0.f, 0.f);
    if (STEM == 1) {
      const int c = (tid % (C / 4)) * 4;
#pragma unroll
      for (int t = 0; t < 9; ++t) stw[t] = *reinterpret_cast<const float4*>(st.w + t * C + c);
      stb = *reinterpret_cast<const float4*>(st.b + c);
    }
    float4 val[ITER];
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int v = tid + i * kThreads;
      val[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (STEM == 1) {
        if (v < nb * 64 * (C / 4)) {
          const int pos = v / (C / 4);
          val[i] = stem4(s_plane[pos >> 6], pos & 63, stw, stb);
        }
      } else if (!(AZ_MX_EXP & 4) && v < nb * 64 * (C / 4)) {
        val[i] = src[v];
      }
    }
    // FP16X2: the boards' max |x| (this thread's values, then the wave, then LDS), and the
    // per-board input scale 2^sx[b] that maps it below 2^15 (fp16's max is 65504)
    float xsc[kBoards];
    if constexpr (G::SCALED) {
      unsigned m[kBoards];
#pragma unroll
      for (int b = 0; b < kBoards; ++b) m[b] = 0u;
#pragma unroll
      for (int i = 0; i < ITER; ++i) {
        const int v = tid + i * kThreads;
        const int bb = (v / (C / 4)) >> 6;
        const unsigned u = max(max(__float_as_uint(fabsf(val[i].x)), __float_as_uint(fabsf(val[i].y))),
                               max(__float_as_uint(fabsf(val[i].z)), __float_as_uint(fabsf(val[i].w))));
#pragma unroll
        for (int b = 0; b < kBoards; ++b)
          if (bb == b) m[b] = max(m[b], u);
      }
#pragma unroll
      for (int b = 0; b < kBoards; ++b) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) m[b] = max(m[b], (unsigned)__shfl_xor((int)m[b], off, 64));
        if ((tid & 63) == 0) atomicMax(&s_amax[b], m[b]);
      }
      __syncthreads();
#pragma unroll
      for (int b = 0; b < kBoards; ++b) {
        const unsigned mb = s_amax[b];
        const int be = (int)((mb >> 23) & 0xff), e = be == 0 ? 0 : be - 126;  // max < 2^e
        xsc[b] = ldexpf(1.0f, 15 - e);
      }
    }
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int v = tid + i * kThreads;
      if ((AZ_MX_EXP & 4) || v >= V) continue;
      const int pos = v / (C / 4), c4 = v % (C / 4);
      char* dst = lds_a + pos * G::APOS + c4 * 8;
      const f32x4 a = {val[i].x, val[i].y, val[i].z, val[i].w};
      if constexpr (G::MODE == AZ_CONV_FP16X2) {
        // the all-zero position (pos = kBoards * 64) takes board 0's scale: zeros either way
        const int bb = (pos >> 6) < kBoards ? (pos >> 6) : 0;
        const f32x4 as = a * xsc[bb];  // exact: a power of two
        const f16x4 hi = __builtin_convertvector(as, f16x4);
        const f16x4 lo = __builtin_convertvector(as - __builtin_convertvector(hi, f32x4), f16x4);
        *reinterpret_cast<f16x4*>(dst) = hi;
        *reinterpret_cast<f16x4*>(dst + C * 2) = lo;
      } else if constexpr (G::MODE == AZ_CONV_SPLIT3) {
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
  __syncthreads();

  // per A tile: this lane's output position and which of the 9 taps land on the board
  int pos0[G::TM], ok9[G::TM];
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi) {
    const int m = 32 * mi + r;
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

  const uint64_t clk0 = (AZ_MX_EXP & 16) ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t rt0 = (AZ_MX_EXP & 16) ? __builtin_amdgcn_s_memrealtime() : 0;
  f32x16 acc[G::TM];
  mx_kloop<G>(acc, lds_a, wq, wlane, pos0, ok9, h, b0f, b1f, b2f, b3f);
  if ((AZ_MX_EXP & 16) && blockIdx.x == 0 && tid == 0) {
    const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    reinterpret_cast<uint64_t*>(y)[0] = clk1 - clk0;
    reinterpret_cast<uint64_t*>(y)[1] = rt1 - rt0;
    return;
  }

  // ---- epilogue: D[row][col], col = lane&31, row = (k&3) + 8*(k>>2) + 4*(lane>>5); a
  // 32-row tile lies inside one board, so the tail-board test is uniform per tile
  const int co = col0 + r;
  const float bv = bias[co];
  // FP16X2: 2^-(sx + sw) per tile's board (exact), sw = the weights' scale from the header
  float osc[G::TM];
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi) osc[mi] = 1.0f;
  if constexpr (G::SCALED) {
    const int sw = reinterpret_cast<const int*>(wq + G::W_BYTES)[1];
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi) {
      const unsigned mb = s_amax[(32 * mi) >> 6];
      const int be = (int)((mb >> 23) & 0xff), e = be == 0 ? 0 : be - 126;
      osc[mi] = ldexpf(1.0f, -(15 - e) - sw);
    }
  }
  float rv[G::TM][16];
  if (RES && STEM == 2) {  // residual = stem(planes) at (row, co), k_conv_stem's fmaf chain
    float sw[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) sw[t] = st.w[t * C + co];
    const float sb = st.b[co];
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int m = 32 * mi + (k & 3) + 8 * (k >> 2) + 4 * h;
        const float* pl = s_plane[(m >> 6) < kBoards ? (m >> 6) : 0];
        const int py = (m >> 3) & 7, px = m & 7;
        float a = sb;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
          if ((unsigned)yy < 8u && (unsigned)xx < 8u)
            a = fmaf(pl[(yy + 1) * 10 + xx + 1], sw[t], a);
        }
        rv[mi][k] = fmaxf(a, 0.f);
      }
    }
  } else if (RES) {  // all residual loads in flight at once
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi) {
      const size_t o0 = ((size_t)b0 * 64 + 32 * mi + 4 * h) * C + co;
      const bool in = ((32 * mi) >> 6) < nb;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        rv[mi][k] = in ? res[o0 + (size_t)((k & 3) + 8 * (k >> 2)) * C] : 0.0f;
    }
  }
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi) {
    if (((32 * mi) >> 6) >= nb) continue;
    const size_t o0 = ((size_t)b0 * 64 + 32 * mi + 4 * h) * C + co;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      float v = (G::SCALED ? acc[mi][k] * osc[mi] : acc[mi][k]) + bv;
      if (RES) v += rv[mi][k];
      if (RELU) v = fmaxf(v, 0.0f);
      if (AZ_MX_EXP & 8) {
        if (v == 12345.f) y[o0] = v;
      } else {
        y[o0 + (size_t)((k & 3) + 8 * (k >> 2)) * C] = v;
      }
    }
  }
}

// FastOthelloNet's whole conv trunk in one launch (az_fast_trunk_gpu): stem -> residual block
// (conv1, conv2 + stem residual) -> conv_add, one board per workgroup, FP16X2.  The same
// arithmetic as the three az_conv3x3_mx_stem_gpu / az_conv3x3_mx_gpu launches (stem values,
// per-board max, split, main loop, epilogue), so the output is bit-identical; what goes is the
// two intermediate activations' HBM round trips and two launches: each conv's epilogue reduces
// its output's max over the workgroup and writes the next conv's fp16 hi / lo image straight
// into LDS from its registers; conv2's residual (the stem output) is recomputed in its
// epilogue, as the separate stem-fused conv does.
struct FastTrunkArgs {
  const float* planes;  // [n][64] canonical boards
  const float* stem_w;  // [9][C]
  const float* stem_b;  // [C]
  const char* wq[3];    // conv1, conv2, conv_add weights (az_conv3x3_mx_prep_gpu, FP16X2)
  const float* bias[3];
  float* y;             // NHWC [n][64][C]: conv_add's output
  int n_boards;
};

// four waves per SIMD: the register allocator fits the kernel into 128 VGPRs (accumulators
// included, ten dwords spilled outside the main loops) so eight one-board workgroups share a CU
// -- the LDS limit (8 x 18 KB) -- and a 2,048-board evaluation is one round of workgroups
// instead of 1.33 rounds at six per CU (three waves: 120 VGPRs + 32 AGPRs): evaluation 105.7 ->
// 97.7-98.4 us, configs[1] +2.6 % same box, same outputs (profiles/r06_c2_fast_trunk_waves_ab.json);
// 0 = the allocator's own choice (A/B builds)
#ifndef AZ_FT_WAVES
#define AZ_FT_WAVES 4
#endif
#if AZ_FT_WAVES > 0
#define AZ_FT_ATTR __attribute__((amdgpu_waves_per_eu(AZ_FT_WAVES)))
#else
#define AZ_FT_ATTR
#endif

template <class G>
__global__ __launch_bounds__(G::THREADS) AZ_FT_ATTR void k_fast_trunk(FastTrunkArgs a) {
  static_assert(G::BOARDS == 1 && G::SCALED, "one board per workgroup, FP16X2");
  constexpr int C = G::C, kThreads = G::THREADS;
  extern __shared__ float4 lds4[];
  __shared__ float s_plane[100];
  __shared__ unsigned s_amax[G::WAVES];
  char* lds_a = reinterpret_cast<char*>(lds4);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int col0 = wave * 32, co = col0 + r;
  const int b = blockIdx.x;
  const int wlane = (col0 + r) * 32 + h * 16;
  BFrag<G> b0f, b1f, b2f, b3f;
  mx_load_b<G>(b0f, a.wq[0], wlane, 0);
  mx_load_b<G>(b1f, a.wq[0], wlane, 1);
  mx_load_b<G>(b2f, a.wq[0], wlane, 2);

  // ---- conv1's input: stem(planes), staged as k_conv3x3_mx<STEM = 1> stages it
  for (int i = tid; i < 100; i += kThreads) {
    const int yy = i / 10 - 1, xx = i % 10 - 1;
    s_plane[i] = (unsigned)yy < 8u && (unsigned)xx < 8u ? a.planes[(size_t)b * 64 + yy * 8 + xx]
                                                        : 0.f;
  }
  if (tid < G::WAVES) s_amax[tid] = 0u;
  __syncthreads();
  int e_in;  // the current conv's input: max |x| < 2^e_in
  {
    constexpr int V = 65 * C / 4, ITER = (V + kThreads - 1) / kThreads;
    static_assert(kThreads % (C / 4) == 0, "one channel quad per thread");
    const int c = (tid % (C / 4)) * 4;
    float4 stw[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) stw[t] = *reinterpret_cast<const float4*>(a.stem_w + t * C + c);
    const float4 stb = *reinterpret_cast<const float4*>(a.stem_b + c);
    float4 val[ITER];
    unsigned m = 0u;
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int v = tid + i * kThreads;
      val[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (v < 64 * (C / 4)) val[i] = stem4(s_plane, v / (C / 4), stw, stb);
      m = max(m, max(max(__float_as_uint(fabsf(val[i].x)), __float_as_uint(fabsf(val[i].y))),
                     max(__float_as_uint(fabsf(val[i].z)), __float_as_uint(fabsf(val[i].w)))));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off, 64));
    if (lane == 0) s_amax[wave] = m;
    __syncthreads();
    unsigned mb = s_amax[0];
#pragma unroll
    for (int w = 1; w < G::WAVES; ++w) mb = max(mb, s_amax[w]);
    const int be = (int)((mb >> 23) & 0xff);
    e_in = be == 0 ? 0 : be - 126;
    const float xsc = ldexpf(1.0f, 15 - e_in);
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int v = tid + i * kThreads;
      if (v >= V) continue;
      char* dst = lds_a + (v / (C / 4)) * G::APOS + (v % (C / 4)) * 8;
      const f32x4 x4 = {val[i].x, val[i].y, val[i].z, val[i].w};
      const f32x4 as = x4 * xsc;
      const f16x4 hi = __builtin_convertvector(as, f16x4);
      const f16x4 lo = __builtin_convertvector(as - __builtin_convertvector(hi, f32x4), f16x4);
      *reinterpret_cast<f16x4*>(dst) = hi;
      *reinterpret_cast<f16x4*>(dst + C * 2) = lo;
    }
  }
  __syncthreads();

  int pos0[G::TM], ok9[G::TM];
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi) {
    const int m = 32 * mi + r;
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

  f32x16 acc[G::TM];
#pragma unroll  // three bodies (one rolled body needed 156 VGPRs)
  for (int layer = 0; layer < 3; ++layer) {
    const char* wq = a.wq[layer];
    mx_kloop<G>(acc, lds_a, wq, wlane, pos0, ok9, h, b0f, b1f, b2f, b3f);
    // epilogue (k_conv3x3_mx's): v = acc * 2^-(sx + sw) + bias (+ stem residual), ReLU
    const int sw = reinterpret_cast<const int*>(wq + G::W_BYTES)[1];
    const float osc = ldexpf(1.0f, -(15 - e_in) - sw);
    const float bv = a.bias[layer][co];
    f32x16(&v)[G::TM] = acc;  // the epilogue's values replace the accumulators in place
    if (layer == 1) {  // residual = stem(planes) at (row, co): k_conv3x3_mx<STEM = 2>'s chain
      // (recomputed: an fp32 copy in LDS would cost occupancy -- 4 workgroups per CU by LDS
      // instead of 6 by registers; A/B: profiles/r06_c2_fast_trunk_ab.json)
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int m = 32 * mi + (k & 3) + 8 * (k >> 2) + 4 * h;
          const int py = (m >> 3) & 7, px = m & 7;
          float rs = a.stem_b[co];
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
            if ((unsigned)yy < 8u && (unsigned)xx < 8u)
              rs = fmaf(s_plane[(yy + 1) * 10 + xx + 1], a.stem_w[t * C + co], rs);
          }
          float x = v[mi][k] * osc + bv;
          x += fmaxf(rs, 0.f);
          v[mi][k] = fmaxf(x, 0.0f);
        }
    } else {
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
        for (int k = 0; k < 16; ++k) v[mi][k] = fmaxf(v[mi][k] * osc + bv, 0.0f);
    }
    if (layer == 2) {  // conv_add's output: NHWC to global memory
      if (b < a.n_boards) {
#pragma unroll
        for (int mi = 0; mi < G::TM; ++mi) {
          const size_t o0 = ((size_t)b * 64 + 32 * mi + 4 * h) * C + co;
#pragma unroll
          for (int k = 0; k < 16; ++k) a.y[o0 + (size_t)((k & 3) + 8 * (k >> 2)) * C] = v[mi][k];
        }
      }
      break;
    }
    // the next conv's input image: the board's max over every wave's values (this barrier
    // also ends every wave's reads of the current image), then hi / lo words from registers
    unsigned m = 0u;
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
      for (int k = 0; k < 16; ++k) m = max(m, __float_as_uint(fabsf(v[mi][k])));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off, 64));
    __syncthreads();  // the previous image's maxima read, every wave's main loop done
    if (lane == 0) s_amax[wave] = m;
    __syncthreads();
    unsigned mb = s_amax[0];
#pragma unroll
    for (int w = 1; w < G::WAVES; ++w) mb = max(mb, s_amax[w]);
    const int be = (int)((mb >> 23) & 0xff);
    e_in = be == 0 ? 0 : be - 126;
    const float xsc = ldexpf(1.0f, 15 - e_in);
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int m = 32 * mi + (k & 3) + 8 * (k >> 2) + 4 * h;
        const float s = v[mi][k] * xsc;  // exact: a power of two
        const _Float16 hi = (_Float16)s;
        const _Float16 lo = (_Float16)(s - (float)hi);
        char* dst = lds_a + m * G::APOS + co * 2;
        *reinterpret_cast<_Float16*>(dst) = hi;
        *reinterpret_cast<_Float16*>(dst + C * 2) = lo;
      }
    // the next conv's first weight steps, in flight across the barrier
    mx_load_b<G>(b0f, a.wq[layer + 1], wlane, 0);
    mx_load_b<G>(b1f, a.wq[layer + 1], wlane, 1);
    mx_load_b<G>(b2f, a.wq[layer + 1], wlane, 2);
    __syncthreads();
  }
}

// w9 [9][Co][Ci] fp32 -> wq [9][Ci/16][PLANES][Co][16] 16-bit words.  FP16X2: w * 2^sw split
// into an fp16 pair; hdr = the 16-byte header after the words: [0] max |w| bits, [1] sw.
// With MAXPASS the kernel only reduces max |w| into hdr[0].
template <int MODE, bool MAXPASS = false>
__global__ void k_conv_mx_prep(const float* __restrict__ w9, uint16_t* __restrict__ wq, int C,
                               unsigned* hdr) {
  constexpr int P = MODE == AZ_CONV_SPLIT3 ? 3 : (MODE == AZ_CONV_FP16X2 ? 2 : 1);
  const int n = 9 * C * C;
  float wsc = 1.0f;
  if constexpr (MODE == AZ_CONV_FP16X2 && !MAXPASS) {
    const unsigned mb = hdr[0];  // max |w| < 2^e
    const int be = (int)((mb >> 23) & 0xff), e = be == 0 ? 0 : be - 126;
    wsc = ldexpf(1.0f, 15 - e);  // scaled max < 2^15
    if (blockIdx.x == 0 && threadIdx.x == 0) hdr[1] = (unsigned)(15 - e);
  }
  unsigned wmax = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int tap = i / (C * C), co = (i / C) % C, ci = i % C;
    const float v = w9[i];
    const size_t base = ((((size_t)tap * (C / 16) + ci / 16) * P) * C + co) * 16 + (ci & 15);
    const size_t pstride = (size_t)C * 16;
    if constexpr (MAXPASS) {
      wmax = max(wmax, __float_as_uint(fabsf(v)));
    } else if constexpr (MODE == AZ_CONV_FP16X2) {
      const float vs = v * wsc;  // exact: a power of two
      const _Float16 hi = (_Float16)vs;
      const _Float16 lo = (_Float16)(vs - (float)hi);
      wq[base] = __builtin_bit_cast(uint16_t, hi);
      wq[base + pstride] = __builtin_bit_cast(uint16_t, lo);
    } else if constexpr (MODE == AZ_CONV_SPLIT3) {
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
  if constexpr (MAXPASS) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wmax = max(wmax, (unsigned)__shfl_xor((int)wmax, off, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(hdr, wmax);
  }
}

template <class G, int STEM>
int launch_mx_t(const float* x, const void* wq, const float* bias, const float* res, float* y,
                int n_boards, int relu, StemArgs st, hipStream_t s) {
  const unsigned grid = (unsigned)((n_boards + G::BOARDS - 1) / G::BOARDS);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS needs the opt-in once per kernel
  if (!attr_set) {
    const void* ks[] = {(const void*)k_conv3x3_mx<G, true, true, STEM>,
                        (const void*)k_conv3x3_mx<G, true, false, STEM>,
                        (const void*)k_conv3x3_mx<G, false, true, STEM>,
                        (const void*)k_conv3x3_mx<G, false, false, STEM>};
    for (const void* k : ks)
      AZ_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)G::LDS_BYTES));
    attr_set = true;
  }
  const char* w = static_cast<const char*>(wq);
  const dim3 blk(G::THREADS);
  const size_t lds = G::LDS_BYTES;
  if (res && relu)
    hipLaunchKernelGGL((k_conv3x3_mx<G, true, true, STEM>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards, st);
  else if (res)
    hipLaunchKernelGGL((k_conv3x3_mx<G, true, false, STEM>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards, st);
  else if (relu)
    hipLaunchKernelGGL((k_conv3x3_mx<G, false, true, STEM>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards, st);
  else
    hipLaunchKernelGGL((k_conv3x3_mx<G, false, false, STEM>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards, st);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

template <class G>
int launch_mx(const float* x, const void* wq, const float* bias, const float* res, float* y,
              int n_boards, int relu, hipStream_t s, StemArgs st = StemArgs{}, int stem = 0) {
  if (stem == 1) return launch_mx_t<G, 1>(x, wq, bias, res, y, n_boards, relu, st, s);
  if (stem == 2) return launch_mx_t<G, 2>(x, wq, bias, res, y, n_boards, relu, st, s);
  return launch_mx_t<G, 0>(x, wq, bias, res, y, n_boards, relu, st, s);
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
    hipLaunchKernelGGL((k_conv_mx_prep<AZ_CONV_SPLIT3>), dim3(grid), dim3(256), 0, s, w9, out, channels, nullptr);
  else if (mode == AZ_CONV_FP16)
    hipLaunchKernelGGL((k_conv_mx_prep<AZ_CONV_FP16>), dim3(grid), dim3(256), 0, s, w9, out, channels, nullptr);
  else if (mode == AZ_CONV_FP16X2) {
    unsigned* hdr = reinterpret_cast<unsigned*>(out + (size_t)9 * channels * channels * 2);
    AZ_HIP(hipMemsetAsync(hdr, 0, 16, s));
    hipLaunchKernelGGL((k_conv_mx_prep<AZ_CONV_FP16X2, true>), dim3(grid), dim3(256), 0, s, w9, out, channels, hdr);
    hipLaunchKernelGGL((k_conv_mx_prep<AZ_CONV_FP16X2>), dim3(grid), dim3(256), 0, s, w9, out, channels, hdr);
  } else
    return azc::set_error(AZ_ERR_ARG, "az_conv3x3_mx_prep_gpu: unknown mode %d", mode);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

namespace {
int launch_mx_cfg(const float* x, const void* wq, const float* bias, const float* res, float* y,
                  int n_boards, int channels, int relu, int mode, int cfg, hipStream_t s,
                  StemArgs st = StemArgs{}, int stem = 0) {
  // cfg 0: 2 boards per workgroup (each weight fragment feeds 4 MFMAs); cfg 1: 1 board
  // (half the LDS, 2-3 workgroups per CU, 2 MFMAs per weight fragment)
  const bool two = cfg == 0;
#define AZ_MX_L(CC, MM)                                                                  \
  return two ? launch_mx<Mx<CC, MM, 2>>(x, wq, bias, res, y, n_boards, relu, s, st, stem) \
             : launch_mx<Mx<CC, MM, 1>>(x, wq, bias, res, y, n_boards, relu, s, st, stem);
  if (channels == 128 && mode == AZ_CONV_SPLIT3) AZ_MX_L(128, AZ_CONV_SPLIT3)
  if (channels == 64 && mode == AZ_CONV_SPLIT3) AZ_MX_L(64, AZ_CONV_SPLIT3)
  if (channels == 128 && mode == AZ_CONV_FP16) AZ_MX_L(128, AZ_CONV_FP16)
  if (channels == 64 && mode == AZ_CONV_FP16) AZ_MX_L(64, AZ_CONV_FP16)
  if (channels == 128 && mode == AZ_CONV_FP16X2) AZ_MX_L(128, AZ_CONV_FP16X2)
  if (channels == 64 && mode == AZ_CONV_FP16X2) AZ_MX_L(64, AZ_CONV_FP16X2)
#undef AZ_MX_L
  return azc::set_error(AZ_ERR_ARG, "az_conv3x3_mx_gpu: channels %d / mode %d unsupported",
                        channels, mode);
}
}  // namespace

extern "C" int64_t az_conv3x3_mx_prep_bytes(int32_t channels, int32_t mode) {
  const int planes = mode == AZ_CONV_SPLIT3 ? 3 : (mode == AZ_CONV_FP16X2 ? 2 : 1);
  return (int64_t)9 * channels * channels * planes * 2 + (mode == AZ_CONV_FP16X2 ? 16 : 0);
}

namespace {
// the default workgroup shape: 1 board (measured faster at every shape in split3,
// profiles/r01_conv_mx.jsonl); AZ_MX_CFG=0 (experiments): 2 boards per workgroup
int mx_default_cfg() {
  static const int cfg = [] {
    const char* e = getenv("AZ_MX_CFG");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return cfg;
}
}  // namespace

extern "C" int az_conv3x3_mx_gpu(const float* x, const void* wq, const float* bias,
                                 const float* res, float* y, int32_t n_boards,
                                 int32_t channels, int32_t relu, int32_t mode, void* stream) {
  return az_conv3x3_mx_cfg_gpu(x, wq, bias, res, y, n_boards, channels, relu, mode,
                               mx_default_cfg(), stream);
}

extern "C" int az_conv3x3_mx_cfg_gpu(const float* x, const void* wq, const float* bias,
                                     const float* res, float* y, int32_t n_boards,
                                     int32_t channels, int32_t relu, int32_t mode, int32_t cfg,
                                     void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_conv3x3_mx_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && wq && bias && y && x != y, AZ_ERR_ARG,
             "az_conv3x3_mx_gpu: null buffer or in-place call");
  AZ_REQUIRE(((uintptr_t)x | (uintptr_t)wq | (uintptr_t)bias) % 16 == 0, AZ_ERR_ARG,
             "az_conv3x3_mx_gpu: buffers must be 16-byte aligned");
  AZ_REQUIRE(cfg == 0 || cfg == 1, AZ_ERR_ARG, "az_conv3x3_mx_gpu: cfg %d", cfg);
  return launch_mx_cfg(x, wq, bias, res, y, n_boards, channels, relu, mode, cfg,
                       azc::as_stream(stream));
}

extern "C" int az_conv3x3_mx_stem_gpu(const float* planes, const float* stem_w,
                                      const float* stem_b, const float* x, const void* wq,
                                      const float* bias, float* y, int32_t n_boards,
                                      int32_t channels, int32_t role, int32_t mode,
                                      void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_conv3x3_mx_stem_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(role == 1 || role == 2, AZ_ERR_ARG, "az_conv3x3_mx_stem_gpu: role %d", role);
  AZ_REQUIRE(planes && stem_w && stem_b && wq && bias && y && (role == 1 || (x && x != y)),
             AZ_ERR_ARG, "az_conv3x3_mx_stem_gpu: null buffer or in-place call");
  AZ_REQUIRE(((uintptr_t)stem_w | (uintptr_t)stem_b | (uintptr_t)wq | (uintptr_t)bias |
              (uintptr_t)(role == 2 ? x : nullptr)) % 16 == 0,
             AZ_ERR_ARG, "az_conv3x3_mx_stem_gpu: buffers must be 16-byte aligned");
  AZ_REQUIRE(channels == 64 || channels == 128, AZ_ERR_ARG,
             "az_conv3x3_mx_stem_gpu: channels must be 64 or 128");
  const StemArgs st{planes, stem_w, stem_b};
  // role 1: input = stem(planes), no residual; role 2: residual = stem(planes) (res is a
  // non-null placeholder that selects the residual epilogue; it is not read)
  return launch_mx_cfg(role == 1 ? stem_b : x, wq, bias, role == 2 ? stem_b : nullptr, y,
                       n_boards, channels, 1, mode, mx_default_cfg(), azc::as_stream(stream), st,
                       role);
}

extern "C" int az_fast_trunk_gpu(const float* planes, const float* stem_w, const float* stem_b,
                                 const void* wq1, const float* bias1, const void* wq2,
                                 const float* bias2, const void* wq3, const float* bias3,
                                 float* y, int32_t n_boards, int32_t channels, int32_t mode,
                                 void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_fast_trunk_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(channels == 64 && mode == AZ_CONV_FP16X2, AZ_ERR_ARG,
             "az_fast_trunk_gpu: 64 channels in FP16X2 only (got %d / mode %d)", channels, mode);
  AZ_REQUIRE(planes && stem_w && stem_b && wq1 && bias1 && wq2 && bias2 && wq3 && bias3 && y,
             AZ_ERR_ARG, "az_fast_trunk_gpu: null buffer");
  AZ_REQUIRE(((uintptr_t)stem_w | (uintptr_t)stem_b | (uintptr_t)wq1 | (uintptr_t)wq2 |
              (uintptr_t)wq3) % 16 == 0,
             AZ_ERR_ARG, "az_fast_trunk_gpu: buffers must be 16-byte aligned");
  using G = Mx<64, AZ_CONV_FP16X2, 1>;
  const FastTrunkArgs a{planes, stem_w, stem_b,
                        {static_cast<const char*>(wq1), static_cast<const char*>(wq2),
                         static_cast<const char*>(wq3)},
                        {bias1, bias2, bias3}, y, n_boards};
  hipLaunchKernelGGL(k_fast_trunk<G>, dim3((unsigned)n_boards), dim3(G::THREADS), G::LDS_BYTES,
                     azc::as_stream(stream), a);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
