// conv_wino.hip — the residual trunk's 3x3 convolution as Winograd F(2x2, 3x3) on the
// 16-bit MFMA pipe, epilogue fused.
//
// Same op and numerics modes as conv16.hip (conv + bias (+ residual) + ReLU, NHWC fp32,
// Ci = Co = C; AZ_CONV_SPLIT3 = fp32 operands as three bf16 words and six partial
// products, fp32-accurate; AZ_CONV_FP16 = one fp16 product), with 2.25x fewer products:
// an 8x8 board is 16 tiles of 2x2 outputs, each read through a 4x4 input window d, and
//     Y = A^T [ sum_ci (G g G^T) (.) (B^T d B) ] A        (Lavin & Gray's F(2x2, 3x3))
// with B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], G = [1 0 0; .5 .5 .5; .5 -.5 .5;
// 0 0 1], A^T = [1 1 1 0; 0 1 -1 -1].  The transforms only add and subtract (B, A) or
// are applied to the weights once in fp64 (G), so the error stays at the direct fp32
// kernel's level (tests/test_nn_gpu.py holds it to the same bar as the direct kernel).
//
// GEMM view: 16 independent GEMMs, one per transform point xi = (k, l):
//     M_xi[tile][co] = sum_ci V_xi[tile][ci] U_xi[ci][co]
// Workgroup = 2 boards (32 tiles = one 32-row MFMA tile) x all C columns, wave w owning
// columns 32w..32w+31 and one fp32 accumulator per point (16 x 16 registers per lane),
// so the output transform and the epilogue run straight from registers.
//   * K loop over 16-channel chunks.  The input transform of chunk c+1 (4x4 windows
//     loaded from HBM/L2 one chunk ahead, rows of B^T d formed at the chunk start, one
//     column combination + bf16x3 split + LDS store per point) is interleaved with chunk
//     c's MFMAs and lands in the other half of a double-buffered LDS image
//     [point][plane][tile][16 ch] (1 KiB per point and plane: conflict-free b128 reads).
//   * U: weights transformed and split once by az_conv3x3_wino_prep_gpu into
//     [chunk][point][plane][Co][16] words; every wave streams its own 32 columns from L2
//     three (chunk, point) steps ahead, as in conv16.hip.
//   * One LDS barrier per chunk (lgkmcnt only: the weight stream stays in flight).
#include <type_traits>

#include "common.h"

// experiment hooks (scripts/exp/wino_exp.py builds copies with bits set): 1 = no A reads in
// the main loop, 2 = no weight loads in the main loop, 4 = no window loads / transform in
// the main loop, 8 = no epilogue stores, 16 = workgroup 0 stamps s_memtime/s_memrealtime
// around its main loop into y[0..3], 32 = no LDS barrier in the main loop, 64 = no
// residual loads.  Product: 0.
#ifndef AZ_WN_EXP
#define AZ_WN_EXP 0
#endif

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

template <int C_, int MODE_>
struct Wn {
  static constexpr int C = C_, MODE = MODE_;
  static constexpr int PLANES = MODE == AZ_CONV_SPLIT3 ? 3 : 1;
  static constexpr int CB = C / 32;                  // 32-column blocks
  static constexpr int WAVES = 2 * CB, THREADS = 64 * WAVES;
  static constexpr int HALF = THREADS / 2;           // threads of one point half
  static constexpr int CHUNKS = C / 16;
  static constexpr int TPT = 256 / HALF;             // transform items per thread
  static constexpr int SLAB = 32 * 32;               // one (point, plane): 32 tiles x 16 ch x 2 B
  static constexpr int BUF = 16 * PLANES * SLAB;
  static constexpr size_t XCH_BYTES = (size_t)CB * 2 * 4 * 2 * 64 * 8;  // epilogue exchange
  static constexpr size_t LDS_BYTES = 2 * BUF > XCH_BYTES ? 2 * BUF : XCH_BYTES;
  static constexpr int STEP_BYTES = PLANES * C * 32; // weight bytes per (chunk, point)
  static constexpr int QSTEPS = CHUNKS * 8;          // steps of one wave (8 points per chunk)
  static_assert(TPT >= 1 && 256 % HALF == 0, "C must be 64 or 128");
};

template <class G>
using Word8 = typename std::conditional<G::MODE == AZ_CONV_SPLIT3, bf16x8, f16x8>::type;

template <class G>
struct Frag {
  Word8<G> v[G::PLANES];
};

// the LDS-only barrier: this wave's LDS stores are complete, then every wave arrives; the
// weight and input loads in flight are not waited for
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// one accumulator element into a VGPR where the epilogue needs it (the compiler would copy
// all 256 accumulator registers out at the loop exit at once, and spill)
__device__ __forceinline__ float acc_read(float a) {
  float v;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(a));
  return v;
}

template <class G>
__device__ __forceinline__ void wn_read_a(Frag<G>& f, const char* buf, int xi, int lane_off) {
#pragma unroll
  for (int pl = 0; pl < G::PLANES; ++pl)
    f.v[pl] = *reinterpret_cast<const Word8<G>*>(buf + (xi * G::PLANES + pl) * G::SLAB + lane_off);
}

template <class G>
__device__ __forceinline__ void wn_load_b(Frag<G>& f, const char* wq, int lane_off, int s) {
  const char* step = wq + (size_t)s * G::STEP_BYTES;
#pragma unroll
  for (int pl = 0; pl < G::PLANES; ++pl)
    f.v[pl] = *reinterpret_cast<const Word8<G>*>(step + lane_off + pl * G::C * 32);
}

template <class G>
__device__ __forceinline__ void wn_mma(f32x16& acc, const Frag<G>& a, const Frag<G>& b) {
  if constexpr (G::MODE == AZ_CONV_SPLIT3) {
    // smallest partial products first (x2y0, x1y1, x0y2, x1y0, x0y1, x0y0)
    constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
    for (int t = 0; t < 6; ++t)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[PA[t]], b.v[PB[t]], acc, 0, 0, 0);
  } else {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[0], b.v[0], acc, 0, 0, 0);
  }
}

// window entries e0 .. e0+NE-1 (of the 12 = rows rbase..rbase+2 this thread's point half
// needs) of this thread's 4x4 input windows (2 channels each) of chunk c; off = element
// offset of window row rbase, column 0, channel 0 of the chunk; msk bit a*4+b = entry (a, b)
// on the board.  Off-board entries read element 0 (a valid address; wn_rows zeroes them, so
// nothing waits for the loads here): every load is issued, with a uniform base and a 32-bit
// lane offset.
template <class G, int NE>
__device__ __forceinline__ void wn_load_raw(f32x2 (&d)[G::TPT][12], const float* x,
                                            const int (&off)[G::TPT], const int (&msk)[G::TPT],
                                            int c, int e0) {
#pragma unroll
  for (int u = 0; u < G::TPT; ++u)
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = e0 + i;
      const bool in = (msk[u] >> e) & 1;
      const uint32_t o = in ? (uint32_t)(off[u] + ((e >> 2) * 8 + (e & 3)) * G::C + c * 16) : 0u;
      d[u][e] = *reinterpret_cast<const f32x2*>(reinterpret_cast<const char*>(x) + o * 4u);
    }
}

// the two rows of B^T d this point half needs (window rows D0..D2 = rows ph..ph+2):
// half 0: rows 0, 1 = D0 - D2, D1 + D2; half 1: rows 2, 3 = D1 - D0, D0 - D2.  Off-board
// window entries count as zeros.
template <class G>
__device__ __forceinline__ void wn_rows(f32x2 (&r)[G::TPT][8], const f32x2 (&raw)[G::TPT][12],
                                        const int (&msk)[G::TPT], int ph) {
#pragma unroll
  for (int u = 0; u < G::TPT; ++u) {
    f32x2 d[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) d[e] = (msk[u] >> e) & 1 ? raw[u][e] : f32x2{0.0f, 0.0f};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (ph == 0) {
        r[u][b] = d[b] - d[8 + b];
        r[u][4 + b] = d[4 + b] + d[8 + b];
      } else {
        r[u][b] = d[4 + b] - d[b];
        r[u][4 + b] = d[b] - d[8 + b];
      }
    }
  }
}

// V at point (k, l) = row k of B^T d times B: column combination l
__device__ __forceinline__ f32x2 wn_point(const f32x2* rk, int l) {
  switch (l) {
    case 0: return rk[0] - rk[2];
    case 1: return rk[1] + rk[2];
    case 2: return rk[2] - rk[1];
    default: return rk[1] - rk[3];
  }
}

// split two transformed values into PLANES 16-bit words and store them in the point's slabs
template <class G>
__device__ __forceinline__ void wn_put(char* slab, f32x2 v) {
  if constexpr (G::MODE == AZ_CONV_SPLIT3) {
    const bf16x2 x0 = __builtin_convertvector(v, bf16x2);
    const f32x2 r1 = v - __builtin_convertvector(x0, f32x2);
    const bf16x2 x1 = __builtin_convertvector(r1, bf16x2);
    const bf16x2 x2 = __builtin_convertvector(r1 - __builtin_convertvector(x1, f32x2), bf16x2);
    *reinterpret_cast<bf16x2*>(slab) = x0;
    *reinterpret_cast<bf16x2*>(slab + G::SLAB) = x1;
    *reinterpret_cast<bf16x2*>(slab + 2 * G::SLAB) = x2;
  } else {
    *reinterpret_cast<f16x2*>(slab) = __builtin_convertvector(v, f16x2);
  }
}

// issue pattern of one (chunk, point) step: the A reads and the transform's VALU work and
// LDS stores in the shadow of the MFMAs, the weight loads behind them; nothing crosses a
// step (otherwise the scheduler hoists every step's loads and spills)
template <class G, int RAW>
__device__ __forceinline__ void wn_sched() {
  constexpr int kMfma = G::MODE == AZ_CONV_SPLIT3 ? 6 : 1;
  constexpr int kDs = G::PLANES;
#pragma unroll
  for (int i = 0; i < kDs; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, kMfma / kDs > 0 ? kMfma / kDs : 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                               // DS read
    __builtin_amdgcn_sched_group_barrier(0x002, 4 * G::TPT, 0);                      // VALU
    __builtin_amdgcn_sched_group_barrier(0x200, G::TPT, 0);                          // DS write
  }
  __builtin_amdgcn_sched_group_barrier(0x008, kMfma, 0);
  __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
  __builtin_amdgcn_sched_group_barrier(0x020, G::PLANES + RAW, 0);  // VMEM read
  __builtin_amdgcn_sched_barrier(0);
}

// One conv layer for board pair `pair` (boards 2*pair, 2*pair+1) by the whole workgroup;
// `lds` = G::LDS_BYTES of LDS.  Ends with a workgroup barrier: its outputs are visible to
// the workgroup and its LDS is free again.
template <class G, bool RES, bool RELU>
__device__ __forceinline__ void wino_pair(const float* __restrict__ x, const char* __restrict__ wq,
                                          const float* __restrict__ bias,
                                          const float* res, float* y,  // may alias (in place)
                                          int n_boards, int pair, char* lds) {
  constexpr int C = G::C, TPT = G::TPT;
  const uint64_t rt_entry = (AZ_WN_EXP & 16) ? __builtin_amdgcn_s_memrealtime() : 0;
  // laundered: nothing lane-dependent is hoisted out of a caller's layer loop (it would sit
  // in registers across every layer and spill)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  // wave = (point half ph, column block cb): points 8ph..8ph+7, columns 32cb..32cb+31.
  // Two waves per SIMD, so one's waits run under the other's MFMAs.
  const int ph = __builtin_amdgcn_readfirstlane(wave / G::CB);
  const int cb = __builtin_amdgcn_readfirstlane(wave % G::CB);
  const int col0 = cb * 32;
  const int b0 = pair * 2;
  const int nb = n_boards - b0 < 2 ? n_boards - b0 : 2;
  constexpr int qlast = G::QSTEPS - 1;
  constexpr int kRing = 4, kPd = 3;  // weight ring and prefetch distance (steps)
  static_assert(8 % kRing == 0 && kPd < kRing, "ring slot of a step = point % kRing");

  // weight step of this wave's q-th step (chunk q/8, point 8ph + q%8)
  const int wlane = (col0 + r) * 32 + h * 16;
  const char* wq_h = wq + (size_t)(8 * ph) * G::STEP_BYTES;
  Frag<G> bf[kRing];

  // transform role: item = (tile T, channel pair) with T = (ht >> 3) + u * HALF/8 (board
  // T>>4, tile row (T>>2)&3, tile column T&3), pair 2*(ht&7) of each chunk, ht = the
  // thread's index within its point half; window rows ph..ph+2
  const int ht = tid % G::HALF;
  int off[TPT], msk[TPT], slab_off[TPT];
#pragma unroll
  for (int u = 0; u < TPT; ++u) {
    const int T = (ht >> 3) + u * (G::HALF / 8);
    const int bd = T >> 4, ty = (T >> 2) & 3, tx = T & 3;
    int m = 0;
#pragma unroll
    for (int e = 0; e < 12; ++e) {
      const int yy = 2 * ty - 1 + ph + (e >> 2), xx = 2 * tx - 1 + (e & 3);
      m |= (bd < nb && (unsigned)yy < 8u && (unsigned)xx < 8u) << e;
    }
    msk[u] = m;
    off[u] = ((b0 + bd) * 64 + (2 * ty - 1 + ph) * 8 + (2 * tx - 1)) * C + 2 * (ht & 7);
    slab_off[u] = (8 * ph) * G::PLANES * G::SLAB + T * 32 + (ht & 7) * 4;
  }

  f32x2 raw[TPT][12], rw[TPT][8];
  // ---- prologue: the windows of chunks 0 and 1 and the first kPd weight steps requested
  // together (one round trip), chunk 0 transformed into buffer 0 (the loop's vmcnt
  // bookkeeping sees the same order on entry as around its back-edge: windows before
  // weights)
  {
    f32x2 raw0[TPT][12];
    wn_load_raw<G, 12>(raw0, x, off, msk, 0, 0);
    wn_load_raw<G, 12>(raw, x, off, msk, G::CHUNKS > 1 ? 1 : 0, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kPd; ++i) wn_load_b<G>(bf[i], wq_h, wlane, (i >> 3) * 16 + (i & 7));
    __builtin_amdgcn_sched_barrier(0);
    wn_rows<G>(rw, raw0, msk, ph);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int u = 0; u < TPT; ++u)
      wn_put<G>(lds + j * G::PLANES * G::SLAB + slab_off[u], wn_point(&rw[u][(j >> 2) * 4], j & 3));
  lds_barrier();

  f32x16 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[j][k] = 0.0f;

  // Step (c, j): MFMAs of point 8ph+j on A set j%2 and B set j%kRing; the next point's A
  // read meanwhile, B of step +kPd requested (clamped to the last step, so every load is
  // issued and vmcnt counts stay exact), window entries of chunk c+2 requested in the first
  // 6 steps (vmcnt is in order: a step's weight wait also waits for the windows requested
  // before it), and point 8ph+j of chunk c+1 transformed into the other buffer.
  const int aoff = (8 * ph) * G::PLANES * G::SLAB + r * 32 + h * 16;
  const uint64_t clk0 = (AZ_WN_EXP & 16) ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t rt0 = (AZ_WN_EXP & 16) ? __builtin_amdgcn_s_memrealtime() : 0;
  Frag<G> af[2];
  wn_read_a<G>(af[0], lds + aoff, 0, 0);
  for (int c = 0; c < G::CHUNKS; ++c) {
    const char* cur = lds + (c & 1) * G::BUF + aoff;
    char* nxt = lds + ((c + 1) & 1) * G::BUF;
    // chunk c+1's windows (requested during chunk c-1) -> rows.  The last chunk transforms
    // a clamped duplicate into the idle buffer (uniform body).
    wn_rows<G>(rw, raw, msk, ph);
    const int craw = c + 2 < G::CHUNKS ? c + 2 : G::CHUNKS - 1;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < 7 && !(AZ_WN_EXP & 1)) wn_read_a<G>(af[(j + 1) & 1], cur, j + 1, 0);
      wn_mma<G>(acc[j], af[j & 1], bf[j % kRing]);
      const int q = c * 8 + j + kPd;
      const int qc = q < qlast ? q : qlast;
      if (!(AZ_WN_EXP & 2)) wn_load_b<G>(bf[(j + kPd) % kRing], wq_h, wlane, (qc >> 3) * 16 + (qc & 7));
      if (j < 6 && !(AZ_WN_EXP & 4)) wn_load_raw<G, 2>(raw, x, off, msk, craw, 2 * j);
      if (!(AZ_WN_EXP & 4)) {
#pragma unroll
        for (int u = 0; u < TPT; ++u)
          wn_put<G>(nxt + j * G::PLANES * G::SLAB + slab_off[u],
                    wn_point(&rw[u][(j >> 2) * 4], j & 3));
      }
      if (j < 6) wn_sched<G, 2 * TPT>();
      else wn_sched<G, 0>();
    }
    if (!(AZ_WN_EXP & 32)) lds_barrier();
    wn_read_a<G>(af[0], lds + ((c + 1) & 1) * G::BUF + aoff, 0, 0);
  }
  uint64_t rt1 = 0;
  if (AZ_WN_EXP & 16) {
    rt1 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0 && tid == 0) {
      reinterpret_cast<uint64_t*>(y)[0] = __builtin_amdgcn_s_memtime() - clk0;
      reinterpret_cast<uint64_t*>(y)[1] = rt1 - rt0;
    }
  }

  // ---- output transform Y = A^T M A and epilogue, per accumulator element k: row (= tile)
  // (k&3) + 8*(k>>2) + 4*h, column co = col0 + r.  Each half forms the four outputs' partial
  // sums over its 8 points (rows k of A^T M: half 0 holds M rows 0,1, half 1 rows 2,3),
  // hands the two outputs the other half finishes through LDS, and finishes its own two:
  // half 0 the tile's top outputs (2ty, 2tx + j), half 1 the bottom ones.
  // Elements k and k+1 (adjacent tile rows of one board) travel together as f32x2, so the
  // transform and epilogue arithmetic issues as packed VALU (no MFMAs to share issue with
  // here) and the exchange as 8-byte LDS accesses.
  // Two rounds of 4 element pairs bound the registers (residuals, own partials).
  const int co = col0 + r;
  const float bv = bias[co];
  const f32x2 bv2 = {bv, bv};
  f32x2* xch = reinterpret_cast<f32x2*>(lds);  // [cb][dest half][k/2 of the round][2][64]
  constexpr int kR = 4;                         // element pairs per round
#pragma unroll
  for (int r0 = 0; r0 < 8; r0 += kR) {
    f32x2 rv[kR][2];
    if (RES) {  // the round's residual loads in flight before its transform arithmetic
#pragma unroll
      for (int i = 0; i < 2 * kR; ++i) {
        const int k = 2 * r0 + i;
        const int T = (k & 3) + 8 * (k >> 2) + 4 * h;
        const int bd = T >> 4, ty = (T >> 2) & 3, tx = T & 3;
        const bool in = bd < nb && !(AZ_WN_EXP & 64);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int pos = (2 * ty + ph) * 8 + 2 * tx + q;
          rv[i >> 1][q][i & 1] = in ? res[((size_t)(b0 + bd) * 64 + pos) * C + co] : 0.0f;
        }
      }
    }
    f32x2 own[kR][2];
    // every wave is done reading the last A buffer (round 0) / the previous round's exchange
    lds_barrier();
#pragma unroll
    for (int i = 0; i < kR; ++i) {
      const int kp = r0 + i;
      f32x2 m[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        m[j] = f32x2{acc_read(acc[j][2 * kp]), acc_read(acc[j][2 * kp + 1])};
      // t0[l] = (A^T M)[0][l] partial, t1[l] = (A^T M)[1][l] partial
      f32x2 t0[4], t1[4];
      if (ph == 0) {
#pragma unroll
        for (int l = 0; l < 4; ++l) {
          t0[l] = m[l] + m[4 + l];
          t1[l] = m[4 + l];
        }
      } else {
#pragma unroll
        for (int l = 0; l < 4; ++l) {
          t0[l] = m[l];
          t1[l] = -m[l] - m[4 + l];
        }
      }
      const f32x2 o0 = t0[0] + t0[1] + t0[2], o1 = t0[1] - t0[2] - t0[3];
      const f32x2 o2 = t1[0] + t1[1] + t1[2], o3 = t1[1] - t1[2] - t1[3];
      f32x2* dst = xch + (((cb * 2 + (1 - ph)) * kR + i) * 2) * 64 + lane;
      if (ph == 0) {
        dst[0] = o2;
        dst[64] = o3;
        own[i][0] = o0;
        own[i][1] = o1;
      } else {
        dst[0] = o0;
        dst[64] = o1;
        own[i][0] = o2;
        own[i][1] = o3;
      }
      __builtin_amdgcn_sched_barrier(0);  // two elements' accumulators in VGPRs at a time
    }
    lds_barrier();
    const f32x2* src = xch + ((cb * 2 + ph) * kR) * 2 * 64 + lane;
#pragma unroll
    for (int i = 0; i < kR; ++i) {
      const int k0 = 2 * (r0 + i);
      const int T0 = (k0 & 3) + 8 * (k0 >> 2) + 4 * h;  // tiles T0, T0 + 1: one board, one row
      const int bd = T0 >> 4, ty = (T0 >> 2) & 3, tx = T0 & 3;
      if (bd >= nb) continue;  // uniform per k pair
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        f32x2 v = own[i][q] + src[(i * 2 + q) * 64] + bv2;
        if (RES) v += rv[i][q];
        if (RELU) v = __builtin_elementwise_max(v, f32x2{0.0f, 0.0f});
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int pos = (2 * ty + ph) * 8 + 2 * (tx + e) + q;
          if (AZ_WN_EXP & 8) {
            if (v[e] == 12345.f) y[0] = v[e];
          } else {
            y[((size_t)(b0 + bd) * 64 + pos) * C + co] = v[e];
          }
        }
      }
    }
  }
  if ((AZ_WN_EXP & 16) && tid == 0) {  // per-workgroup timeline (entry, loop start/end, end)
    uint64_t* t = reinterpret_cast<uint64_t*>(y) + 4 + 4 * pair;
    t[0] = rt_entry;
    t[1] = rt0;
    t[2] = rt1;
    t[3] = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
}

template <class G, bool RES, bool RELU>
__global__ __launch_bounds__(G::THREADS) void k_conv3x3_wino(const float* __restrict__ x,
                                                             const char* __restrict__ wq,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ res,
                                                             float* __restrict__ y,
                                                             int n_boards) {
  extern __shared__ float4 lds4[];
  wino_pair<G, RES, RELU>(x, wq, bias, res, y, n_boards, blockIdx.x, reinterpret_cast<char*>(lds4));
}

// The whole residual trunk in one launch: stem (1 -> C 3x3 conv + bias + ReLU, k_conv_stem's
// fmaf chain) then n_blocks residual blocks (conv + ReLU, conv + residual + ReLU), every
// layer by the same code as k_conv3x3_wino, so the result is bit-identical to the
// layer-by-layer launches.  A convolution only mixes positions within a board, so each
// workgroup carries its board pairs through every layer without a grid-wide barrier: no
// launch gaps, and each layer reads its input from this CU's recent writes (L2) instead of
// a previous kernel's.  Workgroups walk pairs blockIdx.x, +gridDim.x, ...
struct TrunkArgs {
  const float* planes;        // [n][64] canonical boards
  const float* stem_w;        // [9][C]
  const float* stem_b;        // [C]
  const char* const* wq;      // [2 * n_blocks] per-conv Winograd weights (prep layout)
  const float* const* bias;   // [2 * n_blocks]
  float* h;                   // [n][64][C]: the stem output, then each block's output
  float* t;                   // [n][64][C]: each block's first conv output
  int n_boards, n_blocks;
};

template <class G>
__global__ __launch_bounds__(G::THREADS) void k_trunk_wino(TrunkArgs a) {
  constexpr int C = G::C;
  extern __shared__ float4 lds4[];
  char* lds = reinterpret_cast<char*>(lds4);
  const int npairs = (a.n_boards + 1) / 2;
  for (int p = blockIdx.x; p < npairs; p += gridDim.x) {
    // stem of the pair's boards (float4 of channels per item, k_conv_stem's tap order)
    const int nb = a.n_boards - 2 * p < 2 ? a.n_boards - 2 * p : 2;
    for (int i = threadIdx.x; i < nb * 64 * (C / 4); i += G::THREADS) {
      const int pos = i / (C / 4), co = (i % (C / 4)) * 4;
      const int b = 2 * p + (pos >> 6), q = pos & 63, py = q >> 3, px = q & 7;
      const float* in = a.planes + (size_t)b * 64;
      float4 acc = *reinterpret_cast<const float4*>(a.stem_b + co);
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const int yy = py + tp / 3 - 1, xx = px + tp % 3 - 1;
        if ((unsigned)yy < 8u && (unsigned)xx < 8u) {
          const float v = in[yy * 8 + xx];
          const float4 wv = *reinterpret_cast<const float4*>(a.stem_w + tp * C + co);
          acc.x = fmaf(v, wv.x, acc.x);
          acc.y = fmaf(v, wv.y, acc.y);
          acc.z = fmaf(v, wv.z, acc.z);
          acc.w = fmaf(v, wv.w, acc.w);
        }
      }
      acc.x = fmaxf(acc.x, 0.f);
      acc.y = fmaxf(acc.y, 0.f);
      acc.z = fmaxf(acc.z, 0.f);
      acc.w = fmaxf(acc.w, 0.f);
      reinterpret_cast<float4*>(a.h + ((size_t)b * 64 + q) * C)[co / 4] = acc;
    }
    __syncthreads();
    for (int blk = 0; blk < a.n_blocks; ++blk) {
      wino_pair<G, false, true>(a.h, a.wq[2 * blk], a.bias[2 * blk], nullptr, a.t, a.n_boards, p,
                                lds);
      // in place: each output element's residual is read by the lane that then writes it
      wino_pair<G, true, true>(a.t, a.wq[2 * blk + 1], a.bias[2 * blk + 1], a.h, a.h,
                               a.n_boards, p, lds);
    }
  }
}

// w9 [9][Co][Ci] fp32 -> U = G g G^T (fp64, rounded once to fp32) -> wq
// [Ci/16][16 points][PLANES][Co][16] 16-bit words.  FP16X2: U * 2^su split into an fp16
// pair; hdr = the 16-byte header after the words: [0] max |U| bits (k_wino_umax), [1] su.
// With MAXPASS the kernel only reduces max |U| into hdr[0].
template <int MODE, bool MAXPASS = false>
__global__ void k_wino_prep(const float* __restrict__ w9, uint16_t* __restrict__ wq, int C,
                            unsigned* hdr) {
  constexpr int P = MODE == AZ_CONV_SPLIT3 ? 3 : (MODE == AZ_CONV_FP16X2 ? 2 : 1);
  const int n = C * C;
  float usc = 1.0f;
  if constexpr (MODE == AZ_CONV_FP16X2 && !MAXPASS) {
    const unsigned mb = hdr[0];  // max |U| bits: max |U| < 2^e (frexp's exponent)
    const int be = (int)((mb >> 23) & 0xff), e = be == 0 ? 0 : be - 126;
    usc = ldexpf(1.0f, 15 - e);           // scaled max < 2^15 (fp16 max 65504)
    if (blockIdx.x == 0 && threadIdx.x == 0) hdr[1] = (unsigned)(15 - e);
  }
  unsigned umax = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int co = i / C, ci = i % C;
    double g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = (double)w9[(size_t)t * n + i];
    double gg[4][3];  // G g
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      gg[0][j] = g[0][j];
      gg[1][j] = 0.5 * (g[0][j] + g[1][j] + g[2][j]);
      gg[2][j] = 0.5 * (g[0][j] - g[1][j] + g[2][j]);
      gg[3][j] = g[2][j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double u4[4] = {gg[k][0], 0.5 * (gg[k][0] + gg[k][1] + gg[k][2]),
                            0.5 * (gg[k][0] - gg[k][1] + gg[k][2]), gg[k][2]};
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        const float v = (float)u4[l];
        const int xi = k * 4 + l;
        const size_t base = ((((size_t)(ci / 16) * 16 + xi) * P) * C + co) * 16 + (ci & 15);
        const size_t pstride = (size_t)C * 16;
        if constexpr (MAXPASS) {
          umax = max(umax, __float_as_uint(fabsf(v)));
        } else if constexpr (MODE == AZ_CONV_FP16X2) {
          const float vs = v * usc;  // exact: a power of two
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
    }
  }
  if constexpr (MAXPASS) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) umax = max(umax, (unsigned)__shfl_xor((int)umax, off, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(hdr, umax);
  }
}

template <class G>
int launch_wino(const float* x, const void* wq, const float* bias, const float* res, float* y,
                int n_boards, int relu, hipStream_t s) {
  const unsigned grid = (unsigned)((n_boards + 1) / 2);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS needs the opt-in once per kernel
  if (!attr_set) {
    const void* ks[] = {(const void*)k_conv3x3_wino<G, true, true>,
                        (const void*)k_conv3x3_wino<G, true, false>,
                        (const void*)k_conv3x3_wino<G, false, true>,
                        (const void*)k_conv3x3_wino<G, false, false>};
    for (const void* k : ks)
      AZ_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)G::LDS_BYTES));
    attr_set = true;
  }
  const char* w = static_cast<const char*>(wq);
  const dim3 blk(G::THREADS);
  const size_t lds = G::LDS_BYTES;
  if (res && relu)
    hipLaunchKernelGGL((k_conv3x3_wino<G, true, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else if (res)
    hipLaunchKernelGGL((k_conv3x3_wino<G, true, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else if (relu)
    hipLaunchKernelGGL((k_conv3x3_wino<G, false, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else
    hipLaunchKernelGGL((k_conv3x3_wino<G, false, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

}  // namespace

namespace {
template <class G>
int launch_trunk(const TrunkArgs& a, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    AZ_HIP(hipFuncSetAttribute((const void*)k_trunk_wino<G>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS_BYTES));
    attr_set = true;
  }
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    AZ_HIP(hipGetDevice(&dev));
    AZ_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    if (n_cu <= 0) n_cu = 256;
  }
  const int pairs = (a.n_boards + 1) / 2;
  // one workgroup per CU (its LDS and registers allow no second), pairs dealt round robin
  const unsigned grid = (unsigned)(pairs < n_cu ? pairs : n_cu);
  hipLaunchKernelGGL(k_trunk_wino<G>, dim3(grid), dim3(G::THREADS), G::LDS_BYTES, s, a);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
}  // namespace

extern "C" int az_trunk_wino_gpu(const float* planes, const float* stem_w, const float* stem_b,
                                 const void* const* wq, const float* const* bias, float* h,
                                 float* t, int32_t n_boards, int32_t n_blocks, int32_t channels,
                                 int32_t mode, void* stream) {
  AZ_REQUIRE(n_boards >= 0 && n_blocks >= 0, AZ_ERR_ARG, "az_trunk_wino_gpu: negative size");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(planes && stem_w && stem_b && h && t && h != t && (n_blocks == 0 || (wq && bias)),
             AZ_ERR_ARG, "az_trunk_wino_gpu: null or aliased buffer");
  AZ_REQUIRE(((uintptr_t)stem_w | (uintptr_t)stem_b | (uintptr_t)h | (uintptr_t)t) % 16 == 0,
             AZ_ERR_ARG, "az_trunk_wino_gpu: buffers must be 16-byte aligned");
  const TrunkArgs a{planes, stem_w, stem_b, reinterpret_cast<const char* const*>(wq), bias, h, t,
                    n_boards, n_blocks};
  hipStream_t s = azc::as_stream(stream);
  if (channels == 128 && mode == AZ_CONV_SPLIT3) return launch_trunk<Wn<128, AZ_CONV_SPLIT3>>(a, s);
  if (channels == 64 && mode == AZ_CONV_SPLIT3) return launch_trunk<Wn<64, AZ_CONV_SPLIT3>>(a, s);
  if (channels == 128 && mode == AZ_CONV_FP16) return launch_trunk<Wn<128, AZ_CONV_FP16>>(a, s);
  if (channels == 64 && mode == AZ_CONV_FP16) return launch_trunk<Wn<64, AZ_CONV_FP16>>(a, s);
  return azc::set_error(AZ_ERR_ARG, "az_trunk_wino_gpu: channels %d / mode %d unsupported",
                        channels, mode);
}

extern "C" int64_t az_conv3x3_wino_prep_bytes(int32_t channels, int32_t mode) {
  const int planes = mode == AZ_CONV_SPLIT3 ? 3 : (mode == AZ_CONV_FP16X2 ? 2 : 1);
  return (int64_t)16 * channels * channels * planes * 2 + (mode == AZ_CONV_FP16X2 ? 16 : 0);
}

extern "C" int az_conv3x3_wino_prep_gpu(const float* w9, void* wq, int32_t channels,
                                        int32_t mode, void* stream) {
  AZ_REQUIRE(w9 && wq, AZ_ERR_ARG, "az_conv3x3_wino_prep_gpu: null buffer");
  AZ_REQUIRE(channels == 64 || channels == 128, AZ_ERR_ARG,
             "az_conv3x3_wino_prep_gpu: channels must be 64 or 128, got %d", channels);
  hipStream_t s = azc::as_stream(stream);
  const unsigned grid = (unsigned)((channels * channels + 255) / 256);
  uint16_t* out = static_cast<uint16_t*>(wq);
  if (mode == AZ_CONV_SPLIT3)
    hipLaunchKernelGGL((k_wino_prep<AZ_CONV_SPLIT3>), dim3(grid), dim3(256), 0, s, w9, out, channels, nullptr);
  else if (mode == AZ_CONV_FP16)
    hipLaunchKernelGGL((k_wino_prep<AZ_CONV_FP16>), dim3(grid), dim3(256), 0, s, w9, out, channels, nullptr);
  else if (mode == AZ_CONV_FP16X2) {
    unsigned* hdr = reinterpret_cast<unsigned*>(out + (size_t)16 * channels * channels * 2);
    AZ_HIP(hipMemsetAsync(hdr, 0, 16, s));
    hipLaunchKernelGGL((k_wino_prep<AZ_CONV_FP16X2, true>), dim3(grid), dim3(256), 0, s, w9, out, channels, hdr);
    hipLaunchKernelGGL((k_wino_prep<AZ_CONV_FP16X2>), dim3(grid), dim3(256), 0, s, w9, out, channels, hdr);
  } else
    return azc::set_error(AZ_ERR_ARG, "az_conv3x3_wino_prep_gpu: unknown mode %d", mode);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

extern "C" int az_conv3x3_wino_gpu(const float* x, const void* wq, const float* bias,
                                   const float* res, float* y, int32_t n_boards,
                                   int32_t channels, int32_t relu, int32_t mode, void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_conv3x3_wino_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && wq && bias && y && x != y && (!res || res != y), AZ_ERR_ARG,
             "az_conv3x3_wino_gpu: null buffer or in-place call");
  AZ_REQUIRE(((uintptr_t)x | (uintptr_t)wq | (uintptr_t)bias) % 16 == 0, AZ_ERR_ARG,
             "az_conv3x3_wino_gpu: buffers must be 16-byte aligned");
  hipStream_t s = azc::as_stream(stream);
  if (channels == 128 && mode == AZ_CONV_SPLIT3)
    return launch_wino<Wn<128, AZ_CONV_SPLIT3>>(x, wq, bias, res, y, n_boards, relu, s);
  if (channels == 64 && mode == AZ_CONV_SPLIT3)
    return launch_wino<Wn<64, AZ_CONV_SPLIT3>>(x, wq, bias, res, y, n_boards, relu, s);
  if (channels == 128 && mode == AZ_CONV_FP16)
    return launch_wino<Wn<128, AZ_CONV_FP16>>(x, wq, bias, res, y, n_boards, relu, s);
  if (channels == 64 && mode == AZ_CONV_FP16)
    return launch_wino<Wn<64, AZ_CONV_FP16>>(x, wq, bias, res, y, n_boards, relu, s);
  return azc::set_error(AZ_ERR_ARG, "az_conv3x3_wino_gpu: channels %d / mode %d unsupported",
                        channels, mode);
}
