// conv_wino4.hip — the residual trunk's 3x3 convolution (C = 128) as Winograd F(2x2, 3x3)
// on the 16-bit MFMA pipe, with four boards per workgroup and the output transform folded
// into the K loop.
//
// Same op, numerics modes, weight layout (az_conv3x3_wino_prep_gpu) and transforms as
// conv_wino.hip:  Y = A^T [ sum_ci (G g G^T) (.) (B^T d B) ] A,  16 GEMMs (one per
// transform point xi = (k, l)) of  M_xi[tile][co] = sum_ci V_xi[tile][ci] U_xi[ci][co].
//
// Why a second form.  conv_wino.hip keeps all 16 points' accumulators of its tiles live
// (16 x 32 rows x 128 columns fp32 = half the CU's register file), which caps a workgroup
// at two boards; every workgroup then streams the whole transformed weight set (16 x 128 x
// 128 x 6 B split3 = 1.5 MiB) from L2 for two boards, and that L2 -> CU stream, not the
// MFMAs, bounds it.  Here the points are visited row by row of the 4x4
// transform grid ("groups" k = 0..3, four points (k, 0..3) each) and each group's M is
// folded into the four output accumulators right after its K loop:
//     t_j(k) = sum_l A^T[j][l] M_(k,l)     (t_0 = M0 + M1 + M2, t_1 = M1 - M2 - M3)
//     Y[i][j] += A^T[i][k] t_j(k)
// so a tile needs 4 points' M plus its 2x2 outputs Y live instead of 16 points' M: the
// same registers hold 4 boards instead of 2.
//
// Workgroup = 4 boards (64 tiles = two 32-row MFMA tiles) x all 128 columns, 8 waves (two
// per SIMD): wave w = (row tile rt = w / 4, column block cb = w % 4).  Waves w and w + 4
// (same columns, the other row tile) request the same weight fragments at the same step,
// so the second request is served by the CU's L1: the L2 -> CU weight stream per board is
// half of conv_wino.hip's.
//   * Linear chunk L = 0..31 = (group k = L / 8, input-channel chunk c = L % 8 of 16
//     channels); within a chunk, steps l = 0..3 run point (k, l): 6 split3 products (or 1
//     fp16 product) on the wave's 32x32 tile.
//   * V of chunk L+1 is formed while chunk L computes: the two window rows B^T row k needs
//     (d_a +- d_a') are requested one chunk ahead, combined into the row at the chunk start,
//     and each step transforms, splits and stores one point into the other half of a
//     double-buffered LDS image [point][plane][tile][16 ch] (rows XOR-swizzled by 16-byte
//     half so the ds_read_b128 fragment reads are conflict-free).
//   * Weights stream per wave from L2 three steps ahead (ring of 4 fragments).
//   * One LDS barrier per chunk (lgkmcnt only; the weight and window loads stay in flight).
//   * Epilogue straight from the Y registers: + bias (+ residual), ReLU, store.
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "heads_az.h"

#ifndef AZ_W4_IPD3
#define AZ_W4_IPD3 1
#endif
#ifndef AZ_W4_IPD16
#define AZ_W4_IPD16 2
#endif
#ifndef AZ_W4_PD3
#define AZ_W4_PD3 3
#endif
#ifndef AZ_W4_PD16
#define AZ_W4_PD16 7
#endif

#ifndef AZ_W4_STAMP
#define AZ_W4_STAMP 0
#endif
// 1 (product): weight and input slices through buffer descriptors (wave-uniform chunk/step
// offsets in soffset, no per-lane 64-bit address arithmetic), transform-row offsets and
// signs compile-time per group (the group loop's last chunk pair peeled), the input scale
// folded into the row combination; 0 = the round-2 loop (A/B builds)
#ifndef AZ_W4_DIET
#define AZ_W4_DIET 1
#endif
// experiment hooks (scripts/build_variants.py builds with bits set; results wrong):
// 1 = no weight loads in the loop, 2 = no transform / input work in the loop, 4 = no MFMAs,
// 8 = no LDS barrier in the loop, 16 = no A-fragment LDS reads, 32 = weight loads by the
// first row tile's waves only (the other half reuses stale fragments), 64 = no input-slice
// loads / LDS stores in the loop (the windows read stale slots), 128 = no global stores of a
// non-residual conv's output, 256 = no global residual reads (the resident trunk's RES
// epilogues), 512 = no resident-input write-out.  Product: 0.
#ifndef AZ_W4_EXP
#define AZ_W4_EXP 0
#endif
#ifndef AZ_W4_SCHED
#define AZ_W4_SCHED 0
#endif
// wave priority (experiments): 1 = s_setprio 1 once for the younger half of an 8-wave
// workgroup (waves 4-7), 2 = s_setprio 1 / 0 around each step's MFMA cluster
#ifndef AZ_W4_PRIO
#define AZ_W4_PRIO 0
#endif
// streaming cache hint (experiments): bit 0 = the input loads and the residual LDS-DMA
// non-temporal (nt), bit 1 = the output stores non-temporal -- so the activations stream
// past L2 instead of evicting the weight set every workgroup re-reads from it
#ifndef AZ_W4_NT
#define AZ_W4_NT 0
#endif
// timing proxy of a two-plane split (wrong numerics): 2 planes, 3 products
#ifndef AZ_W4_PROXY2
#define AZ_W4_PROXY2 0
#endif
// packed / mixed-precision forms of the transform's and fold's float ops (inline asm where
// the compiler would split them); 0 = the plain vector expressions (A/B builds)
#ifndef AZ_W4_PK
#define AZ_W4_PK 1
#endif
// the lo word of put()'s fp16 split by the mixed-precision FMA (v_fma_mix*_f16); 0 = by
// conversions and a subtraction (same bits)
#ifndef AZ_W4_MIX
#define AZ_W4_MIX AZ_W4_PK
#endif
// the remaining two-wide adds, products and FMAs of the input transform and the fold as one
// packed instruction each (inline asm; the compiler emits about a third of them as two
// scalar ops, profiles/r05_isa_mix.txt): 9 % less loop VALU but twice the hazard s_nops,
// +0.3 % per launch (profiles/r05_conv_micro_ab.json); 0 = the plain vector expressions
#ifndef AZ_W4_PK2
#define AZ_W4_PK2 0
#endif
// the layer's last two chunks skip the pipeline's look-ahead past the end (clamped duplicates:
// input slices, their LDS stores and window reads, the last chunk's weight steps, transform
// and A fragments) -- none of it was ever used: -1.25 % per evaluation at B = 1,024, outputs
// bit-identical (profiles/r04_conv_tail_ab.json); 0 = the uniform look-ahead (A/B builds)
#ifndef AZ_W4_TAIL
#define AZ_W4_TAIL 1
#endif
// the persistent trunk's layer input resident in LDS (see conv_body): 416.2-417.1 -> 368.7-371.3
// us per B = 1,024 trunk + heads launch, configs[2] bench 104.1 -> 116.7 games/s, same box,
// outputs bit-identical (profiles/r05_resident_ab.json); 0 = the per-chunk input slices with
// the two-slice hand-off (AZ_W4_HANDOFF)
#ifndef AZ_W4_RESIDENT
#define AZ_W4_RESIDENT 1
#endif
// with the resident input: a residual conv stages its residual rows in X's odd rows, free
// while the transform-grid row 3 (even input rows only) runs -- half 0 from the end of
// group 2's seventh chunk, half 1 during group 3: 374.9-376.2 -> 344.4-345.9 us per B = 1,024
// trunk + heads launch, configs[2] 116.9 -> 124.5 games/s, same box, bit-identical
// (profiles/r05_resident_ab.json); 0 = read from global memory in the epilogue
#ifndef AZ_W4_RXS
#define AZ_W4_RXS 1
#endif
// boards per workgroup of the persistent trunk (az_trunk_wino4_gpu / _heads_gpu): 2 = two
// workgroups per CU; 4 = one eight-wave workgroup per CU (with the resident input: X 128 KiB +
// two 16 KiB V buffers = all 160 KiB), half the weight stream per board (A/B builds)
#ifndef AZ_W4_TRUNK_BOARDS
#define AZ_W4_TRUNK_BOARDS 2
#endif
// the epilogue's output pairs (2tx, 2tx + 1) as packed f32x2 (scale + bias in one v_pk_fma_f32,
// the staged residual in one packed add): 411.0-411.5 -> 409.0-410.3 us per B = 1,024 trunk
// + heads launch, same box (profiles/r05_conv_micro_ab.json); 0 = one element at a time
#ifndef AZ_W4_EPI_PK
#define AZ_W4_EPI_PK 1
#endif
// the persistent trunk's layer hand-off: a layer's epilogue also writes its output's first two
// 16-channel slices (channels 0-31, held by the column-block-0 wave) into the input slots and
// its per-board max |y| into LDS, so the next layer starts transforming without the global
// round trip of those slices and of its input ranges (same values: bit-identical): 411.0-411.5
// -> 408.0-410.1 us per launch (profiles/r05_conv_micro_ab.json); 0 = off
#ifndef AZ_W4_HANDOFF
#define AZ_W4_HANDOFF 1
#endif

namespace {

#if AZ_W4_STAMP
// experiment builds only (scripts/build_variants.py -DAZ_W4_STAMP=1): per-workgroup
// s_memtime / s_memrealtime stamps [wg][16] in a buffer no kernel reads
__device__ unsigned long long g_w4_stamps[1024 * 16];
#define W4_STAMP(i)                                                                  \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 1024) {                                     \
      g_w4_stamps[blockIdx.x * 16 + 2 * (i)] = __builtin_amdgcn_s_memtime();         \
      g_w4_stamps[blockIdx.x * 16 + 2 * (i) + 1] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                \
  } while (0)
#else
#define W4_STAMP(i) \
  do {              \
  } while (0)
#endif
// experiment builds only (-DAZ_W4_TSTAMP=1, scripts/trunk_stamps.py): the persistent trunk's
// per-layer timeline, workgroup wave 0's s_memtime at each conv's start (after the layer
// fence), after its prologue, before its first epilogue, and at its end, [wg < 1024][layer <
// 16][4], lane 0's vector store
#ifndef AZ_W4_TSTAMP
#define AZ_W4_TSTAMP 0
#endif
#if AZ_W4_TSTAMP
__device__ unsigned long long g_w4_tst[1024 * 16 * 4];
#define W4T_STAMP(layer, i)                                                              \
  do {                                                                                   \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                          \
    if (threadIdx.x == 0 && blockIdx.x < 1024 && (layer) < 16)                           \
      g_w4_tst[(blockIdx.x * 16 + (layer)) * 4 + (i)] = t_;                              \
  } while (0)
#else
#define W4T_STAMP(layer, i) \
  do {                      \
  } while (0)
#endif
// experiment builds only (-DAZ_W4_CSTAMP=1, scripts/w4_chunk_stamps.py): every wave's
// s_memtime at each chunk's start, before and after its closing barrier, [wg < 256][wave]
// [chunk][3], lane 0's vector store
#ifndef AZ_W4_CSTAMP
#define AZ_W4_CSTAMP 0
#endif
#if AZ_W4_CSTAMP
__device__ unsigned long long g_w4_cst[256 * 8 * 32 * 3];
#define W4C_STAMP(v, i)                                                                     \
  do {                                                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 256 && (v) < 32)                            \
      g_w4_cst[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 32 + (v)) * 3 + (i)] = t_;          \
  } while (0)
#else
#define W4C_STAMP(v, i) \
  do {                  \
  } while (0)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

template <int MODE_, int NRT_, int BOARDS_ = 4, int NC_ = 8, int NG_ = 4>
struct W4 {
  static constexpr int C = 128, MODE = MODE_;
  static constexpr int PLANES =
      MODE == AZ_CONV_SPLIT3 ? (AZ_W4_PROXY2 ? 2 : 3) : (MODE == AZ_CONV_FP16X2 ? 2 : 1);
  static constexpr bool SCALED = MODE == AZ_CONV_FP16X2;  // power-of-two operand scaling
  // NRT = MFMA row tiles per wave: 2 -> 4 waves (one per SIMD), each weight fragment feeds
  // both row tiles of its wave; 1 -> 8 waves (two per SIMD), row-tile partners request
  // the same fragments
  // BOARDS = 4: 64 tiles = two row tiles, 8 / NRT waves, one workgroup per CU (LDS);
  // BOARDS = 2: one row tile, 4 waves, two workgroups per CU (independent barriers)
  static constexpr int BOARDS = BOARDS_, ROWS = 16 * BOARDS;
  static constexpr int NRT = NRT_, WAVES = (ROWS / 32) * 4 / NRT, TPT = NRT;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int SLAB = ROWS * 32;            // one (point, plane): 64 tiles x 16 ch x 2 B
  static constexpr int BUF = 4 * PLANES * SLAB;     // one (group, chunk): its four points
  // input chunk slice staged in LDS, zero-padded to 10 x 10 positions per board so a
  // window read never needs a mask: [board][10][10][16 ch] fp32
  static constexpr int IN_ROW = 10 * 64, IN_BOARD = 10 * IN_ROW, IN_SLOT = BOARDS * IN_BOARD;
  static constexpr int IN_OFF = 2 * BUF;             // two slots after the V double buffer
  // residual half (RES kernels): output rows 2ty + I of the 4 boards, [board][ty][8][C] fp32,
  // staged during group 2 + I and added by that half's epilogue
  static constexpr int RES_OFF = 2 * BUF + 2 * IN_SLOT, RES_BYTES = BOARDS * 4 * 8 * C * 4;
  static constexpr int RS = RES_BYTES / 16 / THREADS / 8;  // 16-byte pieces per thread per chunk
  // staged only where it fits beside the rest (not split3's three planes: its residual is
  // read from global memory in the epilogue)
  static constexpr bool RES_FITS = RES_OFF + RES_BYTES <= 160 * 1024 - 128;
  // the persistent trunk's layer hand-off (AZ_W4_HANDOFF): each wave's per-board max |y|,
  // [wave][board] floats after everything else
  static constexpr int RNG_OFF = RES_FITS ? RES_OFF + RES_BYTES : RES_OFF;
  static constexpr int LDS_BYTES = RNG_OFF + 128;
  // the resident layout (AZ_W4_RESIDENT, the persistent trunk): V buffer 0, the layer's whole
  // input X = [board][64 positions][C] fp32 (channel chunk slots swizzled by column pair,
  // xoff), V buffer 1 -- so a board-edge window's out-of-board rows and columns land in
  // finite words (X, or V's fp16 pairs, never an fp32 Inf / NaN pattern) and are masked
  // VPAD: V buffer 0 / 1 rounded up to the 8 KiB a board-edge window reaches before / past X
  // (one board row plus one position: 4.5 KiB); FP16X2's buffers are that size, FP16's half
  static constexpr int VPAD = BUF < 8192 ? 8192 : BUF;
  static constexpr int XOFF = VPAD, XBYTES = BOARDS * 64 * C * 4, V1R = VPAD + XBYTES;
  static constexpr int RSD_BYTES = 2 * VPAD + XBYTES;
  static constexpr int TRUNK_LDS =
      AZ_W4_RESIDENT && RSD_BYTES > LDS_BYTES ? RSD_BYTES : LDS_BYTES;
  static constexpr int LD_PER_THREAD = BOARDS * 64 * 4 / THREADS;  // 16-byte loads per chunk
  static constexpr int STEP_BYTES = PLANES * C * 32;  // weight bytes of one (chunk, point)
  static constexpr int CHUNKS = C / 16;
  static constexpr int LCHUNKS = 4 * CHUNKS;        // (group, chunk) pairs
  static constexpr int QSTEPS = LCHUNKS * 4;        // (group, chunk, point) steps
  // Channel split (small batches, az_conv3x3_wino4_splitk_gpu): a workgroup runs NC of the
  // CHUNKS input-channel chunks of every group -- chunks cs .. cs + NC - 1, cs = NC *
  // blockIdx.y -- and writes its partial output sums; a second kernel adds the splits in
  // order with the epilogue.  Its own chunk sequence is the "virtual" index v = 0 .. VCH-1.
  // NG = 1: the four transform-grid rows split over workgroups too (row g0 = blockIdx.y /
  // (CHUNKS / NC)); the output transform is linear, so those partials add up as well.
  static constexpr int NC = NC_, NG = NG_, VCH = NG * NC, VQ = VCH * 4;
  static constexpr bool SPLIT = NC < CHUNKS || NG < 4;
  static_assert((NC == 1 || NC % 2 == 0) && CHUNKS % NC == 0, "chunk pairs per split");
  static_assert(NG == 4 || NG == 1, "all four transform rows, or one");
  // weight fragment ring and prefetch distance (steps)
  static constexpr int PD = MODE == AZ_CONV_FP16 ? AZ_W4_PD16 : AZ_W4_PD3;
  static constexpr int RING = PD < 4 ? 4 : 8;  // divides the 8 steps of a chunk pair
  // input slices requested IPD chunks ahead of their LDS store (IPD register sets)
  static constexpr int IPD = MODE == AZ_CONV_FP16 ? AZ_W4_IPD16 : AZ_W4_IPD3;
  static_assert(IPD == 1 || IPD == 2, "IPD");
};

template <class G>
using Word8 = typename std::conditional<G::MODE == AZ_CONV_SPLIT3, bf16x8, f16x8>::type;

template <class G>
struct Frag {
  Word8<G> v[G::PLANES];
};

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// frexp's exponent of a non-negative finite float (x < 2^e; 0 -> 0), from its bits
__device__ __forceinline__ int frexp_exp(float x) {
  const int b = (int)((__float_as_uint(x) >> 23) & 0xff);
  return b == 0 ? (x > 0.0f ? -125 : 0) : b - 126;
}

// window rows of group k: B^T row k = sa * d_a0 + sb * d_a1 (B^T = [1 0 -1 0; 0 1 1 0;
// 0 -1 1 0; 0 1 0 -1]); multiplying by +-1 is exact, so this is the transform's own
// add / subtract
__host__ __device__ constexpr int grp_a0(int k) { return k == 0 ? 0 : 1; }
__host__ __device__ constexpr int grp_a1(int k) { return k == 3 ? 3 : 2; }
__host__ __device__ constexpr float grp_sa(int k) { return k == 2 ? -1.0f : 1.0f; }
__host__ __device__ constexpr float grp_sb(int k) { return (k == 1 || k == 2) ? 1.0f : -1.0f; }

// weight fragment of linear step q (chunk L = q / 4 = (group k, channel chunk c), point l)
template <class G>
__device__ __forceinline__ void load_b(Frag<G>& f, const char* wq, int wlane, int q) {
  const int L = q >> 2, l = q & 3, k = L >> 3, c = L & 7;
  const char* step = wq + (size_t)(c * 16 + 4 * k + l) * G::STEP_BYTES;
#pragma unroll
  for (int pl = 0; pl < G::PLANES; ++pl)
    f.v[pl] = *reinterpret_cast<const Word8<G>*>(step + wlane + pl * G::C * 32);
}

// the same through the weights' buffer descriptor: the step's byte offset is wave-uniform
// (soffset), the lane's (wlane) a fixed voffset
template <class G>
__device__ __forceinline__ void load_b(Frag<G>& f, __amdgpu_buffer_rsrc_t rw, int wlane, int q) {
  const int L = q >> 2, l = q & 3, k = L >> 3, c = L & 7;
  const int so = (c * 16 + 4 * k + l) * G::STEP_BYTES;
#pragma unroll
  for (int pl = 0; pl < G::PLANES; ++pl)
    f.v[pl] = __builtin_bit_cast(
        Word8<G>, __builtin_amdgcn_raw_buffer_load_b128(rw, wlane, so + pl * G::C * 32, 0));
}

template <class G>
__device__ __forceinline__ void read_a(Frag<G> (&a)[G::NRT], const char* buf, int l,
                                       const int (&aoff)[G::NRT]) {
#pragma unroll
  for (int t = 0; t < G::NRT; ++t)
#pragma unroll
    for (int pl = 0; pl < G::PLANES; ++pl)
      a[t].v[pl] = *reinterpret_cast<const Word8<G>*>(buf + (l * G::PLANES + pl) * G::SLAB + aoff[t]);
}

// FIRST: the group's first product on this accumulator takes C = 0 (an inline constant)
// instead of a zeroed register set, so no per-group zeroing pass is needed
template <class G, bool FIRST = false>
__device__ __forceinline__ void mma(f32x16& acc, const Frag<G>& a, const Frag<G>& b) {
  if constexpr (FIRST && G::MODE == AZ_CONV_FP16X2) {
    const f32x16 z = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[1], b.v[0], z, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[0], b.v[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[0], b.v[0], acc, 0, 0, 0);
  } else if constexpr (FIRST && G::MODE == AZ_CONV_FP16) {
    const f32x16 z = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[0], b.v[0], z, 0, 0, 0);
  } else if constexpr (FIRST) {
    constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
    constexpr int T0 = AZ_W4_PROXY2 ? 3 : 0;
    const f32x16 z = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[PA[T0]], b.v[PB[T0]], z, 0, 0, 0);
#pragma unroll
    for (int t = T0 + 1; t < 6; ++t)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[PA[t]], b.v[PB[t]], acc, 0, 0, 0);
  } else if constexpr (G::MODE == AZ_CONV_SPLIT3) {
    // smallest partial products first (x2y0, x1y1, x0y2, x1y0, x0y1, x0y0)
    constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
    constexpr int T0 = AZ_W4_PROXY2 ? 3 : 0;  // proxy: the last three products only
#pragma unroll
    for (int t = T0; t < 6; ++t)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[PA[t]], b.v[PB[t]], acc, 0, 0, 0);
  } else if constexpr (G::MODE == AZ_CONV_FP16X2) {
    // lo * hi, hi * lo, hi * hi (the lo * lo term is below fp32's rounding unit)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[1], b.v[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[0], b.v[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[0], b.v[0], acc, 0, 0, 0);
  } else {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.v[0], b.v[0], acc, 0, 0, 0);
  }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// the chunk-L slice of the workgroup's input (4 boards x 64 positions x 16 channels fp32):
// LD_PER_THREAD coalesced 16-byte loads per thread into registers ...
template <class G>
__device__ __forceinline__ void load_in(f32x4 (&ld)[G::LD_PER_THREAD], const float* x,
                                        const int (&goff)[G::LD_PER_THREAD], int L) {
  const int c = L & 7;
#pragma unroll
  for (int j = 0; j < G::LD_PER_THREAD; ++j)
    ld[j] = *reinterpret_cast<const f32x4*>(x + goff[j] + c * 16);
}

// the same through the input's buffer descriptor (goff in bytes; the chunk's channel offset
// is wave-uniform)
template <class G>
__device__ __forceinline__ void load_in(f32x4 (&ld)[G::LD_PER_THREAD], __amdgpu_buffer_rsrc_t rx,
                                        const int (&goff)[G::LD_PER_THREAD], int L) {
  const int c = L & 7;
#pragma unroll
  for (int j = 0; j < G::LD_PER_THREAD; ++j)
    ld[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, goff[j], c * 64,
                                                                             (AZ_W4_NT & 1) ? 2 : 0));
}

// ... and into the slot's padded interior
template <class G>
__device__ __forceinline__ void store_in(char* slot, const f32x4 (&ld)[G::LD_PER_THREAD],
                                         const int (&ldst)[G::LD_PER_THREAD]) {
#pragma unroll
  for (int j = 0; j < G::LD_PER_THREAD; ++j) *reinterpret_cast<f32x4*>(slot + ldst[j]) = ld[j];
}

// Column slot of padded column c (0..9) in a slot row: c ^ (c>>1 & 1) ^ (c>>2 & 1) << 1.  A
// half-wave's window reads hit columns {b, b+2, b+4, b+6} of one row (four tiles), 64 B
// each, and the compiler pairs the two window rows into ds_read2_b64 (16-lane groups, banks
// (a/4) mod 32: columns c, c+2 meet).  Unpermuted, c and c + 2 (ds_read2_b64) or c and
// c + 4 (ds_read_b64, banks (a/4) mod 64) share banks; here c, c+2 differ in 64-B parity and
// {b, b+2, b+4, b+6} are distinct mod 4, so both forms are conflict-free.  The input stores
// (ds_write_b128, 8-lane groups, (a/4) mod 32) pair positions (c, c+2) to match (the load
// lane order below); SQ_LDS_BANK_CONFLICT was 2.2M cycles per launch before.
__host__ __device__ constexpr int col_slot(int c) { return c ^ ((c >> 1) & 1) ^ (((c >> 2) & 1) << 1); }

// B^T row k of this item's 4x4 window (channel pair): the two window rows a0, a1 of group
// k read from the padded slot (off-board entries are the zero border) -- issued first,
// combined once the MFMAs they hide behind are under way.  cols = the window's four column
// slots (col_slot(2tx + b), 8 bits each)
template <class G>
__device__ __forceinline__ void read_rows(f32x2 (&d)[8], const char* slot, int rbase, int cols,
                                          int L) {
  const int k = L >> 3;
  const char* r0 = slot + rbase + grp_a0(k) * G::IN_ROW;
  const char* r1 = slot + rbase + grp_a1(k) * G::IN_ROW;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int co = ((cols >> (8 * b)) & 0xff) * 64;
    d[b] = *reinterpret_cast<const f32x2*>(r0 + co);
    d[4 + b] = *reinterpret_cast<const f32x2*>(r1 + co);
  }
}

__device__ __forceinline__ void combine_rows(f32x2 (&rk)[4], const f32x2 (&d)[8], int L) {
  const int k = L >> 3;
  const f32x2 sa = {grp_sa(k), grp_sa(k)}, sb = {grp_sb(k), grp_sb(k)};
#pragma unroll
  for (int b = 0; b < 4; ++b) rk[b] = sa * d[b] + sb * d[4 + b];
}

template <class G>
__device__ __forceinline__ void make_rows(f32x2 (&rk)[4], const char* slot, int rbase, int cols,
                                          int L) {
  f32x2 d[8];
  read_rows<G>(d, slot, rbase, cols, L);
  combine_rows(rk, d, L);
}

// Compile-time group KK (AZ_W4_DIET): the window rows of slot PAR read with immediate LDS
// offsets from the lane's four column bases cb[b] (rbase + column slot), and combined with
// the input scale folded in -- rk = vsc sa d_a0 + vsc sb d_a1 is vsc times the unscaled
// row exactly (vsc is a power of two), so V and its split are bit-identical to scaling
// each point afterwards
template <class G, int KK, int PAR>
__device__ __forceinline__ void read_rows_k(f32x2 (&d)[8], const char* lds, const int (&cb)[4]) {
  constexpr int base = G::IN_OFF + PAR * G::IN_SLOT;
  constexpr int o0 = base + grp_a0(KK) * G::IN_ROW, o1 = base + grp_a1(KK) * G::IN_ROW;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    d[b] = *reinterpret_cast<const f32x2*>(lds + cb[b] + o0);
    d[4 + b] = *reinterpret_cast<const f32x2*>(lds + cb[b] + o1);
  }
}

// a + b, a * b and fma(a, b, c) on f32x2 as one packed instruction (AZ_W4_PK2), else the
// vector expressions; the same IEEE results element by element
__device__ __forceinline__ f32x2 pk_add(f32x2 a, f32x2 b) {
#if AZ_W4_PK2
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return a + b;
#endif
}
__device__ __forceinline__ f32x2 pk_mul(f32x2 a, f32x2 b) {
#if AZ_W4_PK2
  f32x2 r;
  asm("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return a * b;
#endif
}
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
#if AZ_W4_PK2
  f32x2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return __builtin_elementwise_fma(a, b, c);
#endif
}

template <int KK>
__device__ __forceinline__ void combine_k(f32x2 (&rk)[4], const f32x2 (&d)[8], float vsc) {
  const f32x2 fa = {grp_sa(KK) * vsc, grp_sa(KK) * vsc}, fb = {grp_sb(KK) * vsc, grp_sb(KK) * vsc};
#pragma unroll
  for (int b = 0; b < 4; ++b) rk[b] = pk_fma(fb, d[4 + b], pk_mul(fa, d[b]));
}

// Resident input (AZ_W4_RESIDENT): byte offset in X of (board bd, position pos, channel ch):
// 16-channel chunk slots of 64 B, slot = chunk ^ ((column >> 1) & 3), so the four tiles of
// a half-wave's window read (columns 2tx - 1 + b, tx = 0..3) hit four different bank groups
template <class G>
__device__ __forceinline__ int xoff(int bd, int pos, int ch) {
  return (bd * 64 + pos) * (G::C * 4) + ((((ch >> 4) ^ (((pos & 7) >> 1) & 3)) << 6) | ((ch & 15) << 2));
}

// window rows of group KK for chunk c from X: xb[b] = the window's top-left row and column b
// (unclamped: off-board entries read finite words, masked in combine_kx), chunk 0's slot
template <class G, int KK>
__device__ __forceinline__ void read_rows_x(f32x2 (&d)[8], const char* lds, const int (&xb)[4],
                                            int c) {
  constexpr int RB = 8 * G::C * 4;  // one board row
  constexpr int o0 = G::XOFF + grp_a0(KK) * RB, o1 = G::XOFF + grp_a1(KK) * RB;
  // opaque (an SGPR set here): with a compile-time chunk the compiler would otherwise hoist
  // every peeled chunk's four addresses out of the layer loop (~50 live VGPRs, spills)
  int xc = c << 6;
  asm volatile("" : "+s"(xc));
  // the address as an LDS address, not as lds + offset: the dynamic LDS of the kernels using
  // this (k_trunk_wino4: no static LDS, tests/test_isa_scan_cpu.py checks) starts at address
  // 0, and the symbol's add of 0 cost one VALU per read pair
  (void)lds;
  typedef __attribute__((address_space(3))) const f32x2 lf32x2;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const unsigned a = (unsigned)(xb[b] ^ xc);  // flips the chunk slot bits only
    d[b] = *reinterpret_cast<lf32x2*>((size_t)(a + o0));
    d[4 + b] = *reinterpret_cast<lf32x2*>((size_t)(a + o1));
  }
}

// combine_k with the board-edge masks m = {top row valid, bottom row valid, left column valid,
// right column valid} (0 / 1): a masked term is finite x 0, so the sums are the zero-padded
// slot's (up to the sign of an exact zero)
template <int KK>
__device__ __forceinline__ void combine_kx(f32x2 (&rk)[4], const f32x2 (&d)[8], float vsc,
                                           const float (&m)[4]) {
  float fa_s = grp_sa(KK) * vsc, fb_s = grp_sb(KK) * vsc;
  if constexpr (KK == 0) fa_s *= m[0];  // window row 2ty - 1
  if constexpr (KK == 3) fb_s *= m[1];  // window row 2ty + 2
  const f32x2 fa = {fa_s, fa_s}, fb = {fb_s, fb_s};
#pragma unroll
  for (int b = 0; b < 4; ++b) rk[b] = __builtin_elementwise_fma(fb, d[4 + b], fa * d[b]);
  rk[0] = rk[0] * f32x2{m[2], m[2]};  // window column 2tx - 1
  rk[3] = rk[3] * f32x2{m[3], m[3]};  // window column 2tx + 2
}

// a - b on an f32x2 as ONE v_pk_add_f32 with b negated: the compiler splits a two-wide
// fsub into two v_sub_f32 (and folds an fma by -1 back into that fsub); same IEEE
// differences element by element
__device__ __forceinline__ f32x2 pk_sub(f32x2 a, f32x2 b) {
#if AZ_W4_PK
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return a - b;
#endif
}

// V at point (k, l) = (row k of B^T d) B: column combination l
template <int l>
__device__ __forceinline__ f32x2 col_comb(const f32x2 (&rk)[4]) {
  if constexpr (l == 0) return pk_sub(rk[0], rk[2]);
  if constexpr (l == 1) return pk_add(rk[1], rk[2]);
  if constexpr (l == 2) return pk_sub(rk[2], rk[1]);
  return pk_sub(rk[1], rk[3]);
}

// split two transformed values into PLANES 16-bit words and store them in their slabs
template <class G>
__device__ __forceinline__ void put(char* slab, f32x2 v, float vsc) {
  if constexpr (G::MODE == AZ_CONV_FP16X2) {
    const f32x2 vs = v * vsc;  // exact: a power of two (1 in the DIET path: folded away)
    const f16x2 hi = __builtin_convertvector(vs, f16x2);
#if AZ_W4_MIX
    // lo = RN16(vs - hi) per element by the mixed-precision FMA (hi read as f16, vs - hi
    // exact in f32, rounded once to f16): two v_fma_mix*_f16 instead of two f16 -> f32
    // conversions, the subtraction and a second packed conversion; bit-identical
    uint32_t lo;
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(lo)
        : "v"(__builtin_bit_cast(uint32_t, hi)), "v"(vs.x), "v"(vs.y));
    *reinterpret_cast<f16x2*>(slab) = hi;
    *reinterpret_cast<uint32_t*>(slab + G::SLAB) = lo;
#else
    const f16x2 lo = __builtin_convertvector(vs - __builtin_convertvector(hi, f32x2), f16x2);
    *reinterpret_cast<f16x2*>(slab) = hi;
    *reinterpret_cast<f16x2*>(slab + G::SLAB) = lo;
#endif
  } else if constexpr (G::MODE == AZ_CONV_SPLIT3) {
    const bf16x2 x0 = __builtin_convertvector(v, bf16x2);
    const f32x2 r1 = v - __builtin_convertvector(x0, f32x2);
    const bf16x2 x1 = __builtin_convertvector(r1, bf16x2);
    const bf16x2 x2 = __builtin_convertvector(r1 - __builtin_convertvector(x1, f32x2), bf16x2);
    *reinterpret_cast<bf16x2*>(slab) = x0;
    *reinterpret_cast<bf16x2*>(slab + G::SLAB) = x1;
    if (G::PLANES > 2) *reinterpret_cast<bf16x2*>(slab + 2 * G::SLAB) = x2;
  } else {
    *reinterpret_cast<f16x2*>(slab) = __builtin_convertvector(v, f16x2);
  }
}

template <class G, int l>
__device__ __forceinline__ void put_point(char* buf, const f32x2 (&rk)[4], int soff, float vsc) {
  put<G>(buf + l * G::PLANES * G::SLAB + soff, col_comb<l>(rk), vsc);
}

// group K's M (acc[l][t]) into the output accumulators Y[i][j][t]; K is a compile-time
// constant so every update is straight-line register arithmetic
template <class G, int K>
__device__ __forceinline__ void fold(f32x16 (&acc)[4][G::NRT], f32x16 (&Y)[2][2][G::NRT]) {
  // element pairs (e, e + 1) as f32x2: v_pk_add_f32 on the aligned register pairs, the
  // same IEEE sums element by element
  auto get = [](const f32x16& v, int e) { return f32x2{v[e], v[e + 1]}; };
  auto set = [](f32x16& v, int e, f32x2 x) {
    v[e] = x.x;
    v[e + 1] = x.y;
  };
  auto sub = [](f32x2 a, f32x2 b) { return pk_sub(a, b); };
#pragma unroll
  for (int t = 0; t < G::NRT; ++t)
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      const f32x2 m0 = get(acc[0][t], e), m1 = get(acc[1][t], e), m2 = get(acc[2][t], e),
                  m3 = get(acc[3][t], e);
      const f32x2 t0 = pk_add(pk_add(m0, m1), m2), t1 = sub(sub(m1, m2), m3);
      if constexpr (K == 0 && G::NG == 4) {
        set(Y[0][0][t], e, t0);
        set(Y[0][1][t], e, t1);
      } else if constexpr (K == 0) {  // NG = 1: Y starts at zero (rows of other workgroups)
        set(Y[0][0][t], e, pk_add(get(Y[0][0][t], e), t0));
        set(Y[0][1][t], e, pk_add(get(Y[0][1][t], e), t1));
      } else if constexpr (K == 1) {
        set(Y[0][0][t], e, pk_add(get(Y[0][0][t], e), t0));
        set(Y[0][1][t], e, pk_add(get(Y[0][1][t], e), t1));
        if constexpr (G::NG == 4) {
          set(Y[1][0][t], e, t0);
          set(Y[1][1][t], e, t1);
        } else {
          set(Y[1][0][t], e, pk_add(get(Y[1][0][t], e), t0));
          set(Y[1][1][t], e, pk_add(get(Y[1][1][t], e), t1));
        }
      } else if constexpr (K == 2) {
        set(Y[0][0][t], e, pk_add(get(Y[0][0][t], e), t0));
        set(Y[0][1][t], e, pk_add(get(Y[0][1][t], e), t1));
        set(Y[1][0][t], e, sub(get(Y[1][0][t], e), t0));
        set(Y[1][1][t], e, sub(get(Y[1][1][t], e), t1));
      } else {
        set(Y[1][0][t], e, sub(get(Y[1][0][t], e), t0));
        set(Y[1][1][t], e, sub(get(Y[1][1][t], e), t1));
      }
    }
  // materialise Y here: otherwise the compiler sinks the fold arithmetic past the next
  // group's K loop, keeping this group's M live beside the next one's (and spills)
#pragma unroll
  for (int t = 0; t < G::NRT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if constexpr (K <= 2) asm volatile("" : "+v"(Y[0][0][t][e]), "+v"(Y[0][1][t][e]));
      if constexpr (K >= 1) asm volatile("" : "+v"(Y[1][0][t][e]), "+v"(Y[1][1][t][e]));
    }
}

// a wave's loop state (registers after inlining; one struct so the chunk and group bodies
// below can be separate force-inlined functions)
template <class G>
struct St {
  f32x4 ld[G::IPD][G::LD_PER_THREAD];
  f32x2 rk[G::TPT][4], dr[G::TPT][8];
  Frag<G> bf[G::RING], af[G::NRT];
  f32x16 acc[4][G::NRT];
  f32x16 Y[2][2][G::NRT];
  int goff[G::LD_PER_THREAD], ldst[G::LD_PER_THREAD], rbase[G::TPT], cols[G::TPT], soff[G::TPT], aoff[G::NRT];
  float vsc[G::TPT];  // FP16X2: the item's board input scale 2^sv (1 otherwise)
  int cbase[G::TPT][4];  // AZ_W4_DIET: the item's window column bases in an input slot
  int xb[G::TPT][4];     // AZ_W4_RESIDENT: the item's window bases in X (read_rows_x)
  float xm[G::TPT][4];   // AZ_W4_RESIDENT: its board-edge masks (combine_kx)
  __amdgpu_buffer_rsrc_t rx, rw;  // input and weight descriptors (AZ_W4_DIET)
  int wlane, tid, b0, nb;
  int cs;             // first channel chunk of this workgroup's split (0 unless SPLIT)
  int g0;             // its transform-grid row (NG = 1; 0 otherwise)
  unsigned lds_res;   // LDS byte address of this wave's first residual piece
  const float* x;
  const float* res;
  const char* wq;
  char* lds;
};

// virtual chunk v of this workgroup -> linear chunk L = (group, channel chunk); clamped to the
// last one (the pipeline's look-ahead past the end reads a duplicate, as before)
template <class G>
__device__ __forceinline__ int lmap(const St<G>& S, int v) {
  v = v < G::VCH ? v : G::VCH - 1;
  return (S.g0 + v / G::NC) * G::CHUNKS + S.cs + (v % G::NC);
}
// virtual step vq (= 4 v + point) -> linear weight step
template <class G>
__device__ __forceinline__ int qmap(const St<G>& S, int vq) {
  vq = vq < G::VQ ? vq : G::VQ - 1;
  return lmap<G>(S, vq >> 2) * 4 + (vq & 3);
}

// one 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): lane i's 16 bytes land at LDS
// byte address lds_dst + 16 i.  Issued as asm so the compiler's vmcnt bookkeeping for the
// weight and input loads is not collapsed to vmcnt(0) around it; its completion is waited
// for explicitly (vmcnt(0)) before the barrier that precedes the reads
#if AZ_W4_NT & 1
#define AZ_W4_DMA_CPOL " nt"
#else
#define AZ_W4_DMA_CPOL ""
#endif
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" AZ_W4_DMA_CPOL
      "\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst));
}

__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// residual staging: piece p = (c * RS + s) * THREADS + tid of half I (16 bytes; 256 pieces
// = one 4 KiB [8 positions][C] row segment seg = p / 256 = (board, ty)), DMA'd at chunk c's
// second step straight into LDS (linear: offset 16 p)
template <class G, int I>
__device__ __forceinline__ void res_dma(St<G>& S, int c) {
#pragma unroll
  for (int s = 0; s < G::RS; ++s) {
    const int p = (c * G::RS + s) * G::THREADS + S.tid, seg = p >> 8, w = p & 255;
    const int bd = seg >> 2, ty = seg & 3, bs = bd < S.nb ? bd : S.nb - 1;
    glds16(S.res + ((size_t)(S.b0 + bs) * 64 + (2 * ty + I) * 8) * G::C + 4 * w,
           __builtin_amdgcn_readfirstlane(S.lds_res + 16 * (c * G::RS + s) * G::THREADS));
  }
}

// the resident trunk's residual staging (AZ_W4_RXS): segment c = (board c / 4, ty = c % 4) of
// half I -- row 2ty + I of the board, 8 positions x C fp32 = 4 KiB, one 16-byte piece per
// thread -- into X's row 2ty + 1 of that board (linear [8][C]); S.lds_res = X + 1 KiB x wave
template <class G, int I>
__device__ __forceinline__ void res_dma_x(St<G>& S, int c) {
  // pass c of 8: segments c * SP .. c * SP + SP - 1 (SP = 1 with 256 threads, 2 with 512),
  // 256 threads per 4 KiB segment
  constexpr int SP = G::THREADS / 256;
  static_assert(SP * 8 == G::BOARDS * 4, "eight passes per residual half");
  const int seg = c * SP + (S.tid >> 8);
  const int bd = seg >> 2, ty = seg & 3, bs = bd < S.nb ? bd : S.nb - 1;
  glds16(S.res + ((size_t)(S.b0 + bs) * 64 + (2 * ty + I) * 8) * G::C + 4 * (S.tid & 255),
         __builtin_amdgcn_readfirstlane(S.lds_res + (bd * 64 + (2 * ty + 1) * 8) * G::C * 4));
}

// one chunk L (of parity PAR, so a step's weight ring slot is a compile-time constant): its
// four steps, the next chunk's transform into the other LDS buffer, the windows of the
// chunk after that requested
// KR / KS: the transform-grid rows of chunks v+1 (whose rows are combined here) and v+2
// (whose windows are read at the end), when known at compile time (AZ_W4_DIET); -1 = from
// the chunk map at run time
// TAIL (AZ_W4_TAIL): 1 = the layer's second-to-last chunk (its input-slice look-ahead is past
// the end), 2 = the last (everything after its own MFMAs is)
// RSD (AZ_W4_RESIDENT): the layer input is resident in LDS -- no input-slice loads or stores,
// the windows read from X, V buffer 1 after X
// RDMA >= 0 (the resident trunk's residual staging): after this chunk's window reads, every
// segment of residual half RDMA into X's odd rows (no window reads them from here to the
// layer's end)
template <class G, int PAR, int STAGE, int KR = -1, int KS = -1, bool FIRST = false, int TAIL = 0,
          bool RSD = false, int RDMA = -1>
__device__ __forceinline__ void run_chunk(St<G>& S, int v) {
  constexpr bool CT = AZ_W4_DIET && KR >= 0 && KS >= 0;
  static_assert(!RSD || CT, "the resident input needs the compile-time group rows");
  constexpr bool NO_IN = TAIL >= 1 || RSD, NO_NEXT = TAIL == 2;
  constexpr bool NO_WIN = TAIL >= 1;  // no window reads for chunk v + 2
  constexpr int V1 = RSD ? G::V1R : G::BUF;
  W4C_STAMP(v, 0);
  const int L = lmap<G>(S, v);
  const char* cur = S.lds + (v & 1) * V1;
  char* nxt = S.lds + ((v + 1) & 1) * V1;
  // chunk v+1's rows (its windows were requested during chunk v-1); the last chunk
  // transforms a clamped duplicate into the idle buffer (uniform body)
  const int Lr = lmap<G>(S, v + 1);
  const int Ll = lmap<G>(S, v + 1 + G::IPD);  // loaded
  const int Ls = lmap<G>(S, v + 2);           // stored (slot (v + 2) & 1 = v & 1)
  constexpr int set_l = G::IPD == 1 ? 0 : (PAR + 1) & 1, set_s = G::IPD == 1 ? 0 : PAR;
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    Frag<G> an[G::NRT];
    if (l < 3 && !(AZ_W4_EXP & 16)) read_a<G>(an, cur, l + 1, S.aoff);  // this chunk's: kept
    if (l < 3 && (AZ_W4_EXP & 16)) {
#pragma unroll
      for (int t = 0; t < G::NRT; ++t) an[t] = S.af[t];
    }
    const int slot = (4 * PAR + l) % G::RING;  // = step % RING (folds: l is unrolled)
    if (!(AZ_W4_EXP & 4)) {
      if (AZ_W4_PRIO == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int t = 0; t < G::NRT; ++t) mma<G, FIRST>(S.acc[l][t], S.af[t], S.bf[slot]);
      if (AZ_W4_PRIO == 2) __builtin_amdgcn_s_setprio(0);
    }
    if (l == 0 && !(AZ_W4_EXP & 2) && !NO_NEXT) {
      // chunk L+1's window rows (requested right after the previous barrier) combined
      // behind step 0's MFMAs
#pragma unroll
      for (int u = 0; u < G::TPT; ++u) {
        if constexpr (RSD)
          combine_kx<KR < 4 ? KR : 3>(S.rk[u], S.dr[u], S.vsc[u], S.xm[u]);
        else if constexpr (CT)
          combine_k<KR < 4 ? KR : 3>(S.rk[u], S.dr[u], S.vsc[u]);
        else
          combine_rows(S.rk[u], S.dr[u], Lr);
      }
    }
    if (!(AZ_W4_EXP & 1) && (!(AZ_W4_EXP & 32) || S.tid < 256) && !(NO_NEXT && l + G::PD >= 4)) {
      if constexpr (AZ_W4_DIET)
        load_b<G>(S.bf[(slot + G::PD) % G::RING], S.rw, S.wlane, qmap<G>(S, v * 4 + l + G::PD));
      else
        load_b<G>(S.bf[(slot + G::PD) % G::RING], S.wq, S.wlane, qmap<G>(S, v * 4 + l + G::PD));
    }
    // the chunk-after-next's input slice at the chunk's first step: four steps of latency
    // cover before it is stored to LDS at the chunk's end
    if (l == 0 && !(AZ_W4_EXP & 2) && !(AZ_W4_EXP & 64) && !NO_IN) {
      if constexpr (AZ_W4_DIET)
        load_in<G>(S.ld[set_l], S.rx, S.goff, Ll);
      else
        load_in<G>(S.ld[set_l], S.x, S.goff, Ll);
    }
    if constexpr (STAGE >= 0) {
      if constexpr (RSD) {
        if (l == 1) res_dma_x<G, STAGE>(S, L & 7);
      } else {
        if (l == 1) res_dma<G, STAGE>(S, L & 7);
      }
    }
#pragma unroll
    for (int u = 0; u < G::TPT && !(AZ_W4_EXP & 2) && !NO_NEXT; ++u) {
      const float vs = CT ? 1.0f : S.vsc[u];  // CT: the scale is in rk already
      if (l == 0) put_point<G, 0>(nxt, S.rk[u], S.soff[u], vs);
      if (l == 1) put_point<G, 1>(nxt, S.rk[u], S.soff[u], vs);
      if (l == 2) put_point<G, 2>(nxt, S.rk[u], S.soff[u], vs);
      if (l == 3) put_point<G, 3>(nxt, S.rk[u], S.soff[u], vs);
    }
    if (l < 3) {
#pragma unroll
      for (int t = 0; t < G::NRT; ++t) S.af[t] = an[t];
    }
#if AZ_W4_SCHED
    // interleave: each MFMA followed by a share of the step's VALU and one LDS access, the
    // global loads behind (compile-time instruction placement; the step ends at a barrier)
#pragma unroll
    for (int i = 0; i < 2 * G::NRT * (G::MODE == AZ_CONV_SPLIT3 ? 6 : 1); ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, AZ_W4_SCHED, 0);  // VALU
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
    }
    __builtin_amdgcn_sched_group_barrier(0x020, 8, 0);  // VMEM read
#endif
    __builtin_amdgcn_sched_barrier(0);
  }
  // slot (v+2) & 1 = v & 1 held chunk v's input, whose rows were formed in chunk v-1
  if (!(AZ_W4_EXP & 2) && !(AZ_W4_EXP & 64) && !NO_IN) store_in<G>(S.lds + G::IN_OFF + (v & 1) * G::IN_SLOT, S.ld[set_s], S.ldst);
  W4C_STAMP(v, 1);
  if (!(AZ_W4_EXP & 8)) lds_barrier();
  W4C_STAMP(v, 2);
  if (!NO_NEXT) read_a<G>(S.af, nxt, 0, S.aoff);
  // the next chunk's window rows (chunk L+2, stored just before the barrier)
#pragma unroll
  for (int u = 0; u < G::TPT && !(AZ_W4_EXP & 2) && !NO_WIN; ++u) {
    if constexpr (RSD)
      read_rows_x<G, KS < 4 ? KS : 3>(S.dr[u], S.lds, S.xb[u], Ls & 7);
    else if constexpr (CT)
      read_rows_k<G, KS < 4 ? KS : 3, PAR>(S.dr[u], S.lds, S.cbase[u]);
    else
      read_rows<G>(S.dr[u], S.lds + G::IN_OFF + (v & 1) * G::IN_SLOT, S.rbase[u], S.cols[u], Ls);
  }
  if constexpr (RDMA >= 0) {
#pragma unroll
    for (int c = 0; c < 8; ++c) res_dma_x<G, RDMA>(S, c);
  }
}

// groups whose first chunk starts the accumulators itself (mma<G, true>): the whole-K
// kernel with its first chunk pair peeled (AZ_W4_ZF, default on; 0 = the zeroing pass).
// Not split3: its six-product body grew and measured 15 % slower peeled (63 -> 73 us)
#ifndef AZ_W4_ZF
#define AZ_W4_ZF 1
#endif
template <class G>
constexpr bool zero_free() {
  return AZ_W4_ZF && AZ_W4_DIET && !G::SPLIT && G::NC >= 4 && G::MODE != AZ_CONV_SPLIT3;
}

template <class G>
__device__ __forceinline__ void zero_acc(St<G>& S) {
#pragma unroll
  for (int l = 0; l < 4; ++l)
#pragma unroll
    for (int t = 0; t < G::NRT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) S.acc[l][t][e] = 0.0f;
}

// transform-grid row K (compile time): its eight chunks (staging residual half STAGE, or
// none for -1), then the fold
template <class G, int K, int STAGE = -1, bool RSD = false, int RDMA = -1>
__device__ __forceinline__ void run_group(St<G>& S) {
  static_assert(!RSD || zero_free<G>(), "resident input: the zero-free whole-K kernel only");
  constexpr int KV = G::NG == 4 ? K : 0;  // the group's place in this workgroup's sequence
  if constexpr (G::NC == 1) {
    run_chunk<G, KV & 1, STAGE>(S, KV);  // one chunk per group: the parity alternates by group
  } else if constexpr (zero_free<G>()) {
    // the whole-K kernel: chunks v = 8K + c; the rows combined in chunk v are chunk v+1's,
    // the windows read at its end chunk v+2's -- both in group K except in the last pair,
    // peeled so every group index is a compile-time constant; the first pair peeled too,
    // its first chunk's products starting the accumulators from C = 0
    constexpr int KN = K + 1;
    run_chunk<G, 0, STAGE, K, K, true, 0, RSD>(S, KV * G::NC);
    run_chunk<G, 1, STAGE, K, K, false, 0, RSD>(S, KV * G::NC + 1);
#pragma unroll 1
    for (int c = 2; c < G::NC - 2; c += 2) {
      run_chunk<G, 0, STAGE, K, K, false, 0, RSD>(S, KV * G::NC + c);
      run_chunk<G, 1, STAGE, K, K, false, 0, RSD>(S, KV * G::NC + c + 1);
    }
    constexpr int T1 = AZ_W4_TAIL && K == 3 ? 1 : 0, T2 = AZ_W4_TAIL && K == 3 ? 2 : 0;
    run_chunk<G, 0, STAGE, K, KN, false, T1, RSD, RDMA>(S, KV * G::NC + G::NC - 2);
    run_chunk<G, 1, STAGE, KN, KN, false, T2, RSD>(S, KV * G::NC + G::NC - 1);
  } else if constexpr (AZ_W4_DIET && !G::SPLIT) {
    constexpr int KN = K + 1;
#pragma unroll 1
    for (int c = 0; c < G::NC - 2; c += 2) {
      run_chunk<G, 0, STAGE, K, K>(S, KV * G::NC + c);
      run_chunk<G, 1, STAGE, K, K>(S, KV * G::NC + c + 1);
    }
    run_chunk<G, 0, STAGE, K, KN>(S, KV * G::NC + G::NC - 2);
    run_chunk<G, 1, STAGE, KN, KN>(S, KV * G::NC + G::NC - 1);
  } else {
#pragma unroll 1
    for (int c = 0; c < G::NC; c += 2) {
      run_chunk<G, 0, STAGE>(S, KV * G::NC + c);
      run_chunk<G, 1, STAGE>(S, KV * G::NC + c + 1);
    }
  }
  fold<G, K>(S.acc, S.Y);
  if constexpr (!zero_free<G>()) zero_acc<G>(S);
}

template <class G>
struct Epi {
  float unsc[2 * G::NRT];  // per board of the wave's row tiles: tile 32t + ... -> 2t + (e >= 8)
  float bmax[2 * G::NRT];
  float bv;
  int co;
};

// output half I (rows 2ty + I): accumulator element e of row tile rt = tile 32rt + (e&3) +
// 8(e>>2) + 4h, column co; Y[I][j] = output (2ty + I, 2tx + j); + bias (+ the staged
// residual), ReLU, store, and the boards' max |y|
// RST: the residual is staged in LDS (else read from global memory); NOY: the output is not
// stored to global memory (the resident trunk's conv1 outputs: only the next conv reads them,
// from X)
template <class G, int I, bool RES, bool RELU, bool HEADS = false, bool KEEP = false,
          bool RST = G::RES_FITS, bool NOY = false, bool RXS = false>
__device__ __forceinline__ void epilogue(St<G>& S, Epi<G>& E, const float* __restrict__ res,
                                         float* __restrict__ y, int rt0, int h) {
  constexpr int C = G::C;
#pragma unroll
  for (int t = 0; t < G::NRT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int T = 32 * (rt0 + t) + (e & 3) + 8 * (e >> 2) + 4 * h;
      const int bd = T >> 4, ty = (T >> 2) & 3, tx = T & 3;
      if (bd >= S.nb) continue;
#if AZ_W4_EPI_PK
      // the output pair (2tx, 2tx + 1) of row 2ty + I shares its scale, bias and column: one
      // v_pk_fma_f32 for scale + bias (the power-of-two scaling is exact, so the fused form
      // rounds like the product then the sum), one packed residual add
      if constexpr (!HEADS && G::SCALED && (!RES || RST)) {
        const float u = E.unsc[2 * t + (e >> 3)];
        f32x2 v = __builtin_elementwise_fma(f32x2{S.Y[I][0][t][e], S.Y[I][1][t][e]},
                                            f32x2{u, u}, f32x2{E.bv, E.bv});
        if constexpr (RES) {
          const float* rp = reinterpret_cast<const float*>(
              RXS ? S.lds + G::XOFF + ((bd * 64 + (2 * ty + 1) * 8 + 2 * tx) * C + E.co) * 4
                  : S.lds + G::RES_OFF + (((bd * 4 + ty) * 8 + 2 * tx) * C + E.co) * 4);
          v = v + f32x2{rp[0], rp[C]};
        }
        if (RELU) {
          v.x = fmaxf(v.x, 0.0f);
          v.y = fmaxf(v.y, 0.0f);
        }
        float* yp = &y[((size_t)(S.b0 + bd) * 64 + (2 * ty + I) * 8 + 2 * tx) * C + E.co];
        if (!NOY && !((AZ_W4_EXP & 128) && !RES)) {
          yp[0] = v.x;
          yp[C] = v.y;
        }
        if constexpr (KEEP) {
          S.Y[I][0][t][e] = v.x;
          S.Y[I][1][t][e] = v.y;
        }
        E.bmax[2 * t + (e >> 3)] = fmaxf(E.bmax[2 * t + (e >> 3)], fmaxf(fabsf(v.x), fabsf(v.y)));
        continue;
      }
#endif
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pos = (2 * ty + I) * 8 + 2 * tx + j;
        float v = (G::SCALED ? S.Y[I][j][t][e] * E.unsc[2 * t + (e >> 3)] : S.Y[I][j][t][e]) + E.bv;
        if (RES && RST)
          v += *reinterpret_cast<const float*>(
              RXS ? S.lds + G::XOFF + ((bd * 64 + (2 * ty + 1) * 8 + 2 * tx + j) * C + E.co) * 4
                  : S.lds + G::RES_OFF + (((bd * 4 + ty) * 8 + 2 * tx + j) * C + E.co) * 4);
        else if (RES && !(AZ_W4_EXP & 256))
          v += res[((size_t)(S.b0 + bd) * 64 + pos) * C + E.co];
        if (RELU) v = fmaxf(v, 0.0f);
        if constexpr (HEADS) {  // kept for the fused heads (heads_epilogue), not stored
          S.Y[I][j][t][e] = v;
        } else {
          if constexpr (NOY) {
          } else if constexpr ((AZ_W4_NT & 2) != 0)
            __builtin_nontemporal_store(v, &y[((size_t)(S.b0 + bd) * 64 + pos) * C + E.co]);
          else
            y[((size_t)(S.b0 + bd) * 64 + pos) * C + E.co] = v;
          if constexpr (KEEP) S.Y[I][j][t][e] = v;
          E.bmax[2 * t + (e >> 3)] = fmaxf(E.bmax[2 * t + (e >> 3)], fabsf(v));
        }
      }
    }
}

// The heads' inputs and outputs (az_conv3x3_wino4_heads_gpu); unused otherwise.
struct HeadsOut {
  azh::Weights w;
  float* priors;
  float* values;
};

// Last trunk conv with AlphaZeroNet's heads fused (HEADS): both output halves, final
// (bias, residual, ReLU) in the Y registers, go to an LDS image of the workgroup's NB boards
// [board][square][C] fp32 (NB x 32 KiB over the loop's buffers, free after the barrier), and
// waves 0-3 run the heads on it (heads_az.h: the same code, FC quarters and summation order
// as the stand-alone heads kernel on the same values, so priors and values are
// bit-identical to that path) while the trunk output never goes to global memory.  NB = 2:
// the two-board workgroup of the default trunk conv (four waves, two workgroups per CU);
// NB = 4: the four-board workgroup (eight waves, waves 4-7 only meet the barriers).
template <class G>
__device__ __forceinline__ void heads_epilogue(St<G>& S, const HeadsOut& ho, int rt0, int h,
                                               int co) {
  constexpr int C = G::C, NB = G::BOARDS;
  constexpr int IMG = NB * 64 * C * 4;  // the image; p [NB][128] and v [NB][64] after it
  static_assert(NB <= azh::kQuarters && G::THREADS >= 64 * azh::kQuarters, "heads layout");
  // (the FP16 heads conv runs only as the resident trunk's last layer, in TRUNK_LDS)
  static_assert(IMG + NB * (128 + 64) * 4 <= (G::SCALED ? G::LDS_BYTES : G::TRUNK_LDS),
                "heads LDS");
  // the partial sums (lp at 0, hv at 4,352) overlay the image's first board, written after
  // heads_four's first barrier, when no wave reads the image any more
  static_assert(azh::kQuarters * NB * 65 * 4 <= 4352 &&
                    4352 + azh::kQuarters * NB * 64 * 16 <= IMG,
                "heads scratch inside the image");
  float* img = reinterpret_cast<float*>(S.lds);
  __syncthreads();  // every wave is past its loop and its staged-residual reads
#pragma unroll
  for (int t = 0; t < G::NRT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int T = 32 * (rt0 + t) + (e & 3) + 8 * (e >> 2) + 4 * h;
      const int bd = T >> 4, ty = (T >> 2) & 3, tx = T & 3;
      if (bd >= S.nb) continue;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          img[(bd * 64 + (2 * ty + i) * 8 + 2 * tx + j) * C + co] = S.Y[i][j][t][e];
    }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool active = wave < azh::kQuarters, live = wave < NB && wave < S.nb;
  // a missing board (last workgroup) or a quarter-only wave reads board 0's row: computed
  // by the 1x1 convs only for waves < NB, never stored
  const float4* hp =
      reinterpret_cast<const float4*>(img + ((live ? wave : 0) * 64 + lane) * C);
  char* base = S.lds;
  const azh::ScratchT<NB> L{reinterpret_cast<float(*)[128]>(base + IMG),
                            reinterpret_cast<float(*)[64]>(base + IMG + NB * 128 * 4),
                            reinterpret_cast<float(*)[NB][65]>(base),
                            reinterpret_cast<float4(*)[NB][64]>(base + 4352)};
  azh::heads_four<C, NB>([&](int c) { return hp[c]; }, lane, wave & (azh::kQuarters - 1),
                         S.b0 + wave, live, active, ho.w, L, ho.priors, ho.values);
}

// One conv of this workgroup's boards (the whole kernel of k_conv3x3_wino4; the persistent
// trunk k_trunk_wino4 runs it once per layer on the same boards).
// HIN / HOUT (AZ_W4_HANDOFF, the persistent trunk's layers): HIN = the input's first two
// slices are already in the input slots and its per-board ranges in LDS (written by the
// previous layer's HOUT epilogue, ordered by the layer fence); HOUT = write them for the next
// layer.  Two-board, one-row-tile form only (the trunk's).
// RSD (AZ_W4_RESIDENT, the persistent trunk's layers instead of the hand-off): the layer's whole
// input is resident in LDS (X, G::XOFF) -- XFILL = load it from x first (a launch's first
// conv), else the previous layer wrote it; XOUT = write this layer's output there after the
// last window read (ordered by the layer fence).  No input slices are loaded or stored per
// chunk; the residual is read from global memory in the epilogue (no LDS left to stage it);
// a conv1 output with XOUT is not stored to global memory at all (only the next conv reads it).
template <class G, bool RES, bool RELU, bool HEADS = false, bool LAUNDER = false,
          bool HIN = false, bool HOUT = false, bool RSD = false, bool XFILL = false,
          bool XOUT = false>
__device__ __forceinline__ void conv_body(
    const float* __restrict__ x, const char* __restrict__ wq, const float* __restrict__ bias,
    const float* __restrict__ res, float* __restrict__ y, int n_boards,
    float* __restrict__ in_absmax, float* __restrict__ out_absmax, HeadsOut ho,
    int layer = 0) {
  constexpr int C = G::C;
  static_assert(!(HIN || HOUT) || (G::BOARDS == 2 && G::NRT == 1 && G::IPD == 1 && G::SCALED &&
                                   !G::SPLIT && LAUNDER),
                "the layer hand-off is the persistent two-board fp16x2 trunk's");
  static_assert(!(RSD || XFILL || XOUT) ||
                    (RSD && !HIN && !HOUT && (G::BOARDS == 2 || G::BOARDS == 4) && G::NRT == 1 &&
                     (G::SCALED || G::MODE == AZ_CONV_FP16) &&
                     !G::SPLIT && LAUNDER && AZ_W4_DIET && C == 128),
                "the resident input is the persistent two-board fp16x2 / fp16 trunk's");
  constexpr bool NOY = RSD && XOUT && !RES && !HEADS;

  extern __shared__ float4 lds4[];
  W4_STAMP(0);
  W4T_STAMP(layer, 0);
  St<G> S;
  S.lds = reinterpret_cast<char*>(lds4);
  S.x = x;
  S.wq = wq;
  if constexpr (AZ_W4_DIET) {
    const long long xb = (long long)n_boards * 64 * C * 4;
    S.rx = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, xb < 0x7fffffff ? (int)xb : 0x7fffffff,
                                             0x00020000);
    S.rw = __builtin_amdgcn_make_buffer_rsrc((void*)wq, 0, G::QSTEPS * G::STEP_BYTES, 0x00020000);
  }
  S.res = res;
  // laundered: the persistent trunk runs this body once per layer, and everything derived
  // from the lane index hoisted out of its layer loop would stay live across both bodies
  int tid = threadIdx.x;
  if constexpr (LAUNDER) asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = wave & 3, rt0 = G::NRT == 1 ? wave >> 2 : 0;
  const int r = lane & 31, h = lane >> 5;
  const int col0 = 32 * cb;
  const int b0 = blockIdx.x * G::BOARDS;
  const int nb = n_boards - b0 < G::BOARDS ? n_boards - b0 : G::BOARDS;
  // the input range of board bd (< nb): from the previous layer's LDS hand-off (the max of
  // its waves' maxima: the value the buffer's atomics hold), else the buffer
  auto in_range = [&](int bd) -> float {
    if constexpr (HIN) {
      const float* rng = reinterpret_cast<const float*>(S.lds + G::RNG_OFF);
      float m = rng[bd];
#pragma unroll
      for (int w = 1; w < G::WAVES; ++w) m = fmaxf(m, rng[w * 4 + bd]);
      return m;
    } else {
      return in_absmax[b0 + bd];
    }
  };
  S.tid = tid;
  S.b0 = b0;
  S.nb = nb;
  S.cs = G::SPLIT ? (int)(blockIdx.y % (G::CHUNKS / G::NC)) * G::NC : 0;
  S.g0 = G::NG == 1 ? (int)(blockIdx.y / (G::CHUNKS / G::NC)) : 0;
  if constexpr (G::SPLIT) y += (size_t)blockIdx.y * n_boards * 64 * C;  // this split's partials
  S.lds_res = (unsigned)(uintptr_t)(S.lds + (RSD ? G::XOFF : G::RES_OFF)) +
              16 * 64 * (RSD ? (wave & 3) : wave);
  S.wlane = (col0 + r) * 32 + h * 16;
#pragma unroll
  for (int t = 0; t < G::NRT; ++t)
    S.aoff[t] = (32 * (rt0 + t) + r) * 32 + ((h ^ ((r >> 3) & 1)) << 4);

  // transform items u: tile T = tid / 8 + u * THREADS / 8 (board T / 16, tile row
  // (T / 4) % 4, tile column T % 4), channel pair p = tid % 8 of each 16-channel chunk;
  // the window's top-left entry in the padded slot is position (2ty, 2tx)
#pragma unroll
  for (int u = 0; u < G::TPT; ++u) {
    const int T = (tid >> 3) + u * (G::THREADS / 8), p = tid & 7;
    const int bd = T >> 4, ty = (T >> 2) & 3, tx = T & 3;
    S.rbase[u] = bd * G::IN_BOARD + 2 * ty * G::IN_ROW + p * 8;
    S.cols[u] = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) S.cols[u] |= col_slot(2 * tx + b) << (8 * b);
    S.soff[u] = T * 32 + (((p >> 2) ^ ((T >> 3) & 1)) << 4) + (p & 3) * 4;
#pragma unroll
    for (int b = 0; b < 4; ++b) S.cbase[u][b] = S.rbase[u] + col_slot(2 * tx + b) * 64;
    S.vsc[u] = 1.0f;
    if constexpr (G::SCALED) {
      // |V| <= 4 max |x| < 2^(e+2): scaled by 2^(13-e), the transformed inputs stay below
      // 2^15 (fp16's largest power of two)
      const int e = frexp_exp(bd < nb ? in_range(bd) : 0.0f);
      S.vsc[u] = ldexpf(1.0f, 13 - e);
    }
    if constexpr (RSD) {
      // X byte offset of the window's row 2ty - 1, column 2tx - 1 + b (chunk 0's slot; both
      // may be off the board -- negative for the first board's top-left tile), channel pair p
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int col = 2 * tx - 1 + b;
        S.xb[u][b] = (bd * 64 + (2 * ty - 1) * 8 + col) * (C * 4) + (((col >> 1) & 3) << 6) + p * 8;
      }
      S.xm[u][0] = ty == 0 ? 0.0f : 1.0f;
      S.xm[u][1] = ty == 3 ? 0.0f : 1.0f;
      S.xm[u][2] = tx == 0 ? 0.0f : 1.0f;
      S.xm[u][3] = tx == 3 ? 0.0f : 1.0f;
    }
  }
  // input loads: element e = j * THREADS + tid -> position P = e / 4 (board P / 64, clamped
  // to the last valid board: rows of absent boards are computed but never stored),
  // channel quad e % 4 of the chunk
#pragma unroll
  for (int j = 0; j < G::LD_PER_THREAD; ++j) {
    // lanes 4i..4i+3 load position P; positions of a 4-aligned group are visited in the
    // order 0, 2, 1, 3 so each 8-lane store group writes columns (c, c + 2) (col_slot)
    const int e = j * G::THREADS + tid, P0 = e >> 2, q = e & 3;
    const int P = (P0 & ~3) | ((P0 & 1) << 1) | ((P0 >> 1) & 1);
    const int bd = P >> 6, pos = P & 63;
    const int bs = bd < nb ? bd : nb - 1;
    S.goff[j] = (((b0 + bs) * 64 + pos) * C + 4 * q) * (AZ_W4_DIET ? 4 : 1);  // DIET: bytes
    S.ldst[j] = bd * G::IN_BOARD + ((pos >> 3) + 1) * G::IN_ROW + col_slot((pos & 7) + 1) * 64 + q * 16;
  }

  // ---- prologue: zero both input slots (their borders stay zero), chunk 0 and 1 slices and
  // the first weight steps in flight together; chunk 0 transformed into V buffer 0
  // (the persistent trunk's later layers: the borders are still zero -- interior stores never
  // touch them -- and the layer fence ordered the previous layer's reads)
  const bool fill = !LAUNDER || layer == 0;
  if constexpr (RSD) {
    if constexpr (XFILL) {
      // V buffers zeroed (a board-edge window reads some of their words: finite from here on),
      // and the whole input into X: 16 loads of 16 bytes per thread, in two halves
#pragma unroll
      for (int i = tid * 16; i < G::VPAD; i += G::THREADS * 16) {
        *reinterpret_cast<f32x4*>(S.lds + i) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        *reinterpret_cast<f32x4*>(S.lds + G::V1R + i) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      int xst[G::LD_PER_THREAD];  // X offset of load element j in chunk 0's slot
#pragma unroll
      for (int j = 0; j < G::LD_PER_THREAD; ++j) {
        const int e = j * G::THREADS + tid, P0 = e >> 2, q = e & 3;
        const int P = (P0 & ~3) | ((P0 & 1) << 1) | ((P0 >> 1) & 1);
        xst[j] = xoff<G>(P >> 6, P & 63, 4 * q);
      }
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        f32x4 xl[4][G::LD_PER_THREAD];
#pragma unroll
        for (int c = 0; c < 4; ++c) load_in<G>(xl[c], S.rx, S.goff, 4 * half + c);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int j = 0; j < G::LD_PER_THREAD; ++j)
            *reinterpret_cast<f32x4*>(S.lds + G::XOFF + (xst[j] ^ ((4 * half + c) << 6))) = xl[c][j];
      }
    }
#pragma unroll
    for (int i = 0; i < G::PD; ++i) load_b<G>(S.bf[i], S.rw, S.wlane, qmap<G>(S, i));
    if constexpr (XFILL) lds_barrier();  // X and the zeroed V buffers complete
#pragma unroll
    for (int u = 0; u < G::TPT; ++u) {
      f32x2 d[8];
      read_rows_x<G, 0>(d, S.lds, S.xb[u], 0);
      combine_kx<0>(S.rk[u], d, S.vsc[u], S.xm[u]);
    }
  } else if constexpr (HIN) {
    // chunks 0 and 1 are in the slots already (the previous layer's hand-off, ordered by the
    // layer fence); chunk 2's slice (stored at the end of chunk 0) and the first weight steps
    char* in0 = S.lds + G::IN_OFF;
    load_in<G>(S.ld[0], S.rx, S.goff, lmap<G>(S, 2));
#pragma unroll
    for (int i = 0; i < G::PD; ++i) load_b<G>(S.bf[i], S.rw, S.wlane, qmap<G>(S, i));
#pragma unroll
    for (int u = 0; u < G::TPT; ++u) make_rows<G>(S.rk[u], in0, S.rbase[u], S.cols[u], lmap<G>(S, 0));
  } else {
    char* in0 = S.lds + G::IN_OFF;
    if (fill)
      for (int i = tid * 16; i < 2 * G::IN_SLOT; i += G::THREADS * 16)
        *reinterpret_cast<f32x4*>(in0 + i) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    f32x4 ld0[G::LD_PER_THREAD], ld1[G::LD_PER_THREAD];
    if constexpr (AZ_W4_DIET) {
      load_in<G>(ld0, S.rx, S.goff, lmap<G>(S, 0));
      load_in<G>(G::IPD == 1 ? S.ld[0] : ld1, S.rx, S.goff, lmap<G>(S, 1));
      if (G::IPD == 2) load_in<G>(S.ld[0], S.rx, S.goff, lmap<G>(S, 2));
#pragma unroll
      for (int i = 0; i < G::PD; ++i) load_b<G>(S.bf[i], S.rw, S.wlane, qmap<G>(S, i));
    } else {
      load_in<G>(ld0, x, S.goff, lmap<G>(S, 0));
      load_in<G>(G::IPD == 1 ? S.ld[0] : ld1, x, S.goff, lmap<G>(S, 1));
      if (G::IPD == 2) load_in<G>(S.ld[0], x, S.goff, lmap<G>(S, 2));  // stored at the end of chunk 0
#pragma unroll
      for (int i = 0; i < G::PD; ++i) load_b<G>(S.bf[i], wq, S.wlane, qmap<G>(S, i));
    }
    if (fill) lds_barrier();  // the zero fill before any interior store
    store_in<G>(in0, ld0, S.ldst);
    store_in<G>(in0 + G::IN_SLOT, G::IPD == 1 ? S.ld[0] : ld1, S.ldst);
    if (G::IPD == 1) {  // stored at the end of chunk 0
      if constexpr (AZ_W4_DIET)
        load_in<G>(S.ld[0], S.rx, S.goff, lmap<G>(S, 2));
      else
        load_in<G>(S.ld[0], x, S.goff, lmap<G>(S, 2));
    }
    lds_barrier();
#pragma unroll
    for (int u = 0; u < G::TPT; ++u) make_rows<G>(S.rk[u], in0, S.rbase[u], S.cols[u], lmap<G>(S, 0));
  }
#pragma unroll
  for (int u = 0; u < G::TPT; ++u) {
    const float vs = RSD ? 1.0f : S.vsc[u];  // RSD: the scale is in rk already
    put_point<G, 0>(S.lds, S.rk[u], S.soff[u], vs);
    put_point<G, 1>(S.lds, S.rk[u], S.soff[u], vs);
    put_point<G, 2>(S.lds, S.rk[u], S.soff[u], vs);
    put_point<G, 3>(S.lds, S.rk[u], S.soff[u], vs);
  }
  lds_barrier();

  if constexpr (!zero_free<G>()) zero_acc<G>(S);
  read_a<G>(S.af, S.lds, 0, S.aoff);
#pragma unroll
  for (int u = 0; u < G::TPT; ++u) {
    if constexpr (RSD)
      read_rows_x<G, 0>(S.dr[u], S.lds, S.xb[u], 1);
    else
      read_rows<G>(S.dr[u], S.lds + G::IN_OFF + G::IN_SLOT, S.rbase[u], S.cols[u], lmap<G>(S, 1));
  }
  // epilogue constants: bias, and (FP16X2) the scale M carries, 2^(su + sv_board); removing
  // it is an exact power-of-two product
  Epi<G> E;
  E.co = col0 + r;
  E.bv = G::SPLIT ? 0.0f : bias[E.co];  // split partials: bias etc. in the combining kernel
#pragma unroll
  for (int i = 0; i < 2 * G::NRT; ++i) {
    E.unsc[i] = 1.0f;
    E.bmax[i] = 0.0f;
  }
  if constexpr (G::SCALED) {
    const int su = reinterpret_cast<const int*>(wq + (size_t)G::QSTEPS * G::STEP_BYTES)[1];
#pragma unroll
    for (int i = 0; i < 2 * G::NRT; ++i) {
      const int bd = 2 * rt0 + i;
      const int e = frexp_exp(bd < nb ? in_range(bd) : 0.0f);
      E.unsc[i] = ldexpf(1.0f, -(su + 13 - e));
    }
  }
  W4_STAMP(1);
  W4T_STAMP(layer, 1);
  if (AZ_W4_PRIO == 1 && G::WAVES == 8 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256)
    __builtin_amdgcn_s_setprio(1);
  if constexpr (G::NG == 1) {  // one transform row: its partial outputs, both halves
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < G::NRT; ++t)
#pragma unroll
          for (int e = 0; e < 16; ++e) S.Y[i][j][t][e] = 0.0f;
    switch (S.g0) {
      case 0: run_group<G, 0>(S); break;
      case 1: run_group<G, 1>(S); break;
      case 2: run_group<G, 2>(S); break;
      default: run_group<G, 3>(S); break;
    }
    epilogue<G, 0, false, false>(S, E, res, y, rt0, h);
    epilogue<G, 1, false, false>(S, E, res, y, rt0, h);
    return;
  } else {
  run_group<G, 0, -1, RSD>(S);
  W4_STAMP(2);
  run_group<G, 1, -1, RSD>(S);
  W4_STAMP(3);
  // output rows 2ty (Y[0]) are final after group 2: stored while group 3 computes, with
  // their residual staged through LDS during group 2 (and the odd rows' during group 3)
  // the resident trunk stages its residual in X's odd rows instead (AZ_W4_RXS)
  constexpr bool SX = RSD && RES && AZ_W4_RXS;
  constexpr bool STAGED = (RES && G::RES_FITS && !G::SPLIT && !RSD) || SX;
  constexpr bool KEEPY = HOUT || XOUT;
  run_group<G, 2, STAGED && !SX ? 0 : -1, RSD, SX ? 0 : -1>(S);
  W4_STAMP(4);
  W4T_STAMP(layer, 2);
  if (STAGED) vm_barrier();  // the even-row residual has landed in LDS
  epilogue<G, 0, RES, RELU, HEADS, KEEPY, STAGED, NOY, SX>(S, E, res, y, rt0, h);
  if (STAGED) lds_barrier();  // every wave's even-row residual reads before the odd rows land
  run_group<G, 3, STAGED ? 1 : -1, RSD>(S);
  W4_STAMP(5);
  if (STAGED) vm_barrier();
  epilogue<G, 1, RES, RELU, HEADS, KEEPY, STAGED, NOY, SX>(S, E, res, y, rt0, h);
  if constexpr (SX && XOUT) lds_barrier();  // every wave's odd-row residual reads, then X rewritten
  if constexpr (XOUT && !(AZ_W4_EXP & 512)) {
    // the next layer's input, whole, into X: every window read of this layer's X was issued
    // before the second-to-last chunk's barrier (the tail chunks read none) and completed
    // before the last chunk's; the layer fence orders these stores before the next reads.
    // Element e of half i: tile T = 32 rt0 + (e & 3) + 8 (e >> 2) + 4 h -> board 2 rt0 + (e >> 3), tile column
    // e & 3, tile row (2 (e >> 2) + h) & 3; column slot swizzle (2tx + j) >> 1 = tx
    const int cpart = ((E.co >> 4) << 6) | ((E.co & 15) << 2);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int bd = 2 * rt0 + (e >> 3), tx = e & 3, ty = (2 * (e >> 2) + h) & 3;
        if (bd >= nb) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int pos = (2 * ty + i) * 8 + 2 * tx + j;
          *reinterpret_cast<float*>(S.lds + G::XOFF + (bd * 64 + pos) * (C * 4) +
                                    (cpart ^ (tx << 6))) = S.Y[i][j][0][e];
        }
      }
  }
  if constexpr (HOUT) {
    // the next layer's input: its first two slices (channels 0-31 = column block 0's
    // registers) into the input slots -- free since the last chunk's windows were read,
    // before this layer's last two barriers -- and each wave's per-board max |y|
    if (cb == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int T = (e & 3) + 8 * (e >> 2) + 4 * h;
          const int bd = T >> 4, ty = (T >> 2) & 3, tx = T & 3;
          if (bd >= nb) continue;
#pragma unroll
          for (int j = 0; j < 2; ++j)
            *reinterpret_cast<float*>(S.lds + G::IN_OFF + (r >> 4) * G::IN_SLOT + bd * G::IN_BOARD +
                                      (2 * ty + i + 1) * G::IN_ROW +
                                      col_slot(2 * tx + j + 1) * 64 + (r & 15) * 4) =
                S.Y[i][j][0][e];
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float m = E.bmax[i];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
      if (lane == 0) reinterpret_cast<float*>(S.lds + G::RNG_OFF)[wave * 4 + i] = m;
    }
  }
  if constexpr (HEADS) {
    // in_absmax is consumed (every thread read its entries in the prologue)
    if (threadIdx.x < G::BOARDS && (int)threadIdx.x < nb) in_absmax[b0 + threadIdx.x] = 0.0f;
    heads_epilogue<G>(S, ho, rt0, h, E.co);
    return;
  }
  if (out_absmax && !HOUT) {  // the next layer's in_absmax: one atomic per (wave, board)
#pragma unroll
    for (int i = 0; i < 2 * G::NRT; ++i) {
      float m = E.bmax[i];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
      const int bd = 2 * rt0 + i;
      if (lane == 0 && bd < nb)
        atomicMax(reinterpret_cast<unsigned*>(out_absmax) + b0 + bd, __float_as_uint(m));
    }
  }
  // in_absmax is consumed: reset for its next use as some layer's out_absmax (every thread
  // read its entries in the prologue, before the first barrier)
  if (G::SCALED && !G::SPLIT && tid < G::BOARDS && tid < nb) in_absmax[b0 + tid] = 0.0f;
  W4_STAMP(6);
  W4T_STAMP(layer, 3);
  }
}

template <class G, bool RES, bool RELU, bool HEADS = false>
__global__ __launch_bounds__(G::THREADS, 2 / G::NRT) void k_conv3x3_wino4(
    const float* __restrict__ x, const char* __restrict__ wq, const float* __restrict__ bias,
    const float* __restrict__ res, float* __restrict__ y, int n_boards,
    float* __restrict__ in_absmax, float* __restrict__ out_absmax, HeadsOut ho) {
  conv_body<G, RES, RELU, HEADS>(x, wq, bias, res, y, n_boards, in_absmax, out_absmax, ho);
}

// Persistent trunk (az_trunk_wino4_gpu): a workgroup runs n_convs consecutive 3x3 convs of
// the residual tower on ITS boards -- conv 2i: relu(conv(h)) -> t, conv 2i+1: relu(conv(t) +
// h) -> the other block buffer -- so no layer waits for another workgroup and the 8-9
// kernel boundaries (launch gap + the slowest workgroup's tail, each layer) go.  Every
// activation a layer reads was written by this workgroup, so a barrier with its stores
// drained (vmcnt(0)) and an L1 invalidate (buffer_inv sc0: the ping-pong buffers were read
// by earlier layers) order it; per-board ranges ping-pong amax[0] / amax[1] as between the
// per-layer launches.  Same arithmetic per layer: bit-identical to those launches.
#ifndef AZ_W4_STAGGER
#define AZ_W4_STAGGER 0
#endif
struct TrunkW4 {
  const char* const* wq;     // [n_convs] prepared weights (layer order)
  const float* const* bias;  // [n_convs]
  float* h_in;               // block input (the stem's output): written only with `planes`
  float* hb[2];              // block outputs, ping-pong
  float* t;                  // conv1 outputs
  float* amax[2];            // per-board ranges: amax[0] = h_in's (on entry, or the stem's)
  const float* planes;       // optional: the stem's inputs [n][64] (h_in computed here)
  const float* stem_w;       // [9][C]
  const float* stem_b;       // [C]
  int n_boards, n_convs;
};

// a pointer loaded from device memory (the per-layer weight / bias tables) as a wave-uniform
// value: the compiler loads it with a vector load (the kernel writes global memory, so no
// scalar load) and cannot prove the result uniform, so every buffer descriptor built from it
// became divergent and each buffer load ran in a waterfall loop (v_readfirstlane /
// v_cmp_eq_u64 / s_and_saveexec per load: 1,540 readfirstlanes in the kernel, 1.7x the
// standalone conv's VALU per conv -- profiles/r04_trunk_sq_counters.txt)
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ void layer_fence() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier\n\tbuffer_inv sc0" ::: "memory");
}

// The stem (Ci = 1 -> C = 128, 3x3, bias, ReLU) of board b by a 256-thread workgroup, and the
// board's max |y|: k_conv_stem's (conv.hip) thread mapping, tap order and fmaf chain, so the
// outputs are bit-identical to that kernel's (and to the engine stem's).  s_pl / s_max: LDS.
__device__ __forceinline__ void stem_board(const float* __restrict__ planes,
                                           const float* __restrict__ w,
                                           const float* __restrict__ bias, float* __restrict__ y,
                                           float* __restrict__ absmax, int b, float* s_pl,
                                           float* s_max) {
  constexpr int CO = 128, G4 = CO / 4, PPI = 256 / G4;
  const int tid = threadIdx.x;
  const bool act = tid < 256;  // threads 256.. of a 512-thread workgroup only meet the barriers
  const int co = (tid % G4) * 4;
  float4 wv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wv[t] = *reinterpret_cast<const float4*>(w + t * CO + co);
  const float4 bv = *reinterpret_cast<const float4*>(bias + co);
  __syncthreads();  // the previous board's planes and maxima are no longer read
  if (tid < 64) s_pl[tid] = planes[(size_t)b * 64 + tid];
  __syncthreads();
  float4* out = reinterpret_cast<float4*>(y + (size_t)b * 64 * CO);
  float bmax = 0.0f;
#pragma unroll
  for (int p0 = 0; p0 < 64 && act; p0 += PPI) {
    const int p = p0 + tid / G4, py = p >> 3, px = p & 7;
    float4 acc = bv;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
      if ((unsigned)yy < 8u && (unsigned)xx < 8u) {
        const float v = s_pl[yy * 8 + xx];
        acc.x = fmaf(v, wv[t].x, acc.x);
        acc.y = fmaf(v, wv[t].y, acc.y);
        acc.z = fmaf(v, wv[t].z, acc.z);
        acc.w = fmaf(v, wv[t].w, acc.w);
      }
    }
    acc.x = fmaxf(acc.x, 0.f);
    acc.y = fmaxf(acc.y, 0.f);
    acc.z = fmaxf(acc.z, 0.f);
    acc.w = fmaxf(acc.w, 0.f);
    out[p * G4 + co / 4] = acc;
    bmax = fmaxf(bmax, fmaxf(fmaxf(acc.x, acc.y), fmaxf(acc.z, acc.w)));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) bmax = fmaxf(bmax, __shfl_xor(bmax, off, 64));
  if ((tid & 63) == 0 && act) s_max[tid >> 6] = bmax;
  __syncthreads();
  if (tid == 0) absmax[b] = fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]));
}

// AlphaZeroNet's heads on this workgroup's NB boards of the tower's output y (just written
// by this workgroup, after a layer_fence): heads_four with each board's activations read on
// demand from y (L2), its partial sums in the workgroup's LDS -- the same code and order as
// the separate heads kernel, so bit-identical priors / values.
template <class G>
__device__ __forceinline__ void trunk_heads(const float* __restrict__ y, int n_boards,
                                            const HeadsOut& ho) {
  constexpr int C = G::C, NB = G::BOARDS;
  static_assert(NB <= azh::kQuarters && G::THREADS >= 64 * azh::kQuarters, "heads layout");
  extern __shared__ float4 lds4[];
  char* base = reinterpret_cast<char*>(lds4);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b0 = blockIdx.x * NB;
  const int nb = n_boards - b0 < NB ? n_boards - b0 : NB;
  const bool active = wave < azh::kQuarters, live = wave < NB && wave < nb;
  const float4* hp = reinterpret_cast<const float4*>(
      y + ((size_t)(b0 + (live ? wave : 0)) * 64 + lane) * C);
  // p [NB][128] at 0, v [NB][64] at 1 KiB, lp [4][NB][65] at 2 KiB, hv [4][NB][64] at 4,352
  static_assert(NB * 128 * 4 <= 1024 && 1024 + NB * 64 * 4 <= 2048 &&
                    2048 + azh::kQuarters * NB * 65 * 4 <= 4352,
                "heads scratch layout");
  const azh::ScratchT<NB> L{reinterpret_cast<float(*)[128]>(base),
                            reinterpret_cast<float(*)[64]>(base + 1024),
                            reinterpret_cast<float(*)[NB][65]>(base + 2048),
                            reinterpret_cast<float4(*)[NB][64]>(base + 4352)};
  azh::heads_four<C, NB>([&](int c) { return hp[c]; }, lane, wave & (azh::kQuarters - 1),
                         b0 + wave, live, active, ho.w, L, ho.priors, ho.values);
}

// HEADS: after the last conv (n_convs - 1, a block's second: odd; its output stored as in
// any layer) each workgroup runs AlphaZeroNet's heads on its boards (trunk_heads: priors /
// values bit-identical to az_conv3x3_wino4_heads_gpu and to the separate heads kernel) --
// the tower and the heads in one launch, no kernel boundary before the last layer.  (The
// heads in the last conv's epilogue, inlined here as a third body, spilled ~100 VGPRs into
// the layer loop.)
// AZ_W4_TRUNK_HEADS_EPI (HEADS launches): 1 = the last conv runs after the layer loop as the
// heads-fused body (heads from the accumulators, as az_conv3x3_wino4_heads_gpu; no store and
// read-back of the tower's output; 242 VGPRs, no spills): B = 1,024 evaluation 423.3 vs 424.6
// us for the tower launch + heads-fused conv launch and 431.4 for the read-back form, bench
// +0.2 %, bit-identical (profiles/r04_trunk_heads_epi_ab.json); 0 = the last conv in the loop,
// then trunk_heads (the read-back form)
#ifndef AZ_W4_TRUNK_HEADS_EPI
#define AZ_W4_TRUNK_HEADS_EPI 1
#endif
template <class G, bool HEADS = false>
__global__ __launch_bounds__(G::THREADS, 2 / G::NRT) void k_trunk_wino4(TrunkW4 a,
                                                                      HeadsOut ho) {
  constexpr bool EPI = HEADS && AZ_W4_TRUNK_HEADS_EPI;
#if AZ_W4_STAGGER
  // experiment: the second half of the grid (the second workgroup on each CU when every
  // workgroup is resident) starts later, so the two co-resident workgroups' phases differ
  if (blockIdx.x >= (gridDim.x + 1) / 2) {
    for (int i = 0; i < AZ_W4_STAGGER; ++i) __builtin_amdgcn_s_sleep(8);  // 512 clocks each
  }
#endif
  if (a.planes) {  // the stem of this workgroup's boards first (its output never leaves L2)
    static_assert(G::THREADS >= 256 && G::C == 128, "stem_board's mapping");
    extern __shared__ float4 lds4[];
    float* sp = reinterpret_cast<float*>(lds4);
    const int b0 = blockIdx.x * G::BOARDS;
    for (int bd = 0; bd < G::BOARDS && b0 + bd < a.n_boards; ++bd)
      stem_board(a.planes, a.stem_w, a.stem_b, a.h_in, a.amax[0], b0 + bd, sp, sp + 64);
    layer_fence();
  }
  const float* h = a.h_in;
  int ob = 0;
  const int n_loop = EPI ? a.n_convs - 1 : a.n_convs;
  if constexpr (AZ_W4_RESIDENT) {
    // the resident input: conv1 (even i) reads X, writes t only into X; conv2 reads t from X
    // and the residual h from global memory, writes h to global memory (the next block's
    // residual) and into X.  A launch's first conv loads X; its last writes none
    for (int i = 0; i < n_loop; ++i) {
      if (i > 0) layer_fence();
      const bool xout = i + 1 < a.n_convs;
      if ((i & 1) == 0) {
        if (i == 0 && xout)
          conv_body<G, false, true, false, true, false, false, true, true, true>(
              h, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), nullptr, a.t, a.n_boards,
              a.amax[0], a.amax[1], HeadsOut{}, i);
        else if (i == 0)
          conv_body<G, false, true, false, true, false, false, true, true, false>(
              h, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), nullptr, a.t, a.n_boards,
              a.amax[0], a.amax[1], HeadsOut{}, i);
        else if (xout)
          conv_body<G, false, true, false, true, false, false, true, false, true>(
              h, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), nullptr, a.t, a.n_boards,
              a.amax[0], a.amax[1], HeadsOut{}, i);
        else
          conv_body<G, false, true, false, true, false, false, true, false, false>(
              h, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), nullptr, a.t, a.n_boards,
              a.amax[0], a.amax[1], HeadsOut{}, i);
      } else {
        const bool last_heads = HEADS && i == a.n_convs - 1;
        if (xout)
          conv_body<G, true, true, false, true, false, false, true, false, true>(
              a.t, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), h, a.hb[ob], a.n_boards,
              a.amax[1], last_heads ? nullptr : a.amax[0], HeadsOut{}, i);
        else
          conv_body<G, true, true, false, true, false, false, true, false, false>(
              a.t, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), h, a.hb[ob], a.n_boards,
              a.amax[1], last_heads ? nullptr : a.amax[0], HeadsOut{}, i);
        h = a.hb[ob];
        ob ^= 1;
      }
    }
    if constexpr (EPI) {
      layer_fence();  // the last block's conv1 output in X, ordered for this workgroup
      const int i = a.n_convs - 1;
      conv_body<G, true, true, true, true, false, false, true, false, false>(
          a.t, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), h, nullptr, a.n_boards, a.amax[1],
          nullptr, ho, i);
    } else if constexpr (HEADS) {
      layer_fence();
      trunk_heads<G>(h, a.n_boards, ho);
    }
    return;
  }
  constexpr bool HO = AZ_W4_HANDOFF != 0 && G::BOARDS == 2 && G::SCALED;  // two-board fp16x2 only
  for (int i = 0; i < n_loop; ++i) {
    if (i > 0) layer_fence();
    // a conv whose output the next conv reads hands it off through LDS (every conv but the
    // launch's last); the first conv reads the stem's output from memory
    const bool hout = HO && (i + 1 < a.n_convs);
    if ((i & 1) == 0) {
      if (i == 0 && hout)
        conv_body<G, false, true, false, true, false, HO>(
            h, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), nullptr, a.t, a.n_boards, a.amax[0],
            a.amax[1], HeadsOut{}, i);
      else if (i == 0)
        conv_body<G, false, true, false, true>(h, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]),
                                               nullptr, a.t, a.n_boards,
                                               a.amax[0], a.amax[1], HeadsOut{}, i);
      else if (hout)
        conv_body<G, false, true, false, true, HO, HO>(
            h, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), nullptr, a.t, a.n_boards, a.amax[0],
            a.amax[1], HeadsOut{}, i);
      else
        conv_body<G, false, true, false, true, HO, false>(
            h, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), nullptr, a.t, a.n_boards, a.amax[0],
            a.amax[1], HeadsOut{}, i);
    } else {
      // the last layer of a HEADS launch keeps no range (nothing reads its output as a
      // conv input): amax[0] stays as the stem / caller left it
      const bool last_heads = HEADS && i == a.n_convs - 1;
      if (hout)
        conv_body<G, true, true, false, true, HO, HO>(
            a.t, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), h, a.hb[ob], a.n_boards, a.amax[1],
            last_heads ? nullptr : a.amax[0], HeadsOut{}, i);
      else
        conv_body<G, true, true, false, true, HO, false>(
            a.t, uniform_ptr(a.wq[i]), uniform_ptr(a.bias[i]), h, a.hb[ob], a.n_boards, a.amax[1],
            last_heads ? nullptr : a.amax[0], HeadsOut{}, i);
      h = a.hb[ob];
      ob ^= 1;
    }
  }
  if constexpr (EPI) {
    layer_fence();  // the last block's first conv output (t) visible to this workgroup
    const int i = a.n_convs - 1;
    conv_body<G, true, true, true, true, HO, false>(a.t, uniform_ptr(a.wq[i]),
                                                    uniform_ptr(a.bias[i]), h, nullptr,
                                                    a.n_boards, a.amax[1], nullptr, ho, i);
  } else if constexpr (HEADS) {
    layer_fence();  // the last layer's stores drained and visible to this workgroup's reads
    trunk_heads<G>(h, a.n_boards, ho);
  }
}

template <class G>
int launch_wino4(const float* x, const void* wq, const float* bias, const float* res, float* y,
                 int n_boards, int relu, float* in_absmax, float* out_absmax, hipStream_t s) {
  const unsigned grid = (unsigned)((n_boards + G::BOARDS - 1) / G::BOARDS);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS needs the opt-in once per kernel
  if (!attr_set) {
    const void* ks[] = {(const void*)k_conv3x3_wino4<G, true, true>,
                        (const void*)k_conv3x3_wino4<G, true, false>,
                        (const void*)k_conv3x3_wino4<G, false, true>,
                        (const void*)k_conv3x3_wino4<G, false, false>};
    for (const void* k : ks)
      AZ_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)G::LDS_BYTES));
    attr_set = true;
  }
  const char* w = static_cast<const char*>(wq);
  const dim3 blk(G::THREADS);
  const size_t lds = G::LDS_BYTES;
  if (res && relu)
    hipLaunchKernelGGL((k_conv3x3_wino4<G, true, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards, in_absmax, out_absmax, HeadsOut{});
  else if (res)
    hipLaunchKernelGGL((k_conv3x3_wino4<G, true, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards, in_absmax, out_absmax, HeadsOut{});
  else if (relu)
    hipLaunchKernelGGL((k_conv3x3_wino4<G, false, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards, in_absmax, out_absmax, HeadsOut{});
  else
    hipLaunchKernelGGL((k_conv3x3_wino4<G, false, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards, in_absmax, out_absmax, HeadsOut{});
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

// split-K second pass: y = act(sum over splits s = 0 .. S-1 in order of part[s] + bias (+ res));
// one float4 per thread, every split's load issued before the sums (the pass is load-latency
// bound at a search's few boards), 8 workgroups per board; out_absmax[b] gets the board's
// max |y| (zeros on entry, as for the one-pass kernel), in_absmax[b] is consumed (reset to 0)
template <int S, bool RES, bool RELU>
__global__ __launch_bounds__(256) void k_splitk_combine(
    const float* __restrict__ part, const float* __restrict__ bias,
    const float* __restrict__ res, float* __restrict__ y, int n_boards,
    float* __restrict__ in_absmax, float* __restrict__ out_absmax) {
  constexpr int C = 128, WG_PER_BOARD = 64 * C / 4 / 256;
  const int tid = threadIdx.x, b = blockIdx.x / WG_PER_BOARD;
  const size_t o = 4 * ((size_t)blockIdx.x * 256 + tid);
  const size_t stride = (size_t)n_boards * 64 * C;
  float4 p[S];
#pragma unroll
  for (int s = 0; s < S; ++s) p[s] = *reinterpret_cast<const float4*>(part + s * stride + o);
  const float4 bv = *reinterpret_cast<const float4*>(bias + (o & (C - 1)));
  float4 r = {0.0f, 0.0f, 0.0f, 0.0f};
  if (RES) r = *reinterpret_cast<const float4*>(res + o);
  float4 v = p[0];
#pragma unroll
  for (int s = 1; s < S; ++s) {
    v.x += p[s].x; v.y += p[s].y; v.z += p[s].z; v.w += p[s].w;
  }
  v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
  if (RES) {
    v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
  }
  if (RELU) {
    v.x = fmaxf(v.x, 0.0f); v.y = fmaxf(v.y, 0.0f); v.z = fmaxf(v.z, 0.0f); v.w = fmaxf(v.w, 0.0f);
  }
  *reinterpret_cast<float4*>(y + o) = v;
  if (out_absmax) {
    float m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    __shared__ float s_m[4];
    if ((tid & 63) == 0) s_m[tid >> 6] = m;
    __syncthreads();
    if (tid == 0)
      atomicMax(reinterpret_cast<unsigned*>(out_absmax) + b,
                __float_as_uint(fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]))));
  }
  if (in_absmax && blockIdx.x % WG_PER_BOARD == 0 && tid == 0) in_absmax[b] = 0.0f;
}

// small batches: the channel chunks split over `splits` workgroups per board group (NC =
// CHUNKS / splits chunks each), partial sums to `part`, then k_splitk_combine
template <int NC, int NG = 4>
int launch_wino4_splitk(const float* x, const void* wq, const float* bias, const float* res,
                        float* y, int n_boards, int relu, float* in_absmax, float* out_absmax,
                        float* part, hipStream_t s) {
  using G = W4<AZ_CONV_FP16X2, 1, 4, NC, NG>;
  constexpr int splits = G::CHUNKS / NC * (4 / NG);
  static bool attr_set = false;
  if (!attr_set) {
    AZ_HIP(hipFuncSetAttribute((const void*)k_conv3x3_wino4<G, false, false>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS_BYTES));
    attr_set = true;
  }
  const dim3 grid((unsigned)((n_boards + G::BOARDS - 1) / G::BOARDS), splits);
  hipLaunchKernelGGL((k_conv3x3_wino4<G, false, false>), grid, dim3(G::THREADS),
                     (size_t)G::LDS_BYTES, s, x, static_cast<const char*>(wq), bias, nullptr,
                     part, n_boards, in_absmax, nullptr, HeadsOut{});
  AZ_HIP(hipGetLastError());
  const dim3 cg((unsigned)n_boards * (64 * 128 / 4 / 256));
  if (res && relu)
    hipLaunchKernelGGL((k_splitk_combine<splits, true, true>), cg, dim3(256), 0, s, part, bias, res, y, n_boards, in_absmax, out_absmax);
  else if (res)
    hipLaunchKernelGGL((k_splitk_combine<splits, true, false>), cg, dim3(256), 0, s, part, bias, res, y, n_boards, in_absmax, out_absmax);
  else if (relu)
    hipLaunchKernelGGL((k_splitk_combine<splits, false, true>), cg, dim3(256), 0, s, part, bias, res, y, n_boards, in_absmax, out_absmax);
  else
    hipLaunchKernelGGL((k_splitk_combine<splits, false, false>), cg, dim3(256), 0, s, part, bias, res, y, n_boards, in_absmax, out_absmax);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

}  // namespace

// the buffer-descriptor streams address activations with 32-bit byte offsets (num_records
// is at most 2^31 - 1): n_boards * 64 * 128 channels * 4 B must stay below that
constexpr int32_t kW4MaxBoards = 0x7fffffff / (64 * 128 * 4);

extern "C" int az_conv3x3_wino4_splitk_gpu(const float* x, const void* wq, const float* bias,
                                           const float* res, float* y, int32_t n_boards,
                                           int32_t channels, int32_t relu, int32_t mode,
                                           float* in_absmax, float* out_absmax, float* part,
                                           int32_t splits, void* stream) {
  AZ_REQUIRE(n_boards >= 0 && n_boards <= kW4MaxBoards, AZ_ERR_ARG,
             "az_conv3x3_wino4_splitk_gpu: n_boards %d outside [0, %d] (32-bit buffer offsets)", n_boards,
             kW4MaxBoards);
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && wq && bias && y && part && in_absmax && x != y && (!res || res != y) &&
                 in_absmax != out_absmax,
             AZ_ERR_ARG, "az_conv3x3_wino4_splitk_gpu: null buffer or in-place call");
  AZ_REQUIRE(((uintptr_t)x | (uintptr_t)wq | (uintptr_t)bias | (uintptr_t)y | (uintptr_t)part |
              (uintptr_t)res) % 16 == 0,
             AZ_ERR_ARG, "az_conv3x3_wino4_splitk_gpu: buffers must be 16-byte aligned");
  AZ_REQUIRE(channels == 128 && mode == AZ_CONV_FP16X2, AZ_ERR_ARG,
             "az_conv3x3_wino4_splitk_gpu: 128 channels, FP16X2 only (got %d, mode %d)",
             channels, mode);
  hipStream_t s = azc::as_stream(stream);
  if (splits == 2)
    return launch_wino4_splitk<4>(x, wq, bias, res, y, n_boards, relu, in_absmax, out_absmax, part, s);
  if (splits == 4)
    return launch_wino4_splitk<2>(x, wq, bias, res, y, n_boards, relu, in_absmax, out_absmax, part, s);
  if (splits == 8)
    return launch_wino4_splitk<1>(x, wq, bias, res, y, n_boards, relu, in_absmax, out_absmax, part, s);
  if (splits == 16)  // 4 transform rows x 4 channel splits
    return launch_wino4_splitk<2, 1>(x, wq, bias, res, y, n_boards, relu, in_absmax, out_absmax, part, s);
  if (splits == 32)  // 4 transform rows x 8 channel splits
    return launch_wino4_splitk<1, 1>(x, wq, bias, res, y, n_boards, relu, in_absmax, out_absmax, part, s);
  return azc::set_error(AZ_ERR_ARG,
                        "az_conv3x3_wino4_splitk_gpu: splits must be 2, 4, 8, 16 or 32, got %d",
                        splits);
}

#if AZ_W4_TSTAMP
extern "C" int az_w4_tstamps(unsigned long long* host, int n) {
  AZ_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_w4_tst), sizeof(unsigned long long) * n));
  return AZ_OK;
}
#endif

#if AZ_W4_CSTAMP
extern "C" int az_w4_cstamps(unsigned long long* host, int n) {
  AZ_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_w4_cst), sizeof(unsigned long long) * n));
  return AZ_OK;
}
#endif

#if AZ_W4_STAMP
extern "C" int az_w4_stamps(unsigned long long* host, int n) {
  AZ_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_w4_stamps), sizeof(unsigned long long) * n));
  return AZ_OK;
}
#endif

namespace {
template <class G>
int launch_wino4_heads(const float* x, const void* wq, const float* bias, const float* res,
                       int n_boards, float* in_absmax, const HeadsOut& ho, void* stream) {
  static bool attr_set = false;
  if (!attr_set) {
    AZ_HIP(hipFuncSetAttribute((const void*)k_conv3x3_wino4<G, true, true, true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS_BYTES));
    attr_set = true;
  }
  const unsigned grid = (unsigned)((n_boards + G::BOARDS - 1) / G::BOARDS);
  hipLaunchKernelGGL((k_conv3x3_wino4<G, true, true, true>), dim3(grid), dim3(G::THREADS),
                     (size_t)G::LDS_BYTES, azc::as_stream(stream), x,
                     static_cast<const char*>(wq), bias, res, nullptr, n_boards, in_absmax,
                     nullptr, ho);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
}  // namespace

extern "C" int az_conv3x3_wino4_heads_gpu(const float* x, const void* wq, const float* bias,
                                          const float* res, int32_t n_boards,
                                          int32_t channels, int32_t mode, float* in_absmax,
                                          const float* wpv, const float* bpv,
                                          const float* wpolT, const float* bpol,
                                          const float* w1T, const float* b1, const float* w2,
                                          const float* b2, float* priors, float* values,
                                          void* stream) {
  AZ_REQUIRE(n_boards >= 0 && n_boards <= kW4MaxBoards, AZ_ERR_ARG,
             "az_conv3x3_wino4_heads_gpu: n_boards %d outside [0, %d] (32-bit buffer offsets)", n_boards,
             kW4MaxBoards);
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && wq && bias && res && in_absmax && wpv && bpv && wpolT && bpol && w1T && b1 &&
                 w2 && b2 && priors && values,
             AZ_ERR_ARG, "az_conv3x3_wino4_heads_gpu: null buffer");
  AZ_REQUIRE(((uintptr_t)x | (uintptr_t)wq | (uintptr_t)bias | (uintptr_t)res | (uintptr_t)wpv |
              (uintptr_t)w1T | (uintptr_t)b1 | (uintptr_t)w2) % 16 == 0,
             AZ_ERR_ARG, "az_conv3x3_wino4_heads_gpu: buffers must be 16-byte aligned");
  AZ_REQUIRE(channels == 128 && mode == AZ_CONV_FP16X2, AZ_ERR_ARG,
             "az_conv3x3_wino4_heads_gpu: 128 channels in FP16X2 mode only (got %d, mode %d)",
             channels, mode);
  // AZ_W4_HEADS_BOARDS: 2 = two-board workgroups, two per CU (the trunk conv's default
  // form), 4 = four-board workgroups, one per CU (the round-3 form); read per call so the
  // tests compare the two
  const char* hbe = getenv("AZ_W4_HEADS_BOARDS");
  const int hb = hbe ? atoi(hbe) : 2;
  AZ_REQUIRE(hb == 2 || hb == 4, AZ_ERR_ARG, "AZ_W4_HEADS_BOARDS must be 2 or 4, got %d", hb);
  const HeadsOut ho{{wpv, bpv, wpolT, bpol, w1T, b1, w2, b2}, priors, values};
  if (hb == 2) return launch_wino4_heads<W4<AZ_CONV_FP16X2, 1, 2>>(x, wq, bias, res, n_boards,
                                                                    in_absmax, ho, stream);
  return launch_wino4_heads<W4<AZ_CONV_FP16X2, 1>>(x, wq, bias, res, n_boards, in_absmax, ho,
                                                   stream);
}

extern "C" int az_trunk_wino4_gpu(const void* const* wq, const float* const* bias,
                                  const float* planes, const float* stem_w,
                                  const float* stem_b, float* h_in, float* hb0, float* hb1,
                                  float* t, float* amax0, float* amax1, int32_t n_boards,
                                  int32_t n_convs, int32_t channels, void* stream) {
  AZ_REQUIRE(n_boards >= 0 && n_convs >= 0 && n_boards <= kW4MaxBoards, AZ_ERR_ARG,
             "az_trunk_wino4_gpu: n_boards %d / n_convs %d out of range (n_boards <= %d)",
             n_boards, n_convs, kW4MaxBoards);
  if (n_boards == 0 || (n_convs == 0 && !planes)) return AZ_OK;
  AZ_REQUIRE((n_convs == 0 || (wq && bias)) && h_in && hb0 && hb1 && t && amax0 && amax1,
             AZ_ERR_ARG,
             "az_trunk_wino4_gpu: null buffer");
  AZ_REQUIRE(h_in != hb0 && h_in != hb1 && h_in != t && hb0 != hb1 && hb0 != t && hb1 != t &&
                 amax0 != amax1,
             AZ_ERR_ARG, "az_trunk_wino4_gpu: aliased buffers");
  AZ_REQUIRE(((uintptr_t)h_in | (uintptr_t)hb0 | (uintptr_t)hb1 | (uintptr_t)t) % 16 == 0,
             AZ_ERR_ARG, "az_trunk_wino4_gpu: buffers must be 16-byte aligned");
  AZ_REQUIRE(channels == 128, AZ_ERR_ARG, "az_trunk_wino4_gpu: channels must be 128, got %d",
             channels);
  AZ_REQUIRE(!planes || (stem_w && stem_b && ((uintptr_t)stem_w | (uintptr_t)stem_b) % 16 == 0),
             AZ_ERR_ARG, "az_trunk_wino4_gpu: planes without 16-byte aligned stem weights");
  using G = W4<AZ_CONV_FP16X2, 1, AZ_W4_TRUNK_BOARDS>;  // two-board workgroups, FP16X2
  static bool attr_set = false;
  if (!attr_set) {
    AZ_HIP(hipFuncSetAttribute((const void*)k_trunk_wino4<G>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::TRUNK_LDS));
    attr_set = true;
  }
  const TrunkW4 a{reinterpret_cast<const char* const*>(wq), bias, h_in, {hb0, hb1}, t,
                  {amax0, amax1}, planes, stem_w, stem_b, n_boards, n_convs};
  const unsigned grid = (unsigned)((n_boards + G::BOARDS - 1) / G::BOARDS);
  hipLaunchKernelGGL((k_trunk_wino4<G>), dim3(grid), dim3(G::THREADS), (size_t)G::TRUNK_LDS,
                     azc::as_stream(stream), a, HeadsOut{});
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

template <int MODE>
static int trunk_heads_entry(const char* fn, const void* const* wq, const float* const* bias,
                                        const float* planes, const float* stem_w,
                                        const float* stem_b, float* h_in, float* hb0,
                                        float* hb1, float* t, float* amax0, float* amax1,
                                        int32_t n_boards, int32_t n_convs, int32_t channels,
                                        const float* wpv, const float* bpv,
                                        const float* wpolT, const float* bpol,
                                        const float* w1T, const float* b1, const float* w2,
                                        const float* b2, float* priors, float* values,
                                        void* stream) {
  AZ_REQUIRE(n_boards >= 0 && n_boards <= kW4MaxBoards && n_convs >= 2 && n_convs % 2 == 0,
             AZ_ERR_ARG,
             "%s: n_boards %d (<= %d) / n_convs %d (even, >= 2)", fn, n_boards,
             kW4MaxBoards, n_convs);
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(wq && bias && h_in && hb0 && hb1 && t && amax0 && amax1, AZ_ERR_ARG,
             "%s: null buffer", fn);
  AZ_REQUIRE(h_in != hb0 && h_in != hb1 && h_in != t && hb0 != hb1 && hb0 != t && hb1 != t &&
                 amax0 != amax1,
             AZ_ERR_ARG, "%s: aliased buffers", fn);
  AZ_REQUIRE(((uintptr_t)h_in | (uintptr_t)hb0 | (uintptr_t)hb1 | (uintptr_t)t) % 16 == 0,
             AZ_ERR_ARG, "%s: buffers must be 16-byte aligned", fn);
  AZ_REQUIRE(channels == 128, AZ_ERR_ARG,
             "%s: channels must be 128, got %d", fn, channels);
  AZ_REQUIRE(!planes || (stem_w && stem_b && ((uintptr_t)stem_w | (uintptr_t)stem_b) % 16 == 0),
             AZ_ERR_ARG, "%s: planes without 16-byte aligned stem weights", fn);
  AZ_REQUIRE(wpv && bpv && wpolT && bpol && w1T && b1 && w2 && b2 && priors && values,
             AZ_ERR_ARG, "%s: null heads buffer", fn);
  AZ_REQUIRE(((uintptr_t)wpv | (uintptr_t)w1T | (uintptr_t)b1 | (uintptr_t)w2) % 16 == 0,
             AZ_ERR_ARG, "%s: heads weights must be 16-byte aligned", fn);
  using G = W4<MODE, 1, AZ_W4_TRUNK_BOARDS>;  // two-board workgroups
  static bool attr_set = false;
  if (!attr_set) {
    AZ_HIP(hipFuncSetAttribute((const void*)k_trunk_wino4<G, true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::TRUNK_LDS));
    attr_set = true;
  }
  const TrunkW4 a{reinterpret_cast<const char* const*>(wq), bias, h_in, {hb0, hb1}, t,
                  {amax0, amax1}, planes, stem_w, stem_b, n_boards, n_convs};
  const HeadsOut ho{{wpv, bpv, wpolT, bpol, w1T, b1, w2, b2}, priors, values};
  const unsigned grid = (unsigned)((n_boards + G::BOARDS - 1) / G::BOARDS);
  hipLaunchKernelGGL((k_trunk_wino4<G, true>), dim3(grid), dim3(G::THREADS),
                     (size_t)G::TRUNK_LDS, azc::as_stream(stream), a, ho);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}


#define AZ_TRUNK_HEADS_ARGS                                                                     \
  const void *const *wq, const float *const *bias, const float *planes, const float *stem_w,   \
      const float *stem_b, float *h_in, float *hb0, float *hb1, float *t, float *amax0,        \
      float *amax1, int32_t n_boards, int32_t n_convs, int32_t channels, const float *wpv,     \
      const float *bpv, const float *wpolT, const float *bpol, const float *w1T,                \
      const float *b1, const float *w2, const float *b2, float *priors, float *values,          \
      void *stream
#define AZ_TRUNK_HEADS_PASS                                                                     \
  wq, bias, planes, stem_w, stem_b, h_in, hb0, hb1, t, amax0, amax1, n_boards, n_convs,         \
      channels, wpv, bpv, wpolT, bpol, w1T, b1, w2, b2, priors, values, stream
extern "C" int az_trunk_wino4_heads_gpu(AZ_TRUNK_HEADS_ARGS) {
  return trunk_heads_entry<AZ_CONV_FP16X2>("az_trunk_wino4_heads_gpu", AZ_TRUNK_HEADS_PASS);
}
// the same launch in FP16 (one fp16 product per MFMA step, no operand scaling; the weights
// prepared for the FP16 wino4 conv): configs[4]'s fp16 inference
extern "C" int az_trunk_wino4_heads_fp16_gpu(AZ_TRUNK_HEADS_ARGS) {
  return trunk_heads_entry<AZ_CONV_FP16>("az_trunk_wino4_heads_fp16_gpu", AZ_TRUNK_HEADS_PASS);
}
#undef AZ_TRUNK_HEADS_ARGS
#undef AZ_TRUNK_HEADS_PASS

extern "C" int az_conv3x3_wino4_gpu(const float* x, const void* wq, const float* bias,
                                    const float* res, float* y, int32_t n_boards,
                                    int32_t channels, int32_t relu, int32_t mode,
                                    float* in_absmax, float* out_absmax, void* stream) {
  AZ_REQUIRE(n_boards >= 0 && n_boards <= kW4MaxBoards, AZ_ERR_ARG,
             "az_conv3x3_wino4_gpu: n_boards %d outside [0, %d] (32-bit buffer offsets)", n_boards,
             kW4MaxBoards);
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && wq && bias && y && x != y && (!res || res != y), AZ_ERR_ARG,
             "az_conv3x3_wino4_gpu: null buffer or in-place call");
  AZ_REQUIRE(((uintptr_t)x | (uintptr_t)wq | (uintptr_t)bias) % 16 == 0, AZ_ERR_ARG,
             "az_conv3x3_wino4_gpu: buffers must be 16-byte aligned");
  AZ_REQUIRE(channels == 128, AZ_ERR_ARG, "az_conv3x3_wino4_gpu: channels must be 128, got %d",
             channels);
  AZ_REQUIRE(mode != AZ_CONV_FP16X2 || (in_absmax && in_absmax != out_absmax), AZ_ERR_ARG,
             "az_conv3x3_wino4_gpu: FP16X2 needs in_absmax (distinct from out_absmax)");
  hipStream_t s = azc::as_stream(stream);
  // AZ_W4_NRT (experiments): 1 = eight waves of one row tile (default: two waves per SIMD,
  // no AGPR traffic in the fold; bench 79.7 vs 73.5 games/s same-box), 2 = four waves of two
  static const int nrt = getenv("AZ_W4_NRT") ? atoi(getenv("AZ_W4_NRT")) : 1;
  // Workgroup size (round 3): two boards per workgroup, two workgroups per CU (default for
  // FP16X2 and FP16) -- the same tiles and arithmetic, bit-identical outputs, but each CU
  // holds two independent barrier domains instead of one: configs[2] bench 94.4 -> 97.1
  // games/s same box (profiles/r03_bench_boards2.json; per launch at B = 1,024 -3 % with a
  // residual, equal without, equal at 4,096).  AZ_W4_BOARDS=4: the four-board workgroup (read
  // per call, so tests can compare the two forms).
  const char* nbe = getenv("AZ_W4_BOARDS");
  const int nbw = nbe ? atoi(nbe) : 2;
#define W4_GO(M, N) launch_wino4<W4<M, N>>(x, wq, bias, res, y, n_boards, relu, in_absmax, out_absmax, s)
  if (mode == AZ_CONV_FP16X2 && nbw == 2)
    return launch_wino4<W4<AZ_CONV_FP16X2, 1, 2>>(x, wq, bias, res, y, n_boards, relu, in_absmax,
                                                  out_absmax, s);
  if (mode == AZ_CONV_FP16 && nbw == 2)
    return launch_wino4<W4<AZ_CONV_FP16, 1, 2>>(x, wq, bias, res, y, n_boards, relu, in_absmax,
                                                out_absmax, s);
  if (mode == AZ_CONV_SPLIT3) return nrt == 1 ? W4_GO(AZ_CONV_SPLIT3, 1) : W4_GO(AZ_CONV_SPLIT3, 2);
  if (mode == AZ_CONV_FP16) return nrt == 1 ? W4_GO(AZ_CONV_FP16, 1) : W4_GO(AZ_CONV_FP16, 2);
  if (mode == AZ_CONV_FP16X2) return nrt == 1 ? W4_GO(AZ_CONV_FP16X2, 1) : W4_GO(AZ_CONV_FP16X2, 2);
#undef W4_GO
  return azc::set_error(AZ_ERR_ARG, "az_conv3x3_wino4_gpu: unknown mode %d", mode);
}

namespace {
// one workgroup per board: max |x| over its 64 * C values
__global__ void k_board_absmax(const float* __restrict__ x, int per_board, float* __restrict__ out) {
  const float4* p = reinterpret_cast<const float4*>(x + (size_t)blockIdx.x * per_board);
  float m = 0.0f;
  for (int i = threadIdx.x; i < per_board / 4; i += blockDim.x) {
    const float4 v = p[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  __shared__ float s_m[4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]));
}
}  // namespace

extern "C" int az_board_absmax_gpu(const float* x, int32_t n_boards, int32_t channels, float* out,
                                   void* stream) {
  AZ_REQUIRE(n_boards >= 0 && channels > 0 && channels % 4 == 0, AZ_ERR_ARG,
             "az_board_absmax_gpu: bad sizes");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && out && (uintptr_t)x % 16 == 0, AZ_ERR_ARG,
             "az_board_absmax_gpu: null or unaligned buffer");
  hipLaunchKernelGGL(k_board_absmax, dim3(n_boards), dim3(256), 0, azc::as_stream(stream), x,
                     64 * channels, out);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
