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
// so a wave holds 4 points' M plus the 2x2 outputs Y instead of 16 points' M: room for 64
// tile rows (4 boards), half the weight bytes per board.
//
// Workgroup = 4 boards (64 tiles = two 32-row MFMA tiles) x all 128 columns, 4 waves (one
// per SIMD, 512 registers each): wave w owns columns 32w..32w+31 for all 64 rows, so each
// weight fragment feeds two MFMA row tiles and no two waves stream the same weights.
//   * Linear chunk L = 0..31 = (group k = L / 8, input-channel chunk c = L % 8 of 16
//     channels); within a chunk, steps l = 0..3 run point (k, l): 2 row tiles x (6 split3
//     products | 1 fp16 product) MFMAs.
//   * V of chunk L+1 is formed while chunk L computes: the two window rows B^T row k needs
//     (d_a +- d_a') are loaded one chunk ahead (4 of the 16 loads per step), combined into the
//     row at the chunk start, and each step transforms, splits and stores one point into the
//     other half of a double-buffered LDS image [point][plane][tile][16 ch] (tile rows XOR-
//     swizzled by 16-byte half so the ds_read_b128 fragment reads are conflict-free).
//   * Weights stream per wave from L2 three steps ahead (ring of 4 fragments).
//   * One LDS barrier per chunk (lgkmcnt only; the weight and window loads stay in flight).
//   * Epilogue straight from the Y registers: + bias (+ residual), ReLU, store.
#include <type_traits>

#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

template <int MODE_>
struct W4 {
  static constexpr int C = 128, MODE = MODE_;
  static constexpr int PLANES = MODE == AZ_CONV_SPLIT3 ? 3 : 1;
  static constexpr int BOARDS = 4, ROWS = 64, THREADS = 256;
  static constexpr int SLAB = ROWS * 32;            // one (point, plane): 64 tiles x 16 ch x 2 B
  static constexpr int BUF = 4 * PLANES * SLAB;     // one (group, chunk): its four points
  static constexpr int LDS_BYTES = 2 * BUF;
  static constexpr int STEP_BYTES = PLANES * C * 32;  // weight bytes of one (chunk, point)
  static constexpr int CHUNKS = C / 16;
  static constexpr int LCHUNKS = 4 * CHUNKS;        // (group, chunk) pairs
  static constexpr int QSTEPS = LCHUNKS * 4;        // (group, chunk, point) steps
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

// window rows of group k: B^T row k = sa * d_a0 + sb * d_a1 (B^T = [1 0 -1 0; 0 1 1 0;
// 0 -1 1 0; 0 1 0 -1]); multiplying by +-1 is exact, so this is the transform's own
// add/subtract
__device__ __forceinline__ int grp_a0(int k) { return k == 0 ? 0 : 1; }
__device__ __forceinline__ int grp_a1(int k) { return k == 3 ? 3 : 2; }
__device__ __forceinline__ float grp_sa(int k) { return k == 2 ? -1.0f : 1.0f; }
__device__ __forceinline__ float grp_sb(int k) { return (k == 1 || k == 2) ? 1.0f : -1.0f; }

// weight fragment of linear step q (chunk L = q / 4 = (group k, channel chunk c), point l)
template <class G>
__device__ __forceinline__ void load_b(Frag<G>& f, const char* wq, int wlane, int q) {
  const int L = q >> 2, l = q & 3, k = L >> 3, c = L & 7;
  const char* step = wq + (size_t)(c * 16 + 4 * k + l) * G::STEP_BYTES;
#pragma unroll
  for (int pl = 0; pl < G::PLANES; ++pl)
    f.v[pl] = *reinterpret_cast<const Word8<G>*>(step + wlane + pl * G::C * 32);
}

template <class G>
__device__ __forceinline__ void read_a(Frag<G> (&a)[2], const char* buf, int l,
                                       const int (&aoff)[2]) {
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int pl = 0; pl < G::PLANES; ++pl)
      a[rt].v[pl] = *reinterpret_cast<const Word8<G>*>(buf + (l * G::PLANES + pl) * G::SLAB + aoff[rt]);
}

template <class G>
__device__ __forceinline__ void mma(f32x16& acc, const Frag<G>& a, const Frag<G>& b) {
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

// window entries e0..e0+NE-1 (e = which * 4 + b: window row a0 / a1 of linear chunk L's
// group, column b) of transform item u.  Off-board entries read element 0 (a valid
// address) and are zeroed in make_rows, so every load is issued unconditionally.
template <class G, int NE>
__device__ __forceinline__ void load_raw(f32x2 (&raw)[2][8], const float* x, const int (&off)[2],
                                         const int (&msk)[2], int L, int u, int e0) {
  const int k = L >> 3, c = L & 7;
  const int a0 = grp_a0(k), a1 = grp_a1(k);
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int e = e0 + i, b = e & 3, a = (e >> 2) ? a1 : a0;
    const bool in = (msk[u] >> (a * 4 + b)) & 1;
    const uint32_t o = in ? (uint32_t)(off[u] + (a * 8 + b) * G::C + c * 16) : 0u;
    raw[u][e] = *reinterpret_cast<const f32x2*>(reinterpret_cast<const char*>(x) + o * 4u);
  }
}

template <class G>
__device__ __forceinline__ void make_rows(f32x2 (&rk)[2][4], const f32x2 (&raw)[2][8],
                                          const int (&msk)[2], int L) {
  const int k = L >> 3;
  const int a0 = grp_a0(k), a1 = grp_a1(k);
  const f32x2 sa = {grp_sa(k), grp_sa(k)}, sb = {grp_sb(k), grp_sb(k)};
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const f32x2 d0 = (msk[u] >> (a0 * 4 + b)) & 1 ? raw[u][b] : f32x2{0.0f, 0.0f};
      const f32x2 d1 = (msk[u] >> (a1 * 4 + b)) & 1 ? raw[u][4 + b] : f32x2{0.0f, 0.0f};
      rk[u][b] = sa * d0 + sb * d1;
    }
}

// V at point (k, l) = (row k of B^T d) B: column combination l
template <int l>
__device__ __forceinline__ f32x2 col_comb(const f32x2 (&rk)[4]) {
  if constexpr (l == 0) return rk[0] - rk[2];
  if constexpr (l == 1) return rk[1] + rk[2];
  if constexpr (l == 2) return rk[2] - rk[1];
  return rk[1] - rk[3];
}

// split two transformed values into PLANES 16-bit words and store them in their slabs
template <class G>
__device__ __forceinline__ void put(char* slab, f32x2 v) {
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

template <class G, int l>
__device__ __forceinline__ void put_point(char* buf, const f32x2 (&rk)[2][4], const int (&soff)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) put<G>(buf + l * G::PLANES * G::SLAB + soff[u], col_comb<l>(rk[u]));
}

// group k's M (acc[l][rt]) into the output accumulators Y[i][j][rt]
__device__ __forceinline__ void fold(f32x16 (&acc)[4][2], f32x16 (&Y)[2][2][2], int k) {
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float m0 = acc[0][rt][e], m1 = acc[1][rt][e], m2 = acc[2][rt][e], m3 = acc[3][rt][e];
      const float t0 = (m0 + m1) + m2, t1 = (m1 - m2) - m3;
      if (k == 0) {
        Y[0][0][rt][e] = t0;
        Y[0][1][rt][e] = t1;
      } else if (k == 1) {
        Y[0][0][rt][e] += t0;
        Y[0][1][rt][e] += t1;
        Y[1][0][rt][e] = t0;
        Y[1][1][rt][e] = t1;
      } else if (k == 2) {
        Y[0][0][rt][e] += t0;
        Y[0][1][rt][e] += t1;
        Y[1][0][rt][e] -= t0;
        Y[1][1][rt][e] -= t1;
      } else {
        Y[1][0][rt][e] -= t0;
        Y[1][1][rt][e] -= t1;
      }
    }
}

template <class G, bool RES, bool RELU>
__global__ __launch_bounds__(256, 1) void k_conv3x3_wino4(const float* __restrict__ x,
                                                          const char* __restrict__ wq,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ res,
                                                          float* __restrict__ y, int n_boards) {
  constexpr int C = G::C;
  extern __shared__ float4 lds4[];
  char* lds = reinterpret_cast<char*>(lds4);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int col0 = 32 * wave;
  const int b0 = blockIdx.x * G::BOARDS;
  const int nb = n_boards - b0 < G::BOARDS ? n_boards - b0 : G::BOARDS;
  const int wlane = (col0 + r) * 32 + h * 16;
  const int aoff[2] = {r * 32 + ((h ^ ((r >> 3) & 1)) << 4),
                       (32 + r) * 32 + ((h ^ ((r >> 3) & 1)) << 4)};

  // transform items: u = 0, 1 -> tile T = tid / 8 + 32u (board T / 16, tile row (T / 4) % 4,
  // tile column T % 4), channel pair p = tid % 8 of each 16-channel chunk
  int off[2], msk[2], soff[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int T = (tid >> 3) + 32 * u, p = tid & 7;
    const int bd = T >> 4, ty = (T >> 2) & 3, tx = T & 3;
    int m = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int yy = 2 * ty - 1 + a, xx = 2 * tx - 1 + b;
        m |= (bd < nb && (unsigned)yy < 8u && (unsigned)xx < 8u) << (a * 4 + b);
      }
    msk[u] = m;
    off[u] = ((b0 + bd) * 64 + (2 * ty - 1) * 8 + (2 * tx - 1)) * C + 2 * p;
    soff[u] = T * 32 + (((p >> 2) ^ ((T >> 3) & 1)) << 4) + (p & 3) * 4;
  }

  f32x2 raw[2][8], rk[2][4];
  Frag<G> bf[4];
  // ---- prologue: chunk 0's windows, chunk 1's windows and the first three weight steps in
  // flight together; chunk 0 transformed into buffer 0
  {
    f32x2 raw0[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) load_raw<G, 8>(raw0, x, off, msk, 0, u, 0);
#pragma unroll
    for (int u = 0; u < 2; ++u) load_raw<G, 8>(raw, x, off, msk, 1, u, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 3; ++i) load_b<G>(bf[i], wq, wlane, i);
    __builtin_amdgcn_sched_barrier(0);
    make_rows<G>(rk, raw0, msk, 0);
  }
  put_point<G, 0>(lds, rk, soff);
  put_point<G, 1>(lds, rk, soff);
  put_point<G, 2>(lds, rk, soff);
  put_point<G, 3>(lds, rk, soff);
  lds_barrier();

  f32x16 acc[4][2];
#pragma unroll
  for (int l = 0; l < 4; ++l)
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[l][rt][e] = 0.0f;
  f32x16 Y[2][2][2];

  Frag<G> af[2];
  read_a<G>(af, lds, 0, aoff);
  for (int L = 0; L < G::LCHUNKS; ++L) {
    const char* cur = lds + (L & 1) * G::BUF;
    char* nxt = lds + ((L + 1) & 1) * G::BUF;
    // chunk L+1's rows (its windows were requested during chunk L-1); the last chunk
    // transforms a clamped duplicate into the idle buffer (uniform body)
    const int Lr = L + 1 < G::LCHUNKS ? L + 1 : G::LCHUNKS - 1;
    const int Ll = L + 2 < G::LCHUNKS ? L + 2 : G::LCHUNKS - 1;
    make_rows<G>(rk, raw, msk, Lr);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      Frag<G> an[2];
      if (l < 3) read_a<G>(an, cur, l + 1, aoff);
      mma<G>(acc[l][0], af[0], bf[l]);
      mma<G>(acc[l][1], af[1], bf[l]);
      const int q = L * 4 + l + 3;
      load_b<G>(bf[(l + 3) & 3], wq, wlane, q < G::QSTEPS - 1 ? q : G::QSTEPS - 1);
      load_raw<G, 4>(raw, x, off, msk, Ll, l >> 1, 4 * (l & 1));
      if (l == 0) put_point<G, 0>(nxt, rk, soff);
      if (l == 1) put_point<G, 1>(nxt, rk, soff);
      if (l == 2) put_point<G, 2>(nxt, rk, soff);
      if (l == 3) put_point<G, 3>(nxt, rk, soff);
      if (l < 3) {
        af[0] = an[0];
        af[1] = an[1];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if ((L & 7) == 7) {
      fold(acc, Y, L >> 3);
#pragma unroll
      for (int l = 0; l < 4; ++l)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[l][rt][e] = 0.0f;
    }
    lds_barrier();
    read_a<G>(af, nxt, 0, aoff);
  }

  // ---- epilogue: accumulator element e of row tile rt = tile 32rt + (e&3) + 8(e>>2) + 4h,
  // column col0 + r; Y[i][j] = output (2ty + i, 2tx + j)
  const int co = col0 + r;
  const float bv = bias[co];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int T = 32 * rt + (e & 3) + 8 * (e >> 2) + 4 * h;
      const int bd = T >> 4, ty = (T >> 2) & 3, tx = T & 3;
      if (bd >= nb) continue;  // uniform over the wave half
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const size_t o = ((size_t)(b0 + bd) * 64 + (2 * ty + i) * 8 + 2 * tx + j) * C + co;
          float v = Y[i][j][rt][e] + bv;
          if (RES) v += res[o];
          if (RELU) v = fmaxf(v, 0.0f);
          y[o] = v;
        }
    }
}

template <class G>
int launch_wino4(const float* x, const void* wq, const float* bias, const float* res, float* y,
                 int n_boards, int relu, hipStream_t s) {
  const unsigned grid = (unsigned)((n_boards + G::BOARDS - 1) / G::BOARDS);
  const char* w = static_cast<const char*>(wq);
  const dim3 blk(G::THREADS);
  const size_t lds = G::LDS_BYTES;
  if (res && relu)
    hipLaunchKernelGGL((k_conv3x3_wino4<G, true, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else if (res)
    hipLaunchKernelGGL((k_conv3x3_wino4<G, true, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else if (relu)
    hipLaunchKernelGGL((k_conv3x3_wino4<G, false, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else
    hipLaunchKernelGGL((k_conv3x3_wino4<G, false, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

}  // namespace

extern "C" int az_conv3x3_wino4_gpu(const float* x, const void* wq, const float* bias,
                                    const float* res, float* y, int32_t n_boards,
                                    int32_t channels, int32_t relu, int32_t mode, void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_conv3x3_wino4_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && wq && bias && y && x != y && (!res || res != y), AZ_ERR_ARG,
             "az_conv3x3_wino4_gpu: null buffer or in-place call");
  AZ_REQUIRE(((uintptr_t)x | (uintptr_t)wq | (uintptr_t)bias) % 16 == 0, AZ_ERR_ARG,
             "az_conv3x3_wino4_gpu: buffers must be 16-byte aligned");
  AZ_REQUIRE(channels == 128, AZ_ERR_ARG, "az_conv3x3_wino4_gpu: channels must be 128, got %d",
             channels);
  hipStream_t s = azc::as_stream(stream);
  if (mode == AZ_CONV_SPLIT3)
    return launch_wino4<W4<AZ_CONV_SPLIT3>>(x, wq, bias, res, y, n_boards, relu, s);
  if (mode == AZ_CONV_FP16)
    return launch_wino4<W4<AZ_CONV_FP16>>(x, wq, bias, res, y, n_boards, relu, s);
  return azc::set_error(AZ_ERR_ARG, "az_conv3x3_wino4_gpu: unknown mode %d", mode);
}
