// conv.hip — fp32 MFMA implicit-GEMM 3x3 convolution for 8x8 boards with the epilogue fused.
//
// The residual trunk of the leaf-evaluation net (reference Models.py:72-90, 164-221; the
// BatchNorm of the inference copy folded into weight + bias) is 10 convolutions
// Ci = Co = C over [B, 8, 8, C] activations: ~95 % of a self-play step.  One kernel does
// conv + bias (+ residual) + ReLU:
//
//   GEMM view: M = B*64 output positions, N = C output channels, K = 9 taps x C.
//   Workgroup = 4 waves = 2 boards (M = 128) x all C channels.  The two input boards are
//   staged once into LDS (channels padded +4 floats so ds_read_b128 row gathers are
//   conflict-free); the im2col gather is implicit — for tap (ky,kx) the A row of output
//   position (y,x) is LDS position (y+ky-1, x+kx-1) or zero at the board edge.
//   Weights [9][Co][Ci] stream from L2 into registers (float4 along Ci), one chunk ahead.
//   MFMA v_mfma_f32_32x32x2_f32 (exact f32 fma chain): each float4 of A and of B feeds
//   four MFMAs; the K order inside a chunk is permuted identically for A and B
//   (lane half h, element j  ->  k = ci0 + 4h + j), which leaves the sum unchanged.
//   Epilogue straight from the accumulators: + bias[co], + residual, ReLU, NHWC store.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Tiling: a workgroup of WAVES waves owns BOARDS boards (M = 64*BOARDS rows) x all C
// output channels; each wave a TM x TN block of 32x32 MFMA tiles.
template <int C_, int BOARDS_, int WAVES_, int TM_, int TN_>
struct Geo {
  static constexpr int C = C_, BOARDS = BOARDS_, WAVES = WAVES_, TM = TM_, TN = TN_;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int S = C + 4;       // LDS floats per position (padded: conflict-free rows)
  static constexpr int WM = 32 * TM;    // rows per wave
  static constexpr int WN = 32 * TN;    // cols per wave
  static constexpr int WAVES_N = C / WN;
  static_assert((BOARDS * 64 / WM) * WAVES_N == WAVES, "tiling must cover the workgroup");
};

template <class G, bool RES, bool RELU>
__global__ __launch_bounds__(G::THREADS) void k_conv3x3(const float* __restrict__ x,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ res,
                                                        float* __restrict__ y, int n_boards) {
  constexpr int C = G::C, kBoards = G::BOARDS, kThreads = G::THREADS;
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int b0 = blockIdx.x * kBoards;
  const int nb = n_boards - b0 < kBoards ? n_boards - b0 : kBoards;

  // ---- stage the input boards (NHWC) into LDS, zero-fill a missing tail board; one extra
  // all-zero position (index kBoards*64) is what off-board taps read (branch-free gather)
  {
    constexpr int V = (kBoards * 64 + 1) * C / 4;  // float4s
    constexpr int ITER = (V + kThreads - 1) / kThreads;
    const float4* src = reinterpret_cast<const float4*>(x + (size_t)b0 * 64 * C);
    float4 val[ITER];  // every load issued before the first LDS write
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int v = tid + i * kThreads;
      val[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (v < nb * 64 * (C / 4)) val[i] = src[v];
    }
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int v = tid + i * kThreads;
      if (v >= V) continue;
      const int pos = v / (C / 4), c4 = v % (C / 4);
      *reinterpret_cast<float4*>(lds + pos * G::S + c4 * 4) = val[i];
    }
  }
  __syncthreads();

  const int wm = wave / G::WAVES_N, wn = wave % G::WAVES_N;
  const int row0 = wm * G::WM, col0 = wn * G::WN;
  const int r = lane & 31, h = lane >> 5;

  // per A tile: the output position of this lane's row
  int py[G::TM], px[G::TM], pb[G::TM];
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi) {
    const int m = row0 + 32 * mi + r;
    pb[mi] = m >> 6;
    py[mi] = (m >> 3) & 7;
    px[mi] = m & 7;
  }

  f32x16 acc[G::TM][G::TN];
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[mi][ni][k] = 0.0f;

  // weights: w[tap][co][ci]; lane reads float4 at ci0 + 4h for its column co
  const float* wcol[G::TN];
#pragma unroll
  for (int ni = 0; ni < G::TN; ++ni) wcol[ni] = w + (size_t)(col0 + 32 * ni + r) * C + 4 * h;

  constexpr int CHUNKS = C / 8;      // ci chunks of 8 (two lane halves x float4)
  constexpr int STEPS = 9 * CHUNKS;  // (tap, chunk) iterations

  auto load_b = [&](int s, float4 (&b)[G::TN]) {
    const int tap = s / CHUNKS, ci0 = (s % CHUNKS) * 8;
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni)
      b[ni] = *reinterpret_cast<const float4*>(wcol[ni] + (size_t)tap * C * C + ci0);
  };
  constexpr int kZeroPos = kBoards * 64;
  auto load_a = [&](int s, float4 (&a)[G::TM]) {
    const int tap = s / CHUNKS, ci0 = (s % CHUNKS) * 8;
    const int ky = tap / 3 - 1, kx = tap % 3 - 1;
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi) {
      const int yy = py[mi] + ky, xx = px[mi] + kx;
      const bool ok = (unsigned)yy < 8u && (unsigned)xx < 8u;
      const int pos = ok ? pb[mi] * 64 + yy * 8 + xx : kZeroPos;
      a[mi] = *reinterpret_cast<const float4*>(lds + pos * G::S + ci0 + 4 * h);
    }
  };
  auto mma = [&](const float4 (&a)[G::TM], const float4 (&b)[G::TN]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi) {
        const float av = j == 0 ? a[mi].x : j == 1 ? a[mi].y : j == 2 ? a[mi].z : a[mi].w;
#pragma unroll
        for (int ni = 0; ni < G::TN; ++ni) {
          const float bv = j == 0 ? b[ni].x : j == 1 ? b[ni].y : j == 2 ? b[ni].z : b[ni].w;
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[mi][ni], 0, 0, 0);
        }
      }
    }
  };

  // two chunks in flight: ping-pong register sets, loads for chunk s+2 issued right after
  // chunk s's MFMAs (no register copies, no full drain per chunk)
  static_assert(STEPS % 2 == 0, "even number of (tap, chunk) steps");
  float4 ra0[G::TM], rb0[G::TN], ra1[G::TM], rb1[G::TN];
  load_b(0, rb0);
  load_a(0, ra0);
  load_b(1, rb1);
  load_a(1, ra1);
  // the prefetches are unconditional (clamped to the last chunk) so the compiler's
  // vmcnt/lgkmcnt bookkeeping stays exact: each MFMA group waits only for its own chunk
  for (int s = 0; s < STEPS; s += 2) {
    mma(ra0, rb0);
    const int s2 = s + 2 < STEPS ? s + 2 : STEPS - 2;
    load_b(s2, rb0);
    load_a(s2, ra0);
    mma(ra1, rb1);
    const int s3 = s + 3 < STEPS ? s + 3 : STEPS - 1;
    load_b(s3, rb1);
    load_a(s3, ra1);
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

// Stem: Ci = 1 (the canonical board plane), 9 taps.  One board per workgroup: its 64 plane values in LDS, each thread's 4 channels' 9 tap
// weights in registers, 8 positions per thread; a wave stores two whole 512-byte position
// rows per instruction.  Same tap order and fmaf chain per output as every other stem
// evaluation (az_conv3x3_mx_stem_gpu relies on bit-identity).
template <int CO>
__global__ __launch_bounds__(256) void k_conv_stem(const float* __restrict__ planes,
                                                   const float* __restrict__ w,
                                                   const float* __restrict__ bias,
                                                   float* __restrict__ y, int64_t n_boards,
                                                   float* __restrict__ absmax) {
  __shared__ float s_max[4];
  constexpr int G4 = CO / 4;            // float4 channel groups per position
  constexpr int PPI = 256 / G4;         // positions per pass of the workgroup
  __shared__ float s_pl[64];
  const int tid = threadIdx.x;
  const int co = (tid % G4) * 4;
  float4 wv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wv[t] = *reinterpret_cast<const float4*>(w + t * CO + co);
  const float4 bv = *reinterpret_cast<const float4*>(bias + co);
  for (int64_t b = blockIdx.x; b < n_boards; b += gridDim.x) {
    __syncthreads();  // the previous board's planes are no longer read
    if (tid < 64) s_pl[tid] = planes[b * 64 + tid];
    __syncthreads();
    float4* out = reinterpret_cast<float4*>(y + b * 64 * CO);
    float bmax = 0.0f;
#pragma unroll
    for (int p0 = 0; p0 < 64; p0 += PPI) {
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
    if (absmax) {  // the board's max |y| (outputs are >= 0 after the ReLU)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) bmax = fmaxf(bmax, __shfl_xor(bmax, off, 64));
      if ((tid & 63) == 0) s_max[tid >> 6] = bmax;
      __syncthreads();
      if (tid == 0) absmax[b] = fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]));
    }
  }
}

template <class G>
int launch_conv(const float* x, const float* w, const float* bias, const float* res, float* y,
                int n_boards, int relu, hipStream_t s) {
  const unsigned grid = (unsigned)((n_boards + G::BOARDS - 1) / G::BOARDS);
  const size_t lds = (size_t)(G::BOARDS * 64 + 1) * G::S * sizeof(float);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS needs the opt-in once per kernel
  if (!attr_set) {
    const void* ks[] = {(const void*)k_conv3x3<G, true, true>, (const void*)k_conv3x3<G, true, false>,
                        (const void*)k_conv3x3<G, false, true>, (const void*)k_conv3x3<G, false, false>};
    for (const void* k : ks)
      AZ_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = true;
  }
  const dim3 blk(G::THREADS);
  if (res && relu)
    hipLaunchKernelGGL((k_conv3x3<G, true, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else if (res)
    hipLaunchKernelGGL((k_conv3x3<G, true, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else if (relu)
    hipLaunchKernelGGL((k_conv3x3<G, false, true>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  else
    hipLaunchKernelGGL((k_conv3x3<G, false, false>), dim3(grid), blk, lds, s, x, w, bias, res, y, n_boards);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

// tiling candidates (C, boards, waves, TM, TN); index 0 of each C is the default, picked
// by scripts/conv_bench.py on MI355X with the pipelined main loop (B = 1024, one run:
// C=128 164 us = 118 TFLOP/s vs MIOpen's 191 us for the bare convolution; C=64 49 us vs 57)
using G128_0 = Geo<128, 2, 4, 2, 2>;
using G128_1 = Geo<128, 1, 2, 2, 2>;
using G128_2 = Geo<128, 4, 8, 2, 2>;
using G128_3 = Geo<128, 2, 2, 4, 2>;
using G128_4 = Geo<128, 4, 4, 4, 2>;
using G128_5 = Geo<128, 2, 8, 1, 2>;
using G64_0 = Geo<64, 4, 4, 2, 2>;
using G64_1 = Geo<64, 1, 2, 1, 2>;
using G64_2 = Geo<64, 4, 2, 4, 2>;

int launch_cfg(int cfg, const float* x, const float* w, const float* bias, const float* res,
               float* y, int n_boards, int channels, int relu, hipStream_t s) {
  if (channels == 128) {
    switch (cfg) {
      case 0: return launch_conv<G128_0>(x, w, bias, res, y, n_boards, relu, s);
      case 1: return launch_conv<G128_1>(x, w, bias, res, y, n_boards, relu, s);
      case 2: return launch_conv<G128_2>(x, w, bias, res, y, n_boards, relu, s);
      case 3: return launch_conv<G128_3>(x, w, bias, res, y, n_boards, relu, s);
      case 4: return launch_conv<G128_4>(x, w, bias, res, y, n_boards, relu, s);
      case 5: return launch_conv<G128_5>(x, w, bias, res, y, n_boards, relu, s);
    }
  } else if (channels == 64) {
    switch (cfg) {
      case 0: return launch_conv<G64_0>(x, w, bias, res, y, n_boards, relu, s);
      case 1: return launch_conv<G64_1>(x, w, bias, res, y, n_boards, relu, s);
      case 2: return launch_conv<G64_2>(x, w, bias, res, y, n_boards, relu, s);
    }
  }
  return azc::set_error(AZ_ERR_ARG, "az_conv3x3: no tiling %d for %d channels", cfg, channels);
}

}  // namespace

extern "C" int az_conv3x3_gpu(const float* x, const float* w9, const float* bias,
                              const float* res, float* y, int32_t n_boards, int32_t channels,
                              int32_t relu, void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_conv3x3_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && w9 && bias && y && x != y, AZ_ERR_ARG,
             "az_conv3x3_gpu: null buffer or in-place call");
  AZ_REQUIRE(((uintptr_t)x | (uintptr_t)w9 | (uintptr_t)bias) % 16 == 0, AZ_ERR_ARG,
             "az_conv3x3_gpu: buffers must be 16-byte aligned");
  AZ_REQUIRE(channels == 64 || channels == 128, AZ_ERR_ARG,
             "az_conv3x3_gpu: channels must be 64 or 128, got %d", channels);
  return launch_cfg(0, x, w9, bias, res, y, n_boards, channels, relu, azc::as_stream(stream));
}

// same op with an explicit tiling candidate (benchmarking the tile space)
extern "C" int az_conv3x3_cfg_gpu(const float* x, const float* w9, const float* bias,
                                  const float* res, float* y, int32_t n_boards,
                                  int32_t channels, int32_t relu, int32_t cfg, void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_conv3x3_cfg_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(x && w9 && bias && y && x != y, AZ_ERR_ARG, "az_conv3x3_cfg_gpu: bad buffers");
  return launch_cfg(cfg, x, w9, bias, res, y, n_boards, channels, relu, azc::as_stream(stream));
}

extern "C" int az_conv_stem_gpu(const float* planes, const float* w9, const float* bias,
                                float* y, int32_t n_boards, int32_t channels, void* stream) {
  return az_conv_stem2_gpu(planes, w9, bias, y, n_boards, channels, nullptr, stream);
}

extern "C" int az_conv_stem2_gpu(const float* planes, const float* w9, const float* bias,
                                 float* y, int32_t n_boards, int32_t channels, float* absmax,
                                 void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_conv_stem_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(planes && w9 && bias && y, AZ_ERR_ARG, "az_conv_stem_gpu: null buffer");
  hipStream_t s = azc::as_stream(stream);
  const int64_t blocks = n_boards < 8192 ? n_boards : 8192;  // one board per workgroup pass
  if (channels == 128)
    hipLaunchKernelGGL(k_conv_stem<128>, dim3((unsigned)blocks), dim3(256), 0, s, planes, w9,
                       bias, y, (int64_t)n_boards, absmax);
  else if (channels == 64)
    hipLaunchKernelGGL(k_conv_stem<64>, dim3((unsigned)blocks), dim3(256), 0, s, planes, w9,
                       bias, y, (int64_t)n_boards, absmax);
  else
    return azc::set_error(AZ_ERR_ARG, "az_conv_stem_gpu: channels must be 64 or 128");
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
