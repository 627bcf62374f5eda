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

constexpr int kBoards = 2;  // boards per workgroup
constexpr int kThreads = 256;

template <int C>
struct Geo {
  static constexpr int S = C + 4;                  // LDS floats per position (padded)
  static constexpr int TM = C == 128 ? 2 : 1;      // 32-row MFMA tiles per wave
  static constexpr int TN = 2;                     // 32-col MFMA tiles per wave
  static constexpr int WM = 32 * TM;               // rows per wave
  static constexpr int WN = 32 * TN;               // cols per wave
  static constexpr int WAVES_N = C / WN;           // waves along N
  static_assert((kBoards * 64 / WM) * WAVES_N == 4, "4 waves per workgroup");
};

template <int C, bool RES, bool RELU>
__global__ __launch_bounds__(kThreads, 2) void k_conv3x3(const float* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ res,
                                                         float* __restrict__ y, int n_boards) {
  using G = Geo<C>;
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int b0 = blockIdx.x * kBoards;
  const int nb = n_boards - b0 < kBoards ? n_boards - b0 : kBoards;

  // ---- stage the input boards (NHWC) into LDS, zero-fill a missing tail board
  {
    constexpr int V = kBoards * 64 * C / 4;  // float4s
    const float4* src = reinterpret_cast<const float4*>(x + (size_t)b0 * 64 * C);
    for (int v = tid; v < V; v += kThreads) {
      const int pos = v / (C / 4), c4 = v % (C / 4);
      float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
      if (pos < nb * 64) val = src[v];
      *reinterpret_cast<float4*>(lds + pos * G::S + c4 * 4) = val;
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
  auto load_a = [&](int s, float4 (&a)[G::TM]) {
    const int tap = s / CHUNKS, ci0 = (s % CHUNKS) * 8;
    const int ky = tap / 3 - 1, kx = tap % 3 - 1;
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi) {
      const int yy = py[mi] + ky, xx = px[mi] + kx;
      const bool ok = (unsigned)yy < 8u && (unsigned)xx < 8u;
      const int pos = pb[mi] * 64 + (ok ? yy * 8 + xx : 0);
      const float4 v = *reinterpret_cast<const float4*>(lds + pos * G::S + ci0 + 4 * h);
      a[mi] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };

  float4 a_cur[G::TM], b_cur[G::TN], a_nxt[G::TM], b_nxt[G::TN];
  load_b(0, b_cur);
  load_a(0, a_cur);
  for (int s = 0; s < STEPS; ++s) {
    if (s + 1 < STEPS) {
      load_b(s + 1, b_nxt);
      load_a(s + 1, a_nxt);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi) {
        const float av = j == 0 ? a_cur[mi].x : j == 1 ? a_cur[mi].y : j == 2 ? a_cur[mi].z : a_cur[mi].w;
#pragma unroll
        for (int ni = 0; ni < G::TN; ++ni) {
          const float bv = j == 0 ? b_cur[ni].x : j == 1 ? b_cur[ni].y : j == 2 ? b_cur[ni].z : b_cur[ni].w;
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[mi][ni], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi) a_cur[mi] = a_nxt[mi];
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni) b_cur[ni] = b_nxt[ni];
  }

  // ---- epilogue: D[row][col], col = lane&31, row = (k&3) + 8*(k>>2) + 4*(lane>>5)
#pragma unroll
  for (int ni = 0; ni < G::TN; ++ni) {
    const int co = col0 + 32 * ni + r;
    const float bv = bias[co];
#pragma unroll
    for (int mi = 0; mi < G::TM; ++mi) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int m = row0 + 32 * mi + (k & 3) + 8 * (k >> 2) + 4 * h;
        if ((m >> 6) >= nb) continue;
        const size_t o = ((size_t)b0 * 64 + m) * C + co;
        float v = acc[mi][ni][k] + bv;
        if (RES) v += res[o];
        if (RELU) v = fmaxf(v, 0.0f);
        y[o] = v;
      }
    }
  }
}

// Stem: Ci = 1 (the canonical board plane), 9 taps; one thread per (position, 4 channels).
template <int CO>
__global__ __launch_bounds__(256) void k_conv_stem(const float* __restrict__ planes,
                                                   const float* __restrict__ w,
                                                   const float* __restrict__ bias,
                                                   float* __restrict__ y, int64_t n_out4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_out4;
       i += (int64_t)gridDim.x * 256) {
    const int64_t pos = i / (CO / 4);
    const int co = (int)(i % (CO / 4)) * 4;
    const int64_t b = pos >> 6;
    const int p = (int)(pos & 63), py = p >> 3, px = p & 7;
    const float* in = planes + b * 64;
    float4 acc = *reinterpret_cast<const float4*>(bias + co);
    // same tap order as the MFMA path (tap-major); one fma chain per output
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
      if ((unsigned)yy < 8u && (unsigned)xx < 8u) {
        const float v = in[yy * 8 + xx];
        const float4 wv = *reinterpret_cast<const float4*>(w + t * CO + co);
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
    reinterpret_cast<float4*>(y)[i] = acc;
  }
}

template <int C>
int launch_conv(const float* x, const float* w, const float* bias, const float* res, float* y,
                int n_boards, int relu, hipStream_t s) {
  const unsigned grid = (unsigned)((n_boards + kBoards - 1) / kBoards);
  const size_t lds = (size_t)kBoards * 64 * Geo<C>::S * sizeof(float);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS needs the opt-in once per kernel
  if (!attr_set) {
    const void* ks[] = {(const void*)k_conv3x3<C, true, true>, (const void*)k_conv3x3<C, true, false>,
                        (const void*)k_conv3x3<C, false, true>, (const void*)k_conv3x3<C, false, false>};
    for (const void* k : ks)
      AZ_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = true;
  }
  if (res && relu)
    hipLaunchKernelGGL((k_conv3x3<C, true, true>), dim3(grid), dim3(kThreads), lds, s, x, w, bias, res, y, n_boards);
  else if (res)
    hipLaunchKernelGGL((k_conv3x3<C, true, false>), dim3(grid), dim3(kThreads), lds, s, x, w, bias, res, y, n_boards);
  else if (relu)
    hipLaunchKernelGGL((k_conv3x3<C, false, true>), dim3(grid), dim3(kThreads), lds, s, x, w, bias, res, y, n_boards);
  else
    hipLaunchKernelGGL((k_conv3x3<C, false, false>), dim3(grid), dim3(kThreads), lds, s, x, w, bias, res, y, n_boards);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
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
  hipStream_t s = azc::as_stream(stream);
  if (channels == 128) return launch_conv<128>(x, w9, bias, res, y, n_boards, relu, s);
  if (channels == 64) return launch_conv<64>(x, w9, bias, res, y, n_boards, relu, s);
  return azc::set_error(AZ_ERR_ARG, "az_conv3x3_gpu: channels must be 64 or 128, got %d",
                        channels);
}

extern "C" int az_conv_stem_gpu(const float* planes, const float* w9, const float* bias,
                                float* y, int32_t n_boards, int32_t channels, void* stream) {
  AZ_REQUIRE(n_boards >= 0, AZ_ERR_ARG, "az_conv_stem_gpu: n_boards < 0");
  if (n_boards == 0) return AZ_OK;
  AZ_REQUIRE(planes && w9 && bias && y, AZ_ERR_ARG, "az_conv_stem_gpu: null buffer");
  hipStream_t s = azc::as_stream(stream);
  const int64_t n4 = (int64_t)n_boards * 64 * channels / 4;
  int64_t blocks = (n4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (channels == 128)
    hipLaunchKernelGGL(k_conv_stem<128>, dim3((unsigned)blocks), dim3(256), 0, s, planes, w9,
                       bias, y, n4);
  else if (channels == 64)
    hipLaunchKernelGGL(k_conv_stem<64>, dim3((unsigned)blocks), dim3(256), 0, s, planes, w9,
                       bias, y, n4);
  else
    return azc::set_error(AZ_ERR_ARG, "az_conv_stem_gpu: channels must be 64 or 128");
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
