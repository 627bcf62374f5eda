// nn_fused.hip — fused conv epilogue for the policy/value net's inference copy.
//
// The leaf-evaluation net (reference Models.py:72-221, BatchNorm folded into the
// convolutions) runs its convolutions through MIOpen without a bias; this kernel then
// applies, in one pass over the channels-last (NHWC) activation, what PyTorch would run as
// two to four separate elementwise kernels: + bias[c], + residual (ResidualBlock's
// `out += residual`, Models.py:84-86), ReLU.  HBM-bound: 8 B (no residual) or 12 B
// (residual) per element, 16-byte vector accesses.
#include "common.h"

namespace {

constexpr int kBlock = 256;

template <bool RES, bool RELU>
__global__ __launch_bounds__(kBlock) void k_bias_act4(float4* __restrict__ y,
                                                      const float* __restrict__ bias,
                                                      const float4* __restrict__ res,
                                                      int64_t n4, int C) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n4; j += stride) {
    const int c0 = (int)((j * 4) % C);
    const float4 b = *reinterpret_cast<const float4*>(bias + c0);
    float4 v = y[j];
    v.x += b.x;
    v.y += b.y;
    v.z += b.z;
    v.w += b.w;
    if (RES) {
      const float4 r = res[j];
      v.x += r.x;
      v.y += r.y;
      v.z += r.z;
      v.w += r.w;
    }
    if (RELU) {
      v.x = fmaxf(v.x, 0.0f);
      v.y = fmaxf(v.y, 0.0f);
      v.z = fmaxf(v.z, 0.0f);
      v.w = fmaxf(v.w, 0.0f);
    }
    y[j] = v;
  }
}

__global__ __launch_bounds__(kBlock) void k_bias_act1(float* __restrict__ y,
                                                      const float* __restrict__ bias,
                                                      const float* __restrict__ res, int64_t n,
                                                      int C, int relu) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    float v = y[i] + bias[i % C];
    if (res) v += res[i];
    y[i] = relu ? fmaxf(v, 0.0f) : v;
  }
}

unsigned grid_for(int64_t n) {
  const int64_t b = (n + kBlock - 1) / kBlock;
  return (unsigned)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

}  // namespace

extern "C" int az_bias_act_gpu(float* y, const float* bias, const float* res, int64_t n,
                               int32_t channels, int32_t relu, void* stream) {
  AZ_REQUIRE(n >= 0 && channels > 0, AZ_ERR_ARG, "az_bias_act_gpu: bad n/channels");
  if (n == 0) return AZ_OK;
  AZ_REQUIRE(y && bias && n % channels == 0, AZ_ERR_ARG,
             "az_bias_act_gpu: null buffer or n %% channels != 0");
  hipStream_t s = azc::as_stream(stream);
  const bool vec = channels % 4 == 0 && ((uintptr_t)y % 16) == 0 && ((uintptr_t)bias % 16) == 0 &&
                   (!res || ((uintptr_t)res % 16) == 0);
  if (vec) {
    const int64_t n4 = n / 4;
    float4* y4 = reinterpret_cast<float4*>(y);
    const float4* r4 = reinterpret_cast<const float4*>(res);
    if (res && relu)
      hipLaunchKernelGGL((k_bias_act4<true, true>), dim3(grid_for(n4)), dim3(kBlock), 0, s, y4,
                         bias, r4, n4, channels);
    else if (res)
      hipLaunchKernelGGL((k_bias_act4<true, false>), dim3(grid_for(n4)), dim3(kBlock), 0, s, y4,
                         bias, r4, n4, channels);
    else if (relu)
      hipLaunchKernelGGL((k_bias_act4<false, true>), dim3(grid_for(n4)), dim3(kBlock), 0, s, y4,
                         bias, r4, n4, channels);
    else
      hipLaunchKernelGGL((k_bias_act4<false, false>), dim3(grid_for(n4)), dim3(kBlock), 0, s,
                         y4, bias, r4, n4, channels);
  } else {
    hipLaunchKernelGGL(k_bias_act1, dim3(grid_for(n)), dim3(kBlock), 0, s, y, bias, res, n,
                       channels, relu);
  }
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
