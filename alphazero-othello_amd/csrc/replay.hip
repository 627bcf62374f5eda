// replay.hip — replay-buffer aggregation on the device: the reference's
// Trainer._aggregate_duplicates (train.py:142-173) over bitboard rows.
//
// Rows with equal (own, opp, version) — the reference keys on sha1(int8 canonical board)
// and the model version — collapse into one sample: mean pi (float32 sum in buffer order,
// / count, then / (NumPy-pairwise sum + 1e-12)) and mean value (float64 sum, / count,
// cast to float32), emitted in order of first occurrence.  Bit-exact with the reference
// (tests/test_replay_gpu.py against tests/golden/replay_aggregate.npz).
//
//   1. stable LSD radix sort of row indices by version, then opp, then own (hipCUB):
//      equal keys become adjacent and keep buffer order inside a group;
//   2. group heads flagged and numbered (inclusive scan);
//   3. one wavefront per group sums its rows in order (lane = pi entry) and normalises;
//   4. groups sorted by their first row index (= first occurrence), results gathered.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// NumPy's pairwise sum of a contiguous length-65 float32 vector: eight running partials
// over the first 64 elements, ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the tail element.
__device__ float np_sum65f(float x, float x64) {
  const int lane = lane_id();
  float r = x;
#pragma unroll
  for (int i = 1; i < 8; ++i) r = r + __shfl(x, (lane + 8 * i) & 63, 64);
  const float r0 = __shfl(r, 0, 64), r1 = __shfl(r, 1, 64), r2 = __shfl(r, 2, 64),
              r3 = __shfl(r, 3, 64), r4 = __shfl(r, 4, 64), r5 = __shfl(r, 5, 64),
              r6 = __shfl(r, 6, 64), r7 = __shfl(r, 7, 64);
  return (((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))) + x64;
}

__global__ void k_iota(int32_t* idx, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    idx[i] = (int32_t)i;
}

// keys of the next sort pass, gathered through the current order
__global__ void k_gather_u64(const uint64_t* __restrict__ src, const int32_t* __restrict__ idx,
                             uint64_t* __restrict__ dst, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

__global__ void k_heads(const uint64_t* __restrict__ own, const uint64_t* __restrict__ opp,
                        const int32_t* __restrict__ ver, const int32_t* __restrict__ idx,
                        int32_t* __restrict__ head, int64_t n) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    int32_t h = 1;
    if (j > 0) {
      const int32_t a = idx[j], b = idx[j - 1];
      h = own[a] != own[b] || opp[a] != opp[b] || ver[a] != ver[b];
    }
    head[j] = h;
  }
}

__global__ void k_init_groups(int32_t* __restrict__ first, int32_t* __restrict__ gnum,
                              int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    first[i] = 0x7fffffff;  // slots past the group count sort last
    gnum[i] = (int32_t)i;
  }
}

// group g starts at sorted position start[g]; its first row (in buffer order) keys the
// output order
__global__ void k_starts(const int32_t* __restrict__ head, const int32_t* __restrict__ gid,
                         const int32_t* __restrict__ idx, int32_t* __restrict__ start,
                         int32_t* __restrict__ first, int32_t* __restrict__ gnum,
                         int64_t n) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    if (head[j]) {
      const int g = gid[j] - 1;
      start[g] = (int32_t)j;
      first[g] = idx[j];
      gnum[g] = g;
    }
    if (j == n - 1) start[gid[j]] = (int32_t)n;  // sentinel after the last group
  }
}

// one wavefront per output sample: its group's rows summed in buffer order
__global__ __launch_bounds__(256) void k_reduce(
    const float* __restrict__ pi, const double* __restrict__ v, const uint64_t* __restrict__ own,
    const uint64_t* __restrict__ opp, const int32_t* __restrict__ ver,
    const int32_t* __restrict__ idx, const int32_t* __restrict__ start,
    const int32_t* __restrict__ gorder, const int32_t* __restrict__ n_groups_p,
    uint64_t* __restrict__ own_o, uint64_t* __restrict__ opp_o, int32_t* __restrict__ ver_o,
    float* __restrict__ pi_o, float* __restrict__ v_o, int32_t* __restrict__ count_o) {
  const int lane = lane_id();
  const int n_groups = *n_groups_p;
  for (int o = blockIdx.x * 4 + (threadIdx.x >> 6); o < n_groups; o += gridDim.x * 4) {
    const int g = gorder[o];
    const int j0 = start[g], j1 = start[g + 1];
    float s = 0.f, s64 = 0.f;
    double sv = 0.0;
    for (int j = j0; j < j1; ++j) {
      const int r = idx[j];
      const float x = pi[(size_t)r * 65 + lane];
      const float x64 = pi[(size_t)r * 65 + 64];
      if (j == j0) {  // sum_pi = pi.copy(); sum_v = v
        s = x;
        s64 = x64;
        sv = v[r];
      } else {        // sum_pi += pi; sum_v += v
        s = s + x;
        s64 = s64 + x64;
        sv = sv + v[r];
      }
    }
    const int cnt = j1 - j0;
    const float fc = (float)cnt;
    const float a = s / fc, a64 = s64 / fc;           // sum_pi / cnt
    const float den = np_sum65f(a, a64) + 1e-12f;     // avg_pi.sum() + 1e-12
    pi_o[(size_t)o * 65 + lane] = a / den;
    if (lane == 0) {
      pi_o[(size_t)o * 65 + 64] = a64 / den;
      const int r0 = idx[j0];
      own_o[o] = own[r0];
      opp_o[o] = opp[r0];
      ver_o[o] = ver[r0];
      v_o[o] = (float)(sv / (double)cnt);
      count_o[o] = cnt;
    }
  }
}

unsigned grid1(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

extern "C" int az_replay_aggregate_gpu(const uint64_t* own, const uint64_t* opp,
                                       const int32_t* ver, const float* pi, const double* v,
                                       int64_t n, uint64_t* own_o, uint64_t* opp_o,
                                       int32_t* ver_o, float* pi_o, float* v_o,
                                       int32_t* count_o, int32_t* n_out, void* workspace,
                                       size_t* workspace_bytes, void* stream) {
  AZ_REQUIRE(n >= 0 && n < (int64_t(1) << 31) - 1, AZ_ERR_ARG,
             "az_replay_aggregate_gpu: n=%lld out of range", (long long)n);
  AZ_REQUIRE(workspace_bytes, AZ_ERR_ARG, "az_replay_aggregate_gpu: null workspace_bytes");
  hipStream_t s = azc::as_stream(stream);
  const int N = (int)(n > 0 ? n : 1);
  // workspace: idx x2, keys u64 x2, head, gid, start (N+1), first x2, gnum x2, cub temp
  size_t cub_bytes = 0, t = 0;
  AZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, t, (const uint64_t*)nullptr,
                                            (uint64_t*)nullptr, (const int32_t*)nullptr,
                                            (int32_t*)nullptr, N, 0, 64, s));
  cub_bytes = t > cub_bytes ? t : cub_bytes;
  AZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, t, (const int32_t*)nullptr,
                                            (int32_t*)nullptr, (const int32_t*)nullptr,
                                            (int32_t*)nullptr, N, 0, 32, s));
  cub_bytes = t > cub_bytes ? t : cub_bytes;
  AZ_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, t, (const int32_t*)nullptr,
                                          (int32_t*)nullptr, N, s));
  cub_bytes = t > cub_bytes ? t : cub_bytes;
  const size_t i32 = align256((size_t)(N + 1) * 4), u64 = align256((size_t)N * 8);
  const size_t need = 2 * i32 + 2 * u64 + 2 * i32 + i32 + 4 * i32 + align256(cub_bytes);
  if (!workspace) {
    *workspace_bytes = need;
    return AZ_OK;
  }
  AZ_REQUIRE(*workspace_bytes >= need, AZ_ERR_ARG,
             "az_replay_aggregate_gpu: workspace %zu < %zu bytes", *workspace_bytes, need);
  AZ_REQUIRE(n_out, AZ_ERR_ARG, "az_replay_aggregate_gpu: null n_out");
  if (n == 0) {
    AZ_HIP(hipMemsetAsync(n_out, 0, sizeof(int32_t), s));
    return AZ_OK;
  }
  AZ_REQUIRE(own && opp && ver && pi && v && own_o && opp_o && ver_o && pi_o && v_o && count_o,
             AZ_ERR_ARG, "az_replay_aggregate_gpu: null buffer");
  char* w = static_cast<char*>(workspace);
  auto take = [&](size_t b) { char* p = w; w += b; return p; };
  int32_t* idx_a = (int32_t*)take(i32);
  int32_t* idx_b = (int32_t*)take(i32);
  uint64_t* key_a = (uint64_t*)take(u64);
  uint64_t* key_b = (uint64_t*)take(u64);
  int32_t* head = (int32_t*)take(i32);
  int32_t* gid = (int32_t*)take(i32);
  int32_t* start = (int32_t*)take(i32);
  int32_t* first_a = (int32_t*)take(i32);
  int32_t* first_b = (int32_t*)take(i32);
  int32_t* gnum_a = (int32_t*)take(i32);
  int32_t* gnum_b = (int32_t*)take(i32);
  void* cub_tmp = take(align256(cub_bytes));
  size_t cub_sz = cub_bytes;
  const unsigned g = grid1(n);

  // 1. stable LSD sort: version, then opp, then own
  hipLaunchKernelGGL(k_iota, dim3(g), dim3(256), 0, s, idx_a, n);
  AZ_HIP(hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_sz, ver, (int32_t*)key_b, idx_a, idx_b,
                                            (int)n, 0, 32, s));
  hipLaunchKernelGGL(k_gather_u64, dim3(g), dim3(256), 0, s, opp, idx_b, key_a, n);
  cub_sz = cub_bytes;
  AZ_HIP(hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_sz, key_a, key_b, idx_b, idx_a,
                                            (int)n, 0, 64, s));
  hipLaunchKernelGGL(k_gather_u64, dim3(g), dim3(256), 0, s, own, idx_a, key_a, n);
  cub_sz = cub_bytes;
  AZ_HIP(hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_sz, key_a, key_b, idx_a, idx_b,
                                            (int)n, 0, 64, s));
  // 2. group heads and numbers
  hipLaunchKernelGGL(k_heads, dim3(g), dim3(256), 0, s, own, opp, ver, idx_b, head, n);
  cub_sz = cub_bytes;
  AZ_HIP(hipcub::DeviceScan::InclusiveSum(cub_tmp, cub_sz, head, gid, (int)n, s));
  hipLaunchKernelGGL(k_init_groups, dim3(g), dim3(256), 0, s, first_a, gnum_a, n);
  hipLaunchKernelGGL(k_starts, dim3(g), dim3(256), 0, s, head, gid, idx_b, start, first_a,
                     gnum_a, n);
  // group count = gid[n-1]
  AZ_HIP(hipMemcpyAsync(n_out, gid + (n - 1), sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  // 4. groups in order of first occurrence (the group count is only known on the device:
  // all n slots are sorted, the unused ones keyed INT32_MAX so they land at the end)
  cub_sz = cub_bytes;
  AZ_HIP(hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_sz, first_a, first_b, gnum_a, gnum_b,
                                            (int)n, 0, 32, s));
  // 3. per-group reduction, written in output order
  hipLaunchKernelGGL(k_reduce, dim3(g < 1024 ? g : 1024), dim3(256), 0, s, pi, v, own, opp, ver,
                     idx_b, start, gnum_b, n_out, own_o, opp_o, ver_o, pi_o, v_o, count_o);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}
