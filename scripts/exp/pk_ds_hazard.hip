// pk_ds_hazard.hip -- does an LDS store read its data VGPRs before a just-issued packed-FP32
// (or FP64) VALU result has been written?  (the heads' lanes 48-63 words.)
//
// Each wave repeatedly: moves x, y into v[200:205], runs the producer instruction into
// v[200:201], optionally some filler, then `ds_write_b128 addr, v[200:203]`, waits
// lgkmcnt(0), reads the quad back with plain code and compares it with the producer's result
// computed the ordinary way.  Mismatches are counted per lane (and, separately, those equal to
// the producer's INPUT, i.e. a stale register).  The grid puts 8 waves on every SIMD, and
// every wave runs a chain of independent v_pk_fma_f32 between iterations to keep the packed
// pipe busy -- the contention under which the heads saw the wrong words.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/exp/pk_ds_hazard.hip -o expbuild/pk_ds_hazard
//   ./expbuild/pk_ds_hazard [iters]      -> one JSON line per variant
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

#define CLOB "v200", "v201", "v202", "v203", "v204", "v205", "v206", "memory"
#define LOAD                                                                        \
  "v_mov_b32 v200, %1\n v_mov_b32 v201, %2\n v_mov_b32 v202, %2\n v_mov_b32 v203, %1\n" \
  "v_mov_b32 v204, %2\n v_mov_b32 v205, %1\n s_nop 7\n s_nop 7\n"

// producer + filler variants; result quad = (x+y, y+x, y, x) (f32 forms)
template <int V>
__device__ __forceinline__ void produce_store(unsigned addr, float x, float y) {
  if constexpr (V == 0)  // packed add, store right after
    asm volatile(LOAD "v_pk_add_f32 v[200:201], v[200:201], v[204:205]\n"
                      "ds_write_b128 %0, v[200:203]\n s_waitcnt lgkmcnt(0)\n"
                 :: "v"(addr), "v"(x), "v"(y) : CLOB);
  else if constexpr (V == 1)  // one wait state (s_nop 0) between
    asm volatile(LOAD "v_pk_add_f32 v[200:201], v[200:201], v[204:205]\n s_nop 0\n"
                      "ds_write_b128 %0, v[200:203]\n s_waitcnt lgkmcnt(0)\n"
                 :: "v"(addr), "v"(x), "v"(y) : CLOB);
  else if constexpr (V == 2)  // one independent VALU between
    asm volatile(LOAD "v_pk_add_f32 v[200:201], v[200:201], v[204:205]\n v_mov_b32 v206, 0\n"
                      "ds_write_b128 %0, v[200:203]\n s_waitcnt lgkmcnt(0)\n"
                 :: "v"(addr), "v"(x), "v"(y) : CLOB);
  else if constexpr (V == 3)  // two wait states
    asm volatile(LOAD "v_pk_add_f32 v[200:201], v[200:201], v[204:205]\n s_nop 1\n"
                      "ds_write_b128 %0, v[200:203]\n s_waitcnt lgkmcnt(0)\n"
                 :: "v"(addr), "v"(x), "v"(y) : CLOB);
  else if constexpr (V == 4)  // control: two plain fp32 adds, store right after
    asm volatile(LOAD "v_add_f32 v200, v200, v204\n v_add_f32 v201, v201, v205\n"
                      "ds_write_b128 %0, v[200:203]\n s_waitcnt lgkmcnt(0)\n"
                 :: "v"(addr), "v"(x), "v"(y) : CLOB);
  else if constexpr (V == 5)  // packed mul (x*y, y*x)
    asm volatile(LOAD "v_pk_mul_f32 v[200:201], v[200:201], v[204:205]\n"
                      "ds_write_b128 %0, v[200:203]\n s_waitcnt lgkmcnt(0)\n"
                 :: "v"(addr), "v"(x), "v"(y) : CLOB);
  else if constexpr (V == 6)  // packed fma (x*y + y, y*x + x): src2 = v[202:203]
    asm volatile(LOAD "v_pk_fma_f32 v[200:201], v[200:201], v[204:205], v[202:203]\n"
                      "ds_write_b128 %0, v[200:203]\n s_waitcnt lgkmcnt(0)\n"
                 :: "v"(addr), "v"(x), "v"(y) : CLOB);
}

// V == 7: the heads' sequence (heads_az.h val_fc1 quad, round 3's failing build): a packed mul
// feeding a packed add, an independent packed add into the quad's other half, one SALU, the
// store -- quad = (x + x*y, y + y*x, 2y, 2x)
template <>
__device__ __forceinline__ void produce_store<7>(unsigned addr, float x, float y) {
  asm volatile(LOAD
               "v_pk_mul_f32 v[206:207], v[200:201], v[204:205]\n"
               "v_pk_add_f32 v[200:201], v[200:201], v[206:207]\n"
               "v_pk_add_f32 v[202:203], v[202:203], v[204:205]\n"
               "s_add_i32 s0, 0, 0x10200\n"
               "ds_write_b128 %0, v[200:203]\n s_waitcnt lgkmcnt(0)\n"
               :: "v"(addr), "v"(x), "v"(y) : CLOB, "v207", "s0");
}

template <int V>
__device__ __forceinline__ float4 expect(float x, float y) {
  if constexpr (V == 7)  // no contraction: the asm rounds the product, then the sum
    return {__fadd_rn(x, __fmul_rn(x, y)), __fadd_rn(y, __fmul_rn(y, x)), __fadd_rn(y, y),
            __fadd_rn(x, x)};
  if constexpr (V == 5) return {__fmul_rn(x, y), __fmul_rn(y, x), y, x};
  if constexpr (V == 6) return {__fmaf_rn(x, y, y), __fmaf_rn(y, x, x), y, x};
  return {__fadd_rn(x, y), __fadd_rn(y, x), y, x};
}

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int V>
__global__ __launch_bounds__(512) void k_probe(const float* __restrict__ in,
                                               unsigned* __restrict__ bad,
                                               unsigned* __restrict__ stale, int iters,
                                               int busy) {
  __shared__ float4 buf[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w >= 4) {  // MFMA companions (mfma mode): the same SIMDs kept busy with MFMA chains
    h8 a, b;
    for (int i = 0; i < 8; ++i) {
      a[i] = (_Float16)(in[(lane * 8 + i) & 4095]);
      b[i] = (_Float16)(in[(lane * 8 + i + 99) & 4095]);
    }
    f16v acc = {};
    for (int it = 0; it < iters; ++it)
      for (int k = 0; k < 4; ++k) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    float sgn = 0.f;
    for (int e = 0; e < 16; ++e) sgn += acc[e];
    if (sgn == 12345.f) atomicAdd(&bad[lane], 1u << 30);  // keep the chain alive
    return;
  }
  const unsigned addr = (unsigned)(size_t)(&buf[w][lane]);
  float x = in[(blockIdx.x * 256 + threadIdx.x) & 4095];
  float y = in[(blockIdx.x * 256 + threadIdx.x + 1777) & 4095];
  float2 p = {x, y}, q = {y, x};
  unsigned nb = 0, ns = 0;
  for (int it = 0; it < iters; ++it) {
    produce_store<V>(addr, x, y);
    const float4 got = buf[w][lane];
    const float4 want = expect<V>(x, y);
    if (got.x != want.x || got.y != want.y || got.z != want.z || got.w != want.w) {
      ++nb;
      if (got.x == x || got.y == y) ++ns;  // the producer's input: a stale register
    }
    // keep the packed-FP32 pipe busy (independent of the probe's registers)
    for (int k = 0; k < busy; ++k) {
      asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p) : "v"(q));
    }
    x = x * 1.000061f + 0.25f;
    y = y * 0.999939f - 0.125f;
  }
  if (p.x == 12345.f) nb += 1u << 30;  // keep the busy chain alive
  atomicAdd(&bad[lane], nb);
  atomicAdd(&stale[lane], ns);
}

template <int V>
void run(const char* name, int iters, int busy, int blocks, const float* d_in, unsigned* d_bad,
         unsigned* d_stale) {
  CHECK(hipMemset(d_bad, 0, 64 * 4));
  CHECK(hipMemset(d_stale, 0, 64 * 4));
  const int threads = busy < 0 ? 512 : 256;  // busy < 0: MFMA companion waves
  hipLaunchKernelGGL(k_probe<V>, dim3(blocks), dim3(threads), 0, 0, d_in, d_bad, d_stale, iters,
                     busy < 0 ? 0 : busy);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  unsigned bad[64], stale[64];
  CHECK(hipMemcpy(bad, d_bad, sizeof bad, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(stale, d_stale, sizeof stale, hipMemcpyDeviceToHost));
  unsigned long long tot = 0, st = 0, grp[4] = {0, 0, 0, 0};
  for (int l = 0; l < 64; ++l) {
    tot += bad[l];
    st += stale[l];
    grp[l / 16] += bad[l];
  }
  printf("{\"variant\": \"%s\", \"busy\": %d, \"blocks\": %d, \"iters\": %d, \"checks\": %llu, "
         "\"mismatches\": %llu, \"stale_input\": %llu, \"by_lane_group\": [%llu, %llu, %llu, %llu]}\n",
         name, busy, blocks, iters, (unsigned long long)blocks * 256ull * iters, tot, st, grp[0],
         grp[1], grp[2], grp[3]);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 4;  // up to 4 workgroups per CU (8 waves per SIMD with companions)
  std::vector<float> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = 0.001f * (float)((i * 7919) % 4001) - 2.0f;
  float* d_in;
  unsigned *d_bad, *d_stale;
  CHECK(hipMalloc(&d_in, 4096 * 4));
  CHECK(hipMalloc(&d_bad, 64 * 4));
  CHECK(hipMalloc(&d_stale, 64 * 4));
  CHECK(hipMemcpy(d_in, h.data(), 4096 * 4, hipMemcpyHostToDevice));
  for (int busy : {-1, 8, 0}) {
    for (int nb : {cus, 2 * cus, blocks}) {
      run<7>("heads sequence: pk_mul, pk_add, pk_add, s_add, ds_write_b128", iters, busy, nb, d_in,
             d_bad, d_stale);
      run<0>("pk_add -> ds_write_b128", iters, busy, nb, d_in, d_bad, d_stale);
      run<1>("pk_add, s_nop 0, ds_write_b128", iters, busy, nb, d_in, d_bad, d_stale);
      run<2>("pk_add, v_mov, ds_write_b128", iters, busy, nb, d_in, d_bad, d_stale);
      run<3>("pk_add, s_nop 1, ds_write_b128", iters, busy, nb, d_in, d_bad, d_stale);
      run<4>("2 x v_add_f32 -> ds_write_b128 (control)", iters, busy, nb, d_in, d_bad, d_stale);
      run<5>("pk_mul -> ds_write_b128", iters, busy, nb, d_in, d_bad, d_stale);
      run<6>("pk_fma -> ds_write_b128", iters, busy, nb, d_in, d_bad, d_stale);
    }
  }
  CHECK(hipFree(d_in));
  CHECK(hipFree(d_bad));
  CHECK(hipFree(d_stale));
  return 0;
}
