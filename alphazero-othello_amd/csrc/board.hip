// board.hip — stateless batched board step / legal-mask / D4 entry points.
//
// oth_step_gpu is the north-star kernel: tens of millions of independent positions in
// SoA (own u64[n], opp u64[n], act u8[n]) -> (own' u64, opp' u64, legal u64, status u16),
// 43 algorithmic bytes per position.  The host entry points run the same bitboard.h
// code so single-position Python calls (OthelloGameNew API) and the device agree bit for
// bit.
#include <stdexcept>
#include <string>

#include "bitboard.h"
#include "common.h"

namespace azc {

static thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

}  // namespace azc

// ------------------------------- device kernels --------------------------------------

namespace {

constexpr int kBlock = 256;
__constant__ const azb::RayTable kRays;
static_assert(kBlock == 64 * 4, "k_step stages one up-ray per thread");

// The board step of one position (the body of both k_step forms): branch-free make-move
// with the capture set from the LDS up-ray table, the next side's legal mask, the
// wave-cooperative terminal check (every lane of the wave must call it: uniform control
// flow) and the status word.
__device__ __forceinline__ void step_one(const uint64_t* rays, const azb::WaveLane& L,
                                         uint64_t o, uint64_t p, int a, bool live,
                                         uint64_t& no, uint64_t& np, uint64_t& lg,
                                         uint16_t& st) {
  const azb::Move mv = azb::move_rays_bf(rays, o, p, a);
  const bool ok = live && !mv.illegal;
  lg = ok ? azb::legal(mv.own, mv.opp) : 0ull;
  int tf = azb::terminal_flags_wave(mv.own, mv.opp, lg, ok);
  tf = azb::finish_terminal_wave(tf, mv.own, mv.opp, L);
  no = mv.own;
  np = mv.opp;
  st = mv.illegal ? azb::pack_status(azb::kFlagIllegal, 0)
                  : azb::pack_status(mv.flags | tf, azb::popc(mv.own) - azb::popc(mv.opp));
}

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// Two consecutive positions per lane per iteration, grid-stride: every global access is a
// lane-contiguous 16-byte (own/opp/legal pairs), 2-byte (act pair) or 4-byte (status pair)
// access, non-temporal (each byte is touched once), 32-bit byte offsets off the uniform
// array bases (n < 2^28: the host checks).  Measured at steady state on 2^24 positions
// (scripts/exp/step_variants.hip v41 vs v33): 0.137 vs 0.145 ms for the one-position,
// 8-byte, write-back form below.  Needs 16-byte aligned own/opp/out arrays, a 2-byte
// aligned act and a 4-byte aligned status array (the host checks); an odd n leaves the
// last position to the lane whose pair is half live.
// Grid cap of k_step2: 256 CUs x 64 blocks, i.e. two grid-stride iterations per lane at
// 2^24 positions.  Same-box A/B (scripts/step_ab.py): 0.1268 ms at 16,384 blocks against
// 0.1319 at 8,192, 0.1277 at 32,768 (one iteration), 0.146 at 2,048 (all resident, 16
// iterations); requesting the next iteration's inputs before the current compute
// (software prefetch) measured no gain at 8,192 and a loss at 16,384 (0.1303).
#ifndef AZ_STEP_GRID_CAP
#define AZ_STEP_GRID_CAP (256 * 64)
#endif

// non-temporal output stores (1, the product); 0 = plain stores (A/B builds)
#ifndef AZ_STEP_NT_ST
#define AZ_STEP_NT_ST 1
#endif

template <class T>
__device__ __forceinline__ void st_out(T v, T* p) {
  if constexpr (AZ_STEP_NT_ST)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// one lane's pair of inputs (a = own, b = opp, c = the two actions)
struct PairIn {
  u64x2 a, b;
  uint32_t c;
};

__device__ __forceinline__ PairIn load_pair(const char* own_b, const char* opp_b,
                                            const uint8_t* act, uint32_t j, uint32_t pairs,
                                            uint32_t full) {
  PairIn in;
  in.a = {0ull, 0ull};
  in.b = {0ull, 0ull};
  in.c = azb::kPass | (azb::kPass << 8);
  const uint32_t o16 = j * 16u;
  if (j < full) {
    in.a = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(own_b + o16));
    in.b = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(opp_b + o16));
    in.c = *reinterpret_cast<const uint16_t*>(act + 2u * j);
  } else if (j < pairs) {  // odd n: the last position alone
    in.a.x = *reinterpret_cast<const uint64_t*>(own_b + o16);
    in.b.x = *reinterpret_cast<const uint64_t*>(opp_b + o16);
    in.c = act[2u * j] | (azb::kPass << 8);
  }
  return in;
}

__global__ __launch_bounds__(kBlock) void k_step2(const uint64_t* __restrict__ own,
                                                  const uint64_t* __restrict__ opp,
                                                  const uint8_t* __restrict__ act,
                                                  uint64_t* __restrict__ own_o,
                                                  uint64_t* __restrict__ opp_o,
                                                  uint64_t* __restrict__ legal_o,
                                                  uint16_t* __restrict__ status_o,
                                                  uint32_t n) {
  __shared__ __align__(16) uint64_t rays[64 * 4];
  rays[threadIdx.x] = kRays.r[threadIdx.x];
  const azb::WaveLane L = azb::wave_lane();
  const uint32_t pairs = (n + 1) / 2, full = n / 2;
  const uint32_t stride = gridDim.x * kBlock;
  const uint32_t p_pad = (pairs + kBlock - 1) / kBlock * kBlock;
  const char* own_b = reinterpret_cast<const char*>(own);
  const char* opp_b = reinterpret_cast<const char*>(opp);
  __syncthreads();
  for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < p_pad; j += stride) {
    const PairIn cur = load_pair(own_b, opp_b, act, j, pairs, full);
    const bool live0 = j < pairs, live1 = j < full;
    uint64_t o0, p0, l0, o1, p1, l1;
    uint16_t s0, s1;
    step_one(rays, L, cur.a.x, cur.b.x, cur.c & 0xFF, live0, o0, p0, l0, s0);
    step_one(rays, L, cur.a.y, cur.b.y, cur.c >> 8, live1, o1, p1, l1, s1);
    const uint32_t o16 = j * 16u;
    char* oo = reinterpret_cast<char*>(own_o) + o16;
    char* po = reinterpret_cast<char*>(opp_o) + o16;
    char* lo = reinterpret_cast<char*>(legal_o) + o16;
    if (live1) {
      const u64x2 vo = {o0, o1}, vp = {p0, p1}, vl = {l0, l1};
      st_out(vo, reinterpret_cast<u64x2*>(oo));
      st_out(vp, reinterpret_cast<u64x2*>(po));
      st_out(vl, reinterpret_cast<u64x2*>(lo));
      st_out((uint32_t)s0 | ((uint32_t)s1 << 16), reinterpret_cast<uint32_t*>(status_o) + j);
    } else if (live0) {
      *reinterpret_cast<uint64_t*>(oo) = o0;
      *reinterpret_cast<uint64_t*>(po) = p0;
      *reinterpret_cast<uint64_t*>(lo) = l0;
      status_o[2u * j] = s0;
    }
  }
}

// The ceiling of k_step2's access pattern: the same grid, the same 16-byte own/opp/out,
// 2-byte act and 4-byte status non-temporal accesses per lane (17 B in, 26 B out per
// position), no board arithmetic -- each output is a one-instruction function of the inputs
// so no load is dead.  A measurement probe only (bench.py's roofline.pattern_ceiling_*):
// how close k_step2 gets to what the box moves for its read/write mix.
__global__ __launch_bounds__(kBlock) void k_step2_io(const uint64_t* __restrict__ own,
                                                     const uint64_t* __restrict__ opp,
                                                     const uint8_t* __restrict__ act,
                                                     uint64_t* __restrict__ own_o,
                                                     uint64_t* __restrict__ opp_o,
                                                     uint64_t* __restrict__ legal_o,
                                                     uint16_t* __restrict__ status_o,
                                                     uint32_t n) {
  const uint32_t pairs = (n + 1) / 2, full = n / 2;
  const uint32_t stride = gridDim.x * kBlock;
  const uint32_t p_pad = (pairs + kBlock - 1) / kBlock * kBlock;
  const char* own_b = reinterpret_cast<const char*>(own);
  const char* opp_b = reinterpret_cast<const char*>(opp);
  for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < p_pad; j += stride) {
    const PairIn cur = load_pair(own_b, opp_b, act, j, pairs, full);
    const uint32_t o16 = j * 16u;
    char* oo = reinterpret_cast<char*>(own_o) + o16;
    char* po = reinterpret_cast<char*>(opp_o) + o16;
    char* lo = reinterpret_cast<char*>(legal_o) + o16;
    if (j < full) {
      st_out(cur.b, reinterpret_cast<u64x2*>(oo));
      st_out(cur.a, reinterpret_cast<u64x2*>(po));
      st_out(cur.a | cur.b, reinterpret_cast<u64x2*>(lo));
      st_out(cur.c, reinterpret_cast<uint32_t*>(status_o) + j);
    } else if (j < pairs) {
      *reinterpret_cast<uint64_t*>(oo) = cur.b.x;
      *reinterpret_cast<uint64_t*>(po) = cur.a.x;
      *reinterpret_cast<uint64_t*>(lo) = cur.a.x | cur.b.x;
      status_o[2u * j] = (uint16_t)cur.c;
    }
  }
}

// One position per lane per iteration (any alignment): lane-contiguous 8-byte
// (own/opp/legal), 1-byte (act) and 2-byte (status) accesses.
__global__ __launch_bounds__(kBlock) void k_step(const uint64_t* __restrict__ own,
                                                 const uint64_t* __restrict__ opp,
                                                 const uint8_t* __restrict__ act,
                                                 uint64_t* __restrict__ own_o,
                                                 uint64_t* __restrict__ opp_o,
                                                 uint64_t* __restrict__ legal_o,
                                                 uint16_t* __restrict__ status_o,
                                                 uint32_t n) {
  __shared__ __align__(16) uint64_t rays[64 * 4];
  rays[threadIdx.x] = kRays.r[threadIdx.x];
  __syncthreads();
  const azb::WaveLane L = azb::wave_lane();
  // every lane runs the same number of iterations (the terminal check is wave-cooperative)
  const uint32_t stride = gridDim.x * kBlock;
  const uint32_t n_pad = (n + kBlock - 1) / kBlock * kBlock;
  const char* own_b = reinterpret_cast<const char*>(own);
  const char* opp_b = reinterpret_cast<const char*>(opp);
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n_pad; i += stride) {
    const bool live = i < n;
    const uint32_t o8 = i * 8u;
    uint64_t o = 0, p = 0;
    int a = azb::kPass;
    if (live) {
      o = *reinterpret_cast<const uint64_t*>(own_b + o8);
      p = *reinterpret_cast<const uint64_t*>(opp_b + o8);
      a = act[i];
    }
    uint64_t no, np, lg;
    uint16_t st;
    step_one(rays, L, o, p, a, live, no, np, lg, st);
    if (live) {
      *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(own_o) + o8) = no;
      *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(opp_o) + o8) = np;
      *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(legal_o) + o8) = lg;
      status_o[i] = st;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_legal(const uint64_t* __restrict__ own,
                                                  const uint64_t* __restrict__ opp,
                                                  uint64_t* __restrict__ legal_o, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    legal_o[i] = azb::legal(own[i], opp[i]);
}

__global__ __launch_bounds__(kBlock) void k_d4(const uint64_t* __restrict__ x,
                                               const uint8_t* __restrict__ sym,
                                               uint64_t* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    out[i] = azb::d4(x[i], sym[i] & 7);
}

// the same up-ray table on the host (built once, immutable afterwards)
const uint64_t* host_rays() {
  static const struct Table {
    uint64_t r[64 * 4];
    Table() {
      for (int i = 0; i < 256; ++i) r[i] = azb::ray_up(i >> 2, i & 3);
    }
  } table;
  return table.r;
}

unsigned grid_for(int64_t n, int64_t cap = 256 * 32) {
  // enough waves to cover the chip many times over (256 CUs x 32 blocks); grid-stride for
  // the rest
  const int64_t blocks = (n + kBlock - 1) / kBlock;
  return (unsigned)(blocks < 1 ? 1 : (blocks > cap ? cap : blocks));
}

}  // namespace

// ------------------------------- C ABI: host ------------------------------------------

extern "C" {

const char* az_last_error(void) { return azc::g_last_error.c_str(); }
int az_abi_version(void) { return AZ_ABI_VERSION; }

#ifndef AZ_BUILD_ID
#error "AZ_BUILD_ID must be defined by the build (az_build.py: sha256 of the sources)"
#endif
// the marker prefix lets az_build.py find the id in the .so without loading it
static const char kBuildIdTag[] = "AZ_BUILD_ID=" AZ_BUILD_ID;
const char* az_build_id(void) { return kBuildIdTag + 12; }

int oth_legal_cpu(const uint64_t* own, const uint64_t* opp, uint64_t* legal_o, int64_t n) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_legal_cpu: n=%lld < 0", (long long)n);
  AZ_REQUIRE(n == 0 || (own && opp && legal_o), AZ_ERR_ARG, "oth_legal_cpu: null buffer");
  for (int64_t i = 0; i < n; ++i) legal_o[i] = azb::legal(own[i], opp[i]);
  return AZ_OK;
}

int oth_step_cpu(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
                 uint64_t* own_o, uint64_t* opp_o, uint64_t* legal_o, uint16_t* status_o,
                 int64_t n) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_step_cpu: n=%lld < 0", (long long)n);
  AZ_REQUIRE(n == 0 || (own && opp && act && own_o && opp_o && legal_o && status_o),
             AZ_ERR_ARG, "oth_step_cpu: null buffer");
  const uint64_t* rays = host_rays();
  int64_t first_bad = -1;
  for (int64_t i = 0; i < n; ++i) {
    const azb::Step s = azb::step_rays(rays, own[i], opp[i], act[i]);
    own_o[i] = s.own;
    opp_o[i] = s.opp;
    legal_o[i] = s.legal;
    status_o[i] = s.status;
    if ((s.status & azb::kFlagIllegal) && first_bad < 0) first_bad = i;
  }
  if (first_bad >= 0)
    return azc::set_error(AZ_ERR_ILLEGAL, "Illegal move: %d (position %lld)",
                          (int)act[first_bad], (long long)first_bad);
  return AZ_OK;
}

int oth_make_move_cpu(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
                      uint64_t* own_o, uint64_t* opp_o, int64_t n) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_make_move_cpu: n < 0");
  AZ_REQUIRE(n == 0 || (own && opp && act && own_o && opp_o), AZ_ERR_ARG,
             "oth_make_move_cpu: null buffer");
  for (int64_t i = 0; i < n; ++i) {
    const int a = act[i];
    AZ_REQUIRE(a <= 64, AZ_ERR_ARG, "oth_make_move_cpu: action %d out of range", a);
    // no legality check, exactly like _BitBoard.make_move: an unbounded placement just
    // adds the stone (captured = 0)
    const uint64_t cap = a == azb::kPass ? 0ull : azb::flips(own[i], opp[i], a);
    azb::play(own[i], opp[i], a, cap, own_o + i, opp_o + i);
  }
  return AZ_OK;
}

int oth_pack_np(const int8_t* states, const int8_t* player, uint64_t* own, uint64_t* opp,
                int64_t n) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_pack_np: n < 0");
  AZ_REQUIRE(n == 0 || (states && player && own && opp), AZ_ERR_ARG,
             "oth_pack_np: null buffer");
  for (int64_t i = 0; i < n; ++i) {
    const int8_t* s = states + 64 * i;
    const int p = player[i];
    uint64_t a = 0, b = 0;
    for (int k = 0; k < 64; ++k) {
      a |= (uint64_t)(s[k] == p) << k;
      b |= (uint64_t)(s[k] == -p) << k;
    }
    own[i] = a;
    opp[i] = b;
  }
  return AZ_OK;
}

int oth_unpack_np(const uint64_t* own, const uint64_t* opp, const int8_t* player,
                  int8_t* states, int64_t n) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_unpack_np: n < 0");
  AZ_REQUIRE(n == 0 || (own && opp && player && states), AZ_ERR_ARG,
             "oth_unpack_np: null buffer");
  for (int64_t i = 0; i < n; ++i) {
    int8_t* s = states + 64 * i;
    const int8_t p = player[i];
    for (int k = 0; k < 64; ++k) {
      const int8_t v = (int8_t)(((own[i] >> k) & 1) ? p : (((opp[i] >> k) & 1) ? -p : 0));
      s[k] = v;
    }
  }
  return AZ_OK;
}

int oth_d4_cpu(const uint64_t* x, const uint8_t* sym, uint64_t* out, int64_t n) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_d4_cpu: n < 0");
  AZ_REQUIRE(n == 0 || (x && sym && out), AZ_ERR_ARG, "oth_d4_cpu: null buffer");
  for (int64_t i = 0; i < n; ++i) out[i] = azb::d4(x[i], sym[i] & 7);
  return AZ_OK;
}

// ------------------------------- C ABI: device ----------------------------------------

int oth_legal_gpu(const uint64_t* own, const uint64_t* opp, uint64_t* legal_o, int64_t n,
                  void* stream) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_legal_gpu: n < 0");
  if (n == 0) return AZ_OK;
  AZ_REQUIRE(own && opp && legal_o, AZ_ERR_ARG, "oth_legal_gpu: null buffer");
  hipLaunchKernelGGL(k_legal, dim3(grid_for(n)), dim3(kBlock), 0, azc::as_stream(stream),
                     own, opp, legal_o, n);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

int oth_step_gpu(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
                 uint64_t* own_o, uint64_t* opp_o, uint64_t* legal_o, uint16_t* status_o,
                 int64_t n, void* stream) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_step_gpu: n < 0");
  if (n == 0) return AZ_OK;
  AZ_REQUIRE(own && opp && act && own_o && opp_o && legal_o && status_o, AZ_ERR_ARG,
             "oth_step_gpu: null buffer");
  AZ_REQUIRE(n < (int64_t(1) << 28), AZ_ERR_ARG,
             "oth_step_gpu: n=%lld exceeds 2^28 positions per call", (long long)n);
  const auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15u) == 0; };
  const bool paired = a16(own) && a16(opp) && a16(own_o) && a16(opp_o) && a16(legal_o) &&
                      (reinterpret_cast<uintptr_t>(act) & 1u) == 0 &&
                      (reinterpret_cast<uintptr_t>(status_o) & 3u) == 0;
  if (paired)
    hipLaunchKernelGGL(k_step2, dim3(grid_for((n + 1) / 2, AZ_STEP_GRID_CAP)), dim3(kBlock), 0,
                       azc::as_stream(stream), own, opp, act, own_o, opp_o, legal_o, status_o,
                       (uint32_t)n);
  else
    hipLaunchKernelGGL(k_step, dim3(grid_for(n)), dim3(kBlock), 0, azc::as_stream(stream),
                       own, opp, act, own_o, opp_o, legal_o, status_o, (uint32_t)n);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

int oth_step_io_gpu(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
                    uint64_t* own_o, uint64_t* opp_o, uint64_t* legal_o, uint16_t* status_o,
                    int64_t n, void* stream) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_step_io_gpu: n < 0");
  if (n == 0) return AZ_OK;
  AZ_REQUIRE(own && opp && act && own_o && opp_o && legal_o && status_o, AZ_ERR_ARG,
             "oth_step_io_gpu: null buffer");
  AZ_REQUIRE(n < (int64_t(1) << 28), AZ_ERR_ARG, "oth_step_io_gpu: n exceeds 2^28");
  const auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15u) == 0; };
  AZ_REQUIRE(a16(own) && a16(opp) && a16(own_o) && a16(opp_o) && a16(legal_o) &&
                 (reinterpret_cast<uintptr_t>(act) & 1u) == 0 &&
                 (reinterpret_cast<uintptr_t>(status_o) & 3u) == 0,
             AZ_ERR_ARG, "oth_step_io_gpu: needs k_step2's alignment");
  hipLaunchKernelGGL(k_step2_io, dim3(grid_for((n + 1) / 2, AZ_STEP_GRID_CAP)), dim3(kBlock), 0,
                     azc::as_stream(stream), own, opp, act, own_o, opp_o, legal_o, status_o,
                     (uint32_t)n);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

int oth_d4_gpu(const uint64_t* x, const uint8_t* sym, uint64_t* out, int64_t n,
               void* stream) {
  AZ_REQUIRE(n >= 0, AZ_ERR_ARG, "oth_d4_gpu: n < 0");
  if (n == 0) return AZ_OK;
  AZ_REQUIRE(x && sym && out, AZ_ERR_ARG, "oth_d4_gpu: null buffer");
  hipLaunchKernelGGL(k_d4, dim3(grid_for(n)), dim3(kBlock), 0, azc::as_stream(stream), x,
                     sym, out, n);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

}  // extern "C"
