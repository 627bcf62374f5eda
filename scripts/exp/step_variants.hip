// Experiment harness (not product code): variants of the batched board-step kernel, to find
// what bounds k_step on gfx950.  Built on the GPU box by scripts/exp/run_step_variants.py.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../alphazero-othello_amd/csrc/bitboard.h"

namespace x {
using namespace azb;

__device__ __forceinline__ uint64_t mk(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
template <int K> __device__ __forceinline__ uint64_t shl(uint64_t v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  return mk(lo << K, __builtin_amdgcn_alignbit(hi, lo, 32 - K));
}
template <int K> __device__ __forceinline__ uint64_t shr(uint64_t v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  return mk(__builtin_amdgcn_alignbit(hi, lo, K), hi >> K);
}
template <int D> __device__ __forceinline__ uint64_t moves_dir32(uint64_t P, uint64_t M) {
  uint64_t fl = M & shl<D>(P);
  uint64_t fr = M & shr<D>(P);
  fl |= M & shl<D>(fl);
  fr |= M & shr<D>(fr);
  const uint64_t ml = M & shl<D>(M);
  const uint64_t mr = shr<D>(ml);
  fl |= ml & shl<2 * D>(fl);
  fr |= mr & shr<2 * D>(fr);
  fl |= ml & shl<2 * D>(fl);
  fr |= mr & shr<2 * D>(fr);
  return shl<D>(fl) | shr<D>(fr);
}
__device__ __forceinline__ uint64_t legal32(uint64_t own, uint64_t opp) {
  const uint64_t inner = opp & kInner;
  uint64_t m = moves_dir32<1>(own, inner);
  m |= moves_dir32<8>(own, opp);
  m |= moves_dir32<7>(own, inner);
  m |= moves_dir32<9>(own, inner);
  return m & ~(own | opp);
}
__device__ __forceinline__ Step step32(uint64_t own, uint64_t opp, int act) {
  Step o;
  int flags = 0;
  if (act == kPass) { o.own = opp; o.opp = own; flags = kFlagPassed; }
  else {
    const bool in_range = (unsigned)act < 64u;
    const int sq = act & 63;
    const uint64_t nb = 1ull << sq;
    const uint64_t cap = in_range ? flips(own, opp, sq) : 0ull;
    if (!in_range || cap == 0ull || (nb & (own | opp))) {
      o.own = own; o.opp = opp; o.legal = 0; o.status = pack_status(kFlagIllegal, 0); return o;
    }
    o.own = opp ^ cap; o.opp = (own | nb) ^ cap;
  }
  o.legal = legal32(o.own, o.opp);
  if (!o.legal) flags |= legal32(o.opp, o.own) ? kFlagNoPlace : (kFlagNoPlace | kFlagTerminal);
  o.status = pack_status(flags, popc(o.own) - popc(o.opp));
  return o;
}
}  // namespace x

#define GS for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)

__global__ __launch_bounds__(256) void v0(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  GS { azb::Step s = azb::step(own[i], opp[i], act[i]); oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status; }
}
__global__ __launch_bounds__(256) void v1(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  GS { uint64_t a = own[i], b = opp[i]; int c = act[i]; oo[i] = a ^ c; po[i] = b; lo[i] = a | b; so[i] = (uint16_t)c; }
}
__global__ __launch_bounds__(256) void v2(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  GS { azb::Step s = x::step32(own[i], opp[i], act[i]); oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status; }
}
// two positions per lane, 16-byte I/O
__global__ __launch_bounds__(256) void v3(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const int64_t n2 = n / 2;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n2; j += (int64_t)gridDim.x * 256) {
    const ulonglong2 a = reinterpret_cast<const ulonglong2*>(own)[j];
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(opp)[j];
    const uint16_t c = reinterpret_cast<const uint16_t*>(act)[j];
    azb::Step s0 = x::step32(a.x, b.x, c & 0xFF), s1 = x::step32(a.y, b.y, c >> 8);
    reinterpret_cast<ulonglong2*>(oo)[j] = make_ulonglong2(s0.own, s1.own);
    reinterpret_cast<ulonglong2*>(po)[j] = make_ulonglong2(s0.opp, s1.opp);
    reinterpret_cast<ulonglong2*>(lo)[j] = make_ulonglong2(s0.legal, s1.legal);
    reinterpret_cast<uint32_t*>(so)[j] = (uint32_t)s0.status | ((uint32_t)s1.status << 16);
  }
}
// I/O only, 2 per lane
__global__ __launch_bounds__(256) void v4(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const int64_t n2 = n / 2;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n2; j += (int64_t)gridDim.x * 256) {
    const ulonglong2 a = reinterpret_cast<const ulonglong2*>(own)[j];
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(opp)[j];
    const uint16_t c = reinterpret_cast<const uint16_t*>(act)[j];
    reinterpret_cast<ulonglong2*>(oo)[j] = make_ulonglong2(a.x ^ c, a.y);
    reinterpret_cast<ulonglong2*>(po)[j] = b;
    reinterpret_cast<ulonglong2*>(lo)[j] = make_ulonglong2(a.x | b.x, a.y | b.y);
    reinterpret_cast<uint32_t*>(so)[j] = c;
  }
}
// legal only (no flips): compute cost of the legal mask alone, 64-bit shifts vs 32-bit
__global__ __launch_bounds__(256) void v5(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  GS { lo[i] = azb::legal(own[i], opp[i]); }
}
__global__ __launch_bounds__(256) void v6(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  GS { lo[i] = x::legal32(own[i], opp[i]); }
}

// software-pipelined grid-stride: next iteration's inputs are loaded before this one's compute
__global__ __launch_bounds__(256) void v7(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t a = own[i], b = opp[i]; int c = act[i];
  for (; i < n; i += stride) {
    const int64_t j = i + stride;
    uint64_t a2 = 0, b2 = 0; int c2 = 0;
    if (j < n) { a2 = own[j]; b2 = opp[j]; c2 = act[j]; }
    azb::Step s = azb::step(a, b, c);
    oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status;
    a = a2; b = b2; c = c2;
  }
}
// compute only: inputs synthesised from the index (a corpus-like mix is not needed for an
// op count), one store per lane at the end
__global__ __launch_bounds__(256) void v8(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t base_o = own[t & 32767], base_p = opp[t & 32767];
  const int base_a = act[t & 32767];
  uint64_t acc = 0;
  for (int64_t i = t; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t r = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    azb::Step s = azb::step(base_o ^ (r & 0), base_p ^ (r & 0), (base_a + (int)(i >> 20)) & 63);
    acc ^= s.own ^ s.opp ^ s.legal ^ s.status;
  }
  lo[t] = acc;
}
// one position per lane, no grid-stride loop
__global__ __launch_bounds__(256) void v9(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) { azb::Step s = azb::step(own[i], opp[i], act[i]); oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status; }
}

// --- v10: no terminal check; v11: cooperative terminal check; v12: make-move only
namespace y {
using namespace azb;
__device__ __forceinline__ void step_core(uint64_t own, uint64_t opp, int act, uint64_t& no, uint64_t& np,
                                          int& flags, bool& illegal) {
  flags = 0; illegal = false;
  if (act == kPass) { no = opp; np = own; flags = kFlagPassed; return; }
  const bool in_range = (unsigned)act < 64u;
  const int sq = act & 63;
  const uint64_t nb = 1ull << sq;
  const uint64_t cap = in_range ? flips(own, opp, sq) : 0ull;
  if (!in_range || cap == 0ull || (nb & (own | opp))) { no = own; np = opp; illegal = true; return; }
  no = opp ^ cap; np = (own | nb) ^ cap;
}
// one direction of the legal-move fill (dumb7 with doubling), direction d in 0..7
__device__ __forceinline__ uint64_t dir_moves(uint64_t P, uint64_t O, int d) {
  const uint64_t empty = ~(P | O);
  const uint64_t inner = O & kInner;
  uint64_t M, f, mm;
  int s; bool left;
  switch (d & 3) { case 0: s = 1; M = inner; break; case 1: s = 8; M = O; break;
                   case 2: s = 7; M = inner; break; default: s = 9; M = inner; break; }
  left = d >= 4;
  if (left) {
    f = M & (P << s); f |= M & (f << s); mm = M & (M << s);
    f |= mm & (f << (2 * s)); f |= mm & (f << (2 * s));
    return (f << s) & empty;
  } else {
    f = M & (P >> s); f |= M & (f >> s); mm = M & (M >> s);
    f |= mm & (f >> (2 * s)); f |= mm & (f >> (2 * s));
    return (f >> s) & empty;
  }
}
}  // namespace y

__global__ __launch_bounds__(256) void v10(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  GS {
    uint64_t no, np; int flags; bool ill;
    y::step_core(own[i], opp[i], act[i], no, np, flags, ill);
    uint64_t lg = ill ? 0 : azb::legal(no, np);
    oo[i] = no; po[i] = np; lo[i] = lg;
    so[i] = azb::pack_status(ill ? azb::kFlagIllegal : flags | (lg ? 0 : azb::kFlagNoPlace), ill ? 0 : azb::popc(no) - azb::popc(np));
  }
}
__global__ __launch_bounds__(256) void v11(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t n_pad = (n + 255) / 256 * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pad; i += stride) {
    const bool live = i < n;
    uint64_t no = 0, np = 0; int flags = 0; bool ill = true;
    if (live) y::step_core(own[i], opp[i], act[i], no, np, flags, ill);
    const uint64_t lg = ill ? 0 : azb::legal(no, np);
    // terminal check for the rare lanes with no placement: 8 lanes per position, one
    // direction each (opp' moving against own'), up to 8 positions per pass
    uint64_t need = __ballot(!ill && lg == 0);
    bool other = false;
    while (need) {
      // j-th needed lane for group j = lane / 8
      const int grp = lane >> 3;
      uint64_t mm = need; for (int j = 0; j < grp && mm; ++j) mm &= mm - 1;
      const int src = mm ? __builtin_ctzll(mm) : -1;
      const uint64_t P = __shfl(np, src < 0 ? 0 : src, 64), O = __shfl(no, src < 0 ? 0 : src, 64);
      const uint64_t mv = src < 0 ? 0 : y::dir_moves(P, O, lane & 7);
      const uint64_t got = __ballot(mv != 0);
      // owner lanes read their group's byte
      uint64_t mm2 = need; int k = 0;
      for (; k < 8 && mm2; ++k) { const int l = __builtin_ctzll(mm2); if (l == lane) other = ((got >> (8 * k)) & 0xFF) != 0; mm2 &= mm2 - 1; }
      // drop the processed lanes (the first 8 set bits)
      for (int j = 0; j < 8 && need; ++j) need &= need - 1;
    }
    if (live) {
      if (!ill && lg == 0) flags |= other ? azb::kFlagNoPlace : (azb::kFlagNoPlace | azb::kFlagTerminal);
      oo[i] = no; po[i] = np; lo[i] = lg;
      so[i] = ill ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(flags, azb::popc(no) - azb::popc(np));
    }
  }
}
__global__ __launch_bounds__(256) void v12(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  GS {
    uint64_t no, np; int flags; bool ill;
    y::step_core(own[i], opp[i], act[i], no, np, flags, ill);
    oo[i] = no; po[i] = np; lo[i] = no | np; so[i] = azb::pack_status(flags, azb::popc(no) - azb::popc(np));
  }
}

// v13: product step, two positions per lane (16-byte own/opp/legal I/O)
__global__ __launch_bounds__(256) void v13(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const int64_t n2 = n / 2;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n2; j += (int64_t)gridDim.x * 256) {
    const ulonglong2 a = reinterpret_cast<const ulonglong2*>(own)[j];
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(opp)[j];
    const uint16_t c = reinterpret_cast<const uint16_t*>(act)[j];
    azb::Step s0 = azb::step(a.x, b.x, c & 0xFF), s1 = azb::step(a.y, b.y, c >> 8);
    reinterpret_cast<ulonglong2*>(oo)[j] = make_ulonglong2(s0.own, s1.own);
    reinterpret_cast<ulonglong2*>(po)[j] = make_ulonglong2(s0.opp, s1.opp);
    reinterpret_cast<ulonglong2*>(lo)[j] = make_ulonglong2(s0.legal, s1.legal);
    reinterpret_cast<uint32_t*>(so)[j] = (uint32_t)s0.status | ((uint32_t)s1.status << 16);
  }
}
// v14: product step, block 64 / v15: block 512 (same body as v0)
__global__ __launch_bounds__(64) void v14(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 64) {
    azb::Step s = azb::step(own[i], opp[i], act[i]); oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status; }
}
// v16: four positions per lane, loads for all four issued before any compute
__global__ __launch_bounds__(256) void v16(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const int64_t q = n / 4;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < q; j += stride) {
    uint64_t a[4], b[4]; int c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { const int64_t i = j + k * q; a[k] = own[i]; b[k] = opp[i]; c[k] = act[i]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = j + k * q;
      azb::Step s = azb::step(a[k], b[k], c[k]); oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status;
    }
  }
}


// ---- r01b: ray-table capture set + bop3/carry legal (the product formulation) ----------
#define RAYS __shared__ __align__(16) uint64_t rays[256]; if (threadIdx.x < 256) rays[threadIdx.x] = azb::ray_up(threadIdx.x >> 2, threadIdx.x & 3); __syncthreads();
// v17: plain per-lane step_rays (divergent terminal fill), grid-stride
__global__ __launch_bounds__(256) void v17(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  GS { azb::Step s = azb::step_rays(rays, own[i], opp[i], act[i]); oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status; }
}
// v18: two positions per lane (i and i + n/2), loads of both issued first
__global__ __launch_bounds__(256) void v18(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  const int64_t h = n / 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < h; i += (int64_t)gridDim.x * 256) {
    const uint64_t a0 = own[i], b0 = opp[i], a1 = own[i + h], b1 = opp[i + h];
    const int c0 = act[i], c1 = act[i + h];
    azb::Step s0 = azb::step_rays(rays, a0, b0, c0), s1 = azb::step_rays(rays, a1, b1, c1);
    oo[i] = s0.own; po[i] = s0.opp; lo[i] = s0.legal; so[i] = s0.status;
    oo[i + h] = s1.own; po[i + h] = s1.opp; lo[i + h] = s1.legal; so[i + h] = s1.status;
  }
}
// v19: compute only (one store per lane at the end)
__global__ __launch_bounds__(256) void v19(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t base_o = own[t & 32767], base_p = opp[t & 32767];
  const int base_a = act[t & 32767];
  uint64_t acc = 0;
  for (int64_t i = t; i < n; i += (int64_t)gridDim.x * 256) {
    azb::Step s = azb::step_rays(rays, base_o ^ acc, base_p, (base_a + (int)(i >> 20)) & 63);
    acc ^= (s.own ^ s.opp ^ s.legal ^ s.status) & 1;
  }
  lo[t] = acc;
}
// v20: legal only, new formulation
__global__ __launch_bounds__(256) void v20(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  GS { lo[i] = azb::legal(own[i], opp[i]); }
}
// v21: product step with non-temporal stores
__global__ __launch_bounds__(256) void v21(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  GS { azb::Step s = azb::step_rays(rays, own[i], opp[i], act[i]);
    __builtin_nontemporal_store(s.own, oo + i); __builtin_nontemporal_store(s.opp, po + i);
    __builtin_nontemporal_store(s.legal, lo + i); __builtin_nontemporal_store(s.status, so + i); }
}

// v22: v17 + next iteration's inputs prefetched into registers before this one's compute
__global__ __launch_bounds__(256) void v22(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t a = 0, b = 0; int c = 0;
  if (i < n) { a = own[i]; b = opp[i]; c = act[i]; }
  for (; i < n; i += stride) {
    const int64_t j = i + stride;
    uint64_t a2 = 0, b2 = 0; int c2 = 0;
    if (j < n) { a2 = __builtin_nontemporal_load(own + j); b2 = __builtin_nontemporal_load(opp + j); c2 = __builtin_nontemporal_load(act + j); }
    azb::Step s = azb::step_rays(rays, a, b, c);
    oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status;
    a = a2; b = b2; c = c2;
  }
}
// v23: prefetch distance 2
__global__ __launch_bounds__(256) void v23(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t a = 0, b = 0, a1 = 0, b1 = 0; int c = 0, c1 = 0;
  if (i < n) { a = own[i]; b = opp[i]; c = act[i]; }
  if (i + stride < n) { a1 = own[i + stride]; b1 = opp[i + stride]; c1 = act[i + stride]; }
  for (; i < n; i += stride) {
    const int64_t j = i + 2 * stride;
    uint64_t a2 = 0, b2 = 0; int c2 = 0;
    if (j < n) { a2 = own[j]; b2 = opp[j]; c2 = act[j]; }
    azb::Step s = azb::step_rays(rays, a, b, c);
    oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status;
    a = a1; b = b1; c = c1; a1 = a2; b1 = b2; c1 = c2;
  }
}
// v24: v22 with plain loads
__global__ __launch_bounds__(256) void v24(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t a = 0, b = 0; int c = 0;
  if (i < n) { a = own[i]; b = opp[i]; c = act[i]; }
  for (; i < n; i += stride) {
    const int64_t j = i + stride;
    uint64_t a2 = 0, b2 = 0; int c2 = 0;
    if (j < n) { a2 = own[j]; b2 = opp[j]; c2 = act[j]; }
    azb::Step s = azb::step_rays(rays, a, b, c);
    oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status;
    a = a2; b = b2; c = c2;
  }
}
// v25: one block-tile of 1024 positions per iteration (4 per lane, strided by 256), loads of
// the whole tile issued before any compute
__global__ __launch_bounds__(256) void v25(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  const int64_t tiles = n / 1024;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t base = t * 1024 + threadIdx.x;
    uint64_t a[4], b[4]; int c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { a[k] = own[base + 256 * k]; b[k] = opp[base + 256 * k]; c[k] = act[base + 256 * k]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      azb::Step s = azb::step_rays(rays, a[k], b[k], c[k]);
      const int64_t i = base + 256 * k;
      oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status;
    }
  }
}

// v26: four consecutive positions per lane: 16-byte own/opp/out accesses, 4-byte act, 8-byte status
__global__ __launch_bounds__(256) void v26(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  const int64_t q = n / 4;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < q; j += (int64_t)gridDim.x * 256) {
    const ulonglong2 a0 = reinterpret_cast<const ulonglong2*>(own)[2 * j], a1 = reinterpret_cast<const ulonglong2*>(own)[2 * j + 1];
    const ulonglong2 b0 = reinterpret_cast<const ulonglong2*>(opp)[2 * j], b1 = reinterpret_cast<const ulonglong2*>(opp)[2 * j + 1];
    const uint32_t c = reinterpret_cast<const uint32_t*>(act)[j];
    azb::Step s0 = azb::step_rays(rays, a0.x, b0.x, c & 0xFF), s1 = azb::step_rays(rays, a0.y, b0.y, (c >> 8) & 0xFF);
    azb::Step s2 = azb::step_rays(rays, a1.x, b1.x, (c >> 16) & 0xFF), s3 = azb::step_rays(rays, a1.y, b1.y, c >> 24);
    reinterpret_cast<ulonglong2*>(oo)[2 * j] = make_ulonglong2(s0.own, s1.own); reinterpret_cast<ulonglong2*>(oo)[2 * j + 1] = make_ulonglong2(s2.own, s3.own);
    reinterpret_cast<ulonglong2*>(po)[2 * j] = make_ulonglong2(s0.opp, s1.opp); reinterpret_cast<ulonglong2*>(po)[2 * j + 1] = make_ulonglong2(s2.opp, s3.opp);
    reinterpret_cast<ulonglong2*>(lo)[2 * j] = make_ulonglong2(s0.legal, s1.legal); reinterpret_cast<ulonglong2*>(lo)[2 * j + 1] = make_ulonglong2(s2.legal, s3.legal);
    reinterpret_cast<uint2*>(so)[j] = make_uint2((uint32_t)s0.status | ((uint32_t)s1.status << 16), (uint32_t)s2.status | ((uint32_t)s3.status << 16));
  }
}
// v27: I/O only in v26's pattern
__global__ __launch_bounds__(256) void v27(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const int64_t q = n / 4;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < q; j += (int64_t)gridDim.x * 256) {
    const ulonglong2 a0 = reinterpret_cast<const ulonglong2*>(own)[2 * j], a1 = reinterpret_cast<const ulonglong2*>(own)[2 * j + 1];
    const ulonglong2 b0 = reinterpret_cast<const ulonglong2*>(opp)[2 * j], b1 = reinterpret_cast<const ulonglong2*>(opp)[2 * j + 1];
    const uint32_t c = reinterpret_cast<const uint32_t*>(act)[j];
    reinterpret_cast<ulonglong2*>(oo)[2 * j] = make_ulonglong2(a0.x ^ c, a0.y); reinterpret_cast<ulonglong2*>(oo)[2 * j + 1] = a1;
    reinterpret_cast<ulonglong2*>(po)[2 * j] = b0; reinterpret_cast<ulonglong2*>(po)[2 * j + 1] = b1;
    reinterpret_cast<ulonglong2*>(lo)[2 * j] = make_ulonglong2(a0.x | b0.x, a0.y | b0.y); reinterpret_cast<ulonglong2*>(lo)[2 * j + 1] = make_ulonglong2(a1.x | b1.x, a1.y | b1.y);
    reinterpret_cast<uint2*>(so)[j] = make_uint2(c, c >> 3);
  }
}
// v28: I/O only, one position per lane, nontemporal stores
__global__ __launch_bounds__(256) void v28(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  GS { uint64_t a = own[i], b = opp[i]; int c = act[i];
    __builtin_nontemporal_store(a ^ c, oo + i); __builtin_nontemporal_store(b, po + i);
    __builtin_nontemporal_store(a | b, lo + i); __builtin_nontemporal_store((uint16_t)c, so + i); }
}

// v29 / v30: v17 / v19 with clock stamps (block 0, lane 0): s_memtime (shader clock) and
// s_memrealtime (100 MHz) at start and end, written to oo[n-4 .. n-1] after the work
__global__ __launch_bounds__(256) void v29(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  RAYS
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n - 4; i += (int64_t)gridDim.x * 256) {
    azb::Step s = azb::step_rays(rays, own[i], opp[i], act[i]); oo[i] = s.own; po[i] = s.opp; lo[i] = s.legal; so[i] = s.status; }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) { lo[n - 4] = t0; lo[n - 3] = t1; lo[n - 2] = r0; lo[n - 1] = r1; }
}
__global__ __launch_bounds__(256) void v30(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  RAYS
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t base_o = own[t & 32767], base_p = opp[t & 32767];
  const int base_a = act[t & 32767];
  uint64_t acc = 0;
  for (int64_t i = t; i < n; i += (int64_t)gridDim.x * 256) {
    azb::Step s = azb::step_rays(rays, base_o ^ acc, base_p, (base_a + (int)(i >> 20)) & 63);
    acc ^= (s.own ^ s.opp ^ s.legal ^ s.status) & 1;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t < n - 4) lo[t] = acc;
  if (blockIdx.x == 0 && threadIdx.x == 0) { lo[n - 4] = t0; lo[n - 3] = t1; lo[n - 2] = r0; lo[n - 1] = r1; }
}
// v31: I/O only (v1) with stamps
__global__ __launch_bounds__(256) void v31(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n - 4; i += (int64_t)gridDim.x * 256) {
    uint64_t a = own[i], b = opp[i]; int c = act[i]; oo[i] = a ^ c; po[i] = b; lo[i] = a | b; so[i] = (uint16_t)c; }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) { lo[n - 4] = t0; lo[n - 3] = t1; lo[n - 2] = r0; lo[n - 1] = r1; }
}

// v32: the product k_step body (cooperative terminal check) — A/B reference for v33/v34
__global__ __launch_bounds__(256) void v32(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t n_pad = (n + 255) / 256 * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pad; i += stride) {
    const bool live = i < n;
    uint64_t o = 0, p = 0; int a = azb::kPass;
    if (live) { o = own[i]; p = opp[i]; a = act[i]; }
    const azb::Move mv = azb::move_rays(rays, o, p, a);
    const bool ok = live && !mv.illegal;
    const uint64_t lg = ok ? azb::legal(mv.own, mv.opp) : 0ull;
    int tf = azb::terminal_flags_wave(mv.own, mv.opp, lg, ok);
    tf = azb::finish_terminal_wave(tf, mv.own, mv.opp);
    if (live) {
      oo[i] = mv.own; po[i] = mv.opp; lo[i] = lg;
      so[i] = mv.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(mv.flags | tf, azb::popc(mv.own) - azb::popc(mv.opp));
    }
  }
}
// v33: branch-free move + 32-bit byte offsets (saddr loads/stores)
template <bool BF>
__device__ __forceinline__ void step33(const uint64_t* rays, const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, uint32_t n) {
  const uint32_t stride = gridDim.x * 256;
  const uint32_t n_pad = (n + 255) / 256 * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n_pad; i += stride) {
    const bool live = i < n;
    const uint32_t o8 = i * 8u;
    uint64_t o = 0, p = 0; int a = azb::kPass;
    if (live) {
      o = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(own) + o8);
      p = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(opp) + o8);
      a = act[i];
    }
    const azb::Move mv = BF ? azb::move_rays_bf(rays, o, p, a) : azb::move_rays(rays, o, p, a);
    const bool ok = live && !mv.illegal;
    const uint64_t lg = ok ? azb::legal(mv.own, mv.opp) : 0ull;
    int tf = azb::terminal_flags_wave(mv.own, mv.opp, lg, ok);
    tf = azb::finish_terminal_wave(tf, mv.own, mv.opp);
    if (live) {
      *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(oo) + o8) = mv.own;
      *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(po) + o8) = mv.opp;
      *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(lo) + o8) = lg;
      *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(so) + i * 2u) = mv.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(mv.flags | tf, azb::popc(mv.own) - azb::popc(mv.opp));
    }
  }
}
__global__ __launch_bounds__(256) void v33(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  step33<true>(rays, own, opp, act, oo, po, lo, so, (uint32_t)n);
}
// v34: 32-bit offsets only
__global__ __launch_bounds__(256) void v34(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  step33<false>(rays, own, opp, act, oo, po, lo, so, (uint32_t)n);
}

// v35: v33 with the per-ray validity as a sign mask: xo = x & own is 0 or one bit, so the
// top bit of -xo is (xo != 0); its arithmetic-shifted high word masks R & d in one bitop3
// per half (no compare / select pair per ray)
__device__ __forceinline__ uint64_t ray_flips_s(uint64_t R, uint64_t own, uint64_t nopp) {
  using namespace azb::tt;
  const uint64_t o = R & nopp;
  const uint64_t d = o - 1ull;
  const uint64_t xo = azb::bop3<A & ~B & C>(o, d, own);
  const uint32_t m = xo != 0ull ? 0xFFFFFFFFu : 0u;
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)R, (uint32_t)d, m, A & B & C);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(R >> 32), (uint32_t)(d >> 32), m, A & B & C);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ azb::Move move35(const uint64_t* rays, uint64_t own, uint64_t opp, int act) {
  const int sq = act & 63;
  const uint64_t nb = 1ull << sq;
  const uint64_t* up = rays + 4 * sq;
  const uint64_t* upr = rays + 4 * (63 - sq);
  const uint64_t nopp = ~opp, ownr = azb::rev64(own), noppr = azb::rev64(nopp);
  const uint64_t fu = ray_flips_s(up[0], own, nopp) | ray_flips_s(up[1], own, nopp) |
                      ray_flips_s(up[2], own, nopp) | ray_flips_s(up[3], own, nopp);
  const uint64_t fd = ray_flips_s(upr[0], ownr, noppr) | ray_flips_s(upr[1], ownr, noppr) |
                      ray_flips_s(upr[2], ownr, noppr) | ray_flips_s(upr[3], ownr, noppr);
  const uint64_t cap = fu | azb::rev64(fd);
  const bool place = (unsigned)act < 64u && cap != 0ull && !(nb & (own | opp));
  const bool pass = act == azb::kPass;
  const uint64_t c = place ? cap : 0ull, b = place ? nb : 0ull;
  azb::Move m;
  m.illegal = !(place || pass);
  m.flags = pass ? azb::kFlagPassed : 0;
  m.own = m.illegal ? own : opp ^ c;
  m.opp = m.illegal ? opp : azb::bop3<azb::tt::A ^ azb::tt::B ^ azb::tt::C>(own, b, c);
  return m;
}
__global__ __launch_bounds__(256) void v35(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  RAYS
  const uint32_t n = (uint32_t)n_;
  const uint32_t stride = gridDim.x * 256;
  const uint32_t n_pad = (n + 255) / 256 * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n_pad; i += stride) {
    const bool live = i < n;
    const uint32_t o8 = i * 8u;
    uint64_t o = 0, p = 0; int a = azb::kPass;
    if (live) {
      o = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(own) + o8);
      p = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(opp) + o8);
      a = act[i];
    }
    const azb::Move mv = move35(rays, o, p, a);
    const bool ok = live && !mv.illegal;
    const uint64_t lg = ok ? azb::legal(mv.own, mv.opp) : 0ull;
    int tf = azb::terminal_flags_wave(mv.own, mv.opp, lg, ok);
    tf = azb::finish_terminal_wave(tf, mv.own, mv.opp);
    if (live) {
      *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(oo) + o8) = mv.own;
      *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(po) + o8) = mv.opp;
      *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(lo) + o8) = lg;
      *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(so) + i * 2u) = mv.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(mv.flags | tf, azb::popc(mv.own) - azb::popc(mv.opp));
    }
  }
}

// v36: the product body (branch-free move, cooperative terminal check), two consecutive
// positions per lane: 16-byte own/opp/out accesses, 2-byte act, 4-byte status
__device__ __forceinline__ void body36(const uint64_t* rays, uint64_t o, uint64_t p, int a, bool live,
                                       uint64_t& no, uint64_t& np, uint64_t& lg, uint16_t& st) {
  const azb::Move mv = azb::move_rays_bf(rays, o, p, a);
  const bool ok = live && !mv.illegal;
  lg = ok ? azb::legal(mv.own, mv.opp) : 0ull;
  int tf = azb::terminal_flags_wave(mv.own, mv.opp, lg, ok);
  tf = azb::finish_terminal_wave(tf, mv.own, mv.opp);
  no = mv.own; np = mv.opp;
  st = mv.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(mv.flags | tf, azb::popc(mv.own) - azb::popc(mv.opp));
}
__global__ __launch_bounds__(256) void v36(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  RAYS
  const uint32_t n2 = (uint32_t)(n_ / 2);
  const uint32_t stride = gridDim.x * 256;
  const uint32_t n_pad = (n2 + 255) / 256 * 256;
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n_pad; j += stride) {
    const bool live = j < n2;
    ulonglong2 a = make_ulonglong2(0, 0), b = make_ulonglong2(0, 0);
    uint32_t c = 0x4040;
    if (live) {
      a = *reinterpret_cast<const ulonglong2*>(reinterpret_cast<const char*>(own) + j * 16u);
      b = *reinterpret_cast<const ulonglong2*>(reinterpret_cast<const char*>(opp) + j * 16u);
      c = *reinterpret_cast<const uint16_t*>(act + j * 2u);
    }
    uint64_t o0, p0, l0, o1, p1, l1; uint16_t s0, s1;
    body36(rays, a.x, b.x, c & 0xFF, live, o0, p0, l0, s0);
    body36(rays, a.y, b.y, c >> 8, live, o1, p1, l1, s1);
    if (live) {
      *reinterpret_cast<ulonglong2*>(reinterpret_cast<char*>(oo) + j * 16u) = make_ulonglong2(o0, o1);
      *reinterpret_cast<ulonglong2*>(reinterpret_cast<char*>(po) + j * 16u) = make_ulonglong2(p0, p1);
      *reinterpret_cast<ulonglong2*>(reinterpret_cast<char*>(lo) + j * 16u) = make_ulonglong2(l0, l1);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(so) + j * 4u) = (uint32_t)s0 | ((uint32_t)s1 << 16);
    }
  }
}
// v37: I/O only in v36's pattern
__global__ __launch_bounds__(256) void v37(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  const uint32_t n2 = (uint32_t)(n_ / 2);
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n2; j += stride) {
    const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(reinterpret_cast<const char*>(own) + j * 16u);
    const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(reinterpret_cast<const char*>(opp) + j * 16u);
    const uint32_t c = *reinterpret_cast<const uint16_t*>(act + j * 2u);
    *reinterpret_cast<ulonglong2*>(reinterpret_cast<char*>(oo) + j * 16u) = make_ulonglong2(a.x ^ c, a.y);
    *reinterpret_cast<ulonglong2*>(reinterpret_cast<char*>(po) + j * 16u) = b;
    *reinterpret_cast<ulonglong2*>(reinterpret_cast<char*>(lo) + j * 16u) = make_ulonglong2(a.x | b.x, a.y | b.y);
    *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(so) + j * 4u) = c * 3u;
  }
}
// v38: I/O only, one position per lane, plain stores, 32-bit offsets (the product's pattern)
__global__ __launch_bounds__(256) void v38(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  const uint32_t n = (uint32_t)n_;
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const uint64_t a = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(own) + i * 8u);
    const uint64_t b = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(opp) + i * 8u);
    const uint32_t c = act[i];
    *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(oo) + i * 8u) = a ^ c;
    *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(po) + i * 8u) = b;
    *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(lo) + i * 8u) = a | b;
    *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(so) + i * 2u) = (uint16_t)(c * 3u);
  }
}

// v39 / v41: v36 with non-temporal stores (v41: and non-temporal loads); v40: v33 with
// non-temporal stores
typedef uint64_t u64x2v __attribute__((ext_vector_type(2)));
template <bool NTL>
__device__ __forceinline__ void step39(const uint64_t* rays, const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  const uint32_t n2 = (uint32_t)(n_ / 2);
  const uint32_t stride = gridDim.x * 256;
  const uint32_t n_pad = (n2 + 255) / 256 * 256;
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n_pad; j += stride) {
    const bool live = j < n2;
    u64x2v a = {0, 0}, b = {0, 0};
    uint32_t c = 0x4040;
    if (live) {
      const u64x2v* pa = reinterpret_cast<const u64x2v*>(reinterpret_cast<const char*>(own) + j * 16u);
      const u64x2v* pb = reinterpret_cast<const u64x2v*>(reinterpret_cast<const char*>(opp) + j * 16u);
      if (NTL) { a = __builtin_nontemporal_load(pa); b = __builtin_nontemporal_load(pb); }
      else { a = *pa; b = *pb; }
      c = *reinterpret_cast<const uint16_t*>(act + j * 2u);
    }
    uint64_t o0, p0, l0, o1, p1, l1; uint16_t s0, s1;
    body36(rays, a.x, b.x, c & 0xFF, live, o0, p0, l0, s0);
    body36(rays, a.y, b.y, c >> 8, live, o1, p1, l1, s1);
    if (live) {
      u64x2v vo = {o0, o1}, vp = {p0, p1}, vl = {l0, l1};
      __builtin_nontemporal_store(vo, reinterpret_cast<u64x2v*>(reinterpret_cast<char*>(oo) + j * 16u));
      __builtin_nontemporal_store(vp, reinterpret_cast<u64x2v*>(reinterpret_cast<char*>(po) + j * 16u));
      __builtin_nontemporal_store(vl, reinterpret_cast<u64x2v*>(reinterpret_cast<char*>(lo) + j * 16u));
      __builtin_nontemporal_store((uint32_t)s0 | ((uint32_t)s1 << 16), reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(so) + j * 4u));
    }
  }
}
__global__ __launch_bounds__(256) void v39(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  step39<false>(rays, own, opp, act, oo, po, lo, so, n);
}
__global__ __launch_bounds__(256) void v41(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  step39<true>(rays, own, opp, act, oo, po, lo, so, n);
}
__global__ __launch_bounds__(256) void v40(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  RAYS
  const uint32_t n = (uint32_t)n_;
  const uint32_t stride = gridDim.x * 256;
  const uint32_t n_pad = (n + 255) / 256 * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n_pad; i += stride) {
    const bool live = i < n;
    uint64_t o = 0, p = 0; int a = azb::kPass;
    if (live) { o = own[i]; p = opp[i]; a = act[i]; }
    uint64_t no, np, lg; uint16_t st;
    body36(rays, o, p, a, live, no, np, lg, st);
    if (live) {
      __builtin_nontemporal_store(no, oo + i); __builtin_nontemporal_store(np, po + i);
      __builtin_nontemporal_store(lg, lo + i); __builtin_nontemporal_store(st, so + i);
    }
  }
}

// v42: v41 with two pairs per lane per iteration (pairs j and j + stride/2... as two
// grid-stride streams): both pairs' loads issued before either is computed
__global__ __launch_bounds__(256) void v42(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  RAYS
  const uint32_t n2 = (uint32_t)(n_ / 2);
  const uint32_t stride = gridDim.x * 512;
  for (uint32_t j0 = blockIdx.x * 512 + threadIdx.x; j0 < n2; j0 += stride) {
    const uint32_t j1 = j0 + 256;  // n2 is a multiple of 512 in this harness
    const u64x2v* pa = reinterpret_cast<const u64x2v*>(own);
    const u64x2v* pb = reinterpret_cast<const u64x2v*>(opp);
    const u64x2v a0 = __builtin_nontemporal_load(pa + j0), b0 = __builtin_nontemporal_load(pb + j0);
    const u64x2v a1 = __builtin_nontemporal_load(pa + j1), b1 = __builtin_nontemporal_load(pb + j1);
    const uint32_t c0 = reinterpret_cast<const uint16_t*>(act)[j0], c1 = reinterpret_cast<const uint16_t*>(act)[j1];
    uint64_t o[4], p[4], l[4]; uint16_t st[4];
    body36(rays, a0.x, b0.x, c0 & 0xFF, true, o[0], p[0], l[0], st[0]);
    body36(rays, a0.y, b0.y, c0 >> 8, true, o[1], p[1], l[1], st[1]);
    body36(rays, a1.x, b1.x, c1 & 0xFF, true, o[2], p[2], l[2], st[2]);
    body36(rays, a1.y, b1.y, c1 >> 8, true, o[3], p[3], l[3], st[3]);
    u64x2v* qo = reinterpret_cast<u64x2v*>(oo); u64x2v* qp = reinterpret_cast<u64x2v*>(po); u64x2v* ql = reinterpret_cast<u64x2v*>(lo);
    __builtin_nontemporal_store(u64x2v{o[0], o[1]}, qo + j0); __builtin_nontemporal_store(u64x2v{o[2], o[3]}, qo + j1);
    __builtin_nontemporal_store(u64x2v{p[0], p[1]}, qp + j0); __builtin_nontemporal_store(u64x2v{p[2], p[3]}, qp + j1);
    __builtin_nontemporal_store(u64x2v{l[0], l[1]}, ql + j0); __builtin_nontemporal_store(u64x2v{l[2], l[3]}, ql + j1);
    __builtin_nontemporal_store((uint32_t)st[0] | ((uint32_t)st[1] << 16), reinterpret_cast<uint32_t*>(so) + j0);
    __builtin_nontemporal_store((uint32_t)st[2] | ((uint32_t)st[3] << 16), reinterpret_cast<uint32_t*>(so) + j1);
  }
}
// v43: v41 at 512 threads per block
__global__ __launch_bounds__(512) void v43(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  __shared__ __align__(16) uint64_t rays[256]; if (threadIdx.x < 256) rays[threadIdx.x] = azb::ray_up(threadIdx.x >> 2, threadIdx.x & 3); __syncthreads();
  const uint32_t n2 = (uint32_t)(n / 2);
  const uint32_t stride = gridDim.x * 512;
  for (uint32_t j = blockIdx.x * 512 + threadIdx.x; j < n2; j += stride) {
    const u64x2v a = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(own) + j);
    const u64x2v b = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(opp) + j);
    const uint32_t c = reinterpret_cast<const uint16_t*>(act)[j];
    uint64_t o0, p0, l0, o1, p1, l1; uint16_t s0, s1;
    body36(rays, a.x, b.x, c & 0xFF, true, o0, p0, l0, s0);
    body36(rays, a.y, b.y, c >> 8, true, o1, p1, l1, s1);
    __builtin_nontemporal_store(u64x2v{o0, o1}, reinterpret_cast<u64x2v*>(oo) + j);
    __builtin_nontemporal_store(u64x2v{p0, p1}, reinterpret_cast<u64x2v*>(po) + j);
    __builtin_nontemporal_store(u64x2v{l0, l1}, reinterpret_cast<u64x2v*>(lo) + j);
    __builtin_nontemporal_store((uint32_t)s0 | ((uint32_t)s1 << 16), reinterpret_cast<uint32_t*>(so) + j);
  }
}

// v44: product k_step2 body (lane constants hoisted); v45: the same with the two positions'
// phases separated (both moves, both legal masks, then both terminal checks) for ILP
template <bool SPLIT, int PRE = 1>
__device__ __forceinline__ void pair44(const uint64_t* rays, const azb::WaveLane& L, u64x2v a, u64x2v b, uint32_t c, bool live,
  uint64_t* r) {
  if (SPLIT) {
    const azb::Move m0 = azb::move_rays_bf(rays, a.x, b.x, c & 0xFF);
    const azb::Move m1 = azb::move_rays_bf(rays, a.y, b.y, c >> 8);
    const bool ok0 = live && !m0.illegal, ok1 = live && !m1.illegal;
    const uint64_t l0 = ok0 ? azb::legal(m0.own, m0.opp) : 0ull;
    const uint64_t l1 = ok1 ? azb::legal(m1.own, m1.opp) : 0ull;
    int t0 = azb::terminal_flags_wave(m0.own, m0.opp, l0, ok0);
    int t1 = azb::terminal_flags_wave(m1.own, m1.opp, l1, ok1);
    t0 = azb::finish_terminal_wave(t0, m0.own, m0.opp, L);
    t1 = azb::finish_terminal_wave(t1, m1.own, m1.opp, L);
    r[0] = m0.own; r[1] = m1.own; r[2] = m0.opp; r[3] = m1.opp; r[4] = l0; r[5] = l1;
    const uint16_t s0 = m0.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(m0.flags | t0, azb::popc(m0.own) - azb::popc(m0.opp));
    const uint16_t s1 = m1.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(m1.flags | t1, azb::popc(m1.own) - azb::popc(m1.opp));
    r[6] = (uint32_t)s0 | ((uint32_t)s1 << 16);
  } else {
    for (int k = 0; k < 2; ++k) {
      const azb::Move m = azb::move_rays_bf(rays, k ? a.y : a.x, k ? b.y : b.x, k ? (c >> 8) : (c & 0xFF));
      const bool ok = live && !m.illegal;
      const uint64_t lg = ok ? azb::legal(m.own, m.opp) : 0ull;
      int t = azb::terminal_flags_wave(m.own, m.opp, lg, ok);
      t = azb::finish_terminal_wave<PRE>(t, m.own, m.opp, L);
      r[k] = m.own; r[2 + k] = m.opp; r[4 + k] = lg;
      const uint16_t s = m.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(m.flags | t, azb::popc(m.own) - azb::popc(m.opp));
      r[6] = k ? (r[6] | ((uint32_t)s << 16)) : s;
    }
  }
}
template <bool SPLIT, int PRE = 1>
__device__ __forceinline__ void k44(const uint64_t* rays, const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  const azb::WaveLane L = azb::wave_lane();
  const uint32_t n2 = (uint32_t)(n_ / 2);
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n2; j += stride) {
    const u64x2v a = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(own) + j);
    const u64x2v b = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(opp) + j);
    const uint32_t c = reinterpret_cast<const uint16_t*>(act)[j];
    uint64_t r[7];
    pair44<SPLIT, PRE>(rays, L, a, b, c, true, r);
    __builtin_nontemporal_store(u64x2v{r[0], r[1]}, reinterpret_cast<u64x2v*>(oo) + j);
    __builtin_nontemporal_store(u64x2v{r[2], r[3]}, reinterpret_cast<u64x2v*>(po) + j);
    __builtin_nontemporal_store(u64x2v{r[4], r[5]}, reinterpret_cast<u64x2v*>(lo) + j);
    __builtin_nontemporal_store((uint32_t)r[6], reinterpret_cast<uint32_t*>(so) + j);
  }
}
__global__ __launch_bounds__(256) void v44(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  k44<false>(rays, own, opp, act, oo, po, lo, so, n);
}
__global__ __launch_bounds__(256) void v45(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  k44<true>(rays, own, opp, act, oo, po, lo, so, n);
}

// v46 / v47: sensitivity probes on the product body — 20 extra `s_nop 0` per position
// (are the hazard pads after inline-asm shifts free?) / 20 extra dependent-free VALU per
// position (what does one VALU cost?)
template <int PROBE>
__device__ __forceinline__ void k46(const uint64_t* rays, const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  const azb::WaveLane L = azb::wave_lane();
  const uint32_t n2 = (uint32_t)(n_ / 2);
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n2; j += stride) {
    const u64x2v a = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(own) + j);
    const u64x2v b = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(opp) + j);
    const uint32_t c = reinterpret_cast<const uint16_t*>(act)[j];
    uint64_t r[7];
    pair44<false>(rays, L, a, b, c, true, r);
    if (PROBE == 1) {
#pragma unroll
      for (int k = 0; k < 40; ++k) asm volatile("s_nop 0");
    } else if (PROBE == 2) {
      uint32_t x0 = (uint32_t)r[0], x1 = (uint32_t)r[1], x2 = (uint32_t)r[2], x3 = (uint32_t)r[3];
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        asm volatile("v_xor_b32 %0, %0, %1\n\tv_xor_b32 %1, %1, %0\n\tv_xor_b32 %2, %2, %3\n\tv_xor_b32 %3, %3, %2"
                     : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
      }
      r[6] ^= (x0 ^ x1 ^ x2 ^ x3) & 0x80000000u & (uint32_t)(r[4] >> 63);  // keep them live
    }
    __builtin_nontemporal_store(u64x2v{r[0], r[1]}, reinterpret_cast<u64x2v*>(oo) + j);
    __builtin_nontemporal_store(u64x2v{r[2], r[3]}, reinterpret_cast<u64x2v*>(po) + j);
    __builtin_nontemporal_store(u64x2v{r[4], r[5]}, reinterpret_cast<u64x2v*>(lo) + j);
    __builtin_nontemporal_store((uint32_t)r[6], reinterpret_cast<uint32_t*>(so) + j);
  }
}
__global__ __launch_bounds__(256) void v46(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  k46<1>(rays, own, opp, act, oo, po, lo, so, n);
}
__global__ __launch_bounds__(256) void v47(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  k46<2>(rays, own, opp, act, oo, po, lo, so, n);
}

// v48: probe — v44 without the cooperative terminal pass (terminal flags wrong for real
// passes): what the rare pass costs on this corpus
__global__ __launch_bounds__(256) void v48(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  RAYS
  const uint32_t n2 = (uint32_t)(n_ / 2);
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n2; j += stride) {
    const u64x2v a = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(own) + j);
    const u64x2v b = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(opp) + j);
    const uint32_t c = reinterpret_cast<const uint16_t*>(act)[j];
    uint64_t r[7];
    for (int k = 0; k < 2; ++k) {
      const azb::Move m = azb::move_rays_bf(rays, k ? a.y : a.x, k ? b.y : b.x, k ? (c >> 8) : (c & 0xFF));
      const bool ok = !m.illegal;
      const uint64_t lg = ok ? azb::legal(m.own, m.opp) : 0ull;
      int t = azb::terminal_flags_wave(m.own, m.opp, lg, ok);
      t = t < 0 ? azb::kFlagNoPlace : t;
      r[k] = m.own; r[2 + k] = m.opp; r[4 + k] = lg;
      const uint16_t s = m.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(m.flags | t, azb::popc(m.own) - azb::popc(m.opp));
      r[6] = k ? (r[6] | ((uint32_t)s << 16)) : s;
    }
    __builtin_nontemporal_store(u64x2v{r[0], r[1]}, reinterpret_cast<u64x2v*>(oo) + j);
    __builtin_nontemporal_store(u64x2v{r[2], r[3]}, reinterpret_cast<u64x2v*>(po) + j);
    __builtin_nontemporal_store(u64x2v{r[4], r[5]}, reinterpret_cast<u64x2v*>(lo) + j);
    __builtin_nontemporal_store((uint32_t)r[6], reinterpret_cast<uint32_t*>(so) + j);
  }
}

// v49: v44 without the row pre-test of the cooperative terminal pass (A/B for it)
__global__ __launch_bounds__(256) void v49(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  k44<false, 0>(rays, own, opp, act, oo, po, lo, so, n);
}

// v50: v44 with the row + column pre-test
__global__ __launch_bounds__(256) void v50(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n) {
  RAYS
  k44<false, 2>(rays, own, opp, act, oo, po, lo, so, n);
}

// The terminal check of two positions per lane (a lane's pair, f0/f1 from
// terminal_flags_wave) in ONE sequence of cooperative passes: the pending positions of both
// halves form one list (position 0's pending lanes, then position 1's), eight per pass.
namespace azb {
template <int PRE = 1>
__device__ __forceinline__ void finish_terminal_wave2(int& f0, uint64_t own0, uint64_t opp0,
                                                      int& f1, uint64_t own1, uint64_t opp1,
                                                      const WaveLane& L) {
  uint64_t n0 = __ballot(f0 < 0), n1 = __ballot(f1 < 0);
  if (!(n0 | n1)) return;
  if (PRE) {
    if (f0 < 0) {
      const uint64_t m = moves_row_up(opp0, own0 & kInner) |
                         rev64(moves_row_up(rev64(opp0), rev64(own0) & kInner));
      if (m & ~(own0 | opp0)) f0 = kFlagNoPlace;
    }
    if (f1 < 0) {
      const uint64_t m = moves_row_up(opp1, own1 & kInner) |
                         rev64(moves_row_up(rev64(opp1), rev64(own1) & kInner));
      if (m & ~(own1 | opp1)) f1 = kFlagNoPlace;
    }
    n0 = __ballot(f0 < 0);
    n1 = __ballot(f1 < 0);
  }
  const int c0 = popc(n0), total = c0 + popc(n1);
  const int r0 = popc(n0 & L.below), r1 = c0 + popc(n1 & L.below);
  bool o0 = false, o1 = false;
  for (int base = 0; base < total; base += 8) {
    const int item = base + L.grp;
    const bool second = item >= c0;
    uint64_t m = item < total ? (second ? n1 : n0) : 0ull;
    const int k = second ? item - c0 : item;
    for (int j = 0; j < k && m; ++j) m &= m - 1;
    const int src = m ? __builtin_ctzll(m) : 0;
    const uint64_t P0 = __shfl(opp0, src, 64), O0 = __shfl(own0, src, 64);
    const uint64_t P1 = __shfl(opp1, src, 64), O1 = __shfl(own1, src, 64);
    const uint64_t mv = m ? dir_moves(second ? P1 : P0, second ? O1 : O0, L) : 0ull;
    const uint64_t any = __ballot(mv != 0);
    if (f0 < 0 && r0 >= base && r0 < base + 8) o0 = ((any >> (8 * (r0 - base))) & 0xFFull) != 0;
    if (f1 < 0 && r1 >= base && r1 < base + 8) o1 = ((any >> (8 * (r1 - base))) & 0xFFull) != 0;
  }
  if (f0 < 0) f0 = o0 ? kFlagNoPlace : (kFlagNoPlace | kFlagTerminal);
  if (f1 < 0) f1 = o1 ? kFlagNoPlace : (kFlagNoPlace | kFlagTerminal);
}
}  // namespace azb

// v51: v45 (phases split) with one merged cooperative terminal pass for the pair
__global__ __launch_bounds__(256) void v51(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n_) {
  RAYS
  const azb::WaveLane L = azb::wave_lane();
  const uint32_t n2 = (uint32_t)(n_ / 2);
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n2; j += stride) {
    const u64x2v a = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(own) + j);
    const u64x2v b = __builtin_nontemporal_load(reinterpret_cast<const u64x2v*>(opp) + j);
    const uint32_t c = reinterpret_cast<const uint16_t*>(act)[j];
    const azb::Move m0 = azb::move_rays_bf(rays, a.x, b.x, c & 0xFF);
    const bool ok0 = !m0.illegal;
    const uint64_t l0 = ok0 ? azb::legal(m0.own, m0.opp) : 0ull;
    const azb::Move m1 = azb::move_rays_bf(rays, a.y, b.y, c >> 8);
    const bool ok1 = !m1.illegal;
    const uint64_t l1 = ok1 ? azb::legal(m1.own, m1.opp) : 0ull;
    int t0 = azb::terminal_flags_wave(m0.own, m0.opp, l0, ok0);
    int t1 = azb::terminal_flags_wave(m1.own, m1.opp, l1, ok1);
    azb::finish_terminal_wave2(t0, m0.own, m0.opp, t1, m1.own, m1.opp, L);
    const uint16_t s0 = m0.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(m0.flags | t0, azb::popc(m0.own) - azb::popc(m0.opp));
    const uint16_t s1 = m1.illegal ? azb::pack_status(azb::kFlagIllegal, 0) : azb::pack_status(m1.flags | t1, azb::popc(m1.own) - azb::popc(m1.opp));
    __builtin_nontemporal_store(u64x2v{m0.own, m1.own}, reinterpret_cast<u64x2v*>(oo) + j);
    __builtin_nontemporal_store(u64x2v{m0.opp, m1.opp}, reinterpret_cast<u64x2v*>(po) + j);
    __builtin_nontemporal_store(u64x2v{l0, l1}, reinterpret_cast<u64x2v*>(lo) + j);
    __builtin_nontemporal_store((uint32_t)s0 | ((uint32_t)s1 << 16), reinterpret_cast<uint32_t*>(so) + j);
  }
}

extern "C" int run_variant(int v, const uint64_t* own, const uint64_t* opp, const uint8_t* act,
  uint64_t* oo, uint64_t* po, uint64_t* lo, uint16_t* so, int64_t n, int grid, void* stream) {
  void (*ks[])(const uint64_t*, const uint64_t*, const uint8_t*, uint64_t*, uint64_t*, uint64_t*, uint16_t*, int64_t) =
    {v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v0, v16, v17, v18, v19, v20, v21, v22, v23, v24, v25, v26, v27, v28, v29, v30, v31, v32, v33, v34, v35, v36, v37, v38, v39, v40, v41, v42, v43, v44, v45, v46, v47, v48, v49, v50, v51};
  if (v < 0 || v > 51) return -1;
  const int blk = v == 14 ? 64 : (v == 43 ? 512 : 256);
  hipLaunchKernelGGL(ks[v], dim3(v == 14 ? grid * 4 : grid), dim3(blk), 0, (hipStream_t)stream, own, opp, act, oo, po, lo, so, n);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
