// bitboard.h — 8x8 Othello bitboard primitives shared by the host entry points and
// the gfx950 kernels (one source of truth, compiled by hipcc for both sides).
//
// Layout: bit b <-> board square (r, c) with b = r*8 + c, i.e. the row-major array
// index of the reference's (8,8) int8 state.  This is `_BitBoard`'s own layout
// (reference envs/othello.py:202-212, `to_numpy` uses bit r*8+c); `OthelloGameNew`
// additionally rotates by 180 degrees (envs/othello.py:336-356) but Othello rules and the
// initial position are invariant under that rotation, so every result below is
// bit-identical after the index map.  Boards are always (own, opp) = (side to move,
// opponent), like `_BitBoard.black/white` (envs/othello.py:129-134).
//
// Algorithms are NOT the reference's dumb7 shift loop (envs/othello.py:157-200); they
// compute the same rule-defined sets with fewer integer ops (the rule-defined legal set
// and capture set are unique, so equality with the reference is a property of the rules;
// tests/ check it against the oracle and the reference-generated golden vectors):
//   * legal():  horizontal moves by carry propagation (the downward direction on the
//               bit-reversed board), the other three direction pairs by occluded fill with
//               propagator doubling (3 fill steps per direction instead of 6), every
//               three-input and/or step one v_bitop3_b32 per half on gfx950;
//   * flips():  per-line ray masks built arithmetically, first non-opponent square found
//               with a bit-scan (lowest bit upward, highest bit downward);
//   * flips_rays(): the batched kernels' form — the eight rays of the placed square from
//               a 2 KB up-ray table (down-rays = up-rays of 63 - sq on the bit-reversed
//               board), each ray's capture found with one subtraction (o - 1).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AZ_HD __host__ __device__ __forceinline__

namespace azb {

constexpr uint64_t kInner = 0x7E7E7E7E7E7E7E7Eull;  // columns 1..6
constexpr uint64_t kDiag = 0x8040201008040201ull;   // squares (i, i)
constexpr uint64_t kAnti = 0x0102040810204080ull;   // squares (i, 7 - i)
constexpr uint64_t kInitOwn = 0x0000000810000000ull;  // +1 at (3,4),(4,3): side to move
constexpr uint64_t kInitOpp = 0x0000001008000000ull;  // -1 at (3,3),(4,4)

constexpr int kPass = 64;

// status word of one board step: low byte = flags, high byte = signed disc difference
// (side to move after the step minus its opponent).
enum : int {
  kFlagTerminal = 1,  // neither side has a placement (envs/othello.py:435-454)
  kFlagNoPlace = 2,   // side to move has no placement: only the pass action is valid
  kFlagIllegal = 4,   // input action was not a legal placement (reference: ValueError)
  kFlagPassed = 8,    // input action was the pass (64)
};

AZ_HD int popc(uint64_t x) { return __builtin_popcountll(x); }

// ---- three-input bitwise ops ---------------------------------------------------------
// bop3<T>(a, b, c): any boolean function of three words in one v_bitop3_b32 per 32-bit
// half on gfx950 (the compiler does not form it from 64-bit and/or chains).  T is the
// truth table over a = 0xF0, b = 0xCC, c = 0xAA, e.g. T(a | (b & c)) = 0xF8.
namespace tt {
constexpr uint8_t A = 0xF0, B = 0xCC, C = 0xAA;
}
template <uint8_t T>
AZ_HD uint64_t bop3(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, T);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32),
                                                  (uint32_t)(c >> 32), T);
  return ((uint64_t)hi << 32) | lo;
#else
  uint64_t r = 0;
  for (int i = 0; i < 8; ++i)
    if ((T >> i) & 1) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
  return r;
#endif
}
// 180-degree rotation of the board = bit reversal of the word (v_bfrev_b32 x 2): square
// r*8+c -> (7-r)*8+(7-c), so a ray towards lower bit indices becomes one towards higher.
AZ_HD uint64_t rev64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return ((uint64_t)__builtin_bitreverse32((uint32_t)x) << 32) |
         __builtin_bitreverse32((uint32_t)(x >> 32));
#else
  return __builtin_bitreverse64(x);
#endif
}

// Whole-word shifts by a constant.  On the device they are pinned to one v_lshlrev_b64 /
// v_lshrrev_b64 on a register pair: left to itself the compiler narrows a 64-bit shift
// whose halves feed bop3 into two or three 32-bit ops.
#ifndef AZ_SHIFT_ASM
#define AZ_SHIFT_ASM 1  // measured faster than the alignbit pairs (0.171 vs 0.200 ms / 2^24)
#endif
template <int S>
AZ_HD uint64_t shl(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(S > 0 && S < 32, "constant shifts below one word");
#if AZ_SHIFT_ASM
  uint64_t r;
  asm("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "i"(S), "v"(x));
  return r;
#else
  // two 32-bit ops (v_lshlrev_b32 + v_alignbit_b32), no inline asm (after which the hazard
  // recognizer pads an s_nop); slower here: the 64-bit shift is one full-rate instruction
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, 32 - S) << 32) | (uint32_t)(lo << S);
#endif
#else
  return x << S;
#endif
}
template <int S>
AZ_HD uint64_t shr(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(S > 0 && S < 32, "constant shifts below one word");
#if AZ_SHIFT_ASM
  uint64_t r;
  asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(S), "v"(x));
  return r;
#else
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> S) << 32) | __builtin_amdgcn_alignbit(hi, lo, S);
#endif
#else
  return x >> S;
#endif
}

// a << S and b >> S in one asm statement: the hazard recognizer pads one s_nop after an
// inline-asm block it cannot see into, so pairing the fill's two directions halves them
template <int S>
AZ_HD void shl_shr(uint64_t a, uint64_t b, uint64_t& l, uint64_t& r) {
#if defined(__HIP_DEVICE_COMPILE__) && AZ_SHIFT_ASM
  asm("v_lshlrev_b64 %0, %2, %3\n\tv_lshrrev_b64 %1, %2, %4"
      : "=&v"(l), "=v"(r) : "i"(S), "v"(a), "v"(b));
#else
  l = shl<S>(a);
  r = shr<S>(b);
#endif
}

// Candidate moves of P through masked opponent stones M along +D (l) and -D (r): occluded
// fill with propagator doubling (1 + 1 + 2 + 2 steps cover the six possible run lengths).
template <int D>
AZ_HD void moves_dir2(uint64_t P, uint64_t M, uint64_t& l, uint64_t& r) {
  using namespace tt;
  uint64_t sl, sr;
  shl_shr<D>(P, P, sl, sr);
  uint64_t fl = M & sl;
  uint64_t fr = M & sr;
  shl_shr<D>(fl, fr, sl, sr);
  fl = bop3<A | (B & C)>(fl, M, sl);
  fr = bop3<A | (B & C)>(fr, M, sr);
  const uint64_t ml = M & shl<D>(M);
  const uint64_t mr = shr<D>(ml);
  shl_shr<2 * D>(fl, fr, sl, sr);
  fl = bop3<A | (B & C)>(fl, ml, sl);
  fr = bop3<A | (B & C)>(fr, mr, sr);
  shl_shr<2 * D>(fl, fr, sl, sr);
  fl = bop3<A | (B & C)>(fl, ml, sl);
  fr = bop3<A | (B & C)>(fr, mr, sr);
  shl_shr<D>(fl, fr, l, r);
}

template <int D>
AZ_HD uint64_t moves_dir(uint64_t P, uint64_t M) {
  uint64_t l, r;
  moves_dir2<D>(P, M, l, r);
  return l | r;
}

// Horizontal moves by carry propagation: a run of opponent stones (columns 1..6, so no
// run crosses a row end) starting just above an own stone is cleared by adding its first
// stone, and the carry lands on the square past the run.  The downward direction is the
// upward one on the 180-degree-rotated board.
AZ_HD uint64_t moves_row_up(uint64_t P, uint64_t I) {
  const uint64_t s = (P << 1) & I;
  return (s + I) & ~I;  // landing squares (filtered by `empty` by the caller)
}

// moves_row_up without the final & ~I: the carry word keeps the opponent stones of runs
// that did not start at an own stone, and the caller's `empty` mask removes them (and the
// carries that land on an occupied square) anyway
AZ_HD uint64_t carries_row_up(uint64_t P, uint64_t I) {
  const uint64_t s = (P << 1) & I;
  return s + I;
}

// Legal placements for `own` against `opp` (the rule of reference envs/othello.py:157-166).
AZ_HD uint64_t legal(uint64_t own, uint64_t opp) {
  using namespace tt;
  const uint64_t inner = opp & kInner;
  // eight candidate words (row up / down, three direction pairs) merged by three bop3 and
  // an or, the empty-square mask by a fourth bop3 (round 3: 8 VALU fewer than or-ing each
  // pair first and masking each row word; same-box k_step2 0.1290 vs 0.1293 ms)
  const uint64_t up = carries_row_up(own, inner);
  const uint64_t dn = rev64(carries_row_up(rev64(own), rev64(opp) & kInner));
  uint64_t l8, r8, l7, r7, l9, r9;
  moves_dir2<8>(own, opp, l8, r8);
  moves_dir2<7>(own, inner, l7, r7);
  moves_dir2<9>(own, inner, l9, r9);
  const uint64_t m1 = bop3<A | B | C>(up, dn, l8);
  const uint64_t m2 = bop3<A | B | C>(r8, l7, r7);
  const uint64_t m = bop3<A | B | C>(m1, m2, l9) | r9;
  return bop3<C & ~(A | B)>(own, opp, m);
}

// ---- capture set by ray masks ----------------------------------------------------------
// Up-rays (towards higher bit indices, `sq` excluded) of the four lines through a square:
// k = 0 row (+1), 1 column (+8), 2 diagonal (+9), 3 anti-diagonal (+7).  The down-rays of
// sq are the up-rays of 63 - sq on the rotated board (rev64).
constexpr uint64_t ray_up(int sq, int k) {
  const int dr = k == 0 ? 0 : 1, dc = k == 0 ? 1 : (k == 1 ? 0 : (k == 2 ? 1 : -1));
  uint64_t m = 0;
  int r = (sq >> 3) + dr, c = (sq & 7) + dc;
  while (r < 8 && c >= 0 && c < 8) {
    m |= 1ull << (r * 8 + c);
    r += dr;
    c += dc;
  }
  return m;
}

// The whole [64][4] up-ray table, built at compile time (kernels copy it into LDS with one
// load per thread instead of running ray_up's loop per block).
struct RayTable {
  uint64_t r[64 * 4];
  constexpr RayTable() : r{} {
    for (int i = 0; i < 64 * 4; ++i) r[i] = ray_up(i >> 2, i & 3);
  }
};

// bop3 with the third operand one 32-bit word applied to both halves (a sign mask).
template <uint8_t T>
AZ_HD uint64_t bop3_w(uint64_t a, uint64_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, c, T);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), c, T);
  return ((uint64_t)hi << 32) | lo;
#else
  return bop3<T>(a, b, ((uint64_t)c << 32) | c);
#endif
}

// x - 1 as one v_lshl_add_u64 on a register pair (left alone, the compiler forms it from
// the two halves bop3 produced with an extra 32-bit add)
AZ_HD uint64_t dec64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__) && AZ_SHIFT_ASM
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 0, -1" : "=v"(r) : "v"(x));
  return r;
#else
  return x - 1ull;
#endif
}

// Stones of `opp` captured along one up-ray R by a stone placed below it: the run of
// opponent stones up to the first non-opponent square x, kept only if x holds an own stone.
// x = lowbit(o) with o = R & ~opp; xo = x if it is own, else 0; e = xo - 1 is then the
// squares below x, or all ones when xo = 0 — the only case with the sign bit set (x is at
// most bit 63), so the sign mask of e's high word drops it: 9 VALU per ray, no compare or
// select.
AZ_HD uint64_t ray_flips(uint64_t R, uint64_t own, uint64_t opp) {
  using namespace tt;
  const uint64_t o = R & ~opp;                     // non-opponent squares of the ray
  const uint64_t d = o - 1ull;                     // bits below the first of them set
  const uint64_t xo = bop3<A & ~B & C>(o, d, own); // x itself, if it holds an own stone
  const uint64_t e = dec64(xo);
  const uint32_t neg = (uint32_t)((int32_t)(uint32_t)(e >> 32) >> 31);
  return bop3_w<A & B & ~C>(R, e, neg);
}

// flips() from ray tables: `up` = the four up-rays of sq, `upr` = those of 63 - sq;
// ownr / oppr = the rotated board.
AZ_HD uint64_t flips_rays(const uint64_t* up, const uint64_t* upr, uint64_t own,
                          uint64_t opp, uint64_t ownr, uint64_t oppr) {
  const uint64_t fu = ray_flips(up[0], own, opp) | ray_flips(up[1], own, opp) |
                      ray_flips(up[2], own, opp) | ray_flips(up[3], own, opp);
  const uint64_t fd = ray_flips(upr[0], ownr, oppr) | ray_flips(upr[1], ownr, oppr) |
                      ray_flips(upr[2], ownr, oppr) | ray_flips(upr[3], ownr, oppr);
  return fu | rev64(fd);
}

// Stones captured along one line through `sq`: the ray above sq (towards higher bit
// indices) and the ray below it.
AZ_HD uint64_t line_flips(uint64_t line, uint64_t own, uint64_t opp, int sq) {
  const uint64_t up = line & (~1ull << sq);
  const uint64_t dn = line & ((1ull << sq) - 1ull);
  uint64_t o = up & ~opp;
  const uint64_t x = o & (0ull - o);  // first non-opponent square going up
  uint64_t f = (x & own) ? ((x - 1ull) & up) : 0ull;
  o = dn & ~opp;
  const uint64_t y = o ? (0x8000000000000000ull >> __builtin_clzll(o)) : 0ull;
  f |= (y & own) ? (dn & ~((y << 1) - 1ull)) : 0ull;
  return f;
}

// Stones flipped by `own` placing on `sq` (the capture set of reference
// envs/othello.py:182-194).  Zero means the placement is illegal.
AZ_HD uint64_t flips(uint64_t own, uint64_t opp, int sq) {
  const int r = sq >> 3, c = sq & 7;
  const uint64_t row = 0xFFull << (sq & 56);
  const uint64_t col = 0x0101010101010101ull << c;
  const int k = c - r;
  const uint64_t diag = k >= 0 ? (kDiag >> (8 * k)) : (kDiag << (-8 * k));
  const int s = r + c;
  const uint64_t anti = s <= 7 ? (kAnti >> (8 * (7 - s))) : (kAnti << (8 * (s - 7)));
  return line_flips(row, own, opp, sq) | line_flips(col, own, opp, sq) |
         line_flips(diag, own, opp, sq) | line_flips(anti, own, opp, sq);
}

struct Step {
  uint64_t own, opp, legal;  // next side to move, its opponent, next side's placements
  uint16_t status;           // flags | (uint8 score << 8)
};

AZ_HD uint16_t pack_status(int flags, int score) {
  return (uint16_t)((flags & 0xFF) | (((unsigned)(uint8_t)(int8_t)score) << 8));
}

// Children after a placement / pass: the make-move of reference envs/othello.py:171-200
// (`own' = my ^ captured`, `opp' = opp ^ captured`, then swap sides).
AZ_HD void play(uint64_t own, uint64_t opp, int act, uint64_t cap, uint64_t* nown,
                uint64_t* nopp) {
  if (act == kPass) {
    *nown = opp;
    *nopp = own;
  } else {
    const uint64_t nb = 1ull << act;
    *nown = opp ^ cap;
    *nopp = (own | nb) ^ cap;
  }
}

// Terminal flags / value of a position (side to move = own): reference
// get_value_and_terminated (envs/othello.py:435-454) evaluated for the side to move.
// The opponent's full legal-mask fill runs only when no cheap proof exists: a full board
// or a side without stones ends the game outright (neither side can bound anything), so a
// wavefront skips the divergent second fill unless one of its lanes holds a real pass.
AZ_HD int terminal_flags(uint64_t own, uint64_t opp, uint64_t lg) {
  if (lg) return 0;
  if ((own | opp) == ~0ull || own == 0 || opp == 0) return kFlagNoPlace | kFlagTerminal;
  return legal(opp, own) ? kFlagNoPlace : (kFlagNoPlace | kFlagTerminal);
}

// ---- wave-cooperative terminal check (device) ----------------------------------------
// The lane-dependent constants of the cooperative pass below: computed once per kernel
// (wave_lane()) and kept in registers, so a grid-stride loop does not recompute them for
// every position ahead of the (usually skipped) cooperative branch.
struct WaveLane {
  uint64_t below;  // mask of the lanes below this one
  uint64_t bit;    // this lane's bit
  int grp;         // lane >> 3: which pending position of a pass this lane serves
  int s;           // shift of this lane's direction (1, 8, 7, 9)
  bool up;         // direction towards higher bits (lane & 7 < 4)
  bool col;        // the column direction (no wrap mask)
};

__device__ __forceinline__ WaveLane wave_lane() {
  const int lane = __lane_id();
  const int d = lane & 7;
  WaveLane L;
  L.bit = 1ull << lane;
  L.below = L.bit - 1ull;
  L.grp = lane >> 3;
  L.s = (0x09070801 >> ((d & 3) * 8)) & 0xFF;
  L.up = d < 4;
  L.col = (d & 3) == 1;
  return L;
}

// Legal placements of P against O along ONE direction (the lane's: shifts towards higher
// bits by 1, 8, 7, 9 for lane & 7 = 0..3, the same towards lower bits for 4..7), the fill
// of legal() split by direction so that eight lanes can share one position.
__device__ __forceinline__ uint64_t dir_moves(uint64_t P, uint64_t O, const WaveLane& L) {
  const int s = L.s;
  const uint64_t M = L.col ? O : (O & kInner);
  const bool up = L.up;
  uint64_t x = M & (up ? (P << s) : (P >> s));
#pragma unroll
  for (int i = 0; i < 5; ++i) x |= M & (up ? (x << s) : (x >> s));
  return (up ? (x << s) : (x >> s)) & ~(P | O);
}

// terminal_flags() for one position per lane, computed by the whole wavefront: the rare
// lanes that need the opponent's full fill (no placement, no cheap proof) are served eight
// lanes per position — one direction each — up to eight positions per pass, instead of the
// whole wavefront executing a divergent full legal() for them.  Every lane of the wave must
// call it (uniform control flow); `live` marks lanes that hold a position.
__device__ __forceinline__ int terminal_flags_wave(uint64_t own, uint64_t opp, uint64_t lg,
                                                   bool live) {
  if (!live || lg) return 0;
  if ((own | opp) == ~0ull || own == 0 || opp == 0) return kFlagNoPlace | kFlagTerminal;
  return -1;  // needs the cooperative pass
}

// PRE: a wave with pending lanes first tries the other side's horizontal placements
// (the carry pair of legal(), ~20 VALU once for the wave); only lanes still undecided
// enter the cooperative fill of all eight directions (~70 VALU per pass).
template <int PRE = 1>
__device__ __forceinline__ int finish_terminal_wave(int flags, uint64_t own, uint64_t opp,
                                                    const WaveLane& L) {
  uint64_t need = __ballot(flags < 0);
  if (PRE && need) {
    if (flags < 0) {  // placements of opp against own along the rows (legal(opp, own))
      uint64_t m = moves_row_up(opp, own & kInner) |
                   rev64(moves_row_up(rev64(opp), rev64(own) & kInner));
      if (PRE > 1) m |= moves_dir<8>(opp, own);  // and the columns
      if (m & ~(own | opp)) flags = kFlagNoPlace;
    }
    need = __ballot(flags < 0);
  }
  bool other = false;
  while (need) {
    uint64_t m = need;
    for (int j = 0; j < L.grp && m; ++j) m &= m - 1;
    const int src = m ? __builtin_ctzll(m) : 0;
    const uint64_t P = __shfl(opp, src, 64), O = __shfl(own, src, 64);
    const uint64_t mv = m ? dir_moves(P, O, L) : 0ull;
    const uint64_t any = __ballot(mv != 0);
    if (need & L.bit) {  // this lane's position is pending
      const int rank = popc(need & L.below);
      if (rank < 8) other = ((any >> (8 * rank)) & 0xFFull) != 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) need &= need - 1;
  }
  if (flags >= 0) return flags;
  return other ? kFlagNoPlace : (kFlagNoPlace | kFlagTerminal);
}

__device__ __forceinline__ int finish_terminal_wave(int flags, uint64_t own, uint64_t opp) {
  const WaveLane L = wave_lane();
  return finish_terminal_wave<1>(flags, own, opp, L);
}

struct Move {
  uint64_t own, opp;  // next side to move, its opponent (inputs unchanged when illegal)
  int flags;          // kFlagPassed for the pass
  bool illegal;
};

// The make-move half of step(): placement with flips (or pass), illegal placements
// detected (no capture, occupied square or out of range) and left unchanged.
AZ_HD Move move(uint64_t own, uint64_t opp, int act) {
  Move m;
  m.flags = 0;
  m.illegal = false;
  if (act == kPass) {
    m.own = opp;
    m.opp = own;
    m.flags = kFlagPassed;
    return m;
  }
  const bool in_range = (unsigned)act < 64u;
  const int sq = act & 63;
  const uint64_t nb = 1ull << sq;
  const uint64_t cap = in_range ? flips(own, opp, sq) : 0ull;
  if (!in_range || cap == 0ull || (nb & (own | opp))) {
    m.own = own;
    m.opp = opp;
    m.illegal = true;
    return m;
  }
  m.own = opp ^ cap;
  m.opp = (own | nb) ^ cap;
  return m;
}

// move() with the capture set from ray tables (`rays` = [64][4] up-rays, ray_up()).
AZ_HD Move move_rays(const uint64_t* rays, uint64_t own, uint64_t opp, int act) {
  Move m;
  m.flags = 0;
  m.illegal = false;
  if (act == kPass) {
    m.own = opp;
    m.opp = own;
    m.flags = kFlagPassed;
    return m;
  }
  const int sq = act & 63;
  const uint64_t nb = 1ull << sq;
  const uint64_t cap =
      flips_rays(rays + 4 * sq, rays + 4 * (63 - sq), own, opp, rev64(own), rev64(opp));
  if ((unsigned)act > 64u || cap == 0ull || (nb & (own | opp))) {
    m.own = own;
    m.opp = opp;
    m.illegal = true;
    return m;
  }
  m.own = opp ^ cap;
  m.opp = bop3<(tt::A | tt::B) ^ tt::C>(own, nb, cap);
  return m;
}

// move_rays() without branches (the batched kernel's form: a wave never diverges on the
// pass / illegal cases, which cost four selects instead).
AZ_HD Move move_rays_bf(const uint64_t* rays, uint64_t own, uint64_t opp, int act) {
  const int sq = act & 63;
  const uint64_t nb = 1ull << sq;
  const uint64_t cap =
      flips_rays(rays + 4 * sq, rays + 4 * (63 - sq), own, opp, rev64(own), rev64(opp));
  const bool place = (unsigned)act < 64u && cap != 0ull && !(nb & (own | opp));
  const bool pass = act == kPass;
  const uint64_t c = place ? cap : 0ull, b = place ? nb : 0ull;
  Move m;
  m.illegal = !(place || pass);
  m.flags = pass ? kFlagPassed : 0;
  m.own = m.illegal ? own : opp ^ c;
  m.opp = m.illegal ? opp : bop3<tt::A ^ tt::B ^ tt::C>(own, b, c);
  return m;
}

// One board step for one position: placement or pass, then the next side's legal mask,
// terminal check and disc difference.  Illegal placements leave the board unchanged and
// set kFlagIllegal (the reference raises ValueError at envs/othello.py:419-421).
AZ_HD Step step(uint64_t own, uint64_t opp, int act) {
  Step o;
  const Move m = move(own, opp, act);
  o.own = m.own;
  o.opp = m.opp;
  if (m.illegal) {
    o.legal = 0;
    o.status = pack_status(kFlagIllegal, 0);
    return o;
  }
  o.legal = legal(o.own, o.opp);
  const int flags = m.flags | terminal_flags(o.own, o.opp, o.legal);
  o.status = pack_status(flags, popc(o.own) - popc(o.opp));
  return o;
}

// step() on the ray-table capture set (the batched entry points' formulation).
AZ_HD Step step_rays(const uint64_t* rays, uint64_t own, uint64_t opp, int act) {
  Step o;
  const Move m = move_rays_bf(rays, own, opp, act);
  o.own = m.own;
  o.opp = m.opp;
  if (m.illegal) {
    o.legal = 0;
    o.status = pack_status(kFlagIllegal, 0);
    return o;
  }
  o.legal = legal(o.own, o.opp);
  const int flags = m.flags | terminal_flags(o.own, o.opp, o.legal);
  o.status = pack_status(flags, popc(o.own) - popc(o.opp));
  return o;
}

// ---- dihedral (D4) transforms on the row-major layout -------------------------------
// numpy semantics: rot90(m)[i][j] = m[j][7-i] (anticlockwise), fliplr(m)[i][j] = m[i][7-j].
AZ_HD uint64_t flip_ud(uint64_t x) { return __builtin_bswap64(x); }
AZ_HD uint64_t flip_lr(uint64_t x) {
  x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
  x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
  x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
  return x;
}
AZ_HD uint64_t transpose(uint64_t x) {  // out[i][j] = in[j][i]
  uint64_t t;  // three delta swaps (28, 14, 7)
  t = 0x0F0F0F0F00000000ull & (x ^ (x << 28));
  x ^= t ^ (t >> 28);
  t = 0x3333000033330000ull & (x ^ (x << 14));
  x ^= t ^ (t >> 14);
  t = 0x5500550055005500ull & (x ^ (x << 7));
  x ^= t ^ (t >> 7);
  return x;
}
AZ_HD uint64_t rot90(uint64_t x) { return flip_ud(transpose(x)); }
// sym = k + 4*flip: rot90 applied k times, then fliplr if flip (reference
// MCTS_model.py:15-28 `random_symmetry`, envs/othello.py:501-526).
AZ_HD uint64_t d4(uint64_t x, int sym) {
  for (int i = 0; i < (sym & 3); ++i) x = rot90(x);
  return (sym & 4) ? flip_lr(x) : x;
}
// Square index map of the same transform: out square of input square sq.
AZ_HD int d4_square(int sq, int sym) { return 63 - __builtin_clzll(d4(1ull << sq, sym)); }

}  // namespace azb
