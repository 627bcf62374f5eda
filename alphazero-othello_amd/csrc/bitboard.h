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
//   * legal():  direction-pair occluded fill with propagator doubling (3 fill steps per
//               direction instead of 6);
//   * flips():  per-line ray masks built arithmetically, first non-opponent square found
//               with a bit-scan (lowest bit upward, highest bit downward).
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

// Candidate moves of P through masked opponent stones M along +D and -D.
template <int D>
AZ_HD uint64_t moves_dir(uint64_t P, uint64_t M) {
  uint64_t fl = M & (P << D);
  uint64_t fr = M & (P >> D);
  fl |= M & (fl << D);
  fr |= M & (fr >> D);
  const uint64_t ml = M & (M << D);
  const uint64_t mr = ml >> D;
  fl |= ml & (fl << (2 * D));
  fr |= mr & (fr >> (2 * D));
  fl |= ml & (fl << (2 * D));
  fr |= mr & (fr >> (2 * D));
  return (fl << D) | (fr >> D);
}

// Legal placements for `own` against `opp` (the rule of reference envs/othello.py:157-166).
AZ_HD uint64_t legal(uint64_t own, uint64_t opp) {
  const uint64_t inner = opp & kInner;
  uint64_t m = moves_dir<1>(own, inner);
  m |= moves_dir<8>(own, opp);
  m |= moves_dir<7>(own, inner);
  m |= moves_dir<9>(own, inner);
  return m & ~(own | opp);
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
// Legal placements of P against O along ONE direction d (0..3: shifts towards higher bits
// by 1, 8, 7, 9; 4..7: the same towards lower bits), the fill of legal() split by direction
// so that eight lanes can share one position.
__device__ __forceinline__ uint64_t dir_moves(uint64_t P, uint64_t O, int d) {
  const int s = (0x09070801 >> ((d & 3) * 8)) & 0xFF;
  const uint64_t M = (d & 3) == 1 ? O : (O & kInner);
  const bool up = d < 4;
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

__device__ __forceinline__ int finish_terminal_wave(int flags, uint64_t own, uint64_t opp) {
  const int lane = __lane_id();
  uint64_t need = __ballot(flags < 0);
  bool other = false;
  while (need) {
    const int grp = lane >> 3;
    uint64_t m = need;
    for (int j = 0; j < grp && m; ++j) m &= m - 1;
    const int src = m ? __builtin_ctzll(m) : lane;
    const uint64_t P = __shfl(opp, src, 64), O = __shfl(own, src, 64);
    const uint64_t mv = m ? dir_moves(P, O, lane & 7) : 0ull;
    const uint64_t any = __ballot(mv != 0);
    if ((need >> lane) & 1) {
      const int rank = popc(need & ((1ull << lane) - 1ull));
      if (rank < 8) other = ((any >> (8 * rank)) & 0xFFull) != 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) need &= need - 1;
  }
  if (flags >= 0) return flags;
  return other ? kFlagNoPlace : (kFlagNoPlace | kFlagTerminal);
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
