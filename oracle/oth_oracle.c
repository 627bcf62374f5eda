/* oth_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference's bitboard rules engine, used by tests/ and by
 * bench.py's cpu_baseline leg as the oracle the HIP kernels are compared against.
 * It deliberately follows the reference's own algorithm (the "dumb7" masked shift fill),
 * not the product's faster formulation (csrc/bitboard.h):
 *
 *   masks / shifts      envs/othello.py:112-126  (_MASKS, _LSHIFTS, _RSHIFTS)
 *   _shift              envs/othello.py:147-155
 *   _legal_moves        envs/othello.py:157-166  (1 + 5 fill steps per direction)
 *   make_move           envs/othello.py:171-200  (pass = swap; capture if bounded)
 *   score               envs/othello.py:214-220
 *   get_next_state      envs/othello.py:413-433  (illegal -> error)
 *   get_value_and_terminated envs/othello.py:435-454
 *
 * Layout is `_BitBoard`'s: bit r*8+c.  Pinned against the tests/golden npz fixtures, which were
 * produced by running the reference itself (tests/golden/make_goldens.py).
 */
#include <stdint.h>

static const uint64_t MASKS[8] = {
    0x7F7F7F7F7F7F7F7Full, 0x007F7F7F7F7F7F7Full, 0xFFFFFFFFFFFFFFFFull,
    0x00FEFEFEFEFEFEFEull, 0xFEFEFEFEFEFEFEFEull, 0xFEFEFEFEFEFEFE00ull,
    0xFFFFFFFFFFFFFFFFull, 0x7F7F7F7F7F7F7F00ull};
static const int LSH[8] = {0, 0, 0, 0, 1, 9, 8, 7};
static const int RSH[8] = {1, 9, 8, 7, 0, 0, 0, 0};

static uint64_t shift_dir(uint64_t x, int d) {
  return d < 4 ? ((x >> RSH[d]) & MASKS[d]) : ((x << LSH[d]) & MASKS[d]);
}

uint64_t oracle_legal(uint64_t own, uint64_t opp) {
  uint64_t empty = ~(own | opp), moves = 0;
  for (int d = 0; d < 8; ++d) {
    uint64_t x = shift_dir(own, d) & opp;
    for (int k = 0; k < 5; ++k) x |= shift_dir(x, d) & opp;
    moves |= shift_dir(x, d) & empty;
  }
  return moves;
}

/* make_move on (own, opp); returns the next side's (own, opp) via out pointers. */
void oracle_make_move(uint64_t own, uint64_t opp, int action, uint64_t* nown,
                      uint64_t* nopp) {
  if (action == 64) {
    *nown = opp;
    *nopp = own;
    return;
  }
  uint64_t nw = 1ull << action, my = own | nw, cap = 0;
  for (int d = 0; d < 8; ++d) {
    uint64_t x = shift_dir(nw, d) & opp;
    for (int k = 0; k < 5; ++k) x |= shift_dir(x, d) & opp;
    if (shift_dir(x, d) & my) cap |= x;
  }
  *nown = opp ^ cap; /* swap after `black = my ^ cap; white = opp ^ cap` */
  *nopp = my ^ cap;
}

static int popc(uint64_t x) { return __builtin_popcountll(x); }

/* Batched reference board step with the product's output contract (see
 * include/az_othello.h: status = flags | score << 8).  Returns the index of the first
 * illegal placement, or -1. */
int64_t oracle_step(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
                    uint64_t* own_o, uint64_t* opp_o, uint64_t* legal_o,
                    uint16_t* status_o, int64_t n) {
  int64_t bad = -1;
  for (int64_t i = 0; i < n; ++i) {
    int a = act[i], flags = 0;
    uint64_t o = own[i], p = opp[i], no, np;
    if (a == 64) {
      flags |= 8;
    } else if (a > 64 || !((oracle_legal(o, p) >> a) & 1)) {
      /* get_next_state's illegal-move guard (envs/othello.py:419-421) */
      own_o[i] = o;
      opp_o[i] = p;
      legal_o[i] = 0;
      status_o[i] = 4;
      if (bad < 0) bad = i;
      continue;
    }
    oracle_make_move(o, p, a, &no, &np);
    uint64_t lg = oracle_legal(no, np);
    if (!lg) {
      flags |= 2;
      if (!oracle_legal(np, no)) flags |= 1;
    }
    int score = popc(no) - popc(np);
    own_o[i] = no;
    opp_o[i] = np;
    legal_o[i] = lg;
    status_o[i] = (uint16_t)((flags & 0xFF) | ((unsigned)(uint8_t)(int8_t)score << 8));
  }
  return bad;
}

void oracle_legal_batch(const uint64_t* own, const uint64_t* opp, uint64_t* out,
                        int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = oracle_legal(own[i], opp[i]);
}

/* Random playout from (own, opp) as MCTS._rollout does (MCTS_model.py:276-303): returns
 * the outcome sign from the starting side's view.  Used only for statistical checks. */
int oracle_rollout(uint64_t own, uint64_t opp, uint64_t seed) {
  uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1;
  int side = 1; /* +1: `own` is the original side to move */
  for (int ply = 0; ply < 200; ++ply) {
    uint64_t lg = oracle_legal(own, opp);
    int a = 64;
    if (lg) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      int k = (int)(s % (uint64_t)popc(lg));
      for (int i = 0; i < k; ++i) lg &= lg - 1;
      a = __builtin_ctzll(lg);
    }
    uint64_t no, np;
    oracle_make_move(own, opp, a, &no, &np);
    own = no;
    opp = np;
    side = -side;
    if (!oracle_legal(own, opp) && !oracle_legal(opp, own)) {
      int d = (popc(own) - popc(opp)) * side;
      return d > 0 ? 1 : (d < 0 ? -1 : 0);
    }
  }
  return 0;
}
