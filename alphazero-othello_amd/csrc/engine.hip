// engine.hip — batched MCTS self-play engine for gfx950.
//
// G game slots advance together.  Each slot owns a flat structure-of-arrays node arena
// (the reference's `Node` objects, MCTS_model.py:46-169, as rows of plain arrays) in two
// ping-pong halves: the live tree, and the target of the re-root compaction that
// MCTS.make_move's subtree reuse (MCTS_model.py:200-215) needs.
//
// One batched simulation step (graph-capturable, no host synchronisation):
//   k_select   one wavefront per slot: PUCT descent from the root (MCTS_model.py:362-370,
//              :129-139, ties -> lowest action), terminal leaves backed up in place
//              (:381-384); the first unexpanded leaf is packed as the canonical NN input
//              player*state (Models.py:16) into nn_in[g, 64].
//   (caller)   policy/value net on nn_in -> priors[g, 65] (softmax), values[g] (tanh).
//   k_expand   one wavefront per slot: root Dirichlet noise (:340-343), prior masking and
//              renormalisation (:345-349), eager creation of every legal child — one lane per
//              square runs that child's board step (flip, next-side legal mask, terminal
//              check: envs/othello.py:171-200, :157-166, :435-454) — and the sign-alternating
//              backup (:160-169).
//   k_move     (auto-play) one workgroup per slot whose search is done: pi from visit
//              counts (:244-274), trajectory record (self_play_worker.py:72-73), action
//              sample (:75), the move and terminal check (:77-79), TD(lambda) targets on
//              game end (:8-35, :80-86) and the re-root compaction (make_move).
//
// With one leaf per slot per step the search is exactly the reference with
// args['num_threads'] = 1: the only virtual loss visible in PUCT is the parent's own (+1 in
// the sqrt term), which the descent applies directly.  All float arithmetic reproduces the
// reference's NumPy-2 (NEP 50) promotion; the library is built with -ffp-contract=off.
#include <math.h>

#include <cstdlib>
#include <new>
#include <type_traits>
#include <vector>

#include "bitboard.h"
#include "common.h"
#include "philox.h"

namespace {

constexpr int kWave = 64;
constexpr int kSelBlock = 256;  // 4 slots (waves) per workgroup in select / expand
constexpr int kMoveBlock = 256;
constexpr int kMaxPath = 64;     // one wave lane per path depth for the parallel backup
constexpr int kMaxLeaves = 8;    // leaves_per_step limit (virtual-loss descents per step)

// One leaf per slot and step (K = 1): a select wave starts another descent (after terminal
// ones, backed up in place) only while this launch's descents walked fewer than this many
// tree levels, beside the max_descents cap -- the launch's span is its deepest end-game
// slot's chain of descents (~1.4 us per level at full load).  With one leaf per step a
// slot's sequence of descents and backups does not depend on where the launches split it,
// so games are unchanged; K > 1 keeps the cap alone (its virtual-loss batches would
// change).  14 measured best of 10 / 14 / 18 (profiles/r03_sel_levels_ab.json); 0 = off.
#ifndef AZ_SEL_LEVELS
#define AZ_SEL_LEVELS 14
#endif
// K = 1 select: a terminal descent backs up from the path's N / W held in registers (lane d =
// depth d, loaded by the descent itself) and patches the root's record and its children's
// PUCT inputs in registers instead of reloading them -- two dependent round trips fewer per
// terminal descent, the same stores and the same double additions; 0 = load N / W and reload
// the root (A/B builds)
#ifndef AZ_SEL_REGBACKUP
#define AZ_SEL_REGBACKUP 0
#endif
#ifndef AZ_MOVE_KC
#define AZ_MOVE_KC 4
#endif
#ifndef AZ_ENG_STAMP
#define AZ_ENG_STAMP 0
#endif
#if AZ_ENG_STAMP
// experiment builds only (scripts/build_variants.py -DAZ_ENG_STAMP=1): per-phase
// s_memrealtime stamps of k_move / k_expand workgroups, records of 8 in a ring no product
// kernel reads; scripts/eng_stamps.py summarises them
constexpr int kStampRecs = 1 << 14;
__device__ unsigned long long g_eng_stamps[kStampRecs * 8];
__device__ unsigned int g_eng_stamp_n;
#define ENG_STAMP_BEGIN(kind)                                                    \
  unsigned long long st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};                          \
  st_[0] = (kind);                                                               \
  st_[1] = __builtin_amdgcn_s_memrealtime()
#define ENG_STAMP(i) st_[i] = __builtin_amdgcn_s_memrealtime()
__shared__ unsigned long long g_cst[4];  // compact()'s phase stamps (thread 0)
#define CST(i)                                                  \
  do {                                                          \
    if (threadIdx.x == 0) g_cst[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define ENG_STAMP_END()                                                          \
  do {                                                                           \
    if ((threadIdx.x & 63) == 0) {                                               \
      const unsigned r_ = atomicAdd(&g_eng_stamp_n, 1u) & (kStampRecs - 1);      \
      for (int i_ = 0; i_ < 8; ++i_) g_eng_stamps[r_ * 8 + i_] = st_[i_];        \
    }                                                                            \
  } while (0)
#else
#define ENG_STAMP_BEGIN(kind) \
  do {                        \
  } while (0)
#define ENG_STAMP(i) \
  do {               \
  } while (0)
#define ENG_STAMP_END() \
  do {                  \
  } while (0)
#define CST(i) \
  do {         \
  } while (0)
#endif

enum : uint8_t { kExpanded = 1, kTerminal = 2, kChildF64 = 4 };
enum : int32_t { kIdle = AZ_GAME_IDLE, kActive = AZ_GAME_ACTIVE, kFinished = AZ_GAME_FINISHED,
                 kSearchDone = 3 };

// Node arena: one entry per (half, slot, node).  half in {0,1}, node < cap.
struct Arena {
  uint64_t* own;    // side to move at this node
  uint64_t* opp;
  uint64_t* legal;  // placements of `own`; 0 => only the pass action (envs/othello.py:401-403)
  int32_t* N;       // visit_count
  double* W;        // value_sum (from this node's player's view)
  double* P;        // prior (f32-exact unless the parent carries kChildF64)
  int32_t* parent;
  int32_t* first;   // first child (children contiguous, ascending action)
  uint8_t* nchild;
  uint8_t* action;
  uint8_t* flags;
  int8_t* tval;     // terminal_value for terminal nodes
};

struct Games {
  int32_t* status;
  int32_t* half;       // live arena half
  int32_t* n_nodes;
  int32_t* sims_done;
  int32_t* sims_target;
  unsigned long long* sims_acc;  // simulations completed by the slot (summed into ctr->sims
                                 // by az_counters: no device-wide atomic per wave per step)
  int32_t* leaf;       // [G, K] leaves awaiting evaluation in descent order, -1 ends the list
  int32_t* path;       // [G, K, kMaxPath] root..leaf node indices of each pending leaf
  int32_t* path_len;   // [G, K] entries in `path`; 0 => deeper than kMaxPath, walk parents
  int32_t* ply;
  int32_t* root_player;
  int32_t* winner;
  int32_t* overflow;
  int32_t* start_step; // slot becomes active at this engine step (stagger)
  int32_t* sstep;      // deferred moves: the slot's own step count (its k_select calls)
  int32_t* moving;     // deferred moves: the slot step whose search finished (the next
                       // step's k_select skips the slot while k_move re-roots it)
  uint32_t* rng_event; // per-slot RNG event counter
  uint8_t* sym;        // [G, K] D4 transform of each pending leaf
  int32_t* noise_cur;  // injected-stream cursors
  int32_t* u_cur;
  // K > 1 auto-play: leaves of a batch still open when the launch's descent cap stopped it
  // (rows 0 .. open - 1 hold them, their virtual loss applied; 0 = no open batch)
  int32_t* open;
  // trajectory [G, T]
  uint64_t* t_own;
  uint64_t* t_opp;
  float* t_pi;  // [G, T, 65]
  int8_t* t_player;
  double* t_vroot;
};

struct Counters {  // device-side, 64-bit
  unsigned long long games_started;
  unsigned long long games_finished;
  unsigned long long samples_n;
  unsigned long long samples_dropped;
  unsigned long long overflow;
  unsigned long long step;
  unsigned long long sims;
  unsigned long long moves;
  long long start_budget;  // games still allowed to start (refill)
  int32_t ready_n[2];      // k_move's work lists: slots whose search finished in a step of
                           // parity q (list 0 only, unless moves are deferred)
  int32_t unlimited;       // refill without a start budget
  int32_t move_done;       // k_move workgroups finished this step (the last one resets)
};

struct Samples {
  uint64_t* own;
  uint64_t* opp;
  float* pi;  // [cap, 65]
  double* z;
  int8_t* player;
  int32_t* slot;  // game slot that produced the row
  int64_t cap;
};

struct Params {
  Arena a;
  Games g;
  Samples s;
  Counters* ctr;
  int32_t* ready;  // [2][G] the two work lists
  const double* inj_noise;  // [G, NS, 65]
  const double* inj_u;      // [G, NU]
  int32_t G, C, T, NS, NU;
  int32_t sims;
  int32_t K;  // leaves per slot per step (virtual loss, MCTS_model.py num_threads)
  int32_t n_explore;
  int32_t eval_mode, rng_mode, d4, auto_play, refill;
  int32_t defer;   // deferred moves (az_engine_defer_moves)
  // the evaluation's stem computed by the wave that packs each row (az_engine_set_stem)
  const float* stem_w;  // [9][stem_c] tap-major
  const float* stem_b;  // [stem_c]
  float* stem_y;        // [G*K][64][stem_c] NHWC fp32
  float* stem_amax;     // [G*K] each row's max |y| (optional)
  int32_t stem_c;       // 0 (off), 64 or 128
  double c_puct, alpha, eps, temp, lambd;
  uint64_t seed;
  uint32_t stream_id;
};

__device__ __forceinline__ int64_t nidx(const Params& p, int half, int g, int i) {
  return ((int64_t)half * p.G + g) * (int64_t)p.C + i;
}

// ---------------------------------------------------------------------------------
// wave helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

template <typename T>
__device__ __forceinline__ T shfl(T v, int src) {
  return __shfl(v, src, kWave);
}

// v_readlane_b32 per dword: `lane` must be wave-uniform
template <typename T>
__device__ __forceinline__ T readlane(T v, int lane) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "readlane: 32- or 64-bit values");
  if constexpr (sizeof(T) == 8) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
  }
}

// NumPy's pairwise sum of a contiguous length-65 vector (numpy/_core/src/umath/
// loops_utils.h.src pairwise_sum: eight running partials over the first 64 elements,
// combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the tail element).  x = this lane's
// element (lanes 0..63), x64 = element 64.  Returns the sum in every lane.
template <typename T>
__device__ T np_sum65(T x, T x64) {
  const int lane = lane_id();
  T r = x;
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    const T y = shfl(x, (lane + 8 * i) & 63);
    r = r + y;
  }
  const T r0 = readlane(r, 0), r1 = readlane(r, 1), r2 = readlane(r, 2), r3 = readlane(r, 3);
  const T r4 = readlane(r, 4), r5 = readlane(r, 5), r6 = readlane(r, 6), r7 = readlane(r, 7);
  T res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  res = res + x64;
  return res;
}

__device__ __forceinline__ uint64_t ballot(bool b) { return __ballot(b); }

// Wave argmax with Python max()'s tie rule (the first maximum, i.e. the lowest lane):
// the scores become order-preserving unsigned keys (-0 folded into +0, as a float compare
// sees them; absent lanes 0), the wave maximum comes from the DPP reduction
// __ockl_wfred_max_u32 (VALU data-parallel moves, no LDS round trips), and the lowest lane
// holding it from a ballot.  Called with the whole wave active.
__device__ __forceinline__ uint32_t order_key32(float s) {
  const uint32_t b = __float_as_uint(s + 0.0f);
  return b ^ ((b >> 31) ? 0xffffffffu : 0x80000000u);
}
__device__ __forceinline__ int wave_argmax_f32(float s, bool live) {
  const uint32_t key = live ? order_key32(s) : 0u;
  const uint32_t m = __ockl_wfred_max_u32(key);
  return (int)__builtin_ctzll(ballot(live && key == m));
}
__device__ __forceinline__ int wave_argmax_f64(double s, bool live) {
  const uint64_t b = (uint64_t)__double_as_longlong(s + 0.0);
  const uint64_t key = live ? (b ^ ((b >> 63) ? ~0ull : 0x8000000000000000ull)) : 0ull;
  const uint32_t hi = (uint32_t)(key >> 32), lo = (uint32_t)key;
  const uint32_t mh = __ockl_wfred_max_u32(hi);
  const uint32_t ml = __ockl_wfred_max_u32(hi == mh ? lo : 0u);
  return (int)__builtin_ctzll(ballot(live && hi == mh && lo == ml));
}


// ---------------------------------------------------------------------------------
// node helpers (executed by the whole wave; stores by lane 0 only where noted)

__device__ void init_root(const Params& p, int g, int half, uint64_t own, uint64_t opp) {
  const int64_t r = nidx(p, half, g, 0);
  p.a.own[r] = own;
  p.a.opp[r] = opp;
  p.a.legal[r] = azb::legal(own, opp);
  p.a.N[r] = 0;
  p.a.W[r] = 0.0;
  p.a.P[r] = 0.0;
  p.a.parent[r] = -1;
  p.a.first[r] = -1;
  p.a.nchild[r] = 0;
  p.a.action[r] = 0;
  p.a.flags[r] = 0;  // the root is never terminal-flagged (MCTS_model.py:103-106)
  p.a.tval[r] = 0;
}

// Node.backpropagate (MCTS_model.py:160-169): N += 1, W += sign*v, sign alternating up.
__device__ void backup(const Params& p, int g, int half, int node, double v) {
  double s = 1.0;
  while (node >= 0) {
    const int64_t k = nidx(p, half, g, node);
    p.a.N[k] += 1;
    p.a.W[k] += s * v;
    s = -s;
    node = p.a.parent[k];
  }
}

// The same update with the path held one node per lane (lane d = depth d, leaf at depth
// `leaf_depth` < kMaxPath): every node's N/W is read and written in one round trip instead
// of one dependent parent load per level.  W += (+/-1)*v is the identical double addition.
__device__ void backup_path(const Params& p, int g, int half, int path_node, int leaf_depth,
                            double v) {
  const int lane = lane_id();
  if (lane <= leaf_depth) {
    const int64_t k = nidx(p, half, g, path_node);
    const int n = p.a.N[k];
    const double w = p.a.W[k];
    p.a.N[k] = n + 1;
    p.a.W[k] = w + (((leaf_depth - lane) & 1) ? -v : v);
  }
}

// The net's stem (Models.py:179-180, :209: 3x3 conv 1 -> C, BatchNorm folded, ReLU) on the
// plane row the wave has just packed, when the net hands its stem to the engine
// (az_engine_set_stem): y[row] NHWC fp32 and the row's max |y| (the fp16x2 trunk's input
// range).  k_conv_stem's (conv.hip) fmaf chain in its tap order, so bit-identical to it.
// pl = the plane's value at square `lane`; lane = channels V*lane .. V*lane + V - 1.
#ifndef AZ_STEM_NOSTORE
#define AZ_STEM_NOSTORE 0
#endif
#ifndef AZ_STEM_PK
#define AZ_STEM_PK 1  // 128 channels: the two channels of a lane as packed fp32 fma
#endif
#ifndef AZ_STEM_CODE
#define AZ_STEM_CODE 1  // experiment builds: 0 compiles the engine stem out
#endif
// One board row py of the stem: tap rows dy in [DYLO, DYHI] exist (compile time, as the
// columns: no branch per tap), so the top and bottom rows are separate code and the six
// inner rows one loop.
template <int C, int DYLO, int DYHI, class VecT>
__device__ __forceinline__ void stem_board_row(const VecT (&w)[9], VecT b, float pl, int py,
                                               VecT* __restrict__ y, float& bmax) {
  constexpr int V = C / kWave;
  float v[3][8];  // the plane's rows py-1 .. py+1 (uniform)
#pragma unroll
  for (int dy = DYLO; dy <= DYHI; ++dy)
#pragma unroll
    for (int x = 0; x < 8; ++x) v[dy + 1][x] = readlane(pl, (py + dy) * 8 + x);
#pragma unroll
  for (int px = 0; px < 8; ++px) {
    VecT acc = b;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3 - 1, xx = px + t % 3 - 1;
      if (dy < DYLO || dy > DYHI || xx < 0 || xx > 7) continue;
      if constexpr (V == 2) {
#if AZ_STEM_PK
        // both channels in one v_pk_fma_f32 (per component the same single-rounding fma)
        typedef float f2v __attribute__((ext_vector_type(2)));
        const f2v s2 = {v[dy + 1][xx], v[dy + 1][xx]}, w2 = {w[t].x, w[t].y};
        f2v a2 = {acc.x, acc.y};
        a2 = __builtin_elementwise_fma(s2, w2, a2);
        acc.x = a2.x;
        acc.y = a2.y;
#else
        acc.x = fmaf(v[dy + 1][xx], w[t].x, acc.x);
        acc.y = fmaf(v[dy + 1][xx], w[t].y, acc.y);
#endif
      } else {
        acc = fmaf(v[dy + 1][xx], w[t], acc);
      }
    }
    if constexpr (V == 2) {
      acc.x = fmaxf(acc.x, 0.f);
      acc.y = fmaxf(acc.y, 0.f);
      bmax = fmaxf(bmax, fmaxf(acc.x, acc.y));
    } else {
      acc = fmaxf(acc, 0.f);
      bmax = fmaxf(bmax, acc);
    }
#if !AZ_STEM_NOSTORE  // experiment builds: the stem's arithmetic without its stores
    y[(py * 8 + px) * (C / V)] = acc;
#endif
  }
}

template <int C>
__device__ __forceinline__ void stem_row(const Params& p, int64_t row, float pl) {
  constexpr int V = C / kWave;
  using VecT = typename std::conditional<V == 2, float2, float>::type;
  const int lane = lane_id();
  VecT w[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) w[t] = reinterpret_cast<const VecT*>(p.stem_w + t * C)[lane];
  const VecT b = reinterpret_cast<const VecT*>(p.stem_b)[lane];
  VecT* y = reinterpret_cast<VecT*>(p.stem_y + row * 64 * C) + lane;
  float bmax = 0.0f;
  stem_board_row<C, 0, 1>(w, b, pl, 0, y, bmax);
#pragma unroll 1
  for (int py = 1; py < 7; ++py) stem_board_row<C, -1, 1>(w, b, pl, py, y, bmax);
  stem_board_row<C, -1, 0>(w, b, pl, 7, y, bmax);
  if (p.stem_amax) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bmax = fmaxf(bmax, __shfl_xor(bmax, o, kWave));
    if (lane == 0) p.stem_amax[row] = bmax;
  }
}

__device__ __forceinline__ void emit_stem(const Params& p, int64_t row, float pl) {
#if !AZ_STEM_CODE
  return;
#endif
  if (p.stem_c == 128) stem_row<128>(p, row, pl);
  else if (p.stem_c == 64) stem_row<64>(p, row, pl);
}

// Pack the canonical NN input player*state (Models.py:16): own stones +1, opponent -1,
// optionally through D4 transform `sym` (random_symmetry, MCTS_model.py:15-28; square q of
// the transformed board is bit q of d4(own) / d4(opp)).
// Returns the value stored (the stem's input at square `lane`).
__device__ float emit_leaf(float* nn_in, int64_t row, uint64_t own, uint64_t opp, int sym) {
  const int lane = lane_id();
  const uint64_t P = sym ? azb::d4(own, sym) : own, N = sym ? azb::d4(opp, sym) : opp;
  const float pl = ((P >> lane) & 1) ? 1.0f : (((N >> lane) & 1) ? -1.0f : 0.0f);
  nn_in[row * 64 + lane] = pl;
  return pl;
}

__device__ void emit_none(float* nn_in, int32_t* leaf_o, int64_t row) {
  nn_in[row * 64 + lane_id()] = 0.0f;
  if (lane_id() == 0 && leaf_o) leaf_o[row] = -1;
}

// rows without a leaf (skipped / idle slots): the stem of an empty board
__device__ void emit_none_rows(const Params& p, float* nn_in, int32_t* leaf_o, int64_t row0,
                               int K) {
  for (int j = 0; j < K; ++j) emit_none(nn_in, leaf_o, row0 + j);
  if (p.stem_c)
    for (int j = 0; j < K; ++j) emit_stem(p, row0 + j, 0.0f);
}

// What the descent needs of a node, loaded together with its siblings' PUCT inputs so that
// one round trip per tree level suffices.
struct NodeRec {
  int node;
  int first;         // first child
  int visits;        // N
  int meta;          // flags | nchild << 8 | (uint8)tval << 16
  uint64_t own, opp; // the position (the leaf's NN input, without another load)
  double wv;         // W (AZ_SEL_REGBACKUP: the terminal backup from registers)
};

__device__ __forceinline__ NodeRec load_rec(const Params& p, int g, int half, int node) {
  const int64_t k = nidx(p, half, g, node);
  NodeRec r;
  r.node = node;
  r.first = p.a.first[k];
  r.visits = p.a.N[k];
  r.meta = (int)p.a.flags[k] | ((int)p.a.nchild[k] << 8) | ((int)(uint8_t)p.a.tval[k] << 16);
  r.own = p.a.own[k];
  r.opp = p.a.opp[k];
  r.wv = AZ_SEL_REGBACKUP ? p.a.W[k] : 0.0;
  return r;
}
__device__ __forceinline__ uint8_t rec_flags(const NodeRec& r) { return (uint8_t)r.meta; }
__device__ __forceinline__ int rec_nchild(const NodeRec& r) { return (r.meta >> 8) & 0xff; }
__device__ __forceinline__ int rec_tval(const NodeRec& r) { return (int)(int8_t)(r.meta >> 16); }

// One child's PUCT inputs and record (a select_child lane's loads).
struct KidIn {
  int n, first, meta;
  double w, pr;
  uint64_t own, opp;
};

__device__ __forceinline__ KidIn load_kid(const Params& p, int g, int half, int node) {
  const int64_t c = nidx(p, half, g, node);
  KidIn k;
  k.n = p.a.N[c];
  k.w = p.a.W[c];
  k.pr = p.a.P[c];
  k.first = p.a.first[c];
  k.meta = (int)p.a.flags[c] | ((int)p.a.nchild[c] << 8) | ((int)(uint8_t)p.a.tval[c] << 16);
  k.own = p.a.own[c];
  k.opp = p.a.opp[c];
  return k;
}

// The root's record together with its children's (one round trip): an expanded root's
// children are always nodes 1..nchild -- the root expands into the arena's second slot, and
// the stable re-root compaction keeps a subtree root's child group right behind it -- so
// lane j loads node 1 + j speculatively (in bounds: C >= 128); select_child_rec checks
// first == 1 before using them.
__device__ __forceinline__ NodeRec load_root(const Params& p, int g, int half, KidIn& kid) {
  kid = load_kid(p, g, half, 1 + lane_id());
  return load_rec(p, g, half, 0);
}

// PUCT child choice of MCTS._select_child / Node._get_ucb_score (MCTS_model.py:129-139,
// :362-370).  NumPy-2 promotion: with float32 priors every operation after the Python-float
// sqrt is float32 (c_puct and q are cast to float32); with the Dirichlet-noised root's
// float64 priors it is all float64.  The node's own virtual visit (+1, MCTS_model.py:378)
// enters the sqrt; the children carry none.  max() keeps the first maximum in ascending
// action order, i.e. the lowest child index (wave_argmax_*).
// The parent's record is already in registers, each lane
// loads its child's PUCT inputs AND its record, and the winner's record is read from its
// lane (v_readlane: the winner is wave-uniform) -- the next level starts without another
// load.
__device__ NodeRec select_child_rec(const Params& p, int g, int half, const NodeRec& par,
                                   bool use_pre, const KidIn& pre) {
  const int lane = lane_id();
  const int nc = rec_nchild(par);
  const int fc = par.first;
  const bool f64 = (rec_flags(par) & kChildF64) != 0;
  const double sq = sqrt((double)(par.visits + 1) + 1e-8);
  const bool live = lane < nc;
  NodeRec mine{0, 0, 0, 0, 0ull, 0ull};
  double sd = 0.0;
  float sf = 0.0f;
  if (live) {
    const KidIn k = use_pre && fc == 1 ? pre : load_kid(p, g, half, fc + lane);
    const int n = k.n;
    const double w = k.w;
    const double pr = k.pr;
    mine.first = k.first;
    mine.meta = k.meta;
    mine.visits = n;
    mine.own = k.own;
    mine.opp = k.opp;
    mine.wv = w;
    const double q = -(n == 0 ? 0.0 : w / (double)n);
    if (f64) {
      const double u = p.c_puct * pr * sq / (double)(1 + n);
      sd = q + u;
    } else {
      const float u = (((float)p.c_puct * (float)pr) * (float)sq) / (float)(1 + n);
      sf = (float)q + u;
    }
  }
  const int idx = f64 ? wave_argmax_f64(sd, live) : wave_argmax_f32(sf, live);
  NodeRec r;
  r.node = fc + idx;
  r.first = readlane(mine.first, idx);
  r.visits = readlane(mine.visits, idx);
  r.meta = readlane(mine.meta, idx);
  r.own = readlane(mine.own, idx);
  r.opp = readlane(mine.opp, idx);
  r.wv = AZ_SEL_REGBACKUP ? readlane(mine.wv, idx) : 0.0;
  return r;
}

// list q: 0, or with deferred moves the step's parity; sst: the slot's step (deferred)
__device__ void push_ready(const Params& p, int g, int q = 0, int sst = 0) {
  const int i = atomicAdd(&p.ctr->ready_n[q], 1);
  p.ready[q * p.G + i] = g;
  if (p.defer) p.g.moving[g] = sst;
}

// ---------------------------------------------------------------------------------
// k_select

// Virtual visits of the descents waiting for evaluation in this step (leaves_per_step > 1,
// the reference's num_threads workers, MCTS_model.py:115-118, :196-197): lane d of path[j]
// holds waiting descent j's node at depth d (-1 past its leaf).  A node at depth d can only
// sit at depth d of a path, so its virtual visits are the waiting paths holding it there.
template <int KMAX>
struct Waiting {
  int path[KMAX];
  int n;
};

template <int KMAX>
__device__ __forceinline__ int virtual_visits(const Waiting<KMAX>& w, int depth, int node) {
  int c = 0;
#pragma unroll
  for (int j = 0; j < KMAX; ++j)
    if (j < w.n) c += readlane(w.path[j], depth) == node ? 1 : 0;
  return c;
}

// select_child_rec with virtual loss (Node.value = (W + VV) / (N + VV), the parent's own
// and the waiting descents' visits in the sqrt term, 1 + N + VV below it: MCTS_model.py:
// 110-114, :129-139).  With no waiting descent this is select_child_rec's arithmetic.
template <int KMAX>
__device__ NodeRec select_child_vl(const Params& p, int g, int half, const NodeRec& par,
                                   int depth, const Waiting<KMAX>& w, bool use_pre,
                                   const KidIn& pre) {
  const int lane = lane_id();
  const int nc = rec_nchild(par);
  const int fc = par.first;
  const bool f64 = (rec_flags(par) & kChildF64) != 0;
  const int vvp = 1 + virtual_visits(w, depth, par.node);
  const double sq = sqrt((double)(par.visits + vvp) + 1e-8);
  const int vvc = depth + 1 < kMaxPath ? virtual_visits(w, depth + 1, fc + lane) : 0;
  const bool live = lane < nc;
  NodeRec mine{0, 0, 0, 0, 0ull, 0ull};
  double sd = 0.0;
  float sf = 0.0f;
  if (live) {
    const KidIn k = use_pre && fc == 1 ? pre : load_kid(p, g, half, fc + lane);
    const int n = k.n;
    const double wv = k.w;
    const double pr = k.pr;
    mine.first = k.first;
    mine.meta = k.meta;
    mine.visits = n;
    mine.own = k.own;
    mine.opp = k.opp;
    const int nv = n + vvc;
    const double q = -(nv == 0 ? 0.0 : (wv + (double)vvc) / (double)nv);
    if (f64) {
      const double u = p.c_puct * pr * sq / (double)(1 + nv);
      sd = q + u;
    } else {
      const float u = (((float)p.c_puct * (float)pr) * (float)sq) / (float)(1 + nv);
      sf = (float)q + u;
    }
  }
  const int idx = f64 ? wave_argmax_f64(sd, live) : wave_argmax_f32(sf, live);
  NodeRec r;
  r.node = fc + idx;
  r.first = readlane(mine.first, idx);
  r.visits = readlane(mine.visits, idx);
  r.meta = readlane(mine.meta, idx);
  r.own = readlane(mine.own, idx);
  r.opp = readlane(mine.opp, idx);
  return r;
}

// KMAX = 1: one leaf per slot per step (num_threads = 1).  KMAX > 1: up to K = p.K leaves,
// descents run one after another, each seeing the earlier ones' virtual loss; terminal
// descents back up at once, the others wait for the batched evaluation in rows
// nn_in[g*K + j] (the interleaving tests/golden/make_vl_goldens.py forces on the reference).
__device__ __forceinline__ void move_body(const Params& p, int q, int deferred, int nblocks,
                                          int bid);
template <int KMAX>
__device__ __forceinline__ bool expand_slot(const Params& p, int g,
                                            const float* __restrict__ priors,
                                            const float* __restrict__ values, int par,
                                            int sst_push);

// par / move_blocks (deferred moves, az_select_move): the first move_blocks workgroups run the
// move phase of the previous step's list (par ^ 1) while the others descend; a slot whose
// move is in that list is skipped (nothing of it is read: k_move writes it concurrently, and
// those writes become visible at the launch boundary) and plays again next step.
// FUSED (az_select_move_expand; deferred moves only): each slot's wave first expands and backs
// up the previous step's waiting leaves (expand_slot on priors / values, the evaluation that
// step's net wrote), then descends -- one launch per step instead of select + expand.  A
// search those leaves complete joins this step's move list (moved by the next launch) and
// the slot sits this step out, so each of its moves lands one step later than with k_expand;
// which step a move lands in never changes a game.
template <int KMAX, bool MERGED = false, bool FUSED = false>
__global__ __launch_bounds__(kSelBlock) void k_select(Params p,
                                                      float* __restrict__ nn_in,
                                                      int32_t* __restrict__ leaf_o,
                                                      int max_descents, int par,
                                                      int move_blocks,
                                                      const float* __restrict__ priors,
                                                      const float* __restrict__ values) {
  if constexpr (MERGED) {  // a separate instantiation: the plain one keeps its registers
    if ((int)blockIdx.x < move_blocks) {
      move_body(p, par ^ 1, 1, move_blocks, (int)blockIdx.x);
      return;
    }
  } else {
    move_blocks = 0;
  }
  const int g = ((int)blockIdx.x - move_blocks) * (kSelBlock / kWave) + (threadIdx.x >> 6);
  if (g >= p.G) return;
  const int K = KMAX == 1 ? 1 : p.K;
  const int64_t row0 = (int64_t)g * K;
  const int lane = lane_id();
  // every per-slot word in one round trip
  ENG_STAMP_BEGIN(3);
  int sst = 0;  // deferred moves: this slot's step (its own count of select calls)
  if (p.defer) {
    sst = p.g.sstep[g];
    if (lane == 0) p.g.sstep[g] = sst + 1;
    if (p.g.moving[g] == sst - 1) {
      emit_none_rows(p, nn_in, leaf_o, row0, K);
      return;
    }
  }
  if constexpr (FUSED) {
    if (expand_slot<KMAX>(p, g, priors, values, par, sst)) {
      emit_none_rows(p, nn_in, leaf_o, row0, K);
      return;
    }
    // the expansion's and backup's stores before this wave's descent loads
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
  ENG_STAMP(2);
  const int status = p.g.status[g];
  // the stagger schedule counts steps: the engine's, or the slot's own with deferred moves
  // (the engine's counter is advanced inside a deferred launch)
  const unsigned long long step = p.defer ? (unsigned long long)sst : p.ctr->step;
  const int start_step = p.g.start_step[g];
  const int half = p.g.half[g];
  int sims_done = p.g.sims_done[g];
  const int target = p.g.sims_target[g];
  // the slot's counters as of this point (only this wave writes them from here on): the end
  // of the launch updates them without another load round trip
  const int sims0 = sims_done;
  const unsigned long long acc0 = p.g.sims_acc[g];
  if (status != kActive || (long long)step < (long long)start_step) {
    emit_none_rows(p, nn_in, leaf_o, row0, K);
    return;
  }
  Waiting<KMAX> w;
  w.n = 0;
  float plane[KMAX];  // the packed rows' values at square `lane` (the stem's inputs)
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    w.path[j] = -1;
    plane[j] = 0.0f;
  }
  int open0 = 0;
  if constexpr (KMAX > 1) {
    // an open batch (the last launch's descent cap stopped it before K leaves waited):
    // its leaves keep their rows and virtual loss, and this launch's descents continue it --
    // the reference's schedule (a batch = simulations started until K wait on the net) is
    // the same wherever launches split it
    open0 = p.g.open[g];
    if (open0 > 0) {
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        if (j < open0) {
          const int64_t row = row0 + j;
          const int plen = p.g.path_len[row];
          w.path[j] = lane < plen ? p.g.path[row * kMaxPath + lane] : -1;
          plane[j] = nn_in[row * 64 + lane];
        }
      }
      w.n = open0;
    }
  }
  bool deep = false;  // a waiting path past kMaxPath: its virtual loss could not be tracked
  int depth = 0;      // depth of the current node
  int path_node = 0;  // lane d: node at depth d of the current descent
  KidIn kid0;  // the root's children (load_root)
  NodeRec cur = load_root(p, g, half, kid0);
  // the leaf in `cur` waits for evaluation as row g*K + w.n
  auto wait_leaf = [&]() {
    const int j = w.n;
    const int64_t row = row0 + j;
    int sym = 0;
    if (p.d4) {
      const uint32_t ev = p.g.rng_event[g];
      sym = (int)(azr::uniform1(p.seed, (uint32_t)g, ev, 0x5000u, p.stream_id) * 8.0) & 7;
      if (lane == 0) {
        p.g.rng_event[g] = ev + 1;
        p.g.sym[row] = (uint8_t)sym;
      }
    }
    const float pl = emit_leaf(nn_in, row, cur.own, cur.opp, sym);
#pragma unroll
    for (int jj = 0; jj < KMAX; ++jj)
      if (jj == j) plane[jj] = pl;
    const bool held = depth < kMaxPath && lane <= depth;
    if (held) p.g.path[row * kMaxPath + lane] = path_node;
    if (lane == 0) {
      p.g.path_len[row] = depth < kMaxPath ? depth + 1 : 0;
      p.g.leaf[row] = cur.node;
      if (leaf_o) leaf_o[row] = cur.node;
    }
    if constexpr (KMAX > 1) {
#pragma unroll
      for (int jj = 0; jj < KMAX; ++jj)
        if (jj == j) w.path[jj] = held ? path_node : -1;
      deep = deep || depth >= kMaxPath;
    }
    w.n = j + 1;
  };
  // the root's own expansion (an unexplored root) is a batch of its own, never left open
  bool root_wait = false;
  if (!(rec_flags(cur) & kExpanded)) {
    wait_leaf();  // policy_improve_step expands an unexplored root first (MCTS_model.py:234-235)
    root_wait = true;
  } else {
    int guard = 0;
    // tree levels walked by this launch's descents: the level budget (AZ_SEL_LEVELS, K = 1)
    // applies to auto-play engines only -- a host-driven select (the drop-in MCTS) must
    // keep returning a leaf or the finished search, as its fixed-length graph relies on
    int levels = 0;
    const bool level_budget = KMAX == 1 && AZ_SEL_LEVELS > 0 && p.auto_play;
    constexpr bool RB = KMAX == 1 && AZ_SEL_REGBACKUP;
    bool patched = false;  // RB: the root record and kid0 are current in registers
    NodeRec root = cur;
    int path_n = 0;        // RB: lane d: N and W of the node at depth d
    double path_w = 0.0;
    while (sims_done + w.n < target && w.n < K && guard < max_descents &&
           (!level_budget || levels < AZ_SEL_LEVELS)) {
      if (guard > 0) {  // the last backup changed the root's N
        if (RB && patched)
          cur = root;
        else
          cur = load_root(p, g, half, kid0);
      }
      root = cur;
      patched = false;
      ++guard;
      depth = 0;
      path_node = 0;
      if constexpr (RB) {
        if (lane == 0) {
          path_n = cur.visits;
          path_w = cur.wv;
        }
      }
      while (true) {
        const uint8_t f = rec_flags(cur);
        if (f & kTerminal) {  // MCTS_model.py:381-384
          const double tv = (double)rec_tval(cur);
          if (RB && depth < kMaxPath) {
            // backup_path's stores from the N / W this descent loaded, then the root's record
            // and its children's inputs patched the same way
            if (lane <= depth) {
              const int64_t k = nidx(p, half, g, path_node);
              p.a.N[k] = path_n + 1;
              p.a.W[k] = path_w + (((depth - lane) & 1) ? -tv : tv);
            }
            root.visits += 1;
            root.wv = root.wv + ((depth & 1) ? -tv : tv);
            if (depth >= 1) {
              const int j1 = readlane(path_node, 1) - root.first;
              if (lane == j1) {
                kid0.n += 1;
                kid0.w = kid0.w + (((depth - 1) & 1) ? -tv : tv);
              }
            }
            patched = root.first == 1;  // kid0 holds the root's children only then
          } else if (depth < kMaxPath) {
            backup_path(p, g, half, path_node, depth, tv);
          } else if (lane == 0) {
            backup(p, g, half, cur.node, tv);
          }
          // the N/W stores must be visible to the wave's next PUCT loads
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
          ++sims_done;
          break;
        }
        if (!(f & kExpanded)) {  // MCTS_model.py:386-389
          wait_leaf();
          break;
        }
        if constexpr (KMAX == 1) {
          cur = select_child_rec(p, g, half, cur, depth == 0, kid0);
        } else {
          cur = select_child_vl<KMAX>(p, g, half, cur, depth, w, depth == 0, kid0);
        }
        ++depth;
        if (lane == depth) path_node = cur.node;
        if constexpr (RB) {
          if (lane == depth) {
            path_n = cur.visits;
            path_w = cur.wv;
          }
        }
      }
      levels += depth + 1;
    }
  }
  ENG_STAMP(6);
#if AZ_ENG_STAMP
  st_[7] = (unsigned long long)depth;
#endif
  for (int j = w.n; j < K; ++j) {
    emit_none(nn_in, leaf_o, row0 + j);
    if (KMAX > 1 && lane == 0) p.g.leaf[row0 + j] = -1;
  }
  if (p.stem_c) {
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
      if (j < K) emit_stem(p, row0 + j, plane[j]);
  }
  if (lane == 0) {
    if (sims_done != sims0) {
      p.g.sims_acc[g] = acc0 + (unsigned long long)(sims_done - sims0);
      p.g.sims_done[g] = sims_done;
    }
    if (w.n == 0 && sims_done >= target) {
      if (p.auto_play) push_ready(p, g, par, sst);
      else p.g.status[g] = kSearchDone;
    }
    if (deep) {
      p.g.overflow[g] += 1;
      atomicAdd(&p.ctr->overflow, 1ull);
    }
    if constexpr (KMAX > 1) {
      // stopped by the descent cap with fewer than K leaves waiting and simulations left:
      // the batch stays open (expansion skips it; the next select continues it)
      const int op =
          p.auto_play && !root_wait && w.n > 0 && w.n < K && sims_done + w.n < target ? w.n : 0;
      if (op != open0) p.g.open[g] = op;
    }
  }
  ENG_STAMP(3);
#if AZ_ENG_STAMP
  st_[4] = (unsigned long long)w.n;
  st_[5] = (unsigned long long)sims_done;
#endif
  ENG_STAMP_END();
}

// ---------------------------------------------------------------------------------
// k_expand

// MCTS._rollout (MCTS_model.py:276-303): uniformly random playout; value from the leaf
// player's view.
__device__ double rollout(const Params& p, int g, uint64_t own, uint64_t opp) {
  const uint32_t ev = p.g.rng_event[g];
  p.g.rng_event[g] = ev + 1;
  int side = 1;
  for (uint32_t ply = 0; ply < 256; ++ply) {
    uint64_t lg = azb::legal(own, opp);
    int a = azb::kPass;
    if (lg) {
      const double u = azr::uniform1(p.seed, (uint32_t)g, ev, 0x6000u + ply, p.stream_id);
      int j = (int)(u * azb::popc(lg));
      for (int i = 0; i < j; ++i) lg &= lg - 1;
      a = __builtin_ctzll(lg);
    }
    uint64_t no, np_;
    azb::play(own, opp, a, a == azb::kPass ? 0ull : azb::flips(own, opp, a), &no, &np_);
    own = no;
    opp = np_;
    side = -side;
    if (azb::terminal_flags(own, opp, azb::legal(own, opp)) & azb::kFlagTerminal) {
      const int d = (azb::popc(own) - azb::popc(opp)) * side;
      return d > 0 ? 1.0 : (d < 0 ? -1.0 : 0.0);
    }
  }
  return 0.0;
}

// One waiting leaf (row `row` of the evaluation batch): evaluate, expand and back up
// (MCTS_model.py:325-360).  `repeat`: an earlier descent of this step waits on the same
// leaf -- it is expanded already and this descent only backs up that descent's value `v_in`
// (two reference workers on one leaf both expand it, the second with identical fresh
// children, and both back up).  Returns the value backed up.
// What a waiting leaf's expansion reads that does not depend on the tree: loaded for every
// leaf of the slot in the kernel's first round trip.
struct LeafIn {
  int leaf, plen, pn;  // node, recorded path length, lane's path entry
  float pr, pr64, v;   // evaluation row: this lane's prior (row order), prior 64, value
  int sym;             // D4 transform the leaf was packed through
};

__device__ __forceinline__ LeafIn load_leaf_in(const Params& p, int64_t row,
                                               const float* __restrict__ priors,
                                               const float* __restrict__ values) {
  const int lane = lane_id();
  LeafIn in;
  in.leaf = p.g.leaf[row];
  in.plen = p.g.path_len[row];
  in.pn = p.g.path[row * kMaxPath + lane];
  // (rollout mode: the host passes a zeroed stand-in buffer, so the loads need no branch)
  in.pr = priors[row * 65 + lane];
  in.pr64 = priors[row * 65 + 64];
  in.v = values[row];
  in.sym = p.g.sym[row];  // meaningful only with p.d4 (the caller masks it)
  return in;
}

// n_nodes: the slot's allocation cursor, carried in a register across the step's leaves
// (lane-uniform) and stored once by the caller.
__device__ double expand_backup_leaf(const Params& p, int g, int half, const LeafIn& in,
                                     int& n_nodes, bool repeat, double v_in) {
  const int leaf = in.leaf, plen = in.plen, pn = in.pn;
  const int lane = lane_id();
  const int64_t k = nidx(p, half, g, leaf);
  const uint64_t own = p.a.own[k], opp = p.a.opp[k], lg = p.a.legal[k];
  const bool is_root = leaf == 0;
  // the path's N / W with the leaf's record (nothing here writes them before the backup)
  const bool on_path = plen > 0 && lane < plen;
  int path_n = 0;
  double path_w = 0.0;
  if (on_path) {
    const int64_t pk = nidx(p, half, g, pn);
    path_n = p.a.N[pk];
    path_w = p.a.W[pk];
  }
  double v = v_in;
  if (!repeat) {
    // ---- priors and value (MCTS_model.py:332-337)
    float pr, pr64;
    if (p.eval_mode == AZ_EVAL_ROLLOUT) {
      pr = 1.0f;
      pr64 = 1.0f;
      double vv = 0.0;
      if (lane == 0) vv = rollout(p, g, own, opp);
      v = readlane(vv, 0);
    } else {
      // unsymmetrise_pi (MCTS_model.py:31-43): the net saw the board through `sym`, so
      // lane a takes the row entry of square d4(a)
      pr = in.sym ? __shfl(in.pr, azb::d4_square(lane, in.sym), kWave) : in.pr;
      pr64 = in.pr64;
      v = (double)in.v;
    }
    const bool valid = lg ? ((lg >> lane) & 1) != 0 : false;
    const bool valid64 = lg == 0;

    // ---- noise, mask, renormalise (MCTS_model.py:340-349)
    const bool noise = is_root && p.eps > 0.0;
    double P, P64;
    if (noise) {
      double n, n64;
      if (p.rng_mode == AZ_RNG_INJECTED) {
        const int cur = p.g.noise_cur[g];
        const double* src = p.inj_noise + ((int64_t)g * p.NS + (cur < p.NS ? cur : p.NS - 1)) * 65;
        n = src[lane];
        n64 = src[64];
        if (lane == 0) p.g.noise_cur[g] = cur + 1;
      } else {
        const uint32_t ev = p.g.rng_event[g];
        const double ga = azr::gamma_draw(p.alpha, p.seed, (uint32_t)g, ev, (uint32_t)lane, p.stream_id);
        const double ga64 = azr::gamma_draw(p.alpha, p.seed, (uint32_t)g, ev, 64u, p.stream_id);
        double s = ga;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
        s += ga64;
        n = ga / s;
        n64 = ga64 / s;
        if (lane == 0) p.g.rng_event[g] = ev + 1;
      }
      // (1 - eps) * priors is float32 (Python float x float32 array); + eps * noise is float64
      const float keep = (float)(1.0 - p.eps);
      P = (double)(keep * pr) + p.eps * n;
      P64 = (double)(keep * pr64) + p.eps * n64;
      P = valid ? P : 0.0 * P;  // priors *= valid_mask
      P64 = valid64 ? P64 : 0.0 * P64;
      const double tot = np_sum65<double>(P, P64);
      if (tot > 1e-12) {
        P = P / tot;
        P64 = P64 / tot;
      }
    } else {
      float q = valid ? pr : 0.0f * pr;
      float q64 = valid64 ? pr64 : 0.0f * pr64;
      const float tot = np_sum65<float>(q, q64);
      if (tot > (float)1e-12) {
        q = q / tot;
        q64 = q64 / tot;
      }
      P = (double)q;
      P64 = (double)q64;
    }

    // ---- eager expansion of every legal child (MCTS_model.py:352-357, :146-158)
    const int nc = lg ? azb::popc(lg) : 1;
    int fc = n_nodes;
    if (fc + nc <= p.C) {
      n_nodes = fc + nc;
    } else {
      fc = -1;
      if (lane == 0) {
        p.g.overflow[g] += 1;
        atomicAdd(&p.ctr->overflow, 1ull);
      }
    }
    if (fc >= 0) {
      const bool mine = lg ? valid : (lane == 0);
      const int a = lg ? lane : azb::kPass;
      uint64_t co = 0, cp = 0, clg = 0;
      if (mine) {
        azb::play(own, opp, a, lg ? azb::flips(own, opp, a) : 0ull, &co, &cp);
        clg = azb::legal(co, cp);
      }
      // terminal check of every child, wave-cooperative for the rare real passes
      int tf = azb::terminal_flags_wave(co, cp, clg, mine);
      tf = azb::finish_terminal_wave(tf, co, cp);
      if (mine) {
        const int ci = lg ? azb::popc(lg & ((1ull << lane) - 1ull)) : 0;
        const bool term = (tf & azb::kFlagTerminal) != 0;
        const int d = azb::popc(co) - azb::popc(cp);
        const int64_t c = nidx(p, half, g, fc + ci);
        p.a.own[c] = co;
        p.a.opp[c] = cp;
        p.a.legal[c] = clg;
        p.a.N[c] = 0;
        p.a.W[c] = 0.0;
        p.a.P[c] = lg ? P : P64;
        p.a.parent[c] = leaf;
        p.a.first[c] = -1;
        p.a.nchild[c] = 0;
        p.a.action[c] = (uint8_t)a;
        p.a.flags[c] = term ? kTerminal : 0;
        p.a.tval[c] = (int8_t)(term ? (d > 0 ? 1 : (d < 0 ? -1 : 0)) : 0);
      }
      if (lane == 0) {
        p.a.first[k] = fc;
        p.a.nchild[k] = (uint8_t)nc;
        p.a.flags[k] = p.a.flags[k] | kExpanded | (noise ? kChildF64 : 0);
      }
    }
  }
  // backup (MCTS_model.py:360) along the path k_select recorded (backup_path's update on
  // the values loaded above)
  if (on_path) {
    const int64_t pk = nidx(p, half, g, pn);
    p.a.N[pk] = path_n + 1;
    p.a.W[pk] = path_w + (((plen - 1 - lane) & 1) ? -v : v);
  } else if (plen == 0 && lane == 0) {
    backup(p, g, half, leaf, v);
  }
  return v;
}

// The expansion of slot g's waiting leaves in descent order (rows g*K .. g*K+K-1 of the
// evaluation batch, the list ends at the first -1): k_expand's body, also run by the slot's
// wave at the start of the next select launch (fused expansion, az_select_move_expand).
// Returns whether the slot's search is complete after them (then pushed to move list `par`
// with step sst_push; -1 = this launch's step count minus one, the standalone kernel's).
template <int KMAX>
__device__ __forceinline__ bool expand_slot(const Params& p, int g,
                                            const float* __restrict__ priors,
                                            const float* __restrict__ values, int par,
                                            int sst_push) {
  const int K = KMAX == 1 ? 1 : p.K;
  const int64_t row0 = (int64_t)g * K;
  const int lane = lane_id();
  // one round trip for everything that does not depend on the tree: the slot's words and,
  // for every waiting leaf, its recorded path and evaluation row (the rows are valid memory
  // whatever they hold; they are used only for leaves that wait)
  const int half = p.g.half[g];
  int n_nodes = p.g.n_nodes[g];
  const int sd0 = p.g.sims_done[g], target = p.g.sims_target[g];
  const int open = KMAX > 1 ? p.g.open[g] : 0;
  LeafIn in[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j)
    if (j < K) in[j] = load_leaf_in(p, row0 + j, priors, values);
  // every load above in flight before any is waited for (the compiler would otherwise sink
  // them past the early exit below, one dependent round trip each)
  asm volatile("" ::"v"(half), "v"(n_nodes), "v"(sd0), "v"(target), "v"(open));
#pragma unroll
  for (int j = 0; j < KMAX; ++j)
    if (j < K)
      asm volatile("" ::"v"(in[j].leaf), "v"(in[j].plen), "v"(in[j].pn), "v"(in[j].pr),
                   "v"(in[j].pr64), "v"(in[j].v), "v"(in[j].sym));
#pragma unroll
  for (int j = 0; j < KMAX; ++j) in[j].sym = p.d4 ? in[j].sym : 0;
  // a batch the last select left open (its descent cap) waits for more leaves: the next
  // select continues it, and its leaves are expanded once it closes
  if (in[0].leaf < 0 || open > 0) return false;
  double done_v[KMAX];
  int n_sims = 0;
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    if (j >= K || in[j].leaf < 0) break;
    const int leaf = in[j].leaf;
    // a leaf an earlier descent of this step waits on too: expanded already, this descent
    // only backs up that value
    bool repeat = false;
    double v_in = 0.0;
#pragma unroll
    for (int jj = 0; jj < j; ++jj)
      if (!repeat && in[jj].leaf == leaf) {
        repeat = true;
        v_in = done_v[jj];
      }
    done_v[j] = expand_backup_leaf(p, g, half, in[j], n_nodes, repeat, v_in);
    if (leaf != 0) ++n_sims;  // the search-start root expansion is not one of the simulations
    // the next leaf's path loads must see this backup's N/W stores
    if (KMAX > 1) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
  const int sd = sd0 + n_sims;
  if (lane == 0) {
    p.g.leaf[row0] = -1;
    p.g.n_nodes[g] = n_nodes;
    if (n_sims) {
      p.g.sims_done[g] = sd;
      p.g.sims_acc[g] += (unsigned long long)n_sims;
    }
    if (sd >= target) {
      if (p.auto_play)
        push_ready(p, g, par, sst_push >= 0 ? sst_push : (p.defer ? p.g.sstep[g] - 1 : 0));
      else
        p.g.status[g] = kSearchDone;
    }
  }
  return sd >= target;
}

// One wavefront per slot: expand_slot.
template <int KMAX>
__global__ __launch_bounds__(kSelBlock) void k_expand(Params p, const float* __restrict__ priors,
                                                      const float* __restrict__ values,
                                                      int par) {
  const int g = blockIdx.x * (kSelBlock / kWave) + (threadIdx.x >> 6);
  if (g >= p.G) return;
  ENG_STAMP_BEGIN(2);
  expand_slot<KMAX>(p, g, priors, values, par, -1);
  ENG_STAMP(3);
  ENG_STAMP_END();
}

// ---------------------------------------------------------------------------------
// pi from the root's visit counts (MCTS.policy_improve_step, MCTS_model.py:244-271).
// Wave-level; lane a holds pi[a] on return, lane 0 additionally *pi64.
__device__ float root_pi(const Params& p, int g, int half, double temp, double u_tie,
                         float* pi64) {
  const int lane = lane_id();
  const int64_t r = nidx(p, half, g, 0);
  const int nc = p.a.nchild[r], fc = p.a.first[r];
  const uint64_t lg = p.a.legal[r];
  // counts[a] = child visit count (float32).  The children are every legal action in
  // ascending order (or the single pass): lane j reads child j, lane a gathers from the
  // lane holding its action's rank in the legal mask.
  float c = 0.0f, c64 = 0.0f;
  if (nc > 0) {
    float cnt = 0.0f;
    if (lane < nc) cnt = (float)p.a.N[nidx(p, half, g, fc + lane)];
    const int src = lg ? azb::popc(lg & ((1ull << lane) - 1ull)) : 0;
    const float cj = shfl(cnt, src);
    if (lg) c = ((lg >> lane) & 1) ? cj : 0.0f;
    else c64 = cj;
  }
  float pi, p64;
  if (fabs(temp) < 1e-1) {
    float m = fmaxf(c, c64);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, kWave));
    const uint64_t ties = ballot(c == m);
    const int k = azb::popc(ties) + (c64 == m ? 1 : 0);
    int j = (int)(u_tie * (double)k);
    j = j < 0 ? 0 : (j >= k ? k - 1 : j);
    int best = 64;
    if (j < azb::popc(ties)) {
      uint64_t t = ties;
      for (int i = 0; i < j; ++i) t &= t - 1;
      best = __builtin_ctzll(t);
    }
    const bool any = nc > 0;  // `if len(self.root.valid_actions) != 0`
    pi = (any && best == lane) ? 1.0f : 0.0f;
    p64 = (any && best == 64) ? 1.0f : 0.0f;
  } else {
    const float ex = (float)(1.0 / temp);
    const float ce = temp == 1.0 ? c : powf(c, ex);
    const float ce64 = temp == 1.0 ? c64 : powf(c64, ex);
    const float norm = np_sum65<float>(ce, ce64);
    if (norm < (float)1e-12) {
      // uniform over the root's valid actions (the children)
      const float u = nc > 0 ? (float)(1.0 / (double)nc) : 0.0f;
      pi = (lg >> lane) & 1 ? u : 0.0f;
      p64 = lg == 0 ? u : 0.0f;
    } else {
      pi = ce / norm;
      p64 = ce64 / norm;
    }
  }
  *pi64 = p64;
  return pi;
}

// root_pi on a root record already in registers: nc / legal of the root, `cnt` = this
// lane's child visit count (lane j = child j) -- the same arithmetic as root_pi.
__device__ float root_pi_pre(int nc, uint64_t lg, int cnt_lane, double temp, double u_tie,
                             float* pi64) {
  const int lane = lane_id();
  float c = 0.0f, c64 = 0.0f;
  if (nc > 0) {
    const float cnt = lane < nc ? (float)cnt_lane : 0.0f;
    const int src = lg ? azb::popc(lg & ((1ull << lane) - 1ull)) : 0;
    const float cj = shfl(cnt, src);
    if (lg) c = ((lg >> lane) & 1) ? cj : 0.0f;
    else c64 = cj;
  }
  float pi, p64;
  if (fabs(temp) < 1e-1) {
    float m = fmaxf(c, c64);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, kWave));
    const uint64_t ties = ballot(c == m);
    const int k = azb::popc(ties) + (c64 == m ? 1 : 0);
    int j = (int)(u_tie * (double)k);
    j = j < 0 ? 0 : (j >= k ? k - 1 : j);
    int best = 64;
    if (j < azb::popc(ties)) {
      uint64_t t = ties;
      for (int i = 0; i < j; ++i) t &= t - 1;
      best = __builtin_ctzll(t);
    }
    const bool any = nc > 0;  // `if len(self.root.valid_actions) != 0`
    pi = (any && best == lane) ? 1.0f : 0.0f;
    p64 = (any && best == 64) ? 1.0f : 0.0f;
  } else {
    const float ex = (float)(1.0 / temp);
    const float ce = temp == 1.0 ? c : powf(c, ex);
    const float ce64 = temp == 1.0 ? c64 : powf(c64, ex);
    const float norm = np_sum65<float>(ce, ce64);
    if (norm < (float)1e-12) {
      const float u = nc > 0 ? (float)(1.0 / (double)nc) : 0.0f;
      pi = (lg >> lane) & 1 ? u : 0.0f;
      p64 = lg == 0 ? u : 0.0f;
    } else {
      pi = ce / norm;
      p64 = ce64 / norm;
    }
  }
  *pi64 = p64;
  return pi;
}

// np.random.choice(65, p=pi) given its uniform draw u: cdf = cumsum(float64(pi)) (sequential),
// cdf /= cdf[-1], searchsorted(u, side='right').  Whole wave: lane 0 forms the sequential
// partial sums (NumPy's cumsum order) into `cdf` (LDS, 65 doubles), then every lane divides
// and compares its own entry at once -- the cdf is non-decreasing (pi >= 0) and the
// correctly rounded division is monotone, so the entries <= u are a prefix and the answer is
// their count (all-zero pi: 0/0 compares false everywhere, as in NumPy's loop).
__device__ int sample_action(const float* pis, double u, double* cdf) {
  const int lane = lane_id();
  if (lane == 0) {
    double acc = 0.0;
    for (int a = 0; a < 65; ++a) {
      acc = acc + (double)pis[a];
      cdf[a] = acc;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
  const double last = cdf[64];
  const bool le = cdf[lane] / last <= u;
  const bool le64 = cdf[64] / last <= u;
  const int idx = azb::popc(ballot(le)) + (le64 ? 1 : 0);
  return idx > 64 ? 64 : idx;
}

// Re-root compaction: copy the subtree under old node `child` into the other arena half,
// making it node 0.  Nodes keep their relative arena order (a stable stream compaction):
// every node's parent and every sibling group's allocation precede its own, so `child` maps
// to 0 and each sibling group -- allocated as one block -- stays contiguous and ascending,
// which is all the descent relies on (the oracle's BFS order, oracle/mcts.py make_move,
// yields the same tree).  Membership is found by pointer jumping on the parent links in LDS
// instead of a level-by-level BFS: a handful of global round trips per re-root, not two per
// tree level.  Whole workgroup; `scratch` = LDS of p.C ints, used as two u16 arrays (node
// offsets from `child` are < p.C <= 32768, 0xffff = not in the subtree).
__device__ int compact(const Params& p, int g, int child, int32_t* scratch, int oh,
                       int n_nodes) {
  constexpr uint16_t kOut = 0xffff;
  constexpr int kU = 8;   // LDS link reads in flight per thread (pointer jumping)
  constexpr int kP = 32;  // parent loads in flight per thread (one round trip per 8,192 nodes)
  __shared__ int s_scan[kMoveBlock / kWave];
  uint16_t* rel = reinterpret_cast<uint16_t*>(scratch);  // old offset -> link, then new index
  uint16_t* inv = rel + p.C;                             // new index -> old offset
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int nh = oh ^ 1;
  const int span = n_nodes - child;  // candidates: old nodes child .. n_nodes-1
  CST(0);
  // 1. rel[j] = parent of old node child+j as an offset from `child` (descendants of `child`
  // all lie above it; a parent below it means "not in the subtree")
  for (int j0 = 0; j0 < span; j0 += kMoveBlock * kP) {
    int par[kP];
#pragma unroll
    for (int u = 0; u < kP; ++u) {
      const int j = j0 + u * kMoveBlock + tid;
      par[u] = (j > 0 && j < span) ? p.a.parent[nidx(p, oh, g, child + j)] : child;
    }
#pragma unroll
    for (int u = 0; u < kP; ++u) {
      const int j = j0 + u * kMoveBlock + tid;
      if (j < span) rel[j] = par[u] >= child ? (uint16_t)(par[u] - child) : kOut;
    }
  }
  __syncthreads();
  CST(1);
  // 2. pointer jumping until every link is 0 (member) or kOut; in-place updates only ever
  // replace a link by one of its ancestors' links.  Each round jumps twice, and a thread
  // keeps kU independent LDS reads in flight (the loop is LDS-latency-bound otherwise).
  auto interior = [](uint16_t v) { return v != 0 && v != kOut; };
  for (;;) {
    int more = 0;
    for (int j0 = tid; j0 < span; j0 += kMoveBlock * kU) {
      uint16_t a[kU], b[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int j = j0 + u * kMoveBlock;
        a[u] = j < span ? rel[j] : (uint16_t)0;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) b[u] = interior(a[u]) ? rel[a[u]] : a[u];
#pragma unroll
      for (int u = 0; u < kU; ++u) b[u] = interior(b[u]) ? rel[b[u]] : b[u];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int j = j0 + u * kMoveBlock;
        if (j < span && b[u] != a[u]) rel[j] = b[u];
        more |= interior(b[u]);
      }
    }
    if (!__syncthreads_or(more)) break;
  }
  CST(2);
  // 3. new index = rank among members (block exclusive scan over contiguous thread ranges of
  // a multiple of 8 links, read 16 bytes at a time; entries past `span` are masked)
  const int per = (((span + kMoveBlock - 1) / kMoveBlock) + 7) & ~7;
  const int j0 = tid * per, j1 = min(j0 + per, span);
  int cnt = 0;
  for (int j = j0; j < j1; j += 8) {
    const uint4 v = *reinterpret_cast<const uint4*>(rel + j);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 8; ++k)
      cnt += (j + k < j1 && ((w[k >> 1] >> (16 * (k & 1))) & 0xffffu) == 0) ? 1 : 0;
  }
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(incl, off, kWave);
    if (lane >= off) incl += y;
  }
  if (lane == 63) s_scan[wave] = incl;
  __syncthreads();
  int base = 0, n_new = 0;
  for (int w = 0; w < kMoveBlock / kWave; ++w) {
    if (w < wave) base += s_scan[w];
    n_new += s_scan[w];
  }
  int r = base + incl - cnt;
  for (int j = j0; j < j1; j += 8) {
    const uint4 v = *reinterpret_cast<const uint4*>(rel + j);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool member = ((w[k >> 1] >> (16 * (k & 1))) & 0xffffu) == 0;
      uint32_t nv = kOut;
      if (j + k < j1 && member) {
        inv[r] = (uint16_t)(j + k);
        nv = (uint32_t)r++;
      }
      o[k >> 1] |= (nv & 0xffffu) << (16 * (k & 1));
    }
    // whole 16-byte group written back: links past j1 belong to the next thread's range
    // (or lie past `span`), so only the valid ones are stored
    if (j + 8 <= j1) {
      *reinterpret_cast<uint4*>(rel + j) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (j + k < j1) rel[j + k] = (uint16_t)((o[k >> 1] >> (16 * (k & 1))) & 0xffffu);
    }
  }
  __syncthreads();
  CST(3);
  // 4. copy the members, translating parent / first-child links: kC nodes per thread with
  // every load issued before the first store (one global round trip per kC * block nodes
  // instead of one per block of nodes)
  constexpr int kC = AZ_MOVE_KC;  // 4 (default); experiment builds -DAZ_MOVE_KC=8
  for (int i0 = tid; i0 < n_new; i0 += kMoveBlock * kC) {
    uint64_t own[kC], opp[kC], lg[kC];
    double W[kC], P[kC];
    int N[kC], par[kC], fc[kC];
    uint8_t act[kC], fl[kC], tv[kC], nch[kC];
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      const int i = i0 + u * kMoveBlock;
      if (i < n_new) {
        const int64_t ok = nidx(p, oh, g, child + inv[i]);
        own[u] = p.a.own[ok];
        opp[u] = p.a.opp[ok];
        lg[u] = p.a.legal[ok];
        N[u] = p.a.N[ok];
        W[u] = p.a.W[ok];
        P[u] = p.a.P[ok];
        act[u] = p.a.action[ok];
        fl[u] = p.a.flags[ok];
        tv[u] = p.a.tval[ok];
        nch[u] = p.a.nchild[ok];
        par[u] = p.a.parent[ok];
        fc[u] = p.a.first[ok];
      }
    }
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      const int i = i0 + u * kMoveBlock;
      if (i < n_new) {
        const int64_t nk = nidx(p, nh, g, i);
        const bool ex = (fl[u] & kExpanded) != 0;
        p.a.own[nk] = own[u];
        p.a.opp[nk] = opp[u];
        p.a.legal[nk] = lg[u];
        p.a.N[nk] = N[u];
        p.a.W[nk] = W[u];
        p.a.P[nk] = P[u];
        p.a.action[nk] = act[u];
        p.a.flags[nk] = fl[u];
        p.a.tval[nk] = tv[u];
        p.a.nchild[nk] = ex ? nch[u] : (uint8_t)0;
        p.a.first[nk] = ex ? (int)rel[fc[u] - child] : -1;
        p.a.parent[nk] = i == 0 ? -1 : (int)rel[par[u] - child];
      }
    }
  }
  if (tid == 0) {
    p.g.half[g] = nh;
    p.g.n_nodes[g] = n_new;
  }
  __syncthreads();
  return n_new;
}

__device__ double next_uniform(const Params& p, int g, uint32_t sub) {
  if (p.rng_mode == AZ_RNG_INJECTED) {
    const int cur = p.g.u_cur[g];
    p.g.u_cur[g] = cur + 1;
    return cur < p.NU ? p.inj_u[(int64_t)g * p.NU + cur] : 0.5;
  }
  const uint32_t ev = p.g.rng_event[g];
  p.g.rng_event[g] = ev + 1;
  return azr::uniform1(p.seed, (uint32_t)g, ev, sub, p.stream_id);
}

__device__ void new_game(const Params& p, int g) {
  const int half = p.g.half[g];
  init_root(p, g, half, azb::kInitOwn, azb::kInitOpp);
  p.g.n_nodes[g] = 1;
  p.g.ply[g] = 0;
  p.g.root_player[g] = 1;
  p.g.winner[g] = 0;
  p.g.sims_done[g] = 0;
  p.g.sims_target[g] = p.sims;
  p.g.leaf[(int64_t)g * p.K] = -1;
  p.g.open[g] = 0;
  p.g.status[g] = kActive;
}

// get_training_data (self_play_worker.py:8-35) + append to the sample buffer.
__device__ void finish_game(const Params& p, int g, int n_plies, int winner, int32_t* scratch) {
  __shared__ unsigned long long s_base;
  __shared__ int s_ok;
  const int tid = threadIdx.x;
  const int64_t tb = (int64_t)g * p.T;
  // the return chain below is sequential: stage its inputs in LDS with one parallel load
  // (scratch = the caller's p.C-int LDS block) instead of two dependent loads per ply
  double* s_vr = reinterpret_cast<double*>(scratch);
  int8_t* s_pl = reinterpret_cast<int8_t*>(s_vr + n_plies);
  const bool staged = n_plies * 9 <= p.C * 4;
  if (staged) {
    for (int t = tid; t < n_plies; t += blockDim.x) {
      s_vr[t] = p.g.t_vroot[tb + t];
      s_pl[t] = p.g.t_player[tb + t];
    }
    __syncthreads();
  }
  if (tid == 0) {
    // reserve [base, base + n_plies) only if it fits: the counter advances by a successful
    // compare-and-swap and is never rolled back, so a rejected game cannot lower it under
    // rows another workgroup has already reserved
    unsigned long long base = __hip_atomic_load(&p.ctr->samples_n, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    s_ok = 0;
    while ((int64_t)(base + n_plies) <= p.s.cap) {
      const unsigned long long prev = atomicCAS(&p.ctr->samples_n, base, base + n_plies);
      if (prev == base) {
        s_ok = 1;
        break;
      }
      base = prev;
    }
    if (!s_ok) atomicAdd(&p.ctr->samples_dropped, (unsigned long long)n_plies);
    s_base = base;
    if (s_ok) {
      double g_next = 0.0;
      int p_next = 0;
      for (int t = n_plies - 1; t >= 0; --t) {
        const int pl = staged ? s_pl[t] : p.g.t_player[tb + t];
        const double z = winner == 0 ? 0.0 : (pl == winner ? 1.0 : -1.0);
        double gt;
        if (t == n_plies - 1) {
          gt = z;
        } else {
          const double sign = pl == p_next ? 1.0 : -1.0;
          const double vr = staged ? s_vr[t] : p.g.t_vroot[tb + t];
          gt = (1.0 - p.lambd) * vr + p.lambd * sign * g_next;
        }
        p.s.z[base + t] = gt;
        g_next = gt;
        p_next = pl;
      }
    }
  }
  __syncthreads();
  if (s_ok) {
    const unsigned long long base = s_base;
    for (int t = tid; t < n_plies; t += blockDim.x) {
      p.s.own[base + t] = p.g.t_own[tb + t];
      p.s.opp[base + t] = p.g.t_opp[tb + t];
      p.s.player[base + t] = p.g.t_player[tb + t];
      p.s.slot[base + t] = g;
    }
    constexpr int kU = 8;  // loads in flight per thread
    const int ne = n_plies * 65;
    for (int e0 = 0; e0 < ne; e0 += kMoveBlock * kU) {
      float v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + u * kMoveBlock + tid;
        v[u] = e < ne ? p.g.t_pi[tb * 65 + e] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + u * kMoveBlock + tid;
        if (e < ne) p.s.pi[base * 65 + e] = v[u];
      }
    }
  }
  __syncthreads();
}

// k_move: one workgroup per slot in the ready list.
// The move phase on work list q by `nblocks` workgroups (this one: bid).  deferred: called
// from k_select's extra workgroups for the previous step's list, beside that step's
// descents; the step counter is then advanced but nothing in that launch reads it.
__device__ __forceinline__ void move_body(const Params& p, int q, int deferred, int nblocks,
                                          int bid) {
  extern __shared__ __align__(16) int32_t map[];
  __shared__ float s_pi[65];
  __shared__ double s_cdf[65];
  __shared__ int s_child, s_term, s_winner, s_restart;
  const int tid = threadIdx.x;
  const int n_ready = p.ctr->ready_n[q];
  for (int ri = bid; ri < n_ready; ri += nblocks) {
    ENG_STAMP_BEGIN(1);
    const int g = p.ready[q * p.G + ri];
    const int half = p.g.half[g];
    const int ply = p.g.ply[g];
    const int player = p.g.root_player[g];
    const int n_nodes = p.g.n_nodes[g];
    if (tid < 64) {
      // ---- one round trip for the root record, the children's records (lane j = child j,
      // nodes 1 + j: load_root) and the slot's RNG cursor; everything after works from
      // registers
      const int64_t r = nidx(p, half, g, 0);
      const int64_t ck = nidx(p, half, g, 1 + tid);
      int c_n = p.a.N[ck], c_flags = p.a.flags[ck];
      uint64_t c_own = p.a.own[ck], c_opp = p.a.opp[ck];
      const int nc = p.a.nchild[r], fc = p.a.first[r];
      const uint64_t lg = p.a.legal[r], r_own = p.a.own[r], r_opp = p.a.opp[r];
      const int r_n = p.a.N[r];
      const double r_w = p.a.W[r];
      const bool injected = p.rng_mode == AZ_RNG_INJECTED;
      const uint32_t rng0 = injected ? (uint32_t)p.g.u_cur[g] : p.g.rng_event[g];
      if (fc != 1 && tid < nc) {  // not reached (see load_root); kept for safety
        const int64_t ck2 = nidx(p, half, g, fc + tid);
        c_n = p.a.N[ck2];
        c_flags = p.a.flags[ck2];
        c_own = p.a.own[ck2];
        c_opp = p.a.opp[ck2];
      }
      if (tid >= nc) {
        c_n = 0;
        c_flags = 0;
        c_own = c_opp = 0;
      }
      // ---- the move's uniform draws (next_uniform, in draw order): the tie-break draw
      // when temp < 0.1, then the action sample
      const double temp = ply < p.n_explore ? p.temp : 0.0;
      const bool tie_draw = fabs(temp) < 1e-1;
      double u_tie = 0.0, u_act = 0.0;
      if (tid == 0) {
        auto draw = [&](uint32_t i, uint32_t sub) -> double {
          if (injected) {
            const uint32_t cur = rng0 + i;
            return cur < (uint32_t)p.NU ? p.inj_u[(int64_t)g * p.NU + cur] : 0.5;
          }
          return azr::uniform1(p.seed, (uint32_t)g, rng0 + i, sub, p.stream_id);
        };
        if (tie_draw) u_tie = draw(0, 0x1000u);
        u_act = draw(tie_draw ? 1 : 0, 0x2000u);
        const uint32_t used = tie_draw ? 2u : 1u;
        if (injected) p.g.u_cur[g] = (int)(rng0 + used);
        else p.g.rng_event[g] = rng0 + used;
      }
      u_tie = readlane(u_tie, 0);
      // ---- pi (MCTS_model.py:244-271) and trajectory record (self_play_worker.py:72-73)
      float p64;
      const float pi = root_pi_pre(nc, lg, c_n, temp, u_tie, &p64);
      s_pi[tid] = pi;
      if (tid == 0) s_pi[64] = p64;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      __builtin_amdgcn_wave_barrier();
      const bool room = ply < p.T;
      if (room) p.g.t_pi[((int64_t)g * p.T + ply) * 65 + tid] = pi;
      // ---- action sample (self_play_worker.py:75) and the chosen child (MCTS.make_move,
      // MCTS_model.py:200-215): the children are every legal action in ascending order (or
      // the single pass), so the child's index follows from the root's legal mask
      const int a = sample_action(s_pi, readlane(u_act, 0), s_cdf);
      int jc = -1;
      if (tid == 0) {
        if (room) {
          p.g.t_pi[((int64_t)g * p.T + ply) * 65 + 64] = p64;
          p.g.t_own[(int64_t)g * p.T + ply] = r_own;
          p.g.t_opp[(int64_t)g * p.T + ply] = r_opp;
          p.g.t_player[(int64_t)g * p.T + ply] = (int8_t)player;
          p.g.t_vroot[(int64_t)g * p.T + ply] = r_n == 0 ? 0.0 : r_w / (double)r_n;
        }
        if (nc > 0) {
          if (lg) {
            if (a < 64 && ((lg >> a) & 1)) jc = azb::popc(lg & ((1ull << a) - 1ull));
          } else if (a == azb::kPass) {
            jc = 0;
          }
        }
      }
      jc = readlane(jc, 0);
      const int src = jc >= 0 ? jc : 0;
      const int ch_flags = readlane(c_flags, src);
      const uint64_t ch_own = readlane(c_own, src), ch_opp = readlane(c_opp, src);
      if (tid == 0) {
        s_child = jc >= 0 ? fc + jc : -1;
        int term = 1, winner = 0;
        if (jc >= 0) {
          // get_value_and_terminated from the mover's view (self_play_worker.py:77-86)
          term = (ch_flags & kTerminal) ? 1 : 0;
          const int d = azb::popc(ch_opp) - azb::popc(ch_own);
          winner = d > 0 ? player : (d < 0 ? -player : 0);
        }
        if (!room) term = 1;  // trajectory capacity exhausted (never at T >= 128)
        s_term = term;
        s_winner = winner;
        atomicAdd(&p.ctr->moves, 1ull);
      }
    }
    __syncthreads();
    ENG_STAMP(2);
    if (s_term) {
      const int n_plies = ply + 1 < p.T ? ply + 1 : p.T;
      finish_game(p, g, n_plies, s_winner, map);
      if (tid == 0) {
        p.g.winner[g] = s_winner;
        atomicAdd(&p.ctr->games_finished, 1ull);
        int restart = 0;
        if (p.refill) {
          if (p.ctr->unlimited) {
            restart = 1;
          } else {
            unsigned long long* b = (unsigned long long*)&p.ctr->start_budget;
            const long long prev = (long long)atomicAdd(b, (unsigned long long)(-1ll));
            if (prev > 0) restart = 1;
            else atomicAdd(b, 1ull);
          }
        }
        s_restart = restart;
        if (restart) {
          atomicAdd(&p.ctr->games_started, 1ull);
          p.g.status[g] = kActive;
        } else {
          p.g.status[g] = kFinished;
        }
      }
      __syncthreads();
      if (s_restart && tid == 0) new_game(p, g);
    } else {
      compact(p, g, s_child, map, half, n_nodes);
      if (tid == 0) {
        p.g.ply[g] = ply + 1;
        p.g.root_player[g] = -player;
        p.g.sims_done[g] = 0;
        p.g.sims_target[g] = p.sims;
      }
#if AZ_ENG_STAMP
      for (int i = 0; i < 4; ++i) st_[3 + i] = g_cst[i];
#endif
    }
    __syncthreads();
    ENG_STAMP(7);
    if (threadIdx.x < 64) ENG_STAMP_END();
  }
  __syncthreads();
  // the last workgroup to finish (every workgroup has read ready_n by then) clears the
  // work list for the next step and advances the step counter: no separate memset launch
  if (tid == 0) {
    __threadfence();
    if (atomicAdd(&p.ctr->move_done, 1) == nblocks - 1) {
      p.ctr->ready_n[q] = 0;
      p.ctr->move_done = 0;
      p.ctr->step += 1;
      __threadfence();
    }
  }
  (void)deferred;
}

__global__ __launch_bounds__(kMoveBlock) void k_move(Params p) {
  move_body(p, 0, 0, (int)gridDim.x, (int)blockIdx.x);
}

// ctr->sims = sum of the slots' counters (one workgroup; az_counters only)
__global__ __launch_bounds__(1024) void k_sum_sims(Params p) {
  __shared__ unsigned long long s_part[1024 / kWave];
  unsigned long long v = 0;
  for (int g = threadIdx.x; g < p.G; g += blockDim.x) v += p.g.sims_acc[g];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < (int)(blockDim.x / kWave); ++w) t += s_part[w];
    p.ctr->sims = t;
  }
}

// step counter for engines without auto-play (k_move not launched)
__global__ void k_tick(Counters* c) { c->step += 1; }

// ---------------------------------------------------------------------------------
// host-driven (MCTS API) kernels

__global__ void k_reset(Params p, long long budget, int stagger) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g == 0) {
    p.ctr->games_started = 0;
    p.ctr->games_finished = 0;
    p.ctr->samples_n = 0;
    p.ctr->samples_dropped = 0;
    p.ctr->overflow = 0;
    p.ctr->step = 0;
    p.ctr->sims = 0;
    p.ctr->moves = 0;
    p.ctr->ready_n[0] = 0;
    p.ctr->ready_n[1] = 0;
    p.ctr->move_done = 0;
  }
  if (g >= p.G) return;
  p.g.sstep[g] = 0;
  p.g.moving[g] = -2;
  p.g.half[g] = 0;
  p.g.overflow[g] = 0;
  p.g.sims_acc[g] = 0;
  p.g.rng_event[g] = 0;
  p.g.noise_cur[g] = 0;
  p.g.u_cur[g] = 0;
  p.g.sym[g] = 0;
  p.g.start_step[g] = stagger > 0 ? (int)((long long)g * stagger / p.G) : 0;
  new_game(p, g);
  if (budget >= 0 && g >= budget) p.g.status[g] = kIdle;
  if (g == 0) {
    const long long started = budget < 0 ? p.G : (budget < p.G ? budget : p.G);
    p.ctr->games_started = (unsigned long long)started;
    p.ctr->start_budget = budget < 0 ? 0 : budget - started;
    p.ctr->unlimited = budget < 0 ? 1 : 0;
  }
}

__global__ void k_set_root(Params p, int g, uint64_t own, uint64_t opp, int player) {
  if (threadIdx.x != 0) return;
  p.g.half[g] = 0;
  init_root(p, g, 0, own, opp);
  p.g.n_nodes[g] = 1;
  p.g.root_player[g] = player;
  p.g.leaf[(int64_t)g * p.K] = -1;
  p.g.open[g] = 0;
  p.g.sims_done[g] = 0;
  p.g.sims_target[g] = 0;
  p.g.status[g] = kSearchDone;
}

__global__ void k_begin(Params p, int slot, int sims) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= p.G || (slot >= 0 && g != slot)) return;
  if (p.g.status[g] == kIdle || p.g.status[g] == kFinished) return;
  p.g.sims_done[g] = 0;
  p.g.sims_target[g] = sims;
  p.g.leaf[(int64_t)g * p.K] = -1;
  p.g.open[g] = 0;
  p.g.status[g] = kActive;
}

__global__ void k_policy(Params p, int slot, double temp, double u_tie, float* pi_o,
                         double* vroot_o, int32_t* counts_o) {
  const int g = slot;
  const int lane = threadIdx.x;
  const int half = p.g.half[g];
  float p64;
  const float pi = root_pi(p, g, half, temp, u_tie, &p64);
  pi_o[lane] = pi;
  if (lane == 0) pi_o[64] = p64;
  const int64_t r = nidx(p, half, g, 0);
  if (counts_o) {
    counts_o[lane] = 0;
    if (lane == 0) counts_o[64] = 0;
  }
  if (lane == 0) {
    const int n = p.a.N[r];
    *vroot_o = n == 0 ? 0.0 : p.a.W[r] / (double)n;
    if (counts_o) {
      const int nc = p.a.nchild[r], fc = p.a.first[r];
      for (int j = 0; j < nc; ++j) {
        const int64_t c = nidx(p, half, g, fc + j);
        counts_o[p.a.action[c]] = p.a.N[c];
      }
    }
  }
}

__global__ __launch_bounds__(kMoveBlock) void k_reroot(Params p, int g, int action,
                                                       int32_t* result) {
  extern __shared__ __align__(16) int32_t map[];
  __shared__ int s_child;
  const int half = p.g.half[g];
  if (threadIdx.x == 0) {
    const int64_t r = nidx(p, half, g, 0);
    const int nc = (p.a.flags[r] & kExpanded) ? p.a.nchild[r] : 0, fc = p.a.first[r];
    int child = -1;
    for (int j = 0; j < nc; ++j)
      if (p.a.action[nidx(p, half, g, fc + j)] == action) child = fc + j;
    s_child = child;
    *result = child;
  }
  __syncthreads();
  if (s_child < 0) return;
  const int player = p.g.root_player[g];
  compact(p, g, s_child, map, p.g.half[g], p.g.n_nodes[g]);
  if (threadIdx.x == 0) {
    p.g.root_player[g] = -player;
    p.g.sims_done[g] = 0;
    p.g.sims_target[g] = 0;
    p.g.status[g] = kSearchDone;
  }
}

// ---- batched host-driven control (arena evaluation: many independent searches) -------

__global__ void k_set_roots(Params p, const int32_t* slots, const uint64_t* own,
                            const uint64_t* opp, const int32_t* player, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int g = slots[i];
  if (g < 0 || g >= p.G) return;
  p.g.half[g] = 0;
  init_root(p, g, 0, own[i], opp[i]);
  p.g.n_nodes[g] = 1;
  p.g.root_player[g] = player[i];
  p.g.leaf[(int64_t)g * p.K] = -1;
  p.g.open[g] = 0;
  p.g.sims_done[g] = 0;
  p.g.sims_target[g] = 0;
  p.g.status[g] = kSearchDone;
}

__global__ void k_begin_slots(Params p, const int32_t* slots, int n, int sims) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int g = slots[i];
  if (g < 0 || g >= p.G) return;
  p.g.sims_done[g] = 0;
  p.g.sims_target[g] = sims;
  p.g.leaf[(int64_t)g * p.K] = -1;
  p.g.open[g] = 0;
  p.g.status[g] = kActive;
}

// child visit counts (int32 [G, 65]) and root W/N of every slot: one wave per slot
__global__ __launch_bounds__(kSelBlock) void k_root_stats(Params p, int32_t* counts,
                                                          double* vroot) {
  const int g = blockIdx.x * (kSelBlock / kWave) + (threadIdx.x >> 6);
  if (g >= p.G) return;
  const int lane = lane_id();
  const int half = p.g.half[g];
  const int64_t r = nidx(p, half, g, 0);
  int32_t* row = counts + (int64_t)g * 65;
  row[lane] = 0;
  if (lane == 0) row[64] = 0;
  const int nc = (p.a.flags[r] & kExpanded) ? p.a.nchild[r] : 0, fc = p.a.first[r];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  if (lane < nc) {
    const int64_t c = nidx(p, half, g, fc + lane);
    row[p.a.action[c]] = p.a.N[c];
  }
  if (lane == 0) {
    const int n = p.a.N[r];
    vroot[g] = n == 0 ? 0.0 : p.a.W[r] / (double)n;
  }
}

// re-root every slot with actions[g] >= 0 (MCTS.make_move on many trees at once);
// found[g] = child node or -1 (KeyError / no tree); one workgroup per slot
__global__ __launch_bounds__(kMoveBlock) void k_reroot_slots(Params p, const int32_t* actions,
                                                             int32_t* found) {
  extern __shared__ __align__(16) int32_t map[];
  __shared__ int s_child;
  for (int g = blockIdx.x; g < p.G; g += gridDim.x) {
    const int action = actions[g];
    if (action < 0) {
      if (threadIdx.x == 0) found[g] = -1;
      continue;
    }
    const int half = p.g.half[g];
    if (threadIdx.x == 0) {
      const int64_t r = nidx(p, half, g, 0);
      const int nc = (p.a.flags[r] & kExpanded) ? p.a.nchild[r] : 0, fc = p.a.first[r];
      int child = -1;
      for (int j = 0; j < nc; ++j)
        if (p.a.action[nidx(p, half, g, fc + j)] == action) child = fc + j;
      s_child = child;
      found[g] = child;
    }
    __syncthreads();
    if (s_child >= 0) {
      const int player = p.g.root_player[g];
      compact(p, g, s_child, map, p.g.half[g], p.g.n_nodes[g]);
      if (threadIdx.x == 0) {
        p.g.root_player[g] = -player;
        p.g.sims_done[g] = 0;
        p.g.sims_target[g] = 0;
        p.g.status[g] = kSearchDone;
      }
    }
    __syncthreads();
  }
}

}  // namespace

// ====================================================================================
// host side

struct az_engine {
  az_config cfg;
  // kernels take the parameters by value (kernarg): their pointer fields keep the global
  // address space, so loads and stores through them are global_* instructions (through a
  // pointer to a device copy of Params they compiled to flat_*: round 4, reverted -- it did
  // not change the profiler faults either)
  Params p;
  std::vector<void*> allocs;
  int32_t* d_result = nullptr;
  char* d_scratch = nullptr;  // 1 KiB: az_root_policy outputs
  // batched host-driven control buffers ([G] each, counts [G, 65])
  int32_t* d_slots = nullptr;
  int32_t* d_ivec = nullptr;
  int32_t* d_found = nullptr;
  int32_t* d_counts = nullptr;
  double* d_vroot = nullptr;
  uint64_t* d_own = nullptr;
  uint64_t* d_opp = nullptr;
  float* d_zero_eval = nullptr;  // rollout mode: zeroed [G*K, 66] stand-in priors / values
  size_t lds_move = 0;
};

namespace {

template <typename T>
int dalloc(az_engine* e, T** ptr, size_t count) {
  void* q = nullptr;
  const size_t bytes = count * sizeof(T) > 0 ? count * sizeof(T) : 16;
  hipError_t err = hipMalloc(&q, bytes);
  if (err != hipSuccess)
    return azc::set_error(AZ_ERR_HIP, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(err));
  e->allocs.push_back(q);
  *ptr = static_cast<T*>(q);
  return AZ_OK;
}

#define AZ_TRY(x)            \
  do {                       \
    int rc_ = (x);           \
    if (rc_ != AZ_OK) return rc_; \
  } while (0)

void free_all(az_engine* e) {
  for (void* q : e->allocs) (void)hipFree(q);
  e->allocs.clear();
}

unsigned sel_grid(const az_engine* e) {
  const int per = kSelBlock / kWave;
  return (unsigned)((e->p.G + per - 1) / per);
}

}  // namespace

extern "C" {

#if AZ_ENG_STAMP
int az_eng_stamps(unsigned long long* host, unsigned* n_written) {
  AZ_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_eng_stamps), sizeof(g_eng_stamps)));
  AZ_HIP(hipMemcpyFromSymbol(n_written, HIP_SYMBOL(g_eng_stamp_n), sizeof(unsigned)));
  return AZ_OK;
}
#endif

int az_engine_create(const az_config* cfg_in, az_engine** out) {
  AZ_GUARD_BEGIN
  AZ_REQUIRE(cfg_in && out, AZ_ERR_ARG, "az_engine_create: null argument");
  az_config cfg = *cfg_in;
  if (cfg.node_capacity <= 0) cfg.node_capacity = 16384;
  if (cfg.max_plies <= 0) cfg.max_plies = 128;
  AZ_REQUIRE(cfg.n_games > 0, AZ_ERR_ARG, "n_games must be > 0");
  AZ_REQUIRE(cfg.node_capacity >= 128 && cfg.node_capacity <= 32768, AZ_ERR_ARG,
             "node_capacity must be in [128, 32768] (LDS re-root scratch), got %d",
             cfg.node_capacity);
  AZ_REQUIRE(cfg.num_simulations >= 0, AZ_ERR_ARG, "num_simulations must be >= 0");
  AZ_REQUIRE(cfg.eval_mode == AZ_EVAL_EXTERNAL || cfg.eval_mode == AZ_EVAL_ROLLOUT, AZ_ERR_ARG,
             "bad eval_mode");
  AZ_REQUIRE(cfg.rng_mode == AZ_RNG_DEVICE || cfg.rng_mode == AZ_RNG_INJECTED, AZ_ERR_ARG,
             "bad rng_mode");
  if (cfg.sample_capacity <= 0) cfg.sample_capacity = (int64_t)cfg.n_games * cfg.max_plies * 2;
  if (cfg.inj_noise_slots <= 0) cfg.inj_noise_slots = 1;
  if (cfg.inj_uniform_slots <= 0) cfg.inj_uniform_slots = 1;
  if (cfg.leaves_per_step <= 0) cfg.leaves_per_step = 1;
  AZ_REQUIRE(cfg.leaves_per_step <= kMaxLeaves, AZ_ERR_ARG,
             "leaves_per_step must be in [1, %d], got %d", kMaxLeaves, cfg.leaves_per_step);

  az_engine* e = new (std::nothrow) az_engine();
  AZ_REQUIRE(e, AZ_ERR_ARG, "out of host memory");
  e->cfg = cfg;
  Params& p = e->p;
  p.G = cfg.n_games;
  p.C = cfg.node_capacity;
  p.T = cfg.max_plies;
  p.NS = cfg.inj_noise_slots;
  p.NU = cfg.inj_uniform_slots;
  p.sims = cfg.num_simulations;
  p.K = cfg.leaves_per_step;
  p.n_explore = cfg.num_exploratory_moves;
  p.eval_mode = cfg.eval_mode;
  p.rng_mode = cfg.rng_mode;
  p.d4 = cfg.d4_augment ? 1 : 0;
  p.defer = 0;
  p.auto_play = cfg.auto_play ? 1 : 0;
  p.refill = cfg.refill ? 1 : 0;
  p.c_puct = cfg.c_puct;
  p.alpha = cfg.dirichlet_alpha;
  p.eps = cfg.dirichlet_epsilon;
  p.temp = cfg.temperature;
  p.lambd = cfg.lambd;
  p.seed = cfg.seed;
  p.stream_id = (uint32_t)cfg.stream_id;

  const size_t nodes = (size_t)2 * p.G * p.C;
  const size_t G = p.G, T = p.T;
  int rc = AZ_OK;
  auto chk = [&](int r) {
    if (rc == AZ_OK) rc = r;
  };
  chk(dalloc(e, &p.a.own, nodes));
  chk(dalloc(e, &p.a.opp, nodes));
  chk(dalloc(e, &p.a.legal, nodes));
  chk(dalloc(e, &p.a.N, nodes));
  chk(dalloc(e, &p.a.W, nodes));
  chk(dalloc(e, &p.a.P, nodes));
  chk(dalloc(e, &p.a.parent, nodes));
  chk(dalloc(e, &p.a.first, nodes));
  chk(dalloc(e, &p.a.nchild, nodes));
  chk(dalloc(e, &p.a.action, nodes));
  chk(dalloc(e, &p.a.flags, nodes));
  chk(dalloc(e, &p.a.tval, nodes));
  chk(dalloc(e, &p.g.status, G));
  chk(dalloc(e, &p.g.half, G));
  chk(dalloc(e, &p.g.n_nodes, G));
  chk(dalloc(e, &p.g.sims_done, G));
  chk(dalloc(e, &p.g.sims_target, G));
  chk(dalloc(e, &p.g.sims_acc, G));
  const size_t GK = G * (size_t)p.K;
  chk(dalloc(e, &p.g.leaf, GK));
  chk(dalloc(e, &p.g.path, GK * kMaxPath));
  chk(dalloc(e, &p.g.path_len, GK));
  chk(dalloc(e, &p.g.ply, G));
  chk(dalloc(e, &p.g.root_player, G));
  chk(dalloc(e, &p.g.winner, G));
  chk(dalloc(e, &p.g.overflow, G));
  chk(dalloc(e, &p.g.start_step, G));
  chk(dalloc(e, &p.g.sstep, G));
  chk(dalloc(e, &p.g.moving, G));
  chk(dalloc(e, &p.g.rng_event, G));
  chk(dalloc(e, &p.g.sym, GK));
  chk(dalloc(e, &p.g.noise_cur, G));
  chk(dalloc(e, &p.g.u_cur, G));
  chk(dalloc(e, &p.g.open, G));
  chk(dalloc(e, &p.g.t_own, G * T));
  chk(dalloc(e, &p.g.t_opp, G * T));
  chk(dalloc(e, &p.g.t_pi, G * T * 65));
  chk(dalloc(e, &p.g.t_player, G * T));
  chk(dalloc(e, &p.g.t_vroot, G * T));
  p.s.cap = cfg.sample_capacity;
  chk(dalloc(e, &p.s.own, (size_t)p.s.cap));
  chk(dalloc(e, &p.s.opp, (size_t)p.s.cap));
  chk(dalloc(e, &p.s.pi, (size_t)p.s.cap * 65));
  chk(dalloc(e, &p.s.z, (size_t)p.s.cap));
  chk(dalloc(e, &p.s.player, (size_t)p.s.cap));
  chk(dalloc(e, &p.s.slot, (size_t)p.s.cap));
  chk(dalloc(e, &p.ctr, 1));
  chk(dalloc(e, &p.ready, 2 * G));
  double* noise = nullptr;
  double* uni = nullptr;
  if (cfg.rng_mode == AZ_RNG_INJECTED) {
    chk(dalloc(e, &noise, G * p.NS * 65));
    chk(dalloc(e, &uni, G * p.NU));
  }
  p.inj_noise = noise;
  p.inj_u = uni;
  chk(dalloc(e, &e->d_result, 4));
  chk(dalloc(e, &e->d_scratch, 1024));
  chk(dalloc(e, &e->d_slots, G));
  chk(dalloc(e, &e->d_ivec, G));
  chk(dalloc(e, &e->d_found, G));
  chk(dalloc(e, &e->d_counts, G * 65));
  chk(dalloc(e, &e->d_vroot, G));
  chk(dalloc(e, &e->d_own, G));
  chk(dalloc(e, &e->d_opp, G));
  chk(dalloc(e, &e->d_zero_eval, GK * 66));
  if (rc != AZ_OK) {
    free_all(e);
    delete e;
    return rc;
  }
  e->lds_move = (size_t)p.C * sizeof(int32_t);
  if (hipFuncSetAttribute((const void*)k_move, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_reroot, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_reroot_slots, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      // k_select carries the deferred move phase (az_select_move)
      hipFuncSetAttribute((const void*)k_select<1, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_select<2, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_select<4, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_select<kMaxLeaves, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      // ... and with the fused expansion (az_select_move_expand)
      hipFuncSetAttribute((const void*)k_select<1, true, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_select<2, true, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_select<4, true, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_select<kMaxLeaves, true, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)e->lds_move) != hipSuccess) {
    (void)hipGetLastError();
  }
  // Every per-slot word and every node's flags / child count start zeroed (idle slots on
  // half 0 with an unexpanded empty root): kernels that sweep all slots (k_root_stats,
  // k_select's idle check, ...) read them before the host sets a slot up, and a reused
  // device allocation would otherwise hold a previous engine's values (out-of-range
  // halves, child ranges).
  bool zero_ok = hipMemset(p.ctr, 0, sizeof(Counters)) == hipSuccess &&
                 hipMemset(p.g.moving, 0x80, G * sizeof(int32_t)) == hipSuccess &&  // never a step
                 hipMemset(p.g.leaf, 0xff, GK * sizeof(int32_t)) == hipSuccess &&
                 hipMemset(p.g.path_len, 0, GK * sizeof(int32_t)) == hipSuccess &&
                 hipMemset(p.a.flags, 0, nodes) == hipSuccess &&
                 hipMemset(p.a.nchild, 0, nodes) == hipSuccess;
  for (int32_t* a : {p.g.status, p.g.half, p.g.n_nodes, p.g.sims_done, p.g.sims_target,
                     p.g.ply, p.g.root_player, p.g.winner, p.g.overflow,
                     p.g.start_step, p.g.sstep, p.g.noise_cur, p.g.u_cur, p.g.open})
    zero_ok = zero_ok && hipMemset(a, 0, G * sizeof(int32_t)) == hipSuccess;
  zero_ok = zero_ok && hipMemset(p.g.sims_acc, 0, G * sizeof(unsigned long long)) == hipSuccess &&
            hipMemset(p.g.rng_event, 0, G * sizeof(uint32_t)) == hipSuccess &&
            hipMemset(p.g.sym, 0, GK) == hipSuccess &&
            hipMemset(e->d_zero_eval, 0, GK * 66 * sizeof(float)) == hipSuccess;
  if (!zero_ok) {
    free_all(e);
    delete e;
    return azc::set_error(AZ_ERR_HIP, "hipMemset failed");
  }
  *out = e;
  return AZ_OK;
  AZ_GUARD_END
}

int az_engine_destroy(az_engine* e) {
  if (!e) return AZ_OK;
  (void)hipDeviceSynchronize();
  free_all(e);
  delete e;
  return AZ_OK;
}

int az_reset_all(az_engine* e, int64_t start_budget, int32_t stagger_steps, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  hipStream_t s = azc::as_stream(stream);
  const unsigned grid = (unsigned)((e->p.G + 255) / 256);
  hipLaunchKernelGGL(k_reset, dim3(grid), dim3(256), 0, s, e->p, (long long)start_budget,
                     (int)stagger_steps);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_set_root(az_engine* e, int32_t slot, uint64_t own, uint64_t opp, int32_t player,
                void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(slot >= 0 && slot < e->p.G, AZ_ERR_ARG, "slot %d out of range", slot);
  AZ_REQUIRE((own & opp) == 0, AZ_ERR_ARG, "own and opp overlap");
  AZ_REQUIRE(player == 1 || player == -1, AZ_ERR_ARG, "player must be +1 or -1");
  hipStream_t s = azc::as_stream(stream);
  hipLaunchKernelGGL(k_set_root, dim3(1), dim3(64), 0, s, e->p, (int)slot, own, opp,
                     (int)player);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_begin_search(az_engine* e, int32_t slot, int32_t num_simulations, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(slot >= -1 && slot < e->p.G, AZ_ERR_ARG, "slot %d out of range", slot);
  AZ_REQUIRE(num_simulations >= 0, AZ_ERR_ARG, "num_simulations < 0");
  hipStream_t s = azc::as_stream(stream);
  const unsigned grid = (unsigned)((e->p.G + 255) / 256);
  hipLaunchKernelGGL(k_begin, dim3(grid), dim3(256), 0, s, e->p, (int)slot,
                     (int)num_simulations);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

// k_select (+ the deferred move phase in its first move_blocks workgroups)
static int launch_select(az_engine* e, float* nn_in, int32_t* leaf_o, int par, int move_blocks,
                         hipStream_t s, const float* priors = nullptr,
                         const float* values = nullptr, bool fused = false) {
  // Simulations that end on a terminal node need no evaluation and run inside the select
  // call; cap them per step so one end-game tree (every simulation terminal) cannot hold
  // the whole batched step for hundreds of dependent descents.  Host-driven engines step
  // one search at a time and take them all at once.
  static const int env_md = [] {
    const char* v = getenv("AZ_MAX_DESCENTS");  // experiment knob (scripts/exp), default 4
    return v ? atoi(v) : 0;
  }();
  // (with K leaves per step the cap is 4 K descents: a launch that reaches it with fewer than
  // K leaves waiting leaves its batch open for the next launch -- the same batches)
  const int max_descents = e->p.auto_play ? (env_md > 0 ? env_md : 4 * e->p.K)
                                          : 4 * (e->p.sims + 1) + 64;
  const dim3 grid(sel_grid(e) + (unsigned)move_blocks);
  const size_t lds = move_blocks ? e->lds_move : 0;  // the move phase's re-root scratch
  // the kernels' per-leaf arrays sized to the next power of two >= K (registers)
#define AZ_SEL_GO(KM)                                                                       \
  do {                                                                                     \
    if (fused)                                                                             \
      hipLaunchKernelGGL((k_select<KM, true, true>), grid, dim3(kSelBlock), lds, s, e->p,   \
                         nn_in, leaf_o, max_descents, par, move_blocks, priors, values);   \
    else if (move_blocks)                                                                  \
      hipLaunchKernelGGL((k_select<KM, true>), grid, dim3(kSelBlock), lds, s, e->p, nn_in,  \
                         leaf_o, max_descents, par, move_blocks, nullptr, nullptr);        \
    else                                                                                   \
      hipLaunchKernelGGL((k_select<KM, false>), grid, dim3(kSelBlock), lds, s, e->p, nn_in, \
                         leaf_o, max_descents, par, 0, nullptr, nullptr);                  \
  } while (0)
  if (e->p.K == 1)
    AZ_SEL_GO(1);
  else if (e->p.K <= 2)
    AZ_SEL_GO(2);
  else if (e->p.K <= 4)
    AZ_SEL_GO(4);
  else
    AZ_SEL_GO(kMaxLeaves);
#undef AZ_SEL_GO
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

static int move_blocks_for(const az_engine* e) { return e->p.G < 64 ? e->p.G : 64; }

int az_select(az_engine* e, float* nn_in, int32_t* leaf_o, void* stream) {
  AZ_REQUIRE(e && nn_in, AZ_ERR_ARG, "az_select: null argument");
  AZ_REQUIRE(!e->p.defer, AZ_ERR_STATE, "az_select: deferred moves are on (az_select_move)");
  return launch_select(e, nn_in, leaf_o, 0, 0, azc::as_stream(stream));
}

int az_engine_defer_moves(az_engine* e, int32_t on) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(e->p.auto_play || !on, AZ_ERR_STATE, "deferred moves need an auto-play engine");
  e->p.defer = on ? 1 : 0;
  return AZ_OK;
}

int az_engine_set_stem(az_engine* e, const float* w9, const float* bias, float* y,
                       float* absmax, int32_t channels) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  if (channels == 0) {
    e->p.stem_c = 0;
    e->p.stem_w = e->p.stem_b = nullptr;
    e->p.stem_y = e->p.stem_amax = nullptr;
    return AZ_OK;
  }
  AZ_REQUIRE(channels == 64 || channels == 128, AZ_ERR_ARG,
             "az_engine_set_stem: channels must be 0, 64 or 128, got %d", channels);
  AZ_REQUIRE(w9 && bias && y, AZ_ERR_ARG, "az_engine_set_stem: null buffer");
  AZ_REQUIRE(((uintptr_t)w9 | (uintptr_t)bias | (uintptr_t)y) % 8 == 0, AZ_ERR_ARG,
             "az_engine_set_stem: buffers must be 8-byte aligned");
  e->p.stem_w = w9;
  e->p.stem_b = bias;
  e->p.stem_y = y;
  e->p.stem_amax = absmax;
  e->p.stem_c = channels;
  return AZ_OK;
}

int az_select_move(az_engine* e, float* nn_in, int32_t* leaf_o, int32_t par, void* stream) {
  AZ_REQUIRE(e && nn_in, AZ_ERR_ARG, "az_select_move: null argument");
  AZ_REQUIRE(e->p.defer, AZ_ERR_STATE, "az_select_move: deferred moves are off");
  AZ_REQUIRE(par == 0 || par == 1, AZ_ERR_ARG, "az_select_move: par must be 0 or 1");
  return launch_select(e, nn_in, leaf_o, par, move_blocks_for(e), azc::as_stream(stream));
}

int az_select_move_expand(az_engine* e, float* nn_in, int32_t* leaf_o, const float* priors,
                          const float* values, int32_t par, void* stream) {
  AZ_REQUIRE(e && nn_in, AZ_ERR_ARG, "az_select_move_expand: null argument");
  AZ_REQUIRE(e->p.defer, AZ_ERR_STATE, "az_select_move_expand: deferred moves are off");
  AZ_REQUIRE(par == 0 || par == 1, AZ_ERR_ARG, "az_select_move_expand: par must be 0 or 1");
  AZ_REQUIRE(e->p.eval_mode == AZ_EVAL_ROLLOUT || (priors && values), AZ_ERR_ARG,
             "az_select_move_expand: priors/values required in external-eval mode");
  if (!priors || !values) {  // rollout mode: the expansion loads rows unconditionally
    priors = e->d_zero_eval;
    values = e->d_zero_eval + (size_t)e->p.G * e->p.K * 65;
  }
  return launch_select(e, nn_in, leaf_o, par, move_blocks_for(e), azc::as_stream(stream),
                       priors, values, true);
}

int az_select_expand(az_engine* e, float* nn_in, int32_t* leaf_o, const float* priors,
                     const float* values, void* stream) {
  AZ_REQUIRE(e && nn_in, AZ_ERR_ARG, "az_select_expand: null argument");
  AZ_REQUIRE(!e->p.defer, AZ_ERR_STATE, "az_select_expand: deferred moves are on (az_select_move_expand)");
  AZ_REQUIRE(e->p.eval_mode == AZ_EVAL_ROLLOUT || (priors && values), AZ_ERR_ARG,
             "az_select_expand: priors/values required in external-eval mode");
  if (!priors || !values) {  // rollout mode: the expansion loads rows unconditionally
    priors = e->d_zero_eval;
    values = e->d_zero_eval + (size_t)e->p.G * e->p.K * 65;
  }
  return launch_select(e, nn_in, leaf_o, 0, 0, azc::as_stream(stream), priors, values, true);
}

int az_move_flush(az_engine* e, int32_t par, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(e->p.defer, AZ_ERR_STATE, "az_move_flush: deferred moves are off");
  AZ_REQUIRE(par == 0 || par == 1, AZ_ERR_ARG, "az_move_flush: par must be 0 or 1");
  // the move phase of a step of parity `par` alone: a k_select launch with no slot
  // workgroups (move list par = (par ^ 1) ^ 1)
  hipStream_t s = azc::as_stream(stream);
  const int mb = move_blocks_for(e);
  const dim3 grid((unsigned)mb);
  const int q = par ^ 1;
  if (e->p.K == 1)
    hipLaunchKernelGGL((k_select<1, true>), grid, dim3(kSelBlock), e->lds_move, s, e->p, nullptr,
                       nullptr, 0, q, mb, nullptr, nullptr);
  else if (e->p.K <= 2)
    hipLaunchKernelGGL((k_select<2, true>), grid, dim3(kSelBlock), e->lds_move, s, e->p, nullptr,
                       nullptr, 0, q, mb, nullptr, nullptr);
  else if (e->p.K <= 4)
    hipLaunchKernelGGL((k_select<4, true>), grid, dim3(kSelBlock), e->lds_move, s, e->p, nullptr,
                       nullptr, 0, q, mb, nullptr, nullptr);
  else
    hipLaunchKernelGGL((k_select<kMaxLeaves, true>), grid, dim3(kSelBlock), e->lds_move, s, e->p,
                       nullptr, nullptr, 0, q, mb, nullptr, nullptr);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

static int launch_expand(az_engine* e, const float* priors, const float* values, int par,
                         void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(e->p.eval_mode == AZ_EVAL_ROLLOUT || (priors && values), AZ_ERR_ARG,
             "az_expand_backup: priors/values required in external-eval mode");
  hipStream_t s = azc::as_stream(stream);
  if (!priors || !values) {  // rollout mode: k_expand loads rows unconditionally
    priors = e->d_zero_eval;
    values = e->d_zero_eval + (size_t)e->p.G * e->p.K * 65;
  }
  if (e->p.K == 1)
    hipLaunchKernelGGL(k_expand<1>, dim3(sel_grid(e)), dim3(kSelBlock), 0, s, e->p, priors,
                       values, par);
  else if (e->p.K <= 2)
    hipLaunchKernelGGL(k_expand<2>, dim3(sel_grid(e)), dim3(kSelBlock), 0, s, e->p, priors,
                       values, par);
  else if (e->p.K <= 4)
    hipLaunchKernelGGL(k_expand<4>, dim3(sel_grid(e)), dim3(kSelBlock), 0, s, e->p, priors,
                       values, par);
  else
    hipLaunchKernelGGL(k_expand<kMaxLeaves>, dim3(sel_grid(e)), dim3(kSelBlock), 0, s, e->p,
                       priors, values, par);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

int az_expand_backup(az_engine* e, const float* priors, const float* values, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(!e->p.defer, AZ_ERR_STATE, "az_expand_backup: deferred moves are on (use _par)");
  return launch_expand(e, priors, values, 0, stream);
}

int az_expand_backup_par(az_engine* e, const float* priors, const float* values, int32_t par,
                         void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(e->p.defer, AZ_ERR_STATE, "az_expand_backup_par: deferred moves are off");
  AZ_REQUIRE(par == 0 || par == 1, AZ_ERR_ARG, "az_expand_backup_par: par must be 0 or 1");
  return launch_expand(e, priors, values, par, stream);
}

int az_play(az_engine* e, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(!e->p.defer, AZ_ERR_STATE, "az_play: deferred moves are on (az_select_move)");
  hipStream_t s = azc::as_stream(stream);
  if (!e->p.auto_play) {
    hipLaunchKernelGGL(k_tick, dim3(1), dim3(1), 0, s, e->p.ctr);
    AZ_HIP(hipGetLastError());
    return AZ_OK;
  }
  // the ready list holds a few slots per step (G / (sims + 1) / plies on average): 64
  // workgroups take them grid-stride, and each workgroup's closing atomic on the shared
  // move_done counter stays cheap (one address serialises ~90 atomics per microsecond)
  const int blocks = e->p.G < 64 ? e->p.G : 64;
  hipLaunchKernelGGL(k_move, dim3(blocks), dim3(kMoveBlock), e->lds_move, s, e->p);
  AZ_HIP(hipGetLastError());
  return AZ_OK;
}

int az_inject(az_engine* e, const double* noise, const double* uniforms, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(e->p.rng_mode == AZ_RNG_INJECTED, AZ_ERR_STATE, "engine not in injected-RNG mode");
  hipStream_t s = azc::as_stream(stream);
  const size_t G = e->p.G;
  if (noise)
    AZ_HIP(hipMemcpyAsync((void*)e->p.inj_noise, noise, G * e->p.NS * 65 * sizeof(double),
                          hipMemcpyHostToDevice, s));
  if (uniforms)
    AZ_HIP(hipMemcpyAsync((void*)e->p.inj_u, uniforms, G * e->p.NU * sizeof(double),
                          hipMemcpyHostToDevice, s));
  AZ_HIP(hipMemsetAsync(e->p.g.noise_cur, 0, G * sizeof(int32_t), s));
  AZ_HIP(hipMemsetAsync(e->p.g.u_cur, 0, G * sizeof(int32_t), s));
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_root_policy(az_engine* e, int32_t slot, double temp, double u_tie, float* pi_o,
                   int32_t* counts_o, double* vroot_o, void* stream) {
  AZ_REQUIRE(e && pi_o, AZ_ERR_ARG, "az_root_policy: null argument");
  AZ_REQUIRE(slot >= 0 && slot < e->p.G, AZ_ERR_ARG, "slot out of range");
  hipStream_t s = azc::as_stream(stream);
  float* d_pi = (float*)e->d_scratch;                  // [0, 260)
  double* d_v = (double*)(e->d_scratch + 264);          // [264, 272)
  int32_t* d_c = (int32_t*)(e->d_scratch + 272);        // [272, 532)
  hipLaunchKernelGGL(k_policy, dim3(1), dim3(64), 0, s, e->p, (int)slot, temp, u_tie, d_pi, d_v,
                     d_c);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipMemcpyAsync(pi_o, d_pi, 65 * sizeof(float), hipMemcpyDeviceToHost, s));
  double v = 0.0;
  int32_t c[65];
  AZ_HIP(hipMemcpyAsync(&v, d_v, sizeof(double), hipMemcpyDeviceToHost, s));
  AZ_HIP(hipMemcpyAsync(c, d_c, sizeof(c), hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  if (vroot_o) *vroot_o = v;
  if (counts_o)
    for (int i = 0; i < 65; ++i) counts_o[i] = c[i];
  return AZ_OK;
}

int az_make_move(az_engine* e, int32_t slot, int32_t action, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(slot >= 0 && slot < e->p.G, AZ_ERR_ARG, "slot out of range");
  AZ_REQUIRE(action >= 0 && action <= 64, AZ_ERR_STATE, "%d", action);
  hipStream_t s = azc::as_stream(stream);
  hipLaunchKernelGGL(k_reroot, dim3(1), dim3(kMoveBlock), e->lds_move, s, e->p, (int)slot,
                     (int)action, e->d_result);
  AZ_HIP(hipGetLastError());
  int32_t child = -1;
  AZ_HIP(hipMemcpyAsync(&child, e->d_result, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  // KeyError in the reference (MCTS_model.py:214)
  AZ_REQUIRE(child >= 0, AZ_ERR_STATE, "%d", action);
  return AZ_OK;
}

int az_set_roots(az_engine* e, const int32_t* slots, const uint64_t* own, const uint64_t* opp,
                 const int32_t* player, int32_t n, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(n >= 0 && n <= e->p.G, AZ_ERR_ARG, "az_set_roots: n out of range");
  if (n == 0) return AZ_OK;
  AZ_REQUIRE(slots && own && opp && player, AZ_ERR_ARG, "az_set_roots: null buffer");
  for (int i = 0; i < n; ++i) {
    AZ_REQUIRE(slots[i] >= 0 && slots[i] < e->p.G, AZ_ERR_ARG, "slot %d out of range", slots[i]);
    AZ_REQUIRE((own[i] & opp[i]) == 0, AZ_ERR_ARG, "own and opp overlap (slot %d)", slots[i]);
    AZ_REQUIRE(player[i] == 1 || player[i] == -1, AZ_ERR_ARG, "player must be +1 or -1");
  }
  hipStream_t s = azc::as_stream(stream);
  AZ_HIP(hipMemcpyAsync(e->d_slots, slots, n * 4, hipMemcpyHostToDevice, s));
  AZ_HIP(hipMemcpyAsync(e->d_own, own, n * 8, hipMemcpyHostToDevice, s));
  AZ_HIP(hipMemcpyAsync(e->d_opp, opp, n * 8, hipMemcpyHostToDevice, s));
  AZ_HIP(hipMemcpyAsync(e->d_ivec, player, n * 4, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_set_roots, dim3((n + 255) / 256), dim3(256), 0, s, e->p, e->d_slots,
                     e->d_own, e->d_opp, e->d_ivec, (int)n);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_begin_search_slots(az_engine* e, const int32_t* slots, int32_t n,
                          int32_t num_simulations, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(n >= 0 && n <= e->p.G && num_simulations >= 0, AZ_ERR_ARG,
             "az_begin_search_slots: bad n / num_simulations");
  if (n == 0) return AZ_OK;
  AZ_REQUIRE(slots, AZ_ERR_ARG, "az_begin_search_slots: null slots");
  hipStream_t s = azc::as_stream(stream);
  AZ_HIP(hipMemcpyAsync(e->d_slots, slots, n * 4, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_begin_slots, dim3((n + 255) / 256), dim3(256), 0, s, e->p, e->d_slots,
                     (int)n, (int)num_simulations);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_root_stats(az_engine* e, int32_t* counts, double* vroot, void* stream) {
  AZ_REQUIRE(e && counts, AZ_ERR_ARG, "az_root_stats: null argument");
  hipStream_t s = azc::as_stream(stream);
  hipLaunchKernelGGL(k_root_stats, dim3(sel_grid(e)), dim3(kSelBlock), 0, s, e->p, e->d_counts,
                     e->d_vroot);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipMemcpyAsync(counts, e->d_counts, (size_t)e->p.G * 65 * 4, hipMemcpyDeviceToHost, s));
  if (vroot)
    AZ_HIP(hipMemcpyAsync(vroot, e->d_vroot, (size_t)e->p.G * 8, hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_reroot_slots(az_engine* e, const int32_t* actions, int32_t* found, void* stream) {
  AZ_REQUIRE(e && actions && found, AZ_ERR_ARG, "az_reroot_slots: null argument");
  hipStream_t s = azc::as_stream(stream);
  AZ_HIP(hipMemcpyAsync(e->d_ivec, actions, (size_t)e->p.G * 4, hipMemcpyHostToDevice, s));
  const int blocks = e->p.G < 256 ? e->p.G : 256;
  hipLaunchKernelGGL(k_reroot_slots, dim3(blocks), dim3(kMoveBlock), e->lds_move, s, e->p,
                     e->d_ivec, e->d_found);
  AZ_HIP(hipGetLastError());
  AZ_HIP(hipMemcpyAsync(found, e->d_found, (size_t)e->p.G * 4, hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_counters(az_engine* e, int64_t* out8, void* stream) {
  AZ_REQUIRE(e && out8, AZ_ERR_ARG, "null argument");
  hipStream_t s = azc::as_stream(stream);
  hipLaunchKernelGGL(k_sum_sims, dim3(1), dim3(1024), 0, s, e->p);
  AZ_HIP(hipGetLastError());
  Counters c;
  AZ_HIP(hipMemcpyAsync(&c, e->p.ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  out8[0] = (int64_t)c.games_started;
  out8[1] = (int64_t)c.games_finished;
  out8[2] = (int64_t)c.samples_n;
  out8[3] = (int64_t)c.samples_dropped;
  out8[4] = (int64_t)c.overflow;
  out8[5] = (int64_t)c.step;
  out8[6] = (int64_t)c.sims;
  out8[7] = (int64_t)c.moves;
  return AZ_OK;
}

int az_game_info(az_engine* e, int32_t* status, int32_t* ply, int32_t* winner,
                 int32_t* root_player, int32_t* n_nodes, int32_t* overflow, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  hipStream_t s = azc::as_stream(stream);
  const size_t b = (size_t)e->p.G * sizeof(int32_t);
  if (status) AZ_HIP(hipMemcpyAsync(status, e->p.g.status, b, hipMemcpyDeviceToHost, s));
  if (ply) AZ_HIP(hipMemcpyAsync(ply, e->p.g.ply, b, hipMemcpyDeviceToHost, s));
  if (winner) AZ_HIP(hipMemcpyAsync(winner, e->p.g.winner, b, hipMemcpyDeviceToHost, s));
  if (root_player)
    AZ_HIP(hipMemcpyAsync(root_player, e->p.g.root_player, b, hipMemcpyDeviceToHost, s));
  if (n_nodes) AZ_HIP(hipMemcpyAsync(n_nodes, e->p.g.n_nodes, b, hipMemcpyDeviceToHost, s));
  if (overflow) AZ_HIP(hipMemcpyAsync(overflow, e->p.g.overflow, b, hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_export_tree(az_engine* e, int32_t slot, int32_t max_nodes, uint64_t* own, uint64_t* opp,
                   uint64_t* legal, int32_t* N, double* W, double* prior, int32_t* parent,
                   int32_t* first_child, uint8_t* nchild, uint8_t* action, uint8_t* flags,
                   int8_t* tval, int32_t* n_nodes_o, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(slot >= 0 && slot < e->p.G, AZ_ERR_ARG, "slot out of range");
  hipStream_t s = azc::as_stream(stream);
  int32_t half = 0, n = 0;
  AZ_HIP(hipMemcpyAsync(&half, e->p.g.half + slot, 4, hipMemcpyDeviceToHost, s));
  AZ_HIP(hipMemcpyAsync(&n, e->p.g.n_nodes + slot, 4, hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  if (n_nodes_o) *n_nodes_o = n;
  const int m = n < max_nodes ? n : max_nodes;
  if (m <= 0) return AZ_OK;
  const int64_t off = ((int64_t)half * e->p.G + slot) * e->p.C;
#define CP(dst, src, T)                                                                   \
  if (dst) AZ_HIP(hipMemcpyAsync(dst, e->p.a.src + off, (size_t)m * sizeof(T),             \
                                 hipMemcpyDeviceToHost, s));
  CP(own, own, uint64_t)
  CP(opp, opp, uint64_t)
  CP(legal, legal, uint64_t)
  CP(N, N, int32_t)
  CP(W, W, double)
  CP(prior, P, double)
  CP(parent, parent, int32_t)
  CP(first_child, first, int32_t)
  CP(nchild, nchild, uint8_t)
  CP(action, action, uint8_t)
  CP(flags, flags, uint8_t)
  CP(tval, tval, int8_t)
#undef CP
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_export_trajectory(az_engine* e, int32_t slot, int32_t max_plies, uint64_t* own,
                         uint64_t* opp, float* pi, int8_t* player, double* vroot,
                         int32_t* n_plies_o, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(slot >= 0 && slot < e->p.G, AZ_ERR_ARG, "slot out of range");
  hipStream_t s = azc::as_stream(stream);
  int32_t ply = 0, st = 0;
  AZ_HIP(hipMemcpyAsync(&ply, e->p.g.ply + slot, 4, hipMemcpyDeviceToHost, s));
  AZ_HIP(hipMemcpyAsync(&st, e->p.g.status + slot, 4, hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  int n = st == kFinished ? ply + 1 : ply;
  if (n > e->p.T) n = e->p.T;
  if (n_plies_o) *n_plies_o = n;
  const int m = n < max_plies ? n : max_plies;
  if (m <= 0) return AZ_OK;
  const int64_t off = (int64_t)slot * e->p.T;
  if (own) AZ_HIP(hipMemcpyAsync(own, e->p.g.t_own + off, m * 8, hipMemcpyDeviceToHost, s));
  if (opp) AZ_HIP(hipMemcpyAsync(opp, e->p.g.t_opp + off, m * 8, hipMemcpyDeviceToHost, s));
  if (pi)
    AZ_HIP(hipMemcpyAsync(pi, e->p.g.t_pi + off * 65, (size_t)m * 65 * 4, hipMemcpyDeviceToHost, s));
  if (player)
    AZ_HIP(hipMemcpyAsync(player, e->p.g.t_player + off, m, hipMemcpyDeviceToHost, s));
  if (vroot)
    AZ_HIP(hipMemcpyAsync(vroot, e->p.g.t_vroot + off, m * 8, hipMemcpyDeviceToHost, s));
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_samples(az_engine* e, uint64_t** own, uint64_t** opp, float** pi, double** z,
               int8_t** player, int64_t* n, int64_t* capacity) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  if (own) *own = e->p.s.own;
  if (opp) *opp = e->p.s.opp;
  if (pi) *pi = e->p.s.pi;
  if (z) *z = e->p.s.z;
  if (player) *player = e->p.s.player;
  if (capacity) *capacity = e->p.s.cap;
  if (n) {
    Counters c;
    AZ_HIP(hipMemcpy(&c, e->p.ctr, sizeof(Counters), hipMemcpyDeviceToHost));
    *n = (int64_t)c.samples_n;
  }
  return AZ_OK;
}

int az_copy_samples(az_engine* e, int64_t start, int64_t n, uint64_t* own, uint64_t* opp,
                    float* pi, double* z, int8_t* player, int32_t* slot, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  AZ_REQUIRE(start >= 0 && n >= 0 && start + n <= e->p.s.cap, AZ_ERR_ARG,
             "sample range [%lld, %lld) outside capacity %lld", (long long)start,
             (long long)(start + n), (long long)e->p.s.cap);
  if (n == 0) return AZ_OK;
  hipStream_t s = azc::as_stream(stream);
  const auto k = hipMemcpyDefault;  // host or device destinations (unified addressing)
  if (own) AZ_HIP(hipMemcpyAsync(own, e->p.s.own + start, n * 8, k, s));
  if (opp) AZ_HIP(hipMemcpyAsync(opp, e->p.s.opp + start, n * 8, k, s));
  if (pi) AZ_HIP(hipMemcpyAsync(pi, e->p.s.pi + start * 65, n * 65 * 4, k, s));
  if (z) AZ_HIP(hipMemcpyAsync(z, e->p.s.z + start, n * 8, k, s));
  if (player) AZ_HIP(hipMemcpyAsync(player, e->p.s.player + start, n, k, s));
  if (slot) AZ_HIP(hipMemcpyAsync(slot, e->p.s.slot + start, n * 4, k, s));
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_clear_samples(az_engine* e, void* stream) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  hipStream_t s = azc::as_stream(stream);
  AZ_HIP(hipMemsetAsync(&e->p.ctr->samples_n, 0, sizeof(unsigned long long), s));
  AZ_HIP(hipStreamSynchronize(s));
  return AZ_OK;
}

int az_engine_geometry(az_engine* e, int32_t* n_games, int32_t* node_capacity,
                       int32_t* max_plies) {
  AZ_REQUIRE(e, AZ_ERR_ARG, "null engine");
  if (n_games) *n_games = e->p.G;
  if (node_capacity) *node_capacity = e->p.C;
  if (max_plies) *max_plies = e->p.T;
  return AZ_OK;
}

}  // extern "C"
