/* az_othello.h — C ABI of the MI355X-native Othello self-play engine.
 *
 * The reference (AfoninAndrei/alphaZero-Othello) is pure Python and has no FFI; its
 * drop-in surfaces are duck-typed Python classes.  Every entry point below replaces a
 * reference Python routine, cited as file:line into the reference tree.  The Python
 * host side (alphazero-othello_amd/envs, MCTS_model.py, self_play_worker.py) binds
 * these through ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - every function returns int: AZ_OK (0) or a negative AZ_ERR_* code; az_last_error()
 *     returns a thread-local message for the last failure on the calling thread.  No C++
 *     exception crosses the ABI.
 *   - buffers are caller-owned.  *_cpu functions take host pointers and are reentrant
 *     and stateless.  *_gpu functions take device pointers and are asynchronous on the
 *     given hipStream_t (passed as void*; NULL = the legacy default stream).
 *   - bitboard layout: bit r*8+c <-> square (r, c) of the row-major (8,8) state array
 *     (`_BitBoard` layout, envs/othello.py:202-212).  own = side to move.
 *   - a board step's status word (uint16): low byte = flags (AZ_FLAG_*), high byte =
 *     signed disc difference (side to move after the step minus its opponent).
 *   - an engine handle is NOT thread-safe: one owner thread per engine.
 */
#ifndef AZ_OTHELLO_H
#define AZ_OTHELLO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AZ_ABI_VERSION 1

enum {
  AZ_OK = 0,
  AZ_ERR_ILLEGAL = -1,  /* illegal placement (reference: ValueError, envs/othello.py:421) */
  AZ_ERR_ARG = -2,      /* bad argument / shape */
  AZ_ERR_HIP = -3,      /* HIP runtime failure */
  AZ_ERR_CAPACITY = -4, /* node arena / trajectory capacity exceeded */
  AZ_ERR_STATE = -5,    /* engine state does not allow the call (e.g. not a child: KeyError,
                           MCTS_model.py:214) */
};

enum {
  AZ_FLAG_TERMINAL = 1, /* neither side has a placement (envs/othello.py:435-454) */
  AZ_FLAG_NOPLACE = 2,  /* side to move has no placement: valid mask is {pass} */
  AZ_FLAG_ILLEGAL = 4,  /* the step's action was illegal; outputs = inputs */
  AZ_FLAG_PASSED = 8,   /* the step's action was the pass (64) */
};

const char* az_last_error(void);
int az_abi_version(void);
/* content hash (sha256 hex, 64 chars) of the sources and flags this library was compiled
 * from (alphazero-othello_amd/az_build.py source_hash()): which build a process loaded */
const char* az_build_id(void);

/* ---------------- stateless board entry points: host ---------------------------- */

/* legal placements of own vs opp.  Replaces _BitBoard._legal_moves / valid_mask
 * (envs/othello.py:157-169) and the core of OthelloGameNew.get_valid_moves (:394-411). */
int oth_legal_cpu(const uint64_t* own, const uint64_t* opp, uint64_t* legal_o, int64_t n);

/* one board step per position: act in 0..63 (placement) or 64 (pass).  Outputs are the
 * next side's (own, opp), its legal mask and the status word.  Replaces
 * OthelloGameNew.get_next_state (envs/othello.py:413-433) + _BitBoard.make_move
 * (:171-200) + get_value_and_terminated (:435-454) + _BitBoard.score (:214-220).
 * Returns AZ_ERR_ILLEGAL if any position had an illegal placement (its status carries
 * AZ_FLAG_ILLEGAL and its outputs equal its inputs); all other positions are valid. */
int oth_step_cpu(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
                 uint64_t* own_o, uint64_t* opp_o, uint64_t* legal_o, uint16_t* status_o,
                 int64_t n);

/* raw make-move without a legality check (pass = swap sides): replaces
 * _BitBoard.make_move (envs/othello.py:171-200), which places an unbounded stone with no
 * captures.  Outputs are the next side's (own, opp). */
int oth_make_move_cpu(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
                      uint64_t* own_o, uint64_t* opp_o, int64_t n);

/* int8 (n,8,8) absolute-colour states + int8 player[n] -> (own, opp) bitboards where
 * own = stones equal to player.  Replaces OthelloGameNew._np_to_bitboards
 * (envs/othello.py:358-371) in the row-major layout (no 180-degree rotation). */
int oth_pack_np(const int8_t* states, const int8_t* player, uint64_t* own, uint64_t* opp,
                int64_t n);

/* inverse of oth_pack_np: own stones -> player, opp stones -> -player.  Replaces
 * OthelloGameNew._bitboards_to_np (envs/othello.py:373-388). */
int oth_unpack_np(const uint64_t* own, const uint64_t* opp, const int8_t* player,
                  int8_t* states, int64_t n);

/* dihedral transform sym = k + 4*flip (np.rot90 k times, then np.fliplr if flip) of each
 * bitboard.  Replaces the D4 maps of get_random_symmetry (envs/othello.py:501-526) and
 * random_symmetry (MCTS_model.py:15-28). */
int oth_d4_cpu(const uint64_t* x, const uint8_t* sym, uint64_t* out, int64_t n);

/* ---------------- stateless board entry points: device --------------------------- */
int oth_legal_gpu(const uint64_t* own, const uint64_t* opp, uint64_t* legal_o, int64_t n,
                  void* stream);
/* oth_step_cpu on device, asynchronous on `stream` (device pointers, n < 2^28).  With
 * 16-byte aligned own/opp/own_o/opp_o/legal_o, a 2-byte aligned act and a 4-byte aligned
 * status_o (any torch allocation) it runs two positions per lane with 16-byte
 * non-temporal accesses; other alignments take a one-position-per-lane kernel with the
 * same results.  Illegal placements are reported in status (kFlagIllegal), not as an
 * error code. */
int oth_step_gpu(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
                 uint64_t* own_o, uint64_t* opp_o, uint64_t* legal_o, uint16_t* status_o,
                 int64_t n, void* stream);
int oth_d4_gpu(const uint64_t* x, const uint8_t* sym, uint64_t* out, int64_t n,
               void* stream);
/* Measurement probe, not a reference routine: oth_step_gpu's launch and access pattern
 * (17 B read, 26 B written per position, non-temporal, k_step2's grid) with no board
 * arithmetic -- own_o = opp, opp_o = own, legal_o = own | opp, status_o = the action pair.
 * bench.py times it beside oth_step_gpu as the pattern's ceiling on the box.  Needs
 * k_step2's alignment (AZ_ERR_ARG otherwise). */
int oth_step_io_gpu(const uint64_t* own, const uint64_t* opp, const uint8_t* act,
                    uint64_t* own_o, uint64_t* opp_o, uint64_t* legal_o, uint16_t* status_o,
                    int64_t n, void* stream);

/* ---------------- batched MCTS self-play engine (device) -------------------------
 * G game slots, each with its own flat SoA node arena (the reference's `Node` tree,
 * MCTS_model.py:46-169) in two ping-pong halves (live tree + re-root compaction target),
 * and a trajectory buffer.  One simulation step, all asynchronous on `stream` and
 * graph-capturable (no host synchronisation, no allocation):
 *   az_select        descend every active slot's tree to one leaf (PUCT of
 *                    MCTS_model.py:129-139 / :362-370; terminal leaves are backed up in
 *                    place, :381-384) and pack the leaf's canonical NN input;
 *   (caller)         policy/value net on nn_in -> priors (softmax), values (tanh);
 *   az_expand_backup eager expansion + backup (MCTS_model.py:325-360, :160-169);
 *   az_play          auto-play engines: every slot whose search finished plays its move
 *                    (pi, record, sample, move, terminal check, TD(lambda) targets, re-root;
 *                    MCTS_model.py:200-274, self_play_worker.py:8-88) and finished slots
 *                    restart while the start budget lasts.  Host-driven engines: only
 *                    advances the step counter.
 * With one leaf per slot per step the search is exactly the reference with
 * args['num_threads'] = 1. */

typedef struct az_engine az_engine;

enum { AZ_EVAL_EXTERNAL = 0, AZ_EVAL_ROLLOUT = 1 };
enum { AZ_RNG_DEVICE = 0, AZ_RNG_INJECTED = 1 };
enum { AZ_GAME_IDLE = 0, AZ_GAME_ACTIVE = 1, AZ_GAME_FINISHED = 2, AZ_GAME_SEARCH_DONE = 3 };

typedef struct az_config {
  int32_t n_games;               /* G concurrent game slots */
  int32_t node_capacity;         /* arena nodes per slot and half (0 -> 16384; <= 32768) */
  int32_t max_plies;             /* trajectory capacity per game (0 -> 128) */
  int32_t num_simulations;       /* args['num_simulations'] */
  double c_puct;                 /* args['c_puct'] */
  double dirichlet_alpha;        /* self_play_worker.py:56 */
  double dirichlet_epsilon;      /* self_play_worker.py:57; 0 disables root noise */
  double temperature;            /* args['mcts_temperature'] (self_play_worker.py:66-67) */
  int32_t num_exploratory_moves; /* args['num_exploratory_moves'] */
  double lambd;                  /* args['lambda'] (TD(lambda), self_play_worker.py:8-35) */
  int32_t eval_mode;             /* AZ_EVAL_EXTERNAL (net) or AZ_EVAL_ROLLOUT (policy None) */
  int32_t rng_mode;              /* AZ_RNG_DEVICE (Philox) or AZ_RNG_INJECTED (parity) */
  int32_t d4_augment;            /* 1: random D4 transform per leaf in the NN input pack,
                                    inverse-mapped priors (config #5) */
  int32_t auto_play;             /* 1: az_play plays moves on device (batched self-play);
                                    0: the host drives moves (MCTS class API) */
  int32_t refill;                /* auto-play: finished slots restart a fresh game */
  int64_t sample_capacity;       /* rows of the device sample buffer (0 -> 2*G*max_plies) */
  int32_t inj_noise_slots;       /* AZ_RNG_INJECTED: Dirichlet vectors per slot */
  int32_t inj_uniform_slots;     /* AZ_RNG_INJECTED: uniforms per slot */
  uint64_t seed;                 /* Philox key */
  uint64_t stream_id;            /* Philox sub-stream (rank) */
  int32_t leaves_per_step;       /* K in [1, 8] (0 -> 1): leaves per slot per step, the
                                    reference's args['num_threads'] workers with virtual loss
                                    (MCTS_model.py:115-118, :196-197, :372-395) in one fixed
                                    interleaving; 1 = its deterministic num_threads = 1 search.
                                    The evaluation batch is G*K rows (row g*K + j). */
} az_config;

int az_engine_create(const az_config* cfg, az_engine** out);
int az_engine_destroy(az_engine* eng);
int az_engine_geometry(az_engine* eng, int32_t* n_games, int32_t* node_capacity,
                       int32_t* max_plies);

/* every slot -> a fresh game at the initial position, player +1 (self_play_worker.py:
 * 59-61).  start_budget < 0: unlimited restarts; else at most start_budget games are ever
 * started (slots beyond it stay idle).  Slot g becomes active at step g*stagger/G.
 * Resets the counters.  Synchronous. */
int az_reset_all(az_engine* eng, int64_t start_budget, int32_t stagger_steps, void* stream);

/* slot -> root at an arbitrary position, tree discarded (MCTS.policy_improve_step with
 * root None, MCTS_model.py:223-228).  player in {+1,-1}.  Synchronous. */
int az_set_root(az_engine* eng, int32_t slot, uint64_t own, uint64_t opp, int32_t player,
                void* stream);

/* start a search of num_simulations on one slot (or all, slot = -1): MCTS_model.py:237. */
int az_begin_search(az_engine* eng, int32_t slot, int32_t num_simulations, void* stream);

/* up to K = leaves_per_step leaves per active slot.  nn_in: float [G*K,64], canonical
 * player*state (Models.py:16) of leaf j of slot g in row g*K + j, zeros for rows without a
 * leaf.  leaf_o (optional, int32 [G*K]): leaf node index or -1. */
int az_select(az_engine* eng, float* nn_in, int32_t* leaf_o, void* stream);

/* priors: float [G*K,65] (softmax output), values: float [G*K] (tanh output), rows as
 * az_select's; both ignored in rollout mode. */
int az_expand_backup(az_engine* eng, const float* priors, const float* values, void* stream);

/* auto-play move phase (see above); host-driven engines: step counter only. */
int az_play(az_engine* eng, void* stream);

/* Deferred moves (auto-play engines, reference self_play_worker.py:69-86 per game unchanged):
 * after az_engine_defer_moves(eng, 1) a step is az_select_move -> evaluation ->
 * az_expand_backup_par with the step's parity par (0, 1, 0, 1, ...), and there is no
 * az_play: the move phase of step n runs inside step n+1's az_select_move launch, in extra
 * workgroups beside the descents (which skip the slots being moved; they play again the step
 * after), so the two latency-bound phases overlap in one launch.  Each slot's games, samples
 * and random draws are those of the plain order; only the step a move lands in shifts.
 * az_move_flush(eng, par) applies the moves of the last step (parity par) before results are
 * read.  az_select / az_expand_backup / az_play refuse while deferral is on. */
int az_engine_defer_moves(az_engine* eng, int32_t on);

/* The evaluation's stem inside the select launch (replaces the net's first layer,
 * reference Models.py:179-180, :209, conv0 + bn0 + relu, BatchNorm folded): every row
 * az_select / az_select_move packs is also run through relu(conv3x3_{1->C}(row) + bias)
 * by the wave that packed it, into y (float [G*K][64][C], NHWC) and, if absmax is given,
 * its max |y| into absmax[row] -- bit-identical to az_conv_stem2_gpu on nn_in.
 * w9: float [9][C] tap-major, bias: float [C]; channels 64 or 128, 0 turns it off.  The
 * buffers must stay allocated while it is on. */
int az_engine_set_stem(az_engine* eng, const float* w9, const float* bias, float* y,
                       float* absmax, int32_t channels);
int az_select_move(az_engine* eng, float* nn_in, int32_t* leaf_o, int32_t par, void* stream);
int az_expand_backup_par(az_engine* eng, const float* priors, const float* values, int32_t par,
                         void* stream);
int az_move_flush(az_engine* eng, int32_t par, void* stream);

/* Deferred moves with the expansion fused too (round 3): a step is ONE launch,
 * az_select_move_expand(par) -> evaluation into priors / values, no az_expand_backup_par:
 * each slot's wave first expands and backs up the previous step's waiting leaves from
 * priors / values (the evaluation of that step), then descends; a search those leaves
 * complete is moved by the next launch (the slot sits one step out).  Same games, samples
 * and draws per slot as the plain order.  Before results are read:
 * az_expand_backup_par(par) then az_move_flush(par) for the last step's parity par.
 * Reference MCTS_model.py:325-360 (expand / evaluate / backup) with :372-395 (simulate). */
int az_select_move_expand(az_engine* eng, float* nn_in, int32_t* leaf_o, const float* priors,
                          const float* values, int32_t par, void* stream);

/* The same fusion for engines without deferred moves (the drop-in MCTS's host-driven
 * search): az_select_expand = the expansion of the previous az_select's leaves from priors /
 * values, then az_select's descents, in one launch; a search the expansion completes is
 * marked done and the launch emits no leaf for it.  az_expand_backup after the last one.
 * Reference MCTS_model.py:325-360 with :372-395. */
int az_select_expand(az_engine* eng, float* nn_in, int32_t* leaf_o, const float* priors,
                     const float* values, void* stream);

/* AZ_RNG_INJECTED: per-slot streams, noise double [G, inj_noise_slots, 65] (Dirichlet
 * vectors, consumed at each root expansion with epsilon > 0) and uniforms double
 * [G, inj_uniform_slots] (consumed by the temperature-0 tie break and the action sample,
 * in the reference's np.random call order).  Resets the cursors.  Synchronous. */
int az_inject(az_engine* eng, const double* noise, const double* uniforms, void* stream);

/* pi of one slot's root (MCTS_model.py:244-271) at temperature `temp`; u_tie in [0,1)
 * picks among tied maxima at temp < 0.1 (index floor(u_tie * n_ties)).  Optional outputs:
 * counts int32[65] (child visit counts), vroot (root W/N).  Synchronous. */
int az_root_policy(az_engine* eng, int32_t slot, double temp, double u_tie, float* pi_o,
                   int32_t* counts_o, double* vroot_o, void* stream);

/* re-root one slot on the child reached by `action`, keeping its subtree and statistics
 * (MCTS.make_move, MCTS_model.py:200-215): AZ_ERR_STATE if the root has no such child
 * (KeyError in the reference).  Synchronous. */
int az_make_move(az_engine* eng, int32_t slot, int32_t action, void* stream);

/* ---- batched host-driven control (many independent searches, e.g. arena matches,
 * eval.py:46-178).  Host arrays; synchronous. ---- */
/* roots of n slots at arbitrary positions (as az_set_root, one call). */
int az_set_roots(az_engine* eng, const int32_t* slots, const uint64_t* own, const uint64_t* opp,
                 const int32_t* player, int32_t n, void* stream);
/* start a search of num_simulations on each listed slot. */
int az_begin_search_slots(az_engine* eng, const int32_t* slots, int32_t n,
                          int32_t num_simulations, void* stream);
/* child visit counts int32 [G, 65] (the `counts` of MCTS_model.py:244-247) and root W/N
 * double [G] (vroot may be NULL) of every slot. */
int az_root_stats(az_engine* eng, int32_t* counts, double* vroot, void* stream);
/* MCTS.make_move on every slot with actions[g] >= 0 (int32 [G]); found[g] = the child
 * that became the root, or -1 when the root has no such child (KeyError,
 * MCTS_model.py:214) or actions[g] < 0 — that slot's tree is then unchanged. */
int az_reroot_slots(az_engine* eng, const int32_t* actions, int32_t* found, void* stream);

/* counters: [games_started, games_finished, samples, samples_dropped, arena_overflows,
 * steps, simulations, moves].  Synchronous. */
int az_counters(az_engine* eng, int64_t* out8, void* stream);

/* host copies of per-slot state (int32 [G] each): status (AZ_GAME_*), ply, winner
 * (+1/-1/0), root player, nodes in use, arena overflow count.  Any pointer may be NULL. */
int az_game_info(az_engine* eng, int32_t* status, int32_t* ply, int32_t* winner,
                 int32_t* root_player, int32_t* n_nodes, int32_t* overflow, void* stream);

/* host copy of one slot's tree (root = node 0; children contiguous, ascending action):
 * bitboards (side to move), visit count, value sum, prior, parent, first child, child
 * count, action, flags (bit0 expanded, bit1 terminal, bit2 float64 child priors),
 * terminal value.  Any pointer may be NULL.  Synchronous. */
int az_export_tree(az_engine* eng, int32_t slot, int32_t max_nodes, uint64_t* own,
                   uint64_t* opp, uint64_t* legal, int32_t* N, double* W, double* prior,
                   int32_t* parent, int32_t* first_child, uint8_t* nchild, uint8_t* action,
                   uint8_t* flags, int8_t* tval, int32_t* n_nodes_o, void* stream);

/* host copy of one slot's trajectory: canonical own/opp (state*player,
 * self_play_worker.py:72), pi float[65], player, root value.  Synchronous. */
int az_export_trajectory(az_engine* eng, int32_t slot, int32_t max_plies, uint64_t* own,
                         uint64_t* opp, float* pi, int8_t* player, double* vroot,
                         int32_t* n_plies_o, void* stream);

/* device sample buffer (TD(lambda) rows of finished games, get_training_data,
 * self_play_worker.py:8-35): canonical own/opp u64, pi float[65], z double, player int8.
 * Device pointers owned by the engine. */
int az_samples(az_engine* eng, uint64_t** own, uint64_t** opp, float** pi, double** z,
               int8_t** player, int64_t* n, int64_t* capacity);
/* copy sample rows [start, start+n) to host or device buffers (any pointer may be NULL);
 * slot = the game slot that produced each row.  Synchronous. */
int az_copy_samples(az_engine* eng, int64_t start, int64_t n, uint64_t* own, uint64_t* opp,
                    float* pi, double* z, int8_t* player, int32_t* slot, void* stream);
int az_clear_samples(az_engine* eng, void* stream);

/* ---------------- leaf-evaluation net support (device) ---------------------------
 * Fused conv epilogue of the inference copy of the policy/value net (reference
 * Models.py:72-221 with BatchNorm folded): y = act(y + bias[c] (+ res)) in place over an
 * NHWC (channels-last) float32 activation of n elements and `channels` channels; res may
 * be NULL; relu 0/1.  Replaces the conv bias add, `out += residual` (Models.py:84-86) and
 * F.relu as separate passes. */
int az_bias_act_gpu(float* y, const float* bias, const float* res, int64_t n,
                    int32_t channels, int32_t relu, void* stream);

/* 3x3 convolution, padding 1, over n_boards 8x8 boards, Ci = Co = channels (64 or 128),
 * fp32 MFMA, fused epilogue: y = act(conv(x, w) + bias (+ res)).  x, res, y: NHWC float
 * [n_boards, 8, 8, C]; w9: [9 taps (ky*3+kx)][Co][Ci]; res may be NULL; x != y.  Replaces
 * ResidualBlock.conv1/conv2 + BatchNorm (folded) + skip + ReLU (Models.py:72-90) and
 * FastOthelloNet.conv_add (Models.py:119-121). */
int az_conv3x3_gpu(const float* x, const float* w9, const float* bias, const float* res,
                   float* y, int32_t n_boards, int32_t channels, int32_t relu, void* stream);

/* the same convolution with an explicit tiling candidate `cfg` (benchmarking; 0 = the
 * default tiling used by az_conv3x3_gpu). */
int az_conv3x3_cfg_gpu(const float* x, const float* w9, const float* bias, const float* res,
                       float* y, int32_t n_boards, int32_t channels, int32_t relu, int32_t cfg,
                       void* stream);

/* The same convolution on the 16-bit MFMA pipe (csrc/conv16.hip).  mode:
 *   AZ_CONV_SPLIT3 — fp32-accurate: each fp32 operand split into three bf16 words, the six
 *                    leading partial products accumulated in fp32 (error at fp32's own
 *                    rounding unit; tests/test_nn_gpu.py measures it against fp64);
 *   AZ_CONV_FP16   — one fp16 product (BASELINE configs[4], fp16 inference);
 *   AZ_CONV_FP16X2 — fp32-accurate with half of SPLIT3's products: both operands as an fp16
 *                    pair hi + lo after exact power-of-two scaling (the weights per layer,
 *                    from the prep's header; the inputs per board, from the board's max |x|
 *                    reduced inside the kernel), three products accumulated in fp32, the
 *                    scales removed exactly in the epilogue (FastOthelloNet's 64-channel
 *                    convs, configs[1]).
 * wq: the weights re-laid by az_conv3x3_mx_prep_gpu from w9 [9][Co][Ci] fp32 into
 * [9][Ci/16][planes][Co][16] 16-bit words (planes = 3 for SPLIT3, 1 for FP16, 2 for FP16X2;
 * 16-byte aligned, az_conv3x3_mx_prep_bytes: 9*C*C*planes*2 bytes plus, for FP16X2, a
 * 16-byte scale header after the words).  Replaces the same reference layers as
 * az_conv3x3_gpu. */
enum { AZ_CONV_SPLIT3 = 0, AZ_CONV_FP16 = 1, AZ_CONV_FP16X2 = 2 };
int az_conv3x3_mx_prep_gpu(const float* w9, void* wq, int32_t channels, int32_t mode,
                           void* stream);
int64_t az_conv3x3_mx_prep_bytes(int32_t channels, int32_t mode);
int az_conv3x3_mx_gpu(const float* x, const void* wq, const float* bias, const float* res,
                      float* y, int32_t n_boards, int32_t channels, int32_t relu, int32_t mode,
                      void* stream);
/* the same with an explicit workgroup shape (benchmarking): cfg 0 = 2 boards per workgroup
 * (the default), 1 = 1 board. */
int az_conv3x3_mx_cfg_gpu(const float* x, const void* wq, const float* bias, const float* res,
                          float* y, int32_t n_boards, int32_t channels, int32_t relu,
                          int32_t mode, int32_t cfg, void* stream);

/* az_conv3x3_mx_gpu (1-board workgroups, relu) fused with the stem (1 -> channels 3x3 conv
 * + bias + ReLU of az_conv_stem_gpu, same fmaf chain, bit-identical) so the stem output is
 * never stored: role 1 — the input is stem(planes) (x unused, no residual; the first
 * residual block's conv1); role 2 — the input is x and the residual is stem(planes) (that
 * block's conv2).  planes float [n_boards][64]; stem_w [9][channels]; stem_b [channels].
 * Replaces conv0+bn0+relu (Models.py:186-187) / initial_conv (:103-105) plus the first
 * block's convolutions. */
int az_conv3x3_mx_stem_gpu(const float* planes, const float* stem_w, const float* stem_b,
                           const float* x, const void* wq, const float* bias, float* y,
                           int32_t n_boards, int32_t channels, int32_t role, int32_t mode,
                           void* stream);

/* FastOthelloNet's whole conv trunk in one launch (csrc/conv16.hip, k_fast_trunk): the stem
 * (planes float [n_boards][64], stem_w [9][64], stem_b [64]), the residual block's conv1
 * (wq1 / bias1) and conv2 (wq2 / bias2, + the stem output, ReLU) and conv_add (wq3 / bias3),
 * each conv + bias + ReLU in FP16X2 (weights from az_conv3x3_mx_prep_gpu with
 * AZ_CONV_FP16X2); y NHWC float [n_boards][64][64] = conv_add's output.  One board per
 * workgroup: the activations between the convs stay in LDS (each epilogue writes the next
 * conv's fp16 hi / lo image from its registers), bit-identical to az_conv3x3_mx_stem_gpu
 * (role 1), az_conv3x3_mx_stem_gpu (role 2) and az_conv3x3_mx_gpu in sequence.  channels must
 * be 64 and mode AZ_CONV_FP16X2.  Replaces initial_conv, res_block and conv_add
 * (Models.py:103-116, 144-146). */
int az_fast_trunk_gpu(const float* planes, const float* stem_w, const float* stem_b,
                      const void* wq1, const float* bias1, const void* wq2, const float* bias2,
                      const void* wq3, const float* bias3, float* y, int32_t n_boards,
                      int32_t channels, int32_t mode, void* stream);

/* The same convolution as Winograd F(2x2, 3x3) (csrc/conv_wino.hip): 2.25x fewer MFMA
 * products; the input/output transforms only add and subtract and the weight transform
 * G g G^T is done once in fp64, so SPLIT3 stays at the direct fp32 kernel's error (the
 * test bar of az_conv3x3_mx_gpu).  wq: from az_conv3x3_wino_prep_gpu (w9 [9][Co][Ci] fp32
 * -> [Ci/16][16 points][planes][Co][16] 16-bit words, 16*C*C*planes*2 bytes, 16-byte
 * aligned).  Two boards per workgroup, 96 KiB LDS.  Same reference layers as
 * az_conv3x3_gpu. */
int az_conv3x3_wino_prep_gpu(const float* w9, void* wq, int32_t channels, int32_t mode,
                             void* stream);
/* wq size in bytes for az_conv3x3_wino_prep_gpu: 16*C*C*planes*2 (planes 3 / 1 / 2 for
 * SPLIT3 / FP16 / FP16X2) plus, for FP16X2, 16 bytes of scale header after the words. */
int64_t az_conv3x3_wino_prep_bytes(int32_t channels, int32_t mode);
int az_conv3x3_wino_gpu(const float* x, const void* wq, const float* bias, const float* res,
                        float* y, int32_t n_boards, int32_t channels, int32_t relu,
                        int32_t mode, void* stream);

/* The same op, weights (az_conv3x3_wino_prep_gpu layout) and modes as az_conv3x3_wino_gpu
 * at 128 channels (csrc/conv_wino4.hip): four boards per workgroup, the transform points
 * visited row by row with the output transform folded after each row's K loop, so each
 * streamed weight fragment feeds twice the boards.  One more mode:
 *   AZ_CONV_FP16X2 — fp32-accurate with half the products of SPLIT3: both operands as an
 *                    fp16 pair hi + lo (22 significant bits) after exact power-of-two
 *                    scaling (weights per layer, from az_conv3x3_wino_prep_gpu; inputs per
 *                    board, from in_absmax), the three leading products accumulated in fp32
 *                    and the scale removed exactly in the epilogue.
 * in_absmax: float [n_boards] max |x| of each board (required for FP16X2, ignored
 * otherwise; CONSUMED: the kernel resets its entries to 0).  out_absmax: NULL or float
 * [n_boards] holding zeros: receives max |y| of each output board (the next layer's
 * in_absmax).  Replaces the same reference layers (Models.py:72-90 ResidualBlock convs). */
int az_conv3x3_wino4_gpu(const float* x, const void* wq, const float* bias, const float* res,
                         float* y, int32_t n_boards, int32_t channels, int32_t relu,
                         int32_t mode, float* in_absmax, float* out_absmax, void* stream);

/* The LAST trunk conv (residual + ReLU) of an AlphaZeroNet in FP16X2 mode with the policy and
 * value heads fused into its epilogue: the trunk output stays in LDS and the workgroup's
 * four boards run az_heads_az_gpu's computation on it (csrc/heads_az.h, the same code on the
 * same values: priors and values bit-identical to az_conv3x3_wino4_gpu followed by
 * az_heads_az_gpu).  Same conv arguments as az_conv3x3_wino4_gpu without y / out_absmax
 * (in_absmax consumed); heads weights, priors and values as az_heads_az_gpu.  Replaces the
 * reference's last ResidualBlock conv2 + both heads (Models.py:72-90, 196-221). */
int az_conv3x3_wino4_heads_gpu(const float* x, const void* wq, const float* bias,
                               const float* res, int32_t n_boards, int32_t channels,
                               int32_t mode, float* in_absmax, const float* wpv,
                               const float* bpv, const float* wpolT, const float* bpol,
                               const float* w1T, const float* b1, const float* w2,
                               const float* b2, float* priors, float* values, void* stream);

/* az_conv3x3_wino4_gpu (FP16X2, 128 channels) for small batches -- a search's few leaves per
 * step, where one workgroup per four boards leaves the chip idle: the 128 input channels are
 * split over 2, 4 or 8 workgroups per board group (splits = 16 or 32 also split the four
 * Winograd transform rows, 4 x 4 or 4 x 8), each writing its partial sums to part (float
 * [splits][n_boards][64][128]), and a second kernel adds the splits in order with bias /
 * residual / ReLU and the max |y| of each board.  Same in_absmax / out_absmax contract; fp32
 * sums of the same products in a different order (not bit-identical to the one-pass
 * kernel). */
int az_conv3x3_wino4_splitk_gpu(const float* x, const void* wq, const float* bias,
                                const float* res, float* y, int32_t n_boards, int32_t channels,
                                int32_t relu, int32_t mode, float* in_absmax, float* out_absmax,
                                float* part, int32_t splits, void* stream);

/* out[b] = max |x[b][.]| over each board's 64 * channels fp32 values (NHWC): the
 * in_absmax of az_conv3x3_wino4_gpu for a tensor no kernel produced it for. */
int az_board_absmax_gpu(const float* x, int32_t n_boards, int32_t channels, float* out,
                        void* stream);

/* The whole residual trunk of AlphaZeroNet / FastOthelloNet in one launch
 * (csrc/conv_wino.hip): the stem (az_conv_stem_gpu's arithmetic) then n_blocks residual
 * blocks of two Winograd convolutions (az_conv3x3_wino_gpu's arithmetic: conv + ReLU, conv +
 * residual + ReLU), bit-identical to those launches one layer at a time.  Each workgroup
 * carries whole board pairs through every layer (a conv mixes positions within a board
 * only), so no grid-wide barrier is needed.  planes float [n][64]; stem_w [9][C]; stem_b
 * [C]; wq / bias: device arrays of 2*n_blocks device pointers (az_conv3x3_wino_prep_gpu
 * weights, fp32 biases) in layer order; h [n][64][C] receives the trunk output (NHWC), t
 * [n][64][C] is scratch.  Replaces reference Models.py:209-210 (relu(bn0(conv0)) and the res
 * tower, AlphaZeroNet.forward) / :147-148 (initial_conv + res_block, the FastOthelloNet
 * forward). */
int az_trunk_wino_gpu(const float* planes, const float* stem_w, const float* stem_b,
                      const void* const* wq, const float* const* bias, float* h, float* t,
                      int32_t n_boards, int32_t n_blocks, int32_t channels, int32_t mode,
                      void* stream);

/* The fp16x2 residual tower as one persistent launch (csrc/conv_wino4.hip, round 3): each
 * two-board workgroup runs n_convs consecutive block convs on its own boards -- conv 2i:
 * relu(conv(h)) -> t, conv 2i+1: relu(conv(t) + h) -> hb0 / hb1 alternately (the first
 * block's output in hb0) -- with az_conv3x3_wino4_gpu's arithmetic per layer (bit-identical
 * to those launches), no grid-wide barrier (a conv mixes positions within a board only).
 * h_in [n][64][128] NHWC = the stem output (read only); amax0 = its per-board max |x| on
 * entry, amax1 zeros.  With planes (float [n][64], the canonical boards) and the stem's
 * stem_w [9][128] / stem_b [128], the kernel first runs the stem on each workgroup's boards
 * (az_conv_stem_gpu's arithmetic, bit-identical) into h_in and amax0 (then written, and
 * n_convs may be 0); on return the ranges of the last output are in amax1 (n_convs odd:
 * t) or amax0 (even: the last block output), the other zeroed.  wq / bias: device arrays of
 * n_convs device pointers (az_conv3x3_wino_prep_gpu FP16X2 weights, fp32 biases) in layer
 * order.  Replaces reference Models.py:209-210 (AlphaZeroNet.forward's res tower); an odd
 * n_convs leaves the last block's second conv to az_conv3x3_wino4_heads_gpu. */
int az_trunk_wino4_gpu(const void* const* wq, const float* const* bias, const float* planes,
                       const float* stem_w, const float* stem_b, float* h_in, float* hb0,
                       float* hb1, float* t, float* amax0, float* amax1, int32_t n_boards,
                       int32_t n_convs, int32_t channels, void* stream);

/* az_trunk_wino4_gpu with the tower's last conv (n_convs even: every block, the last
 * block's second conv included) running AlphaZeroNet's policy / value heads in its epilogue,
 * exactly az_conv3x3_wino4_heads_gpu's (heads weights and outputs as there): the whole net
 * after the stem in one launch, the last layer's output never stored.  priors [n][65] /
 * values [n] bit-identical to az_trunk_wino4_gpu (n_convs - 1) + az_conv3x3_wino4_heads_gpu
 * and to the separate az_heads_az_gpu.  Replaces reference Models.py:205-221
 * (AlphaZeroNet.forward after conv0) + the softmax of MCTS_model.py:319. */
int az_trunk_wino4_heads_gpu(const void* const* wq, const float* const* bias,
                             const float* planes, const float* stem_w, const float* stem_b,
                             float* h_in, float* hb0, float* hb1, float* t, float* amax0,
                             float* amax1, int32_t n_boards, int32_t n_convs, int32_t channels,
                             const float* wpv, const float* bpv, const float* wpolT,
                             const float* bpol, const float* w1T, const float* b1,
                             const float* w2, const float* b2, float* priors, float* values,
                             void* stream);

/* az_trunk_wino4_heads_gpu in fp16 (configs[4]'s fp16 inference): one fp16 product per
 * MFMA step, no operand scaling, the block convs' weights prepared for the fp16 wino4 conv
 * (az_conv3x3_wino_prep_gpu with AZ_CONV_FP16); same buffers and heads.  Bit-identical to the
 * per-layer fp16 wino4 convs + the separate heads kernel.  Replaces the same reference span
 * (Models.py:205-221) at configs[4]'s precision. */
int az_trunk_wino4_heads_fp16_gpu(const void* const* wq, const float* const* bias,
                                  const float* planes, const float* stem_w, const float* stem_b,
                                  float* h_in, float* hb0, float* hb1, float* t, float* amax0,
                                  float* amax1, int32_t n_boards, int32_t n_convs,
                                  int32_t channels, const float* wpv, const float* bpv,
                                  const float* wpolT, const float* bpol, const float* w1T,
                                  const float* b1, const float* w2, const float* b2,
                                  float* priors, float* values, void* stream);

/* ---------------- replay buffer (device) -------------------------------------------
 * Trainer._aggregate_duplicates (reference train.py:142-173) on bitboard rows: rows with
 * equal (own, opp, version) — the reference's (sha1(canonical int8 board), version) —
 * collapse to one sample, emitted in order of first occurrence: pi_o = mean pi
 * normalised by (its NumPy-pairwise sum + 1e-12) in float32, v_o = float32(mean v),
 * count_o = group size; *n_out (device int32) = number of samples.  Inputs: own/opp
 * [n], ver [n], pi [n][65] float, v [n] double.  Outputs sized n (the upper bound).
 * Call with workspace = NULL to get *workspace_bytes, then again with that much device
 * memory.  Asynchronous on `stream`. */
int az_replay_aggregate_gpu(const uint64_t* own, const uint64_t* opp, const int32_t* ver,
                            const float* pi, const double* v, int64_t n, uint64_t* own_o,
                            uint64_t* opp_o, int32_t* ver_o, float* pi_o, float* v_o,
                            int32_t* count_o, int32_t* n_out, void* workspace,
                            size_t* workspace_bytes, void* stream);

/* AlphaZeroNet's policy and value heads in one kernel (reference Models.py:196-221 with
 * BatchNorm folded, softmax of MCTS_model.py:319): h NHWC float [n_boards, 8, 8, C];
 * wpv [3][C] (rows: policy ch 0, policy ch 1, value) and bpv [3] the 1x1 convs; wpolT
 * [128][65] = pol_fc.weight^T, bpol [65]; w1T [64][256] = val_fc1.weight^T, b1 [256];
 * w2 [256], b2 [1] = val_fc2.  Writes priors [n_boards][65] (softmax) and values
 * [n_boards] (tanh).  16-byte aligned h / wpv / w1T / b1 / w2. */
int az_heads_az_gpu(const float* h, const float* wpv, const float* bpv, const float* wpolT,
                    const float* bpol, const float* w1T, const float* b1, const float* w2,
                    const float* b2, float* priors, float* values, int32_t n_boards,
                    int32_t channels, void* stream);

/* FastOthelloNet's heads after their input GEMMs (reference Models.py:106-112, softmax of
 * MCTS_model.py:319): logits float [parts][n_boards][ld] (ld >= 129) = the flattened tail
 * output x [fc_policy; fc_value1]^T split over `parts` slices of the reduction (columns 0..64
 * policy logits, 65..128 the value hidden layer before its ReLU), summed here in part order,
 * then + bias [129]; w2 [64], b2 [1] = fc_value2.  Writes priors [n_boards][65] (softmax) and
 * values [n_boards] (tanh). */
int az_heads_fast_finish_gpu(const float* logits, int32_t ld, int32_t parts, const float* bias,
                             const float* w2, const float* b2, float* priors, float* values,
                             int32_t n_boards, void* stream);

/* FastOthelloNet's heads GEMM before az_heads_fast_finish_gpu (csrc/heads.hip): part
 * [splits][n_boards][ld] float = the partial sums over `splits` slices of K = 4,096 of
 * x[b][k] * W[k][n] for the 129 columns [fc_policy; fc_value1] (columns 129 .. ld-1 zeroed),
 * fp32-accurate on the 16-bit MFMA pipe: x = the tail conv's NHWC output [n_boards][4,096]
 * (k = square * 64 + channel), each board's slice scaled by a power of two from its max |x|
 * and split into fp16 hi / lo inside the kernel; wq = columns 0..127 of W * 2^wshift split
 * into fp16 hi / lo words laid out [K/16][2][128][16] (16-byte aligned); w128 = column 128 of
 * W in fp32 [4,096] (fp32 FMAs).  Three MFMA products (lo*hi, hi*lo, hi*hi), fp32
 * accumulation, both scales removed exactly.  Replaces the reference's fc_policy / fc_value1
 * (Models.py:118-124, 150-156).  board_tile = boards per workgroup (32 R: each weight fragment
 * feeds R MFMA row tiles); (board_tile, splits) one of (32, 4), (32, 8), (64, 8), (64, 16),
 * (128, 16). */
int az_heads_fast_gemm_gpu(const float* x, const void* wq, const float* w128, int32_t wshift,
                           float* part, int32_t ld, int32_t splits, int32_t board_tile,
                           int32_t n_boards, void* stream);

/* stem: 1 -> channels 3x3 conv + bias + ReLU on canonical planes float [n_boards, 64];
 * w9: [9][channels]; y NHWC.  Replaces conv0+bn0+relu / initial_conv (Models.py:103-105,
 * 186-187). */
int az_conv_stem_gpu(const float* planes, const float* w9, const float* bias, float* y,
                     int32_t n_boards, int32_t channels, void* stream);
/* the same with each board's max |y| written to absmax[b] (NULL: not computed): the
 * in_absmax of the first trunk conv in FP16X2 mode (az_conv3x3_wino4_gpu) */
int az_conv_stem2_gpu(const float* planes, const float* w9, const float* bias, float* y,
                      int32_t n_boards, int32_t channels, float* absmax, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AZ_OTHELLO_H */
