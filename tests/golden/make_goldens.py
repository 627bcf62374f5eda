"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Runs only in the build container, where the reference tree is mounted read-only at
/root/reference (PYTHONDONTWRITEBYTECODE keeps it untouched).  The GPU box never sees
the reference: it only reads the committed .npz/.json outputs of this script.

    python tests/golden/make_goldens.py            # all fixtures
    python tests/golden/make_goldens.py board mcts # a subset

Fixtures (all boards stored as bitboards in the row-major layout bit r*8+c, with
pos = squares holding +1, neg = squares holding -1 of the absolute-colour state):

  board_corpus.npz    random + lowest-index playouts through OthelloGameNew
                      (envs/othello.py:309-498): valid masks, next states,
                      get_value_and_terminated for both sides, get_score, and the
                      180-degree `_np_to_bitboards` layout for every position.
  bitboard_vectors.npz `_BitBoard` (envs/othello.py:129-220) on random disjoint boards:
                      valid_mask, make_move for every legal square, score.
  edge_cases.npz      pass-only / full / empty / wrap-around / illegal-action tables.
  d4.npz              OthelloGame.get_symmetries (envs/othello.py:286-298) and
                      MCTS_model.random_symmetry / unsymmetrise_pi (:15-43) index maps.
  mcts_cases.npz      reference MCTS (MCTS_model.py) with args['num_threads']=1 and the
                      deterministic mock policy (tests/mock_policy.py): root child visit
                      counts, root value, pi, and the recorded RNG draws.
  selfplay_games.npz  reference one_self_play (self_play_worker.py:38-88) with the mock
                      policy: trajectories, targets, recorded RNG draws.
  training_data.npz   reference get_training_data (self_play_worker.py:8-35) on synthetic
                      trajectories with passes, lambda in {0.98, 1.0}.
  tictactoe_stats.json outcome distribution of rollout self-play on a copy-on-step
                      TicTacToe (statistical pin only).
  augment.npz         reference envs.othello.get_random_symmetry (envs/othello.py:501-526)
                      on canonical boards + policies, with the (k, flip) it drew.
  replay_aggregate.npz reference Trainer._aggregate_duplicates (train.py:142-173) on a
                      synthetic replay buffer with duplicate boards within and across
                      model versions: inputs and the (state, mean pi, mean v) outputs in
                      the reference's first-occurrence order.
"""
import json
import os
import sys
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))  # tests/ (mock_policy)
sys.path.insert(0, REF)

from mock_policy import MockPolicy, MockPolicyNet  # noqa: E402


def bb_from_state(state):
    flat = np.asarray(state).reshape(-1)
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    pos = np.bitwise_or.reduce(np.where(flat == 1, w, np.uint64(0)))
    neg = np.bitwise_or.reduce(np.where(flat == -1, w, np.uint64(0)))
    return np.uint64(pos), np.uint64(neg)


def mask_from_valid(valid):
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    return np.uint64(np.bitwise_or.reduce(np.where(np.asarray(valid)[:64] != 0, w,
                                                   np.uint64(0))))


# ----------------------------------------------------------------------------------------
def gen_board():
    from envs.othello import OthelloGameNew

    g = OthelloGameNew(8)
    rec = {k: [] for k in ("game", "ply", "pos", "neg", "player", "valid", "pass_only",
                           "action", "npos", "nneg", "val_next", "term_next", "val_mover",
                           "term_mover", "score_p1", "rot_own", "rot_opp")}

    def play(game_id, chooser):
        state = g.get_initial_state()
        player = 1
        for ply in range(200):
            valid = g.get_valid_moves(state, player)
            acts = np.nonzero(valid)[0]
            a = int(chooser(acts))
            nxt = g.get_next_state(state, a, player)
            vn, tn = g.get_value_and_terminated(nxt, a, -player)
            vm, tm = g.get_value_and_terminated(nxt, a, player)
            ro, rp = OthelloGameNew._np_to_bitboards(state, player)
            p, n = bb_from_state(state)
            np_, nn_ = bb_from_state(nxt)
            for k, v in (("game", game_id), ("ply", ply), ("pos", p), ("neg", n),
                         ("player", player), ("valid", mask_from_valid(valid)),
                         ("pass_only", int(valid[64])), ("action", a), ("npos", np_),
                         ("nneg", nn_), ("val_next", vn), ("term_next", int(tn)),
                         ("val_mover", vm), ("term_mover", int(tm)),
                         ("score_p1", g.get_score(nxt, 1)), ("rot_own", ro),
                         ("rot_opp", rp)):
                rec[k].append(v)
            state = nxt
            player = -player
            if tn:
                return
        raise RuntimeError("game did not end")

    play(0, lambda acts: acts.min())  # envs/test_equivalence_game.py:117-150 logic
    for first in (19, 26, 37, 44):    # the four openings, then lowest-index
        it = iter([first])
        play(1 + [19, 26, 37, 44].index(first), lambda acts, it=it: next(it, acts.min()))
    n_games = 600
    for gid in range(n_games):
        rng = np.random.default_rng(1000 + gid)
        play(5 + gid, lambda acts, rng=rng: rng.choice(acts))
    out = {}
    for k, v in rec.items():
        dt = np.uint64 if k in ("pos", "neg", "valid", "npos", "nneg", "rot_own",
                                "rot_opp") else np.int32
        out[k] = np.asarray(v, dtype=dt)
    np.savez_compressed(os.path.join(HERE, "board_corpus.npz"), **out)
    print("board_corpus:", len(out["pos"]), "plies")


# ----------------------------------------------------------------------------------------
def gen_bitboard():
    from envs.othello import _BitBoard

    rng = np.random.default_rng(7)
    n = 4000
    blacks, whites, masks, scores = [], [], [], []
    mv_idx, mv_sq, mv_b, mv_w = [], [], [], []
    for i in range(n):
        # random disjoint boards of varying density (many are unreachable in play)
        dens = rng.uniform(0.05, 0.95)
        occ = rng.random(64) < dens
        col = rng.random(64) < rng.uniform(0.2, 0.8)
        w = np.uint64(1) << np.arange(64, dtype=np.uint64)
        b = np.uint64(np.bitwise_or.reduce(np.where(occ & col, w, np.uint64(0))))
        wh = np.uint64(np.bitwise_or.reduce(np.where(occ & ~col, w, np.uint64(0))))
        bb = _BitBoard()
        bb.black, bb.white = b, wh
        m = bb.valid_mask()
        blacks.append(b)
        whites.append(wh)
        masks.append(m)
        scores.append(bb.score())
        mm = int(m)
        while mm:
            sq = (mm & -mm).bit_length() - 1
            mm &= mm - 1
            b2 = _BitBoard()
            b2.black, b2.white = b, wh
            b2.make_move(sq)
            mv_idx.append(i)
            mv_sq.append(sq)
            mv_b.append(b2.black)
            mv_w.append(b2.white)
        if i % 4 == 0:  # pass
            b2 = _BitBoard()
            b2.black, b2.white = b, wh
            b2.make_move(64)
            mv_idx.append(i)
            mv_sq.append(64)
            mv_b.append(b2.black)
            mv_w.append(b2.white)
    np.savez_compressed(os.path.join(HERE, "bitboard_vectors.npz"),
                        black=np.asarray(blacks, np.uint64),
                        white=np.asarray(whites, np.uint64),
                        valid=np.asarray(masks, np.uint64),
                        score=np.asarray(scores, np.int32),
                        mv_board=np.asarray(mv_idx, np.int32),
                        mv_sq=np.asarray(mv_sq, np.int32),
                        mv_black=np.asarray(mv_b, np.uint64),
                        mv_white=np.asarray(mv_w, np.uint64))
    print("bitboard_vectors:", n, "boards,", len(mv_idx), "moves")


# ----------------------------------------------------------------------------------------
def gen_edge():
    from envs.othello import OthelloGameNew, _BitBoard

    g = OthelloGameNew(8)
    out = {}
    # pass-only position of envs/test_equivalence_game.py:241-248
    s = np.zeros((8, 8), np.int8)
    s[:4, :4] = 1
    s[:4, 4:] = 1
    s[4:, :4] = 1
    vm = g.get_valid_moves(s, -1)
    out["passonly_pos"], out["passonly_neg"] = bb_from_state(s)
    out["passonly_valid_m1"] = vm
    out["passonly_valid_p1"] = g.get_valid_moves(s, 1)
    out["passonly_term_m1"] = np.array(g.get_value_and_terminated(s, 64, -1))
    # full / empty / single-stone terminal cases (envs/test_equivalence_game.py:350-363)
    cases = []
    full = np.ones((8, 8), np.int8)
    full[::2, ::3] = -1
    for st in (np.zeros((8, 8), np.int8), full, np.pad(np.ones((1, 1), np.int8), ((0, 7), (0, 7)))):
        for pl in (1, -1):
            v, t = g.get_value_and_terminated(st, 64, pl)
            p, n = bb_from_state(st)
            cases.append((p, n, pl, v, int(t), g.get_score(st, pl)))
    out["term_cases"] = np.array([[int(c[0]), int(c[1])] for c in cases], dtype=np.uint64)
    out["term_meta"] = np.array([c[2:] for c in cases], dtype=np.int32)
    # illegal-action table: every action on a set of reachable positions
    rng = np.random.default_rng(3)
    pos_list, legal_tab = [], []
    for k in range(60):
        state, player = g.get_initial_state(), 1
        for _ in range(int(rng.integers(0, 50))):
            acts = np.nonzero(g.get_valid_moves(state, player))[0]
            a = int(rng.choice(acts))
            state = g.get_next_state(state, a, player)
            player = -player
            if g.get_value_and_terminated(state, a, player)[1]:
                break
        row = []
        for a in range(65):
            try:
                g.get_next_state(state, a, player)
                row.append(1)
            except ValueError:
                row.append(0)
        p, n = bb_from_state(state)
        pos_list.append((int(p), int(n), player))
        legal_tab.append(row)
    out["illegal_pos"] = np.array([[a, b] for a, b, _ in pos_list], dtype=np.uint64)
    out["illegal_player"] = np.array([c for _, _, c in pos_list], dtype=np.int32)
    out["illegal_ok"] = np.array(legal_tab, dtype=np.uint8)
    # wrap-around boards (envs/test_equivalence_game.py:303-327)
    dirs = [(0, 1), (1, 1), (1, 0), (1, -1), (0, -1), (-1, -1), (-1, 0), (-1, 1)]
    wrap = []
    for corner, d, forb in (((4, 7), 0, (4, 0)), ((7, 4), 2, (0, 4)), ((3, 0), 4, (3, 7)),
                            ((0, 3), 6, (7, 3))):
        b = _BitBoard()
        bi = OthelloGameNew._idx_to_bit(corner[0] * 8 + corner[1])
        b.black = np.uint64(1) << np.uint64(bi)
        wi, wj = corner[0] + dirs[d][0], corner[1] + dirs[d][1]
        b.white = np.uint64(0)
        if 0 <= wi < 8 and 0 <= wj < 8:
            b.white = np.uint64(1) << np.uint64(OthelloGameNew._idx_to_bit(wi * 8 + wj))
        wrap.append((int(b.black), int(b.white), int(b.valid_mask()),
                     OthelloGameNew._idx_to_bit(forb[0] * 8 + forb[1])))
    out["wrap"] = np.array(wrap, dtype=np.uint64)
    # random dense states for pack/unpack round trip (:280-293)
    r = np.random.default_rng(5)
    states = r.integers(-1, 2, size=(200, 8, 8)).astype(np.int8)
    rt_own, rt_opp, rt_back = [], [], []
    for st in states:
        o, p = OthelloGameNew._np_to_bitboards(st, 1)
        rt_own.append(o)
        rt_opp.append(p)
        rt_back.append(OthelloGameNew._bitboards_to_np(o, p))
    out["rt_states"] = states
    out["rt_rot_own"] = np.array(rt_own, np.uint64)
    out["rt_rot_opp"] = np.array(rt_opp, np.uint64)
    out["rt_back"] = np.array(rt_back, np.int8)
    out["initial"] = g.get_initial_state()
    np.savez_compressed(os.path.join(HERE, "edge_cases.npz"), **out)
    print("edge_cases: ok")


# ----------------------------------------------------------------------------------------
def gen_d4():
    from envs.othello import OthelloGame
    import MCTS_model

    idx = np.arange(64).reshape(8, 8).astype(np.int64)
    pi = np.arange(65).astype(np.float64)
    syms = OthelloGame(8).get_symmetries(idx, pi)
    gs_board = np.array([s[0].reshape(-1) for s in syms], dtype=np.int64)
    gs_pi = np.array([s[1] for s in syms], dtype=np.float64)
    # random_symmetry / unsymmetrise_pi for every (k, flip)
    rs_board, rs_unpi = [], []
    for flip in (False, True):
        for k in range(4):
            s = np.rot90(idx, k, axes=(-2, -1))
            if flip:
                s = np.flip(s, axis=-1)
            rs_board.append(np.ascontiguousarray(s).reshape(-1))
            rs_unpi.append(MCTS_model.unsymmetrise_pi(pi.copy(), k, flip, 8))
    np.savez_compressed(os.path.join(HERE, "d4.npz"), get_symmetries_board=gs_board,
                        get_symmetries_pi=gs_pi, sym_board=np.array(rs_board),
                        sym_unpi=np.array(rs_unpi))
    print("d4: ok")


# ----------------------------------------------------------------------------------------
class RngRecorder:
    """Wrap np.random.dirichlet / np.random.choice to log every draw the reference
    makes (the wrapped calls return exactly what the originals return)."""

    def __init__(self):
        self.log = []
        self._dir = np.random.dirichlet
        self._choice = np.random.choice

    def __enter__(self):
        rec = self

        def dirichlet(alpha, size=None):
            x = rec._dir(alpha, size)
            rec.log.append(("dirichlet", np.asarray(x, np.float64).copy()))
            return x

        def choice(a, size=None, replace=True, p=None):
            st = np.random.get_state()
            r = rec._choice(a, size, replace, p)
            if p is not None:
                rs = np.random.RandomState()
                rs.set_state(st)
                u = rs.random_sample()
                pp = np.asarray(p, np.float64)
                cdf = pp.cumsum()
                cdf /= cdf[-1]
                assert int(cdf.searchsorted(u, side="right")) == int(r)
                rec.log.append(("choice_p", float(u), int(r)))
            else:
                arr = np.asarray(a)
                k = int(arr) if arr.ndim == 0 else len(arr)
                j = int(np.nonzero(arr == r)[0][0]) if arr.ndim else int(r)
                rec.log.append(("choice_tie", k, j))
            return r

        np.random.dirichlet = dirichlet
        np.random.choice = choice
        return self

    def __exit__(self, *exc):
        np.random.dirichlet = self._dir
        np.random.choice = self._choice


def encode_log(log):
    """(kind, a, b) rows + concatenated dirichlet vectors."""
    kinds, fa, ib, noise = [], [], [], []
    for e in log:
        if e[0] == "dirichlet":
            kinds.append(0)
            fa.append(float(len(noise)))
            ib.append(0)
            noise.append(e[1])
        elif e[0] == "choice_tie":
            kinds.append(1)
            fa.append(float(e[1]))
            ib.append(e[2])
        else:
            kinds.append(2)
            fa.append(e[1])
            ib.append(e[2])
    noise = np.array(noise, np.float64).reshape(-1, 65)
    return np.array(kinds, np.int32), np.array(fa, np.float64), np.array(ib, np.int64), noise


def random_position(g, rng, plies):
    state, player = g.get_initial_state(), 1
    for _ in range(plies):
        acts = np.nonzero(g.get_valid_moves(state, player))[0]
        a = int(rng.choice(acts))
        nxt = g.get_next_state(state, a, player)
        if g.get_value_and_terminated(nxt, a, -player)[1]:
            break
        state, player = nxt, -player
    return state, player


def gen_mcts():
    from envs.othello import OthelloGameNew
    from MCTS_model import MCTS

    g = OthelloGameNew(8)
    rng = np.random.default_rng(11)
    cases = []
    specs = []
    for plies in (0, 3, 10, 20, 30, 40, 50, 55):
        specs.append(random_position(g, rng, plies))
    rows = dict(pos=[], neg=[], player=[], sims=[], c_puct=[], eps=[], alpha=[], temp=[],
                seed=[], moves=[], counts=[], root_value=[], probs=[], root_n=[],
                log_kind=[], log_a=[], log_b=[], log_noise=[], log_case=[], noise_rows=[])
    case_id = 0
    for si, (state, player) in enumerate(specs):
        for sims, cp, eps, temp in ((25, 2.0, 0.0, 1.0), (100, 2.0, 0.0, 0.0),
                                    (100, 1.0, 0.3, 1.0), (400, 2.0, 0.3, 1.0)):
            if sims == 400 and si % 2:
                continue
            seed = 100 + case_id
            np.random.seed(seed)
            args = {"c_puct": cp, "num_simulations": sims, "num_threads": 1}
            m = MCTS(g, args, MockPolicy(), dirichlet_alpha=1.0, dirichlet_epsilon=eps)
            # two consecutive moves with tree reuse: search, move on the most visited
            # child, search again from the child
            st, pl = state.copy(), player
            with RngRecorder() as rec:
                for mv in range(2):
                    probs = m.policy_improve_step(st, pl, temp=temp)
                    counts = np.zeros(65, np.int64)
                    for a, ch in m.root.children.items():
                        counts[a] = ch.visit_count
                    p, n = bb_from_state(st)
                    rows["pos"].append(p)
                    rows["neg"].append(n)
                    rows["player"].append(pl)
                    rows["sims"].append(sims)
                    rows["c_puct"].append(cp)
                    rows["eps"].append(eps)
                    rows["alpha"].append(1.0)
                    rows["temp"].append(temp)
                    rows["seed"].append(seed)
                    rows["moves"].append(mv)
                    rows["counts"].append(counts)
                    rows["root_value"].append(float(m.root.value))
                    rows["probs"].append(np.asarray(probs, np.float32))
                    rows["root_n"].append(m.root.visit_count)
                    rows["log_case"].append(case_id)
                    a = int(np.argmax(counts))
                    nxt = g.get_next_state(st, a, pl)
                    if g.get_value_and_terminated(nxt, a, pl)[1]:
                        break
                    m.make_move(a)
                    st, pl = nxt, -pl
            k, fa, ib, noise = encode_log(rec.log)
            rows["log_kind"].append(k)
            rows["log_a"].append(fa)
            rows["log_b"].append(ib)
            rows["noise_rows"].append(noise)
            case_id += 1
    out = {}
    for k in ("pos", "neg"):
        out[k] = np.array(rows[k], np.uint64)
    for k in ("player", "sims", "seed", "moves", "root_n", "log_case"):
        out[k] = np.array(rows[k], np.int64)
    for k in ("c_puct", "eps", "alpha", "temp", "root_value"):
        out[k] = np.array(rows[k], np.float64)
    out["counts"] = np.array(rows["counts"], np.int64)
    out["probs"] = np.array(rows["probs"], np.float32)
    # per-case RNG logs (ragged -> concatenated with offsets)
    out["n_cases"] = np.int64(case_id)
    offs, noffs = [0], [0]
    for k in rows["log_kind"]:
        offs.append(offs[-1] + len(k))
    for nz in rows["noise_rows"]:
        noffs.append(noffs[-1] + len(nz))
    out["log_offsets"] = np.array(offs, np.int64)
    out["log_kind"] = np.concatenate(rows["log_kind"]) if offs[-1] else np.zeros(0, np.int32)
    out["log_a"] = np.concatenate(rows["log_a"]) if offs[-1] else np.zeros(0)
    out["log_b"] = np.concatenate(rows["log_b"]) if offs[-1] else np.zeros(0, np.int64)
    out["noise_offsets"] = np.array(noffs, np.int64)
    out["noise"] = (np.concatenate(rows["noise_rows"]) if noffs[-1]
                    else np.zeros((0, 65)))
    np.savez_compressed(os.path.join(HERE, "mcts_cases.npz"), **out)
    print("mcts_cases:", case_id, "cases,", len(out["pos"]), "searches")


# ----------------------------------------------------------------------------------------
def gen_selfplay():
    import self_play_worker

    games = [(25, 1), (25, 2), (25, 3), (100, 4), (100, 5), (400, 6)]
    rows = dict(game=[], ply=[], pos=[], neg=[], pi=[], z=[])
    meta, logs, noises = [], [], []
    for gi, (sims, seed) in enumerate(games):
        args = {"c_puct": 2.0, "num_simulations": sims, "num_threads": 1,
                "dirichlet_alpha": 1.0, "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0,
                "num_exploratory_moves": 35, "lambda": 0.98}
        np.random.seed(seed)
        t0 = time.time()
        with RngRecorder() as rec:
            out = self_play_worker.one_self_play(
                (8, args, (MockPolicyNet, {}, {}), None))
        print(f"  selfplay game {gi}: sims={sims} plies={len(out)} "
              f"{time.time() - t0:.1f}s")
        for t, (s, pi, z) in enumerate(out):
            p, n = bb_from_state(s)  # canonical (state*player): +1 = side to move
            rows["game"].append(gi)
            rows["ply"].append(t)
            rows["pos"].append(p)
            rows["neg"].append(n)
            rows["pi"].append(np.asarray(pi, np.float32))
            rows["z"].append(float(z))
        k, fa, ib, nz = encode_log(rec.log)
        logs.append((k, fa, ib))
        noises.append(nz)
        meta.append((sims, seed, len(out)))
    out = {"pos": np.array(rows["pos"], np.uint64), "neg": np.array(rows["neg"], np.uint64),
           "game": np.array(rows["game"], np.int32), "ply": np.array(rows["ply"], np.int32),
           "pi": np.array(rows["pi"], np.float32), "z": np.array(rows["z"], np.float64),
           "meta": np.array(meta, np.int64)}
    offs = [0]
    for k, _, _ in logs:
        offs.append(offs[-1] + len(k))
    out["log_offsets"] = np.array(offs, np.int64)
    out["log_kind"] = np.concatenate([l[0] for l in logs])
    out["log_a"] = np.concatenate([l[1] for l in logs])
    out["log_b"] = np.concatenate([l[2] for l in logs])
    noffs = [0]
    for nz in noises:
        noffs.append(noffs[-1] + len(nz))
    out["noise_offsets"] = np.array(noffs, np.int64)
    out["noise"] = np.concatenate(noises)
    np.savez_compressed(os.path.join(HERE, "selfplay_games.npz"), **out)
    print("selfplay_games:", len(games), "games,", len(out["pos"]), "samples")


# ----------------------------------------------------------------------------------------
def gen_training_data():
    import self_play_worker

    rng = np.random.default_rng(21)
    rows = []
    for case in range(40):
        T = int(rng.integers(1, 70))
        player = 1
        traj = []
        for t in range(T):
            traj.append((np.zeros((8, 8), np.int8), np.zeros(65, np.float32), player,
                         float(np.float32(rng.uniform(-1, 1)))))
            if rng.random() >= 0.1:  # ~10% passes keep the same player next ply
                player = -player
        winner = int(rng.choice([-1, 0, 1]))
        lam = (0.98, 1.0, 0.5)[case % 3]
        out = self_play_worker.get_training_data(traj, winner, lam)
        for t in range(T):
            rows.append((case, t, traj[t][2], traj[t][3], winner, lam, out[t][2]))
    arr = np.array(rows, np.float64)
    np.savez_compressed(os.path.join(HERE, "training_data.npz"), rows=arr)
    print("training_data:", len(rows), "rows")


# ----------------------------------------------------------------------------------------
def gen_tictactoe():
    from envs.tic_tac_toe import TicTacToe
    from MCTS_model import MCTS

    class CopyTicTacToe(TicTacToe):
        """The reference env mutates state in place (envs/tic_tac_toe.py:25-29); this
        copy-on-step wrapper is the only intended deviation."""

        def get_next_state(self, state, action, player):
            return super().get_next_state(state.copy(), action, player)

    env = CopyTicTacToe()
    np.random.seed(0)
    outcomes = {"1": 0, "-1": 0, "0": 0}
    n = 50
    t0 = time.time()
    for _ in range(n):
        m = MCTS(env, {"c_puct": 2.0, "num_simulations": 25, "num_threads": 1}, None)
        state, player = env.get_initial_state(), 1
        while True:
            pi = m.policy_improve_step(state, player, temp=1.0)
            a = int(np.random.choice(9, p=pi))
            m.make_move(a)
            state = env.get_next_state(state, a, player)
            r, done = env.get_value_and_terminated(state, a, player)
            if done:
                w = player if r > 0 else (-player if r < 0 else 0)
                outcomes[str(w)] += 1
                break
            player = -player
    json.dump({"games": n, "sims": 25, "c_puct": 2.0, "outcomes": outcomes,
               "seconds": time.time() - t0},
              open(os.path.join(HERE, "tictactoe_stats.json"), "w"), indent=1)
    print("tictactoe:", outcomes)


# ----------------------------------------------------------------------------------------
def gen_replay():
    import train

    rng = np.random.default_rng(33)
    d = np.load(os.path.join(HERE, "board_corpus.npz"))
    # a small pool of reachable canonical boards so that duplicates are common, plus the
    # initial position (present in every game of a generation)
    pool_idx = rng.choice(len(d["pos"]), size=300, replace=False)
    pool = [(int(d["pos"][i]), int(d["neg"][i])) for i in pool_idx]
    pool.append((0x0000000810000000, 0x0000001008000000))
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)

    def board(pos, neg):
        b = np.zeros(64, np.int8)
        b[(np.uint64(pos) & w) != 0] = 1
        b[(np.uint64(neg) & w) != 0] = -1
        return b.reshape(8, 8)

    n = 4000
    rows = []
    for _ in range(n):
        k = len(pool) - 1 if rng.random() < 0.1 else int(rng.integers(0, len(pool) // 3)) \
            if rng.random() < 0.6 else int(rng.integers(0, len(pool)))
        pi = rng.random(65).astype(np.float32)
        pi[rng.random(65) < 0.7] = 0.0
        pi[int(rng.integers(0, 65))] += np.float32(0.5)
        pi /= pi.sum()
        v = float(rng.uniform(-1, 1))
        ver = int(rng.integers(0, 3))
        rows.append((board(*pool[k]), pi.astype(np.float32), v, ver, pool[k]))

    class Fake:
        pass

    fake = Fake()
    fake.replay_buffer = [(r[0], r[1], r[2], r[3]) for r in rows]
    fake._hash_state = lambda b: train.Trainer._hash_state(fake, b)
    states, policies, values = train.Trainer._aggregate_duplicates(fake)
    out_pos = np.array([int(np.bitwise_or.reduce(np.where(s.reshape(-1) == 1, w, np.uint64(0))))
                        for s in states], np.uint64)
    out_neg = np.array([int(np.bitwise_or.reduce(np.where(s.reshape(-1) == -1, w, np.uint64(0))))
                        for s in states], np.uint64)
    np.savez_compressed(
        os.path.join(HERE, "replay_aggregate.npz"),
        in_pos=np.array([r[4][0] for r in rows], np.uint64),
        in_neg=np.array([r[4][1] for r in rows], np.uint64),
        in_pi=np.stack([r[1] for r in rows]), in_v=np.array([r[2] for r in rows], np.float64),
        in_ver=np.array([r[3] for r in rows], np.int32),
        out_pos=out_pos, out_neg=out_neg, out_pi=np.stack(policies),
        out_v=np.array(values, np.float32))
    print("replay_aggregate:", n, "rows ->", len(states), "buckets")


# ----------------------------------------------------------------------------------------
def gen_augment():
    from envs.othello import get_random_symmetry

    rng = np.random.default_rng(44)
    d = np.load(os.path.join(HERE, "board_corpus.npz"))
    sel = rng.choice(len(d["pos"]), size=512, replace=False)
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    pos, neg = d["pos"][sel].astype(np.uint64), d["neg"][sel].astype(np.uint64)
    states = np.zeros((len(sel), 64), np.float32)
    states[(pos[:, None] & w) != 0] = 1.0
    states[(neg[:, None] & w) != 0] = -1.0
    states = states.reshape(-1, 8, 8)
    pis = rng.random((len(sel), 65)).astype(np.float32)
    pis /= pis.sum(1, keepdims=True)
    np.random.seed(123)
    outs_s, outs_p = [], []
    for i in range(len(sel)):
        s_out, p_out = get_random_symmetry(states[i], pis[i])
        outs_s.append(s_out)
        outs_p.append(p_out)
    np.random.seed(123)  # the same draws, recorded: k = randint(4), flip = rand() < 0.5
    ks, flips = [], []
    for i in range(len(sel)):
        ks.append(np.random.randint(4))
        flips.append(np.random.rand() < 0.5)
    np.savez_compressed(os.path.join(HERE, "augment.npz"), pos=pos, neg=neg, pi=pis,
                        k=np.array(ks, np.int32), flip=np.array(flips, np.int32),
                        out_state=np.stack(outs_s), out_pi=np.stack(outs_p))
    print("augment:", len(sel))


GENS = {"augment": gen_augment, "replay": gen_replay, "board": gen_board, "bitboard": gen_bitboard, "edge": gen_edge, "d4": gen_d4,
        "mcts": gen_mcts, "selfplay": gen_selfplay, "training": gen_training_data,
        "tictactoe": gen_tictactoe}

if __name__ == "__main__":
    which = sys.argv[1:] or list(GENS)
    for w in which:
        t0 = time.time()
        GENS[w]()
        print(f"[{w}] {time.time() - t0:.1f}s")
