"""CPU checks of the product's C ABI and host mirror (no GPU): the library loads and
exports every entry point include/az_othello.h declares; the host build of the bitboard
core matches the reference-generated goldens; the OthelloGameNew drop-in follows the
reference's API (dtypes, errors) and test intents (envs/test_equivalence_*.py)."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, load_golden

nat = pytest.importorskip("az_native")


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "az_othello.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(\w+)\s*\(", src, re.M)))


def declared_arg_counts():
    """name -> number of parameters of every prototype in include/az_othello.h."""
    src = open(os.path.join(ROOT, "include", "az_othello.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:const\s+)?\w+\*?\s+\**(\w+)\s*\(([^)]*)\)\s*;", src, re.M):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_library_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(nat.lib, s), s
    assert set(nat.SIGNATURES) <= set(syms) | {"az_abi_version"}
    assert nat.lib.az_abi_version() == 1


def test_binding_argument_counts_match_header():
    """Every ctypes argtypes list has exactly as many entries as its C prototype (a short
    list would pass the trailing stream as an untyped extra argument)."""
    counts = declared_arg_counts()
    assert len(counts) == len(declared_symbols())
    for name, args in nat.SIGNATURES.items():
        assert len(args) == counts[name], (name, len(args), counts[name])


def test_loaded_library_was_built_from_this_tree():
    """The build id embedded at compile time (sha256 of sources, headers and flags) equals
    the hash of the tree under test: the library loaded is not a stale build."""
    import az_build

    assert nat.build_id() == az_build.source_hash() == az_build.built_id(nat.LIB_PATH)


def own_opp(pos, neg, player):
    return (np.where(player == 1, pos, neg).astype(np.uint64),
            np.where(player == 1, neg, pos).astype(np.uint64))


def test_cpu_step_matches_reference_corpus():
    d = load_golden("board_corpus.npz")
    own, opp = own_opp(d["pos"], d["neg"], d["player"])
    assert (nat.legal_cpu(own, opp) == d["valid"]).all()
    o, p, lg, st = nat.step_cpu(own, opp, d["action"])
    nown, nopp = own_opp(d["npos"], d["nneg"], -d["player"])
    assert (o == nown).all() and (p == nopp).all()
    assert ((nat.status_flags(st) & 1) == d["term_next"]).all()
    assert (nat.status_score(st) * -d["player"] == d["score_p1"]).all()


def test_cpu_illegal_reports_error():
    with pytest.raises(ValueError):
        nat.step_cpu(np.array([0x0000000810000000]), np.array([0x0000001008000000]), [0])
    o, p, lg, st = nat.step_cpu(np.array([0x0000000810000000]), np.array([0x0000001008000000]),
                                [0], raise_illegal=False)
    assert st[0] & nat.AZ_FLAG_ILLEGAL and o[0] == 0x0000000810000000


def test_heads_fast_gemm_rejects_unbuilt_tiles():
    """az_heads_fast_gemm_gpu checks (board_tile, splits) before it touches the device: an
    unbuilt pair is an AZ_ERR_ARG naming both (the buffers are never dereferenced)."""
    fake = 1 << 20  # 16-byte aligned, never read
    rc = nat.lib.az_heads_fast_gemm_gpu(fake, fake, fake, 0, fake, 132, 8, 48, 1, None)
    assert rc != nat.AZ_OK and "board_tile" in nat.last_error()
    rc = nat.lib.az_heads_fast_gemm_gpu(fake, fake, fake, 0, fake, 132, 4, 64, 1, None)
    assert rc != nat.AZ_OK and "(64, 4)" in nat.last_error()


def test_pack_unpack_roundtrip_and_rotated_helpers():
    from envs.othello import OthelloGameNew

    e = load_golden("edge_cases.npz")
    for s, ro, rp, back in zip(e["rt_states"], e["rt_rot_own"], e["rt_rot_opp"], e["rt_back"]):
        o, p = OthelloGameNew._np_to_bitboards(s, 1)
        assert o == ro and p == rp
        assert (OthelloGameNew._bitboards_to_np(ro, rp) == back).all()
        own, opp = nat.pack_np(s, 1)
        assert (nat.unpack_np(own, opp, 1)[0] == s).all()


def test_d4_cpu_matches_numpy_tables():
    d = load_golden("d4.npz")
    rng = np.random.default_rng(1)
    x = rng.integers(0, 2**63, 256, dtype=np.int64).astype(np.uint64)
    for s in range(8):
        got = nat.d4_cpu(x, s)
        bits = ((x[:, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1))
        src = d["sym_board"][s]
        want = np.bitwise_or.reduce(bits[:, src] << np.arange(64, dtype=np.uint64), axis=1)
        assert (got == want).all()


def test_game_api_against_corpus_sample():
    from envs.othello import OthelloGameNew

    g = OthelloGameNew(8)
    d = load_golden("board_corpus.npz")
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    for i in range(0, len(d["pos"]), 37):
        pos, neg, pl, a = int(d["pos"][i]), int(d["neg"][i]), int(d["player"][i]), int(d["action"][i])
        st = (((np.uint64(pos) & w) != 0).astype(np.int8) - ((np.uint64(neg) & w) != 0).astype(np.int8)).reshape(8, 8)
        v = g.get_valid_moves(st, pl)
        assert v.dtype == np.uint8 and v.shape == (65,)
        assert v[64] == d["pass_only"][i]
        nxt = g.get_next_state(st, a, pl)
        assert nxt.dtype == np.int8 and nxt.shape == (8, 8)
        npos = int(np.bitwise_or.reduce(np.where(nxt.reshape(-1) == 1, w, np.uint64(0))))
        assert npos == d["npos"][i]
        assert g.get_value_and_terminated(nxt, a, -pl) == (d["val_next"][i], bool(d["term_next"][i]))
        assert g.get_score(nxt, 1) == d["score_p1"][i]


def test_game_edge_cases():
    from envs.othello import OthelloGameNew, _BitBoard

    g = OthelloGameNew(8)
    e = load_golden("edge_cases.npz")
    assert (g.get_initial_state() == e["initial"]).all()
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)

    def state(pos, neg):
        return (((np.uint64(pos) & w) != 0).astype(np.int8)
                - ((np.uint64(neg) & w) != 0).astype(np.int8)).reshape(8, 8)

    s = state(e["passonly_pos"], e["passonly_neg"])
    assert (g.get_valid_moves(s, -1) == e["passonly_valid_m1"]).all()
    assert (g.get_valid_moves(s, 1) == e["passonly_valid_p1"]).all()
    for (pos, neg), (pl, v, t, sc) in zip(e["term_cases"], e["term_meta"]):
        st = state(pos, neg)
        assert g.get_value_and_terminated(st, 64, pl) == (v, bool(t))
        assert g.get_score(st, pl) == sc
    for (pos, neg), pl, row in zip(e["illegal_pos"], e["illegal_player"], e["illegal_ok"]):
        st = state(pos, neg)
        for a in range(65):
            if row[a]:
                g.get_next_state(st, a, pl)
            else:
                with pytest.raises(ValueError):
                    g.get_next_state(st, a, pl)
    with pytest.raises(AssertionError):
        OthelloGameNew(6)
    # pass returns a copy, never the same object (envs/othello.py:415-416)
    s0 = g.get_initial_state()
    s1 = g.get_next_state(s0, 64, 1)
    assert s1 is not s0 and (s1 == s0).all()
    bb = _BitBoard()
    assert int(bb.valid_mask()) == 0x0000102004080000
    assert bb.score() == 0


def test_bitboard_class_vectors():
    from envs.othello import _BitBoard

    d = load_golden("bitboard_vectors.npz")
    for i in range(0, len(d["mv_sq"]), 11):
        b = _BitBoard()
        k = d["mv_board"][i]
        b.black, b.white = np.uint64(d["black"][k]), np.uint64(d["white"][k])
        assert b.valid_mask() == d["valid"][k]
        b.make_move(int(d["mv_sq"][i]))
        assert b.black == d["mv_black"][i] and b.white == d["mv_white"][i]


def test_full_lowest_index_game_to_double_pass():
    """envs/test_equivalence_game.py:117-150 intent: lowest legal action until the game
    ends; final score as recorded by the reference."""
    from envs.othello import OthelloGameNew

    g = OthelloGameNew(8)
    d = load_golden("board_corpus.npz")
    sel = d["game"] == 0
    s, p = g.get_initial_state(), 1
    for a in d["action"][sel]:
        v = g.get_valid_moves(s, p)
        assert int(a) == int(np.nonzero(v)[0].min())
        s = g.get_next_state(s, int(a), p)
        p = -p
    assert g.get_value_and_terminated(s, 0, p)[1]
    assert g.get_score(s, 1) == d["score_p1"][sel][-1]


def test_get_training_data_matches_reference():
    from self_play_worker import get_training_data

    rows = load_golden("training_data.npz")["rows"]
    for case in np.unique(rows[:, 0]):
        r = rows[rows[:, 0] == case]
        traj = [(None, None, int(p), float(v)) for p, v in zip(r[:, 2], r[:, 3])]
        out = get_training_data(traj, int(r[0, 4]), float(r[0, 5]))
        assert np.array_equal(np.array([o[2] for o in out]), r[:, 6])


def test_cpu_step_random_positions_vs_oracle():
    """Unreachable dense/sparse positions and every action class (legal, occupied, no
    capture, pass, out of range) against the C oracle: the ray-table capture set, the
    carry/fill legal mask and the terminal flags hold on arbitrary boards, not only on the
    corpus."""
    from oracle import board as ob

    rng = np.random.default_rng(7)
    n = 1 << 17
    cells = rng.integers(0, 3, size=(n, 64))
    dense = rng.random(n) < 0.5  # half the boards sparse (mostly empty)
    cells[~dense] = np.where(rng.random((int((~dense).sum()), 64)) < 0.8, 0,
                             cells[~dense])
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    own = np.bitwise_or.reduce(np.where(cells == 1, w, np.uint64(0)), axis=1)
    opp = np.bitwise_or.reduce(np.where(cells == 2, w, np.uint64(0)), axis=1)
    act = rng.integers(0, 70, size=n).astype(np.uint8)
    o, p, lg, st = nat.step_cpu(own, opp, act, raise_illegal=False)
    ro, rp, rl, rs, _ = ob.step_batch(own, opp, act)
    assert (st == rs).all()
    assert (o == ro).all() and (p == rp).all() and (lg == rl).all()
    assert (nat.legal_cpu(own, opp) == ob.legal_batch(own, opp)).all()


def test_augment_tables_match_reference_get_random_symmetry():
    """The pi permutation tables of train_gpu (built from the bitboard D4 map) reproduce the
    reference's get_random_symmetry (envs/othello.py:501-526) for the (k, flip) it drew."""
    from train_gpu import pi_source_tables

    d = load_golden("augment.npz")
    src = pi_source_tables()
    sym = d["k"] + 4 * d["flip"]
    assert np.array_equal(np.take_along_axis(d["pi"], src[sym], 1), d["out_pi"])
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    for i in range(len(sym)):
        o = nat.d4_cpu(d["pos"][i:i + 1], int(sym[i]))[0]
        p = nat.d4_cpu(d["neg"][i:i + 1], int(sym[i]))[0]
        plane = ((o & w) != 0).astype(np.float32) - ((p & w) != 0).astype(np.float32)
        assert np.array_equal(plane.reshape(1, 8, 8), d["out_state"][i])


def test_bench_kernel_inputs_are_legal_playouts():
    """bench.py's kernel-roofline inputs (seeded random playouts, one legal
    action each, or the pass when there is none) are reproducible, every action is legal
    for its position, and the oracle steps all of them without an illegal placement."""
    import bench
    from oracle import board as ob

    own, opp, act = bench.playout_positions(games=64)
    own2, opp2, act2 = bench.playout_positions(games=64)
    assert (own == own2).all() and (opp == opp2).all() and (act == act2).all()
    assert len(own) > 64 * 50  # games run to (near) the end
    lg = ob.legal_batch(own, opp)
    passes = act == 64
    assert (passes == (lg == 0)).all()
    placed = ~passes
    assert ((lg[placed] >> act[placed].astype(np.uint64)) & np.uint64(1)).all()
    _, _, _, _, bad = ob.step_batch(own, opp, act)
    assert bad == -1


def test_splitk_table_picks_the_measured_fastest_form(monkeypatch):
    """FusedInferenceNet.splitk_for: the small-batch trunk conv form per batch size
    (profiles/r02_splitk_sweep.jsonl), AZ_SPLITK overriding it."""
    from Models import FusedInferenceNet as F

    monkeypatch.delenv("AZ_SPLITK", raising=False)
    want = {1: 16, 4: 16, 8: 16, 9: 8, 32: 8, 33: 4, 256: 4, 257: 0, 1024: 0}
    assert {b: F.splitk_for(b) for b in want} == want
    monkeypatch.setenv("AZ_SPLITK", "0")
    assert F.splitk_for(4) == 0


def test_trunk_scratch_is_bounded_and_pinned_under_capture(monkeypatch):
    """FusedInferenceNet keeps per-batch-size trunk scratch: sizes seen during a HIP graph
    capture stay (the graph points at them); other sizes are capped, least recently used
    dropped first; release_scratch() drops the unpinned ones."""
    import torch

    from Models import FusedInferenceNet

    class Net:
        scratch_cap = 2

    net = Net()
    sc = lambda B: FusedInferenceNet._scratch(net, torch.device("cpu"), B)  # noqa: E731
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    pinned = sc(1024)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    for B in range(1, 40):
        sc(B)
    keys = [k[1] for k in net._trunk_scratch]
    assert 1024 in keys and len(keys) == 1 + net.scratch_cap
    assert keys[-2:] == [38, 39]  # the most recent eager sizes
    assert sc(1024) is pinned and pinned["pinned"]
    FusedInferenceNet.release_scratch(net)
    assert [k[1] for k in net._trunk_scratch] == [1024]
