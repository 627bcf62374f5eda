"""Pin the oracle (oracle/) against fixtures produced by the reference itself
(tests/golden/make_goldens.py).  CPU only."""
import numpy as np
import pytest

from conftest import load_golden
from mock_policy import MockPolicy, mock_eval
from oracle import board as ob
from oracle.mcts import LogRng, SeqMCTS
from oracle.selfplay import play_game, td_lambda_targets


def own_opp(pos, neg, player):
    player = np.asarray(player)
    own = np.where(player == 1, pos, neg).astype(np.uint64)
    opp = np.where(player == 1, neg, pos).astype(np.uint64)
    return own, opp


def test_corpus_step_matches_reference():
    d = load_golden("board_corpus.npz")
    own, opp = own_opp(d["pos"], d["neg"], d["player"])
    assert (ob.legal_batch(own, opp) == d["valid"]).all()
    assert ((ob.legal_batch(own, opp) == 0) == (d["pass_only"] == 1)).all()
    o, p, lg, st, bad = ob.step_batch(own, opp, d["action"])
    assert bad == -1
    nown, nopp = own_opp(d["npos"], d["nneg"], -d["player"])
    assert (o == nown).all() and (p == nopp).all()
    flags = st & 0xFF
    score = (st >> 8).astype(np.uint8).view(np.int8).astype(np.int32)
    assert ((flags & 1) == d["term_next"]).all()
    assert ((flags & 1) == d["term_mover"]).all()
    term = d["term_next"] == 1
    assert (np.sign(score[term]) == d["val_next"][term]).all()
    assert (d["val_next"][~term] == 0).all()
    assert (score * -d["player"] == d["score_p1"]).all()
    assert (lg == ob.legal_batch(nown, nopp)).all()


def test_corpus_size_and_shape():
    d = load_golden("board_corpus.npz")
    assert len(d["pos"]) > 30000
    assert len(np.unique(d["game"])) >= 600


def test_bitboard_vectors():
    d = load_golden("bitboard_vectors.npz")
    assert (ob.legal_batch(d["black"], d["white"]) == d["valid"]).all()
    for i in range(len(d["mv_sq"])):
        b = d["mv_board"][i]
        nb, nw = ob.make_move(d["black"][b], d["white"][b], int(d["mv_sq"][i]))
        assert nb == d["mv_black"][i] and nw == d["mv_white"][i]


def test_edge_cases():
    d = load_golden("edge_cases.npz")
    g = ob.OracleGame()
    assert (g.get_initial_state() == d["initial"]).all()
    s = ob.to_state(int(d["passonly_pos"]), int(d["passonly_neg"]), 1)
    assert (g.get_valid_moves(s, -1) == d["passonly_valid_m1"]).all()
    assert (g.get_valid_moves(s, 1) == d["passonly_valid_p1"]).all()
    for (pos, neg), (pl, v, t, sc) in zip(d["term_cases"], d["term_meta"]):
        st = ob.to_state(int(pos), int(neg), 1)
        assert g.get_value_and_terminated(st, 64, pl) == (v, bool(t))
        assert g.get_score(st, pl) == sc
    for (pos, neg), pl, row in zip(d["illegal_pos"], d["illegal_player"], d["illegal_ok"]):
        st = ob.to_state(int(pos), int(neg), 1)
        for a in range(65):
            if row[a]:
                g.get_next_state(st, a, pl)
            else:
                with pytest.raises(ValueError):
                    g.get_next_state(st, a, pl)
    for black, white, mask, forb in d["wrap"]:
        assert ob.legal(black, white) == mask
        assert not (int(mask) >> int(forb)) & 1


def test_d4_tables_consistent():
    d = load_golden("d4.npz")
    idx = np.arange(64).reshape(8, 8)
    for s in range(8):
        k, flip = s % 4, s // 4
        t = np.rot90(idx, k)
        if flip:
            t = np.fliplr(t)
        assert (t.reshape(-1) == d["sym_board"][s]).all()


def replay_case(d, c):
    """Re-run one reference MCTS golden case on the oracle with the recorded draws."""
    rows = np.nonzero(d["log_case"] == c)[0]
    lo, hi = d["log_offsets"][c], d["log_offsets"][c + 1]
    nlo, nhi = d["noise_offsets"][c], d["noise_offsets"][c + 1]
    rng = LogRng(d["log_kind"][lo:hi], d["log_a"][lo:hi], d["log_b"][lo:hi],
                 d["noise"][nlo:nhi])
    r0 = rows[0]
    mp = MockPolicy()

    def evaluate(own, opp, player):
        return mp.inference(ob.to_state(own, opp, player), player)

    m = SeqMCTS(float(d["c_puct"][r0]), int(d["sims"][r0]), evaluate, dirichlet_alpha=1.0,
                dirichlet_epsilon=float(d["eps"][r0]), rng=rng)
    for r in rows:
        own, opp = own_opp(d["pos"][r], d["neg"][r], d["player"][r])
        probs = m.search(int(own), int(opp), int(d["player"][r]), float(d["temp"][r]))
        assert (m.root_counts() == d["counts"][r]).all(), f"case {c} move {d['moves'][r]}"
        assert m.value(m.root) == d["root_value"][r]
        assert (probs.astype(np.float32) == d["probs"][r]).all()
        assert m.N[m.root] == d["root_n"][r]
        a = int(np.argmax(d["counts"][r]))
        if r != rows[-1]:
            m.make_move(a)
    assert rng.i == len(rng.kinds)


@pytest.mark.parametrize("case", range(28))
def test_mcts_cases_match_reference(case):
    d = load_golden("mcts_cases.npz")
    assert int(d["n_cases"]) == 28
    replay_case(d, case)


def replay_vl_case(d, c):
    """One multi-leaf (virtual-loss) golden case: the reference's threaded search forced
    into the engine's interleaving (tests/golden/make_vl_goldens.py), on the oracle."""
    rows = np.nonzero(d["log_case"] == c)[0]
    nlo, nhi = d["noise_offsets"][c], d["noise_offsets"][c + 1]
    n = nhi - nlo
    rng = LogRng(np.zeros(n, np.int32), np.arange(n, dtype=np.float64), np.zeros(n, np.int64),
                 d["noise"][nlo:nhi])
    r0 = rows[0]
    mp = MockPolicy()

    def evaluate(own, opp, player):
        return mp.inference(ob.to_state(own, opp, player), player)

    m = SeqMCTS(float(d["c_puct"][r0]), int(d["sims"][r0]), evaluate, dirichlet_alpha=1.0,
                dirichlet_epsilon=float(d["eps"][r0]), rng=rng, leaves_per_step=int(d["k"][r0]))
    for r in rows:
        own, opp = own_opp(d["pos"][r], d["neg"][r], d["player"][r])
        probs = m.search(int(own), int(opp), int(d["player"][r]), 1.0)
        assert (m.root_counts() == d["counts"][r]).all(), f"case {c} move {d['moves'][r]}"
        assert m.value(m.root) == d["root_value"][r]
        assert (probs.astype(np.float32) == d["probs"][r]).all()
        assert m.N[m.root] == d["root_n"][r]
        if r != rows[-1]:
            m.make_move(int(np.argmax(d["counts"][r])))
    assert rng.i == len(rng.kinds)


@pytest.mark.parametrize("case", range(28))
def test_mcts_virtual_loss_cases_match_reference(case):
    d = load_golden("mcts_vl_cases.npz")
    assert int(d["n_cases"]) == 28
    replay_vl_case(d, case)


def test_virtual_loss_cases_differ_from_single_leaf():
    """The K-leaf goldens are not the num_threads=1 search (the virtual loss matters)."""
    d = load_golden("mcts_vl_cases.npz")
    mp = MockPolicy()

    def evaluate(own, opp, player):
        return mp.inference(ob.to_state(own, opp, player), player)

    differ = 0
    for r in np.nonzero(d["moves"] == 0)[0]:
        if d["eps"][r] > 0:
            continue
        m = SeqMCTS(float(d["c_puct"][r]), int(d["sims"][r]), evaluate)
        own, opp = own_opp(d["pos"][r], d["neg"][r], d["player"][r])
        m.search(int(own), int(opp), int(d["player"][r]), 1.0)
        differ += int((m.root_counts() != d["counts"][r]).any())
    assert differ >= 3


def _selfplay_args(sims):
    return {"c_puct": 2.0, "num_simulations": sims, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}


@pytest.mark.parametrize("game", [0, 1, 2, 3])
def test_selfplay_games_match_reference(game):
    d = load_golden("selfplay_games.npz")
    sims, seed, plies = d["meta"][game]
    lo, hi = d["log_offsets"][game], d["log_offsets"][game + 1]
    nlo, nhi = d["noise_offsets"][game], d["noise_offsets"][game + 1]
    rng = LogRng(d["log_kind"][lo:hi], d["log_a"][lo:hi], d["log_b"][lo:hi],
                 d["noise"][nlo:nhi])
    mp = MockPolicy()

    def evaluate(own, opp, player):
        return mp.inference(ob.to_state(own, opp, player), player)

    samples, _ = play_game(_selfplay_args(int(sims)), evaluate, rng=rng)
    sel = d["game"] == game
    assert len(samples) == plies == sel.sum()
    for t, (s, pi, z) in enumerate(samples):
        pos, neg = ob.to_bitboards(s, 1)
        assert pos == d["pos"][sel][t] and neg == d["neg"][sel][t]
        assert (pi.astype(np.float32) == d["pi"][sel][t]).all()
        assert z == d["z"][sel][t]


@pytest.mark.parametrize("game", [0, 3, 4, 5])
def test_deep_selfplay_games_match_reference(game):
    """selfplay_deep.npz (make_deep_goldens.py): 400-simulation games with one worker, and
    games under the forced K = 4 worker schedule -- the oracle's K-leaf self-play without a
    descent cap is that schedule."""
    d = load_golden("selfplay_deep.npz")
    sims, seed, plies, K = d["meta"][game]
    lo, hi = d["log_offsets"][game], d["log_offsets"][game + 1]
    nlo, nhi = d["noise_offsets"][game], d["noise_offsets"][game + 1]
    rng = LogRng(d["log_kind"][lo:hi], d["log_a"][lo:hi], d["log_b"][lo:hi],
                 d["noise"][nlo:nhi])
    mp = MockPolicy()

    def evaluate(own, opp, player):
        return mp.inference(ob.to_state(own, opp, player), player)

    samples, _ = play_game(_selfplay_args(int(sims)), evaluate, rng=rng,
                           leaves_per_step=int(K))
    sel = d["game"] == game
    assert len(samples) == plies == sel.sum()
    for t, (s, pi, z) in enumerate(samples):
        pos, neg = ob.to_bitboards(s, 1)
        assert pos == d["pos"][sel][t] and neg == d["neg"][sel][t]
        assert (pi.astype(np.float32) == d["pi"][sel][t]).all()
        assert z == d["z"][sel][t]


def test_training_data_matches_reference():
    rows = load_golden("training_data.npz")["rows"]
    for case in np.unique(rows[:, 0]):
        r = rows[rows[:, 0] == case]
        g = td_lambda_targets(list(r[:, 2].astype(int)), list(r[:, 3]), int(r[0, 4]),
                              float(r[0, 5]))
        assert np.array_equal(np.array(g), r[:, 6])


def test_mock_policy_is_float32_exact():
    x = np.random.default_rng(0).integers(-1, 2, size=(100, 64))
    p, v = mock_eval(x)
    assert p.dtype == np.float32
    assert (p * 1024 == np.rint(p * 1024)).all()
    assert (np.float32(v).astype(np.float64) == v).all()


def test_replay_aggregate_oracle_matches_reference():
    """oracle/replay.py against the reference's Trainer._aggregate_duplicates output
    (train.py:142-173), bit for bit, order included."""
    from oracle import replay

    d = load_golden("replay_aggregate.npz")
    own, opp, ver, pi, v, cnt = replay.aggregate(d["in_pos"], d["in_neg"], d["in_ver"],
                                                 d["in_pi"], d["in_v"])
    assert (own == d["out_pos"]).all() and (opp == d["out_neg"]).all()
    assert np.array_equal(pi, d["out_pi"])
    assert np.array_equal(v, d["out_v"])
    assert cnt.sum() == len(d["in_pos"])
