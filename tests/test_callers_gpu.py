"""the interactive callers run unchanged on the drop-in MCTS.

play_othello.py:39-94 (human vs MCTS) and play_mcts_vs_egaroucid.py:191-240 (MCTS vs an
external engine) drive one `MCTS(env, {'c_puct', 'num_simulations'}, net,
apply_symmetry=True)` through a whole game: `policy_improve_step(state, player, temp=0.0)`
on the bot's turns, the opponent's move chosen outside MCTS, `mcts.make_move(a)` after
EVERY ply (both sides, tree reuse), and `(mcts.root.value + 1) / 2 if mcts.root` read as
the win probability.  Here the opponent is a seeded random legal mover (the human / the
Egaroucid engine stand-in) and the net is the deterministic mock policy; the expected
moves and root values come from the oracle's restatement of the reference MCTS
(oracle/mcts.py, pinned to reference-run goldens) -- with the reference's default of 4
worker threads (MCTS_model.py:196: these callers pass no num_threads), i.e. the 4-leaf
virtual-loss search (tests/golden/make_vl_goldens.py) -- with np.random seeded identically
before every search (temp 0 breaks count ties with np.random.choice, MCTS_model.py:247).
Bit-exact: every bot move, every root value and visit count."""
import numpy as np
import pytest

from mock_policy import MockPolicy, mock_eval

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from MCTS_model import MCTS  # noqa: E402
from envs.othello import OthelloGameNew  # noqa: E402
from oracle import board as ob  # noqa: E402
from oracle.mcts import SeqMCTS  # noqa: E402


def _oracle_eval(own, opp, player):
    st = ob.to_state(own, opp, player)
    p, v = mock_eval((player * st).reshape(-1))
    return p.astype(np.float32), float(v)


def _play(bot_player, sims, seed):
    env = OthelloGameNew(8)
    args = {"c_puct": 3.0, "num_simulations": sims}  # play_othello.py:41's keys
    mcts = MCTS(env, args, MockPolicy(), apply_symmetry=True)
    ref = SeqMCTS(args["c_puct"], sims, _oracle_eval, leaves_per_step=4)
    opp_rng = np.random.default_rng(seed)
    game = ob.OracleGame()
    state, ostate = env.get_initial_state(), game.get_initial_state()
    player, plies, bot_moves = 1, 0, 0
    while True:
        assert (np.asarray(state) == np.asarray(ostate)).all()
        if player == bot_player:
            np.random.seed(seed * 1000 + plies)
            probs = mcts.policy_improve_step(state, player, temp=0.0)
            np.random.seed(seed * 1000 + plies)
            own, opp = ob.to_bitboards(ostate, player)
            rprobs = ref.search(own, opp, player, 0.0)
            action = int(np.argmax(probs))
            assert action == int(np.argmax(rprobs)), plies
            got = np.array([c.visit_count if c else 0 for c in
                            (mcts.root.children.get(a) for a in range(65))])
            assert (got == ref.root_counts()).all(), plies
            bot_moves += 1
        else:
            valid = np.flatnonzero(env.get_valid_moves(state, player))
            action = int(opp_rng.choice(valid))
        mcts.make_move(action)
        if ref.root >= 0:
            ref.make_move(action)
        # play_othello.py:71
        win_prob = (mcts.root.value + 1) / 2 if mcts.root else 0.0
        exp = (ref.value(0) + 1) / 2 if ref.root >= 0 else 0.0
        assert win_prob == exp, plies
        state = env.get_next_state(state, action, player)
        ostate = game.get_next_state(ostate, action, player)
        value, done = env.get_value_and_terminated(state, action, player)
        ovalue, odone = game.get_value_and_terminated(ostate, action, player)
        assert (value, done) == (ovalue, odone)
        plies += 1
        if done:
            return plies, bot_moves
        player = env.get_opponent(player)


@pytest.mark.parametrize("bot_player,seed", [(1, 1), (-1, 2)])
def test_interactive_caller_loop_matches_reference(bot_player, seed):
    plies, bot_moves = _play(bot_player, sims=24, seed=seed)
    assert plies >= 30 and bot_moves >= 15


@pytest.mark.parametrize("threads", [1, 4])
def test_dropin_net_search_graph_replay_equals_eager(threads, monkeypatch):
    """The path real callers take with a Models.py net (train.py's pool, eval.py): the
    drop-in MCTS evaluates on the fused HIP inference copy and runs each search as replays
    of one captured select -> net -> expand graph, ceil(sims / K) + 1 of them.  The same
    searches run eagerly (no graph) must give identical root visit counts and root values
    over several plies of tree reuse, so the captured graph is replayed on later searches
    with the engine's current buffers."""
    import torch

    from MCTS_model import _EngineSearch
    from Models import AlphaZeroNet

    def run(use_graph, fuse=True):
        monkeypatch.setattr(_EngineSearch, "use_graph", use_graph)
        monkeypatch.setattr(_EngineSearch, "fuse_expand", fuse)
        torch.manual_seed(0)
        net = AlphaZeroNet(8, 65, 5, 128)
        env = OthelloGameNew(8)
        mcts = MCTS(env, {"c_puct": 2.0, "num_simulations": 48, "num_threads": threads}, net,
                    dirichlet_alpha=1.0, dirichlet_epsilon=0.3)
        state, player = env.get_initial_state(), 1
        out = []
        for ply in range(6):
            np.random.seed(100 + ply)
            probs = mcts.policy_improve_step(state, player, temp=1.0)
            counts = np.array([c.visit_count if c else 0 for c in
                               (mcts.root.children.get(a) for a in range(65))])
            out.append((counts, mcts.root.value, mcts.root.visit_count, probs))
            action = int(np.flatnonzero(counts == counts.max())[0])
            mcts.make_move(action)
            state = env.get_next_state(state, action, player)
            player = -player
        assert (getattr(mcts._impl, "_graph", None) is not None) == use_graph
        return out

    # fused (az_select_expand: each iteration's expansion in the next select launch, the
    # default) and unfused iterations, replayed and eager: the same searches
    e = run(False, False)
    for other in (run(True, True), run(False, True), run(True, False)):
        for ply, (a, b) in enumerate(zip(other, e)):
            assert np.array_equal(a[0], b[0]), ply
            assert a[1] == b[1] and a[2] == b[2], ply
            assert np.array_equal(a[3], b[3]), ply


def _endgame_positions(n, max_empty, seed):
    """Positions of seeded random playouts with at most max_empty empty squares left and a
    placement for the side to move (most simulations from them end on terminal nodes)."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        own, opp, player = 0x0000000810000000, 0x0000001008000000, 1
        while True:
            lg = ob.legal(own, opp)
            empty = 64 - bin(own | opp).count("1")
            if lg and empty <= max_empty:
                out.append((own, opp, player))
                break
            if not lg and not ob.legal(opp, own):
                break
            moves = [a for a in range(64) if (lg >> a) & 1] or [64]
            own, opp = ob.make_move(own, opp, int(rng.choice(moves)))
            player = -player
    return out


@pytest.mark.parametrize("threads", [1, 4])
def test_dropin_endgame_searches_terminal_heavy(threads):
    """the drop-in search raises after 1,000 selects without progress.  Under the
    reference's settings a host-driven select's descent budget covers every simulation, so
    terminal-heavy end-game trees (1-4 empty squares: nearly every simulation ends on a
    terminal node, backed up in place) finish without the guard firing, at the reference's
    worker count of 4 and at 1 -- visit counts equal to the oracle's."""
    env = OthelloGameNew(8)
    for max_empty in (1, 2, 4):
        for own, opp, player in _endgame_positions(3, max_empty, 17 + max_empty):
            state = ob.to_state(own, opp, player)
            args = {"c_puct": 2.0, "num_simulations": 64, "num_threads": threads}
            mcts = MCTS(env, args, MockPolicy())
            ref = SeqMCTS(args["c_puct"], 64, _oracle_eval, leaves_per_step=threads)
            np.random.seed(5)
            mcts.policy_improve_step(state, player, temp=1.0)
            np.random.seed(5)
            ref.search(own, opp, player, 1.0)
            got = np.array([c.visit_count if c else 0 for c in
                            (mcts.root.children.get(a) for a in range(65))])
            assert (got == ref.root_counts()).all(), (max_empty, threads)
