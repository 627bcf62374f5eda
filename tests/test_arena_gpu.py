"""Batched arena (eval.py play_match semantics on the GPU engine) against the oracle's
restatement of play_match (sequential MCTS per player with tree reuse, eval.py:134-178),
two distinct deterministic policies, lowest-index tie break on both sides: identical
results and game lengths for every match, both colours."""
import numpy as np
import pytest

from mock_policy import mock_eval, mock_eval_torch

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("az_native")
from arena import BatchedArena, tie_break_lowest  # noqa: E402
from oracle import board as ob  # noqa: E402
from oracle.mcts import SeqMCTS  # noqa: E402


class LowestTie:
    def choice_tie(self, best):
        return best[0]


def oracle_play_match(first_salt, second_salt, args):
    def ev(salt):
        def f(own, opp, player):
            st = ob.to_state(own, opp, player)
            p, v = mock_eval((player * st).reshape(-1), salt)
            return p.astype(np.float32), float(v)
        return f

    K = args.get("num_threads", 4)  # the reference's default worker count (MCTS_model.py:196)
    trees = {1: SeqMCTS(args["c_puct"], args["num_simulations"], ev(first_salt), rng=LowestTie(),
                        leaves_per_step=K),
             -1: SeqMCTS(args["c_puct"], args["num_simulations"], ev(second_salt), rng=LowestTie(),
                         leaves_per_step=K)}
    game = ob.OracleGame()
    state, player, plies = game.get_initial_state(), 1, 0
    while True:
        own, opp = ob.to_bitboards(state, player)
        probs = trees[player].search(own, opp, player, 0.0)
        action = int(np.argmax(probs))
        state = game.get_next_state(state, action, player)
        plies += 1
        reward, done = game.get_value_and_terminated(state, action, player)
        if done:
            if reward == 0:
                return 0, plies
            first_won = (reward == 1) == (player == 1)
            return (1 if first_won else -1), plies
        for t in trees.values():
            if t.root >= 0:
                t.make_move(action)
        player = -player


@pytest.mark.parametrize("threads", [None, 1])
def test_arena_matches_oracle_play_match(threads):
    # eval.py's args carry no num_threads: the reference's default of 4 workers
    args = {"c_puct": 2.0, "num_simulations": 16}
    if threads is not None:
        args["num_threads"] = threads
    arena = BatchedArena(lambda x: mock_eval_torch(x, 1), lambda x: mock_eval_torch(x, 2), args,
                         n_slots=4, tie_break=tie_break_lowest)
    wa, wb, dr, plies = arena.play(4)
    exp_wa = exp_wb = exp_dr = 0
    exp_plies = []
    for m in range(4):
        a_first = m % 2 == 0
        r, pl = oracle_play_match(1 if a_first else 2, 2 if a_first else 1, args)
        exp_plies.append(pl)
        if r == 0:
            exp_dr += 1
        elif (r == 1) == a_first:
            exp_wa += 1
        else:
            exp_wb += 1
    assert (wa, wb, dr) == (exp_wa, exp_wb, exp_dr)
    assert plies == exp_plies


def test_evaluate_models_batched_with_nets():
    from arena import evaluate_models_batched
    from Models import FastOthelloNet

    net = FastOthelloNet(8, 65)
    ps = (FastOthelloNet, net.get_config(), net.state_dict())
    a, b = evaluate_models_batched(8, {"c_puct": 2.0, "num_simulations": 8}, ps, ps, n_matches=6)
    assert 0.0 <= a <= 1.0 and 0.0 <= b <= 1.0 and a + b <= 1.0


@pytest.mark.parametrize("threads", [None, 1])
def test_arena_graph_replay_equals_oracle(threads):
    """The graph-replayed search (nets with evaluate_into: select -> net on the searching
    half's rows -> expand, captured once per plan) plays exactly the oracle's matches, with
    more matches than slots (two waves)."""
    from mock_policy import MockNet

    args = {"c_puct": 2.0, "num_simulations": 24}
    if threads is not None:
        args["num_threads"] = threads
    arena = BatchedArena(MockNet(1).cuda(), MockNet(2).cuda(), args, n_slots=6,
                         tie_break=tie_break_lowest)
    assert arena.use_graph
    wa, wb, dr, plies = arena.play(10)
    assert arena._graphs  # the searches ran from captured graphs
    exp = [0, 0, 0]
    exp_plies = []
    for m in range(10):
        a_first = m % 2 == 0
        r, pl = oracle_play_match(1 if a_first else 2, 2 if a_first else 1, args)
        exp_plies.append(pl)
        exp[2 if r == 0 else (0 if (r == 1) == a_first else 1)] += 1
    assert (wa, wb, dr) == tuple(exp)
    assert plies == exp_plies


def test_arena_graphs_follow_simulation_count_changes():
    """the arena's HIP graphs freeze the engines' Params and the evaluators'
    buffers; a caller that changes num_simulations between play() calls (bench's warm-up
    plays 8 sims, then the timed 400) must still get exactly the oracle's matches at the new
    count -- the graph cache is keyed on what it was captured under."""
    from mock_policy import MockNet

    args = {"c_puct": 2.0, "num_simulations": 8}
    arena = BatchedArena(MockNet(1).cuda(), MockNet(2).cuda(), args, n_slots=4,
                         tie_break=tie_break_lowest)
    for sims in (8, 24, 8):
        args["num_simulations"] = sims
        wa, wb, dr, plies = arena.play(4)
        exp = [0, 0, 0]
        exp_plies = []
        for m in range(4):
            a_first = m % 2 == 0
            r, pl = oracle_play_match(1 if a_first else 2, 2 if a_first else 1, args)
            exp_plies.append(pl)
            exp[2 if r == 0 else (0 if (r == 1) == a_first else 1)] += 1
        assert (wa, wb, dr) == tuple(exp), sims
        assert plies == exp_plies, sims
        assert arena._graph_state[1] == sims
