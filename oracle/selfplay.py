"""TEST INFRASTRUCTURE ONLY — restatement of self_play_worker.py.

  td_lambda_targets   get_training_data (self_play_worker.py:8-35)
  play_game           one_self_play's loop (self_play_worker.py:55-88) on the oracle MCTS
"""
import numpy as np

from . import board as ob
from .mcts import NumpyRng, SeqMCTS


def td_lambda_targets(players, v_roots, winner, lambd):
    """G_T = z(player_T); G_t = (1-lambda) v_t + lambda * s * G_{t+1}, s = +1 when the
    side to move did not change between t and t+1 (a pass), else -1."""
    T = len(players)
    out = [0.0] * T
    g_next, p_next = None, None
    for t in range(T - 1, -1, -1):
        p = players[t]
        z = 0.0 if winner == 0 else (1.0 if p == winner else -1.0)
        if g_next is None:
            g = z
        else:
            s = 1.0 if p == p_next else -1.0
            g = (1.0 - lambd) * v_roots[t] + lambd * s * g_next
        out[t] = g
        g_next, p_next = g, p
    return out


def play_game(args, evaluate, rng=None, max_plies=200, leaves_per_step=1):
    """One self-play game; returns (samples, winner) where samples are
    (canonical int8 (8,8), pi float32[65], target float) as one_self_play returns."""
    rng = rng or NumpyRng()
    m = SeqMCTS(args["c_puct"], args["num_simulations"], evaluate,
                dirichlet_alpha=args["dirichlet_alpha"],
                dirichlet_epsilon=args["dirichlet_epsilon"], rng=rng,
                leaves_per_step=leaves_per_step)
    game = ob.OracleGame()
    state = game.get_initial_state()
    player = 1
    traj = []
    for _ in range(max_plies):
        temp = args["mcts_temperature"] if len(traj) < args["num_exploratory_moves"] else 0.0
        own, opp = ob.to_bitboards(state, player)
        pi = m.search(own, opp, player, temp)
        v_root = m.value(m.root)
        traj.append(((state * player).astype(np.int8), pi.copy(), player, v_root))
        action = int(rng.choice_p(65, pi))
        m.make_move(action)
        state = game.get_next_state(state, action, player)
        reward, done = game.get_value_and_terminated(state, action, player)
        if done:
            winner = player if reward > 0 else (-player if reward < 0 else 0)
            g = td_lambda_targets([t[2] for t in traj], [t[3] for t in traj], winner,
                                  args["lambda"])
            return [(t[0], t[1], g[i]) for i, t in enumerate(traj)], winner
        player = -player
    raise RuntimeError("game did not terminate")
