"""Games/s of the UNCHANGED-caller path: the reference's own drivers calling the drop-in
`MCTS` one game at a time (no batching), on one GPU.

  * self-play: `self_play_worker.one_self_play` (reference self_play_worker.py:38-88, what
    train.py:199-225's spawn pool runs per worker), AlphaZeroNet(5,128) random init,
    configs[2] args (400 sims, Dirichlet root noise, T = 1 for 35 moves) -> one complete
    game, games/s and ms per move;
  * arena: eval.py:134-178 play_match's per-move call, `policy_improve_step(temp=0)` +
    `make_move` on two drop-in MCTS (two nets), ms per move over one game.
Both with the callers' own args -- train.py:399-423 / eval.py:191 pass no num_threads, so
the reference default of 4 workers (MCTS_model.py:196) = 4 virtual-loss leaves per engine
step -- and with num_threads = 1 (the sequential search).
One JSON line.  The batched engine (bench.py) is the production path; this measures what a
caller gets without changing a line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
from Models import AlphaZeroNet  # noqa: E402
from MCTS_model import MCTS  # noqa: E402
from envs.othello import OthelloGameNew  # noqa: E402
import self_play_worker  # noqa: E402


def run(threads, sims):
    torch.manual_seed(0)
    np.random.seed(0)
    net = AlphaZeroNet(8, 65, 5, 128).eval()
    args = {"c_puct": 2.0, "num_simulations": sims, "dirichlet_alpha": 1.0,
            "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0, "num_exploratory_moves": 35,
            "lambda": 0.98}
    if threads is not None:
        args["num_threads"] = threads
    ps = (AlphaZeroNet, {"board_size": 8, "action_size": 65, "n_res_blocks": 5, "channels": 128},
          net.state_dict())
    # warm-up game (captures the graphs, loads the kernels)
    self_play_worker.one_self_play((8, dict(args, num_simulations=8), ps, None))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = self_play_worker.one_self_play((8, args, ps, None))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = {"self_play": {"games_per_s": round(1.0 / dt, 4), "plies": len(out),
                         "ms_per_move": round(dt / len(out) * 1e3, 2), "sims": sims,
                         "net": "AlphaZeroNet(5,128) random init, fused HIP inference copy"}}

    # eval.py play_match's per-move loop on two drop-in MCTS
    env = OthelloGameNew(8)
    net2 = AlphaZeroNet(8, 65, 5, 128).eval()
    a = {"c_puct": 2.0, "num_simulations": sims}
    if threads is not None:
        a["num_threads"] = threads
    players = {1: MCTS(env, a, net), -1: MCTS(env, a, net2)}
    state, player, moves, t = env.get_initial_state(), 1, 0, 0.0
    while True:
        t0 = time.perf_counter()
        probs = players[player].policy_improve_step(state, player, temp=0.0)
        action = int(np.argmax(probs))
        for m in players.values():
            m.make_move(action)
        t += time.perf_counter() - t0
        moves += 1
        state = env.get_next_state(state, action, player)
        _, done = env.get_value_and_terminated(state, action, player)
        if done:
            break
        player = -player
    res["arena_play_match"] = {"ms_per_move": round(t / moves * 1e3, 2), "moves": moves,
                               "sims": sims}
    return res


def main():
    sims = int(os.environ.get("SIMS", 400))
    res = {"num_threads_default_4": run(None, sims), "num_threads_1": run(1, sims),
           "device": torch.cuda.get_device_name(0)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
