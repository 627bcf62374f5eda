"""Self-play driver drop-in (reference self_play_worker.py:1-88).

`get_training_data` is the reference's TD(lambda) target rule (host copy of what the
engine's finish kernel computes on device for batched self-play).  `one_self_play` keeps
the reference's signature so train.py's process pool (train.py:199-225) works unchanged;
the game itself runs through the MCTS drop-in on the GPU engine.  `collect_self_play_games`
is the batched replacement for that whole pool: one engine, G concurrent games on the GPU.
"""
import numpy as np
import torch

from envs.othello import OthelloGameNew as OthelloGame
from MCTS_model import MCTS


def get_training_data(trajectory, winning_player, lambd: float = 1.0):
    """G_T = z(player_T); G_t = (1-lambda) v_t + lambda * s * G_{t+1} with s = +1 when the
    side to move is unchanged between t and t+1 (around a pass), else -1
    (self_play_worker.py:8-35)."""

    def z_for(p):
        if winning_player == 0:
            return 0.0
        return 1.0 if p == winning_player else -1.0

    out = [None] * len(trajectory)
    g_next = None
    p_next = None
    for t in range(len(trajectory) - 1, -1, -1):
        state, pi, player, v_root = trajectory[t]
        if g_next is None:
            g = z_for(player)
        else:
            s = 1.0 if player == p_next else -1.0
            g = (1.0 - lambd) * v_root + lambd * s * g_next
        out[t] = (state, pi, g)
        g_next, p_next = g, player
    return out


# one_self_play's per-process game batch (AZ_DROPIN_BATCH): games played together on the
# batched engine at the first call, handed out one per call while the policy and args match
_BATCH = {"key": None, "games": []}


def _dropin_batch_size(args=None):
    """AZ_DROPIN_BATCH (default 32), capped at this worker's share of the generation when
    the args carry train.py's num_self_play / num_workers (train.py:413, 420): with the
    reference's 300 games over os.cpu_count() workers a worker plays ceil(300 / workers)
    games per batch instead of 32 it would mostly discard."""
    import os

    n = int(os.environ.get("AZ_DROPIN_BATCH", "32"))
    args = args or {}
    try:
        games, workers = int(args["num_self_play"]), int(args["num_workers"])
    except (KeyError, TypeError, ValueError):
        return n
    if n > 1 and games > 0 and workers > 0:
        n = min(n, -(-games // workers))
    return n


def _batch_key(board_size, args, policy_state):
    """Identity of what a batch was played with: the policy class, config, every state_dict
    tensor (bytes) and the args."""
    import hashlib

    cls, cfg, sd = policy_state
    h = hashlib.sha1(repr((board_size, getattr(cls, "__qualname__", str(cls)),
                           sorted(cfg.items()), sorted((k, repr(v)) for k, v in args.items())))
                     .encode())
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def _games_from_rows(rows):
    """Engine sample rows -> one list of reference tuples per game, in SLOT order.  A game's
    rows are contiguous in the sample ring (finish_game reserves them at once) and each starts
    at the initial position, the only position with four stones.  The ring itself is in
    completion order -- all of a batch's games start together, so that is game-length order --
    and handing games out in it would return the shortest games first; a slot plays one
    game of the batch from its own Philox stream, so slot order does not depend on the
    outcome (games of one slot keep their ring order)."""
    own = np.asarray(rows["own"]).view(np.uint64)
    opp = np.asarray(rows["opp"]).view(np.uint64)
    occ = own | opp
    stones = np.zeros(len(own), np.int64)
    for sh in range(64):
        stones += ((occ >> np.uint64(sh)) & np.uint64(1)).astype(np.int64)
    starts = list(np.flatnonzero(stones == 4)) + [len(own)]
    tuples = _rows_to_tuples(rows)
    games = [tuples[a:b] for a, b in zip(starts[:-1], starts[1:])]
    if "slot" in rows and len(games):
        slot = np.asarray(rows["slot"])[np.asarray(starts[:-1])]
        games = [games[i] for i in np.argsort(slot, kind="stable")]
    return games


@torch.no_grad()
def one_self_play(args_tuple):
    """One complete game (self_play_worker.py:38-88); returns [(state, pi, G)].

    train.py's spawn pool (train.py:199-225) calls this once per game in each worker
    process.  By default (AZ_DROPIN_BATCH = 32, capped at the worker's share
    ceil(num_self_play / num_workers) when args carry them) the worker's first call plays that
    many games at once on the batched GPU engine (BatchedSelfPlay: the same search, K =
    args['num_threads'] virtual-loss leaves per step, Dirichlet root noise, temperature
    schedule and TD(lambda) targets; its Philox seed drawn from np.random, which the pool's
    _worker_init seeds) and hands them out one per call while the policy weights and args
    are unchanged, in slot order (independent of the games' lengths and outcomes:
    _games_from_rows) -- games distributed like the reference's, the engine's rate instead of
    one search at a time.  AZ_DROPIN_BATCH <= 1: one game per call through the drop-in MCTS
    (np.random draws in the reference's order)."""
    board_size, args, policy_state, _ = args_tuple
    if _dropin_batch_size() <= 1:
        return _one_game(args_tuple)
    n = _dropin_batch_size(args)
    assert board_size == 8
    key = _batch_key(board_size, args, policy_state)
    if _BATCH["key"] != key:
        _BATCH["key"], _BATCH["games"] = key, []
    if not _BATCH["games"]:
        policy_class, policy_config, policy_state_dict = policy_state
        policy = policy_class(**policy_config)
        policy.load_state_dict(policy_state_dict)
        policy.eval()
        seed = int(np.random.randint(0, 2**31 - 1))
        rows = _local_rows(policy, args, n, None, seed, 0, False, torch.float32)
        _BATCH["games"] = _games_from_rows(rows)
        assert len(_BATCH["games"]) == n, (len(_BATCH["games"]), n)
    return _BATCH["games"].pop(0)


@torch.no_grad()
def _one_game(args_tuple):
    """One complete game through the drop-in MCTS (self_play_worker.py:38-88)."""
    board_size, args, policy_state, inference_cache = args_tuple
    env = OthelloGame(board_size)
    policy_class, policy_config, policy_state_dict = policy_state
    policy = policy_class(**policy_config)
    policy.load_state_dict(policy_state_dict)
    policy.eval()
    mcts = MCTS(env, args, policy, dirichlet_alpha=args["dirichlet_alpha"],
                dirichlet_epsilon=args["dirichlet_epsilon"], inference_cache=inference_cache)
    trajectory = []
    state = env.get_initial_state()
    player = 1
    while True:
        temp = args["mcts_temperature"] if len(trajectory) < args["num_exploratory_moves"] else 0.0
        probs = mcts.policy_improve_step(state, player, temp=temp)
        trajectory.append((state.copy() * player, probs.copy(), player, mcts.root.value))
        action = np.random.choice(env.action_size, p=probs)
        mcts.make_move(action)
        state = env.get_next_state(state, action, player)
        reward, done = env.get_value_and_terminated(state, action, player)
        if done:
            winner = player if reward > 0 else (-player if reward < 0 else 0)
            return get_training_data(trajectory, winner, args["lambda"])
        player = env.get_opponent(player)


def collect_self_play_games(policy, args, num_games, n_slots=None, seed=0, stream_id=0,
                            d4_augment=False, dtype=torch.float32, group=None,
                            sync_weights=True, pipelines=1):
    """Batched replacement of Trainer.collect_self_play_games' pool (train.py:199-225):
    `num_games` games on the GPU, `n_slots` at a time (default min(games, 4096)), each
    searching with args['num_threads'] virtual-loss leaves per step (the reference's worker
    count, default 4: MCTS_model.py:196).  Returns the training tuples of all games.

    Under torch.distributed (one process per GPU, `group` or the default group, world > 1)
    this is one generation of the whole node: rank r plays its share of
    `num_games` (num_games // world, the first num_games % world ranks one more) on its own
    Philox sub-stream (stream_id + r), with the best net's weights first broadcast from rank
    0 (`sync_weights`; the reference hands every pool worker the best net's state_dict,
    train.py:205-207), and ONE all-gather (dist_replay.allgather_samples: RCCL over xGMI
    with the "nccl" backend) pools every rank's rows on every rank -- each rank returns the
    same list, rank 0's games first.

    pipelines > 1: the rank's slots as that many independent pipelines on their own HIP
    streams (engine.PipelinedSelfPlay; +8-10 % on configs[1] / configs[4]-sized batches,
    profiles/r04_pipelines_ab.json)."""
    import torch.distributed as dist

    distributed = dist.is_available() and dist.is_initialized() and \
        dist.get_world_size(group) > 1
    if not distributed:
        rows = _local_rows(policy, args, num_games, n_slots, seed, stream_id, d4_augment, dtype,
                           pipelines)
        return _rows_to_tuples(rows)
    from dist_replay import allgather_samples, broadcast_state_dict

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = _collective_device(group)
    if sync_weights and policy is not None:
        home = next(iter(policy.parameters())).device
        broadcast_state_dict(policy.to(dev), src=0, group=group)
        policy.to(home)
    mine = num_games // world + (1 if rank < num_games % world else 0)
    rows = _local_rows(policy, args, mine, n_slots, seed, stream_id + rank, d4_augment, dtype,
                       pipelines)
    pooled, _ = allgather_samples(rows, dev, group=group)
    return _rows_to_tuples({k: v.cpu().numpy() for k, v in pooled.items()})


def _collective_device(group=None):
    """Tensors for the group's backend: the rank's GPU for RCCL ("nccl"), the host for gloo."""
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _local_rows(policy, args, num_games, n_slots, seed, stream_id, d4_augment, dtype,
                pipelines=1):
    """This process's games as engine sample rows (numpy: own/opp canonical bitboards, pi,
    z, player); none when num_games is 0."""
    if num_games <= 0:
        return {"own": np.zeros(0, np.uint64), "opp": np.zeros(0, np.uint64),
                "pi": np.zeros((0, 65), np.float32), "z": np.zeros(0, np.float64),
                "player": np.zeros(0, np.int8)}
    from engine import BatchedSelfPlay, PipelinedSelfPlay

    n_slots = n_slots or min(num_games, 4096)
    kw = dict(seed=seed, stream_id=stream_id, d4_augment=d4_augment, dtype=dtype,
              sample_capacity=num_games * 130,
              leaves_per_step=min(8, max(1, int(args.get("num_threads", 4)))))
    if pipelines > 1 and n_slots >= pipelines:
        n_slots -= n_slots % pipelines
        sp = PipelinedSelfPlay(policy, args, n_slots, pipelines=pipelines, **kw)
        return sp.play_games(num_games, tuples=False)
    sp = BatchedSelfPlay(policy, args, n_slots, **kw)
    sp.play_games(num_games)
    return sp.engine.samples()


def _rows_to_tuples(rows):
    """Sample rows -> the reference's [(state int8 (8,8), pi float32 (65,), G float)] with
    state = the canonical board (own stones +1, self_play_worker.py:72)."""
    from engine import samples_to_tuples

    return samples_to_tuples({"own": np.asarray(rows["own"]).view(np.uint64),
                              "opp": np.asarray(rows["opp"]).view(np.uint64),
                              "pi": np.asarray(rows["pi"], np.float32),
                              "z": np.asarray(rows["z"], np.float64)})
