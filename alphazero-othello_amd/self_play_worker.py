"""Self-play driver drop-in (reference self_play_worker.py:1-88).

`get_training_data` is the reference's TD(lambda) target rule (host copy of what the
engine's finish kernel computes on device for batched self-play).  `one_self_play` keeps
the reference's signature so train.py's process pool (train.py:199-225) works unchanged;
the game itself runs through the MCTS drop-in on the GPU engine.  `collect_self_play_games`
is the batched replacement for that whole pool: one engine, G concurrent games on the GPU.
"""
import os
import shutil
import time

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


# one_self_play's shared generation (AZ_DROPIN_SHARED, default on when the args carry train.py's
# num_self_play): the pool's workers coordinate through a directory named by the batch key
# (policy weights + args: the same for every task of a generation).  The first worker to create
# its `producer` file plays ALL num_self_play games in one batch on the GPU engine and publishes
# the sample rows (rows.npz, written under another name and renamed into place, then `done`);
# every call of every worker claims the next unclaimed game index with an O_EXCL file
# (claim.<i>), so each game is handed out exactly once, in slot order of the one batch.  The
# other workers never touch the GPU.  A worker that has read its game leaves read.<i>; the
# reader that completes the set removes the directory.  A producer that died before `done`
# (or failed: its waiters raise the error) has its directory retired -- renamed away -- and the
# next caller produces anew.
_SHARED = {"key": None, "games": None, "next": 0}


def _shared_root():
    """AZ_DROPIN_DIR, default .dropin_gen/ beside this module (inside the checkout)."""
    return os.environ.get("AZ_DROPIN_DIR") or os.path.join(
        os.path.dirname(os.path.abspath(__file__)), ".dropin_gen")


def _excl(path, text=""):
    """Create `path` exclusively (atomic on a local file system); False if it exists."""
    try:
        fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o600)
    except FileExistsError:
        return False
    with os.fdopen(fd, "w") as f:
        f.write(text)
    return True


def _pid_alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


def _retire_stale(root, keep, max_age_s=600.0):
    """Remove other generations' directories untouched for max_age_s (a generation whose
    games were not all claimed -- e.g. a warm-up -- is never completed by its readers), except
    one whose producer is still alive and playing (no `done` yet)."""
    now = time.time()
    for name in os.listdir(root):
        path = os.path.join(root, name)
        if name == keep or not os.path.isdir(path):
            continue
        try:
            if now - os.stat(path).st_mtime <= max_age_s:
                continue
            if not os.path.exists(os.path.join(path, "done")):
                with open(os.path.join(path, "producer")) as f:
                    pid = int(f.read() or 0)
                if pid and _pid_alive(pid):
                    continue
        except (OSError, ValueError):
            pass
        shutil.rmtree(path, ignore_errors=True)


def _shared_game(key, total, produce, poll_s=0.02):
    """Game i of the generation `key` (total games, rows from produce(total)), or None when
    every game has been claimed.  Returns a list of reference tuples."""
    root = _shared_root()
    os.makedirs(root, exist_ok=True)
    name = key[:40]
    d = os.path.join(root, name)
    while True:
        os.makedirs(d, exist_ok=True)
        if _excl(os.path.join(d, "producer"), str(os.getpid())):
            _retire_stale(root, name)
            try:
                rows = produce(total)
                tmp = os.path.join(d, f"rows.{os.getpid()}.npz")
                with open(tmp, "wb") as f:
                    np.savez(f, **{k: np.asarray(v) for k, v in rows.items()})
                os.replace(tmp, os.path.join(d, "rows.npz"))
                tok = os.path.join(d, f"done.{os.getpid()}")
                with open(tok, "w") as f:
                    f.write(f"{os.getpid()}.{time.time_ns()}")
                os.replace(tok, os.path.join(d, "done"))  # appears with its token
            except BaseException as ex:
                # waiters that see `failed` raise it; the directory is then retired, so a later
                # call (or a waiter that missed it) produces anew
                _excl(os.path.join(d, "failed"), repr(ex))
                try:
                    os.rename(d, f"{d}.failed.{os.getpid()}")
                except OSError:
                    pass
                raise
            break
        retired = False
        while not os.path.exists(os.path.join(d, "done")):
            if not os.path.isdir(d):  # retired meanwhile: start over
                retired = True
                break
            if os.path.exists(os.path.join(d, "failed")):
                with open(os.path.join(d, "failed")) as f:
                    raise RuntimeError(f"one_self_play: the generation's producer failed: {f.read()}")
            try:
                with open(os.path.join(d, "producer")) as f:
                    pid = int(f.read() or 0)
            except (OSError, ValueError):
                pid = 0
            if pid and not _pid_alive(pid):  # died before publishing: retire, start over
                try:
                    os.rename(d, f"{d}.dead.{pid}.{os.getpid()}")
                except OSError:
                    pass
                retired = True
                break
            time.sleep(poll_s)
        if not retired:
            break
    try:
        with open(os.path.join(d, "done")) as f:
            gen = (key, f.read())  # this publication (the same key can return in a later pool)
    except FileNotFoundError:  # completed and removed meanwhile: every game was claimed
        return None
    if _SHARED["key"] != gen:
        _SHARED.update(key=gen, games=None, next=0)
    for i in range(_SHARED["next"], total):
        if _excl(os.path.join(d, f"claim.{i}"), str(os.getpid())):
            break
    else:
        return None
    _SHARED["next"] = i + 1
    if _SHARED["games"] is None:
        with np.load(os.path.join(d, "rows.npz")) as z:
            _SHARED["games"] = _games_from_rows({k: z[k] for k in z.files})
    game = _SHARED["games"][i]
    _excl(os.path.join(d, f"read.{i}"))
    try:
        if sum(n.startswith("read.") for n in os.listdir(d)) == total:
            shutil.rmtree(d, ignore_errors=True)
    except OSError:
        pass
    return game


def _shared_total(args):
    """The generation's game count when one_self_play shares it (AZ_DROPIN_SHARED, default
    on): train.py's num_self_play from the args; None = per-worker batches."""
    if os.environ.get("AZ_DROPIN_SHARED", "1") != "1":
        return None
    try:
        total = int((args or {})["num_self_play"])
    except (KeyError, TypeError, ValueError):
        return None
    return total if total > 0 else None


@torch.no_grad()
def one_self_play(args_tuple):
    """One complete game (self_play_worker.py:38-88); returns [(state, pi, G)].

    train.py's spawn pool (train.py:199-225) calls this once per game in each worker
    process.  When the args carry train.py's num_self_play (AZ_DROPIN_SHARED, default on),
    the pool's workers share ONE batch of that many games: the first call of the generation
    plays all of them on the GPU engine and every call returns the next unclaimed one
    (_shared_game: one producer, the other workers never touch the GPU; coordination files
    under AZ_DROPIN_DIR, default .dropin_gen/ beside this module).  Otherwise
    (AZ_DROPIN_BATCH = 32, capped at the worker's share
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
    assert board_size == 8
    key = _batch_key(board_size, args, policy_state)
    total = _shared_total(args)
    if total is not None:
        def produce(n):
            policy_class, policy_config, policy_state_dict = policy_state
            policy = policy_class(**policy_config)
            policy.load_state_dict(policy_state_dict)
            policy.eval()
            seed = int(np.random.randint(0, 2**31 - 1))
            # AZ_DROPIN_PIPELINES (experiments): the generation's slots as that many pipelines
            pipes = int(os.environ.get("AZ_DROPIN_PIPELINES", "1"))
            rows = _local_rows(policy, args, n, None, seed, 0, False, torch.float32, pipes)
            assert len(_games_from_rows(rows)) == n
            return rows

        game = _shared_game(key, total, produce)
        if game is not None:
            return game
        # more calls than the generation's games: this worker's own batches from here on
    n = _dropin_batch_size(args)
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
