"""Batched arena evaluation on the GPU engine: eval.py's play_match / evaluate_models
(eval.py:12-44, 46-74, 134-178) for many matches at once.

Each net owns one host-driven engine whose slot g is that net's tree in match g (the
reference gives each player its own `MCTS` with tree reuse).  Per ply, every match's side
to move searches in its own engine (temperature 0, no root noise: eval.py builds its
trees with the default dirichlet_epsilon = 0); both engines' searches run concurrently,
`args['num_threads']` virtual-loss leaves per searching slot per step (the reference's
worker count, default 4, MCTS_model.py:196); the action is the argmax of the
root visit counts
with the reference's random tie break (np.random.choice over the tied maxima,
MCTS_model.py:250-254); the board advances through the C-ABI step; both trees re-root on
the action (eval.py:176-177).  Colours alternate by match index as in
evaluate_models_parallel (even: A plays first).
"""
import numpy as np
import torch

import az_native as nat
from engine import Engine

INIT_OWN, INIT_OPP = 0x0000000810000000, 0x0000001008000000


def _as_evaluator(net, device):
    """nn.Module -> its fused inference copy (evaluate_into straight into the engine's
    buffers, graph-capturable); callables pass through (device-side test policies: eager
    steps); None = rollout evaluation."""
    if net is None or callable(net) and not isinstance(net, torch.nn.Module):
        return net
    if hasattr(net, "evaluate_into"):  # already an inference form (FusedInferenceNet, ...)
        return net
    from Models import inference_copy

    return inference_copy(net, device)


def tie_break_random(best):
    return int(np.random.choice(best))


def tie_break_lowest(best):
    return int(best[0])


class BatchedArena:
    """Two host-driven engines (one per net), slot g of each holding that net's tree of
    match g.  A search is replayed from HIP graphs: ceil(sims / K) + 1 iterations of
    select -> net -> expand complete every searching slot (a host-driven select waits on
    min(K, remaining) leaves or finishes its search), with one status check after them.
    Matches are laid out so that a net's searching slots are one contiguous half of the
    wave (the matches where it plays first, then the others: with colours alternating, the
    side to move at a ply is one colour in every match), and the net evaluates only that
    half's rows."""

    def __init__(self, net_a, net_b, args, n_slots, device=None, seed=0,
                 tie_break=tie_break_random, node_capacity=0, use_graph=True,
                 steps_per_graph=8):
        self.args = args
        self.G = n_slots
        self.K = min(8, max(1, int(args.get("num_threads", 4))))
        kw = dict(c_puct=args["c_puct"], auto_play=False, node_capacity=node_capacity,
                  device=device, leaves_per_step=self.K)
        self.eng = [Engine(n_slots, args["num_simulations"], rollout=net_a is None, seed=seed,
                           **kw),
                    Engine(n_slots, args["num_simulations"], rollout=net_b is None,
                           seed=seed + 1, **kw)]
        dev = self.eng[0].device
        self.eval = [_as_evaluator(net_a, dev), _as_evaluator(net_b, dev)]
        self.tie_break = tie_break
        # graphs need every evaluator on device buffers only (rollout or a fused inference
        # copy); test callables run eagerly
        self.use_graph = use_graph and all(ev is None or hasattr(ev, "evaluate_into")
                                           for ev in self.eval)
        self.steps_per_graph = max(1, int(steps_per_graph))
        self._graphs = {}
        self._graph_state = None  # what the cached graphs were captured under (_run)
        self._bounds = (0, n_slots, n_slots)  # (0, end of the first-player half, n)
        self.iterations = 0  # select -> net -> expand iterations run (per searching engine)

    def _row_range(self, sel):
        """The slot range whose rows a net evaluates: the half of the wave holding every
        searching slot, else the whole wave."""
        lo, mid, hi = self._bounds
        if sel.min() >= lo and sel.max() < mid:
            return (lo, mid)
        if sel.min() >= mid and sel.max() < hi:
            return (mid, hi)
        return (lo, hi)

    def _iteration(self, plan):
        """One select -> net -> expand per (engine, slot range) of the plan."""
        K = self.K
        for k, (lo, hi) in plan:
            e = self.eng[k]
            e.select()
            ev = self.eval[k]
            r0, r1 = lo * K, hi * K
            if ev is None:
                pass  # rollout: the expansion evaluates on device
            elif hasattr(ev, "evaluate_into"):
                ev.evaluate_into(e.nn_in[r0:r1], e.priors[r0:r1], e.values[r0:r1])
            else:
                pr, va = ev(e.nn_in[r0:r1])
                e.priors[r0:r1].copy_(pr)
                e.values[r0:r1].copy_(va)
            e.expand()

    def _run(self, plan, n):
        """n iterations of the plan: graphs of steps_per_graph iterations (and single ones
        for the remainder), each captured on first use after one eager iteration."""
        self.iterations += n
        if not self.use_graph:
            for _ in range(n):
                self._iteration(plan)
            return
        # the captured launches freeze each engine's Params (kernel arguments by value) and the
        # evaluators' buffers: a graph is reused only under the same engine parameters and
        # simulation count, otherwise the cache is dropped and recaptured
        key_state = (tuple(e.param_epoch for e in self.eng), self.args["num_simulations"],
                     tuple(id(ev) for ev in self.eval))
        if key_state != self._graph_state:
            self._graphs = {}
            self._graph_state = key_state
        while n > 0:
            m = self.steps_per_graph if n >= self.steps_per_graph else 1
            g = self._graphs.get((plan, m))
            if g is None:
                s = torch.cuda.Stream(device=self.eng[0].device)
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    self._iteration(plan)  # warms the kernels and caches; real work
                torch.cuda.current_stream().wait_stream(s)
                n -= 1
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(m):
                        self._iteration(plan)
                self._graphs[(plan, m)] = g
                continue
            g.replay()
            n -= m

    @torch.no_grad()
    def _search(self, slots):
        sims = self.args["num_simulations"]
        plan = []
        for k in (0, 1):
            if len(slots[k]):
                self.eng[k].begin_search_slots(slots[k], sims)
                plan.append((k, self._row_range(slots[k])))
        plan = tuple(plan)
        # every searching slot finishes within ceil(sims / K) + 1 iterations (the root's
        # expansion included); the loop confirms, and would finish a straggler step by step
        self._run(plan, -(-sims // self.K) + 1)
        for _ in range(1000):
            plan = tuple((k, r) for k, r in plan
                         if (self.eng[k].game_info()["status"] == nat.AZ_GAME_ACTIVE).any())
            if not plan:
                break
            self._run(plan, 1)
        else:
            raise RuntimeError("arena search did not finish")
        for k in (0, 1):
            # a skipped expansion (node arena full, or a waiting descent deeper than the
            # tracked path) makes that search differ from the reference's: never score it
            n = self.eng[k].counters()["arena_overflows"]
            if n:
                raise RuntimeError(f"arena engine {k}: node arena overflowed {n} times; the "
                                   "searches diverged from the reference (raise node_capacity)")

    def play(self, n_matches):
        """Play n_matches (in waves of G) and return (wins_a, wins_b, draws, plies)."""
        wins_a = wins_b = draws = 0
        plies = []
        for base in range(0, n_matches, self.G):
            n = min(self.G, n_matches - base)
            # colours alternate by match index (eval.py:114-121: even -> A first); slot s of
            # the wave holds match perm[s], the matches where A plays first in the first
            # slots, so each net's searching slots at a ply are one half
            a_first_m = (np.arange(base, base + n) % 2) == 0
            perm = np.argsort(~a_first_m, kind="stable")
            self._bounds = (0, int(a_first_m.sum()), n)
            res, pl_s = self._play_wave(a_first_m[perm])
            pl = np.empty(n, np.int64)
            pl[perm] = pl_s  # plies in match order
            pl = [int(x) for x in pl]
            wins_a += int((res == 1).sum())
            wins_b += int((res == -1).sum())
            draws += int((res == 0).sum())
            plies.extend(pl)
        return wins_a, wins_b, draws, plies

    def _play_wave(self, a_first):
        n = len(a_first)
        own = np.full(n, INIT_OWN, np.uint64)
        opp = np.full(n, INIT_OPP, np.uint64)
        player = np.ones(n, np.int32)
        live = np.ones(n, bool)
        has_root = np.zeros((2, n), bool)
        result = np.zeros(n, np.int32)  # +1 A won, -1 B won, 0 draw
        ply = np.zeros(n, np.int32)
        while live.any():
            # engine of the side to move: 0 (A) when A plays this colour
            mover = np.where((player == 1) == a_first, 0, 1)
            slots = []
            for k in (0, 1):
                sel = np.nonzero(live & (mover == k))[0]
                fresh = sel[~has_root[k][sel]]
                if len(fresh):  # policy_improve_step with root None (MCTS_model.py:223-228)
                    self.eng[k].set_roots(fresh, own[fresh], opp[fresh], player[fresh])
                    has_root[k][fresh] = True
                slots.append(sel.astype(np.int32))
            self._search(slots)
            actions = np.full(n, -1, np.int64)
            for k in (0, 1):
                if not len(slots[k]):
                    continue
                counts, _ = self.eng[k].root_stats()
                for g in slots[k]:
                    c = counts[g].astype(np.float32)
                    best = np.where(c == c.max())[0]
                    actions[g] = self.tie_break(best)
            idx = np.nonzero(live)[0]
            o, p, _, st = nat.step_cpu(own[idx], opp[idx], actions[idx].astype(np.uint8))
            terminal = (nat.status_flags(st) & nat.AZ_FLAG_TERMINAL) != 0
            score = nat.status_score(st)  # side to move after the step minus the mover
            for j, g in enumerate(idx):
                ply[g] += 1
                if terminal[j]:
                    # reward from the mover's view (eval.py:163-175)
                    d = -score[j]
                    winner_is_a = (mover[g] == 0) if d > 0 else (mover[g] == 1)
                    result[g] = 0 if d == 0 else (1 if winner_is_a else -1)
                    live[g] = False
            own[idx], opp[idx] = o, p
            player[idx] = -player[idx]
            # both trees re-root on the action (eval.py:176-177); no-op without a root
            for k in (0, 1):
                act = np.full(self.G, -1, np.int32)
                sel = np.nonzero(live & has_root[k])[0]
                act[sel] = actions[sel]
                if len(sel):
                    found = self.eng[k].reroot_slots(act)
                    missing = sel[found[sel] < 0]
                    if len(missing):
                        raise KeyError(int(actions[missing[0]]))
        return result, list(ply)


def evaluate_models_batched(board_size, args, policy_state, best_policy_state, n_matches=20,
                            n_slots=None, device=None):
    """Drop-in for evaluate_models_parallel (eval.py:46-74): returns
    (win rate of `policy`, win rate of `best_policy`)."""
    assert board_size == 8

    def build(ps):
        if ps is None:
            return None
        cls, cfg, sd = ps
        net = cls(**cfg)
        net.load_state_dict(sd)
        return net.eval()

    arena = BatchedArena(build(policy_state), build(best_policy_state), args,
                         n_slots or min(n_matches, 1024), device=device)
    wa, wb, _, _ = arena.play(n_matches)
    return wa / n_matches, wb / n_matches
