"""MCTS drop-in (reference MCTS_model.py:1-395): same constructor, `policy_improve_step`,
`make_move`, `.root` and argument keys, so self_play_worker.py, eval.py, play_othello.py
and diagnostic_plots.py run unchanged.

For OthelloGameNew the tree lives on the GPU in the batched engine's SoA node arena (one
game slot, host-driven): each simulation is az_select (PUCT descent, wavefront argmax) ->
policy evaluation -> az_expand_backup (eager expansion: one lane per child board step).
args['num_threads'] (the reference's worker count, default 4, MCTS_model.py:196) becomes the
engine's leaves_per_step K (<= 8): K virtual-loss descents per step, evaluated as one batch —
the reference's threaded search in one fixed interleaving of its workers (pinned by goldens the
reference itself produced under that schedule, tests/golden/make_vl_goldens.py); num_threads
= 1 is its deterministic sequential mode.  Host-side draws
keep the reference's np.random call order: Dirichlet root noise (np.random.dirichlet, :341)
is injected into the engine and the temperature-0 tie break (np.random.choice, :251) is
drawn here, so a seeded np.random reproduces the reference's search exactly (tests/).

A torch policy (the Models.py nets) is evaluated on the device directly on the engine's
packed planes; any other policy object is called through its `inference(state, player)`
duck type (MCTS_model.py:305-307) with the canonical board and player +1, which is what the
reference's Inference mixin computes from (player*state, Models.py:16).
`inference_cache` / `apply_symmetry` are accepted and, as in the reference, have no effect
(the cache is never populated: SURVEY.md 0.9).

Other `Game` environments (TicTacToe, config #1: CPU plumbing) use `_TreeSearch`, a
host-side restatement of the same algorithm on the environment's own methods.
"""
import math
import os

import numpy as np

os.environ.setdefault("OMP_NUM_THREADS", "1")

EPS = 1e-8
VIRTUAL_LOSS = 1.0


def random_symmetry(state):
    """One D4 element (MCTS_model.py:15-28): rot90 k times, then optional left-right flip."""
    k = np.random.randint(4)
    flip = bool(np.random.randint(2))
    s = np.rot90(state, k, axes=(-2, -1))
    if flip:
        s = np.flip(s, axis=-1)
    return s, k, flip


def unsymmetrise_pi(pi_sym, k, flip, n):
    """Inverse of random_symmetry on an (n*n+1,) policy (MCTS_model.py:31-43)."""
    pb = pi_sym[:-1].reshape(n, n)
    if flip:
        pb = np.flip(pb, axis=-1)
    pb = np.rot90(pb, -k)
    return np.concatenate([pb.ravel(), pi_sym[-1:]])


def _pi_from_counts(counts, temp, valid_actions):
    """policy_improve_step's tail (MCTS_model.py:244-274), NumPy semantics unchanged."""
    if abs(temp) < 1e-1:
        best_actions = np.where(counts == counts.max())[0]
        best_action = np.random.choice(best_actions)
        probs = np.zeros_like(counts)
        if len(valid_actions) != 0:
            probs[best_action] = 1.0
        return probs
    counts_exp = counts ** (1.0 / temp)
    norm = np.sum(counts_exp)
    if norm < 1e-12:
        probs = np.zeros(len(counts), dtype=np.float32)
        for a in valid_actions:
            probs[a] = 1.0 / len(valid_actions)
        return probs
    return counts_exp / norm


# ---------------------------------------------------------------------------------------
# read-only views of the device tree (what callers read from `mcts.root`)

class _NodeView:
    __slots__ = ("_t", "_i", "_player", "_state_fn", "parent")

    def __init__(self, tree, i, player, state_fn, parent=None):
        self._t, self._i, self._player, self._state_fn, self.parent = tree, i, player, state_fn, parent

    @property
    def visit_count(self):
        return int(self._t["N"][self._i])

    @property
    def value_sum(self):
        return float(self._t["W"][self._i])

    virtual_visits = 0
    virtual_value = 0.0

    @property
    def value(self):
        n = self.visit_count
        return 0.0 if n == 0 else self.value_sum / n

    @property
    def prior(self):
        p = self._t["prior"][self._i]
        f64 = self.parent is not None and self._t["flags"][self.parent._i] & 4
        return np.float64(p) if f64 else np.float32(p)

    @property
    def player(self):
        return self._player

    @property
    def action(self):
        return None if self._i == 0 else int(self._t["action"][self._i])

    @property
    def state(self):
        return self._state_fn(self._i, self._player)

    @property
    def is_terminal(self):
        return bool(self._t["flags"][self._i] & 2)

    @property
    def terminal_value(self):
        return int(self._t["tval"][self._i])

    @property
    def valid_mask(self):
        lg = int(self._t["legal"][self._i])
        v = np.zeros(65, np.uint8)
        if lg == 0:
            v[64] = 1
        else:
            v[:64] = (np.uint64(lg) >> np.arange(64, dtype=np.uint64)) & np.uint64(1)
        return v

    @property
    def valid_actions(self):
        return np.nonzero(self.valid_mask)[0]

    @property
    def children(self):
        t, i = self._t, self._i
        if not t["flags"][i] & 1 or i >= len(t["N"]):
            return {}
        fc, nc = int(t["first"][i]), int(t["nchild"][i])
        return {int(t["action"][c]): _NodeView(t, c, -self._player, self._state_fn, self)
                for c in range(fc, fc + nc) if c < len(t["N"])}

    def is_leaf(self):
        return len(self.children) == 0


class _EngineSearch:
    """One host-driven slot of the GPU engine."""

    def __init__(self, env, args, policy, dirichlet_alpha, dirichlet_epsilon):
        self.env, self.args, self.policy = env, args, policy
        self.alpha, self.eps = dirichlet_alpha, dirichlet_epsilon
        self.engine = None
        self.has_root = False
        self.root_state = None
        self.root_player = None
        self.dev_policy = None
        self._tree = None
        self.K = min(8, max(1, int(args.get("num_threads", 4))))

    def _ensure(self):
        if self.engine is not None:
            return
        import torch

        from engine import Engine

        self.engine = Engine(1, self.args["num_simulations"], c_puct=self.args["c_puct"],
                             dirichlet_alpha=self.alpha, dirichlet_epsilon=self.eps,
                             rollout=self.policy is None, injected_rng=True, auto_play=False,
                             leaves_per_step=self.K)
        if isinstance(self.policy, torch.nn.Module) and hasattr(self.policy, "evaluate_planes"):
            import copy

            from Models import AlphaZeroNet, FastOthelloNet, inference_copy

            if isinstance(self.policy, (AlphaZeroNet, FastOthelloNet)):
                # the same fused HIP inference copy the batched engine runs (fp32-accurate)
                self.dev_policy = inference_copy(self.policy, self.engine.device)
            else:
                self.dev_policy = copy.deepcopy(self.policy).to(self.engine.device).eval()

    def reset(self):
        self.has_root = False
        self._tree = None

    def _evaluate(self):
        import torch

        e = self.engine
        if self.dev_policy is not None:
            with torch.no_grad():
                if hasattr(self.dev_policy, "evaluate_into"):
                    self.dev_policy.evaluate_into(e.nn_in, e.priors, e.values)
                else:
                    pr, va = self.dev_policy.evaluate_planes(e.nn_in)
                    e.priors.copy_(pr)
                    e.values.copy_(va)
            return
        # every waiting leaf's row (rows are packed from 0; -1 ends the list)
        leaves = e.leaf.cpu().numpy()
        planes = np.rint(e.nn_in.cpu().numpy()).astype(np.int8)
        pr = np.zeros((len(leaves), 65), np.float32)
        va = np.zeros(len(leaves), np.float32)
        for j in np.flatnonzero(leaves >= 0):
            priors, value = self.policy.inference(planes[j].reshape(8, 8), 1)
            pr[j] = np.asarray(priors, np.float32).reshape(65)
            va[j] = float(value)
        e.priors.copy_(torch.from_numpy(pr))
        e.values.copy_(torch.from_numpy(va))

    def _device_iteration(self):
        e = self.engine
        if self.fuse_expand:
            e.select_expand()  # the previous iteration's leaves, then this one's descents
            self._evaluate()
            return
        e.select()
        self._evaluate()
        e.expand()

    # False: the same n iterations run eagerly (tests/test_callers_gpu.py compares the two)
    use_graph = True
    # True: each iteration is az_select_expand -> net (the expansion runs in the next
    # iteration's select launch, one launch fewer per iteration; az_expand_backup after the
    # last).  Off by default: one game's search is a latency chain, and the merged launch
    # (the expansion's registers) measured no faster -- one_self_play 1.04-1.05 vs 1.07
    # games/s unfused, same box (profiles/r03_dropin_fuse_expand_ab.json); AZ_DROPIN_FUSE=1
    fuse_expand = os.environ.get("AZ_DROPIN_FUSE", "0") == "1"

    def _run_on_device(self, n):
        """n select -> net -> expand iterations with no host synchronisation, replayed from
        one captured HIP graph of a single iteration (captured on first use)."""
        import torch

        self._run_iterations(n)
        if self.fuse_expand and n > 0:
            with torch.no_grad():
                self.engine.expand()  # the last iteration's leaves

    def _run_iterations(self, n):
        import torch

        if not self.use_graph:
            with torch.no_grad():
                for _ in range(n):
                    self._device_iteration()
            return
        if getattr(self, "_graph", None) is None:
            s = torch.cuda.Stream(device=self.engine.device)
            s.wait_stream(torch.cuda.current_stream())
            with torch.no_grad(), torch.cuda.stream(s):
                # the first iteration runs eagerly (it also warms the kernels up); capturing
                # does not execute the captured work
                self._device_iteration()
            torch.cuda.current_stream().wait_stream(s)
            n -= 1
            g = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(g):
                self._device_iteration()
            self._graph = g
        for _ in range(n):
            self._graph.replay()

    def search(self, init_state, init_player, temp):
        self._ensure()
        e = self.engine
        self._tree = None
        if not self.has_root:
            own, opp = _pack(init_state, init_player)
            e.set_root(0, own, opp, init_player)
            self.root_state = np.array(init_state, copy=True)
            self.root_player = init_player
            self.has_root = True
        else:
            assert np.all(self.root_state == init_state)
            assert self.root_player == init_player
        root = e.export_tree(0, max_nodes=1)
        if not root["flags"][0] & 1 and self.eps > 0:
            # the root will be expanded inside this call: Dirichlet noise (MCTS_model.py:340)
            e.inject(noise=np.random.dirichlet([self.alpha] * 65).reshape(1, 1, 65))
        e.begin_search(0, self.args["num_simulations"])
        if self.dev_policy is not None:
            # a host-driven select always waits on min(K, remaining) leaves or finishes the
            # search (its descent budget covers all simulations), so ceil(sims / K) + 1
            # iterations (the root expansion included) complete it: no per-simulation host
            # round trip (the loop below confirms)
            self._run_on_device(-(-self.args["num_simulations"] // self.K) + 1)
        guard = 0
        while True:
            e.select()
            leaf = int(e.leaf[0].item())
            if leaf < 0:
                info = e.game_info()
                if info["status"][0] != 1:
                    break
                guard += 1
                if guard > 1000:
                    raise RuntimeError("MCTS search made no progress in 1,000 selects "
                                       "(engine descent budget exhausted)")
                continue
            if self.policy is not None:
                self._evaluate()
            e.expand()
        if info["overflow"][0]:
            # an expansion was skipped (engine.hip k_expand): no longer the reference's search
            raise RuntimeError("MCTS node arena overflow: the search diverged from the reference")
        _, counts, _ = e.root_policy(0, 1.0)
        tree = self.root_tree()
        return _pi_from_counts(counts.astype(np.float32), temp,
                               _NodeView(tree, 0, self.root_player, self._state_of).valid_actions)

    def make_move(self, action):
        if not self.has_root:
            return
        self.engine.make_move(0, int(action))  # KeyError when not a child (:214)
        self._tree = None
        t = self.root_tree(max_nodes=1)
        self.root_player = -self.root_player
        self.root_state = _unpack(t["own"][0], t["opp"][0], self.root_player)

    def root_tree(self, max_nodes=None):
        if self._tree is None or max_nodes is None and len(self._tree["N"]) < self._tree["n_nodes"]:
            self._tree = self.engine.export_tree(0, max_nodes)
        return self._tree

    def _state_of(self, i, player):
        t = self.root_tree()
        return _unpack(t["own"][i], t["opp"][i], player)

    def root_view(self):
        if not self.has_root:
            return None
        return _NodeView(self.root_tree(), 0, self.root_player, self._state_of)


def _pack(state, player):
    import az_native as nat

    own, opp = nat.pack_np(np.asarray(state), player)
    return int(own[0]), int(opp[0])


def _unpack(own, opp, player):
    import az_native as nat

    return nat.unpack_np(np.array([own], np.uint64), np.array([opp], np.uint64), player)[0]


# ---------------------------------------------------------------------------------------
# generic environments (config #1 TicTacToe): host restatement of the same algorithm

class Node:
    """The reference Node (MCTS_model.py:46-169) for generic environments."""

    __slots__ = ("env", "args", "state", "player", "action", "prior", "value_sum",
                 "visit_count", "virtual_visits", "virtual_value", "parent", "children",
                 "valid_mask", "valid_actions", "terminal_value", "is_terminal")

    def __init__(self, env, args, state, player, action=None, prior=0.0, parent=None):
        self.env, self.args, self.state, self.player = env, args, state, player
        self.action, self.prior, self.parent = action, prior, parent
        self.value_sum, self.visit_count = 0.0, 0
        self.virtual_visits, self.virtual_value = 0, 0.0
        self.children = {}
        self.valid_mask = env.get_valid_moves(state, player)
        self.valid_actions = np.nonzero(self.valid_mask)[0]
        if action is not None:
            self.terminal_value, self.is_terminal = env.get_value_and_terminated(
                state, action, player)
        else:
            self.terminal_value, self.is_terminal = 0, False

    @property
    def value(self):
        n = self.visit_count + self.virtual_visits
        return 0.0 if n == 0 else (self.value_sum + self.virtual_value) / n

    def is_leaf(self):
        return len(self.children) == 0

    def backpropagate(self, value):
        node, sign = self, 1
        while node is not None:
            node.visit_count += 1
            node.value_sum += sign * value
            sign = -sign
            node = node.parent


class _TreeSearch:
    def __init__(self, env, args, policy, dirichlet_alpha, dirichlet_epsilon):
        self.env, self.args, self.policy = env, args, policy
        self.alpha, self.eps = dirichlet_alpha, dirichlet_epsilon
        self.root = None

    def reset(self):
        self.root = None

    def _ucb(self, node, child):
        sq = math.sqrt(node.visit_count + node.virtual_visits + EPS)
        q = -child.value
        return q + (self.args["c_puct"] * child.prior * sq /
                    (1 + child.visit_count + child.virtual_visits))

    def _rollout(self, state, player):
        cur, cp = state.copy(), player
        while True:
            acts = np.where(self.env.get_valid_moves(cur, cp) == 1)[0]
            if len(acts) == 0:
                return 0.0
            a = np.random.choice(acts)
            cur = self.env.get_next_state(cur, a, cp)
            v, term = self.env.get_value_and_terminated(cur, a, player)
            if term:
                return v
            cp = self.env.get_opponent(cp)

    def _expand(self, leaf):
        if self.policy is None:
            priors = np.ones(self.env.action_size, dtype=np.float32)
            v = self._rollout(leaf.state, leaf.player)
        else:
            priors, v = self.policy.inference(leaf.state, leaf.player)
        if leaf is self.root and self.eps > 0:
            noise = np.random.dirichlet([self.alpha] * len(priors))
            priors = (1 - self.eps) * priors + self.eps * noise
        priors = priors * leaf.valid_mask
        s = priors.sum()
        if s > 1e-12:
            priors = priors / s
        for a in leaf.valid_actions:
            a = int(a)
            st = self.env.get_next_state(leaf.state, a, leaf.player)
            leaf.children[a] = Node(self.env, self.args, st, self.env.get_opponent(leaf.player),
                                    a, priors[a], leaf)
        leaf.backpropagate(v)

    def _simulate(self):
        node, path = self.root, []
        while True:
            node.virtual_visits += 1
            node.virtual_value += VIRTUAL_LOSS
            path.append(node)
            if node.is_terminal:
                node.backpropagate(node.terminal_value)
                break
            if node.is_leaf():
                self._expand(node)
                break
            node = max(node.children.values(), key=lambda c, n=node: self._ucb(n, c))
        for n in path:
            n.virtual_visits -= 1
            n.virtual_value -= VIRTUAL_LOSS

    def search(self, init_state, init_player, temp):
        if self.root is None:
            self.root = Node(self.env, self.args, init_state.copy(), init_player)
        else:
            assert np.all(self.root.state == init_state)
            assert self.root.player == init_player
        if self.root.is_leaf():
            self._expand(self.root)
        for _ in range(self.args["num_simulations"]):
            self._simulate()
        counts = np.zeros(self.env.action_size, dtype=np.float32)
        for a, c in self.root.children.items():
            counts[a] = c.visit_count
        return _pi_from_counts(counts, temp, self.root.valid_actions)

    def make_move(self, action):
        if not self.root:
            return
        self.root = self.root.children[int(action)]
        self.root.parent = None

    def root_view(self):
        return self.root


class MCTS:
    """Drop-in for the reference MCTS (MCTS_model.py:172-395)."""

    def __init__(self, env, args, policy, apply_symmetry=False, dirichlet_alpha=0.03,
                 dirichlet_epsilon=0.0, inference_cache=None):
        from envs.othello import OthelloGameNew

        self.env = env
        self.args = args
        self.policy = policy
        self.use_rollout = policy is None
        self.num_actions = env.action_size
        self.apply_symmetry = apply_symmetry
        self.dirichlet_alpha = dirichlet_alpha
        self.dirichlet_epsilon = dirichlet_epsilon
        self.inference_cache = inference_cache
        self.num_threads = max(1, args.get("num_threads", 4))
        impl = _EngineSearch if isinstance(env, OthelloGameNew) else _TreeSearch
        self._impl = impl(env, args, policy, dirichlet_alpha, dirichlet_epsilon)

    @property
    def root(self):
        return self._impl.root_view()

    @root.setter
    def root(self, value):
        if value is not None:
            raise ValueError("MCTS.root can only be reset to None")
        self._impl.reset()

    def make_move(self, action):
        self._impl.make_move(action)

    def policy_improve_step(self, init_state, init_player, temp=1):
        return self._impl.search(init_state, init_player, temp)
