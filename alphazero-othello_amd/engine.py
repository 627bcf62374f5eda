"""Batched GPU self-play: the owner of an `az_engine` handle (include/az_othello.h) and the
driver loop that replaces the reference's process-pool of `one_self_play` calls
(train.py:199-225, self_play_worker.py:38-88).

Per simulation step (all on one HIP stream, no host synchronisation, replayed from HIP
graphs of 8 steps).  The plain sequence (Engine's host-driven API, the drop-in MCTS):

    az_select         leaves of every active game -> canonical planes nn_in [G*K, 64]
                      (K = leaves_per_step: virtual-loss descents per game per step)
    net               the leaf evaluation on nn_in -> priors [G*K, 65], values [G*K]
    az_expand_backup  expansion + backup
    az_play           games whose search finished: pi, record, sample, move, TD(lambda)
                      targets on game end, re-root; finished slots restart

BatchedSelfPlay's default merges them into two launches per step: az_select_move_expand
(the previous step's expansions, the descents, the previous step's moves and the net's stem,
one wave per game) and the net (Models.FusedInferenceNet: the persistent HIP trunk with the
policy / value heads in its last conv).

The host only reads counters.  Finished games' samples accumulate in a device buffer in
the reference's training-tuple layout (canonical state, pi, target).
"""
import ctypes
import os

import numpy as np
import torch

import az_native as nat

SAMPLE_FIELDS = ("own", "opp", "pi", "z", "player", "slot")


class Engine:
    """RAII owner of one az_engine handle plus its per-step device buffers."""

    def __init__(self, n_games, num_simulations, c_puct=2.0, dirichlet_alpha=1.0,
                 dirichlet_epsilon=0.0, temperature=1.0, num_exploratory_moves=0,
                 lambd=1.0, rollout=False, injected_rng=False, d4_augment=False,
                 auto_play=True, refill=False, node_capacity=0, max_plies=0,
                 sample_capacity=0, inj_noise_slots=1, inj_uniform_slots=1, seed=0,
                 stream_id=0, device=None, leaves_per_step=1):
        if not torch.cuda.is_available():
            raise RuntimeError("the self-play engine needs a HIP device (no CPU fallback)")
        self.device = torch.device(device if device is not None else "cuda")
        cfg = nat.AzConfig()
        cfg.n_games = int(n_games)
        cfg.node_capacity = int(node_capacity)
        cfg.max_plies = int(max_plies)
        cfg.num_simulations = int(num_simulations)
        cfg.c_puct = float(c_puct)
        cfg.dirichlet_alpha = float(dirichlet_alpha)
        cfg.dirichlet_epsilon = float(dirichlet_epsilon)
        cfg.temperature = float(temperature)
        cfg.num_exploratory_moves = int(num_exploratory_moves)
        cfg.lambd = float(lambd)
        cfg.eval_mode = nat.AZ_EVAL_ROLLOUT if rollout else nat.AZ_EVAL_EXTERNAL
        cfg.rng_mode = nat.AZ_RNG_INJECTED if injected_rng else nat.AZ_RNG_DEVICE
        cfg.d4_augment = int(bool(d4_augment))
        cfg.auto_play = int(bool(auto_play))
        cfg.refill = int(bool(refill))
        cfg.sample_capacity = int(sample_capacity)
        cfg.inj_noise_slots = int(inj_noise_slots)
        cfg.inj_uniform_slots = int(inj_uniform_slots)
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        cfg.stream_id = int(stream_id)
        cfg.leaves_per_step = int(leaves_per_step)
        self.cfg = cfg
        # bumped whenever a host call changes the Params the kernels take by value
        # (defer_moves, set_stem): HIP graphs captured before it are stale
        self.param_epoch = 0
        self.K = max(1, int(leaves_per_step))
        self.rollout = rollout
        with torch.cuda.device(self.device):
            h = ctypes.c_void_p()
            nat.check(nat.lib.az_engine_create(ctypes.byref(cfg), ctypes.byref(h)),
                      "az_engine_create")
            self.h = h
            G, C, T = (ctypes.c_int32() for _ in range(3))
            nat.check(nat.lib.az_engine_geometry(h, ctypes.byref(G), ctypes.byref(C),
                                                 ctypes.byref(T)), "az_engine_geometry")
            self.G, self.C, self.T = G.value, C.value, T.value
            d = self.device
            R = self.G * self.K  # evaluation rows: leaf j of slot g is row g*K + j
            self.nn_in = torch.zeros(R, 64, dtype=torch.float32, device=d)
            self.leaf = torch.full((R,), -1, dtype=torch.int32, device=d)
            self.priors = torch.zeros(R, 65, dtype=torch.float32, device=d)
            self.values = torch.zeros(R, dtype=torch.float32, device=d)

    def close(self):
        if getattr(self, "h", None):
            nat.lib.az_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- async step pieces (current torch stream) -----------------------------------
    def _s(self):
        return nat.stream_ptr()

    def select(self):
        nat.check(nat.lib.az_select(self.h, nat.ptr(self.nn_in), nat.ptr(self.leaf), self._s()),
                  "az_select")

    def expand(self, priors=None, values=None):
        pr = self.priors if priors is None else priors
        va = self.values if values is None else values
        R = self.G * self.K
        assert pr.dtype == torch.float32 and pr.is_contiguous() and pr.shape == (R, 65)
        assert va.dtype == torch.float32 and va.is_contiguous() and va.numel() == R
        nat.check(nat.lib.az_expand_backup(self.h, nat.ptr(pr), nat.ptr(va), self._s()),
                  "az_expand_backup")

    def play(self):
        nat.check(nat.lib.az_play(self.h, self._s()), "az_play")

    # deferred moves (include/az_othello.h): step n's move phase inside step n+1's select launch
    def defer_moves(self, on=True):
        nat.check(nat.lib.az_engine_defer_moves(self.h, int(bool(on))), "az_engine_defer_moves")
        self.param_epoch += 1

    def select_move(self, par):
        nat.check(nat.lib.az_select_move(self.h, nat.ptr(self.nn_in), nat.ptr(self.leaf), int(par),
                                         self._s()), "az_select_move")

    def expand_par(self, par, priors=None, values=None):
        pr = self.priors if priors is None else priors
        va = self.values if values is None else values
        nat.check(nat.lib.az_expand_backup_par(self.h, nat.ptr(pr), nat.ptr(va), int(par),
                                               self._s()), "az_expand_backup_par")

    def select_move_expand(self, par, priors=None, values=None):
        """One launch per step (az_select_move_expand): the previous step's leaves expanded
        from priors / values, then this step's descents (+ the moves of the step before)."""
        pr = self.priors if priors is None else priors
        va = self.values if values is None else values
        nat.check(nat.lib.az_select_move_expand(self.h, nat.ptr(self.nn_in), nat.ptr(self.leaf),
                                                nat.ptr(pr), nat.ptr(va), int(par), self._s()),
                  "az_select_move_expand")

    def select_expand(self, priors=None, values=None):
        """az_select_expand: the previous select's leaves expanded from priors / values, then
        this select's descents, one launch (engines without deferred moves)."""
        pr = self.priors if priors is None else priors
        va = self.values if values is None else values
        nat.check(nat.lib.az_select_expand(self.h, nat.ptr(self.nn_in), nat.ptr(self.leaf),
                                           nat.ptr(pr), nat.ptr(va), self._s()),
                  "az_select_expand")

    def move_flush(self, par):
        nat.check(nat.lib.az_move_flush(self.h, int(par), self._s()), "az_move_flush")

    def set_stem(self, w9, bias, y, absmax=None):
        """Run the net's stem inside the select launch (az_engine_set_stem): y float32 NHWC
        [G*K, C, 8, 8] receives relu(conv3x3(nn_in row) + bias) of every packed row, absmax
        float32 [G*K] each row's max |y|.  The tensors are kept referenced here.  None turns it
        off."""
        self.param_epoch += 1  # the kernels take Params by value: captured graphs are stale
        if w9 is None:
            self._stem = None
            nat.check(nat.lib.az_engine_set_stem(self.h, None, None, None, None, 0),
                      "az_engine_set_stem")
            return
        R = self.G * self.K
        C = bias.numel()
        assert w9.dtype == bias.dtype == y.dtype == torch.float32 and w9.shape == (9, C)
        assert y.numel() == R * 64 * C and y.is_contiguous(memory_format=torch.channels_last)
        assert absmax is None or (absmax.dtype == torch.float32 and absmax.numel() == R)
        self._stem = (w9, bias, y, absmax)
        nat.check(nat.lib.az_engine_set_stem(self.h, nat.ptr(w9), nat.ptr(bias), nat.ptr(y),
                                             nat.ptr(absmax), C), "az_engine_set_stem")

    # ---- synchronous control --------------------------------------------------------
    def reset_all(self, start_budget=-1, stagger_steps=0):
        nat.check(nat.lib.az_reset_all(self.h, int(start_budget), int(stagger_steps), self._s()),
                  "az_reset_all")

    def set_root(self, slot, own, opp, player):
        nat.check(nat.lib.az_set_root(self.h, int(slot), int(own), int(opp), int(player),
                                      self._s()), "az_set_root")

    def begin_search(self, slot, sims):
        nat.check(nat.lib.az_begin_search(self.h, int(slot), int(sims), self._s()),
                  "az_begin_search")

    def inject(self, noise=None, uniforms=None):
        n = None if noise is None else np.ascontiguousarray(noise, np.float64)
        u = None if uniforms is None else np.ascontiguousarray(uniforms, np.float64)
        nat.check(nat.lib.az_inject(self.h, nat.ptr(n), nat.ptr(u), self._s()), "az_inject")

    def root_policy(self, slot, temp, u_tie=0.0):
        pi = np.zeros(65, np.float32)
        counts = np.zeros(65, np.int32)
        v = ctypes.c_double()
        nat.check(nat.lib.az_root_policy(self.h, int(slot), float(temp), float(u_tie),
                                         nat.ptr(pi), nat.ptr(counts), ctypes.byref(v),
                                         self._s()), "az_root_policy")
        return pi, counts, v.value

    def make_move(self, slot, action):
        nat.check(nat.lib.az_make_move(self.h, int(slot), int(action), self._s()),
                  "az_make_move")

    # ---- batched host-driven control (arena) ----------------------------------------
    def set_roots(self, slots, own, opp, player):
        slots = np.ascontiguousarray(slots, np.int32)
        own = np.ascontiguousarray(own, np.uint64)
        opp = np.ascontiguousarray(opp, np.uint64)
        player = np.ascontiguousarray(player, np.int32)
        nat.check(nat.lib.az_set_roots(self.h, nat.ptr(slots), nat.ptr(own), nat.ptr(opp),
                                       nat.ptr(player), len(slots), self._s()), "az_set_roots")

    def begin_search_slots(self, slots, sims):
        slots = np.ascontiguousarray(slots, np.int32)
        nat.check(nat.lib.az_begin_search_slots(self.h, nat.ptr(slots), len(slots), int(sims),
                                                self._s()), "az_begin_search_slots")

    def root_stats(self):
        counts = np.zeros((self.G, 65), np.int32)
        vroot = np.zeros(self.G, np.float64)
        nat.check(nat.lib.az_root_stats(self.h, nat.ptr(counts), nat.ptr(vroot), self._s()),
                  "az_root_stats")
        return counts, vroot

    def reroot_slots(self, actions):
        actions = np.ascontiguousarray(actions, np.int32)
        assert actions.shape == (self.G,)
        found = np.zeros(self.G, np.int32)
        nat.check(nat.lib.az_reroot_slots(self.h, nat.ptr(actions), nat.ptr(found), self._s()),
                  "az_reroot_slots")
        return found

    def counters(self):
        out = np.zeros(8, np.int64)
        nat.check(nat.lib.az_counters(self.h, nat.ptr(out), self._s()), "az_counters")
        keys = ("games_started", "games_finished", "samples", "samples_dropped",
                "arena_overflows", "steps", "simulations", "moves")
        return dict(zip(keys, (int(x) for x in out)))

    def game_info(self):
        arrs = [np.zeros(self.G, np.int32) for _ in range(6)]
        nat.check(nat.lib.az_game_info(self.h, *[nat.ptr(a) for a in arrs], self._s()),
                  "az_game_info")
        return dict(zip(("status", "ply", "winner", "root_player", "n_nodes", "overflow"),
                        arrs))

    def export_tree(self, slot, max_nodes=None):
        n = ctypes.c_int32()
        nat.check(nat.lib.az_export_tree(self.h, int(slot), 0, *([None] * 12),
                                         ctypes.byref(n), self._s()), "az_export_tree")
        m = n.value if max_nodes is None else min(n.value, max_nodes)
        t = {"own": np.zeros(m, np.uint64), "opp": np.zeros(m, np.uint64),
             "legal": np.zeros(m, np.uint64), "N": np.zeros(m, np.int32),
             "W": np.zeros(m, np.float64), "prior": np.zeros(m, np.float64),
             "parent": np.zeros(m, np.int32), "first": np.zeros(m, np.int32),
             "nchild": np.zeros(m, np.uint8), "action": np.zeros(m, np.uint8),
             "flags": np.zeros(m, np.uint8), "tval": np.zeros(m, np.int8)}
        nat.check(nat.lib.az_export_tree(self.h, int(slot), m, *[nat.ptr(t[k]) for k in t],
                                         ctypes.byref(n), self._s()), "az_export_tree")
        t["n_nodes"] = n.value
        return t

    def export_trajectory(self, slot):
        T = self.T
        own, opp = np.zeros(T, np.uint64), np.zeros(T, np.uint64)
        pi, player = np.zeros((T, 65), np.float32), np.zeros(T, np.int8)
        vroot, n = np.zeros(T, np.float64), ctypes.c_int32()
        nat.check(nat.lib.az_export_trajectory(self.h, int(slot), T, nat.ptr(own), nat.ptr(opp),
                                               nat.ptr(pi), nat.ptr(player), nat.ptr(vroot),
                                               ctypes.byref(n), self._s()),
                  "az_export_trajectory")
        k = n.value
        return {"own": own[:k], "opp": opp[:k], "pi": pi[:k], "player": player[:k],
                "vroot": vroot[:k]}

    def samples(self, start=0, n=None, device=False):
        """Sample rows [start, start+n) as numpy (device=False) or torch device tensors."""
        if n is None:
            n = self.counters()["samples"] - start
        if device:
            out = {"own": torch.empty(n, dtype=torch.int64, device=self.device),
                   "opp": torch.empty(n, dtype=torch.int64, device=self.device),
                   "pi": torch.empty(n, 65, dtype=torch.float32, device=self.device),
                   "z": torch.empty(n, dtype=torch.float64, device=self.device),
                   "player": torch.empty(n, dtype=torch.int8, device=self.device),
                   "slot": torch.empty(n, dtype=torch.int32, device=self.device)}
        else:
            out = {"own": np.zeros(n, np.uint64), "opp": np.zeros(n, np.uint64),
                   "pi": np.zeros((n, 65), np.float32), "z": np.zeros(n, np.float64),
                   "player": np.zeros(n, np.int8), "slot": np.zeros(n, np.int32)}
        nat.check(nat.lib.az_copy_samples(self.h, int(start), int(n),
                                          *[nat.ptr(out[k]) for k in SAMPLE_FIELDS],
                                          self._s()), "az_copy_samples")
        return out

    def clear_samples(self):
        nat.check(nat.lib.az_clear_samples(self.h, self._s()), "az_clear_samples")


def samples_to_tuples(s):
    """Device sample rows -> the reference's training tuples
    [(state int8 (8,8), pi float32 (65,), G float)] (self_play_worker.py:33-35), with
    state = canonical board state*player (own stones +1)."""
    n = len(s["z"])
    ones = np.ones(n, np.int8)
    boards = nat.unpack_np(s["own"], s["opp"], ones)
    return [(boards[i], s["pi"][i].copy(), float(s["z"][i])) for i in range(n)]


class BatchedSelfPlay:
    """G concurrent self-play games on one GPU with a policy/value net.

    `net` is any module with the reference forward signature ([B,1,8,8] -> (logits [B,65],
    value [B,1])); it is evaluated through `Models.inference_copy` (BatchNorm folded,
    channels-last, trunk `precision` "fp16x2" (fp32-accurate, default for fp32) / "split3" / "fp32" /
    "fp16" = config #5).  `args` uses the reference's keys
    (train.py:399-423): c_puct, num_simulations, dirichlet_alpha, dirichlet_epsilon,
    mcts_temperature, num_exploratory_moves, lambda.
    """

    def __init__(self, net, args, n_games, seed=0, stream_id=0, d4_augment=False,
                 dtype=torch.float32, node_capacity=0, sample_capacity=0, use_graph=True,
                 device=None, fold=True, steps_per_graph=8, precision=None, leaves_per_step=1,
                 require_graph=False, defer_moves=True, engine_stem=None, fuse_expand=None,
                 injected_rng=False, inj_noise_slots=1, inj_uniform_slots=1):
        from Models import inference_copy

        self.args = dict(args)
        self.engine = Engine(
            n_games, args["num_simulations"], c_puct=args["c_puct"],
            dirichlet_alpha=args.get("dirichlet_alpha", 1.0),
            dirichlet_epsilon=args.get("dirichlet_epsilon", 0.0),
            temperature=args.get("mcts_temperature", 1.0),
            num_exploratory_moves=args.get("num_exploratory_moves", 0),
            lambd=args.get("lambda", 1.0), rollout=net is None, d4_augment=d4_augment,
            auto_play=True, refill=True, node_capacity=node_capacity,
            sample_capacity=sample_capacity, seed=seed, stream_id=stream_id, device=device,
            leaves_per_step=leaves_per_step, injected_rng=injected_rng,
            inj_noise_slots=inj_noise_slots, inj_uniform_slots=inj_uniform_slots)
        self.device = self.engine.device
        if net is None:
            self.net = None
        elif fold:
            self.net = inference_copy(net, self.device, dtype, precision=precision)
        else:
            self.net = net.to(self.device).eval()
        # defer_moves: each step's move phase (pi, sample, record, re-root) runs in the next
        # step's select launch beside its descents instead of after expand (per game nothing
        # changes); steps alternate a parity the graphs are captured with
        self.defer_moves = bool(defer_moves)
        if self.defer_moves:
            self.engine.defer_moves(True)
        self._par = 0  # parity of the next step (deferred moves)
        # fuse_expand (deferred moves only): the expansion of step n's leaves runs at the start
        # of step n+1's select launch, by each slot's own wave -- one launch per step; default
        # on, AZ_FUSE_EXPAND=0 turns it off (separate k_expand after the evaluation)
        if fuse_expand is None:
            fuse_expand = os.environ.get("AZ_FUSE_EXPAND", "1") != "0"
        self.fuse_expand = bool(fuse_expand) and self.defer_moves
        # engine_stem: the net's stem runs in the select launch, by the wave that packs each
        # row (bit-identical; one launch and the planes' round trip fewer per step); default
        # on where the net supports it, AZ_ENGINE_STEM=0 turns it off
        if engine_stem is None:
            engine_stem = os.environ.get("AZ_ENGINE_STEM", "1") != "0"
        self.engine_stem = False
        if engine_stem and self.net is not None and hasattr(self.net, "engine_stem"):
            st = self.net.engine_stem(self.device, self.engine.G * self.engine.K)
            if st is not None:
                self.engine.set_stem(st["w9"], st["bias"], st["y"], st["absmax"])
                self.engine_stem = True
        self.use_graph = use_graph
        # require_graph: a failed capture raises instead of running eagerly (bench.py: a
        # regression must not show up only as lost throughput)
        self.require_graph = require_graph
        self.graph_error = None
        self.steps_per_graph = max(1, int(steps_per_graph))
        self.graph = None  # {steps: CUDAGraph}: one replay = that many simulation steps

    def _step_body(self, par=0):
        e = self.engine
        if self.fuse_expand:
            e.select_move_expand(par)  # the previous step's leaves, descents, its moves
        elif self.defer_moves:
            e.select_move(par)  # + the previous step's moves
        else:
            e.select()
        if self.net is not None:
            if self.engine_stem:
                self.net.evaluate_into(e.nn_in, e.priors, e.values, stem_done=True)
            elif hasattr(self.net, "evaluate_into"):
                self.net.evaluate_into(e.nn_in, e.priors, e.values)
            else:
                pr, va = self.net.evaluate_planes(e.nn_in)
                e.priors.copy_(pr)
                e.values.copy_(va)
        if self.fuse_expand:
            pass  # expanded by the next step's launch (or step()'s flush)
        elif self.defer_moves:
            e.expand_par(par)
        else:
            e.expand()
            e.play()

    def _capture(self):
        """Capture the step into HIP graphs: one of `steps_per_graph` consecutive steps (the
        host launches one graph per that many steps, so launch cost never paces the GPU)
        and one single step for remainders.  The steps are pure device work on engine state
        in HBM, so replaying a captured sequence is the same computation."""
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm MIOpen / hipBLASLt solution caches outside capture
                self._step_body(self._par)
                self._par ^= 1
        torch.cuda.current_stream().wait_stream(s)
        # graphs keyed by (steps, parity of their first step): the multi-step graph starts at
        # parity 0 (an even number of steps keeps it there), one single step per parity
        k = self.steps_per_graph + (self.steps_per_graph & 1 if self.defer_moves else 0)
        self.steps_per_graph = k
        graphs = {}
        for key in [(k, 0), (1, 0), (1, 1)] if self.defer_moves else [(k, 0), (1, 0)]:
            if key in graphs:
                continue
            n, par = key
            g = torch.cuda.CUDAGraph()  # private memory pool per graph
            with torch.no_grad(), torch.cuda.graph(g):
                for i in range(n):
                    self._step_body(par ^ (i & 1))
            graphs[key] = g
        self.graph = graphs

    def reset(self, start_budget=-1, stagger_steps=0):
        self.engine.reset_all(start_budget, stagger_steps)

    def inject(self, noise=None, uniforms=None):
        """Injected-RNG engines (injected_rng=True): per-slot Dirichlet vectors
        [G, inj_noise_slots, 65] and uniforms [G, inj_uniform_slots] (Engine.inject) replace the
        device Philox draws, so recorded reference games replay through this exact path
        (tests/test_bench_path_gpu.py).  A slot's cursors run on across its games."""
        self.engine.inject(noise, uniforms)

    @torch.no_grad()
    def step(self, n=1):
        self._advance(n)
        if n > 0:
            self._flush()

    def _advance(self, n):
        """n simulation steps on the current stream, without the closing flush."""
        if self.use_graph and self.graph is None:
            try:
                self._capture()
            except Exception as ex:  # capture unsupported for this net: run eagerly
                if self.require_graph:
                    raise
                import warnings

                self.use_graph = False
                self.graph_error = repr(ex)
                warnings.warn(f"HIP graph capture failed, running the step eagerly: {ex!r}")
        if self.graph is None:
            for _ in range(n):
                self._step_body(self._par)
                if self.defer_moves:
                    self._par ^= 1
        else:
            k = self.steps_per_graph
            left = n
            while left > 0:
                if left >= k and self._par == 0:
                    self.graph[(k, 0)].replay()  # k even with deferred moves: parity kept
                    left -= k
                else:
                    self.graph[(1, self._par)].replay()
                    left -= 1
                    if self.defer_moves:
                        self._par ^= 1

    def _flush(self):
        if self.defer_moves:
            # the last step's leaves (fused expansion) and moves, so results read after step()
            # returns are complete
            if self.fuse_expand:
                self.engine.expand_par(self._par ^ 1)
            self.engine.move_flush(self._par ^ 1)

    def counters(self):
        return self.engine.counters()

    def samples_since(self, c0, device=False):
        """Sample rows recorded since counters() returned c0."""
        n = self.counters()["samples"] - c0["samples"]
        return self.engine.samples(c0["samples"], n, device=device)

    def play_games(self, n_games, max_steps=None, check_every=256):
        """Play exactly n_games complete games (slots restart until the budget is used);
        returns the reference's training tuples of every game."""
        e = self.engine
        self.reset(start_budget=n_games)
        limit = max_steps or (n_games // max(1, e.G) + 2) * 200 * (self.args["num_simulations"] + 2)
        done = 0
        steps = 0
        while done < n_games and steps < limit:
            self.step(check_every)
            steps += check_every
            done = e.counters()["games_finished"]
        check_complete(e.counters(), n_games)
        return samples_to_tuples(e.samples())


class PipelinedSelfPlay:
    """G concurrent self-play games as P independent BatchedSelfPlay pipelines of G / P slots,
    each replaying its own HIP graphs on its own HIP stream.  A pipeline's step is dependent
    launches (select + expansion + moves, then the net: the persistent trunk with the heads); the
    select launch leaves most of the chip idle while its slowest descents finish (DESIGN.md
    §5), and with two pipelines the other one's trunk fills it.  Per pipeline nothing changes
    (same kernels and games as a BatchedSelfPlay of G / P slots with its seed and stream id:
    tests/test_pipelined_gpu.py); the host enqueues `steps_per_graph` steps of each pipeline in
    turn.  Pipeline i draws Philox stream stream_id * P + i; its sample rows' slot ids are
    offset by i * G / P."""

    def __init__(self, net, args, n_games, pipelines=2, seed=0, stream_id=0, **kw):
        if pipelines < 1 or n_games % pipelines:
            raise ValueError(f"{n_games} games do not split into {pipelines} pipelines")
        self.P, self.G = int(pipelines), int(n_games)
        self.parts = [BatchedSelfPlay(net, args, n_games // pipelines, seed=seed,
                                      stream_id=stream_id * pipelines + i, **kw)
                      for i in range(pipelines)]
        p0 = self.parts[0]
        self.device = p0.device
        # AZ_PIPE_PRIO (experiments): comma-separated stream priorities per pipeline (lower =
        # higher priority; torch.cuda.Stream.priority_range())
        pr = [int(x) for x in os.environ.get("AZ_PIPE_PRIO", "").split(",") if x.strip()]
        self.streams = [torch.cuda.Stream(device=self.device,
                                          priority=pr[i] if i < len(pr) else 0)
                        for i in range(len(self.parts))]
        self.args, self.net = p0.args, p0.net
        self.defer_moves, self.engine_stem = p0.defer_moves, p0.engine_stem

    @property
    def graph(self):
        return self.parts[0].graph

    @property
    def graph_error(self):
        return next((p.graph_error for p in self.parts if p.graph_error), None)

    def reset(self, start_budget=-1, stagger_steps=0):
        for i, p in enumerate(self.parts):
            b = -1 if start_budget < 0 else start_budget // self.P + (i < start_budget % self.P)
            p.reset(b, stagger_steps)

    @torch.no_grad()
    def step(self, n=1):
        cur = torch.cuda.current_stream(self.device)
        for s in self.streams:
            s.wait_stream(cur)
        k = max(p.steps_per_graph for p in self.parts)
        left = n
        while left > 0:  # round-robin, k steps of each pipeline at a time
            m = min(k, left)
            for p, s in zip(self.parts, self.streams):
                with torch.cuda.stream(s):
                    p._advance(m)
            left -= m
        if n > 0:
            for p, s in zip(self.parts, self.streams):
                with torch.cuda.stream(s):
                    p._flush()
        for s in self.streams:
            cur.wait_stream(s)

    def counters(self):
        per = [p.counters() for p in self.parts]
        out = {k: sum(c[k] for c in per) for k in per[0]}
        out["per_part"] = per
        return out

    def samples_since(self, c0, device=False):
        rows = [p.samples_since(c, device=device) for p, c in zip(self.parts, c0["per_part"])]
        cat = (lambda xs: torch.cat(xs)) if device else (lambda xs: np.concatenate(xs))
        for i, r in enumerate(rows):
            r["slot"] = r["slot"] + i * (self.G // self.P)
        return {k: cat([r[k] for r in rows]) for k in rows[0]}

    def play_games(self, n_games, max_steps=None, check_every=256, tuples=True):
        """Play exactly n_games complete games over the pipelines; returns the reference's
        training tuples of every game (tuples=False: the sample rows)."""
        self.reset(start_budget=n_games)
        c0 = {"samples": 0, "per_part": [{"samples": 0} for _ in self.parts]}
        G = self.G // self.P
        limit = max_steps or (n_games // max(1, G) + 2) * 200 * (self.args["num_simulations"] + 2)
        steps = 0
        while self.counters()["games_finished"] < n_games and steps < limit:
            self.step(check_every)
            steps += check_every
        for i, p in enumerate(self.parts):
            check_complete(p.counters(), n_games // self.P + (i < n_games % self.P))
        rows = self.samples_since(c0)
        return samples_to_tuples(rows) if tuples else rows


def check_complete(c, n_games):
    """Raise unless every requested game finished with the reference's semantics: a node
    arena overflow skips an expansion (engine.hip k_expand), so that search is no longer the
    reference's; dropped sample rows or unfinished games are lost data."""
    if c["arena_overflows"]:
        raise RuntimeError(f"node arena overflowed {c['arena_overflows']} times: the search "
                           "diverged from the reference (raise node_capacity)")
    if c["samples_dropped"]:
        raise RuntimeError(f"{c['samples_dropped']} sample rows dropped: the sample buffer is "
                           "full (raise sample_capacity)")
    if c["games_finished"] < n_games:
        raise RuntimeError(f"only {c['games_finished']} of {n_games} games finished within the "
                           "step limit")
