"""Self-play throughput benchmark: games/sec at 400 MCTS simulations per move.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU, RCCL)

Workload (BASELINE.json configs[2], the one the metric is quoted on): 8x8 Othello,
400 sims/move, AlphaZeroNet(8, 65, 5, 128) random init (no checkpoints offline), batched leaf
eval = 1,024: two pipelines of 1,024 concurrent games per GPU on their own HIP streams (one
pipeline's select launch beside the other's trunk), each evaluating its games' one leaf per
step as one batch of 1,024 (--pipelines 1: one 1,024-game pipeline); the reference's
self-play settings (train.py:399-423): c_puct 2, Dirichlet alpha 1 / eps 0.3 at the root,
temperature 1 for 35 plies then 0, lambda 0.98.  The net is fp32-accurate: the 3x3 trunk runs
fp32 operands as exactly scaled fp16 hi + lo pairs, three fp16 MFMA products with fp32
accumulation (Winograd F(2x2,3x3), csrc/conv_wino4.hip; error bounded by the fp32 MFMA
kernel's, tests/test_nn_gpu.py); --conv-precision split3 / fp32 select the bf16x3 and the
plain fp32 MFMA kernels.

A step is one batched simulation over every game slot: select (descent + leaf pack) ->
net forward -> expand+backup -> move phase (with two pipelines, one step of each); games
restart as they finish (weak scaling: 2,048 games per GPU).  Slot starts are staggered over one game length ((sims+1) x 60
steps) so that when the window opens every slot is playing and the slots' game phases are
spread evenly over a game (the continuous self-play steady state: end-game simulations are
cheaper, so a window at one game phase would mis-measure); the untimed warmup runs
max(W, that stagger) steps to get there (reported as warmup_steps_run).  value = simulations run by all ranks in the
timed window / (sims per move x mean plies per game of the games completed in the run) /
window seconds — every move costs exactly `sims` simulations, so this is the game rate,
and it holds for any window length (a window shorter than one move would see few or no
move completions).  The window also contains the per-generation RCCL all-gather of the
finished games' samples.  The move-completion rate and the games that actually finished in
the window are reported beside it.

Also measured in the same run:
  roofline      the bitboard-step kernel (oth_step_gpu, the north-star kernel) on 2^24
                positions of seeded random playouts, timed before the
                self-play warmup and again after the window: 43 algorithmic bytes per
                position (read own, opp, act = 17; write own', opp', legal, status = 26),
                HIP events on the launch stream; traffic = HBM bytes from rocprofv3 PMC
                (profiles/oth_step_traffic.json), or null.
  cpu_baseline  the oracle's restatement of the reference self-play (oracle/mcts.py:
                sequential MCTS, batch-1 torch-CPU inference of the same net, the C board
                oracle) in --cpu-workers single-threaded processes (default: every CPU this
                job is allotted) for a bounded sample of moves each; the per-core rate times
                os.cpu_count() is the whole host's.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "alphazero-othello_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

SELFPLAY_ARGS = {"c_puct": 2.0, "num_simulations": 400, "dirichlet_alpha": 1.0,
                 "dirichlet_epsilon": 0.3, "mcts_temperature": 1.0,
                 "num_exploratory_moves": 35, "lambda": 0.98}
REF_PLIES_PER_GAME = 60.0  # SURVEY.md 6 (measured on the reference at 400 sims)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_COPY_GBS = 6290.0      # the guide's measured float4 copy rate (MI355X_MICROARCH.md)
STEP_BYTES = 43            # algorithmic bytes per board step
MFMA16_PEAK = 2500.0       # dense bf16 / fp16 MFMA TFLOP/s (MI355X_MICROARCH.md)
MFMA32_PEAK = 157.3        # dense fp32 MFMA TFLOP/s
L2_PEAK_TBPS = 34.5        # aggregate L2 bandwidth, 8 XCDs x 4 MiB (MI355X_MICROARCH.md)
DTYPE_LABEL = {
    "split3": "fp32-accurate net (trunk: fp32 operands split into 3 bf16 words, 6 bf16 MFMA "
              "partial products, fp32 accumulation; error <= 2x the fp32 MFMA kernel's vs fp64), int64 bitboards",
    "fp16x2": "fp32-accurate net (trunk: fp32 operands as scaled fp16 hi+lo pairs, 3 fp16 MFMA "
              "partial products, fp32 accumulation; error <= 2x the fp32 MFMA kernel's vs fp64), int64 bitboards",
    "fp32": "fp32 (net), int64 bitboards",
    "fp16": "fp16 trunk operands, fp32 accumulation (net), int64 bitboards",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8000)
    ap.add_argument("--warmup", type=int, default=24000,
                    help="untimed steps; the default (about one game length at 400 sims) lets "
                         "the first games finish so plies/game is measured in this run")
    ap.add_argument("--settle", type=int, default=3,
                    help="untimed windows of --steps steps, each bracketed like the timed one, "
                         "between the warmup and the timed window (the post-load power "
                         "transient: profiles/r06_window_power.json)")
    ap.add_argument("--sustained-steps", type=int, default=2000,
                    help="the warmup's last block of this many steps, timed on its own and "
                         "reported as detail.sustained_ms_per_step (0 = off)")
    ap.add_argument("--warmup-exact", action="store_true",
                    help="run exactly --warmup untimed steps, not the steady-state minimum "
                         "(short profiler runs; the value is then not steady state)")
    ap.add_argument("--workload", default="c3", choices=["c2", "c3", "c4", "c5", "arena"],
                    help="BASELINE.json configs: c2 = configs[1], 4096 games x 100 sims "
                         "FastOthelloNet; c3 = configs[2], 1024 games x 400 sims "
                         "AlphaZeroNet(5x128) fp32 (the metric's config, default); c4 = "
                         "configs[3], 4096 games per GPU x 400 sims AlphaZeroNet(5x128) fp32 "
                         "(32,768 on 8 GPUs, RCCL all-gather); c5 = configs[4], c4 + fused D4 "
                         "symmetry per leaf + fp16 inference; arena = eval.py's play_match / "
                         "evaluate_models_parallel (SURVEY 8(f)1) on configs[2]'s net and sims: "
                         "--matches matches of two random-init AlphaZeroNet(5x128), temperature "
                         "0, colours alternating, the reference's 4 search workers")
    ap.add_argument("--matches", type=int, default=1024,
                    help="arena workload: matches played (and concurrent, one wave)")
    ap.add_argument("--games", type=int, default=None, help="concurrent games per GPU")
    ap.add_argument("--leaves", type=int, default=1,
                    help="virtual-loss leaves per game per step (the reference's num_threads; "
                         "SURVEY 8d C3 allows 256 games x 4 leaves = a 1,024-row leaf batch)")
    ap.add_argument("--sims", type=int, default=None)
    ap.add_argument("--net", default=None, choices=["az5x128", "fast"])
    ap.add_argument("--conv-precision", default=None, choices=["fp16x2", "split3", "fp32", "fp16"],
                    help="3x3 trunk arithmetic: fp16x2 = scaled fp16 hi+lo operand pairs, 3 "
                         "products, fp32 accumulation, fp32-accurate (default for c2-c4; "
                         "64-channel convs use split3); split3 = bf16x3-split operands, 6 "
                         "products, fp32-accurate; fp32 = fp32 MFMA; fp16 = fp16 operands "
                         "(c5's fp16 inference)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-defer", action="store_true",
                    help="the move phase after expand (az_play) instead of inside the next "
                         "step's select launch (deferred moves, the default)")
    ap.add_argument("--no-engine-stem", action="store_true",
                    help="the net's stem as its own kernel on the packed planes instead of "
                         "inside the select launch (az_engine_set_stem, the default where the "
                         "net has a stored fp16x2 stem)")
    ap.add_argument("--steps-per-graph", type=int, default=8,
                    help="simulation steps captured per HIP graph (rocprofv3's kernel tracer "
                         "records 8-step graphs completely: DESIGN.md section 5)")
    ap.add_argument("--pipelines", type=int, default=None,
                    help="the GPU's games as this many independent pipelines, each on its own "
                         "HIP stream (engine.PipelinedSelfPlay: one pipeline's select launch "
                         "overlaps another's trunk); default 2 (measured c2 +8, c3 +4.6, c4 "
                         "+2, c5 +10 %%: profiles/r04_pipelines_ab.json, r05_pipelines_ab.json); "
                         "c3's default games = 1,024 per pipeline, so every evaluation is "
                         "configs[2]'s batch of 1,024 leaves")
    ap.add_argument("--kernel-n", type=int, default=1 << 24)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--cpu-workers", type=int, default=None,
                    help="host cores (one single-threaded process each) for cpu_baseline; "
                         "default: every CPU allotted to this job (host_cpu_share)")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--skip-kernel", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "oth_step_traffic.json"))
    a = ap.parse_args()
    preset = {"c2": (4096, 100, "fast", False, "fp32"), "c3": (1024, 400, "az5x128", False, "fp32"),
              "arena": (1024, 400, "az5x128", False, "fp32"),
              "c4": (4096, 400, "az5x128", False, "fp32"),
              "c5": (4096, 400, "az5x128", True, "fp16")}[a.workload]
    if a.pipelines is None:
        a.pipelines = 2 if a.workload in ("c2", "c3", "c4", "c5") else 1
    # c3 (configs[2]: "batched leaf eval = 1024"): 1,024 concurrent games per pipeline
    a.games = a.games or (1024 * a.pipelines if a.workload == "c3" else preset[0])
    a.sims = a.sims or preset[1]
    a.net = a.net or preset[2]
    a.d4, a.precision = preset[3], preset[4]
    a.conv_precision = a.conv_precision or ("fp16" if a.precision == "fp16" else "fp16x2")
    if a.games % a.pipelines:
        a.pipelines = 1
    return a


def make_net(kind):
    from Models import AlphaZeroNet, FastOthelloNet

    torch.manual_seed(0)
    return AlphaZeroNet(8, 65, 5, 128) if kind == "az5x128" else FastOthelloNet(8, 65)


class _HipEvents:
    """HIP events created with hipEventDisableSystemFence (HIP's timing mode: recording the
    event performs no system-scope cache writeback / invalidate inside the timed interval,
    which a default event -- torch.cuda.Event -- does: "can improve the accuracy of timing
    measurements", hip_runtime_api.h).  Through the HIP runtime torch already loaded (the
    same libamdhip64.so soname, so the same runtime and streams)."""
    FLAG_DISABLE_SYSTEM_FENCE = 0x20000000

    def __init__(self):
        import ctypes

        self.ct = ctypes
        self.lib = ctypes.CDLL("libamdhip64.so")
        self.lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        self.lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                                 ctypes.c_void_p]
        self.lib.hipEventDestroy.argtypes = [ctypes.c_void_p]

    def create(self):
        ev = self.ct.c_void_p()
        assert self.lib.hipEventCreateWithFlags(self.ct.byref(ev), self.FLAG_DISABLE_SYSTEM_FENCE) == 0
        return ev

    def record(self, ev):
        assert self.lib.hipEventRecord(ev, self.ct.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0

    def elapsed_ms(self, e0, e1):
        ms = self.ct.c_float()
        assert self.lib.hipEventElapsedTime(self.ct.byref(ms), e0, e1) == 0
        return ms.value

    def destroy(self, ev):
        self.lib.hipEventDestroy(ev)


class _ProfilerWindow:
    """AZ_PROF_WINDOW=1 under `rocprofv3 --selected-regions`: the profiler records only
    between roctxProfilerResume and roctxProfilerPause, i.e. the timed window (the warmup's
    tens of thousands of graph launches are not traced).  A no-op otherwise."""

    def __init__(self):
        self.lib = None
        if os.environ.get("AZ_PROF_WINDOW") == "1":
            import ctypes

            self.lib = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
            self.lib.roctxProfilerResume.argtypes = [ctypes.c_uint64]
            self.lib.roctxProfilerPause.argtypes = [ctypes.c_uint64]

    def resume(self):
        if self.lib is not None:
            torch.cuda.synchronize()
            self.lib.roctxProfilerResume(0)

    def pause(self):
        if self.lib is not None:
            torch.cuda.synchronize()
            self.lib.roctxProfilerPause(0)


def launch_ms(launch, reps, system_fence=False, before=None):
    """Average duration of one launch: a HIP event pair around each launch on its stream
    (the current torch stream, which the entry points are given), so the figure is the
    kernel's own duration -- the quantity rocprofv3 --kernel-trace reports -- and not the
    back-to-back loop's inter-launch gaps.  Events without the system-scope fence
    (_HipEvents) by default; system_fence=True: torch's default events (each record
    writes back and invalidates the caches inside the interval -- reported beside the
    figure).  before(): untimed work ahead of each pair (e.g. restoring consumed inputs)."""
    if system_fence:
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(reps)]
        for e0, e1 in evs:
            if before:
                before()
            e0.record()
            launch()
            e1.record()
        torch.cuda.synchronize()
        return sum(e0.elapsed_time(e1) for e0, e1 in evs) / reps
    he = _HipEvents()
    evs = [(he.create(), he.create()) for _ in range(reps)]
    for e0, e1 in evs:
        if before:
            before()
        he.record(e0)
        launch()
        he.record(e1)
    torch.cuda.synchronize()
    ms = sum(he.elapsed_ms(e0, e1) for e0, e1 in evs) / reps
    for e0, e1 in evs:
        he.destroy(e0)
        he.destroy(e1)
    return ms


def playout_positions(games=4096, plies=60, seed=0xC0FFEE):
    """SURVEY.md 8(d)'s kernel-bench inputs: positions of seeded uniform-random playouts from
    the initial position (one per game and ply, plies 0..59, finished games dropped), each
    with one uniformly drawn legal action (or the pass).  Played on the product's host entry
    points (oth_legal_cpu / oth_step_cpu, the same bitboard.h code as the kernel)."""
    import az_native as nat

    rng = np.random.default_rng(seed)
    own = np.full(games, 0x0000000810000000, np.uint64)
    opp = np.full(games, 0x0000001008000000, np.uint64)
    live = np.ones(games, bool)
    P, O, A = [], [], []
    bitv = (np.uint64(1) << np.arange(64, dtype=np.uint64))
    for _ in range(plies):
        lg = nat.legal_cpu(own, opp)
        bits = (lg[:, None] & bitv[None, :]) != 0
        # uniform legal placement: argmax of random keys over the set bits; none -> pass
        keys = np.where(bits, rng.random(bits.shape), -1.0)
        act = np.where(bits.any(1), keys.argmax(1), 64).astype(np.uint8)
        P.append(own[live]), O.append(opp[live]), A.append(act[live])
        no, np_, _, st = nat.step_cpu(own, opp, act)
        own, opp = no, np_
        live &= (st & 1) == 0  # terminal flag: the game is over
        if not live.any():
            break
    return np.concatenate(P), np.concatenate(O), np.concatenate(A)


class StepKernelBench:
    """oth_step_gpu over n positions resident in HBM (the playout corpus tiled to n)."""

    def __init__(self, n, device):
        import az_native as nat

        self.nat, self.n = nat, n
        own, opp, act = playout_positions()
        self.host = (own, opp, act)
        reps = -(-n // len(own))
        t = lambda a: torch.from_numpy(np.ascontiguousarray(np.tile(a, reps)[:n])).to(device)
        self.inp = (t(own.view(np.int64)), t(opp.view(np.int64)), t(act))
        self.outs = [torch.empty(n, dtype=torch.int64, device=device) for _ in range(3)]
        self.st = torch.empty(n, dtype=torch.int16, device=device)
        self.args = [nat.ptr(x) for x in self.inp] + [nat.ptr(x) for x in self.outs] + \
            [nat.ptr(self.st), n, nat.stream_ptr()]

    def time_ms(self, warm=400, reps=100, system_fence=False):
        """Average launch time at steady state: `warm` untimed back-to-back launches first
        (the chip's power management takes ~8-200 launches of sustained load to settle
        from a cold start, during which launches run up to 40 % slower:
        profiles/r01_step_steady.json), then `reps` launches, each timed by its own event pair."""
        nat = self.nat
        for _ in range(warm):
            nat.check(nat.lib.oth_step_gpu(*self.args), "oth_step_gpu")
        torch.cuda.synchronize()
        ms = launch_ms(lambda: nat.lib.oth_step_gpu(*self.args), reps, system_fence)
        # spot-check the timed outputs against the host build of the same entry point
        own, opp, act = self.host
        k = min(self.n, len(own))
        co, cp, cl, cs = nat.step_cpu(own[:k], opp[:k], act[:k], raise_illegal=False)
        assert (self.outs[0][:k].cpu().numpy().view(np.uint64) == co).all()
        assert (self.outs[2][:k].cpu().numpy().view(np.uint64) == cl).all()
        assert (self.st[:k].cpu().numpy().view(np.uint16) == cs).all()
        return ms

    def time_io_ms(self, warm=400, reps=100):
        """The same launches of oth_step_io_gpu: k_step2's grid and access pattern (17 B in,
        26 B out per position, non-temporal) with no board arithmetic -- the ceiling of the
        pattern on this box (roofline.pattern_ceiling_*).  Run right after time_ms, so both
        see the chip in the same state."""
        nat = self.nat
        for _ in range(warm):
            nat.check(nat.lib.oth_step_io_gpu(*self.args), "oth_step_io_gpu")
        torch.cuda.synchronize()
        ms = launch_ms(lambda: nat.lib.oth_step_io_gpu(*self.args), reps)
        # the probe really moved the data (no dead loads): own_o = opp, opp_o = own
        k = min(self.n, 4096)
        assert torch.equal(self.outs[0][:k], self.inp[1][:k])
        assert torch.equal(self.outs[1][:k], self.inp[0][:k])
        return ms

    def release(self):
        self.inp = self.outs = self.st = self.args = None


def conv_roofline(sp, device, n_boards):
    """The step's dominant kernel (the fused 3x3 trunk conv: ~90 % of a step's GPU time)
    timed with HIP events on its launch stream, at the bench's leaf batch, with the net's
    own weights.  achieved = MFMA FLOP executed per launch / average launch time against
    the dense peak of the pipe it runs on: split3 executes 6 bf16 products per fp32
    multiply-add (2*B*64*C*C*9 algorithmic FLOP x 6) against 2.5 PFLOP/s; fp16 1x against
    2.5 PFLOP/s; fp32 1x against 157.3 TFLOP/s (MI355X_MICROARCH.md)."""
    import az_native as nat

    conv = sp.net.c2[0]
    C = conv.channels
    refill = lambda: None  # noqa: E731  (wino4: restore the consumed per-board ranges)
    # post-ReLU-like synthetic activations (about half zeros, as the trunk's inputs are):
    # MFMA power -- and with it the clock the chip holds -- depends on the operand values
    x = torch.randn(n_boards, C, 8, 8, device=device).relu().contiguous(
        memory_format=torch.channels_last)
    r = torch.randn_like(x).relu().contiguous(memory_format=torch.channels_last)
    y = torch.empty_like(x)
    if conv.precision == "fp32":
        fn = nat.lib.az_conv3x3_gpu
        args = [nat.ptr(x), nat.ptr(conv.w9), nat.ptr(conv.bias), nat.ptr(r), nat.ptr(y),
                n_boards, C, 1, nat.stream_ptr()]
        kname, mult, peak = "k_conv3x3 (az_conv3x3_gpu, fp32 MFMA)", 1, MFMA32_PEAK
    else:
        algo = getattr(conv, "algo", "direct")
        args = [nat.ptr(x), nat.ptr(conv.wq), nat.ptr(conv.bias), nat.ptr(r), nat.ptr(y),
                n_boards, C, 1, conv.mode]
        mult = {"split3": 6, "fp16x2": 3}.get(conv.precision, 1)
        if algo == "wino4":
            from Models import board_absmax

            # in_absmax is consumed by every launch: refill a work copy beside (outside)
            # each timed launch
            amax = board_absmax(x)
            work = amax.clone()
            fn = nat.lib.az_conv3x3_wino4_gpu
            args += [nat.ptr(work), None]
            refill = lambda: work.copy_(amax)  # noqa: E731
            nbw = int(os.environ.get("AZ_W4_BOARDS", "2"))  # the library's default: 2
            kname = (f"k_conv3x3_wino4 (az_conv3x3_wino4_gpu, Winograd F(2x2,3x3), {nbw} boards "
                     f"per workgroup, {conv.precision})")
        elif algo == "wino":
            fn = nat.lib.az_conv3x3_wino_gpu
            kname = f"k_conv3x3_wino (az_conv3x3_wino_gpu, Winograd F(2x2,3x3), {conv.precision})"
        else:
            fn = nat.lib.az_conv3x3_mx_gpu
            kname = f"k_conv3x3_mx (az_conv3x3_mx_gpu, {conv.precision})"
        if algo in ("wino", "wino4"):  # 16 products per 2x2-output tile instead of 36
            mult = mult * 256 / 576
        args += [nat.stream_ptr()]
        peak = MFMA16_PEAK
    for _ in range(400):  # past the power-management transient (StepKernelBench.time_ms)
        refill()
        nat.check(fn(*args), kname)
    torch.cuda.synchronize()
    ms = launch_ms(lambda: fn(*args), 100, before=refill)  # refill outside the timed pair
    flop = 2.0 * n_boards * 64 * C * C * 9
    achieved = mult * flop / (ms * 1e-3) / 1e12
    traffic = None  # HBM bytes per launch, PMC (scripts/pmc_conv.sh), for the default form
    tj = os.path.join(ROOT, "profiles", "conv_traffic.json")
    if os.path.exists(tj):
        try:
            tjd = json.load(open(tj))
            if tjd.get("kernel_tag") == f"{getattr(conv, 'algo', 'direct')}_{conv.precision}_{C}":
                traffic = tjd.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    out = {"kernel": kname + ", fused bias+residual+ReLU", "bound": "mfma",
           "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
           "frac": round(achieved / peak, 4), "traffic": traffic, "boards": n_boards,
           "channels": C, "avg_launch_ms": round(ms, 4), "flop_per_launch": flop,
           "mfma_flop_per_algorithmic_flop": round(mult, 4),
           "algorithmic_tflops": round(flop / (ms * 1e-3) / 1e12, 1)}
    if conv.precision != "fp32":
        # every workgroup streams the whole pre-split weight set from L2
        algo = getattr(conv, "algo", "direct")
        per_wg = (16 if algo in ("wino", "wino4") else 9) * C * C * \
            {"split3": 3, "fp16x2": 2}.get(conv.precision, 1) * 2
        nbw = int(os.environ.get("AZ_W4_BOARDS", "2"))
        wgs = {"wino": (n_boards + 1) // 2,
               "wino4": (n_boards + nbw - 1) // nbw}.get(algo, n_boards)
        out["l2_weight_stream"] = {"bytes_per_launch": per_wg * wgs,
                                   "achieved_TBps": round(per_wg * wgs / (ms * 1e-3) / 1e12, 2),
                                   "peak_TBps": L2_PEAK_TBPS}
    return out


CALIBRATION_JSON = os.path.join(ROOT, "profiles", "cpu_calibration.json")


def trunk_roofline(sp, device, n_boards):
    """The step's dominant launch since round 4 -- the whole net after the engine's select
    launch: k_trunk_wino4, the stem, every block conv and the heads in one persistent kernel
    (FusedInferenceNet.evaluate_into on canonical planes) -- timed with HIP events on its
    launch stream at the bench's leaf batch.  achieved = the block convs' MFMA FLOP per launch
    (2*B*64*C*C*9 algorithmic per conv x 16/36 Winograd x 3 fp16x2 products) / the average
    launch time, against the dense fp16 MFMA peak; the stem and heads (< 1 % of the FLOP) are
    inside the time but not counted.  configs[4]'s fp16 net runs the same launch in fp16
    (az_trunk_wino4_heads_fp16_gpu: one product); above 4 x CUs boards the evaluation is one
    launch per resident chunk and the time is the evaluation's."""
    net = sp.net
    if not (hasattr(net, "c1") and getattr(net, "conv_impl", "") == "hip" and net.c1):
        return None
    prec = net.c1[0].precision
    if not (prec in ("fp16x2", "fp16")
            and all(getattr(c, "algo", "") == "wino4" and c.precision == prec
                    for c in list(net.c1) + list(net.c2))):
        return None
    C, n_convs = net.c1[0].channels, 2 * len(net.c1)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randint(-1, 2, (n_boards, 64), generator=g).float().to(device)
    pr = torch.empty(n_boards, 65, device=device)
    va = torch.empty(n_boards, device=device)
    with torch.no_grad():
        for _ in range(200):  # past the power-management transient
            net.evaluate_into(x, pr, va)
        torch.cuda.synchronize()
        ms = launch_ms(lambda: net.evaluate_into(x, pr, va), 50)
    flop = 2.0 * n_boards * 64 * C * C * 9 * n_convs
    mult = (3 if prec == "fp16x2" else 1) * 256 / 576
    executed = mult * flop / (ms * 1e-3) / 1e12
    # the whole net's algorithmic FLOP per evaluation (189.0 MFLOP for
    # AlphaZeroNet(5x128)): stem 3x3 (1 -> C), the block convs, the 1x1 policy (2) + value (1)
    # convs, pol_fc (128 -> 65), val_fc1 (64 -> 256), val_fc2 (256 -> 1)
    per_eval = (2 * 64 * C * 9 + 2 * 64 * C * C * 9 * n_convs + 2 * 64 * C * 3
                + 2 * 128 * 65 + 2 * 64 * 256 + 2 * 256)
    algorithmic = per_eval * n_boards / (ms * 1e-3) / 1e12
    # HBM bytes per launch from the committed PMC summary (scripts/trunk_traffic.py), used only
    # while the trunk kernel is the one it was measured on: the file records the hash of the
    # trunk's sources, and the loaded library must be the build of the tree's sources (a kernel
    # change makes the figure stale: reported as such, traffic null)
    traffic, source = None, None
    tj = os.path.join(ROOT, "profiles", "trunk_traffic.json")
    if n_boards == 1024 and prec == "fp16x2" and os.path.exists(tj):
        try:
            import az_build
            import az_native as nat

            tjd = json.load(open(tj))
            kernel = az_build.sources_hash(az_build.TRUNK_SOURCES)
            source = {"file": "profiles/trunk_traffic.json", "measured": tjd.get("source"),
                      "trunk_sources_hash": tjd.get("trunk_sources_hash"),
                      "current_trunk_sources_hash": kernel,
                      "library_is_tree_build": nat.build_id() == az_build.source_hash()}
            if tjd.get("trunk_sources_hash") == kernel and source["library_is_tree_build"]:
                traffic = tjd.get("hbm_bytes_per_launch")
            else:
                source["stale"] = "measured on another trunk kernel: not reported"
        except (OSError, ValueError):
            traffic = None
    fn = "az_trunk_wino4_heads_gpu" if prec == "fp16x2" else "az_trunk_wino4_heads_fp16_gpu"
    cap = net._trunk4_cap(device)
    return {"kernel": "k_trunk_wino4 (%s: stem + %d block convs, Winograd F(2x2,3x3) %s, two "
                      "boards per workgroup, each layer's input resident in LDS, + heads)"
                      % (fn, n_convs, prec),
            "launches_per_evaluation": -(-n_boards // cap),
            "bound": "mfma", "achieved": round(algorithmic, 1), "peak": MFMA16_PEAK,
            "unit": "TFLOP/s", "frac": round(algorithmic / MFMA16_PEAK, 4), "traffic": traffic,
            "traffic_source": source,
            "achieved_basis": "algorithmic: the net's %.1f MFLOP per evaluation x boards / launch "
                              "time" % (per_eval / 1e6),
            "mfma_executed_tflops": round(executed, 1),
            "frac_mfma_executed": round(executed / MFMA16_PEAK, 4),
            "boards": n_boards, "avg_launch_ms": round(ms, 4), "conv_flop_per_launch": flop,
            "algorithmic_flop_per_eval": per_eval,
            "mfma_flop_per_algorithmic_flop": round(mult, 4),
            "us_per_conv": round(ms * 1e3 / n_convs, 2)}


def cpu_baseline(net_kind, sims, seconds, seed=0, start_ply=0, full_games=0):
    """The oracle's restatement of one_self_play (reference algorithm, sequential MCTS,
    batch-1 torch-CPU inference, C board oracle) on one core.  The worker reaches ply
    `start_ply` with seeded uniformly random legal moves (no search), then runs 400-sim
    moves (fresh tree, then tree reuse as the reference does) until `seconds` are used,
    starting over from the same ply when a game ends; games/s = 1 / (seconds per move x
    plies per game).  full_games > 0: play that many complete games from the initial
    position instead (the calibration against the reference pool, scripts/
    calibrate_cpu_baseline.py)."""
    from oracle import board as ob
    from oracle.mcts import SeqMCTS

    torch.set_num_threads(1)
    cpu_net = make_net(net_kind).cpu().eval()

    def evaluate(own, opp, player):
        s = ob.to_state(own, opp, player)
        x = torch.from_numpy((player * s).astype(np.float32)).unsqueeze(0)
        with torch.no_grad():
            logits, v = cpu_net(x)
            p = torch.softmax(logits, -1)
        return p[0].numpy(), float(v[0, 0])

    np.random.seed(seed)
    rng = np.random.default_rng(seed)
    a = SELFPLAY_ARGS
    game = ob.OracleGame()

    def opening(plies):
        state, player = game.get_initial_state(), 1
        for _ in range(plies):
            valid = np.nonzero(game.get_valid_moves(state, player))[0]
            act = int(rng.choice(valid))
            nxt = game.get_next_state(state, act, player)
            if game.get_value_and_terminated(nxt, act, player)[1]:
                break
            state, player = nxt, -player
        return state, player

    moves, games = 0, 0
    t0 = time.perf_counter()
    while True:
        m = SeqMCTS(a["c_puct"], sims, evaluate, dirichlet_alpha=a["dirichlet_alpha"],
                    dirichlet_epsilon=a["dirichlet_epsilon"])
        state, player = opening(0 if full_games else start_ply)
        ply = 0 if full_games else start_ply
        while True:
            own, opp = ob.to_bitboards(state, player)
            temp = a["mcts_temperature"] if ply < a["num_exploratory_moves"] else 0.0
            pi = m.search(own, opp, player, temp)
            action = int(np.random.choice(65, p=pi))
            m.make_move(action)
            state = game.get_next_state(state, action, player)
            moves += 1
            ply += 1
            done = game.get_value_and_terminated(state, action, player)[1]
            if done or (not full_games and time.perf_counter() - t0 >= seconds):
                break
            player = -player
        if done:
            games += 1
        if full_games and games >= full_games:
            break
        if not full_games and time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    if full_games:
        return {"moves": moves, "seconds": dt, "games": games, "games_per_s": games / dt}
    return {"moves": moves, "seconds": dt, "start_ply": start_ply,
            "games_per_s": 1.0 / (dt / moves * REF_PLIES_PER_GAME)}


def _cpu_pool(net_kind, sims, seconds, workers, full_games=0):
    import subprocess

    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
               ROCR_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    procs = []
    for w in range(workers):
        # start plies spread uniformly over a game (0, 7, 15, ..., 52 for 8 workers)
        ply = int(w * REF_PLIES_PER_GAME / workers)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker",
                                       net_kind, str(sims), str(seconds), str(w), str(ply),
                                       str(full_games)],
                                      stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env))
    outs = []
    for pr in procs:
        out, _ = pr.communicate(timeout=(seconds + 600) * 10 if not full_games else 7200)
        if pr.returncode != 0:
            raise RuntimeError(f"cpu baseline worker failed ({pr.returncode})")
        outs.append(json.loads(out.decode().strip().splitlines()[-1]))
    return outs


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpu_share():
    """CPUs this process may actually run on: the affinity mask, capped by a cgroup-v2 CPU
    quota (a GPU box shows the whole machine in os.cpu_count() but allots a job a share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def calibration_for(cal, net_kind, sims, model, n_cpus):
    """The reference/port ratio of profiles/cpu_calibration.json, applicable only to the
    same net and sims on the same CPU model with the same CPU count it was measured on (the
    gap between the reference's threaded Python search and the port depends on the CPU)."""
    if not cal or cal.get("net") != net_kind or cal.get("sims") != sims:
        return None
    if cal.get("cpu_model") != model or cal.get("os_cpu_count") != n_cpus:
        return None
    return cal.get("ratio_reference_over_port")


def cpu_baseline_pool(net_kind, sims, seconds, workers):
    """cpu_baseline on `workers` host cores at once, one single-threaded process each
    (started before any GPU work of theirs could exist: they hide the GPUs), like the
    reference's spawn-pool self-play workers (train.py:210-222, one per host core); worker w
    samples the game from ply w*60/workers, so the moves cover the whole game.  Games are
    independent processes, so the host's rate is the per-core rate x os.cpu_count()
    (BASELINE.md section 3): `value` with `cores` = os.cpu_count(), the measured cores beside
    it.  The calibration ratio (reference pool / port, full games) scales `value` only on
    the CPU model and count it was measured on; elsewhere it is reported, not applied."""
    outs = _cpu_pool(net_kind, sims, seconds, workers)
    moves = sum(o["moves"] for o in outs)
    # worker w times the plies from w*60/W on, so a game's length in seconds is 60 x the
    # MEAN seconds per move over the workers (averaging per-worker game rates instead
    # would let the cheap end-game moves of the last workers dominate)
    s_per_move = [o["seconds"] / max(1, o["moves"]) for o in outs]
    s_per_game = REF_PLIES_PER_GAME * float(np.mean(s_per_move))
    per_core = 1.0 / s_per_game
    port = per_core * workers  # the measured cores together
    n_host = os.cpu_count() or workers
    model = cpu_model()
    cal = json.load(open(CALIBRATION_JSON)) if os.path.exists(CALIBRATION_JSON) else None
    ratio = calibration_for(cal, net_kind, sims, model, n_host)
    host = per_core * n_host
    net_name = "AlphaZeroNet(5,128)" if net_kind == "az5x128" else "FastOthelloNet"
    cal_note = None
    if cal:
        cal_note = {"ratio_reference_over_port": cal.get("ratio_reference_over_port"),
                    "cpu_model": cal.get("cpu_model"), "os_cpu_count": cal.get("os_cpu_count"),
                    "games_per_side": (cal.get("reference") or {}).get("games"),
                    "applied": ratio is not None}
    return {"value": host * ratio if ratio else host, "unit": "games/s",
            "cores": n_host, "kind": "port", "cores_measured": workers,
            "per_core_games_per_s": per_core, "measured_cores_games_per_s": port,
            "calibration_ratio": ratio, "calibration": cal_note,
            "cpu_model": model, "os_cpu_count": n_host,
            "sample": f"{workers} single-threaded worker processes (the CPUs allotted to this "
                      f"job) at once; worker w plays from ply w*{int(REF_PLIES_PER_GAME)}/"
                      f"{workers} (seeded random opening) for {seconds:.0f} s of {sims}-sim "
                      f"moves ({moves} moves in all); {net_name} fp32 batch-1 torch-CPU, "
                      f"oracle/mcts.py SeqMCTS; seconds per game = {REF_PLIES_PER_GAME:.0f} x the "
                      f"mean seconds per move over the workers ({s_per_game:.1f} s); value = "
                      f"os.cpu_count() = {n_host} cores / seconds per game (independent game "
                      "processes scale by core; on an SMT host this overstates the CPU)"
                      + (f" x calibration_ratio {ratio:.3f}" if ratio else
                         "; uncalibrated: the calibration's CPU differs, and the port is faster "
                         "than the reference there (ratio < 1), so this overstates the CPU"),
            "seconds_per_game": round(s_per_game, 3),
            "per_worker_s_per_move": [round(t, 4) for t in s_per_move]}


STAT_KEYS = ("moves", "games_done", "sims", "plies_total", "games_total", "window_s")


def gather_stats(stats, dist, world):
    """Every rank's window statistics (a float64 vector in STAT_KEYS order) as a
    [world, 6] array on every rank (one all_gather; a plain copy at world 1)."""
    if dist is None:
        return stats.cpu().numpy()[None]
    allst = [torch.zeros_like(stats) for _ in range(world)]
    dist.all_gather(allst, stats)
    return torch.stack(allst).cpu().numpy()


def aggregate_stats(allst, sims_per_move):
    """Whole-job figures from gather_stats' rows: counts summed over ranks, the window =
    the slowest rank's (max over ranks), plies per game from every rank's completed games
    (the reference's 60 until 16 exist).  Every slot always has a game in progress and runs
    one simulation per step; a move is exactly `sims` simulations, so games/s =
    simulations/s / (sims x plies per game).  (Game completions inside the window follow the
    start schedule of the first game generation rather than the steady state, so they are
    reported, not used.)"""
    allst = np.asarray(allst, np.float64).reshape(-1, len(STAT_KEYS))
    tot = allst.sum(0)
    t_max = float(allst[:, 5].max())
    gtot = tot[4]
    plies_per_game = float(tot[3] / gtot) if gtot >= 16 else REF_PLIES_PER_GAME
    return {"value": float(tot[2] / sims_per_move / plies_per_game / t_max),
            "moves": float(tot[0]), "games_done": float(tot[1]), "sims": float(tot[2]),
            "plies_per_game": plies_per_game, "window_s": t_max,
            "per_rank": [{"sims": int(r[2]), "moves": int(r[0]), "window_s": round(float(r[5]), 4)}
                         for r in allst]}


def main_arena(a):
    """eval.py's evaluate_models_parallel (eval.py:47-74) with play_match (:134-178) per match,
    as arena.BatchedArena plays it: matches/s.  Two random-init nets of configs[2]'s
    architecture, 400 sims, no num_threads in args (the reference's default of 4 workers =
    4 virtual-loss leaves per searching slot per step), temperature 0, colours alternating.
    A warm-up wave at 8 sims captures the search graphs first (the graphs do not depend on
    the simulation count); the timed region is one arena.play over --matches matches."""
    from arena import BatchedArena
    from Models import AlphaZeroNet

    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    torch.manual_seed(0)
    net_a = AlphaZeroNet(8, 65, 5, 128)
    torch.manual_seed(1)
    net_b = AlphaZeroNet(8, 65, 5, 128)
    args = {"c_puct": 2.0, "num_simulations": a.sims}
    n = a.matches
    arena = BatchedArena(net_a, net_b, args, n, device=device, seed=1234)
    np.random.seed(0)
    arena.args = dict(args, num_simulations=8)
    arena.play(n)  # warm-up: the same wave layout, so every graph of the timed run exists
    arena.args = args
    torch.cuda.synchronize()
    it0 = arena.iterations
    t0 = time.perf_counter()
    wa, wb, dr, plies = arena.play(n)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    its = arena.iterations - it0
    result = {
        "metric": f"arena matches/sec (eval.py play_match), 8x8 Othello @ {a.sims} MCTS sims/move",
        "value": round(n / dt, 4), "unit": "matches/s", "n_gpus": 1, "steps": its,
        "warmup": 1, "ms_per_step": round(dt * 1000.0 / max(1, its), 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": DTYPE_LABEL[a.conv_precision],
        "data": "synthetic: matches from the initial position, two random-init nets",
        "config": {"workload": "SURVEY 8(f)1 arena: eval.py evaluate_models_parallel on the "
                               "GPU engine, configs[2]'s AlphaZeroNet(5x128) fp32 and sims",
                   "matches": n, "sims": a.sims, "leaves_per_step": arena.K,
                   "hip_graph": arena.use_graph, "graphs": len(arena._graphs)},
        "value_basis": "matches / wall seconds of one arena.play (a step = one select -> net "
                       "-> expand iteration of every searching engine)",
        "detail": {"wins_a": wa, "wins_b": wb, "draws": dr,
                   "mean_plies": round(float(np.mean(plies)), 2), "window_s": round(dt, 3),
                   "iterations": its}}
    print(json.dumps(result), flush=True)


def main():
    a = parse()
    if a.workload == "arena":
        return main_arena(a)
    if os.environ.get("AZ_FAULTHANDLER"):  # diagnostics: every thread's Python stack on a fault
        import faulthandler

        faulthandler.enable(all_threads=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AZ_BENCH_REHEARSE=1: every rank on cuda:0 with gloo collectives (rehearses the N>1
    # path on a one-GPU box); otherwise one GPU per rank and RCCL ("nccl")
    rehearse = os.environ.get("AZ_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    coll_device = torch.device("cpu") if rehearse else device
    dist = None
    if world > 1:
        import torch.distributed as dist

        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    from engine import BatchedSelfPlay, PipelinedSelfPlay

    net = make_net(a.net)
    args = dict(SELFPLAY_ARGS, num_simulations=a.sims)
    kw = dict(seed=1234, stream_id=rank, use_graph=not a.no_graph, require_graph=not a.no_graph,
              device=device, d4_augment=a.d4,
              dtype=torch.float16 if a.precision == "fp16" else torch.float32,
              sample_capacity=a.games // a.pipelines * 130 * 4, steps_per_graph=a.steps_per_graph,
              defer_moves=not a.no_defer, engine_stem=not a.no_engine_stem,
              precision=a.conv_precision, leaves_per_step=a.leaves)
    if a.pipelines > 1:
        sp = PipelinedSelfPlay(net, args, a.games, pipelines=a.pipelines, **kw)
    else:
        sp = BatchedSelfPlay(net, args, a.games, **kw)
    if os.environ.get("AZ_DUMP_MAPS"):  # diagnostics: the address map, to place a fault's PC
        with open("/proc/self/maps") as f_in, open(os.environ["AZ_DUMP_MAPS"], "w") as f_out:
            f_out.write(f_in.read())
    # stagger slot starts over one game length: at the end of the warmup every slot plays
    # and the game phases are uniform (steady state of continuous self-play)
    stagger = (-(-a.sims // a.leaves) + 1) * int(REF_PLIES_PER_GAME)
    warmup_run = a.warmup if a.warmup_exact else max(a.warmup, stagger)
    sp.reset(start_budget=-1, stagger_steps=stagger)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    # the north-star kernel first, with the chip in the state the profiler run also sees it
    # in (rocprofv3 serialises the self-play, which then heats the chip less): the figure
    # agrees with the committed rocprof summary; it is re-timed after the window below
    kb = None
    if rank == 0 and not a.skip_kernel:
        kb = StepKernelBench(a.kernel_n, device)
        ms_step_kernel = kb.time_ms()
        ms_io_kernel = kb.time_io_ms()
    sp.step(warmup_run)
    barrier()
    # the sustained rate (reported beside the line, never part of value): the untimed warmup's
    # continuation, --sustained-steps more steps in one block
    sustained = None
    if a.sustained_steps > 0:
        ts = time.perf_counter()
        sp.step(a.sustained_steps)
        barrier()
        sustained = (time.perf_counter() - ts) * 1000.0 / a.sustained_steps
    # settle windows (untimed): --settle blocks of exactly the timed window's shape (barrier,
    # counters, --steps steps, counters, barrier).  After seconds of sustained full load the
    # chip's power management makes the next one or two short windows up to ~25 % slower than
    # both the sustained rate and every later window (profiles/r06_window_power.json: a
    # window's time also grows with the idle pause before it); these blocks let that transient
    # pass before the timed window, which then sees the conditions every later window does
    settle = []
    for _ in range(a.settle):
        barrier()
        sp.counters()
        tq = time.perf_counter()
        sp.step(a.steps)
        sp.counters()
        barrier()
        settle.append(round((time.perf_counter() - tq) * 1000.0 / a.steps, 4))
    barrier()
    prof = _ProfilerWindow()  # AZ_PROF_WINDOW=1: rocprofv3 --selected-regions traces the window only
    c0 = sp.counters()
    t0 = time.perf_counter()
    prof.resume()
    sp.step(a.steps)
    # per-generation exchange: all-gather the finished games' samples over RCCL/xGMI
    c_mid = sp.counters()
    n_new = c_mid["samples"] - c0["samples"]
    allgather_rows = n_new
    if dist is not None:
        from dist_replay import allgather_samples

        pooled, counts = allgather_samples(sp.samples_since(c0, device=not rehearse), coll_device)
        allgather_rows = int(sum(counts))
    barrier()
    dt = time.perf_counter() - t0
    prof.pause()
    c1 = sp.counters()
    # AZ_BENCH_REPEAT=k (diagnostics): k more windows of the same length after the timed one,
    # timed the same way, reported beside the line (never part of value)
    repeat = []
    for _ in range(int(os.environ.get("AZ_BENCH_REPEAT", "0"))):
        barrier()
        sp.counters()
        tr = time.perf_counter()
        sp.step(a.steps)
        sp.counters()
        barrier()
        repeat.append(round((time.perf_counter() - tr) * 1000.0 / a.steps, 4))
    moves = c1["moves"] - c0["moves"]
    games_done = c1["games_finished"] - c0["games_finished"]
    sims = c1["simulations"] - c0["simulations"]
    plies_total = c1["samples"]
    games_total = c1["games_finished"]
    stats = torch.tensor([moves, games_done, sims, plies_total, games_total, dt],
                         dtype=torch.float64, device=coll_device)
    allst = gather_stats(stats, dist, world)
    agg = aggregate_stats(allst, a.sims)
    t_max, plies_per_game, value = agg["window_s"], agg["plies_per_game"], agg["value"]
    moves_all, games_all, sims_all = agg["moves"], agg["games_done"], agg["sims"]
    basis = ("simulations in the window / (sims per move x mean plies per completed game) / "
             "window seconds (all ranks)")

    result = {
        "metric": f"self-play games/sec (whole node), 8x8 Othello @ {a.sims} MCTS sims/move",
        "value": round(float(value), 4), "unit": "games/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "warmup_steps_run": warmup_run + max(0, a.sustained_steps) + a.settle * a.steps,
        "ms_per_step": round(t_max * 1000.0 / a.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": DTYPE_LABEL[a.conv_precision],
        "data": "synthetic: self-play from the initial position, random-init net weights",
        "config": {"workload": {"c3": "configs[2]: 8x8 Othello, 400 sims/move, AlphaZeroNet(5x128) "
                                      "random init fp32, batched leaf eval = 1024 (each "
                                      "pipeline's concurrent games, one leaf each per step)",
                                "c2": "configs[1]: 8x8 Othello, 4096 concurrent games, 100 sims/move, "
                                      "FastOthelloNet random init fp32",
                                "c4": "configs[3]: 8x8 Othello, 4096 concurrent games per GPU "
                                      f"({4096 * world} on {world} GPU(s)), 400 sims/move, "
                                      "AlphaZeroNet(5x128) random init fp32, RCCL all-gather "
                                      "of the generation's samples",
                                "c5": "configs[4]: configs[3] (4096 games per GPU) + fused D4 "
                                      "symmetry per leaf + fp16 net inference"}[a.workload],
                   "d4_augment": a.d4,
                   "games_per_gpu": a.games, "sims": a.sims, "net": a.net,
                   "leaves_per_step": a.leaves,
                   "leaf_batch": a.games // a.pipelines * a.leaves,
                   "parallelism": f"dp{world} (independent games per GPU)",
                   "pipelines": a.pipelines,
                   "hip_graph": sp.graph is not None, "graph_error": sp.graph_error,
                   "deferred_moves": sp.defer_moves, "engine_stem": sp.engine_stem},
        "value_basis": basis,
        "detail": {"moves": int(moves_all),
                   "moves_based_games_per_s": round(float(moves_all / plies_per_game / t_max), 4), "games_finished_in_window": int(games_all),
                   "simulations": int(sims_all), "plies_per_game": round(float(plies_per_game), 2),
                   "sims_per_s": round(float(sims_all / t_max), 1),
                   "window_s": round(t_max, 3), "allgather_rows": allgather_rows,
                   "arena_overflows": int(c1["arena_overflows"]),
                   "samples_dropped": int(c1["samples_dropped"])},
    }
    if repeat:
        result["detail"]["repeat_ms_per_step"] = repeat
    if settle:
        result["detail"]["settle_ms_per_step"] = settle
    if sustained is not None:
        result["detail"]["sustained_ms_per_step"] = round(sustained, 4)
        result["detail"]["sustained_steps"] = a.sustained_steps
    if dist is not None:
        # what the process group actually was, and every rank's share (a SCALE line shows
        # by itself that N ranks ran and how value was formed)
        result["dist"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                          "per_rank": agg["per_rank"]}
    if kb is not None:
        ms, n = ms_step_kernel, a.kernel_n
        ms_hot = kb.time_ms()
        # the same launches timed with default (system-fence) events, last: for comparison
        # only (each record writes back and invalidates the caches, and the launch after it
        # starts cold: profiles/r03_step_rocprof_timed_fencefree.json)
        ms_step_fenced = kb.time_ms(warm=100, system_fence=True)
        kb.release()
        achieved = STEP_BYTES * n / (ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(a.traffic_json):
            try:
                traffic = json.load(open(a.traffic_json)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        result["roofline"] = {"kernel": "oth_step_gpu (k_step2, two positions per lane)", "bound": "hbm",
                              "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                              "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),
                              "traffic": traffic, "positions": n,
                              "avg_launch_ms": round(ms, 4),
                              "gsteps_per_s": round(n / (ms * 1e-3) / 1e9, 2),
                              "inputs": "seeded random playouts (SURVEY.md 8d: seed 0xC0FFEE, "
                                        "plies 0-59, one legal action each), tiled to 2^24",
                              "timing": "HIP event pair per launch on its stream, events "
                                        "without the system-scope fence (hipEventDisableSystemFence)",
                              "avg_launch_ms_default_events": round(ms_step_fenced, 4),
                              "frac_default_events": round(STEP_BYTES * n / (ms_step_fenced * 1e-3)
                                                           / 1e9 / HBM_PEAK_GBS, 4),
                              "pattern_ceiling_ms": round(ms_io_kernel, 4),
                              "pattern_ceiling_GBps": round(STEP_BYTES * n / (ms_io_kernel * 1e-3) / 1e9, 1),
                              "pattern_ceiling_frac": round(ms_io_kernel / ms, 4),
                              "pattern_ceiling": "oth_step_io_gpu: the same grid and 17 B in / 26 B "
                                                 "out non-temporal accesses with no board "
                                                 "arithmetic, timed right after; "
                                                 "pattern_ceiling_frac = its time / k_step2's",
                              "avg_launch_ms_after_selfplay": round(ms_hot, 4),
                              "frac_after_selfplay": round(STEP_BYTES * n / (ms_hot * 1e-3)
                                                           / 1e9 / HBM_PEAK_GBS, 4)}
    if rank == 0 and not a.skip_kernel and hasattr(sp.net, "c2") \
            and getattr(sp.net, "conv_impl", "") == "hip":
        lb = a.games // a.pipelines * a.leaves  # one evaluation's boards
        result["roofline_conv"] = conv_roofline(sp, device, lb)
        rt = trunk_roofline(sp, device, lb)  # above 4 x CUs boards: one launch per chunk
        if rt is not None:
            result["roofline_trunk"] = rt
    if rank == 0 and world == 1 and not a.skip_cpu:  # the contract: rank 0 at N = 1 only
        result["cpu_baseline"] = cpu_baseline_pool(a.net, a.sims, a.cpu_seconds,
                                                   a.cpu_workers or host_cpu_share())
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu-worker":  # cpu_baseline_pool's workers
        print(json.dumps(cpu_baseline(sys.argv[2], int(sys.argv[3]), float(sys.argv[4]),
                                      int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7]))),
              flush=True)
    else:
        main()
