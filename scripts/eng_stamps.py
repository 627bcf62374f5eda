"""Per-phase latency of the engine kernels at steady state, from an AZ_ENG_STAMP build
(scripts/build_variants.py stamp "-DAZ_ENG_STAMP=1", loaded through AZ_LIB_PATH):
k_move per ready game (root/children load + pi + sample; compaction: parent loads, pointer
jumping, scan, copy; end) and k_expand per sampled slot (first round trip, the rest), in
microseconds (s_memrealtime, 100 MHz): medians / 90th percentiles over the last records.

    AZ_LIB_PATH=... python scripts/eng_stamps.py [warm_steps] > out.json"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alphazero-othello_amd")]
import az_native as nat  # noqa: E402
import bench  # noqa: E402
from engine import BatchedSelfPlay  # noqa: E402
from Models import AlphaZeroNet  # noqa: E402


def stats(x):
    x = np.asarray(x, np.float64) / 100.0  # 100 MHz ticks -> us
    if not len(x):
        return {"n": 0}
    return {"n": int(len(x)), "p50": round(float(np.median(x)), 2),
            "p90": round(float(np.percentile(x, 90)), 2), "mean": round(float(x.mean()), 2)}


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 26000
    torch.manual_seed(0)
    sp = BatchedSelfPlay(AlphaZeroNet(8, 65, 5, 128), bench.SELFPLAY_ARGS, 1024, seed=1,
                         precision="fp16x2")
    sp.reset(-1, 401 * 60)
    for _ in range(warm // 2000):
        sp.step(2000)
        torch.cuda.synchronize()
        print("warm", file=sys.stderr, flush=True)
    sp.step(400)
    torch.cuda.synchronize()
    recs = (ctypes.c_ulonglong * (16384 * 8))()
    n = ctypes.c_uint()
    nat.lib.az_eng_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    nat.check(nat.lib.az_eng_stamps(ctypes.addressof(recs), ctypes.byref(n)), "az_eng_stamps")
    a = np.frombuffer(recs, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
    a = a[a[:, 1] > 0]
    mv, ex = a[a[:, 0] == 1], a[a[:, 0] == 2]
    cmp_ = mv[mv[:, 3] > 0]
    out = {"records": int(n.value),
           "k_move": {"total": stats(mv[:, 7] - mv[:, 1]), "root_pi_sample": stats(mv[:, 2] - mv[:, 1]),
                      "compact_parents": stats(cmp_[:, 4] - cmp_[:, 3]),
                      "compact_jumping": stats(cmp_[:, 5] - cmp_[:, 4]),
                      "compact_scan": stats(cmp_[:, 6] - cmp_[:, 5]),
                      "compact_copy": stats(cmp_[:, 7] - cmp_[:, 6]),
                      "game_end_total": stats((mv[mv[:, 3] == 0][:, 7] - mv[mv[:, 3] == 0][:, 1]))},
           "k_expand": {"total": stats(ex[:, 3] - ex[:, 1]), "first_round_trip": stats(ex[:, 2] - ex[:, 1]),
                        "rest": stats(ex[:, 3] - ex[:, 2])}}
    # per launch: waves of one launch start within a few us of each other; launches are
    # separated by the rest of the step (>= 400 us): split on gaps in the start stamps
    for kind, name in ((2, "k_expand"), (3, "k_select")):
        r = a[a[:, 0] == kind]
        r = r[np.argsort(r[:, 1])]
        if not len(r):
            continue
        cut = np.flatnonzero(np.diff(r[:, 1]) > 10000) + 1  # 100 us
        spans, starts, ends = [], [], []
        for grp in np.split(r, cut):
            if len(grp) < 256:
                continue
            spans.append(grp[:, 3].max() - grp[:, 1].min())
            starts.append(np.percentile(grp[:, 1] - grp[:, 1].min(), 90))
            ends.append(np.percentile(grp[:, 3] - grp[:, 1].min(), 50))
        out.setdefault(name, {})
        out[name]["launch_span_first_start_to_last_end"] = stats(spans)
        out[name]["launch_p90_wave_start_offset"] = stats(starts)
        out[name]["launch_median_wave_end_offset"] = stats(ends)
        if kind == 3:
            out[name]["wave_total"] = stats(r[:, 3] - r[:, 1])
    # the merged select launch (deferred moves + fused expansion): per launch, when each
    # select wave's phases end relative to the launch's first start (expansion -> [2],
    # descent -> [6], stem / bookkeeping -> [3]; [7] = the last descent's depth) and when the
    # move workgroups (kind 1, ends at [7]) end
    r = a[(a[:, 0] == 3) | (a[:, 0] == 1)]
    r = r[np.argsort(r[:, 1])]
    if len(r):
        cut = np.flatnonzero(np.diff(r[:, 1]) > 10000) + 1
        lw = {"span": [], "slowest_select_start": [], "slowest_select_expand": [],
              "slowest_select_descent": [], "slowest_select_finish": [], "slowest_select_depth": [],
              "slowest_is_move": [], "move_end_max": [], "select_end_p50": [], "select_end_p99": []}
        ph = {"expand": [], "descent": [], "finish": [], "depth": []}
        for grp in np.split(r, cut):
            sel, mvg = grp[grp[:, 0] == 3], grp[grp[:, 0] == 1]
            if len(sel) < 256:
                continue
            t0 = grp[:, 1].min()
            send = sel[:, 3] - t0
            mend = (mvg[:, 7] - t0) if len(mvg) else np.zeros(1, np.int64)
            lw["span"].append(max(send.max(), mend.max()))
            lw["move_end_max"].append(mend.max())
            lw["select_end_p50"].append(np.percentile(send, 50))
            lw["select_end_p99"].append(np.percentile(send, 99))
            lw["slowest_is_move"].append(100 * int(mend.max() > send.max()))
            w = sel[np.argmax(send)]
            lw["slowest_select_start"].append(w[1] - t0)
            lw["slowest_select_expand"].append(w[2] - w[1])
            lw["slowest_select_descent"].append(w[6] - w[2])
            lw["slowest_select_finish"].append(w[3] - w[6])
            lw["slowest_select_depth"].append(100 * w[7])
            ph["expand"] += list(sel[:, 2] - sel[:, 1])
            ph["descent"] += list(sel[:, 6] - sel[:, 2])
            ph["finish"] += list(sel[:, 3] - sel[:, 6])
            ph["depth"] += list(100 * sel[:, 7])
        out["merged_select_per_launch"] = {k: stats(v) for k, v in lw.items()}
        out["merged_select_wave_phases"] = {k: stats(v) for k, v in ph.items()}
        out["merged_select_note"] = ("us; *_depth and slowest_is_move are x100 "
                                     "(depth in levels, is_move as a percentage)")
    # the slowest k_expand waves: leaf (0 = a root expansion), path length, arena size, slot
    ex = ex[np.argsort(ex[:, 3] - ex[:, 1])]
    out["k_expand_slowest"] = [{"us": round((r[3] - r[1]) / 100.0, 2), "leaf": int(r[4]),
                                "plen": int(r[5]), "n_nodes": int(r[6]), "slot": int(r[7])}
                               for r in ex[-12:]]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
