"""Is the slow first short window after a long load the chip's power management?  bench.py's
configs[2] engine (1 or 2 pipelines) and warmup; then, repeatedly: `load` untimed steps
(sustained full load), synchronize, an idle pause of `pause_ms`, and one 20-step window timed
as bench.py times it.  If the window's time falls with the pause, the controller's memory of
the sustained load (not the engine) sets the short window's speed.
    python scripts/window_power.py <pipelines> [load steps]"""
import json
import sys
import time

import torch

import window_probe as wp  # noqa: E402  (scripts/ on sys.path when run from the repo root)


def main():
    P = int(sys.argv[1])
    load = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    sp, stagger = wp.build(P)
    sp.step(stagger)
    torch.cuda.synchronize()
    for rep in range(2):
        for pause_ms in (0, 2, 10, 50, 200, 1000):
            sp.step(load)
            torch.cuda.synchronize()
            time.sleep(pause_ms / 1000.0)
            w = wp.window(sp, 20, events=False)
            w2 = wp.window(sp, 20, events=False)  # the next one, right after
            print(json.dumps({"pipelines": P, "load_steps": load, "pause_ms": pause_ms,
                              "rep": rep, "ms_per_step": w["ms_per_step"],
                              "next_ms_per_step": w2["ms_per_step"]}), flush=True)


if __name__ == "__main__":
    main()
