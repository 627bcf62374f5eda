"""Host side of the pipelined self-play (no GPU): the split is checked before anything is
allocated, and bench.py pipelines every workload by default (measured gains); configs[2] keeps
its batch of 1,024 leaves per evaluation (1,024 games per pipeline)."""
import sys

import pytest

import bench


def test_pipelines_must_divide_the_games():
    from engine import PipelinedSelfPlay

    with pytest.raises(ValueError):
        PipelinedSelfPlay(None, {"num_simulations": 8}, 1023, pipelines=2)
    with pytest.raises(ValueError):
        PipelinedSelfPlay(None, {"num_simulations": 8}, 64, pipelines=0)


@pytest.mark.parametrize("argv,want", [([], 2), (["--workload", "c4"], 2),
                                       (["--workload", "c2"], 2), (["--workload", "c5"], 2),
                                       (["--pipelines", "2"], 2),
                                       (["--workload", "c5", "--games", "1023"], 1)])
def test_bench_pipeline_defaults(monkeypatch, argv, want):
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    assert bench.parse().pipelines == want


@pytest.mark.parametrize("argv,games,pipes", [([], 2048, 2), (["--pipelines", "1"], 1024, 1),
                                              (["--pipelines", "4"], 4096, 4),
                                              (["--games", "1024"], 1024, 2)])
def test_bench_configs2_leaf_batch(monkeypatch, argv, games, pipes):
    """configs[2] ("batched leaf eval = 1024"): by default 1,024 games per pipeline."""
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    a = bench.parse()
    assert (a.games, a.pipelines) == (games, pipes)


def test_bench_window_protocol_defaults(monkeypatch):
    """The driver's command (--steps 20 --warmup 5) gets the sustained block and the settle
    windows between the warmup and the timed window."""
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "20", "--warmup", "5"])
    a = bench.parse()
    assert (a.steps, a.warmup, a.settle, a.sustained_steps) == (20, 5, 3, 2000)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--settle", "0", "--sustained-steps", "0"])
    a = bench.parse()
    assert (a.settle, a.sustained_steps) == (0, 0)
