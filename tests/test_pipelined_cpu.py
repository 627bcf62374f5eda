"""Host side of the pipelined self-play (no GPU): the split is checked before anything is
allocated, and bench.py pipelines configs[2] by default, nothing else."""
import sys

import pytest

import bench


def test_pipelines_must_divide_the_games():
    from engine import PipelinedSelfPlay

    with pytest.raises(ValueError):
        PipelinedSelfPlay(None, {"num_simulations": 8}, 1023, pipelines=2)
    with pytest.raises(ValueError):
        PipelinedSelfPlay(None, {"num_simulations": 8}, 64, pipelines=0)


@pytest.mark.parametrize("argv,want", [([], 2), (["--workload", "c4"], 1),
                                       (["--workload", "c2"], 1), (["--pipelines", "1"], 1),
                                       (["--games", "1023"], 1)])
def test_bench_pipeline_defaults(monkeypatch, argv, want):
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    assert bench.parse().pipelines == want
