"""Host side of the pipelined self-play (no GPU): the split is checked before anything is
allocated, and bench.py pipelines configs[1] and configs[4] by default (measured gains), not
configs[2] / configs[3]."""
import sys

import pytest

import bench


def test_pipelines_must_divide_the_games():
    from engine import PipelinedSelfPlay

    with pytest.raises(ValueError):
        PipelinedSelfPlay(None, {"num_simulations": 8}, 1023, pipelines=2)
    with pytest.raises(ValueError):
        PipelinedSelfPlay(None, {"num_simulations": 8}, 64, pipelines=0)


@pytest.mark.parametrize("argv,want", [([], 1), (["--workload", "c4"], 1),
                                       (["--workload", "c2"], 2), (["--workload", "c5"], 2),
                                       (["--pipelines", "2"], 2),
                                       (["--workload", "c5", "--games", "1023"], 1)])
def test_bench_pipeline_defaults(monkeypatch, argv, want):
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    assert bench.parse().pipelines == want
