"""RCCL channel / protocol knobs (CPU): parsing, env plumbing, and the sweep's winner selection."""
import os

import pytest

from ddpx.parallel.comm import parse_channels, set_rccl_protocol


def test_parse_channels():
    assert parse_channels(None) is None and parse_channels("") is None and parse_channels(0) is None
    assert parse_channels(8) == (8, 8)
    assert parse_channels("12") == (12, 12)
    assert parse_channels("4:16") == (4, 16)
    assert parse_channels((0, 8)) == (0, 8)
    with pytest.raises(ValueError):
        parse_channels("16:4")
    with pytest.raises(ValueError):
        parse_channels(-1)


def test_set_rccl_protocol(monkeypatch):
    monkeypatch.delenv("NCCL_PROTO", raising=False)
    set_rccl_protocol(None)
    assert "NCCL_PROTO" not in os.environ
    set_rccl_protocol("LL128")
    assert os.environ["NCCL_PROTO"] == "LL128"


def test_bench_flags_reach_the_parser():
    import bench
    a = bench.parse(["--rccl_channels", "4:16", "--rccl_proto", "Simple"])
    assert a.rccl_channels == "4:16" and a.rccl_proto == "Simple"
    from ddpx.train.app import build_parser
    b = build_parser("t").parse_args(["1", "1", "--rccl_channels", "8"])
    assert b.rccl_channels == "8" and b.rccl_proto is None


def test_sweep_picks_fastest_per_op_and_size():
    import importlib.util
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("rccl_sweep", os.path.join(here, "benchmarks", "rccl_sweep.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    rows = [{"op": "all_reduce", "bytes": 64, "us": 9.0, "proto": "default", "channels": "0"},
            {"op": "all_reduce", "bytes": 64, "us": 7.0, "proto": "LL", "channels": "8"},
            {"op": "all_reduce", "bytes": 128, "us": 5.0, "proto": "Simple", "channels": "16"},
            {"op": "all_gather", "bytes": 64, "us": 3.0, "proto": "default", "channels": "0"}]
    best = m.best_rows(rows)
    assert best[("all_reduce", 64)]["proto"] == "LL"
    assert best[("all_reduce", 128)]["channels"] == "16"
    assert best[("all_gather", 64)]["us"] == 3.0
