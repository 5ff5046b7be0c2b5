"""bench.py's driver line: the last stdout line must be one JSON object under 8 KB
carrying the contract keys, `roofline` (numeric traffic) and `cpu_baseline`, built here from a
recorded full result of round 5 (profiles/r05/s5/bench.json, whose single 20-KB line the driver
could not parse)."""
import io
import json
import os
import contextlib

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORDED = os.path.join(REPO, "profiles", "r05", "s5", "bench.json")

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "build", "roofline", "cpu_baseline")


def _recorded():
    if not os.path.exists(RECORDED):
        pytest.skip("recorded round-5 result not in this tree")
    with open(RECORDED) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_compact_line_from_recorded_result(tmp_path):
    full = _recorded()
    assert len(json.dumps(full)) > bench.FINAL_LINE_MAX  # the case that failed in round 5
    details = str(tmp_path / "details.json")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.emit(full, details)
    lines = buf.getvalue().splitlines()
    assert len(lines) == 1
    line = lines[-1]
    assert len(line.encode()) <= bench.FINAL_LINE_MAX
    d = json.loads(line)
    for k in CONTRACT:
        assert k in d, k
    assert d["value"] == full["value"] and d["ms_per_step"] == full["ms_per_step"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert isinstance(r["traffic"], (int, float))
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-3)
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb
    assert cb["legs"]["dcn_4096"]["gpu_over_cpu"] >= 10  # the north star's DCN-4096 leg stays
    assert d["models"]["dcn"]["sps"] == full["models"]["dcn"]["samples_per_s"]
    assert "gather_frac" in d["models"]["deepfm"]
    # the side file holds every leg in full
    with open(details) as f:
        assert json.load(f) == full


def test_compact_line_falls_back_when_extras_grow(tmp_path):
    full = _recorded()
    full["models"] = {f"m{i}": {"samples_per_s": 1.0, "ms_per_step": 1.0, "roofline": {"frac": 0.5}}
                      for i in range(400)}
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.emit(full, str(tmp_path / "d.json"))
    line = buf.getvalue().splitlines()[-1]
    assert len(line.encode()) <= bench.FINAL_LINE_MAX
    d = json.loads(line)
    assert "models" not in d and d["roofline"]["frac"] == full["roofline"]["frac"]


def test_counter_staleness_tags():
    bench._LIB_SRC = "abc"
    try:
        assert bench.counter_staleness({"src": "abc"}) == "current"
        assert bench.counter_staleness({"src": "def"}).startswith("stale")
        assert bench.counter_staleness({}) == "unknown"
    finally:
        bench._LIB_SRC = None
