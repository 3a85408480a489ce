"""bench.py's output contract (one JSON line with the driver's keys, roofline and
cpu_baseline objects) on a short run; the bench runs as a child process."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_line_contract():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--cpu-sample", str(1 << 16)],
                       cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["higher_is_better"] is True and d["value"] > 0 and d["parity_spot_check"] is True
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["algorithmic_bytes_per_launch"] == 9 * 26_214_400 * 4
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0
    assert cb["matches_gpu"] is True
    assert "workload" in d["config"]


@pytest.mark.gpu
def test_bench_sharded_mode_line():
    """Config-5 mode on one GPU (the collectives are identities): a JSON line whose
    aggregate passes its own parity spot check."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--mode", "sharded", "--steps", "2",
                        "--warmup", "1", "--values", str(1 << 22)],
                       cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["parity_spot_check"] is True
    assert d["config"]["values_per_worker"] == 1 << 22
