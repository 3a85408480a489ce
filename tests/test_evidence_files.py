"""The committed evidence is self-consistent: the bench line carries the contract's
objects, the PMC traffic file matches it, and DESIGN.md's kernel table can be regenerated
from profiles/ (tools/design_table.py) without a missing row."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")
RD = os.environ.get("INA_EVIDENCE_ROUND", "r02")


def test_bench_line_and_traffic_agree():
    b = json.load(open(os.path.join(P, RD, "bench.json")))
    t = json.load(open(os.path.join(P, "traffic_sum_reduce_c3.json")))
    rf = b["roofline"]
    assert rf["bound"] == "hbm" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert t["algorithmic_bytes"] == rf["algorithmic_bytes_per_launch"] == 9 * 26_214_400 * 4
    assert 0.99 < t["traffic_over_algorithmic"] < 1.05
    assert b["cpu_baseline"]["matches_gpu"] is True and b["parity_spot_check"] is True


def test_design_table_regenerates_from_profiles():
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "design_table.py"), "check", "--check"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("\n| ") >= 20
