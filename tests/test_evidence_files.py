"""The committed evidence is self-consistent: the bench line carries the contract's
objects and the PMC traffic file matches it."""
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")
RD = os.environ.get("INA_EVIDENCE_ROUND", "r03")


def test_bench_line_and_traffic_agree():
    b = json.load(open(os.path.join(P, RD, "bench.json")))
    t = json.load(open(os.path.join(P, "traffic_sum_reduce_c3.json")))
    rf = b["roofline"]
    assert rf["bound"] == "hbm" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert t["algorithmic_bytes"] == rf["algorithmic_bytes_per_launch"] == 9 * 26_214_400 * 4
    assert 0.99 < t["traffic_over_algorithmic"] < 1.05
    assert b["cpu_baseline"]["matches_gpu"] is True and b["parity_spot_check"] is True


def test_bench_line_carries_every_leg():
    """The round's committed line has the single-GPU configs and the PCIe rate with their
    rooflines and parity checks, and config 5's xGMI roofline."""
    b = json.load(open(os.path.join(P, RD, "bench.json")))
    for leg in ("c2_fused", "c4_int16", "e2e_pcie"):
        assert b[leg]["parity_spot_check"] is True and 0 < b[leg]["roofline"]["frac"] < 1, leg
    assert b["sharded_c5"]["roofline"]["bound"] == "xgmi"
    assert b["cpu_baseline"]["cores"] <= b["cpu_baseline"]["affinity_cores"]
