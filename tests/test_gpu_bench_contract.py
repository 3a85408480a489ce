"""bench.py's output contract (one JSON line with the driver's keys, roofline,
cpu_baseline, sharded_c5 and switch_c3 objects) on short runs; the bench runs as a child process.
The two-rank rehearsal puts both ranks on the one GPU of the test box with a gloo group
(bench.py --gpus 2 launching its own ranks, INA_BENCH_BACKEND=gloo): the launcher, the
group-size assertion, the per-rank slot ranges and the config-5 path through
ShardedAggregator at world size 2 -- the RCCL run itself needs the 8-GPU node."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _run(*args, env=None, timeout=300):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO,
                          capture_output=True, text=True, timeout=timeout, env=e)


@pytest.mark.gpu
def test_bench_json_line_contract():
    d = _line(_run("--steps", "3", "--warmup", "1", "--cpu-sample", str(1 << 16),
                   "--c5-values", str(1 << 22), "--c5-steps", "2"))
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline",
                "rccl_world", "sharded_c5"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["rccl_world"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["scaling"] == "weak"
    assert d["higher_is_better"] is True and d["value"] > 0 and d["parity_spot_check"] is True
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["algorithmic_bytes_per_launch"] == 9 * 26_214_400 * 4
    src = rf["traffic_source"]                  # where `traffic` came from, or why it is null
    assert src["file"].endswith(".json")
    if rf["traffic"] is not None:
        assert src["matches_kernel_and_size"] is True and src["session"]
        assert "k_sum_reduce_i32_vec<8, 4, true>" in src["kernel"] or "k_sum_reduce_i32_vec<8,4,true>" in src["kernel"]
    assert "every 997th over the whole bucket" in d["parity_sample"]
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["value"] > 0
    aff = len(os.sched_getaffinity(0))
    assert cb["affinity_cores"] == aff and 1 <= cb["cores"] <= aff      # cores = CPUs granted
    assert str(cb["threads"]) in cb["value_by_threads"]                 # threads = best count
    assert cb["value"] == max(cb["value_by_threads"].values()) == cb["value_by_threads"][str(cb["threads"])]
    if cb["cgroup_cpu_quota"]:
        assert cb["cores"] == min(aff, max(1, int(cb["cgroup_cpu_quota"])))
    assert cb["matches_gpu"] is True and cb["value_1core"] > 0
    assert "workload" in d["config"] and "independent replicas" in d["config"]["parallelism"]
    # the single-GPU BASELINE configs 2 and 4 and the PCIe-inclusive rate, each with a
    # roofline and a parity spot check
    c2, c4, e2e = d["c2_fused"], d["c4_int16"], d["e2e_pcie"]
    for leg, kern, algo in ((c2, "k_quant_reduce_i32<4>", 20 * 25_557_032),
                            (c4, "k_quant_reduce_i16<16>", 66 * 25_557_032 + 99_833)):
        rf = leg["roofline"]
        assert leg["parity_spot_check"] is True and rf["bound"] == "hbm" and kern in rf["kernel"]
        assert rf["algorithmic_bytes_per_launch"] == algo and 0 < rf["frac"] < 1
        assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert c4["overflow_slots"] == c4["overflow_slots_injected"] > 0
    assert e2e["parity_spot_check"] is True and e2e["roofline"]["bound"] == "pcie_h2d"
    assert e2e["copy_pipeline"]["parity_spot_check"] is True and e2e["copy_pipeline"]["value"] > 0
    assert 0 < e2e["roofline"]["frac"] and e2e["roofline"]["peak"] > 0
    c5 = d["sharded_c5"]
    assert c5["parity_spot_check"] is True and c5["rccl_world"] == 1 and c5["values_per_rank"] == 1 << 22
    assert c5["layout_b"]["parity_spot_check"] is True and c5["layout_b"]["value"] > 0
    assert "allreduce" not in c5 and "pipelined" not in c5   # one rank: no collective to compare
    for r in (c5["roofline"], c5["layout_b"]["roofline"]):   # one rank: no xGMI bytes, null fields
        assert r["bound"] == "xgmi" and r["peak"] == 7 * 153.0
        assert r["achieved"] is None and r["frac"] is None
        assert all(p["frac"] > 0 for p in r["hbm_phases"].values())   # 16 MiB: may replay from MALL
    sw = d["switch_c3"]                          # the packet-stream switch, measured live
    assert sw["algorithmic_bytes"] == 819_200 * 1040 + 102_400 * (1040 + 1029) + 819_200
    paths = {"worker_major": "runs", "worker_major_split": "runs", "round_robin": "in_order",
             "worker_major_sorted": "sorted", "shuffled": "sorted"}
    for order, path in paths.items():
        assert sw[order]["ok"] is True and sw[order]["slots_completed"] == 102_400
        assert 0 < sw[order]["frac"] < 1 and sw[order]["batch_path"] == path, order
        assert sw[order]["parity_spot_check"] is True, order
    v32 = d["switch_c3_v32"]                     # the P4's own NGA-32 at config-3 size
    assert v32["V"] == 32 and v32["stride"] == 144
    assert v32["algorithmic_bytes"] == 6_553_600 * 144 + 819_200 * (144 + 133) + 6_553_600
    for order, path in (("worker_major", "runs"), ("worker_major_split", "runs"), ("round_robin", "in_order"),
                        ("round_robin_split", "in_order"), ("shuffled", "sorted")):
        assert v32[order]["ok"] is True and v32[order]["slots_completed"] == 819_200, order
        assert v32[order]["parity_spot_check"] is True and v32[order]["batch_path"] == path, order
        assert 0 < v32[order]["frac"] < 1, order
    pp = d["packet_path"]                        # the whole INA step, PS fused, steady state
    assert pp["parity_spot_check"] is True and pp["value"] > 0 and pp["ms_per_step"] > 0
    assert pp["roofline"]["bound"] == "hbm" and 0 < pp["roofline"]["frac"] < 1
    assert abs(pp["roofline"]["frac"] - pp["roofline"]["achieved"] / pp["roofline"]["peak"]) < 1e-3
    for leg in (pp, d["packet_path_packed"]):    # split rows, and packed rows (same datagrams)
        assert leg["parity_spot_check"] is True and leg["value"] > 0 and leg["switch_batch_path"] == "runs"
        ph = leg["phases"]                       # the packs and the switch + PS pass apart
        assert 0 < ph["worker_packs"]["frac"] < 1 and 0 < ph["switch_and_ps"]["frac"] < 1
        assert ph["worker_packs"]["bytes"] + ph["switch_and_ps"]["bytes"] == leg["roofline"]["path_bytes_per_step"]
    assert pp["rows"] == "split" and d["packet_path_packed"]["rows"] == "packed"
    assert not any(isinstance(v, dict) and "error" in v for v in d.values())   # no leg raised


@pytest.mark.gpu
def test_bench_sharded_mode_line():
    """Config-5 mode on one GPU (the collectives are identities), both wires."""
    for wire in ("i32", "i16"):
        d = _line(_run("--mode", "sharded", "--c5-steps", "2", "--c5-values", str(1 << 22),
                       "--wire", wire))
        assert d["n_gpus"] == 1 and d["value"] > 0 and d["parity_spot_check"] is True, wire
        assert d["config"]["values_per_worker"] == 1 << 22
        assert d["layout_b"]["parity_spot_check"] is True, wire


@pytest.mark.gpu
def test_bench_two_rank_rehearsal_on_one_gpu():
    """bench.py --gpus 2 starts two ranks itself; both on cuda:0 with gloo."""
    d = _line(_run("--gpus", "2", "--steps", "3", "--warmup", "1", "--values", str(1 << 22),
                   "--c5-values", str(1 << 22), "--c5-steps", "2",
                   env={"INA_BENCH_BACKEND": "gloo"}, timeout=400))
    assert d["n_gpus"] == 2 and d["rccl_world"] == 2 and d["backend"] == "gloo"
    assert d["parity_spot_check"] is True and "cpu_baseline" not in d
    assert "independent replicas x 2" in d["config"]["parallelism"]
    rf = d["roofline"]                           # the slowest rank's launch: frac = min over ranks
    assert rf["per_rank_frac_min"] == rf["frac"] <= rf["per_rank_frac_max"]
    for leg in ("c2_fused", "c4_int16", "e2e_pcie"):
        assert d[leg]["parity_spot_check"] is True, leg
    c5 = d["sharded_c5"]
    assert c5["rccl_world"] == 2 and c5["parity_spot_check"] is True
    assert c5["xgmi"]["rs_send_bytes_per_rank"] == c5["shard_values"] * 4
    assert c5["layout_b"]["parity_spot_check"] is True
    assert c5["layout_b"]["xgmi"]["ag_recv_bytes_per_rank"] == c5["shard_values"] * 4
    ar = c5["allreduce"]                         # the one-collective variant, same bits
    assert ar["collective"] == "allreduce" and ar["parity_spot_check"] is True
    assert ar["xgmi"]["allreduce_bytes_per_rank"] == 2 * c5["shard_values"] * 4
    a2 = c5["a2a"]                               # all-to-all + device sum, same bits
    assert a2["collective"] == "a2a" and a2["parity_spot_check"] is True
    assert a2["roofline"]["bytes_per_rank"] == c5["roofline"]["bytes_per_rank"]
    pl = c5["pipelined"]                         # chunked, async RCCL work, same bits
    assert pl["chunks"] > 1 and pl["parity_spot_check"] is True
    # every variant carries an xGMI roofline with the per-rank bytes it moved
    assert c5["roofline"]["bytes_per_rank"] == 2 * c5["shard_values"] * 4
    assert c5["layout_b"]["roofline"]["bytes_per_rank"] == c5["shard_values"] * 4
    assert ar["roofline"]["bytes_per_rank"] == 2 * c5["shard_values"] * 4
    assert pl["roofline"]["bytes_per_rank"] == pl["xgmi"]["rs_send_bytes_per_rank"] + pl["xgmi"]["ag_recv_bytes_per_rank"]
    for r in (c5["roofline"], c5["layout_b"]["roofline"], ar["roofline"], pl["roofline"], a2["roofline"]):
        assert r["bound"] == "xgmi" and r["achieved"] > 0 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert set(c5["roofline"]["hbm_phases"]) == {"quantize", "decode"}
    sw = d["switch_c3"]                          # every rank switched its own bucket
    assert sw["ranks"] == 2 and sw["worker_major"]["ok"] is True and sw["round_robin"]["ok"] is True
    assert d["packet_path"]["parity_spot_check"] is True
    assert sw["worker_major"]["aggregate_GBps"] > 0
    d = _line(_run("--gpus", "2", "--mode", "sharded", "--wire", "i16", "--c5-values", "1000003",
                   "--c5-steps", "2", env={"INA_BENCH_BACKEND": "gloo"}, timeout=400))
    assert d["n_gpus"] == 2 and d["parity_spot_check"] is True
    assert d["layout_b"]["parity_spot_check"] is True
    shard = d["config"]["shard_values"]          # the i16 wire gathers int16 sums + slot flags
    assert d["xgmi"]["ag_recv_bytes_per_rank"] == 2 * shard + shard // 256
    assert d["xgmi"]["rs_send_bytes_per_rank"] == 4 * shard
    assert d["allreduce"]["parity_spot_check"] is True and d["pipelined"]["parity_spot_check"] is True
    assert d["a2a"]["parity_spot_check"] is True
