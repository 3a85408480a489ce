"""bench.py's multi-rank launcher on CPU: `bench.py --gpus N` with no launcher around it
starts N ranks itself (torch.distributed.run on 127.0.0.1), every rank asserts the group
size, and rank 0 prints one line with n_gpus == N.  --check-launch does no GPU work, so
this runs here with gloo; the GPU rehearsal is tests/test_gpu_bench_contract.py."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import REPO


def _bench(*args, env=None, timeout=240):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO,
                          capture_output=True, text=True, timeout=timeout, env=e)


@pytest.mark.parametrize("n", [1, 2, 3, 8])         # 8: the driver's largest scaling run
def test_bench_gpus_n_spawns_n_ranks(n):
    r = _bench("--gpus", str(n), "--check-launch")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["rccl_world"] == n and d["ranks"] == list(range(n))
    assert d["backend"] == ("gloo" if n > 1 else "none")


def test_bench_refuses_a_group_of_the_wrong_size():
    r = _bench("--gpus", "2", "--check-launch", env={"WORLD_SIZE": "1"})
    assert r.returncode != 0
    assert "--gpus 2 but the launcher started 1 ranks" in r.stderr


def test_cgroup_quota_reader_is_safe():
    sys.path.insert(0, REPO)
    import bench
    q = bench.cgroup_cpus()
    assert q is None or q > 0


def test_run_leg_reports_a_failing_leg_and_keeps_the_line():
    sys.path.insert(0, REPO)
    import bench
    line = {"value": 1.0}
    ok = bench.run_leg(line, "a", lambda: {"frac": 0.8})
    assert ok == {"frac": 0.8} and line["a"] is ok

    def boom():
        raise RuntimeError("NCCL error: unhandled system error")
    bad = bench.run_leg(line, "b", boom)
    assert bad["error"].startswith("RuntimeError: NCCL error")
    bench.run_leg(bad, "sub", lambda: {"x": 1})        # sub-legs attach to an errored parent
    assert line["b"]["sub"] == {"x": 1} and line["value"] == 1.0
    json.dumps(line)


def test_legs_summary_is_compact_and_last():
    sys.path.insert(0, REPO)
    import bench
    line = {"value": 5.0, "roofline": {"avg_launch_us": 146.4, "frac": 0.81}, "parity_spot_check": True,
            "c2_fused": {"roofline": {"avg_launch_us": 79.8, "frac": 0.8}, "parity_spot_check": True},
            "e2e_pcie": {"ms_per_step": 15.05, "roofline": {"frac": 0.97}, "parity_spot_check": True},
            "switch_c3_v32": {"workload": "w", "round_robin_split": {"us": 243.5, "frac": 0.6,
                                                                     "parity_spot_check": True,
                                                                     "batch_path": "in_order"},
                              "parity_sample": "s"},
            "packet_path_v32": {"error": "RuntimeError: out of memory"}}
    line["legs"] = bench.legs_summary(line)
    legs = json.loads(json.dumps(line))["legs"]
    assert list(json.loads(json.dumps(line)))[-1] == "legs"
    assert legs["headline"] == {"us": 146.4, "frac": 0.81, "parity": True}
    assert legs["c2_fused"]["us"] == 79.8 and legs["e2e_pcie"]["us"] == 15050.0
    assert legs["switch_c3_v32.round_robin_split"] == {"us": 243.5, "frac": 0.6, "parity": True,
                                                       "path": "in_order"}
    assert legs["packet_path_v32"]["error"].startswith("RuntimeError")


def test_leg_tuning_is_restored_when_a_leg_raises(monkeypatch):
    sys.path.insert(0, REPO)
    import bench
    from ina_amd import ops
    seen = []
    monkeypatch.setattr(ops, "set_tuning", lambda **kw: seen.append(kw))
    with pytest.raises(RuntimeError):
        with bench._tuning(switch_runs=False):
            raise RuntimeError("leg failed")
    assert seen == [{"switch_runs": False}, {"switch_runs": True}]
