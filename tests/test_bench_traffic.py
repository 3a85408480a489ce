"""bench.py's roofline.traffic provenance (CPU): the committed PMC file is quoted only for the
kernel symbol and size it measured, and the line says which file and session it came from."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def _write(tmp_path, **kw):
    t = {"kernel": "void ina::k_sum_reduce_i32_vec<8, 4, true>(ina::PtrPack<int>, int*, unsigned long, "
                   "unsigned long)", "session": "r04x", "workers": 8, "values": 26_214_400,
         "hbm_bytes_per_launch": 943_779_840}
    t.update(kw)
    p = tmp_path / "traffic.json"
    p.write_text(json.dumps(t))
    return str(p)


def test_traffic_quoted_for_its_kernel(tmp_path):
    b, src = bench.load_traffic(_write(tmp_path), 8, 26_214_400)
    assert b == 943_779_840 and src["matches_kernel_and_size"] is True and src["session"] == "r04x"


def test_traffic_nulled_for_another_kernel_or_size(tmp_path):
    b, src = bench.load_traffic(_write(tmp_path, kernel="void ina::k_sum_reduce_i32_vec<8, 2, true>(x)"),
                                8, 26_214_400)
    assert b is None and src["matches_kernel_and_size"] is False
    b, src = bench.load_traffic(_write(tmp_path), 8, 1000)
    assert b is None and src["matches_kernel_and_size"] is False
    b, src = bench.load_traffic(str(tmp_path / "missing.json"), 8, 26_214_400)
    assert b is None and "error" in src


def test_committed_traffic_file_names_the_headline_kernel():
    t = json.load(open(os.path.join(REPO, "profiles", "traffic_sum_reduce_c3.json")))
    assert bench._kernel_symbol(t["kernel"]) == bench._kernel_symbol(bench.HEADLINE_KERNEL)
