"""The CPU oracle pinned against the reference's own outputs (tests/golden/).

C-128 bytes come from the reference's communicator.cc (compiled here, sendto
captured); NGA-32 datagrams from DataManager._send_data; PS combine vectors
from launch.py / launch_async.py aggregate().  See tests/golden/gen_golden.py.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from tests._golden import load_capture, manifest, ps_cases

C128 = manifest("c128_cases.json")
NGA = manifest("nga_cases.json")


@pytest.mark.parametrize("case", C128, ids=[c["name"] for c in C128])
def test_c128_oracle_matches_reference_bytes(case):
    data, pkts = load_capture(case["file"])
    assert all(len(p) == orc.C128_BYTES for p in pkts)
    if case["kind"] == "wrapper":
        got = orc.pack_c128(data, case["packet_num"], case["worker_id"],
                            case["aggregator_index"], case["tensor_index"])
        assert got.tobytes() == b"".join(pkts)
    elif case["kind"] == "single":
        # communicator.py:41-42: int(len/128) packets, tail values dropped, ids 0
        npk = len(data) // orc.C128_V
        assert len(pkts) == npk
        got = orc.pack_c128(data, npk, 0, 0, 0)
        assert got.tobytes() == b"".join(pkts)
    else:
        # communicator.py:133-157: floor(pkts/P) per thread, remainder to the last,
        # tensor_index = value offset of the slice; thread order is racy -> compare sets
        P = case["threads"]
        total = len(data) // orc.C128_V
        per, rem = divmod(total, P)
        want, off = [], 0
        for t in range(P):
            cnt = per + (rem if t == P - 1 else 0)
            g = orc.pack_c128(data[off:], cnt, 0, 0, off)
            want += [g[i * 524:(i + 1) * 524].tobytes() for i in range(cnt)]
            off += per * orc.C128_V
        assert sorted(want) == sorted(pkts)


def test_c128_worker0_shift_is_x86_masked():
    assert orc.c128_bitmap(0) == 0x80000000
    assert orc.c128_bitmap(1) == 1
    assert orc.c128_bitmap(3) == 4


@pytest.mark.parametrize("case", NGA, ids=[c["name"] for c in NGA])
def test_nga_oracle_matches_reference_datagrams(case):
    q, pkts = load_capture(case["file"])
    seq0 = {"send_data": 1, "fast_send_data": 0, "_send_data_end": 5}[case["entry"]]
    data_pkts = [p for p in pkts if len(p) == orc.nga_packet_bytes(32)]
    got = orc.pack_nga(q, 32, bitmap=case["worker_id"], count=case["degree"] & 0xFF,
                       switch_id=case["switch_id"] & 0xFF, seq0=seq0)
    assert len(got) == len(data_pkts) == -(-case["n"] // 32)
    for g, p in zip(got, data_pkts):
        assert g.tobytes() == p
    # unpack round trip (PS side, headers.p4 layout)
    f, vals = orc.unpack_nga(got.reshape(-1), 32)
    assert np.array_equal(vals[:q.size], q) and not vals[q.size:].any()
    assert (f["frag_id"] == seq0 + np.arange(len(got))).all()
    assert (f["index"] == (seq0 + np.arange(len(got))) % 16384).all()
    end = [p for p in pkts if len(p) == orc.NGA_HDR]
    if case["entry"] == "_send_data_end":
        # end marker: header only, index 0, frag 0 (DataManager.py:155-164)
        assert len(end) == 1
        want = orc.pack_nga(np.zeros(0, np.int32), 32, case["worker_id"], case["degree"],
                            case["switch_id"], 0)
        hdr = bytearray(15)
        hdr[0:4] = case["worker_id"].to_bytes(4, "big")
        hdr[4] = case["degree"] & 0xFF
        hdr[10] = case["switch_id"]
        assert end[0] == bytes(hdr) and want.size == 0
    else:
        assert not end   # send_data never sends it (positional-arg bug, DataManager.py:106)


def test_ps_combine_oracle_matches_reference_aggregate():
    cases = ps_cases()
    assert len(cases) >= 5
    for name, c in cases.items():
        W, K = int(c["W"]), int(c["K"])
        paras = list(c["paras"])
        if K > 0:
            paras, weight = paras[:K], 1.0 / K
        else:
            weight = 1.0 / (W + 1)
        got = orc.ps_combine_f32(c["local"], paras, weight * float(c["step"]))
        assert np.array_equal(got.view(np.uint32), c["out"].view(np.uint32)), name
