"""Host-side drop-in surfaces that need no GPU: packet headers (NGAPacket.py /
header_config.py), the communicator.py slice fan-out, the PS TCP framing and
communication_parallel (launch.py:111-130), and refusal of CPU-resident models."""
import socket
import threading

import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests._golden import load_capture


def test_header_build_parse_matches_oracle_and_reference():
    from ina_amd import packet
    q, pkts = load_capture("nga_send_n70.bin")
    f = packet.parse_header(pkts[0])
    assert (f["bitmap"], f["count"], f["index"], f["switch_id"], f["frag_id"]) == (6, 3, 1, 2, 1)
    hdr = packet.build_header(6, 3, 0, 1, 2, 1)
    assert hdr == pkts[0][:15]
    o = orc.pack_nga(q, 32, 6, 3, 2, 1)
    assert o[0][:15].tobytes() == hdr
    assert packet.HEADER_BYTE == 35 and packet.packet_bytes(32) == 143


def test_end_marker_matches_reference():
    from ina_amd import packet
    _, pkts = load_capture("nga_send_end_marker_n40.bin")
    assert packet.end_marker(2, 2, 1) == pkts[-1]


def test_ack_sets_flag_and_keeps_slot():
    from ina_amd import packet
    h = packet.build_header(1, 8, packet.FLAG_OVERFLOW, 77, 1, 12345)
    a = packet.parse_header(packet.ack_for(h))
    assert a["is_ack"] == 1 and a["index"] == 77 and a["frag_id"] == 12345 and a["overflow"] == 0


def test_communicator_slices_follow_reference_split():
    from ina_amd import communicator as cm
    data = np.arange(1000, dtype=np.uint32)
    sl = list(cm._slices(3, data))
    # 7 packets: 2, 2, 3 (remainder to the last), tensor_index = value offset
    assert [n for _, n, _ in sl] == [2, 2, 3]
    assert [off for _, _, off in sl] == [0, 256, 512]
    assert cm.ip2int("172.16.210.33") == (172 << 24) | (16 << 16) | (210 << 8) | 33
    assert cm.PARA_LEN == 25557032 and cm.AGGREGATOR_SIZE == -(-cm.PARA_LEN // 128)


def test_tcp_framing_round_trip():
    from ina_amd import ps
    a, b = socket.socketpair()
    try:
        t = torch.arange(10, dtype=torch.float32)
        th = threading.Thread(target=ps.send_timestamp_data, args=(a, 12.5, t))
        th.start()
        ts, got = ps.get_timestamp_data(b)
        th.join()
        assert ts == 12.5 and torch.equal(got, t)
    finally:
        a.close()
        b.close()


def test_communication_parallel_runs_every_worker():
    from ina_amd import ps
    calls = []

    class W:
        def __init__(self, i):
            self.i = i

        def get_trained_model(self):
            calls.append(("pull", self.i))

        def send_data(self, d):
            calls.append(("push", self.i, d))

        def launch(self, para, part):
            calls.append(("init", self.i, para, part))

    ws = [W(i) for i in range(4)]
    ps.communication_parallel(ws, "pull")
    ps.communication_parallel(ws, "push", updated_data=7)
    ps.communication_parallel(ws, "init", para=1, partition=2)
    assert sorted(c for c in calls if c[0] == "pull") == [("pull", i) for i in range(4)]
    assert len([c for c in calls if c[0] == "push" and c[2] == 7]) == 4
    assert len([c for c in calls if c[0] == "init"]) == 4


def test_aggregate_requires_device_model():
    from ina_amd import ps
    m = torch.nn.Linear(4, 4)

    class Wk:
        updated_paras = torch.zeros(20)
    with pytest.raises(ValueError, match="GPU"):
        ps.aggregate(m, [Wk()], 1)


def test_data_manager_byte_range_checks():
    from ina_amd.data_manager import _signed_byte
    assert _signed_byte("degree", -1) == 0xFF and _signed_byte("degree", 127) == 127
    with pytest.raises(ValueError):
        _signed_byte("degree", 128)


def test_spawn_pools_start_warm():
    """multi_process_send / multi_process_send_futures_P start their spawned workers and
    run the warm-up initializer (HIP start-up + a barrier over every worker) before the
    clock starts; the pools come up and drain here without a GPU."""
    from concurrent.futures import ProcessPoolExecutor

    from ina_amd import communicator as cm
    with cm._SPAWN.Pool(3, **cm._warm_pool_args(3)) as pool:
        assert pool.map(cm._noop, range(3), chunksize=1) == [None] * 3
    with ProcessPoolExecutor(max_workers=2, mp_context=cm._SPAWN, **cm._warm_pool_args(2)) as ex:
        assert list(ex.map(cm._noop, range(2))) == [None, None]
