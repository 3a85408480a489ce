"""Edge cases on the device path: empty inputs, one value, W at the ABI maximum (64),
ragged tails at every residue, packet ingest with a skipped IPv4 header, and UDP
loopback egress (the wire path the reference's raw sockets take)."""
import socket

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def ops():
    from ina_amd import ops as o
    return o


def test_empty_inputs_are_no_ops():
    o = ops()
    e32 = torch.empty(0, dtype=torch.int32, device="cuda")
    ef = torch.empty(0, dtype=torch.float32, device="cuda")
    assert o.sum_reduce([e32, e32]).numel() == 0
    assert o.quantize(ef, 16).numel() == 0
    assert o.dequantize(e32, 16).numel() == 0
    assert o.quantize_reduce([ef, ef], 16).numel() == 0
    q, f = o.quantize_i16(ef, 10, 32)
    assert q.numel() == 0 and f.numel() == 0
    assert o.pack_nga(e32, 32, 1, 2, 1, 1).shape[0] == 0
    cs = o.checksum(e32)
    torch.cuda.synchronize()
    assert int(cs.item()) == 0


def test_max_workers_and_one_value():
    rng = np.random.default_rng(64)
    bufs = [rng.integers(-2**31, 2**31, 1, dtype=np.int64).astype(np.int32) for _ in range(64)]
    got = ops().sum_reduce([torch.from_numpy(b).cuda() for b in bufs]).cpu().numpy()
    assert np.array_equal(got, orc.sum_reduce_i32(bufs))
    with pytest.raises(ValueError):
        ops().sum_reduce([torch.zeros(4, dtype=torch.int32, device="cuda")] * 65)


@pytest.mark.parametrize("n", list(range(1, 18)) + [255, 256, 257, 1023, 1025])
def test_ragged_tails_every_kernel(n):
    o = ops()
    rng = np.random.default_rng(n)
    ints = [rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32) for _ in range(3)]
    flts = [(rng.standard_normal(n) * 100).astype(np.float32) for _ in range(3)]
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    assert np.array_equal(o.sum_reduce([d(a) for a in ints]).cpu().numpy(), orc.sum_reduce_i32(ints))
    assert np.array_equal(o.quantize_reduce([d(a) for a in flts], 8).cpu().numpy(),
                          orc.quantize_reduce_i32(flts, 8))
    q, f = o.quantize_reduce_i16([d(a) for a in flts], 8, 8)
    wq, wf = orc.quantize_reduce_i16_sat(flts, 8, 8)
    assert np.array_equal(q.cpu().numpy(), wq) and np.array_equal(f.cpu().numpy(), wf)
    pk = o.pack_nga(d(ints[0]), 32, 7, 3, 1, 9)
    assert np.array_equal(pk.cpu().numpy(), orc.pack_nga(ints[0], 32, 7, 3, 1, 9, stride=144))
    assert o.checksum(d(ints[0])).cpu().numpy().view(np.uint32)[0] == orc.checksum_i32(ints[0])


def test_ring_recv_skips_ip_header():
    """get_data_from_nic reads IPv4 header + NGA packet (utils.py:61-64); skip=20 drops
    the IP header so packets land at offset 0 of each ring row."""
    from ina_amd.nic import PacketRing
    V = 32
    vals = np.arange(3 * V, dtype=np.int32) - 40
    pk = orc.pack_nga(vals, V, 5, 2, 1, 1)
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    try:
        for row in pk:
            a.send(bytes(range(20)) + row.tobytes())
        ring = PacketRing(8, V)
        n = ring.recv(b, max_pkts=3, timeout_ms=2000, skip=20)
        assert n == 3 and list(ring.lens[:3]) == [143] * 3
        got = ring.to_device(n)
        f, v = ops().unpack_nga(got, V)
        assert np.array_equal(v.cpu().numpy(), vals)
        assert ring.recv(b, max_pkts=1, timeout_ms=50) == 0        # deadline, nothing queued
    finally:
        a.close()
        b.close()


def test_udp_loopback_egress_and_ingest():
    from ina_amd.nic import PacketRing, send_device_packets
    V = 256
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 22)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.connect(rx.getsockname())
    try:
        vals = torch.arange(40 * V, dtype=torch.int32, device="cuda") * 7919
        pk = ops().pack_nga(vals, V, 1, 2, 1, 100)
        assert send_device_packets(tx, pk, 15 + 4 * V) == 40
        ring = PacketRing(64, V)
        got = 0
        while got < 40:
            r = ring.recv(rx, max_pkts=40 - got, timeout_ms=2000, offset=got)
            assert r > 0
            got += r
        assert torch.equal(ring.to_device(got)[:, :15 + 4 * V], pk[:, :15 + 4 * V])
    finally:
        tx.close()
        rx.close()
