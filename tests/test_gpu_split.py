"""GPU parity of the split NGA rows (include/ina.h: 16-byte header rows + 4V-byte payload
rows, the same datagrams as the packed rows of DataManager._send_data, DataManager.py:111-165
/ headers.p4:27-80): every split entry point against the packed one on the same inputs --
pack, fused worker pack, unpack, the switch (sort, run table, in-order and small-batch
paths, wide and narrow V) and the fused PS step -- and the wire bytes over a socket pair.
Packed rows are pinned to the reference and the oracle elsewhere (test_gpu_parity.py), so
equality here carries that parity over."""
import socket

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ina_amd import ops  # noqa: F401


def ops():
    from ina_amd import ops as o
    return o


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def to_split(packed: np.ndarray, V: int):
    """Packed rows -> (header rows [n, 16] with a zero 16th byte, payload rows [n, 4V])."""
    hdr = np.zeros((len(packed), 16), np.uint8)
    hdr[:, :15] = packed[:, :15]
    return hdr, np.ascontiguousarray(packed[:, 15:15 + 4 * V])


def from_split(hdr: np.ndarray, pay: np.ndarray, stride: int):
    out = np.zeros((len(hdr), stride), np.uint8)
    out[:, :15] = hdr[:, :15]
    out[:, 15:15 + pay.shape[1]] = pay
    return out


@pytest.mark.parametrize("V", [4, 12, 32, 64, 256])
@pytest.mark.parametrize("tail", [0, 3])
def test_pack_split_equals_packed(V, tail):
    o = ops()
    rng = np.random.default_rng(V + tail)
    n = 137 * V - tail
    vals = torch.from_numpy(rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)).to(DEV)
    npk = -(-n // V)
    ovf = torch.from_numpy((rng.random(npk) < 0.2).astype(np.uint8)).to(DEV)
    pk, d0 = o.pack_nga(vals, V, 7, 3, 2, 4_000_000_000, flags=0x10, num_slots=1000, overflow=ovf, desc=True)
    hdr, pay, d1 = o.pack_nga_split(vals, V, 7, 3, 2, 4_000_000_000, flags=0x10, num_slots=1000, overflow=ovf,
                                    desc=True)
    h, p = to_split(host(pk), V)
    assert np.array_equal(host(hdr), h) and np.array_equal(host(pay), p)
    assert torch.equal(d0, d1)
    f0, v0 = o.unpack_nga(pk, V)
    f1, v1 = o.unpack_nga_split(hdr, pay, V)
    assert torch.equal(v0, v1)
    for key in f0:
        assert torch.equal(f0[key], f1[key]), key


@pytest.mark.parametrize("V,W", [(256, 8), (256, 9), (32, 8), (64, 3), (4, 1)])
@pytest.mark.parametrize("with_base", [False, True])
def test_quantize_pack_multi_split_equals_packed(V, W, with_base):
    o = ops()
    rng = np.random.default_rng(V * W + with_base)
    n = 301 * V - 5
    xs = [torch.from_numpy((rng.standard_normal(n) * 1e-2).astype(np.float32)).to(DEV) for _ in range(W)]
    base = torch.from_numpy((rng.standard_normal(n) * 1e-2).astype(np.float32)).to(DEV) if with_base else None
    outs, ds0 = o.quantize_pack_nga_multi(xs, 16, V, list(range(1, W + 1)), W, 1, 9, base=base,
                                          num_slots=1 << 13, descs=True)
    hdrs, pays, ds1 = o.quantize_pack_nga_multi_split(xs, 16, V, list(range(1, W + 1)), W, 1, 9, base=base,
                                                      num_slots=1 << 13, descs=True)
    for w in range(W):
        h, p = to_split(host(outs[w]), V)
        assert np.array_equal(host(hdrs[w]), h), w
        assert np.array_equal(host(pays[w]), p), w
        assert torch.equal(ds0[w], ds1[w]), w


def _switch_both(o, V, stream, num_slots, write_dropped, use_desc, batches=2):
    """The same batches through a packed-row switch and a split-row switch."""
    stride = stream[0].shape[1]
    sw0 = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=write_dropped)
    sw1 = o.Switch(V, num_slots=num_slots, switch_id=1, device=DEV, write_dropped=write_dropped)
    for i, b in enumerate(stream):
        d0 = torch.from_numpy(b).to(DEV)
        h, p = to_split(b, V)
        hd, pd = torch.from_numpy(h).to(DEV), torch.from_numpy(p).to(DEV)
        desc = o.nga_descriptors(d0) if use_desc else None
        a0 = sw0.process(d0, desc=desc)
        a1 = sw1.process_split(hd, pd, desc=desc)
        assert np.array_equal(host(a0), host(a1)), i
        assert np.array_equal(from_split(host(hd), host(pd), stride), _wire(host(d0), V, stride)), i
        if len(b) > 768 and num_slots < (1 << 22):
            assert sw0.batch_path(len(b)) == sw1.batch_path(len(b)), i
    for x, y in ((sw0.count, sw1.count), (sw0.frag, sw1.frag), (sw0.regs, sw1.regs)):
        assert torch.equal(x, y)


def _wire(packed, V, stride):
    """Packed rows with everything past the datagram's 15 + 4V bytes zeroed (split rows do
    not hold the packed row's padding)."""
    out = packed.copy()
    out[:, 15 + 4 * V:] = 0
    return out


def _pad_zero(stream, V):
    s = stream.copy()
    s[:, 15 + 4 * V:] = 0
    return s


@pytest.mark.parametrize("write_dropped", [True, False])
@pytest.mark.parametrize("V,num_slots,W,used,order", [
    (256, 1 << 17, 8, 700, "worker"), (256, 1 << 17, 8, 700, "round_robin"), (256, 1 << 17, 8, 700, "shuffled"),
    (32, 1 << 13, 8, 500, "worker"), (32, 1 << 13, 8, 500, "shuffled"), (64, 1 << 10, 4, 300, "shuffled"),
    (4, 16, 16, 60, "shuffled"), (32, 64, 3, 20, "worker"), (256, 1 << 20, 8, 300, "worker"),
    (128, 4096, 2, 40, "shuffled")])
def test_switch_split_equals_packed(V, num_slots, W, used, order, write_dropped):
    """Random streams (collisions, acks, foreign packets, mixed degrees) through both row
    layouts: same actions, registers after every batch, and the same datagram bytes after
    the switch rewrote them (collision flags, running sums).  Covers the run table, the
    in-order and bucket-sort paths, the digit widths of 2^20 pools, narrow (V <= 32) and wide
    run kernels and the one-launch small batches."""
    o = ops()
    rng = np.random.default_rng(V + num_slots + W + used + write_dropped)
    stride = o.nga_stride(V)
    batches = []
    for _ in range(2):
        pk = []
        for s in range(used):
            idx = s + 5
            deg = int(rng.choice([W, W, W, 1, 2]))
            frag = 1000 + s if rng.random() > 0.05 else 7
            for w in range(W):
                f = frag if rng.random() > 0.03 else frag + 1
                flags = orc.FLAG_ACK if rng.random() < 0.05 else 0
                sw = 2 if rng.random() < 0.03 else 1
                vals = rng.integers(-2**31, 2**31, V, dtype=np.int64).astype(np.int32)
                p = orc.pack_nga(vals, V, w + 1, deg, sw, 0, flags=flags, stride=stride)[0].copy()
                p[6:10] = np.frombuffer(idx.to_bytes(4, "big"), np.uint8)
                p[11:15] = np.frombuffer(f.to_bytes(4, "big"), np.uint8)
                pk.append(p)
        pk = np.stack(pk)                               # round-robin: slot-major already
        if order == "worker":
            pk = pk.reshape(used, W, stride).transpose(1, 0, 2).reshape(-1, stride).copy()
        elif order == "shuffled":
            pk = pk[rng.permutation(len(pk))]
        batches.append(_pad_zero(pk, V))
    _switch_both(o, V, batches, num_slots, write_dropped, use_desc=bool(rng.integers(0, 2)))


@pytest.mark.parametrize("V,W,per", [(256, 8, 700), (32, 8, 3000), (64, 4, 200), (256, 3, 30)])
def test_process_apply_split_equals_packed(V, W, per):
    """The packet path's steady state in both layouts: the fused worker packs, the acks of
    step t in front of step t+1's packets, the switch with the PS fused -- same actions, PS
    update (bit for bit), ack rows (their 15 wire bytes) and ack descriptors, registers."""
    o = ops()
    rng = np.random.default_rng(V + W + per)
    n = V * per - 3
    npk = -(-n // V)
    stride = o.nga_stride(V)
    slots = 1 << 13
    xs = [torch.from_numpy((rng.standard_normal(n) * 1e-2).astype(np.float32)).to(DEV) for _ in range(W)]
    glob0 = torch.from_numpy((rng.standard_normal(n) * 1e-2).astype(np.float32)).to(DEV)
    res = {}
    for split in (False, True):
        glob = glob0.clone()
        upd = torch.empty_like(glob)
        acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=DEV)
        desc = torch.zeros((W + 1) * npk, dtype=torch.int64, device=DEV)
        sw = o.Switch(V, num_slots=slots, switch_id=1, device=DEV)
        steps = []
        if split:
            hdr = torch.zeros(((W + 1) * npk, 16), dtype=torch.uint8, device=DEV)
            pay = torch.zeros(((W + 1) * npk, 4 * V), dtype=torch.uint8, device=DEV)
            hw, pw = hdr[npk:].view(W, npk, 16), pay[npk:].view(W, npk, 4 * V)
        else:
            big = torch.zeros(((W + 1) * npk, stride), dtype=torch.uint8, device=DEV)
            rows = big[npk:].view(W, npk, stride)
        for step in range(3):
            wd = list(desc[npk:].view(W, npk).unbind(0))
            if split:
                o.quantize_pack_nga_multi_split(xs, 16, V, list(range(1, W + 1)), W, 1, 1, base=glob,
                                                num_slots=slots, hdrs=list(hw.unbind(0)), pays=list(pw.unbind(0)),
                                                descs=wd)
                if step == 0:
                    o.nga_descriptors(hdr[:npk], out=desc[:npk])
                sw.process_apply_split(hdr, pay, 1, glob, 16, 1.0 / (W + 1), out=upd, ack_hdr=hdr[:npk],
                                       ack_desc=desc[:npk], keep_forwarded=False, actions=acts, desc=desc)
                ack = host(hdr[:npk])[:, :15]
            else:
                o.quantize_pack_nga_multi(xs, 16, V, list(range(1, W + 1)), W, 1, 1, base=glob,
                                          num_slots=slots, outs=list(rows.unbind(0)), descs=wd)
                if step == 0:
                    o.nga_descriptors(big[:npk], out=desc[:npk])
                sw.process_apply(big, 1, glob, 16, 1.0 / (W + 1), out=upd, acks=big[:npk],
                                 ack_desc=desc[:npk], keep_forwarded=False, actions=acts, desc=desc)
                ack = host(big[:npk])[:, :15]
            steps.append((host(acts).copy(), host(upd).view(np.uint32).copy(), ack.copy(), host(desc[:npk]).copy()))
            glob.copy_(upd)
        res[split] = (steps, host(sw.count), host(sw.frag), host(sw.regs))
    (s0, c0, f0, r0), (s1, c1, f1, r1) = res[False], res[True]
    for (a0, u0, k0, d0), (a1, u1, k1, d1) in zip(s0, s1):
        assert np.array_equal(a0, a1)
        assert np.array_equal(u0, u1)
        assert np.array_equal(k0, k1)
        assert np.array_equal(d0, d1)
    assert np.array_equal(c0, c1) and np.array_equal(f0, f1) and np.array_equal(r0, r1)
    assert int((s1[2][0] == orc.ACT_FWD_AGG).sum()) == npk


@pytest.mark.parametrize("V", [32, 256])
def test_split_rows_on_the_wire(V):
    """send_device_split (two iovecs per datagram) puts the packed rows' datagrams on the
    socket byte for byte; SplitPacketRing.recv scatters datagrams back into split rows."""
    from ina_amd import nic
    o = ops()
    rng = np.random.default_rng(V)
    n = 40 * V - 1
    vals = torch.from_numpy(rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)).to(DEV)
    pk = o.pack_nga(vals, V, 3, 2, 1, 77)
    hdr, pay = o.pack_nga_split(vals, V, 3, 2, 1, 77)
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    try:
        for s_ in (a, b):
            s_.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 22)
            s_.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 1 << 22)
        npk = pk.shape[0]
        assert nic.send_device_split(a, hdr, pay, V) == npk
        got = [b.recv(4096) for _ in range(npk)]
        want = host(pk)[:, :15 + 4 * V]
        assert all(g == w.tobytes() for g, w in zip(got, want))
        nic.send_device_packets(a, pk, 15 + 4 * V)
        ring = nic.SplitPacketRing(npk, V, device=DEV)
        assert ring.recv(b, timeout_ms=2000) == npk
        h, p = ring.to_device(npk)
        assert torch.equal(h, hdr) and torch.equal(p, pay)
        assert (ring.lens[:npk] == 15 + 4 * V).all()
    finally:
        a.close()
        b.close()
