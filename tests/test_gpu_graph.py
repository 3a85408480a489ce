"""GPU: the device path is capture-safe -- one PS epoch (workers' fused quantise+pack,
the packet-stream switch, the fused completed-slot apply and the PS acks that free the
slots) recorded once as a hipGraph and replayed on fresh inputs gives the same bytes as
running the ops eagerly.  Every ina_* entry point is asynchronous on the caller's stream
and neither allocates nor synchronises."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _epoch(o, sw, xs, base, local, V, k, W, seq0, slots, pk_buf, acks, out):
    torch.cat([o.quantize_pack_nga(x, k, V, bitmap=w + 1, count=W, switch_id=1, seq0=seq0,
                                   base=base, num_slots=slots) for w, x in enumerate(xs)],
              out=pk_buf)
    act = sw.process(pk_buf)
    o.apply_completed(pk_buf, act, V, seq0, local, k, 1.0 / (W + 1), out=out, acks=acks)
    sw.process(acks)                      # PS acks clear each slot's frag (fragcheck.p4:26-31)
    return act


@pytest.mark.parametrize("V,n,W", [(256, 256 * 300 + 77, 4), (32, 32 * 500 + 5, 2)])
def test_epoch_replays_as_hip_graph(V, n, W):
    from ina_amd import ops as o
    k, slots, seq0 = 16, 4096, 1
    npk = -(-n // V)
    stride = o.nga_stride(V)
    g = torch.Generator(device=DEV).manual_seed(n)
    xs = [torch.empty(n, device=DEV) for _ in range(W)]
    base = torch.empty(n, device=DEV)
    local = torch.empty(n, device=DEV)
    pk_buf = torch.empty((W * npk, stride), dtype=torch.uint8, device=DEV)
    acks = torch.zeros((npk, stride), dtype=torch.uint8, device=DEV)
    out = torch.empty(n, device=DEV)
    sw = o.Switch(V, num_slots=slots, switch_id=1, device=DEV)

    def fill(i):
        for w, x in enumerate(xs):
            x.copy_(torch.randn(n, device=DEV, generator=g) * 1e-2 * (i + 1) + w)
        base.copy_(torch.randn(n, device=DEV, generator=g) * 1e-3)
        local.copy_(torch.randn(n, device=DEV, generator=g))

    # eager reference for three epochs (switch state carries over, as in training)
    want = []
    fill(0)
    s = torch.cuda.Stream(DEV)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):             # warm-up on the capture stream (scratch, kernels)
        _epoch(o, sw, xs, base, local, V, k, W, seq0, slots, pk_buf, acks, out)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    sw_ref = o.Switch(V, num_slots=slots, switch_id=1, device=DEV)
    sw_ref.count.copy_(sw.count)
    sw_ref.frag.copy_(sw.frag)
    sw_ref.regs.copy_(sw.regs)
    inputs = []
    for i in range(1, 4):
        fill(i)
        inputs.append([t.clone() for t in (*xs, base, local)])
        pk2 = torch.empty_like(pk_buf)
        acks2 = torch.zeros_like(acks)
        out2 = torch.empty_like(out)
        act = _epoch(o, sw_ref, xs, base, local, V, k, W, seq0, slots, pk2, acks2, out2)
        want.append((out2.clone(), act.clone(), pk2.clone()))

    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        act_g = _epoch(o, sw, xs, base, local, V, k, W, seq0, slots, pk_buf, acks, out)
    for i, inp in enumerate(inputs):
        for t, v in zip((*xs, base, local), inp):
            t.copy_(v)
        graph.replay()
        torch.cuda.synchronize()
        w_out, w_act, w_pk = want[i]
        assert torch.equal(act_g, w_act), i
        assert torch.equal(out, w_out), i
        fwd = w_act == 1
        assert torch.equal(pk_buf[fwd], w_pk[fwd]), i
        assert int(fwd.sum()) == npk
    assert torch.equal(sw.count, sw_ref.count) and torch.equal(sw.frag, sw_ref.frag)
    assert np.array_equal(sw.regs.cpu().numpy(), sw_ref.regs.cpu().numpy())
