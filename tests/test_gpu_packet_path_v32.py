"""The INA packet path in the P4 program's own NGA-32 format (headers.p4:40-73) at full
config-3 size, as bench.py's packet_path_v32 leg runs it: 8 workers x 26,214,400 fp32 ->
quantise(p_w - p_global, k=16) + NGA-32 split packs (ina_quantize_pack_nga_multi_split, one
launch) -> one switch batch of the previous step's 819,200 PS acks in front of 6,553,600
worker packets (2^20-slot pool) -> every completed slot applied to p_global by the fused PS
step (ina_switch (split rows + PS step), launch.py:46-50).  Three steady-state steps: every
worker packet completes its slot exactly once, every ack frees one, and the update at a
strided sample equals the oracle's PS combine (oracle.ps_combine_ina_f32, the C restatement
of ps.py's quantised aggregation) bit for bit."""
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
    from ina_amd import ops  # noqa: F401  (fails loudly if libina.so is missing)


def test_packet_path_v32_full_c3_vs_oracle():
    from ina_amd import ops as o
    W, n, V, k, slots = 8, 26_214_400, 32, 16, 1 << 20
    npk = n // V
    ws = 1.0 / (W + 1)
    g = torch.Generator(device=DEV).manual_seed(6032)
    xs = [torch.randn(n, device=DEV, generator=g) * 1e-2 for _ in range(W)]
    glob = torch.randn(n, device=DEV, generator=g) * 1e-2
    upd = torch.empty_like(glob)
    hdr = torch.zeros(((W + 1) * npk, 16), dtype=torch.uint8, device=DEV)      # [acks | workers]
    pay = torch.zeros(((W + 1) * npk, 4 * V), dtype=torch.uint8, device=DEV)
    desc = torch.empty((W + 1) * npk, dtype=torch.int64, device=DEV)
    acts = torch.empty((W + 1) * npk, dtype=torch.uint8, device=DEV)
    hw, pw = list(hdr[npk:].view(W, npk, 16).unbind(0)), list(pay[npk:].view(W, npk, 4 * V).unbind(0))
    dw = list(desc[npk:].view(W, npk).unbind(0))
    sw = o.Switch(V, num_slots=slots, switch_id=1, device=DEV)
    o.nga_descriptors(hdr[:npk], out=desc[:npk])         # step 0's "acks": another switch's rows
    # a strided sample, both ends and a whole slot at a 4 Ki boundary
    idx = np.unique(np.concatenate([np.arange(0, n, 1009), np.arange(n - 64, n), np.arange(4096 * V, 4097 * V)]))
    ti = torch.from_numpy(idx).to(DEV)
    xs_s = [x[ti].cpu().numpy() for x in xs]
    for step in range(3):
        local = glob[ti].cpu().numpy()
        o.quantize_pack_nga_multi_split(xs, k, V, [w + 1 for w in range(W)], W, 1, 1, base=glob,
                                        num_slots=slots, hdrs=hw, pays=pw, descs=dw)
        sw.process_apply_split(hdr, pay, 1, glob, k, ws, out=upd, ack_hdr=hdr[:npk], ack_desc=desc[:npk],
                               keep_forwarded=False, actions=acts, desc=desc)
        torch.cuda.synchronize()
        a = acts.cpu().numpy()
        assert int((a[npk:] == orc.ACT_FWD_AGG).sum()) == npk, step       # each slot completes once
        if step > 0:
            assert (a[:npk] == orc.ACT_FWD_ACK).all(), step                # every ack frees its slot
        if step > 0:                                                      # 9 dense runs: no sort
            assert sw.batch_path((W + 1) * npk) == "runs", step
        want = orc.ps_combine_ina_f32(local, xs_s, k, ws)
        got = upd[ti].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), step
        glob.copy_(upd)
