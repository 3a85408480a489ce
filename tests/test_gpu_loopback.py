"""Config-1 flow on one GPU box: a PS process and W=2 worker processes over loopback
sockets, the switch replaced by the PS GPU's packet-stream aggregator (ops.Switch)
fed by recvmmsg, workers quantising and packing on their GPU and sending with
sendmmsg.  The PS's parameters after every epoch must equal, bit for bit, the
oracle's INA update  local + 1/(W+1) * dequant(sum_w q(p_w - local))."""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import oracle as orc
from tests.conftest import PKG_ROOT, REPO

pytestmark = pytest.mark.gpu

K = 16
SIZES = {"small": (100, 1000), "big": (100, 6000)}   # big: 606,000 params -> 18,938 NGA-32 packets


def make_small():
    return torch.nn.Linear(*SIZES["small"])


def make_big():
    return torch.nn.Linear(*SIZES["big"])


def noise(idx, epoch, n):
    g = torch.Generator().manual_seed(1000 * idx + epoch)
    return (torch.randn(n, generator=g) * 1e-2).numpy().astype(np.float32)


def train_step(model, idx, epoch):
    with torch.no_grad():
        v = torch.nn.utils.parameters_to_vector(model.parameters())
        v += torch.from_numpy(noise(idx, epoch, v.numel())).to(v.device)
        torch.nn.utils.vector_to_parameters(v, model.parameters())


def _worker(idx, W, port, path, size):
    for p in (REPO, PKG_ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    from ina_amd.loopback import worker_serve
    worker_serve(idx, W, port, path, make_big if size == "big" else make_small, train_step)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("V,size", [(256, "small"), (32, "small"), (32, "big")])
def test_loopback_two_workers_bit_exact(V, size):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ina_amd.loopback import ps_serve
    W, epochs = 2, 3
    torch.manual_seed(0)
    model = (make_big if size == "big" else make_small)().cuda()
    local0 = torch.nn.utils.parameters_to_vector(model.parameters()).detach().cpu().numpy()
    port = _free_port()
    seen = []
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "switch.sock")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker, args=(i, W, port, path, size)) for i in range(W)]
        # the PS binds first; workers retry their connect inside create_connection's backlog
        import threading
        out = {}
        th = threading.Thread(target=lambda: out.setdefault(
            "r", ps_serve(model, W, epochs, port, path, k=K, V=V,
                          on_epoch=lambda e, v, ta, tt: seen.append(v.cpu().numpy().copy()))))
        th.start()
        import time
        time.sleep(1.0)
        for p in procs:
            p.start()
        th.join(timeout=240)
        for p in procs:
            p.join(timeout=60)
        assert not th.is_alive()
        assert all(p.exitcode == 0 for p in procs)
    assert len(seen) == epochs
    local = local0
    for e in range(epochs):
        paras = [(local + noise(i, e, local.size)).astype(np.float32) for i in range(W)]
        local = orc.ps_combine_ina_f32(local, paras, K, 1.0 / (W + 1))
        assert np.array_equal(seen[e].view(np.uint32), local.view(np.uint32)), e
