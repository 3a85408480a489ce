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
PARA_LEN = 25_557_032          # ResNet-50, communicator.py:11 (config 1's model size)


def make_small():
    return torch.nn.Linear(*SIZES["small"])


def make_big():
    return torch.nn.Linear(*SIZES["big"])


class FlatResNet50(torch.nn.Module):
    """Config 1 at its size: ResNet-50's 25,557,032 parameters as ONE flat Parameter --
    aggregate() sees only parameters_to_vector (launch.py:42-52), so the layer layout
    does not change the aggregation path."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(50)
        self.flat = torch.nn.Parameter(torch.randn(PARA_LEN, generator=g) * 0.05)


MAKERS = {"small": make_small, "big": make_big, "resnet50": FlatResNet50}


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
    worker_serve(idx, W, port, path, MAKERS[size], train_step)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("V,size,epochs", [(256, "small", 3), (32, "small", 3), (32, "big", 3),
                                           (256, "resnet50", 2), (32, "resnet50", 2)])
def test_loopback_two_workers_bit_exact(V, size, epochs):
    """resnet50: config 1 at its size -- 25,557,032 parameters, W = 2 -> 2 x 99,833
    NGA-256 (or 2 x 798,657 NGA-32) packets per epoch through recvmmsg and the device
    switch, every epoch bit-exact against the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ina_amd.loopback import ps_serve
    W = 2
    torch.manual_seed(0)
    model = MAKERS[size]().cuda()
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
        th.join(timeout=420 if size == "resnet50" else 240)
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
