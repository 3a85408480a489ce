"""GPU tests of the drop-in host surfaces: DataManager (DataManager.py),
communicator (communicator.py fan-out over the legacy send_gradients path),
launch.py's aggregate() and the sharded aggregator, each through libina.so's
device kernels and checked against the oracle / the reference's own outputs."""
import socket

import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests._golden import load_capture, ps_cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _drain(sock, n):
    return [sock.recv(4096) for _ in range(n)]


@pytest.mark.parametrize("n,entry", [(70, "send"), (64, "send"), (1, "send"), (96, "fast"),
                                     (40, "end")])
def test_data_manager_datagrams(n, entry):
    from ina_amd.data_manager import DataManager
    x = (np.random.default_rng(n).standard_normal(n) * 0.5).astype(np.float32)
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    try:
        dm = DataManager("10.0.0.1", "10.0.0.2", data=x, sock=a)
        if entry == "send":
            dm.send_data(6, 2, 3)
            seq0, end = 1, False
        elif entry == "fast":
            dm.fast_send_data(6, 2, 3)
            seq0, end = 0, False
        else:
            dm._send_data(6, 2, 3, 0, n, 5, True)
            seq0, end = 5, True
        npk = -(-n // 32)
        got = _drain(b, npk + (1 if end else 0))
    finally:
        a.close()
        b.close()
    want = orc.pack_nga(orc.quantize_i32(x, 16), 32, 6, 3, 2, seq0)
    assert [g for g in got[:npk]] == [w.tobytes() for w in want]
    if end:
        assert got[-1] == bytes([0, 0, 0, 6, 3, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0])


def test_communicator_thread_fanout_matches_reference_packets():
    from ina_amd import communicator as cm
    data, pkts = load_capture("c128_threads3_1000.bin")
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    b.settimeout(10)
    try:
        cm.send_fd = a.fileno()
        cm.multi_thread_send_threading(3, data)
        got = _drain(b, len(pkts))
    finally:
        cm.send_fd = None
        a.close()
        b.close()
    assert sorted(got) == sorted(pkts)


@pytest.mark.parametrize("fanout", ["multi_process_send", "multi_process_send_futures_P"])
def test_communicator_process_fanout_after_gpu_use(fanout):
    """The process fan-outs after the parent has initialised HIP (a device op first):
    workers are spawned, not forked, and send on the parent's socket; the
    packets equal the reference's captured bytes."""
    from ina_amd import communicator as cm
    from ina_amd import ops
    ops.checksum(torch.arange(1024, dtype=torch.int32, device="cuda"))   # HIP is live here
    torch.cuda.synchronize()
    data, pkts = load_capture("c128_threads3_1000.bin")
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    b.settimeout(60)
    try:
        cm.send_fd = a.fileno()
        getattr(cm, fanout)(3, data)
        got = _drain(b, len(pkts))
    finally:
        cm.send_fd = None
        a.close()
        b.close()
    assert sorted(got) == sorted(pkts)


def _model_with(vec):
    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Parameter(torch.zeros(len(vec) // 2))
            self.b = torch.nn.Parameter(torch.zeros(len(vec) - len(vec) // 2))
    m = M().cuda()
    torch.nn.utils.vector_to_parameters(torch.from_numpy(vec).cuda(), m.parameters())
    return m


class _Wk:
    def __init__(self, p):
        self.updated_paras = p


def test_aggregate_fp32_matches_reference_outputs():
    from ina_amd import ps
    for name, c in ps_cases().items():
        W, K = int(c["W"]), int(c["K"])
        m = _model_with(c["local"])
        wl = [_Wk(torch.from_numpy(p)) for p in c["paras"]]       # CPU tensors, as unpickled
        with torch.no_grad():
            ps.aggregate(m, wl, float(c["step"]), None if K < 0 else K)
        got = torch.nn.utils.parameters_to_vector(m.parameters()).detach().cpu().numpy()
        assert np.array_equal(got.view(np.uint32), c["out"].view(np.uint32)), name


@pytest.mark.parametrize("mode", ["fp32", "ina"])
def test_aggregate_cpu_model_matches_reference_outputs(mode):
    """A PS whose global model stays on the CPU (launch.py:38,207 moves it to cuda only when
    it sees a GPU): aggregate() stages it through pinned memory, runs the same kernel and
    writes the CPU parameters back -- bit-exact against the reference's own aggregate()
    outputs (fp32), and equal to the same call on a GPU model (ina mode)."""
    from ina_amd import ps
    for name, c in ps_cases().items():
        W, K = int(c["W"]), int(c["K"])
        cpu_model = _model_with(c["local"]).cpu()
        assert next(cpu_model.parameters()).device.type == "cpu"
        wl = [_Wk(torch.from_numpy(p)) for p in c["paras"]]
        with torch.no_grad():
            ps.aggregate(cpu_model, wl, float(c["step"]), None if K < 0 else K, mode=mode)
        got = torch.nn.utils.parameters_to_vector(cpu_model.parameters()).detach().numpy()
        assert next(cpu_model.parameters()).device.type == "cpu"
        if mode == "fp32":
            want = c["out"]
        else:
            gpu_model = _model_with(c["local"])
            with torch.no_grad():
                ps.aggregate(gpu_model, wl, float(c["step"]), None if K < 0 else K, mode=mode)
            want = torch.nn.utils.parameters_to_vector(gpu_model.parameters()).detach().cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), name


def test_aggregate_ina_mode_matches_oracle():
    from ina_amd import ps
    rng = np.random.default_rng(4)
    n, W, k = 300_001, 6, 18
    local = rng.standard_normal(n).astype(np.float32)
    paras = [local + (rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(W)]
    m = _model_with(local)
    with torch.no_grad():
        ps.aggregate(m, [_Wk(torch.from_numpy(p).cuda()) for p in paras], 1.0, mode="ina", k=k)
    got = torch.nn.utils.parameters_to_vector(m.parameters()).detach().cpu().numpy()
    want = orc.ps_combine_ina_f32(local, paras, k, 1.0 / (W + 1))
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    ref = orc.ps_combine_f32(local, paras, 1.0 / (W + 1))
    assert np.abs(got - ref).max() <= W * 2.0 ** -(k + 1) / (W + 1) + 2e-7 * np.abs(ref).max()


def test_sharded_aggregator_single_rank():
    from ina_amd.dist import ShardedAggregator
    n, k = 1_000_003, 16
    g = (np.random.default_rng(9).standard_normal(n) * 1e-2).astype(np.float32)
    agg = ShardedAggregator(n, k=k)
    out = agg(torch.from_numpy(g).cuda()).cpu().numpy()
    want = orc.dequantize_i32(orc.quantize_i32(g, k), k)
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32))


def test_float_to_int_helpers():
    from ina_amd.data_manager import float_to_int, int_to_float
    x = np.array([0.5, -1.25, 3e-6, 1e9], np.float32)
    q = float_to_int(x)
    assert np.array_equal(q.cpu().numpy(), orc.quantize_i32(x, 16))
    assert np.array_equal(int_to_float(q.cpu().numpy()).cpu().numpy(),
                          orc.dequantize_i32(orc.quantize_i32(x, 16), 16))
