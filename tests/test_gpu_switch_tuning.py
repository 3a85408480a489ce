"""The switch's tuning snapshot (include/ina.h, ina_switch phases): a sort queued alone records
the switch keys it ran under, and the run over its scratch follows that record -- so another
thread that flips keys 12 (slot sort), 18 (run table) and 19 (split first pass) between sort()
and run() changes nothing in that batch (the run used to re-read key 19 and read
arrays the sort never wrote).  Every arrival order the sort distinguishes (in slot order, dense
runs, near-sorted, shuffled), both directions of the flip: actions, rewritten packets and
registers equal a one-call process() of the same batch on a fresh switch."""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
FLIPPED = dict(switch_sort=3, switch_runs=False, switch_pre_all=False)
DEFAULT = dict(switch_sort=0, switch_runs=True, switch_pre_all=True)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ina_amd import ops  # noqa: F401  (fails loudly if libina.so is missing)


def _batch(order, W=8, npw=20_000, V=32, slots=1 << 17, seed=5):
    from ina_amd import ops
    g = torch.Generator(device=DEV).manual_seed(seed)
    rows, descs = [], []
    for w in range(W):
        b = torch.randint(-(1 << 30), 1 << 30, (npw * V,), dtype=torch.int32, device=DEV, generator=g)
        p, d = ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True)
        rows.append(p)
        descs.append(d)
    pk, ds = torch.cat(rows), torch.cat(descs)
    N = W * npw
    rr = torch.arange(N, device=DEV).view(W, npw).t().reshape(-1)
    if order == "worker_major":
        perm = None
    elif order == "round_robin":
        perm = rr
    elif order == "jitter":
        key = torch.arange(N, device=DEV) + torch.randint(0, 64, (N,), device=DEV, generator=g)
        perm = rr[torch.sort(key, stable=True).indices]
    else:
        perm = torch.randperm(N, device=DEV, generator=g)
    if perm is not None:
        pk, ds = pk[perm].contiguous(), ds[perm].contiguous()
    return pk, ds, V, slots


def _flip_on_thread(keys):
    from ina_amd import ops
    t = threading.Thread(target=lambda: ops.set_tuning(**keys))
    t.start()
    t.join()


@pytest.mark.parametrize("order", ["round_robin", "worker_major", "jitter", "shuffled"])
@pytest.mark.parametrize("sort_under,run_under", [(DEFAULT, FLIPPED), (FLIPPED, DEFAULT)])
def test_keys_flipped_between_sort_and_run(order, sort_under, run_under):
    from ina_amd import ops
    pk, ds, V, slots = _batch(order)
    try:
        ops.set_tuning(**DEFAULT)
        ref = ops.Switch(V, num_slots=slots, switch_id=1, device=DEV)
        want_pk = pk.clone()
        want_act = ref.process(want_pk, desc=ds)
        ops.set_tuning(**sort_under)
        sw = ops.Switch(V, num_slots=slots, switch_id=1, device=DEV)
        got_pk = pk.clone()
        act = sw.sort(got_pk, ds)
        _flip_on_thread(run_under)                 # another thread tunes mid-batch
        sw.run(got_pk, act)
        torch.cuda.synchronize()
    finally:
        ops.set_tuning(**DEFAULT)
    assert torch.equal(act, want_act), order
    assert torch.equal(got_pk, want_pk), order
    for x, y in ((sw.count, ref.count), (sw.frag, ref.frag), (sw.regs, ref.regs)):
        assert torch.equal(x, y), order
    assert int((act == 1).sum()) == pk.shape[0] // 8


def test_run_without_its_sort_is_refused():
    """A run whose batch no sort queued into the scratch (here: a shorter batch) is refused
    by the library itself, not only by the Python pairing check."""
    from ina_amd import _lib, ops
    import ctypes as C
    pk, ds, V, slots = _batch("round_robin", W=2, npw=2_000)
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=DEV)
    act = sw.sort(pk, ds)
    npk, stride = pk.shape
    b = _lib.SwitchBatch(pk.data_ptr(), None, npk - 1, stride, None, act.data_ptr(), sw._scratch.data_ptr())
    rc = _lib.load().ina_switch(C.byref(sw._state), C.byref(b), None, _lib.INA_SWITCH_RUN,
                                torch.cuda.current_stream().cuda_stream)
    assert rc == _lib.INA_EINVAL
    sw.run(pk, act)                                # the real pair still runs
    torch.cuda.synchronize()
    assert int((act == 1).sum()) == npk // 2


def test_run_must_name_the_sorted_batch():
    """the sort stores every dropped and foreign packet's action byte, so a run that
    names another actions buffer (or other rows, or another switch id) would leave those bytes
    unwritten -- the library refuses it; a run consumes its sort, so a second run is refused."""
    from ina_amd import _lib, ops
    import ctypes as C
    pk, ds, V, slots = _batch("jitter", W=2, npw=4_000)
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=DEV)
    act = sw.sort(pk, ds)
    npk, stride = pk.shape
    lib = _lib.load()
    cs = torch.cuda.current_stream().cuda_stream
    other_act = torch.empty_like(act)
    other_pk = pk.clone()
    for rows, a in ((pk, other_act), (other_pk, act)):
        b = _lib.SwitchBatch(rows.data_ptr(), None, npk, stride, None, a.data_ptr(), sw._scratch.data_ptr())
        assert lib.ina_switch(C.byref(sw._state), C.byref(b), None, _lib.INA_SWITCH_RUN, cs) == _lib.INA_EINVAL
    st2 = _lib.SwitchState.from_buffer_copy(sw._state)
    st2.switch_id = 2
    b = _lib.SwitchBatch(pk.data_ptr(), None, npk, stride, None, act.data_ptr(), sw._scratch.data_ptr())
    assert lib.ina_switch(C.byref(st2), C.byref(b), None, _lib.INA_SWITCH_RUN, cs) == _lib.INA_EINVAL
    assert lib.ina_switch(C.byref(sw._state), C.byref(b), None, _lib.INA_SWITCH_RUN, cs) == 0
    assert lib.ina_switch(C.byref(sw._state), C.byref(b), None, _lib.INA_SWITCH_RUN, cs) == _lib.INA_EINVAL
    torch.cuda.synchronize()
    assert int((act == 1).sum()) == npk // 2
