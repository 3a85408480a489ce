"""Parameter-server surface of src/distributed_training/launch.py kept as a drop-in.

aggregate(global_model, worker_list, step_size[, worker_num]) has the signature
and meaning of launch.py:42-52 (sync: weight 1/(W+1)) and launch_async.py:42-57
(worker_num=K: the first K workers, weight 1/K).  The sum runs on the GPU:

  mode="fp32" (default)  one fused kernel (ina_ps_combine_f32) reproducing torch's
                         fp32 op sequence bit for bit;
  mode="ina"             the in-network semantics: each worker's delta p_w - local
                         is quantised (2^k fixed point), summed as wrapping int32 --
                         the switch's Processor add -- and dequantised into the
                         update (ina_ps_combine_ina_f32), one pass over HBM;
                         k="auto" picks the largest non-saturating scale from the
                         deltas' absmax (ops.scale_for_workers).

Worker.updated_paras may be CPU tensors (unpickled from the worker socket,
worker.py:78) or device tensors; CPU ones are staged through pinned memory.  The global
model may live on the GPU or -- as launch.py:38,207 leaves it when the PS sees no GPU of
its own -- on the CPU: its parameters are then staged to the aggregating GPU (`device`,
default the current one) through pinned memory, the same kernel runs, and the result is
written back into the CPU parameters.  There is no CPU compute path: without a GPU the
call raises.
communication_parallel (launch.py:111-130) and the TCP framing helpers
(trans.py:43-54, worker.py:63-79) are kept with the reference's wire format.
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import pickle
import socket
import struct

import torch

from . import ops


def _device_of(model) -> torch.device:
    for p in model.parameters():
        return p.device
    return torch.device("cuda")


def _staged(t: torch.Tensor, dev: torch.device) -> torch.Tensor:
    t = t.detach().reshape(-1)
    if t.device == dev:
        return t.contiguous().float() if t.dtype != torch.float32 else t.contiguous()
    if not t.is_pinned():
        t = t.float().contiguous().pin_memory()
    return t.to(dev, dtype=torch.float32, non_blocking=True)


def aggregate(global_model, worker_list, step_size, worker_num: int | None = None,
              mode: str = "fp32", k: int | str = 16, device: str | torch.device | None = None):
    home = _device_of(global_model)
    if home.type == "cuda":
        dev = home
    else:                                            # a CPU model: aggregate on a GPU
        if not torch.cuda.is_available():
            raise ValueError("aggregate: no GPU to aggregate on (the INA path has no CPU fallback)")
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    local = torch.nn.utils.parameters_to_vector(global_model.parameters()).detach()
    if home.type != "cuda":
        local = _staged(local, dev)
    if worker_num is not None:                       # launch_async.py:45-47
        weight = 1.0 / worker_num
        worker_list = worker_list[:worker_num]
    else:                                            # launch.py:45 / launch_async.py:49
        weight = 1.0 / (len(worker_list) + 1)
    paras = [_staged(w.updated_paras, dev) for w in worker_list]
    ws = weight * step_size                          # python float, as in launch.py:47-48
    if mode == "fp32":
        out = ops.ps_combine(local, paras, ws)
    elif mode == "ina":
        out = combine_ina(local, paras, k, ws)
    else:
        raise ValueError(f"unknown mode {mode!r}")
    if home.type != "cuda":                          # back into the CPU parameters
        host = torch.empty(out.shape, dtype=out.dtype, pin_memory=True)
        host.copy_(out)                              # synchronous: the update is complete
        out = host
    torch.nn.utils.vector_to_parameters(out, global_model.parameters())
    return out


def combine_ina(local: torch.Tensor, paras, k, weight_step: float, out=None):
    """local + float(weight_step) * dequant(sum_w q(paras[w] - local)) on the GPU.
    k="auto": the largest scale at which no delta and no W-way sum saturates
    (ops.scale_for_workers over the deltas; one host read)."""
    from . import _lib
    ops._req(local, torch.float32, "local")
    paras, n = ops._bufs(paras, torch.float32, "paras")
    if k == "auto":
        k = ops.scale_for_workers(paras, base=local)
    out = torch.empty_like(local) if out is None else out
    arr = _lib.ptr_array([p.data_ptr() for p in paras])
    _lib.check(_lib.load().ina_ps_combine_ina_f32(local.data_ptr(), arr, len(paras), k,
                                                  float(weight_step), out.data_ptr(), n,
                                                  ops._stream(local)), "ps_combine_ina")
    return out


def communication_parallel(worker_list, action, para=None, updated_data=None, partition=None):
    """launch.py:111-130: run one action on every worker concurrently."""
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    executor = concurrent.futures.ThreadPoolExecutor(max_workers=max(1, len(worker_list)))
    tasks = []
    for w in worker_list:
        if action == "init":
            tasks.append(loop.run_in_executor(executor, w.launch, para, partition))
        elif action == "pull":
            tasks.append(loop.run_in_executor(executor, w.get_trained_model))
        elif action == "push":
            tasks.append(loop.run_in_executor(executor, w.send_data, updated_data))
    if tasks:
        loop.run_until_complete(asyncio.wait(tasks))
    loop.close()
    executor.shutdown(wait=True)


# ---- TCP framing (trans.py:43-54, worker.py:63-79), wire-compatible ------------------------
def send_data(s: socket.socket, data):
    ser = pickle.dumps(data)
    s.sendall(struct.pack(">I", len(ser)))
    s.sendall(ser)


def send_timestamp_data(s: socket.socket, timestamp: float, data):
    s.sendall(struct.pack(">d", timestamp))
    send_data(s, data)


def _recv_exact(s: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = s.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return bytes(buf)


def get_data(s: socket.socket):
    (n,) = struct.unpack(">I", _recv_exact(s, 4))
    return pickle.loads(_recv_exact(s, n))   # the reference's trusted-peer protocol


def get_timestamp_data(s: socket.socket):
    (ts,) = struct.unpack(">d", _recv_exact(s, 8))
    return ts, get_data(s)
