"""Loopback INA training flow with the GPU as the software stand-in for the switch
(BASELINE config 1: worker_num=2, loopback sockets, software stand-in for src/p4).

Control plane exactly as the reference: the PS listens on TCP, pushes the flat
parameter vector to every worker (length-prefixed pickle, worker.py:63-66) and
pulls results back (trans.py:43-54).  Data plane as the INA design intends (and as
the reference never wired together): each worker quantises its update
d_w = p_w - p_global on its GPU, packs NGA-V packets on the GPU and sends them with
sendmmsg to the "switch" socket; the PS runs the P4 state machine
(ngaa.p4:120-196) on its GPU over the received batch (ops.Switch), unpacks the
completed slots, acks them (fragcheck.p4:26-31) and applies
p_global += 1/(W+1) * dequant(sum) -- aggregate()'s update (launch.py:42-52) with
the switch's integer sum in place of the float sum.

The data socket is an AF_UNIX datagram socket by default (loopback, lossless: the
reference has no loss recovery -- its resend bit is unused, headers.p4:33); a UDP
socket on 127.0.0.1 works the same way when the receive buffer is large enough.
"""
from __future__ import annotations

import socket
import time

import torch

from . import _lib, control, ops, ps
from .nic import PacketRing, send_device_packets


class SwitchStandIn:
    """The Tofino's role on the PS GPU for one bucket of n values from W workers."""

    def __init__(self, n: int, W: int, V: int = 256, switch_id: int = 1, device="cuda",
                 num_slots: int | None = None, cp: control.ControlPlane | None = None,
                 ps_addr: str = "127.0.0.1", ps_port: int = 0):
        """cp: the switch's tables (switch_check / ipRoute, ngaa.p4:27-61); by default
        switch_id aggregates and the PS address routes to ps_port.  Only completed
        slots that ipRoute sends to ps_port reach the PS."""
        self.n, self.W, self.V = n, W, V
        if cp is None:
            cp = control.ControlPlane()
            cp.Ingress.switch_check.add_with_set_agg(switch_id)
            cp.Ingress.ipRoute.add_with_ipv4_forward(ps_addr, dst_mac=0, port=ps_port)
        self.cp, self.ps_addr, self.ps_port = cp, control.ip2int(ps_addr), ps_port
        self.npk = -(-n // V)
        # The Tofino pool is 16,384 slots (config.p4:5) and the reference sends a whole
        # bucket with index = seq mod 16384 (DataManager.py:119), so buckets of more
        # packets collide there.  HBM holds a pool for the whole bucket instead.
        self.num_slots = num_slots or max(_lib.NUM_REGISTER, self.npk)
        self.switch = cp.make_switch(V, self.num_slots, device)
        self.ring = PacketRing(W * self.npk, V, device)
        self.out = torch.empty(self.npk * V, dtype=torch.int32, device=device)
        self.acks = torch.zeros((self.npk, self.ring.stride), dtype=torch.uint8, device=device)
        self.device = torch.device(device)

    def _switch_batch(self, sock, timeout_ms):
        want = self.W * self.npk
        got = 0
        while got < want:
            r = self.ring.recv(sock, want - got, timeout_ms, offset=got)
            if r == 0:
                raise TimeoutError(f"switch stand-in: {got}/{want} packets after {timeout_ms} ms")
            got += r
        pk = self.ring.to_device(got)
        act = self.switch.process(pk)
        eg = self.cp.egress(act, dst_default=self.ps_addr)       # ipRoute, ngaa.p4:39-61
        routed = torch.where(eg == self.ps_port, act, torch.zeros_like(act))
        ndone = int((routed == _lib.ACT_FWD_AGG).sum())
        if ndone != self.npk:
            bad = int((act == _lib.ACT_FWD_COLLISION).sum())
            raise RuntimeError(f"{ndone}/{self.npk} slots completed and routed to the PS "
                               f"({bad} collisions)")
        act = routed
        return pk, act

    def aggregate_apply(self, sock, seq0: int, local: torch.Tensor, k: int, weight_step: float,
                        timeout_ms: int = 30000) -> torch.Tensor:
        """Receive, switch, then ONE fused kernel: completed slots -> dequantise -> update
        (local + weight_step * sum * 2^-k) and PS acks, which then free the slots."""
        pk, act = self._switch_batch(sock, timeout_ms)
        new = ops.apply_completed(pk, act, self.V, seq0, local, k, weight_step, acks=self.acks)
        self.switch.process(self.acks)
        return new

    def aggregate(self, sock, seq0: int, timeout_ms: int = 30000) -> torch.Tensor:
        """Receive W x npk packets, run them through the switch, return int32 [n]."""
        pk, act = self._switch_batch(sock, timeout_ms)
        done = torch.nonzero(act == _lib.ACT_FWD_AGG).flatten()
        fin = pk.index_select(0, done)
        fields, vals = ops.unpack_nga(fin, self.V)
        slot = (fields["frag_id"].to(torch.int64) - seq0) % (1 << 32)
        self.out.view(self.npk, self.V).index_copy_(0, slot, vals.view(self.npk, self.V))
        fin[:, 5] = _lib.FLAG_ACK                        # PS ack clears each slot's frag
        self.switch.process(fin)
        return self.out[: self.n]


def worker_send(sock, params: torch.Tensor, base: torch.Tensor, worker_id: int, W: int, V: int,
                k: int, seq0: int, switch_id: int = 1, num_slots: int = _lib.NUM_REGISTER) -> int:
    """Worker data plane: quantise(params - base) + NGA-V pack in one GPU pass, then
    sendmmsg.  num_slots must be the aggregator's pool size (index = seq mod num_slots,
    DataManager.py:119)."""
    pk = ops.quantize_pack_nga(params.reshape(-1).contiguous(), k, V, bitmap=worker_id, count=W,
                               switch_id=switch_id, seq0=seq0, base=base.reshape(-1).contiguous(),
                               num_slots=num_slots)
    return send_device_packets(sock, pk, _lib.NGA_HDR_BYTES + 4 * V)


def seq_base(epoch: int, npk: int) -> int:
    return (1 + epoch * npk) & 0xFFFFFFFF      # send_data numbers from 1 (DataManager.py:106)


def ps_serve(model, W: int, epochs: int, tcp_port: int, data_path: str, k: int = 16,
             V: int = 256, on_epoch=None, timeout_ms: int = 60000):
    """PS side (master_loop's epoch, launch.py:209-242, with the INA data plane)."""
    dev = next(model.parameters()).device
    local = torch.nn.utils.parameters_to_vector(model.parameters()).detach()
    n = local.numel()
    sw = SwitchStandIn(n, W, V, device=dev)
    data = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
    data.bind(data_path)
    data.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 24)
    srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind(("127.0.0.1", tcp_port))
    srv.listen(W)
    conns = []
    try:
        for _ in range(W):
            c, _ = srv.accept()
            conns.append(c)
        for c in conns:                                   # init (worker.py:56-61)
            ps.send_data(c, {"para": local.cpu(), "epochs": epochs, "k": k, "V": V,
                             "num_slots": sw.num_slots})
        for epoch in range(epochs):
            t0 = time.time()
            new = sw.aggregate_apply(data, seq_base(epoch, sw.npk), local, k, 1.0 / (W + 1),
                                     timeout_ms)
            t_agg = time.time()
            torch.nn.utils.vector_to_parameters(new, model.parameters())
            local = new
            host = local.cpu()
            for c in conns:                               # push (launch.py:222-227)
                ps.send_data(c, host)
            if on_epoch:
                on_epoch(epoch, local, t_agg - t0, time.time() - t0)
    finally:
        for c in conns:
            c.close()
        srv.close()
        data.close()
    return local


def worker_serve(idx: int, W: int, tcp_port: int, data_path: str, make_model, train_step,
                 device="cuda"):
    """Worker side (worker_loop, launch.py:248-322, with the INA data plane)."""
    ctl = socket.create_connection(("127.0.0.1", tcp_port))
    data = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
    data.connect(data_path)
    try:
        cfg = ps.get_data(ctl)
        k, V, epochs = cfg["k"], cfg["V"], cfg["epochs"]
        model = make_model().to(device)
        glob = cfg["para"].to(device)
        torch.nn.utils.vector_to_parameters(glob, model.parameters())
        npk = -(-glob.numel() // V)
        for epoch in range(epochs):
            train_step(model, idx, epoch)
            p = torch.nn.utils.parameters_to_vector(model.parameters()).detach()
            worker_send(data, p, glob, idx + 1, W, V, k, seq_base(epoch, npk),
                        num_slots=cfg["num_slots"])
            glob = ps.get_data(ctl).to(device)
            torch.nn.utils.vector_to_parameters(glob, model.parameters())
    finally:
        data.close()
        ctl.close()
