"""Host packet I/O for the device path.

The reference receives one datagram per recvfrom() into a Python list
(get_data_from_nic, utils.py:61-64; RecvThread/RecvProcess 67-94) and sends one per
sendto() (DataManager.py:134,153; communicator.cc:37).  Here datagrams move in
recvmmsg()/sendmmsg() batches between the socket and a pinned host ring laid out
exactly like the device packet buffers (stride = ops.nga_stride(V)), so one
hipMemcpyAsync moves a whole batch to or from HBM.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib, ops


class PacketRing:
    """Pinned host buffer + device buffer of `capacity` packets at the NGA stride."""

    def __init__(self, capacity: int, V: int, device="cuda", stride: int | None = None):
        self.capacity, self.V = capacity, V
        self.stride = stride or ops.nga_stride(V)
        self.host = torch.empty((capacity, self.stride), dtype=torch.uint8, pin_memory=True)
        self.dev = torch.empty((capacity, self.stride), dtype=torch.uint8, device=device)
        self.lens = np.zeros(capacity, np.uint32)

    def recv(self, sock, max_pkts: int | None = None, timeout_ms: int = 1000, skip: int = 0,
             offset: int = 0) -> int:
        """Receive up to max_pkts datagrams into slots [offset, offset+n); returns n."""
        max_pkts = self.capacity - offset if max_pkts is None else max_pkts
        if offset + max_pkts > self.capacity:
            raise ValueError("ring overflow")
        base = self.host.data_ptr() + offset * self.stride
        lp = self.lens.ctypes.data + 4 * offset
        rc = _lib.load().ina_recv_packets_fd(sock.fileno(), base, max_pkts, self.stride, skip,
                                             timeout_ms, lp)
        return _lib.check(rc, "ina_recv_packets_fd")

    def to_device(self, n: int) -> torch.Tensor:
        self.dev[:n].copy_(self.host[:n], non_blocking=True)
        return self.dev[:n]


def send_device_packets(sock, pkts: torch.Tensor, pkt_len: int, dst_ip: int = 0,
                        staging: torch.Tensor | None = None) -> int:
    """D2H a uint8 [npkts, stride] device packet batch into pinned memory and sendmmsg it
    (pkt_len wire bytes of each row).  Returns packets sent."""
    npk, stride = pkts.shape
    if staging is None or staging.shape[0] < npk or staging.shape[1] != stride:
        staging = torch.empty((npk, stride), dtype=torch.uint8, pin_memory=True)
    staging[:npk].copy_(pkts)
    rc = _lib.load().ina_send_packets_fd(sock.fileno(), staging.data_ptr(), npk, stride, pkt_len,
                                         dst_ip)
    return _lib.check(rc, "ina_send_packets_fd")


class SplitPacketRing:
    """The same ring for split rows (include/ina.h): pinned header rows [capacity, 16] and
    payload rows [capacity, 4V]; recvmmsg scatters each datagram's 15 header bytes and 4V
    payload bytes into them (two iovecs), so the device copies are aligned row arrays."""

    def __init__(self, capacity: int, V: int, device="cuda"):
        self.capacity, self.V = capacity, V
        self.host_hdr = torch.zeros((capacity, 16), dtype=torch.uint8, pin_memory=True)
        self.host_pay = torch.empty((capacity, 4 * V), dtype=torch.uint8, pin_memory=True)
        self.hdr = torch.zeros((capacity, 16), dtype=torch.uint8, device=device)
        self.pay = torch.empty((capacity, 4 * V), dtype=torch.uint8, device=device)
        self.lens = np.zeros(capacity, np.uint32)

    def recv(self, sock, max_pkts: int | None = None, timeout_ms: int = 1000, skip: int = 0,
             offset: int = 0) -> int:
        max_pkts = self.capacity - offset if max_pkts is None else max_pkts
        if offset + max_pkts > self.capacity:
            raise ValueError("ring overflow")
        rc = _lib.load().ina_recv_packets_split_fd(
            sock.fileno(), self.host_hdr.data_ptr() + 16 * offset, self.host_pay.data_ptr() + 4 * self.V * offset,
            max_pkts, self.V, skip, timeout_ms, self.lens.ctypes.data + 4 * offset)
        return _lib.check(rc, "ina_recv_packets_split_fd")

    def to_device(self, n: int):
        self.hdr[:n].copy_(self.host_hdr[:n], non_blocking=True)
        self.pay[:n].copy_(self.host_pay[:n], non_blocking=True)
        return self.hdr[:n], self.pay[:n]


def send_device_split(sock, hdr: torch.Tensor, pay: torch.Tensor, V: int, dst_ip: int = 0) -> int:
    """D2H split rows (uint8 [npkts, 16] + [npkts, 4V]) into pinned memory and sendmmsg them,
    two iovecs per datagram: the same wire bytes as the packed rows.  Returns packets sent."""
    npk = hdr.shape[0]
    sh = torch.empty((npk, 16), dtype=torch.uint8, pin_memory=True)
    sp = torch.empty((npk, 4 * V), dtype=torch.uint8, pin_memory=True)
    sh.copy_(hdr[:npk])
    sp.copy_(pay[:npk])
    rc = _lib.load().ina_send_packets_split_fd(sock.fileno(), sh.data_ptr(), sp.data_ptr(), npk, V, dst_ip)
    return _lib.check(rc, "ina_send_packets_split_fd")
