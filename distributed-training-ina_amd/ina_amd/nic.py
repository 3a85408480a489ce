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
