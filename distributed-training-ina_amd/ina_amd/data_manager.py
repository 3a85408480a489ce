"""Drop-in for src/common/DataManager.py (DataManager.py:33-168).

DataManager(src_ip, dst_ip, data, interface, thread_num) quantises its gradient
at construction and on update_data (DataManager.py:37,168) and sends it as NGA
packets with send_data / fast_send_data (104-109, 42-102).  Here the quantiser
(the build's float_to_int: sat(rne(x * 2^k))), the packetiser (15-byte header +
V big-endian words, zero-padded tail; DataManager.py:116-153) run on the GPU;
the packets come back into one pinned buffer and leave in sendmmsg batches on a
raw IPv4 socket with protocol 0x12 (DataManager.py:112), or on a caller-provided
datagram socket (`sock=`).

Reference behaviour kept: send_data numbers packets from sequence 1 and never
emits the end marker (its `True` binds to `sequence`, DataManager.py:106);
fast_send_data numbers from 0; index = sequence mod 16384 (119); the header is
'!IbbIbI' = worker_id, degree, 0, index, switch_id, sequence (122-130), so
degree and switch_id must fit a signed byte as struct.pack requires.
"""
from __future__ import annotations

import socket
import time

import numpy as np
import torch

from . import _lib, ops
from .packet import NGA_TYPE, end_marker


def _signed_byte(name, v):
    if not -128 <= v <= 127:   # struct.pack('b') range, DataManager.py:122
        raise ValueError(f"{name} must fit a signed byte ('b'), got {v}")
    return v & 0xFF


class DataManager:
    def __init__(self, src_ip, dst_ip, data=None, interface="eth0", thread_num=4, k=16, V=32,
                 device="cuda", sock=None):
        self.src_ip = src_ip
        self.dst_ip = dst_ip
        self.iface = interface
        self.thread_num = thread_num          # kept for signature parity; sendmmsg batches instead
        self.k, self.V = k, V
        self.device = torch.device(device)
        self._sock = sock
        self.data = None
        if data is not None:
            self.update_data(data)

    # DataManager.py:167-168
    def update_data(self, new_data):
        x = torch.as_tensor(new_data, dtype=torch.float32)
        x = x.reshape(-1).to(self.device, non_blocking=True).contiguous()
        self.data = ops.quantize(x, self.k)

    def _socket(self):
        if self._sock is None:
            self._sock = socket.socket(socket.AF_INET, socket.SOCK_RAW, NGA_TYPE)
        return self._sock

    def packets(self, worker_id, switch_id, degree, sequence=0, offset=0, step=None):
        """Device uint8 [npkts, stride] NGA-V packets for data[offset:offset+step]."""
        step = self.data.numel() - offset if step is None else step
        vals = self.data[offset: offset + step]
        return ops.pack_nga(vals, self.V, bitmap=worker_id, count=_signed_byte("degree", degree),
                            switch_id=_signed_byte("switch_id", switch_id), seq0=sequence)

    def _send_data(self, worker_id, switch_id, degree, offset, step, sequence=0, end=False):
        """DataManager.py:111-165; returns the number of payload values sent."""
        if step <= 0:
            pk = None
        else:
            pk = self.packets(worker_id, switch_id, degree, sequence, offset, step)
        s = self._socket()
        dst = 0 if self._sock_is_connected(s) else _ip2int(self.dst_ip)
        if pk is not None:
            host = torch.empty(pk.shape, dtype=torch.uint8, pin_memory=True)
            host.copy_(pk)                    # D2H into pinned memory (synchronous copy)
            plen = 15 + 4 * self.V
            rc = _lib.load().ina_send_packets_fd(s.fileno(), host.data_ptr(), pk.shape[0],
                                                 pk.shape[1], plen, dst)
            _lib.check(rc, "ina_send_packets_fd")
        if end is True:
            s.sendto(end_marker(worker_id, degree, switch_id), (self.dst_ip, 0)) if dst else \
                s.send(end_marker(worker_id, degree, switch_id))
        return max(step, 0)

    @staticmethod
    def _sock_is_connected(s):
        try:
            s.getpeername()
            return True
        except OSError:
            return s.family == socket.AF_UNIX

    def send_data(self, worker_id, switch_id, degree):
        start_time = time.time()
        self._send_data(worker_id, switch_id, degree, 0, self.data.numel(), True)   # sic: seq 1
        print("END: send to nic.")
        print("Total time: {}.".format(time.time() - start_time))

    def fast_send_data(self, worker_id, switch_id, degree, send_step=10000):
        print("send to nic...")
        start_time = time.time()
        count = self._send_data(worker_id, switch_id, degree, 0, self.data.numel())
        print("END: send to nic.")
        print("Total time: {}, byte count: {}.".format(time.time() - start_time, count))


def _ip2int(ip: str) -> int:
    a, b, c, d = (int(x) for x in ip.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def float_to_int(data, k=16, device="cuda") -> torch.Tensor:
    """The quantiser the reference imports from the missing utils.comm_utils (device)."""
    return ops.quantize(torch.as_tensor(np.asarray(data, np.float32)).to(device), k)


def int_to_float(data, k=16, device="cuda") -> torch.Tensor:
    """The dequantiser the reference imports from the missing utils.comm_utils (device)."""
    t = torch.as_tensor(np.asarray(data, np.int32)).to(device)
    return ops.dequantize(t, k)
