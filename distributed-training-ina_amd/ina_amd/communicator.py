"""Drop-in for src/common/communicator.py (communicator.py:1-158).

Same module surface -- TENSOR_NUM_PER_PACKET, AGGREGATOR_SIZE, PARA_LEN,
dst_ip_str, ip2int, c_send_wrapper, single_process_send, multi_process_send,
multi_thread_send_futures, multi_process_send_futures_P, multi_thread_send_threading
-- bound to libina.so's send_gradients instead of ./send.so.  The symbol keeps the
reference signature (communicator.h:27); behind it the 524-byte packet_t packets
are built on the GPU and sent with sendmmsg (csrc/ina_send.cpp).

Behaviour kept: packet counts are int(len/128), so a partial tail packet is
dropped (communicator.py:42,48); the P-way split gives floor(pkts/P) to each
slice and the remainder to the last, with tensor_index = the slice's VALUE offset
(communicator.py:44-63).  Behaviour fixed: the reference's multi_* functions end
in NameError on the undefined `data_size` (communicator.py:65,91,117,157); here
data_size is the slice's byte count.

Set `send_fd` to an open datagram socket to send there (ina_send_gradients_fd)
instead of the raw IPPROTO_UDP socket send_gradients opens per call.

The process fan-outs (multi_process_send, multi_process_send_futures_P) start their
workers with the "spawn" method, never fork: send_gradients runs HIP (the packets are
built on the GPU), and a child forked from a parent that has initialised HIP is not
supported.  A `send_fd` travels to the spawned workers as a socket object (its
descriptor is duplicated into the child by multiprocessing's resource sharer).  Timing:
the reference starts its clock before `Pool(process_num)` (communicator.py:45-47,
95-97), so its printed time includes starting forked workers.  A spawned worker costs
far more to start (interpreter, imports, HIP initialisation), so the process fan-outs
print two lines: the reference's line over the reference's timed region (pool start-up
included, comparable with the reference's output), then the same figures for the sends
alone, timed after every worker is started and warm.
"""
from __future__ import annotations

import ctypes as C
import multiprocessing
import os
import socket
import threading
import time
from concurrent.futures import ProcessPoolExecutor, ThreadPoolExecutor
from ctypes import POINTER, c_int, c_uint32

from . import _lib

TENSOR_NUM_PER_PACKET = 128        # communicator.py:9
AGGREGATOR_SIZE = 199665           # communicator.py:10 (ResNet-50 / 128)
PARA_LEN = 25557032                # communicator.py:11
dst_ip_str = "172.16.210.33"       # communicator.py:13

send_fd: int | None = None          # optional datagram socket (tests / pre-opened sockets)

_send = _lib.load()                 # communicator.py:15 loaded ./send.so


def ip2int(ip: str) -> int:
    a, b, c, d = (int(x) for x in ip.strip().split("."))
    return a * 256 ** 3 + b * 256 ** 2 + c * 256 + d


def c_send_wrapper(gradient, packet_num, dst_ip: int, worker_id, aggregator_index,
                   tensor_index: int):
    """communicator.py:32-39: hand a uint32 numpy slice to the C ABI (GIL released)."""
    ptr = gradient.ctypes.data_as(POINTER(c_uint32))
    if send_fd is None:
        _send.send_gradients(ptr, c_int(packet_num), c_uint32(dst_ip), c_int(worker_id),
                             c_uint32(aggregator_index), c_int(tensor_index))
        return packet_num
    rc = _send.ina_send_gradients_fd(send_fd, C.cast(ptr, C.c_void_p), packet_num, dst_ip,
                                     worker_id, aggregator_index, tensor_index)
    return _lib.check(rc, "ina_send_gradients_fd")


def single_process_send(data):
    return c_send_wrapper(data, int(len(data) / TENSOR_NUM_PER_PACKET), ip2int(dst_ip_str),
                          0, 0, 0)


def _slices(process_num, data):
    total_packet = int(len(data) / TENSOR_NUM_PER_PACKET)
    per = int(total_packet / process_num)
    rem = int(total_packet % process_num)
    offset = 0
    for i in range(process_num):
        if i != process_num - 1:
            yield data[offset: offset + per * TENSOR_NUM_PER_PACKET], per, offset
        else:
            yield data[offset:], per + rem, offset
        offset += per * TENSOR_NUM_PER_PACKET


def _report(process_num, data, start, sends_start=None):
    """The reference's line (communicator.py:65); with sends_start, a second line for the
    sends alone (the spawned pool's start-up excluded)."""
    end = time.time()
    data_size = data.nbytes / 1e9
    print("{} processes cost: {} sec; Throuthput {} GBps".format(
        process_num, end - start, data_size / max(end - start, 1e-12)))
    if sends_start is not None:
        print("{} processes, sends only (pool started and warm): {} sec; Throughput {} GBps".format(
            process_num, end - sends_start, data_size / max(end - sends_start, 1e-12)))


_SPAWN = multiprocessing.get_context("spawn")    # never fork a HIP-initialised parent


def _child_send(sock, gradient, packet_num, dst_ip, worker_id, aggregator_index, tensor_index):
    """Runs in a spawned worker: send on the parent's socket when it passed one."""
    global send_fd
    send_fd = sock.fileno() if sock is not None else None
    try:
        return c_send_wrapper(gradient, packet_num, dst_ip, worker_id, aggregator_index,
                              tensor_index)
    finally:
        send_fd = None
        if sock is not None:
            sock.close()


def _shared_socket():
    """The caller's send_fd as a socket object a spawned worker can receive (a dup)."""
    return socket.socket(fileno=os.dup(send_fd)) if send_fd is not None else None


def _warm_worker(barrier):
    """Pool initializer: start the HIP runtime (hipFree(NULL) initialises it; libina.so is
    already loaded by this module's import) and wait until every worker got this far, so
    the timed region holds the sends only -- not interpreter start-up, library loading and
    HIP initialisation, which a spawned worker pays and the reference's forked ones did not."""
    try:
        C.CDLL("libamdhip64.so").hipFree(None)
    except (OSError, AttributeError):   # no HIP runtime here: the first send initialises it
        pass
    try:
        barrier.wait(timeout=300)
    except threading.BrokenBarrierError:   # a worker never started: warm-up only, go on
        pass


def _noop(_):
    return None


def _warm_pool_args(process_num):
    return {"initializer": _warm_worker, "initargs": (_SPAWN.Barrier(process_num),)}


def multi_process_send(process_num, data):
    sock = _shared_socket()
    start = time.time()                               # the reference's clock: before Pool()
    try:
        with _SPAWN.Pool(process_num, **_warm_pool_args(process_num)) as pool:
            pool.map(_noop, range(process_num), chunksize=1)   # every worker started and warm
            sends = time.time()
            rs = [pool.apply_async(_child_send, (sock, s, n, ip2int(dst_ip_str), 0, 0, off))
                  for s, n, off in _slices(process_num, data)]
            for r in rs:
                r.get()
    finally:
        if sock is not None:
            sock.close()
    _report(process_num, data, start, sends)


def multi_thread_send_futures(process_num, data):
    start = time.time()
    with ThreadPoolExecutor() as ex:
        fs = [ex.submit(c_send_wrapper, s, n, ip2int(dst_ip_str), 0, 0, off)
              for s, n, off in _slices(process_num, data)]
        for f in fs:
            f.result()
    _report(process_num, data, start)


def multi_process_send_futures_P(process_num, data):
    sock = _shared_socket()
    start = time.time()                               # the reference's clock: before the pool
    try:
        # process_num workers (one per slice; the reference's default pool size only adds
        # idle processes), started and warmed before the sends' clock starts
        with ProcessPoolExecutor(max_workers=process_num, mp_context=_SPAWN,
                                 **_warm_pool_args(process_num)) as ex:
            list(ex.map(_noop, range(process_num)))
            sends = time.time()
            fs = [ex.submit(_child_send, sock, s, n, ip2int(dst_ip_str), 0, 0, off)
                  for s, n, off in _slices(process_num, data)]
            for f in fs:
                f.result()
    finally:
        if sock is not None:
            sock.close()
    _report(process_num, data, start, sends)


class myThread(threading.Thread):   # communicator.py:120-131
    def __init__(self, threadID, gradient, packet_num, dst_ip, worker_id, aggregator_index,
                 tensor_index):
        threading.Thread.__init__(self)
        self.threadID = threadID
        self.gradient = gradient
        self.packet_num = packet_num
        self.dst_ip = dst_ip
        self.worker_id = worker_id
        self.aggregator_index = aggregator_index
        self.tensor_index = tensor_index
        self.error = None

    def run(self):
        try:
            c_send_wrapper(self.gradient, self.packet_num, self.dst_ip, self.worker_id,
                           self.aggregator_index, self.tensor_index)
        except Exception as e:   # surfaced by multi_thread_send_threading
            self.error = e


def multi_thread_send_threading(process_num, data):
    start = time.time()
    ts = [myThread(i, s, n, ip2int(dst_ip_str), 0, 0, off)
          for i, (s, n, off) in enumerate(_slices(process_num, data))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for t in ts:
        if t.error:
            raise t.error
    _report(process_num, data, start)
