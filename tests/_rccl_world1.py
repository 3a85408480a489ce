"""One RCCL rank (backend nccl, world size 1), launched by torch.distributed.run from
tests/test_gpu_dist.py: the collective calls the config-5 path makes at N > 1 --
reduce_scatter_tensor(int32, SUM), all_to_all_single(int32), all_gather_into_tensor of fp32 values, int16 sums
(the i16 wire) and uint8 slot flags, all_reduce(float64, MAX/MIN) of bench.py's max-over-ranks timing -- issued
through RCCL on this image, with a device-kernel quantise/dequantise around them.  At
world size 1 every collective is a copy, so results are checked exactly; what this run
proves is that RCCL initialises with device_id and takes these dtypes and calls here."""
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))


def main():
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    from ina_amd import ops
    n, k = 1 << 20, 16
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(n, device=dev, generator=g) * 1e-2
    q = ops.quantize(x, k)
    s = torch.empty_like(q)
    dist.reduce_scatter_tensor(s, q, op=dist.ReduceOp.SUM)
    assert torch.equal(s, q)
    y = ops.dequantize(s, k)
    full = torch.empty_like(y)
    dist.all_gather_into_tensor(full, y)
    assert torch.equal(full, ops.dequantize(q, k))
    s16 = (torch.arange(4096, device=dev, dtype=torch.int32) * 37 - 70000).clamp(-32768, 32767)
    s16 = s16.to(torch.int16)
    f16 = torch.empty_like(s16)       # RCCL has no int16: dist.all_gather_shards' uint8 view
    dist.all_gather_into_tensor(f16.view(torch.uint8), s16.view(torch.uint8))
    assert torch.equal(f16, s16)
    flags = (torch.arange(4096, device=dev) % 3 == 0).to(torch.uint8)
    fo = torch.empty_like(flags)
    dist.all_gather_into_tensor(fo, flags)
    assert torch.equal(fo, flags)
    # the pipelined variant's calls: async work on views into one buffer, waited later
    buf = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    buf[n:] = q
    part = torch.empty(n, dtype=torch.int32, device=dev)
    w = dist.reduce_scatter_tensor(part, buf[n:], op=dist.ReduceOp.SUM, async_op=True)
    w.wait()
    fbuf = torch.zeros(2 * n, device=dev)
    w = dist.all_gather_into_tensor(fbuf[n:], ops.dequantize(part, k), async_op=True)
    w.wait()
    assert torch.equal(fbuf[n:], y) and not fbuf[:n].any()
    # the a2a variant's exchange: all_to_all_single of the int32 wire
    recv = torch.empty_like(q)
    dist.all_to_all_single(recv, q)
    assert torch.equal(recv, q)
    t = torch.tensor([1.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    assert float(t.item()) == 1.5
    dist.barrier()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("rccl world-1 collectives ok")


if __name__ == "__main__":
    main()
