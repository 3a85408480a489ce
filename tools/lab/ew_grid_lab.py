"""Lab: grid cap of the chunk-loop elementwise kernels (quantise, dequantise, int16 wire
quantise / decode) at config 2's bucket (25,557,032 values) and config 5's (268,435,456
values = 1 GiB fp32), interleaved rounds, HIP events, median.  The grid cap is
ina_set_tuning keys 4 (stream_blocks: packet / fused kernels) and 14 (ew_blocks: one-in
one-out kernels), set together here; results never change, only speed.

  python tools/lab/ew_grid_lab.py [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
from ina_amd import ops  # noqa: E402

GRIDS = [int(g) for g in os.environ.get("GRIDS", "2048,4096,8192,16384,32768,65536").split(",")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = {}
    s = torch.cuda.current_stream()
    for n in (25_557_032, 268_435_456):
        x = torch.randn(n, device=dev) * 1e-2
        q = torch.empty(n, dtype=torch.int32, device=dev)
        y = torch.empty(n, dtype=torch.float32, device=dev)
        kern = {"quantize": (lambda: ops.quantize(x, 16, out=q), 8 * n),
                "dequantize": (lambda: ops.dequantize(q, 16, out=y), 8 * n),
                "quantize_i16_wire": (lambda: ops.quantize_i16_wire(x, 20, out=q), 8 * n),
                "i16_wire_finish_y": (lambda: ops.i16_wire_finish(q, 20, 256, y=y, want_out16=False),
                                      8 * n + n // 256)}
        if n < 100_000_000:                        # config-2/3-sized packet and fused kernels
            V = 256
            npk = -(-n // V)
            pk = torch.empty((npk, ops.nga_stride(V)), dtype=torch.uint8, device=dev)
            xs = [torch.randn(n, device=dev) for _ in range(4)]
            loc = torch.randn(n, device=dev)
            kern.update({
                "pack_nga": (lambda: ops.pack_nga(q, V, 1, 8, 1, 1, out=pk), 4 * n + pk.numel()),
                "unpack_nga": (lambda: ops.unpack_nga(pk, V), pk.numel() + 4 * n + 15 * npk),
                "quantize_pack_nga": (lambda: ops.quantize_pack_nga(x, 16, V, 1, 8, 1, 1, base=loc, out=pk),
                                      8 * n + pk.numel()),
                "quantize_reduce W=4": (lambda: ops.quantize_reduce(xs, 16, out=q), 20 * n),
                "ps_apply": (lambda: ops.ps_apply(loc, q, 16, 0.25, out=y), 12 * n)})
        times = {}
        for _ in range(a.rounds):
            for g in GRIDS:
                ops.set_tuning(stream_blocks=g, ew_blocks=g)
                for name, (fn, nbytes) in kern.items():
                    fn()
                    ts = []
                    for _ in range(5):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(s)
                        fn()
                        e1.record(s)
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    times.setdefault((name, g), []).extend(ts)
        for (name, g), ts in times.items():
            us = statistics.median(ts)
            res.setdefault(f"{name} n={n}", {})[g] = {"us": round(us, 1),
                                                      "frac": round(kern[name][1] / (us * 1e-6) / 8e12, 4)}
        del x, q, y, kern
    ops.set_tuning(stream_blocks=8192, ew_blocks=1 << 24)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
