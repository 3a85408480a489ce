#!/usr/bin/env python3
"""Lab: grid cap (ina_set_tuning key 4, stream_blocks) of the flat packet kernels --
pack_nga, unpack_nga (header fields + values), the worker's fused
quantise+pack -- at config 3's bucket (V = 256), including a grid that covers every
16-byte chunk with one thread (no grid-stride loop).  Interleaved rounds, cold caches
(a 512 MiB read between timed launches), HIP events, median; outputs checked equal
across grids.

  python tools/lab/stream_grid_lab.py [--rounds 5]
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

GRIDS = [int(g) for g in os.environ.get("GRIDS", "4096,8192,16384,32768,16777216").split(",")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    n, V = 26_214_400, 256
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
    xf = torch.randn(n, device=dev, generator=g) * 1e-2
    bf = torch.randn(n, device=dev, generator=g) * 1e-2
    pk = ops.pack_nga(x, V, 1, 8, 1, 1)
    npk, stride = pk.shape
    out_pk = torch.empty_like(pk)
    flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)
    cases = {
        "pack_nga": (lambda: ops.pack_nga(x, V, 1, 8, 1, 1, out=out_pk), 4 * n + npk * stride),
        "unpack_nga fields+values": (lambda: ops.unpack_nga(pk, V)[1], npk * stride + 4 * n + 15 * npk),
        "quantize_pack_nga (worker, fused)": (
            lambda: ops.quantize_pack_nga(xf, 16, V, 1, 8, 1, 1, base=bf, out=out_pk), 8 * n + npk * stride),
    }
    times = {(c, gr): [] for c in cases for gr in GRIDS}
    ref = {}
    for _ in range(a.rounds):
        for gr in GRIDS:
            ops.set_tuning(stream_blocks=gr)
            for c, (fn, _) in cases.items():
                for _ in range(4):
                    ops.checksum(flush)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    r = fn()
                    e1.record()
                    torch.cuda.synchronize()
                    times[(c, gr)].append(e0.elapsed_time(e1) * 1e3)
                key = c
                if key not in ref:
                    ref[key] = r.clone()
                elif not torch.equal(ref[key], r):
                    raise SystemExit(f"{c} at grid {gr}: output differs")
    ops.set_tuning(stream_blocks=8192)
    res = []
    for (c, gr), ts in times.items():
        us = statistics.median(ts)
        res.append({"kernel": c, "stream_blocks": gr, "us": round(us, 2),
                    "frac": round(cases[c][1] / (us * 1e-6) / 8e12, 4)})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
