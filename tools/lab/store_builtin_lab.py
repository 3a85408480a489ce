#!/usr/bin/env python3
"""Store-helper A/B lab (experiment only): libina.so with the compiler-visible sc1 store
(`__builtin_amdgcn_raw_buffer_store_b*`, csrc/ina_device.h) against the round-3 library
whose stream_store was inline asm (`tools/lab/libina_asmstore.so`, built from the round-3
sources by `git archive 84f5acb distributed-training-ina_amd/csrc include` + make OUT=...).
Headline (C3 W = 8 int32), C2 (4 x ResNet-50 fp32 fused quantise + reduce), C4 (16 x
ResNet-50 int16 saturating) and the 1 GiB quantise / dequantise, timed back to back (20
launches, two alternating input sets, HIP events) interleaved A/B/A/B over rounds; every
output compared byte for byte between the two libraries, and the reduce at W = 1..17, 32,
64 against torch's wrapping int32 sum."""
import ctypes as C
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
LIBS = {"builtin": os.path.join(REPO, "distributed-training-ina_amd", "ina_amd", "libina.so"),
        "asm": os.path.join(HERE, "libina_asmstore.so")}
libs = {k: C.CDLL(p) for k, p in LIBS.items()}
VP = C.c_void_p
for L in libs.values():
    L.ina_sum_reduce_i32.argtypes = [VP, C.c_int, VP, C.c_size_t, VP]
    L.ina_quantize_reduce_f32_i32.argtypes = [VP, C.c_int, VP, C.c_size_t, C.c_int, VP]
    L.ina_quantize_reduce_f32_i16_sat.argtypes = [VP, C.c_int, VP, C.c_size_t, C.c_int, C.c_int, VP, VP]
    L.ina_quantize_f32_i32.argtypes = [VP, VP, C.c_size_t, C.c_int, VP]
    L.ina_dequantize_i32_f32.argtypes = [VP, VP, C.c_size_t, C.c_int, VP]
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(5)
st = VP(torch.cuda.current_stream().cuda_stream)
K, ROUNDS = int(os.environ.get("K", 20)), int(os.environ.get("ROUNDS", 6))
NR = 25_557_032


def ptrs(ts):
    return (VP * len(ts))(*[t.data_ptr() for t in ts])


def case_c3():
    n, W = 26_214_400, 8
    sets = [[torch.randint(-(1 << 30), 1 << 30, (n,), dtype=torch.int32, device=dev, generator=g) for _ in range(W)]
            for _ in range(2)]
    arrs = [ptrs(s) for s in sets]
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
    return lambda L, s: L.ina_sum_reduce_i32(arrs[s], W, outs[s].data_ptr(), n, st), outs, (W + 1) * n * 4


def case_c2():
    n, W = NR, 4
    sets = [[torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)] for _ in range(2)]
    arrs = [ptrs(s) for s in sets]
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
    return lambda L, s: L.ina_quantize_reduce_f32_i32(arrs[s], W, outs[s].data_ptr(), n, 16, st), outs, (4 * W + 4) * n


def case_c4():
    n, W, V = NR, 16, 256
    sets = [[torch.randn(n, device=dev, generator=g) * 1e-2 for _ in range(W)] for _ in range(2)]
    arrs = [ptrs(s) for s in sets]
    outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
    flags = [torch.empty((n + V - 1) // V, dtype=torch.uint8, device=dev) for _ in range(2)]
    return (lambda L, s: L.ina_quantize_reduce_f32_i16_sat(arrs[s], W, outs[s].data_ptr(), n, 12, V,
                                                           flags[s].data_ptr(), st),
            outs, (4 * W + 2) * n)


def case_quant():
    n = 1 << 28
    xs = [torch.randn(n, device=dev, generator=g) for _ in range(2)]
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
    return lambda L, s: L.ina_quantize_f32_i32(xs[s].data_ptr(), outs[s].data_ptr(), n, 16, st), outs, 8 * n


def case_dequant():
    n = 1 << 28
    xs = [torch.randint(-(1 << 30), 1 << 30, (n,), dtype=torch.int32, device=dev, generator=g) for _ in range(2)]
    outs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(2)]
    return lambda L, s: L.ina_dequantize_i32_f32(xs[s].data_ptr(), outs[s].data_ptr(), n, 16, st), outs, 8 * n


def wsweep():
    bad = []
    n = 1_000_003
    for W in list(range(1, 18)) + [32, 64]:
        bufs = [torch.randint(-(1 << 31), (1 << 31) - 1, (n,), dtype=torch.int32, device=dev, generator=g)
                for _ in range(W)]
        want = torch.stack([b.to(torch.int64) for b in bufs]).sum(0)
        want = ((want + (1 << 31)) % (1 << 32) - (1 << 31)).to(torch.int32)
        for name, L in libs.items():
            out = torch.empty(n, dtype=torch.int32, device=dev)
            assert L.ina_sum_reduce_i32(ptrs(bufs), W, out.data_ptr(), n, st) == 0
            torch.cuda.synchronize()
            if not torch.equal(out, want):
                bad.append((name, W))
    return bad


def main():
    res = {"wsweep_mismatch": wsweep()}
    print("wsweep", res["wsweep_mismatch"], flush=True)
    for cname, mk in [("c3", case_c3), ("c2", case_c2), ("c4", case_c4), ("quant_1g", case_quant),
                      ("dequant_1g", case_dequant)]:
        launch, outs, nbytes = mk()
        ref = {}
        for name, L in libs.items():
            assert launch(L, 0) == 0
            torch.cuda.synchronize()
            ref[name] = outs[0].clone()
        equal = torch.equal(ref["builtin"], ref["asm"])
        del ref
        t = {k: [] for k in libs}
        for _ in range(ROUNDS):
            for name, L in libs.items():
                for i in range(10):
                    launch(L, i % 2)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for i in range(K):
                    launch(L, i % 2)
                b.record()
                torch.cuda.synchronize()
                t[name].append(a.elapsed_time(b) * 1e3 / K)
        row = {"bytes_equal": equal}
        for name in libs:
            med = statistics.median(t[name])
            row[name] = {"us_median": round(med, 2), "us_all": [round(x, 2) for x in t[name]],
                         "frac": round(nbytes / med / 8e6, 4)}
        row["builtin_over_asm"] = round(row["builtin"]["us_median"] / row["asm"]["us_median"], 4)
        res[cname] = row
        print(cname, json.dumps(row), flush=True)
        del launch, outs
        torch.cuda.empty_cache()
    out = sys.argv[1] if len(sys.argv) > 1 else None
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
