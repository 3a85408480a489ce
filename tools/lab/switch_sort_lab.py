"""Lab: ina_switch_process on config 3's packet stream (8 workers x 102,400 NGA-256
packets, 2^17-slot pool) per slot-sort variant -- the r01 passes vs the one-sweep sort vs bucket + local,
keys from the packet headers vs from the pack kernel's descriptors, one-sweep tile sizes.
Interleaved rounds, HIP events around each process() call, median per variant; every
variant's actions are checked against the first one's.

  python tools/lab/switch_sort_lab.py [--rounds 5] [--reps 5]
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

VARIANTS = {                      # name: (sort, rounds, use descriptors)
    "r01_hdr": (3, 0, False),
    "r01_desc": (3, 0, True),
    "r01_desc_r4": (3, 4, True),
    "r01_desc_r8": (3, 8, True),
    "os_hdr": (1, 0, False),
    "os_desc": (1, 0, True),
    "os_desc_r4": (1, 4, True),
    "os_desc_r8": (1, 8, True),
    "os_desc_r16": (1, 16, True),
    "hyb_hdr": (2, 0, False),
    "hyb_desc": (2, 0, True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--values", type=int, default=26_214_400)
    ap.add_argument("--only", default="", help="comma-separated variant names (default: all)")
    a = ap.parse_args()
    variants = {k: v for k, v in VARIANTS.items() if not a.only or k in a.only.split(",")}
    n, W, V, slots = a.values, 8, 256, 1 << 17
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1)
    packed = []
    for w in range(W):
        b = torch.randint(-(1 << 20), 1 << 20, (n,), dtype=torch.int32, device=dev, generator=g)
        packed.append(ops.pack_nga(b, V, w + 1, W, 1, 1, num_slots=slots, desc=True))
        del b
    clean = torch.cat([p for p, _ in packed])
    desc = torch.cat([d for _, d in packed])
    del packed
    stream = torch.empty_like(clean)
    sw = ops.Switch(V, num_slots=slots, switch_id=1, device=dev)
    acts = torch.empty(clean.shape[0], dtype=torch.uint8, device=dev)
    times = {k: [] for k in variants}
    ref = None
    s = torch.cuda.current_stream()
    for _ in range(a.rounds):
        for name, (sort, rounds, use_desc) in variants.items():
            ops.set_tuning(switch_sort=sort, switch_sort_rounds=rounds)
            for _ in range(a.reps):
                stream.copy_(clean)
                sw.count.zero_()
                sw.frag.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                sw.process(stream, acts, desc=desc if use_desc else None)
                e1.record(s)
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) * 1e3)
            if ref is None:
                ref = acts.clone()
            elif not torch.equal(acts, ref):
                raise SystemExit(f"{name}: actions differ from the first variant")
    ops.set_tuning(switch_sort=0, switch_sort_rounds=0)
    algo = clean.shape[0] * clean.shape[1] + (n // V) * (clean.shape[1] + 4 * V + 5) + clean.shape[0]
    res = {k: {"median_us": round(statistics.median(v), 1), "min_us": round(min(v), 1),
               "frac": round(algo / (statistics.median(v) * 1e-6) / 8e12, 4)} for k, v in times.items()}
    print(json.dumps({"packets": clean.shape[0], "algorithmic_bytes": algo, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
