#!/usr/bin/env python3
"""Regenerate the "Measured (MI355X)" column of DESIGN.md's kernel table (§4) from the
committed evidence of one round (INA_EVIDENCE_ROUND, default r02): profiles/<round>/bench.json,
bench_extra.json, kernel_stats_bench.csv, traffic_switch.json, profiles/traffic_sum_reduce_c3.json,
and the driver's own bench line of the previous round (BENCH_r*.json at the repo root).  Static notes (what a row's
history was, lab references) are kept verbatim after the numbers.

usage: design_table.py SESSION_TAG [--check]
"""
import csv
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")
RD = os.environ.get("INA_EVIDENCE_ROUND", "r02")


def driver_bench():
    """(file, avg_launch_us, frac) of the newest driver BENCH_rNN.json, or None."""
    fs = sorted(f for f in os.listdir(REPO) if re.fullmatch(r"BENCH_r\d+\.json", f))
    for f in reversed(fs):
        try:
            rf = json.load(open(os.path.join(REPO, f)))["parsed"]["roofline"]
            return f, rf["avg_launch_us"], rf["frac"]
        except Exception:
            continue
    return None


def load():
    bench = json.load(open(os.path.join(P, RD, "bench.json")))
    extra = {r["kernel"]: r for r in json.load(open(os.path.join(P, RD, "bench_extra.json")))["rows"]}
    sw = json.load(open(os.path.join(P, RD, "traffic_switch.json")))["kernels"]
    tr = json.load(open(os.path.join(P, "traffic_sum_reduce_c3.json")))
    prof_us = None
    for r in csv.DictReader(open(os.path.join(P, RD, "kernel_stats_bench.csv"))):
        if "k_sum_reduce_i32_vec<8, 4, true>" in r["Name"]:
            prof_us = float(r["AverageNs"]) / 1e3
    return bench, extra, sw, tr, prof_us


def fmt(r):
    return f"{r['us']:.1f} µs, {r['GB/s'] / 1e3:.2f} TB/s ({100 * r['frac']:.0f} %)"


def row_cells(tag):
    bench, ex, sw, tr, prof_us = load()
    e = lambda k: ex[k] if k in ex else ex[k.replace("slot sort", "radix sort")]   # noqa: E731 (r01 names)
    rf = bench["roofline"]
    d = driver_bench()
    drv = (f"the driver's {d[0]}: {d[1]:.2f} µs = {100 * d[2]:.1f} %" if d else "no driver bench yet")
    keys = sorted(sw, key=lambda k: -sw[k]["avg_us"])
    run2 = next(k for k in keys if "k_switch_run2" in k)
    kk = next(k for k in keys if "k_switch_keys" in k)
    sort_us = sum(sw[k]["avg_us"] for k in keys if "k_rs_" in k)
    path = e("INA packet path step: 8 x quantise+pack -> switch -> apply -> acks (8 x 100 MiB fp32)")
    small = [r for k, r in ex.items() if k.startswith("switch_process small batch")]
    return {
        "`k_sum_reduce_i32_vec<W=8,U=4>`":
            f"**{rf['avg_launch_us']:.1f} µs, {rf['achieved'] / 1e3:.2f} TB/s = {100 * rf['frac']:.1f} %** "
            f"on the {tag} box (bench.py events; rocprof {prof_us:.1f} µs; {drv}; "
            f"{e('sum_reduce_i32 W=8')['us']:.1f} µs with the cold flush of this "
            f"table); PMC traffic {tr['hbm_bytes_per_launch']:,} B = {tr['traffic_over_algorithmic']:.5f}× "
            f"algorithmic",
        "same, W = 2 / 4 / 16":
            " / ".join(f"{e(f'sum_reduce_i32 W={w}')['GB/s'] / 1e3:.2f}" for w in (2, 4, 16)) + " TB/s ("
            + " / ".join(f"{100 * e(f'sum_reduce_i32 W={w}')['frac']:.0f}" for w in (2, 4, 16)) + " %)",
        "`k_quantize_i32`": fmt(e("quantize_f32_i32")),
        "`k_dequantize_i32`": fmt(e("dequantize_i32_f32")),
        "`k_quant_reduce_i32<4>`": fmt(e("quantize_reduce_f32_i32 W=4 (C2)")),
        "`k_quant_reduce_i16<16>`": fmt(e("quantize_reduce_f32_i16 W=16 V=256 (C4)")),
        "`k_quantize_i16`": fmt(e("quantize_f32_i16_sat V=256 (C4 worker)")),
        "`k_dequantize_i16`": fmt(e("dequantize_i16_f32 (C4 aggregate)")),
        "`k_ps_combine_f32<4>`": fmt(e("ps_combine_f32 W=4")),
        "`k_ps_combine_ina<4>`": fmt(e("ps_combine_ina_f32 W=4")),
        "`k_pack_nga_flat<SrcI32>`": fmt(e("pack_nga V=256")),
        "`k_pack_nga_flat<SrcQ32>`": fmt(e("quantize_pack_nga V=256 ResNet-50 delta (worker side, fused)")),
        "`k_unpack_nga_flat`": fmt(e("unpack_nga V=256")),
        "`k_apply_completed_nga`": fmt(e("apply_completed_nga V=256 (PS side, fused; 102,400 completed of 819,200)")),
        "`k_absmax_f32`": fmt(e("absmax_f32 ResNet-50 delta (dynamic scale)")),
        "`k_pack_c128`": fmt(e("pack_c128 ResNet-50")),
        "`ina_switch_process` (819,200":
            fmt(e("switch_process 8x NGA-256 (819,200 pkts, incl. slot sort; keys from descriptors)"))
            + " with keys from the pack kernels' descriptors ("
            + fmt(e("switch_process 8x NGA-256 (819,200 pkts, incl. slot sort; keys from headers)"))
            + " from the headers)"
            + f" event-timed; under rocprof ({tag}, `profiles/{RD}/traffic_switch.json`) `k_switch_run2` "
              f"{sw[run2]['avg_us']:.1f} µs moving "
              f"{(sw[run2]['hbm_read_bytes'] + sw[run2]['hbm_write_bytes']) / 1e9:.2f} GB at "
              f"{sw[run2]['TB_per_s']:.1f} TB/s, keys {sw[kk]['avg_us']:.1f} µs "
              f"({sw[kk]['hbm_read_bytes'] / 1e6:.1f} MB read), sort passes {sort_us:.1f} µs",
        "`ina_switch_process`, other arrival orders":
            (lambda a, b: f"round-robin over the workers (a NIC's interleave: a slot's packets adjacent) "
                          f"{fmt(a)}; random {fmt(b)}")(
                e("switch_process 8x NGA-256 (819,200 pkts, incl. slot sort; round-robin over workers arrival)"),
                e("switch_process 8x NGA-256 (819,200 pkts, incl. slot sort; random arrival)"))
            if "switch_process 8x NGA-256 (819,200 pkts, incl. slot sort; random arrival)" in ex
            else "(not in this session's bench_extra)",
        "`ina_switch_process`, small batches":
            ", ".join(f"{k.split(': ')[1].split(' NGA')[0]} packets {r['us']:.1f} µs"
                      for k, r in ((r['kernel'], r) for r in small))
            + " (up to 128 packets ONE launch -- sort and run in one workgroup; up to 768 the one-workgroup "
              "sort + run kernel: 2 launches; the bucket sort above -- thresholds from `tools/lab/tiny_lab.py`)",
        "INA packet path step, steady state, PS fused":
            (lambda r: f"{r['us']:.0f} µs per step = {r['aggregated_GBps']:,.0f} GB/s of worker gradients; "
                       f"{r['GB/s'] / 1e3:.1f} TB/s = {100 * r['frac']:.0f} % of peak for the path's bytes")(
                e("INA packet path step, steady state, PS fused into the switch pass"))
            if "INA packet path step, steady state, PS fused into the switch pass" in ex
            else "(not in this session's bench_extra)",
        "INA packet path step, steady state":
            (lambda r: f"{r['us']:.0f} µs per step = {r['aggregated_GBps']:,.0f} GB/s of worker gradients; "
                       f"{r['GB/s'] / 1e3:.1f} TB/s = {100 * r['frac']:.0f} % of peak for the path's bytes")(
                e("INA packet path step, steady state: step t's acks ride in front of step t+1's packets"))
            if "INA packet path step, steady state: step t's acks ride in front of step t+1's packets" in ex
            else "(not in this session's bench_extra)",
        "INA packet path step":
            f"{path['us']:.0f} µs per 8 × 100 MiB = {path['aggregated_GBps']:,.0f} GB/s of worker "
            f"gradients; 4.02 GB / {path['us']:.0f} µs = {path['GB/s'] / 1e3:.1f} TB/s = "
            f"{100 * path['frac']:.0f} % of peak for the path as a whole",
    }


# static notes kept after the generated numbers, by row key
NOTES = {
    "`k_quant_reduce_i16<16>`": " after the split-halves layout (a wave covers 512 values, lane l the 4 at 4l of each half: every load instruction reads 1 KiB contiguous); 8 consecutive values per lane (32-byte lane stride) was 292–305 µs (69–71 %), `profiles/r01/lab/q16_lab.log`",
    "`k_quantize_i16`": "; 30.2 µs before the split layout",
    "`k_dequantize_i16`": ": 4 values per lane (8-byte load, 16-byte store); was one 2-byte value per thread",
    "`k_pack_nga_flat<SrcQ32>`": "; was 80.9 µs (48 %) as a thread-per-chunk kernel that re-read and re-quantised a 5th value per chunk",
    "`k_apply_completed_nga`": "; was 98.6 µs (40 %) as one lane group per packet over every packet",
    "`k_absmax_f32`": " at 256 workgroups; 86 µs at 8192 (one atomicMax per workgroup on one word); a read-before-atomic skip changed nothing at 256 and larger grids stay slower with it (`profiles/r02/lab/absmax_skip_lab.log`)",
    "`k_unpack_nga_flat`": "; the SoA header fields by a thread-per-packet pass inside the kernel (coalesced stores) instead of six narrow stores from each packet's chunk-0 lane: 42.6 -> 39.3 us (`profiles/r02/lab/unpack_hdr_lab.log`); a thread-per-output-chunk variant (unbroken store stream, header chunks skipped by the loads) was 3 % faster without the header fields and 4 % slower with them (`profiles/r01/lab/unpack_out_lab.log`)",
    "`k_pack_c128`": ": 4 wire words per thread with one 16-byte store (4-byte gradient loads, one 32-bit divide by 131), 38.7 -> 35.7 µs against a word per thread (`profiles/r02/lab/c128_lab.log`); round 1's aligned-8-word-window variant was slower, 41.6 µs",
}


def main():
    tag = sys.argv[1]
    path = os.path.join(REPO, "DESIGN.md")
    s = open(path).read()
    head = "| Kernel | Bound | Algorithmic bytes | Measured (MI355X) |"
    i = s.index(head)
    j = s.index("\n\n", i)
    lines = s[i:j].split("\n")
    cells = row_cells(tag)
    out = lines[:2]
    for ln in lines[2:]:
        c = [x.strip() for x in ln.strip().strip("|").split(" | ")]
        key = next((k for k in cells if c[0].startswith(k)), None)
        if key is None:
            raise SystemExit(f"no generator for row {c[0][:50]!r}")
        c[3] = cells[key] + NOTES.get(key, "")
        out.append("| " + " | ".join(c) + " |")
    s2 = s[:i] + "\n".join(out) + s[j:]
    s2 = re.sub(r"`profiles/r\d+/bench_extra\.json` \(session ", f"`profiles/{RD}/bench_extra.json` (session ", s2, 1)
    k = s2.index(f"`profiles/{RD}/bench_extra.json` (session ") + len(f"`profiles/{RD}/bench_extra.json` (session ")
    s2 = s2[:k] + tag + s2[s2.index(",", k):]
    if "--check" in sys.argv:
        print("\n".join(out))
        return
    open(path, "w").write(s2)
    print(f"DESIGN.md table regenerated from {tag}")


if __name__ == "__main__":
    main()
