#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of one csrc source (hipcc's
kernel-resource-usage remarks, gfx950): the check before a GPU A/B that a change did not spill
or cost occupancy.  usage: kernel_resources.py <file.hip> [name filter ...] [-- extra hipcc flags]"""
import re
import subprocess
import sys

CSRC = __file__.rsplit("/", 3)[0] + "/distributed-training-ina_amd/csrc"
KEYS = {"VGPRs": "vgpr", "AGPRs": "agpr", "TotalSGPRs": "sgpr", "ScratchSize [bytes/lane]": "scratch",
        "Occupancy [waves/SIMD]": "waves", "SGPRs Spill": "sspill", "VGPRs Spill": "vspill",
        "LDS Size [bytes/block]": "lds"}


def main():
    argv = sys.argv[1:]
    extra = argv[argv.index("--") + 1:] if "--" in argv else []
    argv = argv[:argv.index("--")] if "--" in argv else argv
    src, filt = argv[0], argv[1:]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-ffp-contract=off",
           "-I../../include", "-I.", *extra, "-c", src, "-o", "/tmp/kernel_resources.o",
           "-Rpass-analysis=kernel-resource-usage"]
    err = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr
    rows, cur = {}, None
    for line in err.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            continue
        m = re.search(r"remark:\s+(.+?): (\d+)", line)
        if m and cur and m.group(1) in KEYS:
            rows.setdefault(cur, {})[KEYS[m.group(1)]] = int(m.group(2))
    for name in sorted(rows):
        if filt and not any(f in name for f in filt):
            continue
        print(name[:72].ljust(72), " ".join(f"{k}={v}" for k, v in rows[name].items()))


if __name__ == "__main__":
    main()
