"""Readers for the committed golden fixtures (format written by gen_golden.py)."""
import json
import os
import struct

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_capture(fname):
    with open(os.path.join(GOLDEN, fname), "rb") as f:
        data = np.load(f)
        (npk,) = struct.unpack("<I", f.read(4))
        pkts = []
        for _ in range(npk):
            (n,) = struct.unpack("<I", f.read(4))
            pkts.append(f.read(n))
    return data, pkts


def manifest(name):
    return json.load(open(os.path.join(GOLDEN, name)))


def ps_cases():
    z = np.load(os.path.join(GOLDEN, "ps_aggregate.npz"))
    names = sorted({k.split("__")[0] for k in z.files})
    return {n: {k.split("__")[1]: z[k] for k in z.files if k.startswith(n + "__")} for n in names}
