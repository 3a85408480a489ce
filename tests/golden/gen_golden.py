"""gen_golden.py -- CONTAINER-ONLY fixture generator (needs /root/reference).

Produces the small golden vectors under tests/golden/ that pin the CPU oracle
to the reference's own code.  The reference never travels to the GPU box; only
the data files written here do.  Nothing from the reference is copied: its
C packetiser is compiled where it lies (oracle/Makefile `ref`) and its Python
modules are imported from /root/reference with the missing/unavailable
dependencies (scapy, torchvision, the absent utils.comm_utils) replaced by
stubs defined in this file.

Fixtures:
  c128_cases.json + c128_<name>.bin  captured bytes of communicator.cc's
      send_gradients (communicator.cc:3-47) driven through the reference's own
      ctypes wrapper (communicator.py:32-39,41-42,133-157), sendto() redirected
      into a file by oracle/capture_shim.c.
  nga_cases.json + nga_<name>.bin    captured datagrams of
      DataManager._send_data (DataManager.py:104-165).  The payload words come
      from a build-supplied float_to_int stub (the reference's is missing), so
      only header/framing/tail-padding/sequence numbering are pinned.
  ps_aggregate.npz                   inputs/outputs of launch.py:42-52 and
      launch_async.py:42-57 aggregate() on small synthetic parameter vectors.

Run:  make -C oracle ref && python tests/golden/gen_golden.py
"""
from __future__ import annotations

import json
import os
import struct
import subprocess
import sys
import tempfile
import textwrap
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("INA_REFERENCE", "/root/reference")
REF_OUT = os.path.join(REPO, "oracle", "_ref")


def read_capture(path):
    out = []
    if not os.path.exists(path):
        return out
    raw = open(path, "rb").read()
    off = 0
    while off < len(raw):
        (n,) = struct.unpack_from("<I", raw, off)
        out.append(raw[off + 4: off + 4 + n])
        off += 4 + n
    return out


# ---------------------------------------------------------------------------
# C-128: communicator.cc via communicator.py
# ---------------------------------------------------------------------------
C128_DRIVER = textwrap.dedent(r"""
    import os, sys, json
    import numpy as np
    sys.path.insert(0, os.environ["REF_COMMON"])
    import communicator as cm          # loads ./send.so (communicator.py:15)
    case = json.loads(os.environ["CASE"])
    rng = np.random.default_rng(case["seed"])
    data = rng.integers(0, 2**32, size=case["n"], dtype=np.uint64).astype(np.uint32)
    np.save(os.environ["DATA_OUT"], data)
    kind = case["kind"]
    if kind == "wrapper":
        cm.c_send_wrapper(data, case["packet_num"], cm.ip2int("10.0.0.2"), case["worker_id"],
                          case["aggregator_index"], case["tensor_index"])
    elif kind == "single":
        cm.single_process_send(data)
    elif kind == "threads":
        try:
            cm.multi_thread_send_threading(case["threads"], data)
        except NameError as e:          # communicator.py:157 data_size is undefined
            print("NameError:", e)
""")

C128_CASES = [
    dict(name="w3_agg7_t10", kind="wrapper", n=3 * 128, packet_num=3, worker_id=3,
         aggregator_index=7, tensor_index=10, seed=11),
    dict(name="w1_agg0_t0", kind="wrapper", n=2 * 128, packet_num=2, worker_id=1,
         aggregator_index=0, tensor_index=0, seed=12),
    dict(name="w32_aggmax", kind="wrapper", n=128, packet_num=1, worker_id=32,
         aggregator_index=0xFFFFFFFF, tensor_index=-5, seed=13),
    dict(name="w0_ub_shift", kind="wrapper", n=128, packet_num=1, worker_id=0,
         aggregator_index=199665, tensor_index=1, seed=14),
    dict(name="single_300_tail_dropped", kind="single", n=300, seed=15),
    dict(name="threads3_1000", kind="threads", n=1000, threads=3, seed=16),
]


def gen_c128():
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True,
                   stdout=subprocess.DEVNULL)
    manifest = []
    for case in C128_CASES:
        with tempfile.TemporaryDirectory() as td:
            cap = os.path.join(td, "cap.bin")
            dat = os.path.join(td, "data.npy")
            env = dict(os.environ)
            pre = os.path.join(REF_OUT, "libcapture.so")
            env["LD_PRELOAD"] = (pre + " " + env["LD_PRELOAD"]).strip() if env.get("LD_PRELOAD") else pre
            env.update(INA_CAPTURE_FILE=cap, CASE=json.dumps(case), DATA_OUT=dat,
                       REF_COMMON=os.path.join(REF, "src", "common"))
            r = subprocess.run([sys.executable, "-c", C128_DRIVER], cwd=REF_OUT, env=env,
                               capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"c128 case {case['name']} failed:\n{r.stderr}")
            pkts = read_capture(cap)
            data = np.load(dat)
        blob = b"".join(pkts)
        fname = f"c128_{case['name']}.bin"
        with open(os.path.join(HERE, fname), "wb") as f:
            np.save(f, data)
            f.write(struct.pack("<I", len(pkts)))
            for p in pkts:
                f.write(struct.pack("<I", len(p)))
                f.write(p)
        manifest.append(dict(case, file=fname, packets=len(pkts),
                             packet_bytes=sorted({len(p) for p in pkts}),
                             stdout=r.stdout.strip().splitlines()[-1:] if r.stdout else []))
        print(f"c128 {case['name']}: {len(pkts)} packets, {len(blob)} B")
    json.dump(manifest, open(os.path.join(HERE, "c128_cases.json"), "w"), indent=1)


# ---------------------------------------------------------------------------
# NGA-32: DataManager._send_data with stubbed scapy / comm_utils / socket
# ---------------------------------------------------------------------------
class _CaptureSocket:
    sent: list = []

    def __init__(self, *a):
        self.args = a

    def sendto(self, data, addr):
        _CaptureSocket.sent.append(bytes(data))
        return len(data)


def _float_to_int_stub(data):
    """Build-supplied stand-in for the missing utils.comm_utils.float_to_int:
    q = sat32(rne(x * 2^16)), each as 4 big-endian bytes (what `nga += d`
    at DataManager.py:131-133 concatenates)."""
    x = np.asarray(data, np.float32)
    y = np.rint(x.astype(np.float64) * 65536.0)
    y = np.clip(y, -2**31, 2**31 - 1).astype(np.int64)
    return [int(v).to_bytes(4, "big", signed=True) for v in y]


def _install_dm_stubs():
    sockmod = types.SimpleNamespace(socket=_CaptureSocket, AF_INET=2, SOCK_RAW=3)
    scapy_all = types.ModuleType("scapy.all")
    scapy_all.socket = sockmod
    scapy_all.get_if_list = lambda: ["eth0"]
    scapy_all.sys = sys
    scapy_all.__all__ = ["socket", "get_if_list", "sys"]
    for name in ("scapy", "scapy.layers", "scapy.layers.inet", "scapy.layers.l2"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["scapy.all"] = scapy_all
    sys.modules["scapy.layers.inet"].IP = object
    sys.modules["scapy.layers.l2"].Ether = object
    utils = types.ModuleType("utils")
    utils.__path__ = []
    ngapkt = types.ModuleType("utils.NGAPacket")
    ngapkt.NGA_TYPE, ngapkt.DATA_NUM = 0x12, 32
    ngapkt.__all__ = ["NGA_TYPE", "DATA_NUM"]
    cu = types.ModuleType("utils.comm_utils")
    cu.float_to_int = _float_to_int_stub
    cu.int_to_float = lambda d: d
    sys.modules.update({"utils": utils, "utils.NGAPacket": ngapkt, "utils.comm_utils": cu})


NGA_CASES = [  # (name, n, entry, worker_id, switch_id, degree)
    ("send_n1", 1, "send_data", 3, 1, 2),
    ("send_n31", 31, "send_data", 1, 1, 2),
    ("send_n32", 32, "send_data", 2, 1, 4),
    ("send_n33", 33, "send_data", 4, 7, 8),
    ("send_n64", 64, "send_data", 5, 1, 16),
    ("send_n70", 70, "send_data", 6, 2, 3),
    ("send_n300", 300, "send_data", 7, 1, 127),
    ("fast_n70", 70, "fast_send_data", 9, 3, 5),
    ("fast_n96", 96, "fast_send_data", 1, 1, 2),
    ("send_end_marker_n40", 40, "_send_data_end", 2, 1, 2),
    ("send_negdeg_n8", 8, "send_data", 0xFFFFFFFF, 127, -1),
]


def gen_nga():
    _install_dm_stubs()
    sys.path.insert(0, os.path.join(REF, "src", "common"))
    import DataManager as dm   # noqa: E402  (reference module, imported from /root/reference)
    manifest = []
    rng = np.random.default_rng(2024)
    for name, n, entry, wid, sw, deg in NGA_CASES:
        x = (rng.standard_normal(n) * 0.5).astype(np.float32)
        m = dm.DataManager("10.0.0.1", "10.0.0.2", data=x, interface="eth0", thread_num=1)
        _CaptureSocket.sent = []
        if entry == "send_data":
            m.send_data(wid, sw, deg)
        elif entry == "fast_send_data":
            m.fast_send_data(wid, sw, deg)
        else:   # the end marker path send_data never reaches (DataManager.py:106,155-164)
            m._send_data(wid, sw, deg, 0, len(m.data), 5, True)
        pkts = list(_CaptureSocket.sent)
        q = np.array([int.from_bytes(b, "big", signed=True) for b in m.data], np.int32)
        fname = f"nga_{name}.bin"
        with open(os.path.join(HERE, fname), "wb") as f:
            np.save(f, q)
            f.write(struct.pack("<I", len(pkts)))
            for p in pkts:
                f.write(struct.pack("<I", len(p)))
                f.write(p)
        manifest.append(dict(name=name, n=n, entry=entry, worker_id=wid, switch_id=sw,
                             degree=deg, file=fname, packets=len(pkts),
                             packet_bytes=[len(p) for p in pkts]))
        print(f"nga {name}: {len(pkts)} packets {[len(p) for p in pkts][:4]}")
    json.dump(manifest, open(os.path.join(HERE, "nga_cases.json"), "w"), indent=1)


# ---------------------------------------------------------------------------
# PS combine: launch.py / launch_async.py aggregate()
# ---------------------------------------------------------------------------
PS_DRIVER = textwrap.dedent(r"""
    import os, sys, types
    import numpy as np
    import torch
    for name in ("torchvision", "torchvision.datasets", "torchvision.transforms",
                 "torchvision.models"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["torchvision"].datasets = sys.modules["torchvision.datasets"]
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.modules["torchvision"].models = sys.modules["torchvision.models"]
    sys.path.insert(0, os.environ["REF_DT"])
    sys.argv = ["launch.py", "--master", "1"]
    import importlib
    mod = importlib.import_module(os.environ["MODULE"])
    rng = np.random.default_rng(int(os.environ["SEED"]))
    W, n = int(os.environ["W"]), int(os.environ["N"])
    step = float(os.environ["STEP"])
    K = os.environ.get("K")

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Parameter(torch.zeros(n // 2))
            self.b = torch.nn.Parameter(torch.zeros(n - n // 2))
    model = M()
    local = rng.standard_normal(n).astype(np.float32)
    local[:4] = [0.0, -0.0, 1e-30, -3.5]
    torch.nn.utils.vector_to_parameters(torch.from_numpy(local.copy()), model.parameters())
    paras = []
    class Wk: pass
    wl = []
    for w in range(W):
        p = (local + rng.standard_normal(n).astype(np.float32) * 0.01).astype(np.float32)
        p[1] = -0.0 if w % 2 else 0.0
        paras.append(p)
        o = Wk(); o.updated_paras = torch.from_numpy(p.copy()); wl.append(o)
    with torch.no_grad():
        if K is None:
            mod.aggregate(model, wl, step)
        else:
            mod.aggregate(model, wl, step, int(K))
    out = torch.nn.utils.parameters_to_vector(model.parameters()).detach().numpy()
    np.savez(os.environ["OUT"], local=local, paras=np.stack(paras), out=out,
             step=np.float64(step), W=W, K=-1 if K is None else int(K))
""")

PS_CASES = [  # (name, module, W, n, step, K)
    ("sync_w2", "launch", 2, 1000, 1.0, None),
    ("sync_w4", "launch", 4, 777, 1.0, None),
    ("sync_w3_step05", "launch", 3, 513, 0.5, None),
    ("async_w5_k3", "launch_async", 5, 600, 1.0, 3),
    ("async_w4_none", "launch_async", 4, 300, 1.0, None),
]


def gen_ps():
    files = {}
    for i, (name, module, W, n, step, K) in enumerate(PS_CASES):
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "o.npz")
            env = dict(os.environ, REF_DT=os.path.join(REF, "src", "distributed_training"),
                       MODULE=module, SEED=str(100 + i), W=str(W), N=str(n), STEP=str(step),
                       OUT=out)
            if K is not None:
                env["K"] = str(K)
            r = subprocess.run([sys.executable, "-c", PS_DRIVER], cwd=td, env=env,
                               capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"ps case {name} failed:\n{r.stderr}")
            z = np.load(out)
            for k in z.files:
                files[f"{name}__{k}"] = z[k]
        print(f"ps {name}: ok")
    np.savez_compressed(os.path.join(HERE, "ps_aggregate.npz"), **files)


if __name__ == "__main__":
    gen_c128()
    gen_nga()
    gen_ps()
