"""flow_ab.py — measurement tool (not product): launch forms of the flow-key kernel
(nfcs_exp_time_flow in tools/exp/nfcs_exp.hip) on C1 frames, HIP events per launch; parity: every
form's keys and hashes byte-equal to the product's on the same batch.
  python tools/exp/flow_ab.py [--variants 0,1,2] [--packets 1048576]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
os.environ.setdefault("NFCS_LIB", os.path.join(HERE, "libnfcs_exp.so"))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="0,1,2")
ap.add_argument("--packets", type=int, default=1 << 20)
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()
L = nf.lib()
fn = L.nfcs_exp_time_flow
fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
               ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
eng = nf.Engine(0)
n = a.packets
arena, nbytes, desc, hd = eng.config_batch(1, 20250620, 0, n, 128)
keys, hashes = eng.alloc(64 * n), eng.alloc(4 * n)
ms = ctypes.c_float()
ref = None
for v in [int(x) for x in a.variants.split(",")]:
    for _ in range(3):
        assert fn(v, arena.ptr, nbytes, desc.ptr, n, keys.ptr, hashes.ptr, 20, eng.stream, ctypes.byref(ms)) == 0
    assert fn(v, arena.ptr, nbytes, desc.ptr, n, keys.ptr, hashes.ptr, a.iters, eng.stream, ctypes.byref(ms)) == 0
    per = ms.value / a.iters
    out = (keys.download(np.uint8, 64 * n).tobytes(), hashes.download(np.uint8, 4 * n).tobytes())
    ref = out if ref is None else ref
    print(json.dumps({"variant": v, "packets": n, "kernel_us": round(per * 1e3, 2),
                      "Mpkt_per_s": round(n / (per * 1e-3) / 1e6, 1), "parity": out == ref}), flush=True)
eng.close()
