"""bin_probe.py — measurement tool (not product): what would length-class binning buy on C3?

Splits the C3 batch's descriptors (4M frames of U{64..1500} B) at a length threshold T into a
short and a long list (host side, numpy, order kept), and times the existing launch forms of
tools/exp/nfcs_exp.hip over each list separately and over the whole batch (HIP events, the same
arena). If the two class launches together take much less than the whole-batch launch, a
class-specific kernel for the short list has room to pay; if the long list alone already takes
about as long as the whole batch, binning cannot reach the target.
  python tools/exp/bin_probe.py [--thresholds 256,384,512] [--variants 0,1,2]
"""
import argparse
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
os.environ.setdefault("NFCS_LIB", os.path.join(HERE, "libnfcs_exp.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import netflow_amd as nf  # noqa: E402

SEED = 20250620


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--thresholds", default="256,384,512")
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    L = nf.lib()
    fn = L.nfcs_exp_time_update
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                   ctypes.c_void_p, ctypes.c_uint, ctypes.c_int, ctypes.c_void_p,
                   ctypes.POINTER(ctypes.c_float)]
    eng = nf.Engine(0)
    n = 1 << 22
    a, nb, d, hd = eng.config_batch(3, SEED, 0, n, 128)
    ws = eng.alloc(8 * n)
    ms = ctypes.c_float()

    def time_list(v, dptr, m):
        def run():
            if fn(v, a.ptr, nb, dptr, m, ws.ptr, 0, 1, eng.stream, ctypes.byref(ms)):
                raise SystemExit(f"variant {v} failed")
            return ms.value
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            run()
        return sum(run() for _ in range(args.iters)) / args.iters

    lens = hd["len"].astype(np.int64)
    for v in [int(x) for x in args.variants.split(",")]:
        full = time_list(v, d.ptr, n)
        print(json.dumps({"variant": v, "list": "all", "packets": n, "bytes": int(lens.sum()),
                          "kernel_ms": round(full, 4)}), flush=True)
    for T in [int(x) for x in args.thresholds.split(",")]:
        for name, sel in (("short", lens <= T), ("long", lens > T)):
            sub = np.ascontiguousarray(hd[sel])
            dd = eng.alloc(max(sub.nbytes, 16)).upload(sub)
            for v in [int(x) for x in args.variants.split(",")]:
                t = time_list(v, dd.ptr, len(sub))
                print(json.dumps({"variant": v, "list": name, "T": T, "packets": int(len(sub)),
                                  "bytes": int(lens[sel].sum()), "kernel_ms": round(t, 4)}), flush=True)
            dd.free()
    ws.free()
    a.free()
    d.free()
    eng.close()


if __name__ == "__main__":
    main()
