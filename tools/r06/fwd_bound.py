"""fwd_bound.py — measurement tool (not product): the fused forward's bound on BASELINE C3's mix
(tools/r06/fwd_bound.hip). Calls rotate over 2 separately generated 4M-frame C3
batches (the steady state), HIP events around --iters back-to-back calls, variants alternating within each
round; TTLs are restored (regenerated batches) before every timed forward. Then the product forward once
on each fresh batch, digest against the reference's (tests/golden/configs.json l3fwd_more). One JSON line
per (variant, round).
  python3 tools/r06/fwd_bound.py --variants 0,1,2,3,4,5 --rounds 3 [--align 128]
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
os.environ.setdefault("NFCS_LIB", os.path.join(HERE, "libnfcs_fwdb.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import netflow_amd as nf  # noqa: E402

SEED = 20250620
NAMES = {0: "product forward", 1: "forward pattern, read only", 2: "forward pattern, read + 64-byte segment stores",
         3: "64-byte segment stores alone", 4: "product update", 5: "update's frames_read floor"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3,4,5")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--align", type=int, default=128)
    a = ap.parse_args()
    L = nf.lib()
    fn = L.nfcs_r6_fwd_time
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                   ctypes.POINTER(ctypes.c_float)]
    eng = nf.Engine(0)
    n = 1 << 22
    bs = [eng.config_batch(3, SEED, 0, n, a.align) for _ in range(2)]
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
    table = np.frombuffer(bytes.fromhex(g["l3fwd_c1"]["table"]), dtype=np.uint8).copy()
    d_tab = eng.alloc(table.nbytes).upload(table)
    d_nh = eng.alloc(4 * n).upload((np.arange(n) % 9).astype(np.uint32))
    sink = eng.alloc(4096)
    frames = float(bs[0][3]["len"].astype("f8").sum())
    algo = {0: frames + 37.0 * n, 4: frames + 12.0 * n}
    want = next(x["digest_out"] for x in g["l3fwd_more"] if x["config"] == 3 and x["first"] == 0 and x["n"] == n)
    arenas = (ctypes.c_void_p * 2)(*[b[0].ptr for b in bs])
    sizes = (ctypes.c_uint64 * 2)(*[b[1] for b in bs])
    descs = (ctypes.c_void_p * 2)(*[b[2].ptr for b in bs])
    variants = [int(x) for x in a.variants.split(",")]
    ms = ctypes.c_float()

    def regen():
        for arena, nbytes, desc, _ in bs:
            eng.gen_config_device(3, SEED, 0, n, arena, nbytes, desc)
        eng.sync()

    def timed(v, iters):
        rc = fn(eng.ctx, v, 2, arenas, sizes, descs, n, iters, d_nh.ptr, d_tab.ptr, 8, sink.ptr, ctypes.byref(ms))
        if rc:
            raise SystemExit(f"variant {v}: rc {rc}")
        return ms.value / iters

    timed(4, 60)  # warm the clocks
    for r in range(1, a.rounds + 1):
        for v in variants:
            regen()
            timed(v, 8)
            if v in (0, 3):
                regen()  # fresh TTLs / frames for the timed forward; the write-only probe zeroes headers
            t = timed(v, a.iters)
            row = {"work": "c3_fwd_bound", "align": a.align, "variant": v, "what": NAMES[v], "round": r,
                   "ms_per_call": round(t, 4)}
            if v in algo:
                row["frac"] = round(algo[v] / (t * 1e-3) / 1e9 / 8000.0, 4)
            print(json.dumps(row), flush=True)
    regen()
    got = []
    for arena, nbytes, desc, _ in bs:
        one = (ctypes.c_void_p * 1)(arena.ptr)
        sz = (ctypes.c_uint64 * 1)(nbytes)
        de = (ctypes.c_void_p * 1)(desc.ptr)
        fn(eng.ctx, 0, 1, one, sz, de, n, 1, d_nh.ptr, d_tab.ptr, 8, sink.ptr, ctypes.byref(ms))
        got.append(f"{eng.digest_device(arena, nbytes, desc, n, 0):016x}")
    print(json.dumps({"work": "c3_fwd_bound", "variant": 0, "parity": all(x == want for x in got), "digests": got}),
          flush=True)


if __name__ == "__main__":
    main()
