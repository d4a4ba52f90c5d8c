"""c3_forms.py — measurement tool (not product): the C3 write schedules of tools/r05/c3_exp.hip against
the product, calls rotating over 2 separately generated 4M-frame C3 batches (the steady state), HIP
events around --iters back-to-back calls, variants alternating within each round; then each variant
once on a freshly generated batch, digest against the reference's (tests/golden/configs.json).
One JSON line per (variant, round).
  python3 tools/r05/c3_forms.py --variants 0,1,2,3,4,5 --rounds 3
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
os.environ.setdefault("NFCS_LIB", os.path.join(HERE, "libnfcs_c3x.so"))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402

SEED = 20250620


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3,4,5")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    L = nf.lib()
    fn = L.nfcs_r5_c3_time
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
    eng = nf.Engine(0)
    n = 1 << 22
    bs = [eng.config_batch(3, SEED, 0, n, 128) for _ in range(2)]
    ws = eng.alloc(16 << 20)
    algo = float(bs[0][3]["len"].astype("f8").sum()) + 12.0 * n
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))["configs"]["3"]["digest_out"]
    arenas = (ctypes.c_void_p * 2)(*[b[0].ptr for b in bs])
    sizes = (ctypes.c_uint64 * 2)(*[b[1] for b in bs])
    descs = (ctypes.c_void_p * 2)(*[b[2].ptr for b in bs])
    variants = [int(x) for x in a.variants.split(",")]
    ms = ctypes.c_float()

    def timed(v, iters):
        rc = fn(eng.ctx, v, 2, arenas, sizes, descs, n, iters, ws.ptr, ctypes.byref(ms))
        if rc:
            raise SystemExit(f"variant {v}: rc {rc}")
        return ms.value / iters

    timed(0, 60)  # warm the clocks
    for r in range(1, a.rounds + 1):
        for v in variants:
            timed(v, 6)
            t = timed(v, a.iters)
            print(json.dumps({"work": "c3", "variant": v, "round": r, "ms_per_call": round(t, 4),
                              "frac": round(algo / (t * 1e-3) / 1e9 / 8000.0, 4)}), flush=True)
    for v in variants:
        if v == 4:
            continue
        arena, nbytes, desc, _ = bs[0]
        eng.gen_config_device(3, SEED, 0, n, arena, nbytes, desc)
        eng.sync()
        one = (ctypes.c_void_p * 1)(arena.ptr)
        sz = (ctypes.c_uint64 * 1)(nbytes)
        de = (ctypes.c_void_p * 1)(desc.ptr)
        rc = fn(eng.ctx, v, 1, one, sz, de, n, 1, ws.ptr, ctypes.byref(ms))
        got = f"{eng.digest_device(arena, nbytes, desc, n, 0):016x}"
        print(json.dumps({"work": "c3", "variant": v, "parity": got == want, "digest": got, "rc": rc}), flush=True)


if __name__ == "__main__":
    main()
