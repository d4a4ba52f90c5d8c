"""fresh_forms.py — measurement tool (not product): the store forms of tools/r04/fresh_exp.hip on
1500-byte frames, replayed (the same batch every call) and rotated over --batches separately generated
batches (a NIC ring's steady state: no call touches what the previous call wrote), HIP events around
--iters back-to-back calls; then each variant once on a freshly generated batch, digest against the
reference's (tests/golden/configs.json). One JSON line per (work, variant, mode, round).
  python3 tools/r04/fresh_forms.py --variants 0,1,4,7 [--work c1,c4shard] [--rounds 2]
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
os.environ.setdefault("NFCS_LIB", os.path.join(HERE, "libnfcs_r4.so"))
sys.path.insert(0, ROOT)
if "--torch" in sys.argv:  # torch's bundled HIP runtime loaded first, as bench.py does (libnfcs binds to it)
    import torch  # noqa: E402
    torch.cuda.set_device(0)
    torch.cuda.init()
import netflow_amd as nf  # noqa: E402

SEED = 20250620
WORK = {"c1": (1, 1 << 20), "c4shard": (1, 1 << 22), "c2": (2, 1 << 20), "c3": (3, 1 << 22)}


def golden(config, first, n):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
    c = g["configs"].get(str(config))
    if c and c["first"] == first and c["n"] == n:
        return c["digest_out"]
    for sh in g.get("c1_rank_shards", []) + g.get("c4_rank_shards", []):
        if config == 1 and sh["first"] == first and sh["n"] == n:
            return sh["digest_out"]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--work", default="c1")
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--modes", default="replay,rotate")
    ap.add_argument("--torch", action="store_true", help="load torch's HIP runtime first (as bench.py)")
    a = ap.parse_args()
    L = nf.lib()
    fn = L.nfcs_r4_time
    fn.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
    eng = nf.Engine(0)
    variants = [int(x) for x in a.variants.split(",")]
    for w in a.work.split(","):
        cfg, n = WORK[w]
        bs = [eng.config_batch(cfg, SEED, 0, n, 128) for _ in range(a.batches)]
        ws = eng.alloc(8 * (1 << 22) + 64 * n)  # 8-byte records, then SF_REC64's 64-byte ones
        algo = float(bs[0][3]["len"].astype("f8").sum()) + 12.0 * n
        want = golden(cfg, 0, n)

        def run(v, k):
            sel = bs[:k]
            arenas = (ctypes.c_void_p * k)(*[b[0].ptr for b in sel])
            sizes = (ctypes.c_uint64 * k)(*[b[1] for b in sel])
            descs = (ctypes.c_void_p * k)(*[b[2].ptr for b in sel])
            ms = ctypes.c_float()
            rc = fn(v, k, arenas, sizes, descs, n, ws.ptr, a.iters, eng.stream, ctypes.byref(ms))
            if rc:
                raise SystemExit(f"variant {v}: hip error {rc}")
            return ms.value / a.iters

        for v in variants:  # warm every form once
            run(v, a.batches)
        for r in range(a.rounds):
            for v in variants:
                for mode in a.modes.split(","):
                    k = 1 if mode == "replay" else a.batches
                    run(v, k)  # the launch pattern warm
                    t = run(v, k)
                    print(json.dumps({"work": w, "variant": v, "mode": mode, "round": r, "ms": round(t, 4),
                                      "frac": round(algo / (t * 1e-3) / 1e9 / 8000.0, 4)}), flush=True)
        for v in variants:
            arena, nbytes, desc, _ = bs[0]
            eng.gen_config_device(cfg, SEED, 0, n, arena, nbytes, desc)
            eng.sync()
            k1 = (ctypes.c_void_p * 1)(arena.ptr)
            s1 = (ctypes.c_uint64 * 1)(nbytes)
            d1 = (ctypes.c_void_p * 1)(desc.ptr)
            ms = ctypes.c_float()
            if fn(v, 1, k1, s1, d1, n, ws.ptr, 1, eng.stream, ctypes.byref(ms)):
                raise SystemExit("apply failed")
            got = f"{eng.digest_device(arena, nbytes, desc, n, 0):016x}"
            print(json.dumps({"work": w, "variant": v, "parity": got == want, "digest": got, "want": want}), flush=True)
        for b in bs:
            b[0].free()
            b[2].free()
        ws.free()


if __name__ == "__main__":
    main()
