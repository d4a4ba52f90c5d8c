"""ab.py — measurement tool (not product): A/B of the launch forms in tools/exp/nfcs_exp.hip.

For each (workload, variant): kernel time per launch by HIP events over --iters launches after a
0.5 s warm-up, on the engine's stream, then parity: the variant applied once to a freshly generated
batch, whole-arena digest against the reference's (tests/golden/configs.json) where one exists.
`--fresh R` rotates the launches over R separately generated batches of the same shape (so no
launch re-processes what the previous one just wrote, as on a NIC ring); default 1 = the same
batch every launch (bench.py's replay). One JSON line per run.
  python tools/exp/ab.py --variants 0,1,4 --work c1,c4shard,c3 [--fresh 4] [--lds 0]
Work "c<k>n<N>": the first N packets of config k (burst-size sweeps). Work "u<L>": 1M IPv4+UDP frames all of length L (128-byte aligned), built here with numpy (no
reference digest: parity is every variant's output digest equal to variant 0's on the same input).
"""
import argparse
import ctypes

import numpy as np
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
os.environ.setdefault("NFCS_LIB", os.path.join(HERE, "libnfcs_exp.so"))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402

SEED = 20250620
WORK = {"c1": (1, 1 << 20), "c2": (2, 1 << 20), "c3": (3, 1 << 22), "c4shard": (1, 1 << 22),
        "c1half": (1, 1 << 19)}


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
    ap.add_argument("--variants", default="0")
    ap.add_argument("--work", default="c1")
    ap.add_argument("--fresh", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lds", type=int, default=0)
    args = ap.parse_args()
    L = nf.lib()
    fn = L.nfcs_exp_time_update
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                   ctypes.c_void_p, ctypes.c_uint, ctypes.c_int, ctypes.c_void_p,
                   ctypes.POINTER(ctypes.c_float)]
    eng = nf.Engine(0)
    for w in args.work.split(","):
        if w.startswith("u"):
            uniform(eng, int(w[1:]), args, fn)
            continue
        if w == "imix":  # simple IMIX: 64 / 570 / 1500-byte frames in the ratio 7:4:1
            lens = np.random.default_rng(7).choice([64, 570, 1500], size=1 << 20, p=[7 / 12, 4 / 12, 1 / 12])
            uniform(eng, lens, args, fn)
            continue
        if w[0] == "c" and "n" in w[1:] and w[1:w.index("n", 1)].isdigit():  # c<k>n<N>: N packets of Ck
            cfg, n = int(w[1:w.index("n", 1)]), int(w[w.index("n", 1) + 1:])
        else:
            cfg, n = WORK[w]
        bs = [eng.config_batch(cfg, SEED, 0, n, 128) for _ in range(args.fresh)]
        ws = eng.alloc(8 * n)
        hd = bs[0][3]
        algo = float(hd["len"].astype("f8").sum()) + 12.0 * n
        for v in [int(x) for x in args.variants.split(",")]:
            ms = ctypes.c_float()

            def run(k, iters):
                a, nb, d, _ = bs[k % len(bs)]
                rc = fn(v, a.ptr, nb, d.ptr, n, ws.ptr, args.lds, iters, eng.stream, ctypes.byref(ms))
                if rc:
                    raise SystemExit(f"variant {v}: hip error {rc}")
                return ms.value
            t0 = time.perf_counter()
            k = 0
            while time.perf_counter() - t0 < 0.5:
                run(k, 1)
                k += 1
            tot = 0.0
            for i in range(args.iters):
                tot += run(k + i, 1)
            per = tot / args.iters
            # parity on a fresh batch
            a, nb, d, _ = bs[0]
            eng.gen_config_device(cfg, SEED, 0, n, a, nb, d)
            eng.sync()
            run(0, 1)
            got = f"{eng.digest_device(a, nb, d, n, 0):016x}"
            want = golden(cfg, 0, n)
            print(json.dumps({"work": w, "variant": v, "fresh": args.fresh, "lds": args.lds,
                              "kernel_ms": round(per, 4), "frac": round(algo / (per * 1e-3) / 8e12, 4),
                              "parity": None if want is None else got == want}), flush=True)
        for b in bs:
            b[0].free()
            b[2].free()
        ws.free()
    eng.close()


def uniform(eng, L, args, fn, n=1 << 20):
    """1M IPv4+UDP frames of length L (an int, or one length per frame): random bytes, then the
    header fields of DESIGN.md §6; 128-byte aligned slots."""
    import numpy as np
    lens = np.full(n, L, dtype=np.int64) if np.isscalar(L) else np.asarray(L, dtype=np.int64)
    n = len(lens)
    slots = (lens + 127) // 128 * 128
    starts = np.concatenate([[0], np.cumsum(slots)[:-1]])
    rng = np.random.default_rng(int(lens[0]) * 7 + n)
    host = rng.integers(0, 256, size=int(slots.sum()), dtype=np.uint8)
    tail = np.arange(int(slots.max()))
    for Lv in np.unique(lens):  # zero each slot's bytes past its frame
        idx = np.nonzero(lens == Lv)[0]
        pad = tail[int(Lv):int((Lv + 127) // 128 * 128)]
        if len(pad):
            host[(starts[idx][:, None] + pad[None, :]).ravel()] = 0
    def put(o, v):
        host[starts + o] = v
    put(12, 0x08); put(13, 0x00); put(14, 0x45); put(15, 0x00)
    put(16, (lens - 14) >> 8); put(17, (lens - 14) & 0xFF)
    put(22, 64); put(23, 17)
    host[starts + 24] |= 1
    put(38, (lens - 34) >> 8); put(39, (lens - 34) & 0xFF)
    desc = np.zeros(n, dtype=nf.DESC_DTYPE)
    desc["off16"] = (starts // 16).astype(np.uint32)
    desc["len"] = lens.astype(np.uint32)
    arenas = [eng.alloc(host.nbytes).upload(host) for _ in range(args.fresh)]
    d_desc = eng.alloc(desc.nbytes).upload(desc)
    ws = eng.alloc(8 * n)
    algo = float(lens.sum()) + 12.0 * n
    L = "imix" if not np.isscalar(L) else L
    ms = ctypes.c_float()
    ref = None
    for v in [int(x) for x in args.variants.split(",")]:
        def run(k):
            a = arenas[k % len(arenas)]
            if fn(v, a.ptr, host.nbytes, d_desc.ptr, n, ws.ptr, args.lds, 1, eng.stream, ctypes.byref(ms)):
                raise SystemExit(f"variant {v} failed")
            return ms.value
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 0.5:
            run(k)
            k += 1
        per = sum(run(k + i) for i in range(args.iters)) / args.iters
        arenas[0].upload(host)
        run(0)
        got = eng.digest_device(arenas[0], host.nbytes, d_desc, n, 0)
        ref = got if ref is None else ref
        print(json.dumps({"work": f"u{L}", "variant": v, "fresh": args.fresh, "lds": args.lds,
                          "kernel_ms": round(per, 4), "frac": round(algo / (per * 1e-3) / 8e12, 4),
                          "parity": got == ref}), flush=True)
    for a in arenas:
        a.free()
    d_desc.free()
    ws.free()


if __name__ == "__main__":
    main()
