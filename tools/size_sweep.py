"""size_sweep.py — measurement tool (not product): does the checksum kernel's rate depend on the
batch size, and does cutting a large batch into sub-launches change it?

For C1-shaped batches (1500 B IPv4+UDP, 128-B aligned) of 1M..4M packets it times
`nfcs_update_device` over the whole batch, and over the same batch cut into sub-batches of
`chunk` packets (the descriptor pointer advanced per sub-launch; same arena), on the engine's
stream, wall clock around `iters` back-to-back steps after a 0.5 s warm-up. One JSON line each.
    python tools/size_sweep.py [--sizes 1,2,4] [--chunks 0,262144,1048576]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import netflow_amd as nf  # noqa: E402

SEED = 20250620


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,2,4", help="batch sizes in units of 1M packets")
    ap.add_argument("--chunks", default="0,262144,524288,1048576", help="0 = one launch")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--first-only", action="store_true",
                    help="each step processes only the first sub-batch (same region every step)")
    ap.add_argument("--flush-probe", action="store_true")
    args = ap.parse_args()
    if args.flush_probe:
        return flush_probe()
    eng = nf.Engine(0)
    for m in [int(x) for x in args.sizes.split(",")]:
        n = m << 20
        d_arena, nbytes, d_desc, hdesc = eng.config_batch(args.config, SEED, 0, n, 128)
        fb = float(hdesc["len"].astype("f8").sum())
        for chunk in [int(x) for x in args.chunks.split(",")]:
            if chunk >= n:
                continue
            c = chunk or n

            def step():
                for s in range(0, c if args.first_only else n, c):
                    eng.update_device(d_arena, nbytes, d_desc.ptr + 8 * s, min(c, n - s))
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.5:
                step()
                eng.sync()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                step()
            eng.sync()
            dt = (time.perf_counter() - t0) / args.iters
            if args.first_only:
                fb1 = float(hdesc["len"][:c].astype("f8").sum())
                print(json.dumps({"arena_packets": n, "packets": c, "ms": round(dt * 1e3, 4),
                                  "algo_frac": round((fb1 + 12.0 * c) / dt / 8e12, 4),
                                  "variant": os.environ.get("NFCS_VARIANT", "0")}), flush=True)
                continue
            print(json.dumps({"variant": os.environ.get("NFCS_VARIANT", "0"), "packets": n, "chunk": c, "launches": (n + c - 1) // c,
                              "ms": round(dt * 1e3, 4), "frame_GBps": round(fb / dt / 1e9, 1),
                              "algo_frac": round((fb + 12.0 * n) / dt / 8e12, 4)}), flush=True)
        d_arena.free()
        d_desc.free()




def flush_probe(iters: int = 30, flush_packets: int = 200_000):
    """Is the cross-launch gain (the same region re-processed runs faster than fresh regions)
    held in the Infinity Cache or in the address translations? Between launches over the same
    1M-packet C1 batch, read a separate ~300 MB arena (digest_device: a read-only pass, more
    than the 256 MB Infinity Cache, ~150 translations of 2 MiB). Kernel time by HIP events."""
    eng = nf.Engine(0)
    n = 1 << 20
    d_arena, nbytes, d_desc, hdesc = eng.config_batch(1, SEED, 0, n, 128)
    f_arena, f_bytes, f_desc, _ = eng.config_batch(1, SEED + 1, 0, flush_packets, 128)
    fb = float(hdesc["len"].astype("f8").sum()) + 12.0 * n
    for mode in ("control", "flush", "control"):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            eng.update_device(d_arena, nbytes, d_desc, n)
            eng.sync()
        ms = []
        for _ in range(iters):
            if mode == "flush":
                eng.digest_device(f_arena, f_bytes, f_desc, flush_packets)
            ms.append(eng.time_update_device(d_arena, nbytes, d_desc, n, 1))
        ms.sort()
        med = ms[len(ms) // 2]
        print(json.dumps({"probe": mode, "flush_MB": round(f_bytes / 1e6) if mode == "flush" else 0,
                          "kernel_ms_median": round(med, 4), "algo_frac": round(fb / (med * 1e-3) / 8e12, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
