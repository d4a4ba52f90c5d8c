"""fresh_probe.py — measurement tool (not product): why a C1 call over a batch the previous call did
not touch (bench.py's `fresh` sub-line) is slower than a replayed one.

Per-call HIP-event times of nfcs_update_device on 1M x 1500 B frames (128-byte starts), median of
`--calls` calls, for: replay (the same batch every call); rotation over K separately allocated
batches (K = 2, 4, 8: TLB reach grows with K, the memory-side cache holds none of them); replay with
a read of a separate `--flush-mb` buffer between calls (evicts the 256 MB memory-side cache, touches
few new pages). One JSON line per mode.
  python3 tools/r03/fresh_probe.py [--calls 30] [--flush-mb 512]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402

SEED = 20250620


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--flush-mb", type=int, default=512)
    a = ap.parse_args()
    eng = nf.Engine(0)
    n = 1 << 20
    batches = [eng.config_batch(1, SEED, 0, n, 128) for _ in range(8)]
    algo = float(batches[0][3]["len"].astype("float64").sum()) + 12.0 * n
    flush = eng.alloc(a.flush_mb << 20)

    def call(k):
        arena, nbytes, desc, _ = batches[k]
        return eng.time_update_device(arena, nbytes, desc, n, 1)

    for _ in range(20):  # warm
        call(0)
    modes = [("replay", 1, False), ("rotate", 2, False), ("rotate", 4, False), ("rotate", 8, False),
             ("replay_flush", 1, True), ("rotate_flush", 8, True)]
    for name, k, fl in modes:
        ts = []
        for i in range(a.calls + k):
            if fl:
                eng.time_stream_read(flush, a.flush_mb << 20, 1, form=5)
            t = call(i % k)
            if i >= k:  # every batch touched once before timing
                ts.append(t)
        med = statistics.median(ts)
        print(json.dumps({"mode": name, "batches": k, "flush_MB": a.flush_mb if fl else 0,
                          "call_ms_median": round(med, 4), "call_ms_min": round(min(ts), 4),
                          "frac": round(algo / (med * 1e-3) / 1e9 / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
