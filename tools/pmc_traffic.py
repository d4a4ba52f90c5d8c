#!/usr/bin/env python3
"""HBM traffic per launch of the checksum kernel from rocprofv3 PMC counters.

Runs bench.py under rocprofv3 twice per config — one pass with FETCH_SIZE, one with
WRITE_SIZE (they do not fit one TCC pass on gfx950; counters are never combined with
sys/runtime tracing) — and applies the MI355X_MICROARCH.md HBM correction: on gfx950
FETCH_SIZE reports exactly half of the bytes of a wide (16 B/lane) coalesced streaming read,
so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE (KB) is taken as is.

  python3 tools/pmc_traffic.py --out gpurun_out/pmc --configs 1 2 3
writes <out>/traffic.json: {"C1": {"fetch_bytes": .., "write_bytes": .., "hbm_bytes": ..,
"per_packet": .., "launches": ..}, ...}; copy it to profiles/traffic.json to have bench.py
report it as roofline.traffic.
"""
import argparse
import csv
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PACKETS = {0: 1024, 1: 1 << 20, 2: 1 << 20, 3: 1 << 22}


def run_pass(out, cfg, counter, steps):
    d = os.path.join(out, f"c{cfg}_{counter}")
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", d,
           "-o", "p", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--config", str(cfg),
           "--steps", str(steps), "--warmup", "1", "--no-cpu"]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise SystemExit(f"rocprofv3 failed ({r.returncode}): {r.stderr[-2000:]}")
    vals = []
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for row in csv.DictReader(open(os.path.join(root, f))):
                    if "update_rows_kernel" in row["Kernel_Name"] and row["Counter_Name"] == counter:
                        vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} samples for the update kernel in {d}")
    return statistics.median(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    ap.add_argument("--configs", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, --kernel-trace; "
                     "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 correction), write = WRITE_SIZE x 1024; "
                     "median over launches of bench.py"}
    for cfg in a.configs:
        f, nf_ = run_pass(a.out, cfg, "FETCH_SIZE", a.steps)
        w, nw = run_pass(a.out, cfg, "WRITE_SIZE", a.steps)
        fb, wb = 2 * f * 1024, w * 1024
        res[f"C{cfg}"] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                          "per_packet": (fb + wb) / PACKETS[cfg], "launches": min(nf_, nw)}
        print(f"C{cfg}: read {fb / 1e9:.3f} GB  write {wb / 1e6:.1f} MB per launch", flush=True)
    with open(os.path.join(a.out, "traffic.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
