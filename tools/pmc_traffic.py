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


# the kernels of one call of the op: nfcs_update_device is the read pass and, for waves of long
# frames, the write pass (apply_bytes_kernel); per call = the sum of the per-kernel medians
KERNEL = {"update": ("update_rows_kernel", "apply_bytes_kernel"), "l3fwd": ("update_rows_kernel", "apply_fwd_kernel"),
          "vlan": ("vlan_rows_kernel",), "flowkey": ("flow_keys_lanes_kernel",)}


def threads_per_packet(kernel_name: str) -> int:
    """Work items per packet of a dispatch of one of the op's kernels, from its template arguments:
    update_rows_kernel<K, R, ...> and vlan_rows_kernel<K, K2, POL, R, ...> run an R-lane row per
    packet; the write passes and the flow-key kernel one lane per packet."""
    if "update_rows_kernel<" in kernel_name:
        return int(kernel_name.split("update_rows_kernel<", 1)[1].split(",")[1])
    if "vlan_rows_kernel<" in kernel_name:
        return int(kernel_name.split("vlan_rows_kernel<", 1)[1].split(",")[3])
    return 1


def run_pass(out, cfg, counters, steps, op="update", packets=0, align=128):
    """One rocprofv3 pass with the given counters; per counter, the sum over the op's kernels of the
    median over that kernel's dispatches of the counter per packet the dispatch covers (its grid size
    / work items per packet), times the call's packets. A call that runs as several sub-batches
    (nfcs_update_device above 512K long frames, the forward's deferred bursts) is so counted whole
    from the dispatches the trace holds, whatever the thresholds (the number of sub-batches
    is no longer predicted here)."""
    d = os.path.join(out, f"c{cfg}{'_' + str(packets) if packets else ''}_a{align}_{op}_{counters[0]}")
    cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc", *counters, "--kernel-trace", "--output-format", "csv", "-d", d,
           "-o", "p", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--config", str(cfg),
           "--steps", str(steps), "--warmup", "1", "--warm-seconds", "0", "--no-cpu", "--no-replay", "--no-host", "--no-c4", "--op", op, "--align", str(align)] + (["--packets", str(packets)] if packets else [])
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise SystemExit(f"rocprofv3 failed ({r.returncode}): {r.stderr[-2000:]}")
    n = packets or PACKETS[cfg]
    vals = {(k, c): [] for k in KERNEL[op] for c in counters}
    covered = {k: 0.0 for k in KERNEL[op]}
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for row in csv.DictReader(open(os.path.join(root, f))):
                    for k in KERNEL[op]:
                        if k in row["Kernel_Name"] and (k, row["Counter_Name"]) in vals:
                            pk = int(row["Grid_Size"]) / threads_per_packet(row["Kernel_Name"])
                            vals[(k, row["Counter_Name"])].append(float(row["Counter_Value"]) / pk)
                            if row["Counter_Name"] == counters[0]:
                                covered[k] += pk
    if not vals[(KERNEL[op][0], counters[0])]:
        raise SystemExit(f"no {counters[0]} samples for {KERNEL[op][0]} in {d}")
    med = {c: sum(statistics.median(vals[(k, c)]) * n for k in KERNEL[op] if vals[(k, c)]) for c in counters}
    # launches per call: the read-pass dispatches over the packets they covered, per n packets
    per_call = len(vals[(KERNEL[op][0], counters[0])]) * n / covered[KERNEL[op][0]]
    return med, len(vals[(KERNEL[op][0], counters[0])]), per_call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    ap.add_argument("--configs", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--ops", nargs="+", default=["update"], choices=list(KERNEL))
    ap.add_argument("--merge", help="existing traffic.json to extend")
    ap.add_argument("--packets", type=int, default=0,
                    help="packets per launch instead of the config's (C1 with 4194304 = the C4 shard)")
    ap.add_argument("--align", type=int, default=128, help="frame start alignment (bench.py --align)")
    a = ap.parse_args()
    a.out = os.path.abspath(a.out)  # rocprofv3 runs with cwd /tmp
    os.makedirs(a.out, exist_ok=True)
    res = {"method": "rocprofv3 --pmc, --kernel-trace only, separate passes; read bytes = "
                     "2 x FETCH_SIZE x 1024 (gfx950 correction), write = WRITE_SIZE x 1024; "
                     "cross-check: TCC_EA0_RDREQ x 128 B (gfx950 read requests are whole 128-B "
                     "lines; the stock 64-B expression under-counts by the same factor 2), "
                     "EA0_WRREQ(_64B) write requests; median over launches of bench.py"}
    if a.merge:
        res = json.load(open(a.merge))
    for cfg, op in [(c, o) for o in a.ops for c in a.configs]:
        P = a.packets
        f, nf_, sub = run_pass(a.out, cfg, ["FETCH_SIZE"], a.steps, op, P, a.align)
        w, nw, _ = run_pass(a.out, cfg, ["WRITE_SIZE"], a.steps, op, P, a.align)
        q, _, _ = run_pass(a.out, cfg, ["TCC_BUBBLE_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"],
                           a.steps, op, P, a.align)
        wq, _, _ = run_pass(a.out, cfg, ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"], a.steps, op, P, a.align)
        key = ("C4_shard" if (cfg == 1 and P == 1 << 22) else f"C{cfg}" + (f"_{P}" if P else "")) + \
            ("" if op == "update" else f"_{op}") + ("" if a.align == 128 else f"_align{a.align}")
        fb, wb = 2 * f["FETCH_SIZE"] * 1024, w["WRITE_SIZE"] * 1024
        rq = q["TCC_EA0_RDREQ_sum"]
        rb_req = rq * 128
        res[key] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                          "per_packet": (fb + wb) / (P or PACKETS[cfg]), "launches": min(nf_, nw),
                    "launches_per_call": round(sub, 3),
                          "read_bytes_from_requests": rb_req, "read_requests": rq,
                          "write_requests": wq["TCC_EA0_WRREQ_sum"],
                          "write_requests_64B": wq["TCC_EA0_WRREQ_64B_sum"]}
        print(f"{key} {op}: read {fb / 1e9:.3f} GB (requests: {rb_req / 1e9:.3f} GB)  write "
              f"{wb / 1e6:.1f} MB in {wq['TCC_EA0_WRREQ_sum']:.0f} requests per call", flush=True)
    with open(os.path.join(a.out, "traffic.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
