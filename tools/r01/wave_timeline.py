"""Per-wave timeline of the checksum kernel (measurement build only; not product, not a test).

Runs a timeline variant of update_rows_kernel (90/91: 256-/64-thread workgroups; 92/93: the same
without frame stores) once over a BASELINE config and summarises, per wave of 4 packets, the
shader-clock stamps the kernel takes:

  T0 wave start  -> T1 descriptors landed (scalar load)  -> T2 header slot landed (first of 6
  loads) -> T3 all 6 slots landed and summed -> T4 frame stores issued -> T5 stores acknowledged

plus the wave's start on the 100 MHz real-time clock and its XCC / hardware id, from which the
waves resident per CU over time follow.

  NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so python3 tools/wave_timeline.py --config 3 --variant 91
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402

SEED = 20250620
N = {1: 1 << 20, 2: 1 << 20, 3: 1 << 22}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--variant", type=int, default=91)
    ap.add_argument("--warm", type=int, default=20, help="untimed launches of the default kernel first")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    n = N[args.config]
    lib = nf.lib()
    if not hasattr(lib, "nfcs_exp_wave_timeline"):
        raise SystemExit("needs the measurement build: NFCS_LIB=.../libnfcs_exp.so")
    lib.nfcs_exp_wave_timeline.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_void_p]
    waves = (n + 3) // 4
    with nf.Engine(0) as eng:
        d_arena, nbytes, d_desc, _ = eng.config_batch(args.config, SEED, 0, n, 128)
        d_ts = eng.alloc(waves * 64)
        for _ in range(args.warm):
            eng.update_device(d_arena, nbytes, d_desc, n)
        eng.sync()
        rc = lib.nfcs_exp_wave_timeline(eng.ctx, d_arena.ptr, nbytes, d_desc.ptr, n, args.variant,
                                        d_ts.ptr)
        if rc != 0:
            raise SystemExit(f"nfcs_exp_wave_timeline rc={rc}")
        t = d_ts.download(np.uint64).reshape(waves, 8).astype(np.int64)
    d = {
        "desc": t[:, 1] - t[:, 0],
        "first_slot": t[:, 2] - t[:, 1],
        "all_slots": t[:, 3] - t[:, 2],
        "to_stores": t[:, 4] - t[:, 3],
        "store_ack": t[:, 5] - t[:, 4],
        "life": t[:, 5] - t[:, 0],
    }
    rt = t[:, 6]
    span_us = (rt.max() - rt.min()) / 100.0  # wave starts, 100 MHz real-time clock
    res = {"config": args.config, "variant": args.variant, "waves": waves,
           "start_span_us": round(span_us, 1)}
    # shader clock: s_memtime is per CU, so compare it with the real-time clock within one CU
    # (HW_ID bits 8-15: CU, SH, SE; plus the XCC id)
    cu = ((t[:, 7] >> 32) << 8) | ((t[:, 7] >> 8) & 0xFF)
    order = np.argsort(cu, kind="stable")
    cu_s, t0_s, rt_s = cu[order], t[order, 0], rt[order]
    bounds = np.flatnonzero(np.diff(cu_s)) + 1
    rates = []
    for a, b in zip(np.r_[0, bounds], np.r_[bounds, len(cu_s)]):
        if b - a > 50 and rt_s[a:b].max() > rt_s[a:b].min():
            rates.append((t0_s[a:b].max() - t0_s[a:b].min()) / ((rt_s[a:b].max() - rt_s[a:b].min()) / 100e6))
    ghz = float(np.median(rates)) / 1e9 if rates else None
    res["shader_clock_GHz_est"] = round(ghz, 3) if ghz else None
    res["cus_seen"] = int(len(np.unique(cu)))
    for k, v in d.items():
        res[k] = {"mean_cyc": round(float(v.mean()), 1), "p50": int(np.median(v)),
                  "p90": int(np.percentile(v, 90)),
                  "mean_us": round(float(v.mean()) / (ghz * 1e3), 3) if ghz else None}
    if ghz:  # average waves resident = sum of lifetimes / span of the launch
        res["resident_waves_est"] = round(float(d["life"].sum()) / (ghz * 1e3) / span_us, 0)
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
