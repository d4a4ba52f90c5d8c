#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rate of the host-memory path, nfcs_update_host.

Frames start and end in host memory (NIC/socket buffers): the engine stages them through its
pinned ring (H2D copy, kernel, D2H copy, overlapped on two streams). Measures, for config C1:
  * pageable host arena, whole frames copied back;
  * pageable host arena, only 8-byte patch records copied back and applied on the host;
  * pinned host arena (nfcs_host_alloc), staged, whole frames / patch records copied back;
  * pinned host arena, zero-copy (the kernel reads the frames over PCIe in place).
Every mode's result must equal the reference's (C1 digest, tests/golden/configs.json).
Prints one JSON object per mode (GB/s of frame bytes, host wall clock).
  python3 tools/e2e_host.py [--packets 1024 16384 1048576] [--reps 5]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402


def result_digest(eng, arena, d_desc, n):
    """Order-independent digest of the updated frames (nfcs_digest_device on a device copy),
    compared with the reference's C1 digest (tests/golden/configs.json)."""
    d = eng.alloc(arena.nbytes).upload(arena)
    g = eng.digest_device(d, arena.nbytes, d_desc, n, 0)
    d.free()
    return g


def main(n=1 << 20, reps=5):
    eng = nf.Engine(0)
    d_arena, nbytes, d_desc, hdesc = eng.config_batch(1, 20250620, 0, n)
    src = d_arena.download(np.uint8, nbytes)
    frame_bytes = float(hdesc["len"].astype(np.float64).sum())
    out = []
    if n == 1 << 20:
        want = int(json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
                   ["configs"]["1"]["digest_out"], 16)
    else:  # a burst of another size: the device path's result (itself checked by the GPU tests)
        eng.update_device(d_arena, nbytes, d_desc, n)
        eng.sync()
        want = eng.digest_device(d_arena, nbytes, d_desc, n, 0)
    pinned = eng.host_array(nbytes)
    node, local = eng.host_numa()
    print(json.dumps({"gpu_numa_node": node, "staging_bound_to_node": local}), flush=True)
    for mode in ("pageable_frames", "pageable_patch", "pinned_frames", "pinned_patch", "pinned_zero_copy"):
        arena = pinned if mode.startswith("pinned") else np.empty(nbytes, dtype=np.uint8)
        kw = dict(want_status=False, mode=mode.split("_", 1)[1])
        arena[:] = src
        eng.update_host(arena, hdesc, **kw)  # warm
        assert result_digest(eng, arena, d_desc, n) == want, mode
        ts = []
        for _ in range(reps):
            arena[:] = src
            t0 = time.perf_counter()
            eng.update_host(arena, hdesc, **kw)
            ts.append(time.perf_counter() - t0)
        assert result_digest(eng, arena, d_desc, n) == want, mode
        t = min(ts)
        r = {"mode": mode, "packets": n, "frame_bytes": frame_bytes, "seconds": t,
             "GBps": frame_bytes / t / 1e9, "digest": f"{want:016x}", "numa_node": node,
             "staging_numa_local": local}
        print(json.dumps(r), flush=True)
        out.append(r)
    eng.host_free(pinned)
    eng.close()
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, nargs="+", default=[1 << 20], help="burst sizes (C1 frames)")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    for p in a.packets:
        main(p, a.reps)
