#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rate of the host-memory path, nfcs_update_host.

Frames start and end in host memory (NIC/socket buffers): the engine stages them through its
pinned ring (H2D copy, kernel, D2H copy, overlapped on two streams). Measures, for config C1:
  * pageable host arena, whole frames copied back;
  * pageable host arena, only 8-byte patch records copied back and applied on the host;
  * pinned host arena (nfcs_host_alloc), whole frames copied back.
Prints one JSON object per mode (GB/s of frame bytes, host wall clock).
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


def main(n=1 << 20, reps=5):
    eng = nf.Engine(0)
    d_arena, nbytes, d_desc, hdesc = eng.config_batch(1, 20250620, 0, n)
    src = d_arena.download(np.uint8, nbytes)
    frame_bytes = float(hdesc["len"].astype(np.float64).sum())
    out = []
    for mode in ("pageable_frames", "pageable_patch", "pinned_frames"):
        if mode.startswith("pinned"):
            p = ctypes.c_void_p()
            nf._check(nf.lib().nfcs_host_alloc(eng.ctx, nbytes, ctypes.byref(p)), "host_alloc")
            arena = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))
        else:
            arena = np.empty(nbytes, dtype=np.uint8)
        arena[:] = src
        eng.update_host(arena, hdesc, want_status=False, patch_only=mode.endswith("patch"))  # warm
        ts = []
        for _ in range(reps):
            arena[:] = src
            t0 = time.perf_counter()
            eng.update_host(arena, hdesc, want_status=False, patch_only=mode.endswith("patch"))
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        r = {"mode": mode, "packets": n, "frame_bytes": frame_bytes, "seconds": t,
             "GBps": frame_bytes / t / 1e9}
        print(json.dumps(r), flush=True)
        out.append(r)
    return out


if __name__ == "__main__":
    main()
