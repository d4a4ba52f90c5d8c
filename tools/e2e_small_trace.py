#!/usr/bin/env python3
"""Measurement tool (not product): one small-burst host-path mode in a loop, for a rocprofv3
timeline of where a call's time goes (copies, kernel, gaps).
  rocprofv3 --kernel-trace --memory-copy-trace -d <dir> -o t -- python3 tools/e2e_small_trace.py 16384 pinned_patch
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
mode = sys.argv[2] if len(sys.argv) > 2 else "pinned_patch"
eng = nf.Engine(0)
d_arena, nbytes, d_desc, hdesc = eng.config_batch(1, 20250620, 0, n)
src = d_arena.download(np.uint8, nbytes)
arena = eng.host_array(nbytes) if mode.startswith("pinned") else np.empty(nbytes, dtype=np.uint8)
arena[:] = src
kw = dict(want_status=False, mode=mode.split("_", 1)[1])
for _ in range(5):
    eng.update_host(arena, hdesc, **kw)
ts = []
for _ in range(50):
    t0 = time.perf_counter()
    eng.update_host(arena, hdesc, **kw)
    ts.append(time.perf_counter() - t0)
print(f"{mode} n={n}: min {min(ts) * 1e6:.1f} us, median {sorted(ts)[25] * 1e6:.1f} us per call")
if mode.startswith("pinned"):
    eng.host_free(arena)
eng.close()
