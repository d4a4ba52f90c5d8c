"""bimodal.py — measurement tool (not product): a 4M-frame mix of 64-byte and 1500-byte IPv4/UDP
frames in random order (`--long-frac` of them long), 128-byte starts, so the checksum kernel runs its
short shape (mean footprint ~830 B) with many groups of 4 averaging >= 1280 B (deferral candidates).
Times nfcs_update_device by HIP events, replayed and over 4 rotating copies (wall clock), with the
library NFCS_LIB names; prints one JSON line with the arena digest after one call (equal across
libraries when both are correct).
  NFCS_LIB=... python3 tools/r03/bimodal.py [--long-frac 0.5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402


def build(n, long_frac, seed):
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(n) < long_frac, 1500, 64).astype(np.uint32)
    slots = (lens.astype(np.uint64) + 127) // 128 * 128
    offs = np.concatenate([[0], np.cumsum(slots)[:-1]]).astype(np.uint64)
    total = int(offs[-1] + slots[-1])
    arena = rng.integers(0, 256, total, dtype=np.uint8)
    o = offs.astype(np.int64)
    arena[o + 12] = 0x08
    arena[o + 13] = 0x00
    arena[o + 14] = 0x45
    arena[o + 15] = 0
    tl = lens - 14
    arena[o + 16] = (tl >> 8).astype(np.uint8)
    arena[o + 17] = (tl & 0xFF).astype(np.uint8)
    arena[o + 22] = 64
    arena[o + 23] = 17
    ul = lens - 34
    arena[o + 38] = (ul >> 8).astype(np.uint8)
    arena[o + 39] = (ul & 0xFF).astype(np.uint8)
    desc = np.zeros(n, dtype=nf.DESC_DTYPE)
    desc["off16"] = (offs // 16).astype(np.uint32)
    desc["len"] = lens
    return arena, desc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--long-frac", type=float, default=0.5)
    ap.add_argument("--packets", type=int, default=1 << 22)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    eng = nf.Engine(0)
    arena, desc = build(a.packets, a.long_frac, 7)
    n = len(desc)
    frame_bytes = float(desc["len"].astype(np.float64).sum())
    algo = frame_bytes + 12.0 * n
    copies = []
    for _ in range(4):
        d_a = eng.alloc(arena.nbytes).upload(arena)
        d_d = eng.alloc(desc.nbytes).upload(desc)
        copies.append((d_a, d_d))
    d_a, d_d = copies[0]
    for _ in range(10):
        eng.update_device(d_a, arena.nbytes, d_d, n)
    eng.sync()
    ev = eng.time_update_device(d_a, arena.nbytes, d_d, n, a.steps) / a.steps
    for k in range(8):
        eng.update_device(copies[k % 4][0], arena.nbytes, copies[k % 4][1], n)
    eng.sync()
    t0 = time.perf_counter()
    for k in range(a.steps):
        eng.update_device(copies[k % 4][0], arena.nbytes, copies[k % 4][1], n)
    eng.sync()
    fresh = (time.perf_counter() - t0) / a.steps
    # digest of one call on a fresh copy of the input
    d_a.upload(arena)
    eng.update_device(d_a, arena.nbytes, d_d, n)
    eng.sync()
    dg = f"{eng.digest_device(d_a, arena.nbytes, d_d, n, 0):016x}"
    print(json.dumps({"lib": os.path.basename(nf.LIB_PATH), "long_frac": a.long_frac, "packets": n,
                      "kernel_ms": round(ev, 4), "frac": round(algo / (ev * 1e-3) / 1e9 / 8000.0, 4),
                      "fresh_ms": round(fresh * 1e3, 4), "fresh_frac": round(algo / fresh / 1e9 / 8000.0, 4),
                      "digest": dg}), flush=True)


if __name__ == "__main__":
    main()
