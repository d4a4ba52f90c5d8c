"""Shared inputs for the fused L3 forward tests: the fixture frames of
tests/golden/l3fwd_ref.npz are regenerated from the oracle's fuzz generator with the TTL
overrides stored in the fixture (same recipe as tests/golden/make_golden.py:l3_inputs)."""
import os

import numpy as np

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def l3_fixture():
    z = np.load(os.path.join(GOLD, "l3fwd_ref.npz"))
    n = len(z["lens"])
    frames = oracle.fuzz_frames(int(z["seed"]), 0, n)
    out = []
    for i, f in enumerate(frames):
        b = bytearray(f)
        l2 = 18 if len(b) >= 14 and b[12:14] == b"\x81\x00" else 14
        t = int(z["ttl_set"][i])
        if t != 255 and len(b) > l2 + 8:
            b[l2 + 8] = t
        out.append(bytes(b))
    return z, out


def frame_hashes(arena, desc):
    L = oracle.lib()
    return np.array([L.nfo_frame_hash(oracle._ptr(arena[int(d["off16"]) * 16:]), int(d["len"]))
                     for d in desc], dtype=np.uint64)


def random_l3_case(seed: int, n: int, table_n: int = 8):
    """Fresh fuzz frames with TTLs in {0,1,2,keep} and next hops (incl. none / out of range)."""
    rng = np.random.default_rng(seed)
    frames = []
    for f in oracle.fuzz_frames(seed, 0, n):
        b = bytearray(f)
        l2 = 18 if len(b) >= 14 and b[12:14] == b"\x81\x00" else 14
        r = rng.random()
        if r < 0.3 and len(b) > l2 + 8:
            b[l2 + 8] = int(rng.integers(0, 3))
        frames.append(bytes(b))
    table = rng.integers(0, 256, size=(table_n, 12), dtype=np.uint8)
    nh = rng.integers(0, table_n + 2, size=n).astype(np.uint32)
    nh[rng.random(n) < 0.05] = 0xFFFFFFFF
    return frames, table, nh
