"""Shared inputs for the VLAN push/pop tests: the fixture frames of
tests/golden/vlan_ref.npz are the oracle fuzz frames of its seed, with the per-frame edit words
and buffer capacities stored in the fixture (recipe: tests/golden/make_golden.py:vlan_inputs)."""
import json
import os

import numpy as np

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def vlan_kats():
    return json.load(open(os.path.join(GOLD, "kat_vlan.json")))


def vlan_fixture():
    z = np.load(os.path.join(GOLD, "vlan_ref.npz"))
    frames = oracle.fuzz_frames(int(z["seed"]), 0, len(z["lens"]))
    return z, frames


def window_hashes(arena, desc_in):
    """frame_hash of each frame's edit window (vlan_window(len_in) bytes from its start)."""
    L = oracle.lib()
    out = np.zeros(len(desc_in), dtype=np.uint64)
    for i, d in enumerate(desc_in):
        o, w = int(d["off16"]) * 16, oracle.vlan_window(int(d["len"]))
        out[i] = L.nfo_frame_hash(oracle._ptr(arena[o:o + w]), w)
    return out


def random_vlan_case(seed: int, n: int):
    """Fresh fuzz frames with random edits (push / pop / none) and capacities."""
    rng = np.random.default_rng(seed)
    frames = oracle.fuzz_frames(seed, 0, n)
    ops = np.zeros(n, dtype=np.uint32)
    caps = np.zeros(n, dtype=np.uint32)
    for i, f in enumerate(frames):
        r = rng.random()
        if r < 0.45:
            ops[i] = oracle.vlan_op("push", int(rng.integers(0, 4096)), int(rng.integers(0, 8)))
        elif r < 0.9:
            ops[i] = oracle.vlan_op("pop")
        caps[i] = len(f) + int(rng.integers(0, 6)) if rng.random() < 0.3 else len(f) + 4
    # make a quarter of the pops land on tagged frames built from untagged ones
    for i in range(0, n, 4):
        f = frames[i]
        if len(f) >= 14 and f[12:14] != b"\x81\x00":
            frames[i] = f[:12] + bytes([0x81, 0x00, 0x20 | (i & 0x0F), i & 0xFF]) + f[12:]
            ops[i] = oracle.vlan_op("pop")
            caps[i] = len(frames[i])
    return frames, ops, caps
