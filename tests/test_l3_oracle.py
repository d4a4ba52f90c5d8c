"""CPU tests of the fused L3 forward restatement (oracle) against the reference's own output:
tests/golden/kat_l3.json and l3fwd_ref.npz were produced by driving the reference's Packet
through the switch.hpp:247-294 data path (tests/golden/make_golden.py, oracle/ref_shim.cpp)."""
import json
import os

import numpy as np
import pytest

import oracle
from l3_common import GOLD, frame_hashes, l3_fixture, random_l3_case


def test_l3_kat_matches_reference(oracle_lib):
    kat = json.load(open(os.path.join(GOLD, "kat_l3.json")))
    assert len(kat) >= 20
    for name, k in kat.items():
        nh = None if k["nh"] is None else bytes.fromhex(k["nh"])
        out, st = oracle.l3_forward_frame(bytes.fromhex(k["in"]), nh)
        assert out.hex() == k["out"], name
        assert st == k["status"], name
        assert bool(st & 0x80) == bool(k["forwarded"]), name


def test_l3_fixture_matches_reference(oracle_lib):
    z, frames = l3_fixture()
    arena, desc = oracle.pack_frames(frames)
    assert np.array_equal(frame_hashes(arena, desc), z["hash_in"])  # same inputs as the reference saw
    st = oracle.l3_forward_batch(arena, desc, z["nh_index"], z["table"])
    assert np.array_equal(st, z["oracle_status"])
    dom = (st & 0x3F) != 14
    h = frame_hashes(arena, desc)
    assert np.array_equal(h[dom], z["hash_out"][dom])
    assert np.array_equal((st[dom] & 0x80) != 0, z["forwarded"][dom] != 0)
    # every outcome is represented
    for s in (11, 12, 13):
        assert (st == s).sum() > 100, s
    assert ((st & 0x80) != 0).sum() > 1000


@pytest.mark.skipif(not oracle.ref_available(), reason="reference shim not built here")
def test_l3_oracle_vs_reference_fresh():
    frames, table, nh = random_l3_case(11, 4000)
    for i, f in enumerate(frames):
        h = bytes(table[nh[i]]) if nh[i] < len(table) else None
        o, st = oracle.l3_forward_frame(f, h)
        if (st & 0x3F) == 14:
            continue
        r, fw = oracle.ref_l3_forward_frame(f, h)
        assert o == r and bool(st & 0x80) == bool(fw), i


def test_l3_oracle_reproduces_c3_bench_digest(oracle_lib):
    """The reference's digest of one fused forward over C3's 4M mixed frames (configs.json
    l3fwd_more, bench.py --op l3fwd --config 3), reproduced by the restatement chunk by chunk."""
    g = json.load(open(os.path.join(GOLD, "configs.json")))
    want = next(x for x in g["l3fwd_more"] if x["config"] == 3)
    table = np.frombuffer(bytes.fromhex(g["l3fwd_c1"]["table"]), dtype=np.uint8).reshape(-1, 12)
    n, chunk, d = want["n"], 1 << 18, 0
    for lo in range(0, n, chunk):
        m = min(chunk, n - lo)
        arena, desc = oracle.gen_config(3, 20250620, lo, m)
        oracle.l3_forward_batch(arena, desc, (np.arange(lo, lo + m) % 9).astype(np.uint32), table)
        d = (d + oracle.digest(arena, desc, lo)) % (1 << 64)
    assert f"{d:016x}" == want["digest_out"]
