"""GPU parity of the fused L3 forward (nfcs_l3_forward_device) through the C
ABI against the reference's own output (tests/golden/kat_l3.json, l3fwd_ref.npz) and against
the oracle on fresh seeded inputs, byte for byte."""
import json
import os

import numpy as np
import pytest

import netflow_amd as nf
import oracle
from l3_common import GOLD, frame_hashes, l3_fixture, random_l3_case

pytestmark = pytest.mark.gpu


def run_l3(engine, arena, desc, nh, table):
    n = len(desc)
    table = np.ascontiguousarray(table, dtype=np.uint8).reshape(-1, 12)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(max(desc.nbytes, 16)).upload(desc)
    d_nh = engine.alloc(max(4 * n, 16)).upload(np.ascontiguousarray(nh, dtype=np.uint32))
    d_tab = engine.alloc(max(table.nbytes, 16))
    if table.size:
        d_tab.upload(table)
    d_st = engine.alloc(max(n, 16))
    engine.l3_forward_device(d_arena, arena.nbytes, d_desc, d_nh, n, d_tab, len(table), d_st)
    engine.sync()
    return d_arena.download(np.uint8, arena.nbytes), d_st.download(np.uint8, n)


def test_l3_kat_matches_reference(engine):
    kat = json.load(open(os.path.join(GOLD, "kat_l3.json")))
    names = sorted(kat)
    frames = [bytes.fromhex(kat[k]["in"]) for k in names]
    table = np.stack([np.frombuffer(bytes.fromhex(kat[k]["nh"]), dtype=np.uint8)
                      for k in names if kat[k]["nh"]] or [np.zeros(12, np.uint8)])
    nh, t = [], 0
    for k in names:
        if kat[k]["nh"] is None:
            nh.append(0xFFFFFFFF)
        else:
            nh.append(t)
            t += 1
    arena, desc = oracle.pack_frames(frames)
    out, st = run_l3(engine, arena, desc, np.array(nh, np.uint32), table)
    for name, g, s in zip(names, oracle.unpack_frames(out, desc), st):
        assert g.hex() == kat[name]["out"], name
        assert s == kat[name]["status"], name


@pytest.mark.parametrize("align", [16, 128])
def test_l3_fixture_matches_reference(engine, align):
    z, frames = l3_fixture()
    arena, desc = oracle.pack_frames(frames, align=align)
    orig = arena.copy()
    out, st = run_l3(engine, arena, desc, z["nh_index"], z["table"])
    assert np.array_equal(st, z["oracle_status"])
    dom = (st & 0x3F) != 14
    h = frame_hashes(out, desc)
    bad = np.nonzero(h[dom] != z["hash_out"][dom])[0]
    assert len(bad) == 0, f"{len(bad)} frames differ from the reference, first {bad[:5]}"
    # not forwarded: untouched
    for i in np.nonzero((st & 0x80) == 0)[0][:2000]:
        o, ln = int(desc[i]["off16"]) * 16, int(desc[i]["len"])
        assert np.array_equal(out[o:o + ln], orig[o:o + ln]), i


@pytest.mark.parametrize("seed,table_n", [(21, 8), (22, 1), (23, 0)])
def test_l3_fresh_vs_oracle(engine, seed, table_n):
    frames, table, nh = random_l3_case(seed, 30000, table_n=max(table_n, 1))
    table = table[:table_n]
    arena, desc = oracle.pack_frames(frames)
    ref = arena.copy()
    rst = oracle.l3_forward_batch(ref, desc, nh, table)
    out, st = run_l3(engine, arena, desc, nh, table)
    assert np.array_equal(st, rst)
    assert np.array_equal(out, ref)


def test_l3_config_batch_vs_oracle(engine):
    """C3-shaped batch (mixed lengths, TCP/UDP) on the device generator, every packet routed."""
    n = 1 << 16
    d_arena, nbytes, d_desc, hdesc = engine.config_batch(3, 20250620, 0, n, 128)
    arena, desc = oracle.gen_config(3, 20250620, 0, n, 128)
    assert np.array_equal(d_arena.download(np.uint8, nbytes), arena[:nbytes])
    rng = np.random.default_rng(5)
    table = rng.integers(0, 256, size=(16, 12), dtype=np.uint8)
    nh = (np.arange(n) % 17).astype(np.uint32)  # 16 = no route
    rst = oracle.l3_forward_batch(arena, desc, nh, table)
    d_nh = engine.alloc(4 * n).upload(nh)
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_st = engine.alloc(n)
    engine.l3_forward_device(d_arena, nbytes, d_desc, d_nh, n, d_tab, 16, d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    assert np.array_equal(d_arena.download(np.uint8, nbytes), arena[:nbytes])
    assert ((rst & 0x80) != 0).sum() == (nh < 16).sum()  # TTL 64 everywhere: all routed ones go
    assert (rst[nh == 16] == nf.ST_NO_ROUTE).all()


def _pad_groups(frames, rng, keep_every=5):
    """Long-frame groups: in every aligned group of 4 frames except one in `keep_every`, each frame
    is extended to 1300-1500 bytes with random payload (its headers, and so its parse and bounds
    checks, stay those of the fuzz frame), so the batch runs the long-frame shape with every header
    kind of the fuzz in it."""
    out = []
    for i, f in enumerate(frames):
        if (i // 4) % keep_every != 0 and len(f) < 1300:
            f = f + rng.integers(0, 256, size=int(rng.integers(1300, 1501)) - len(f), dtype=np.uint8).tobytes()
        out.append(f)
    return out


@pytest.mark.parametrize("align,n", [(16, 100_003), (128, 100_003), (128, 60_001)])
def test_l3_long_frame_fuzz_vs_oracle(engine, align, n):
    """Bursts of mostly long frames (the long-frame shape, 16-lane rows) with every header kind of
    the fuzz (tagged, options, IHL < 5, IPv6, ICMP, expired TTLs, no route): bytes and statuses
    against the oracle. 100K packets take the deferred form (forward records + apply_fwd_kernel,
    above kFwdDeferAbovePackets), 60K the inline segment stores; both end ragged (a partial last
    group of 4)."""
    rng = np.random.default_rng(align + 7)
    frames, table, nh = random_l3_case(31 + align, n, table_n=8)
    frames = _pad_groups(frames, rng)
    arena, desc = oracle.pack_frames(frames, align=align)
    ref = arena.copy()
    rst = oracle.l3_forward_batch(ref, desc, nh, table)
    out, st = run_l3(engine, arena, desc, nh, table)
    assert np.array_equal(st, rst)
    assert np.array_equal(out, ref)
    assert ((rst & 0x80) != 0).sum() > n // 4  # about a third of the fuzz frames forward


def test_l3_large_batch_vs_oracle(engine):
    """1.2M C1 frames (1.8 GB, larger than the memory-side cache) with expired TTLs, missing routes
    and a ragged tail in one call, against the oracle byte for byte."""
    n = 1_200_003
    arena, desc = oracle.gen_config(1, 20250620, 0, n, 128)
    idx = np.arange(n)
    ttl_at = desc["off16"].astype(np.int64) * 16 + 22
    arena[ttl_at[idx % 7 == 3]] = 1  # TTL 1: expired, untouched
    rng = np.random.default_rng(12)
    table = rng.integers(0, 256, size=(8, 12), dtype=np.uint8)
    nh = (idx % 9).astype(np.uint32)  # 8 = no route
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_nh = engine.alloc(4 * n).upload(nh)
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_st = engine.alloc(n)
    rst = oracle.l3_forward_batch(arena, desc, nh, table)
    engine.l3_forward_device(d_arena, arena.nbytes, d_desc, d_nh, n, d_tab, 8, d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), arena)
    assert (rst[idx % 7 == 3] == nf.ST_TTL_EXPIRED).all()
    assert (rst[(idx % 9 == 8) & (idx % 7 != 3)] == nf.ST_NO_ROUTE).all()


def test_l3_deferred_sub_batches_fuzz_vs_oracle(engine):
    """Above kFwdDeferAbovePackets (64K) the forward defers the stores of its long-frame waves: per
    512K-packet sub-batch, a read pass writing 8-byte forward records, then apply_fwd_kernel writing
    each forwarded packet's bytes from its record. 1.2M mostly long fuzz frames (every header
    kind, expired TTLs, no route, deferring and inline groups side by side, a partial last group):
    bytes and statuses against the oracle."""
    rng = np.random.default_rng(77)
    frames, table, nh = random_l3_case(41, 300_001, table_n=8)
    frames = _pad_groups(frames, rng)
    n = 4 * len(frames) - 1
    frames = (frames * 4)[:n]
    nh = np.tile(nh, 4)[:n]
    arena, desc = oracle.pack_frames(frames, align=128)
    ref = arena.copy()
    rst = oracle.l3_forward_batch(ref, desc, nh, table)
    out, st = run_l3(engine, arena, desc, nh, table)
    assert np.array_equal(st, rst)
    assert np.array_equal(out, ref)


def test_l3_deferred_misaligned_descriptors(engine):
    """Descriptors and next hops need only their natural alignment (8 and 4 bytes): the deferred
    forward over 1.1M C1 frames with both arrays at an address = 8 mod 16, against the oracle."""
    n = 1_100_001
    arena, desc = oracle.gen_config(1, 20250620, 0, n, 128)
    rng = np.random.default_rng(13)
    table = rng.integers(0, 256, size=(8, 12), dtype=np.uint8)
    nh = (np.arange(n) % 9).astype(np.uint32)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes + 16).upload(np.concatenate([np.zeros(8, np.uint8), desc.view(np.uint8)]))
    d_nh = engine.alloc(4 * n + 16).upload(np.concatenate([np.zeros(2, np.uint32), nh]))
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_st = engine.alloc(n)
    rst = oracle.l3_forward_batch(arena, desc, nh, table)
    engine.l3_forward_device(d_arena, arena.nbytes, d_desc.ptr + 8, d_nh.ptr + 8, n, d_tab, 8, d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), arena)


@pytest.mark.parametrize("config,n", [(3, 1 << 22), (1, 1 << 22)])
def test_l3_full_size_digests_match_reference(engine, config, n):
    """The bench's forward workloads at full size against the compiled reference's digests
    (configs.json l3fwd_more): the C3 mix (4M x U{64..1500} B, 8-lane rows of 12 slots) and 4M x
    1500 B (512K sub-batches, the record-only write pass), next hop i % 9 into the fixture's table."""
    g = json.load(open(os.path.join(GOLD, "configs.json")))
    want = [x for x in g["l3fwd_more"] if x["config"] == config and x["first"] == 0 and x["n"] == n]
    assert want
    table = np.frombuffer(bytes.fromhex(g["l3fwd_c1"]["table"]), dtype=np.uint8).copy()
    d_arena, nbytes, d_desc, _ = engine.config_batch(config, 20250620, 0, n, 128)
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_nh = engine.alloc(4 * n).upload((np.arange(n) % 9).astype(np.uint32))
    try:
        engine.l3_forward_device(d_arena, nbytes, d_desc, d_nh, n, d_tab, 8)
        engine.sync()
        assert f"{engine.digest_device(d_arena, nbytes, d_desc, n, 0):016x}" == want[0]["digest_out"]
    finally:
        for b in (d_arena, d_desc, d_tab, d_nh):
            b.free()
