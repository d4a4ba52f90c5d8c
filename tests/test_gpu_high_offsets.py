"""Maximum-size addressing: a descriptor's off16 is a u32 count of 16-byte units, so an arena can
reach 64 GiB and a frame's byte offset needs 36 bits. Frames placed past 32 GiB (off16 >= 2^31: a
signed 32-bit offset would go negative, a 32-bit byte offset would wrap) through every device entry
point — the checksum update (inline and deferred stores), the fused L3 forward, VLAN push/pop,
flow keys and the digest — must give the oracle's bytes, byte for byte, and leave the arena
around them untouched. The region's own offsets are shifted by the base for the device."""
import numpy as np
import pytest

import netflow_amd as nf
import oracle
from l3_common import random_l3_case
from vlan_common import random_vlan_case

pytestmark = pytest.mark.gpu
BASE = (32 << 30) + 4096  # byte offset of the region: off16 = 2^31 + 256
GUARD = 1 << 20           # arena bytes after the region (checked untouched)


@pytest.fixture(scope="module")
def big(engine):
    b = engine.alloc(BASE + (96 << 20) + GUARD)
    yield b
    b.free()


def place(engine, big, arena, desc):
    """Upload the region at BASE with a guard pattern after it; device descriptors shifted."""
    big.upload(arena, BASE)
    big.upload(np.full(GUARD, 0xA5, np.uint8), BASE + arena.nbytes)
    d = desc.copy()
    d["off16"] = d["off16"].astype(np.uint64) + BASE // 16
    assert int(d["off16"].min()) >= 1 << 31
    return engine.alloc(max(d.nbytes, 16)).upload(d), BASE + arena.nbytes + GUARD


def region(big, nbytes):
    out = big.download(np.uint8, nbytes + GUARD, BASE)
    assert (out[nbytes:] == 0xA5).all()  # nothing written past the region
    return out[:nbytes]


def test_update_past_32_gib(engine, big):
    frames = oracle.fuzz_frames(51, 0, 70000)  # > kInlineMaxPackets: inline and deferred waves
    arena, desc = oracle.pack_frames(frames, align=128)
    n = len(desc)
    assert arena.nbytes + GUARD <= (96 << 20) + GUARD
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    d_desc, nbytes = place(engine, big, arena, desc)
    d_st = engine.alloc(n)
    assert engine.digest_device(big, nbytes, d_desc, n) == oracle.digest(arena, desc)
    engine.update_device(big, nbytes, d_desc, n, d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    assert np.array_equal(region(big, arena.nbytes), ref)
    assert engine.digest_device(big, nbytes, d_desc, n) == oracle.digest(ref, desc)
    d_desc.free()
    d_st.free()


def test_l3_forward_past_32_gib(engine, big):
    frames, table, nh = random_l3_case(52, 20000, table_n=8)
    arena, desc = oracle.pack_frames(frames)
    n = len(desc)
    ref = arena.copy()
    rst = oracle.l3_forward_batch(ref, desc, nh, table)
    table = np.ascontiguousarray(table, dtype=np.uint8).reshape(-1, 12)
    d_desc, nbytes = place(engine, big, arena, desc)
    d_nh = engine.alloc(4 * n).upload(np.ascontiguousarray(nh, dtype=np.uint32))
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_st = engine.alloc(n)
    engine.l3_forward_device(big, nbytes, d_desc, d_nh, n, d_tab, len(table), d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    assert np.array_equal(region(big, arena.nbytes), ref)
    for b in (d_desc, d_nh, d_tab, d_st):
        b.free()


def test_vlan_past_32_gib(engine, big):
    frames, ops, caps = random_vlan_case(53, 20000)
    arena, desc = oracle.pack_frames(frames, room=4)
    n = len(desc)
    ref, rdesc = arena.copy(), desc.copy()
    rst = oracle.vlan_batch(ref, rdesc, ops, caps)
    d_desc, nbytes = place(engine, big, arena, desc)
    d_ops = engine.alloc(4 * n).upload(np.ascontiguousarray(ops, dtype=np.uint32))
    d_caps = engine.alloc(4 * n).upload(np.ascontiguousarray(caps, dtype=np.uint32))
    d_st = engine.alloc(n)
    engine.vlan_device(big, nbytes, d_desc, n, d_ops, 0, d_caps, 0, d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    got = d_desc.download(nf.DESC_DTYPE, n)
    assert np.array_equal(got["len"], rdesc["len"])
    assert np.array_equal(got["off16"].astype(np.uint64) - BASE // 16, rdesc["off16"].astype(np.uint64))
    assert np.array_equal(region(big, arena.nbytes), ref)
    for b in (d_desc, d_ops, d_caps, d_st):
        b.free()


def test_flow_keys_past_32_gib(engine, big):
    frames = oracle.fuzz_frames(54, 0, 20000)
    arena, desc = oracle.pack_frames(frames)
    n = len(desc)
    rrecs, rh = oracle.flow_keys_batch(arena, desc)
    d_desc, nbytes = place(engine, big, arena, desc)
    d_keys = engine.alloc(64 * n)
    d_hash = engine.alloc(4 * n)
    engine.flow_keys_device(big, nbytes, d_desc, n, d_keys, d_hash)
    engine.sync()
    assert np.array_equal(d_keys.download(np.uint8, 64 * n).reshape(n, 64), rrecs)
    assert np.array_equal(d_hash.download(np.uint32, n), rh)
    assert np.array_equal(region(big, arena.nbytes), arena)  # read only
    for b in (d_desc, d_keys, d_hash):
        b.free()


@pytest.mark.parametrize("slot", [0, 1536, 900, 256])
def test_update_waves_spanning_32_gib(engine, big, slot):
    """Rows of one wave with frames 32 GiB apart: even packets in a region at the arena's start,
    odd ones in the region past 32 GiB, so every wave's frames span more than the 4 GB a per-wave
    buffer resource addresses and its rows load through global addresses (row_stage's fallback);
    the last wave is partial. Every launch shape (no hint: the long shape; slot hints: long, short,
    tiny), bytes and statuses against the oracle, region by region, the guard untouched."""
    frames = oracle.fuzz_frames(53, 0, 20001)
    fa, fb = frames[0::2], frames[1::2]
    arena_a, desc_a = oracle.pack_frames(fa, align=128)
    arena_b, desc_b = oracle.pack_frames(fb, align=128)
    ref_a, ref_b = arena_a.copy(), arena_b.copy()
    st_a, _ = oracle.update_batch(ref_a, desc_a, nthreads=8)
    st_b, _ = oracle.update_batch(ref_b, desc_b, nthreads=8)
    lo = 4096
    assert lo + arena_a.nbytes < BASE
    big.upload(arena_a, lo)
    big.upload(arena_b, BASE)
    big.upload(np.full(GUARD, 0xA5, np.uint8), BASE + arena_b.nbytes)
    n = len(frames)
    desc = np.zeros(n, dtype=desc_a.dtype)
    desc[0::2] = desc_a
    desc[1::2] = desc_b
    desc["off16"][0::2] = desc_a["off16"].astype(np.uint64) + lo // 16
    desc["off16"][1::2] = desc_b["off16"].astype(np.uint64) + BASE // 16
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_st = engine.alloc(n)
    try:
        engine.set_slot_bytes(slot)
        engine.update_device(big, BASE + arena_b.nbytes + GUARD, d_desc, n, d_st)
        engine.sync()
        st = d_st.download(np.uint8, n)
        assert np.array_equal(st[0::2], st_a) and np.array_equal(st[1::2], st_b)
        assert np.array_equal(big.download(np.uint8, arena_a.nbytes, lo), ref_a)
        assert np.array_equal(region(big, arena_b.nbytes), ref_b)
    finally:
        engine.set_slot_bytes(0)
        d_desc.free()
        d_st.free()


@pytest.mark.parametrize("delta16", [(1 << 28) - (1 << 13) - 1, (1 << 28) - (1 << 13)])
def test_update_waves_at_the_wave_buffer_span_boundary(engine, big, delta16):
    """The short shape's per-wave buffer resource (nfcs_kernels.hip wave_buf): a wave whose
    rows' frames span delta16 16-byte units — kBufSpan16 - 1 (the last span the buffer path takes,
    offsets up to 4 GiB - 128 KiB into the wave's buffer) and kBufSpan16 (the first the global-load
    path takes). Rows 0-2 of every wave lie in one region, row 3 exactly delta16 units above row 0, so
    every wave's span is exactly delta16. An off-by-one in the span check or the out-of-range offset
    would not fault: the lanes would read zeros and the checksums would differ from the oracle's."""
    waves = 5000
    n = 4 * waves
    frames = [f[:1500] if len(f) > 1500 else f for f in oracle.fuzz_frames(55, 0, n)]
    lo = 4096
    off = np.zeros(n, np.uint64)
    for w in range(waves):
        a = lo + w * 3 * 1536
        off[4 * w: 4 * w + 3] = [a, a + 1536, a + 3072]
        off[4 * w + 3] = a + delta16 * 16
    assert int(off.max()) + 1536 < BASE
    packed, pdesc = oracle.pack_frames(frames)
    ref = packed.copy()
    rst, _ = oracle.update_batch(ref, pdesc, nthreads=8)
    region_a = np.zeros(waves * 3 * 1536, np.uint8)
    region_b = np.zeros(waves * 3 * 1536 + 1536, np.uint8)
    b0 = lo + delta16 * 16
    for i, f in enumerate(frames):
        o = int(off[i])
        dst, base = (region_a, lo) if i % 4 != 3 else (region_b, b0)
        dst[o - base: o - base + len(f)] = np.frombuffer(f, np.uint8)
    big.upload(region_a, lo)
    big.upload(region_b, b0)
    desc = np.zeros(n, dtype=nf.DESC_DTYPE)
    desc["off16"] = (off // 16).astype(np.uint32)
    desc["len"] = [len(f) for f in frames]
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_st = engine.alloc(n)
    try:
        engine.set_slot_bytes(900)  # the short shape (16-lane rows in 256-thread workgroups, frame-relative windows, buffer loads)
        engine.update_device(big, b0 + region_b.nbytes, d_desc, n, d_st)
        engine.sync()
        assert np.array_equal(d_st.download(np.uint8, n), rst)
        got_a = big.download(np.uint8, region_a.nbytes, lo)
        got_b = big.download(np.uint8, region_b.nbytes, b0)
        for i, f in enumerate(frames):
            o = int(off[i])
            g, base = (got_a, lo) if i % 4 != 3 else (got_b, b0)
            p = int(pdesc[i]["off16"]) * 16
            assert np.array_equal(g[o - base: o - base + len(f)], ref[p: p + len(f)]), i
    finally:
        engine.set_slot_bytes(0)
        d_desc.free()
        d_st.free()
