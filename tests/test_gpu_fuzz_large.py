"""Large fresh fuzz batches through every entry point on the GPU, byte for byte against the
oracle (itself pinned to the reference by the golden fixtures): 300k frames per op (VLAN-tagged,
IPv4 with options and IHL < 5, IPv6, ICMP, runts, odd lengths, jumbo), packed (16-byte) and
NIC-aligned (128-byte) layouts. These batches are large enough that every wave shape, store form
and cold path of the kernels runs many times in one launch."""
import numpy as np
import pytest

import netflow_amd as nf
import oracle
from vlan_common import random_vlan_case

pytestmark = pytest.mark.gpu

N = 300_000


@pytest.fixture(scope="module")
def frames():
    return oracle.fuzz_frames(9091, 0, N)


@pytest.mark.parametrize("align", [16, 128])
def test_update_large_fuzz(engine, frames, align):
    arena, desc = oracle.pack_frames(frames, align=align)
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_st = engine.alloc(N)
    engine.update_device(d_arena, arena.nbytes, d_desc, N, d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, N), rst)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)


@pytest.mark.parametrize("align", [16, 128])
def test_l3_forward_large_fuzz(engine, frames, align):
    arena, desc = oracle.pack_frames(frames, align=align)
    rng = np.random.default_rng(align)
    table = rng.integers(0, 256, size=(7, 12), dtype=np.uint8)
    nh = rng.integers(0, 8, size=N).astype(np.uint32)  # 7 = no route
    ref = arena.copy()
    rst = oracle.l3_forward_batch(ref, desc, nh, table)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_nh = engine.alloc(nh.nbytes).upload(nh)
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_st = engine.alloc(N)
    engine.l3_forward_device(d_arena, arena.nbytes, d_desc, d_nh, N, d_tab, 7, d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, N), rst)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)


@pytest.mark.parametrize("align", [16, 128])
def test_vlan_large_fuzz(engine, align):
    fr, ops, caps = random_vlan_case(9092 + align, N)
    arena, desc = oracle.pack_frames(fr, align=align, room=4)
    ref, rdesc = arena.copy(), desc.copy()
    rst = oracle.vlan_batch(ref, rdesc, ops, caps)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_ops = engine.alloc(ops.nbytes).upload(np.ascontiguousarray(ops, np.uint32))
    d_caps = engine.alloc(caps.nbytes).upload(np.ascontiguousarray(caps, np.uint32))
    d_st = engine.alloc(N)
    engine.vlan_device(d_arena, arena.nbytes, d_desc, N, d_ops, 0, d_caps, 0, d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, N), rst)
    assert np.array_equal(d_desc.download(nf.DESC_DTYPE, N), rdesc)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)


@pytest.mark.parametrize("align", [16, 128])
def test_flow_keys_large_fuzz(engine, frames, align):
    arena, desc = oracle.pack_frames(frames, align=align)
    recs, hashes = oracle.flow_keys_batch(arena, desc)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_keys = engine.alloc(64 * N)
    d_hash = engine.alloc(4 * N)
    engine.flow_keys_device(d_arena, arena.nbytes, d_desc, N, d_keys, d_hash)
    engine.sync()
    assert np.array_equal(d_keys.download(np.uint8, 64 * N).reshape(N, 64), recs)
    assert np.array_equal(d_hash.download(np.uint32, N), hashes)
