"""Edge cases on the GPU, every entry point against the oracle (pinned to the reference by the
fixtures): empty batches, zero-length and runt frames, and maximum-size frames — IPv4 with
total_length 65535 (a 65,549-byte frame, 65,553 with a tag) and IPv6 with payload_length 65535 —
through update_checksums, the fused L3 forward, VLAN push/pop and flow-key extraction."""
import numpy as np
import pytest

import netflow_amd as nf
import oracle

pytestmark = pytest.mark.gpu


def be16(v):
    return bytes([(v >> 8) & 0xFF, v & 0xFF])


def max_frames(rng):
    out = []
    for tag in (False, True):
        l2 = bytes(rng.integers(0, 256, 12, dtype=np.uint8)) + ((b"\x81\x00" + be16(0x2123)) if tag else b"")
        # IPv4 + UDP / TCP / ICMP with total_length 65535
        for proto in (17, 6, 1):
            payload = bytes(rng.integers(0, 256, 65535 - 20, dtype=np.uint8))
            ip = bytes([0x45, 0]) + be16(65535) + bytes(4) + bytes([64, proto]) + bytes([0x12, 0x34]) + \
                bytes(rng.integers(0, 256, 8, dtype=np.uint8))
            if proto == 17:
                payload = bytes(4) + be16(65535 - 20) + payload[6:]
            elif proto == 6:
                payload = payload[:12] + bytes([0x50]) + payload[13:]
            out.append(l2 + b"\x08\x00" + ip + payload)
        # IPv6 + UDP with payload_length 65535 (UDP length = 65535)
        ip6 = bytes([0x60, 0, 0, 0]) + be16(65535) + bytes([17, 64]) + bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        udp = bytes(4) + be16(65535) + bytes(2) + bytes(rng.integers(0, 256, 65535 - 8, dtype=np.uint8))
        out.append(l2 + b"\x86\xdd" + ip6 + udp)
    return out


def ragged(rng, n=3000):
    frames = oracle.fuzz_frames(99, 0, n)
    for i in range(0, n, 7):
        frames[i] = frames[i][: int(rng.integers(0, 40))]  # zero-length and runt frames
    return frames


def test_empty_batches(engine):
    d = engine.alloc(64)
    engine.update_device(d, 64, d, 0)
    engine.l3_forward_device(d, 64, d, d, 0, d, 1)
    engine.vlan_device(d, 64, d, 0, None, nf.VLAN_POP, None, 64)
    engine.flow_keys_device(d, 64, d, 0, d, d)
    engine.sync()
    st = engine.update_host(np.zeros(16, np.uint8), np.zeros(0, dtype=nf.DESC_DTYPE))
    assert st is None or len(st) == 0


@pytest.mark.parametrize("which", ["max", "ragged"])
def test_update_edges(engine, which):
    rng = np.random.default_rng(5)
    frames = max_frames(rng) if which == "max" else ragged(rng)
    arena, desc = oracle.pack_frames(frames)
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(max(desc.nbytes, 16)).upload(desc)
    d_st = engine.alloc(max(len(desc), 16))
    engine.update_device(d_arena, arena.nbytes, d_desc, len(desc), d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, len(desc)), rst)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)
    if which == "max":
        assert set(rst.tolist()) >= {nf.ST_V4_UDP, nf.ST_V4_TCP, nf.ST_V4_ICMP, nf.ST_V6_UDP}


@pytest.mark.parametrize("which", ["max", "ragged"])
def test_l3_forward_edges(engine, which):
    rng = np.random.default_rng(6)
    frames = max_frames(rng) if which == "max" else ragged(rng)
    arena, desc = oracle.pack_frames(frames)
    table = rng.integers(0, 256, size=(4, 12), dtype=np.uint8)
    nh = (np.arange(len(frames)) % 5).astype(np.uint32)  # 4 = no route
    ref = arena.copy()
    rst = oracle.l3_forward_batch(ref, desc, nh, table)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(max(desc.nbytes, 16)).upload(desc)
    d_nh = engine.alloc(max(nh.nbytes, 16)).upload(nh)
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_st = engine.alloc(max(len(desc), 16))
    engine.l3_forward_device(d_arena, arena.nbytes, d_desc, d_nh, len(desc), d_tab, 4, d_st)
    engine.sync()
    assert np.array_equal(d_st.download(np.uint8, len(desc)), rst)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)


@pytest.mark.parametrize("which", ["max", "ragged"])
def test_vlan_edges(engine, which):
    rng = np.random.default_rng(7)
    frames = max_frames(rng) if which == "max" else ragged(rng)
    arena, desc = oracle.pack_frames(frames, room=4)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(max(desc.nbytes, 16)).upload(desc)
    d_st = engine.alloc(max(len(desc), 16))
    caps = (desc["len"].astype(np.uint32) + 4)
    d_caps = engine.alloc(max(caps.nbytes, 16)).upload(caps)
    for op in (nf.vlan_push_op(4094, 6), nf.VLAN_POP, nf.VLAN_POP):  # push, pop, pop again
        rst = oracle.vlan_batch(arena, desc, None, caps, op_all=op)
        engine.vlan_device(d_arena, arena.nbytes, d_desc, len(desc), None, op, d_caps, 0, d_st)
        engine.sync()
        assert np.array_equal(d_st.download(np.uint8, len(desc)), rst)
        assert np.array_equal(d_desc.download(nf.DESC_DTYPE, len(desc)), desc)
        assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), arena)


@pytest.mark.parametrize("which", ["max", "ragged"])
def test_flow_keys_edges(engine, which):
    rng = np.random.default_rng(8)
    frames = max_frames(rng) if which == "max" else ragged(rng)
    arena, desc = oracle.pack_frames(frames)
    recs, hashes = oracle.flow_keys_batch(arena, desc)
    n = len(desc)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(max(desc.nbytes, 16)).upload(desc)
    d_keys = engine.alloc(64 * n)
    d_hash = engine.alloc(max(4 * n, 16))
    engine.flow_keys_device(d_arena, arena.nbytes, d_desc, n, d_keys, d_hash)
    engine.sync()
    assert np.array_equal(d_keys.download(np.uint8, 64 * n).reshape(n, 64), recs)
    assert np.array_equal(d_hash.download(np.uint32, n), hashes)
