"""Line-aligned row windows (netflow_amd/csrc/nfcs_kernels.hip row_stage): the long
shape reads each frame from the 128-byte line in which it starts, so frame chunk j sits in lane
(j + mis) % 16 of slot (j + mis) / 16, where mis (0..7) is the frame's 16-byte offset in that line.
This sweep places frames at every one of the 8 line offsets, with lengths around the places where
that mapping changes — the end of slot 0 (256 bytes), the 7 slots of one row pass (1792 bytes),
continuation batches of jumbo frames — and with every header kind of the fuzz generator (802.1Q,
IPv6, ICMP, IP options and IHL < 5 for the cold path, runts), in waves that mix aligned and
misaligned rows. The update (long shape forced by the slot-size hint, above kInlineMaxPackets so
deferred waves take part), the fused L3 forward, VLAN push / pop and the flow keys must equal the
oracle."""
import numpy as np
import pytest

import oracle
from l3_common import random_l3_case

pytestmark = pytest.mark.gpu


def be16(v):
    return bytes([(v >> 8) & 0xFF, v & 0xFF])


def udp_frame(rng, length, tagged=False):
    """An IPv4/UDP frame of `length` bytes (length >= 42 + 4*tagged) with stale checksums."""
    l2 = bytes(rng.integers(0, 256, 12, dtype=np.uint8)) + ((b"\x81\x00" + be16(0x0123)) if tagged else b"")
    tl = length - len(l2) - 2
    ip = bytes([0x45, 0]) + be16(tl) + bytes(4) + bytes([64, 17]) + bytes([0xAB, 0xCD]) + \
        bytes(rng.integers(0, 256, 8, dtype=np.uint8))
    payload = bytes(rng.integers(0, 256, tl - 20 - 8, dtype=np.uint8))
    return l2 + b"\x08\x00" + ip + be16(1234) + be16(80) + be16(tl - 20) + b"\x5a\xa5" + payload


def boundary_frames(rng):
    out = []
    for base in (64, 240, 256, 272, 1500, 1664, 1776, 1792, 1808, 3584, 9000):
        for d in (-17, -16, -1, 0, 1, 15, 16):
            length = base + d
            if length >= 46:
                out.append(udp_frame(rng, length, tagged=bool(length & 1)))
    return out


def place(frames, offsets, room=0):
    """One arena: frame i starts `offsets[i]` 16-byte chunks past a 128-byte line."""
    desc = np.zeros(len(frames), dtype=oracle.DESC_DTYPE)
    off = 0
    for i, f in enumerate(frames):
        off = (off + 127) // 128 * 128 + 16 * int(offsets[i])
        desc[i] = (off // 16, len(f))
        off += (len(f) + room + 15) // 16 * 16
    arena = np.zeros(max(off, 16), dtype=np.uint8)
    for i, f in enumerate(frames):
        o = int(desc[i]["off16"]) * 16
        arena[o:o + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return arena, desc


@pytest.fixture
def long_shape(engine):
    engine.set_slot_bytes(4096)  # the long shape whatever the arena's footprint
    yield engine
    engine.set_slot_bytes(0)


def sweep(rng, n_fuzz):
    bf = boundary_frames(rng)
    frames = (bf * 8) + oracle.fuzz_frames(61, 0, n_fuzz)
    # every boundary frame at each of the 8 line offsets; fuzz frames at random offsets, so waves
    # hold aligned and misaligned rows side by side
    offsets = np.concatenate([np.repeat(np.arange(8), len(bf)), rng.integers(0, 8, n_fuzz)])
    return frames, offsets


def test_update_every_line_offset(long_shape):
    rng = np.random.default_rng(17)
    frames, offsets = sweep(rng, 70000)  # > kInlineMaxPackets: deferred and inline waves
    arena, desc = place(frames, offsets)
    n = len(desc)
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    d_arena = long_shape.alloc(arena.nbytes).upload(arena)
    d_desc = long_shape.alloc(desc.nbytes).upload(desc)
    d_st = long_shape.alloc(n)
    long_shape.update_device(d_arena, arena.nbytes, d_desc, n, d_st)
    long_shape.sync()
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)
    for b in (d_arena, d_desc, d_st):
        b.free()


def test_l3_forward_every_line_offset(long_shape):
    rng = np.random.default_rng(19)
    frames, table, nh = random_l3_case(29, 30000, table_n=8)
    frames = boundary_frames(rng) * 8 + frames
    nh = np.concatenate([np.arange(len(frames) - len(nh)) % 8, nh]).astype(np.uint32)
    offsets = np.concatenate([np.repeat(np.arange(8), len(frames) - 30000 >> 3), rng.integers(0, 8, 30000)])
    arena, desc = place(frames, offsets)
    n = len(desc)
    ref = arena.copy()
    rst = oracle.l3_forward_batch(ref, desc, nh, table)
    table = np.ascontiguousarray(table, dtype=np.uint8).reshape(-1, 12)
    d_arena = long_shape.alloc(arena.nbytes).upload(arena)
    d_desc = long_shape.alloc(desc.nbytes).upload(desc)
    d_nh = long_shape.alloc(4 * n).upload(nh)
    d_tab = long_shape.alloc(table.nbytes).upload(table)
    d_st = long_shape.alloc(n)
    long_shape.l3_forward_device(d_arena, arena.nbytes, d_desc, d_nh, n, d_tab, len(table), d_st)
    long_shape.sync()
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)
    for b in (d_arena, d_desc, d_nh, d_tab, d_st):
        b.free()


def test_flow_keys_every_line_offset(engine):
    """The flow keys load header bytes 0..47 first and the rest only for long headers: at every line
    offset the records and hashes equal the oracle's."""
    rng = np.random.default_rng(23)
    frames, offsets = sweep(rng, 20000)
    arena, desc = place(frames, offsets)
    n = len(desc)
    keys, hashes = oracle.flow_keys_batch(arena, desc)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_keys = engine.alloc(64 * n)
    d_hash = engine.alloc(4 * n)
    engine.flow_keys_device(d_arena, arena.nbytes, d_desc, n, d_keys, d_hash)
    engine.sync()
    assert np.array_equal(d_hash.download(np.uint32, n), hashes)
    assert np.array_equal(d_keys.download(np.uint8, 64 * n).reshape(n, 64), np.asarray(keys).reshape(n, 64))
    for b in (d_arena, d_desc, d_keys, d_hash):
        b.free()


def test_vlan_every_line_offset(long_shape):
    """VLAN push / pop / re-tag with line-aligned windows (vlan_rows_kernel, long shape): frames at
    every line offset, lengths around the slot boundaries and the fuzz generator's header kinds,
    each with room for a push; bytes, lengths and statuses equal the oracle's."""
    import netflow_amd as nf
    from vlan_common import random_vlan_case
    rng = np.random.default_rng(29)
    bf = boundary_frames(rng)
    fr, ops, caps = random_vlan_case(31, 30000)
    frames = bf * 8 + fr
    kinds = [oracle.vlan_op("push", 100, 3), oracle.vlan_op("pop"), oracle.vlan_op("push", 7, 1)]
    ops = np.concatenate([np.array([kinds[i % 3] for i in range(8 * len(bf))], dtype=np.uint32), ops])
    caps = np.concatenate([np.array([len(f) + 4 for f in bf * 8], dtype=np.uint32), caps])
    offsets = np.concatenate([np.repeat(np.arange(8), len(bf)), rng.integers(0, 8, len(fr))])
    arena, desc = place(frames, offsets, room=4)
    n = len(desc)
    ref, rdesc = arena.copy(), desc.copy()
    rst = oracle.vlan_batch(ref, rdesc, ops=ops, caps=caps)
    d_arena = long_shape.alloc(arena.nbytes).upload(arena)
    d_desc = long_shape.alloc(desc.nbytes).upload(desc)
    d_ops = long_shape.alloc(ops.nbytes).upload(ops)
    d_caps = long_shape.alloc(caps.nbytes).upload(caps)
    d_st = long_shape.alloc(n)
    long_shape.vlan_device(d_arena, arena.nbytes, d_desc, n, d_ops, 0, d_caps, 0, d_st)
    long_shape.sync()
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    assert np.array_equal(d_desc.download(nf.DESC_DTYPE, n), rdesc)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)
    for b in (d_arena, d_desc, d_ops, d_caps, d_st):
        b.free()
