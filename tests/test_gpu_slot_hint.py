"""The launch-shape hint (nfcs_ctx_set_slot_bytes, include/nfcs.h): a burst that fills a small part
of a large arena (a NIC ring) runs the shape its frames call for when the caller states their mean
slot size. The hint picks speed only: every shape (8-lane rows, 16-lane one-wave workgroups,
256-thread workgroups with deferred stores) must give the reference's bytes, statuses and lengths
for the update, the fused L3 forward and VLAN push/pop, checked against the oracle."""
import numpy as np
import pytest

import netflow_amd as nf
import oracle
from l3_common import random_l3_case
from vlan_common import random_vlan_case

pytestmark = pytest.mark.gpu
HINTS = (0, 128, 512, 1000, 4096)  # 0 = arena_bytes / n; then tiny (VLAN: sc1, nt) / short / long shapes
SLACK = 256 << 20  # arena bytes past the burst: with no hint the long shape runs


@pytest.fixture
def hinted(engine):
    yield engine
    engine.set_slot_bytes(0)  # the session engine goes back to arena_bytes / n


@pytest.mark.parametrize("align", [128, 16, 64])
def test_update_every_shape_matches_oracle(hinted, align):
    """Also frames that start mid-line (packed 16-byte and 64-byte starts): the long shape reads
    line-aligned windows (row_stage), whose header view and sums must give the same bytes."""
    frames = oracle.fuzz_frames(33, 0, 70003)  # above kInlineMaxPackets (deferral applies); a partial last wave
    arena, desc = oracle.pack_frames(frames, align=align)
    n = len(desc)
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    d_desc = hinted.alloc(desc.nbytes).upload(desc)
    d_st = hinted.alloc(n)
    d_arena = hinted.alloc(arena.nbytes + SLACK)
    for hint in HINTS:
        hinted.set_slot_bytes(hint)
        d_arena.upload(arena)
        hinted.update_device(d_arena, arena.nbytes + SLACK, d_desc, n, d_st)
        hinted.sync()
        assert np.array_equal(d_st.download(np.uint8, n), rst), hint
        assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref), hint
    for b in (d_arena, d_desc, d_st):
        b.free()


@pytest.mark.parametrize("align", [16, 128])
def test_l3_forward_every_shape_matches_oracle(hinted, align):
    frames, table, nh = random_l3_case(24, 30001, table_n=8)
    arena, desc = oracle.pack_frames(frames, align=align)
    n = len(desc)
    ref = arena.copy()
    rst = oracle.l3_forward_batch(ref, desc, nh, table)
    table = np.ascontiguousarray(table, dtype=np.uint8).reshape(-1, 12)
    d_desc = hinted.alloc(desc.nbytes).upload(desc)
    d_nh = hinted.alloc(4 * n).upload(np.ascontiguousarray(nh, dtype=np.uint32))
    d_tab = hinted.alloc(table.nbytes).upload(table)
    d_st = hinted.alloc(n)
    d_arena = hinted.alloc(arena.nbytes + SLACK)
    for hint in HINTS:
        hinted.set_slot_bytes(hint)
        d_arena.upload(arena)
        hinted.l3_forward_device(d_arena, arena.nbytes + SLACK, d_desc, d_nh, n, d_tab, len(table), d_st)
        hinted.sync()
        assert np.array_equal(d_st.download(np.uint8, n), rst), hint
        assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref), hint
    for b in (d_arena, d_desc, d_nh, d_tab, d_st):
        b.free()


def test_vlan_every_shape_matches_oracle(hinted):
    frames, ops, caps = random_vlan_case(44, 20003)
    arena, desc = oracle.pack_frames(frames, room=4)
    n = len(desc)
    ref, rdesc = arena.copy(), desc.copy()
    rst = oracle.vlan_batch(ref, rdesc, ops, caps)
    d_desc = hinted.alloc(desc.nbytes)
    d_ops = hinted.alloc(4 * n).upload(np.ascontiguousarray(ops, dtype=np.uint32))
    d_caps = hinted.alloc(4 * n).upload(np.ascontiguousarray(caps, dtype=np.uint32))
    d_st = hinted.alloc(n)
    d_arena = hinted.alloc(arena.nbytes + SLACK)
    for hint in HINTS:
        hinted.set_slot_bytes(hint)
        d_arena.upload(arena)
        d_desc.upload(desc)
        hinted.vlan_device(d_arena, arena.nbytes + SLACK, d_desc, n, d_ops, 0, d_caps, 0, d_st)
        hinted.sync()
        assert np.array_equal(d_st.download(np.uint8, n), rst), hint
        assert np.array_equal(d_desc.download(np.dtype(desc.dtype), n), rdesc), hint
        assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref), hint
    for b in (d_arena, d_desc, d_ops, d_caps, d_st):
        b.free()


def ring_burst(n, L, slot, seed):
    """n IPv4/UDP frames of L bytes at the starts of `slot`-byte slots (a NIC ring's layout)."""
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, size=(n, slot), dtype=np.uint8)
    host[:, L:] = 0
    host[:, 12], host[:, 13], host[:, 14], host[:, 15] = 0x08, 0x00, 0x45, 0x00
    host[:, 16], host[:, 17] = (L - 14) >> 8, (L - 14) & 0xFF
    host[:, 22], host[:, 23] = 64, 17
    host[:, 38], host[:, 39] = (L - 34) >> 8, (L - 34) & 0xFF
    desc = np.zeros(n, dtype=oracle.DESC_DTYPE)
    desc["off16"] = np.arange(n, dtype=np.uint32) * (slot // 16)
    desc["len"] = L
    return host.reshape(-1), desc


def test_ring_burst_adapts_without_hint(engine):
    """1M 64-byte frames at the start of a 4 GiB ring, NO slot-size hint: arena_bytes / n (4 KiB)
    says long frames, so the first call runs the long shape and samples the frames' footprint
    (sample_footprint); from the second call over the same burst the launch runs the shape the
    sample calls for (8-lane rows below kTinyMeanBytes = 800). The shape is read back directly
    (nfcs_ctx_launch_footprint), not inferred from timings; bytes equal the oracle's at every call
    (the shape picks speed only). The times are printed for the record, never asserted."""
    n, L, slot, ring = 1 << 20, 64, 128, 4 << 30
    host, desc = ring_burst(n, L, slot, 7)
    ref = host.copy()
    oracle.update_batch(ref, desc, nthreads=8)
    engine.set_slot_bytes(0)
    a = engine.alloc(ring)
    d = engine.alloc(desc.nbytes).upload(desc)
    try:
        a.upload(host)
        assert engine.launch_footprint(ring, d, n) == ring // n  # nothing sampled yet: the long shape
        first = engine.time_update_device(a, ring, d, n, 1)  # the long shape + the sample
        engine.sync()
        assert np.array_equal(a.download(np.uint8, host.nbytes), ref)
        fp = engine.launch_footprint(ring, d, n)
        assert fp < 800 and fp >= slot, fp  # the sample: 128-byte slots -> 8-lane rows from now on
        assert engine.launch_footprint(ring, d, n - 4) == ring // (n - 4)  # another burst: not its sample
        engine.time_update_device(a, ring, d, n, 10)  # warm
        adapted = engine.time_update_device(a, ring, d, n, 40) / 40
        assert np.array_equal(a.download(np.uint8, host.nbytes), ref)  # idempotent
        engine.set_slot_bytes(slot)
        assert engine.launch_footprint(ring, d, n) == slot
        engine.time_update_device(a, ring, d, n, 10)
        hinted = engine.time_update_device(a, ring, d, n, 40) / 40
        print(f"1M x 64 B in a 4 GiB ring: first call {first * 1e3:.1f} us, adapted {adapted * 1e3:.1f} us, "
              f"with the hint {hinted * 1e3:.1f} us")
        # VLAN push/pop on the same ring adapts the same way (its kernel samples too); an even
        # number of alternating push / pop calls leaves every frame as it was
        engine.set_slot_bytes(0)
        push = nf.vlan_push_op(100, 3)
        vfirst = engine.time_vlan_device(a, ring, d, n, push, nf.VLAN_POP, slot, 2)
        fp = engine.launch_footprint(ring, d, n)
        assert fp < 800 and fp >= slot, fp
        engine.time_vlan_device(a, ring, d, n, push, nf.VLAN_POP, slot, 10)
        vadapted = engine.time_vlan_device(a, ring, d, n, push, nf.VLAN_POP, slot, 40) / 40
        engine.set_slot_bytes(slot)
        engine.time_vlan_device(a, ring, d, n, push, nf.VLAN_POP, slot, 10)
        vhinted = engine.time_vlan_device(a, ring, d, n, push, nf.VLAN_POP, slot, 40) / 40
        # frames equal within their length (a pop leaves the pushed frame's last 4 bytes past the
        # new end, as the reference's memmove does)
        got = a.download(np.uint8, host.nbytes).reshape(n, slot)
        assert np.array_equal(got[:, :L], ref.reshape(n, slot)[:, :L])
        print(f"VLAN push/pop: first pair {vfirst / 2 * 1e3:.1f} us per call, adapted {vadapted * 1e3:.1f} us, "
              f"with the hint {vhinted * 1e3:.1f} us")
    finally:
        engine.set_slot_bytes(0)
        a.free()
        d.free()


def test_footprint_sampled_over_the_whole_sub_batched_call(engine):
    """A 1M-packet burst in a ring of 2176-byte slots whose first 512K frames are 1500 bytes long and
    whose last 512K are 64 bytes (arena_bytes / n = 2176 says long, so the call runs as two 512K
    sub-batches and samples): the footprint read back reflects BOTH halves, (1536 + 128) / 2 = 832
    bytes, not the first sub-batch's 1536 (round 5: the first sub-batch samples 256 descriptors
    spread over the whole call). Bytes equal the oracle's."""
    n, slot = 1 << 20, 2176
    h1, d1 = ring_burst(n // 2, 1500, slot, 21)
    h2, d2 = ring_burst(n // 2, 64, slot, 22)
    host = np.concatenate([h1, h2])
    desc = np.concatenate([d1, d2])
    desc["off16"][n // 2:] += (n // 2) * (slot // 16)
    ring = host.nbytes
    ref = host.copy()
    oracle.update_batch(ref, desc, nthreads=8)
    engine.set_slot_bytes(0)
    a = engine.alloc(ring).upload(host)
    d = engine.alloc(desc.nbytes).upload(desc)
    try:
        assert engine.launch_footprint(ring, d, n) == slot
        engine.update_device(a, ring, d, n)
        engine.sync()
        assert np.array_equal(a.download(np.uint8, ring), ref)
        fp = engine.launch_footprint(ring, d, n)
        assert 700 <= fp <= 960, fp
        engine.update_device(a, ring, d, n)  # now the short shape: same bytes (idempotent)
        engine.sync()
        assert np.array_equal(a.download(np.uint8, ring), ref)
    finally:
        a.free()
        d.free()


def test_footprint_kept_per_burst_across_a_rotation(engine):
    """Calls rotating over three bursts (descriptor arrays) of 64-byte frames in 4 KiB-slot rings, no
    hint: each burst keeps its own sample (8 observation slots per context, least recently used
    replaced), so every one adapts after its first call — round 4 kept one, and a rotation never
    adapted. A sample of a replaced burst's generation is never taken for another's."""
    n, L, slot = 1 << 16, 64, 4096
    bursts = []
    engine.set_slot_bytes(0)
    try:
        for k in range(3):
            host, desc = ring_burst(n, L, slot, 30 + k)
            ref = host.copy()
            oracle.update_batch(ref, desc, nthreads=8)
            bursts.append((engine.alloc(host.nbytes).upload(host), engine.alloc(desc.nbytes).upload(desc), ref))
        for rnd in range(2):
            for a, d, ref in bursts:
                engine.update_device(a, ref.nbytes, d, n)
                engine.sync()
                assert np.array_equal(a.download(np.uint8, ref.nbytes), ref)
        for a, d, ref in bursts:
            fp = engine.launch_footprint(ref.nbytes, d, n)
            assert 128 <= fp < 800, fp  # each burst's own sample: 64-byte frames round up to 128
        # 8 more bursts push the first three out: their footprint is arena_bytes / n again
        others = [engine.alloc(16 * n) for _ in range(8)]
        try:
            for k, o in enumerate(others):
                od = np.zeros(n, dtype=oracle.DESC_DTYPE)
                od["off16"] = np.arange(n, dtype=np.uint32) * (slot // 16)
                od["len"] = L
                o.upload(od)
                engine.update_device(bursts[k % 3][0], bursts[k % 3][2].nbytes, o, n)
            engine.sync()
            for a, d, ref in bursts:
                assert engine.launch_footprint(ref.nbytes, d, n) == ref.nbytes // n
        finally:
            for o in others:
                o.free()
    finally:
        for a, d, _ in bursts:
            a.free()
            d.free()


def packed_udp(lengths, seed):
    """IPv4/UDP frames of the given lengths, packed at 16-byte starts (SURVEY §8d's arena layout)."""
    rng = np.random.default_rng(seed)
    frames = []
    for L in lengths:
        f = rng.integers(0, 256, int(L), dtype=np.uint8)
        f[12:16] = (0x08, 0x00, 0x45, 0x00)
        f[16], f[17] = (L - 14) >> 8, (L - 14) & 0xFF
        f[22], f[23] = 64, 17
        f[38], f[39] = (L - 34) >> 8, (L - 34) & 0xFF
        frames.append(f.tobytes())
    return oracle.pack_frames(frames, align=16)


@pytest.mark.parametrize("mix", ["c3", "imix", "bimodal25"])
def test_packed_mix_shape_follows_its_sample(engine, mix):
    """A densely packed burst whose arena_bytes / n says 8-lane rows (< kTinyMeanBytes): the first call
    runs them and samples its frames. C3's mix (U{64..1500}, 782 B per packet packed; half its frames
    need a second 8-lane row pass) then runs the 16-lane short shape (footprint read back >= 800:
    round 6, packed C3 0.655 against 0.79-0.82 ms per call in 8-lane rows); IMIX 7:4:1 (64/570/1500 B,
    one frame in 12 longer than a row pass) stays on 8-lane rows, and so does a mix of 64-byte frames
    with 25% 1500-byte ones (many long frames, but a 424-byte mean: below kTinyMixMeanBytes, where the
    shape audit measured 8-lane rows 15-25% faster). Bytes and statuses equal the oracle's at every
    call (the shape picks speed only)."""
    n = 1 << 17
    if mix == "c3":
        arena, desc = oracle.gen_config(3, 20250620, 0, n)
    elif mix == "imix":
        lens = np.random.default_rng(62).permutation(np.tile([64] * 7 + [570] * 4 + [1500], n // 12 + 1)[:n])
        arena, desc = packed_udp(lens, 61)
    else:
        lens = np.random.default_rng(64).permutation(np.tile([64] * 3 + [1500], n // 4))
        arena, desc = packed_udp(lens, 63)
    est = arena.nbytes // n
    assert est < 800, est
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    engine.set_slot_bytes(0)
    a = engine.alloc(arena.nbytes).upload(arena)
    d = engine.alloc(desc.nbytes).upload(desc)
    st = engine.alloc(n)
    try:
        assert engine.launch_footprint(arena.nbytes, d, n) == est  # nothing sampled: 8-lane rows
        for k in range(3):
            engine.update_device(a, arena.nbytes, d, n, st)
            engine.sync()
            assert np.array_equal(a.download(np.uint8, arena.nbytes), ref), k
            assert np.array_equal(st.download(np.uint8, n), rst), k
            fp = engine.launch_footprint(arena.nbytes, d, n)
            if mix == "c3":
                assert 800 <= fp < 1200, fp  # the short shape from the second call on
            else:
                assert fp < 800, fp  # 8-lane rows stay
    finally:
        for b in (a, d, st):
            b.free()


def test_packed_mix_forward_and_vlan_follow_the_sample(engine):
    """The same shape rule for the fused L3 forward and VLAN push/pop (their launches sample too): C3's
    mix packed at 16-byte starts, three forwards in a row (8-lane rows of 6 slots, then the short-mix
    shape once the sample has counted the long frames) and a push / pop / push sequence, each call's
    bytes, statuses and lengths against the oracle applied as many times."""
    n = 1 << 16
    arena0, desc0 = oracle.gen_config(3, 20250620, 0, n)
    frames = oracle.unpack_frames(arena0, desc0)
    arena, desc = oracle.pack_frames(frames, align=16, room=4)
    caps = np.diff(np.append(desc["off16"].astype(np.int64), arena.nbytes // 16)) * 16
    rng = np.random.default_rng(63)
    table = rng.integers(0, 256, (8, 12), dtype=np.uint8)
    nh = (np.arange(n) % 9).astype(np.uint32)  # index 8: no route
    engine.set_slot_bytes(0)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_nh = engine.alloc(4 * n).upload(nh)
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_caps = engine.alloc(8 * n).upload(np.ascontiguousarray(caps, dtype=np.uint32))
    d_st = engine.alloc(n)
    try:
        assert engine.launch_footprint(arena.nbytes, d_desc, n) < 800
        ref = arena.copy()
        for k in range(3):
            rst = oracle.l3_forward_batch(ref, desc, nh, table)
            engine.l3_forward_device(d_arena, arena.nbytes, d_desc, d_nh, n, d_tab, 8, d_st)
            engine.sync()
            assert np.array_equal(d_st.download(np.uint8, n), rst), k
            assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref), k
        assert engine.launch_footprint(arena.nbytes, d_desc, n) >= 800  # the forward's sample moved it
        rdesc = desc.copy()
        for k, op in enumerate(["push", "pop", "push"]):
            word = oracle.vlan_op(op, 100 + k, 3)
            rst = oracle.vlan_batch(ref, rdesc, None, caps, op_all=word)
            engine.vlan_device(d_arena, arena.nbytes, d_desc, n, None, word, d_caps, 0, d_st)
            engine.sync()
            assert np.array_equal(d_st.download(np.uint8, n), rst), op
            assert np.array_equal(d_desc.download(np.dtype(desc.dtype), n), rdesc), op
            assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref), op
    finally:
        engine.set_slot_bytes(0)
        for b in (d_arena, d_desc, d_nh, d_tab, d_caps, d_st):
            b.free()


@pytest.mark.parametrize("align", [16, 128])
def test_packed_imix_vlan_follows_the_sample(engine, align):
    """VLAN push/pop on IMIX 7:4:1 (mean footprint under kTinyMeanBytes: 8-lane rows). The first call
    samples the frames; from the second on, frames of varying lengths (and, packed at 16-byte starts,
    frames sharing lines) store write-through in 8-lane rows (nfcs_internal.h kVlanWtMeanBytes; the
    round-6 audit measured them 15-31% faster than past the caches). Each call's bytes, statuses and
    lengths equal the oracle's applied as many times (the store policy picks speed only)."""
    n = 1 << 16
    lens = np.random.default_rng(65).permutation(np.tile([64] * 7 + [570] * 4 + [1500], n // 12 + 1)[:n])
    arena0, desc0 = packed_udp(lens, 66)
    frames = oracle.unpack_frames(arena0, desc0)
    arena, desc = oracle.pack_frames(frames, align=align, room=4)
    caps = np.diff(np.append(desc["off16"].astype(np.int64), arena.nbytes // 16)) * 16
    engine.set_slot_bytes(0)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_caps = engine.alloc(4 * n).upload(np.ascontiguousarray(caps, dtype=np.uint32))
    d_st = engine.alloc(n)
    try:
        assert engine.launch_footprint(arena.nbytes, d_desc, n) < 800
        ref, rdesc = arena.copy(), desc.copy()
        for k, op in enumerate(["push", "pop", "push", "pop"]):
            word = oracle.vlan_op(op, 200 + k, 5)
            rst = oracle.vlan_batch(ref, rdesc, None, caps, op_all=word)
            engine.vlan_device(d_arena, arena.nbytes, d_desc, n, None, word, d_caps, 0, d_st)
            engine.sync()
            assert np.array_equal(d_st.download(np.uint8, n), rst), op
            assert np.array_equal(d_desc.download(np.dtype(desc.dtype), n), rdesc), op
            assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref), op
        assert engine.launch_footprint(arena.nbytes, d_desc, n) < 800  # still 8-lane rows
    finally:
        engine.set_slot_bytes(0)
        for b in (d_arena, d_desc, d_caps, d_st):
            b.free()


def test_packed_bimodal_forward_matches_oracle(engine):
    """The fused forward on a 64/1500 mix with 40% full-size frames packed at 16-byte starts: its
    sample finds hardly any frames between minimum and full size, so from the second call on it keeps
    8-lane rows of 6 slots where the update's rule would move to 16-lane rows (kObsMidShift; the round-6
    audit measured them 27-34% faster for such mixes). Three forwards in a row, each call's bytes and
    statuses against the oracle applied as many times."""
    n = 1 << 16
    lens = np.random.default_rng(67).permutation(np.tile([64] * 3 + [1500] * 2, n // 5 + 1)[:n])
    arena, desc = packed_udp(lens, 68)
    rng = np.random.default_rng(69)
    table = rng.integers(0, 256, (8, 12), dtype=np.uint8)
    nh = (np.arange(n) % 9).astype(np.uint32)
    engine.set_slot_bytes(0)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_nh = engine.alloc(4 * n).upload(nh)
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_st = engine.alloc(n)
    try:
        ref = arena.copy()
        for k in range(3):
            rst = oracle.l3_forward_batch(ref, desc, nh, table)
            engine.l3_forward_device(d_arena, arena.nbytes, d_desc, d_nh, n, d_tab, 8, d_st)
            engine.sync()
            assert np.array_equal(d_st.download(np.uint8, n), rst), k
            assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref), k
    finally:
        for b in (d_arena, d_desc, d_nh, d_tab, d_st):
            b.free()


@pytest.mark.parametrize("mixed", [False, True])
def test_ring_of_mid_size_frames_runs_eight_lane_rows(engine, mixed):
    """A burst in a ring of 2 KiB slots, no hint: arena_bytes / n says long, so the first call samples.
    Frames of one length (1024 B) on their own lines then run 8-lane rows (footprint read back just under
    kTinyMeanBytes; round 6 audit: 13-16% faster than the short shape), while frames of varying length
    (U{512..1500}, same slots) keep the mean's shape. Bytes equal the oracle's at every call."""
    n, slot = 1 << 16, 2048
    rng = np.random.default_rng(70 + mixed)
    lens = rng.integers(512, 1501, n) if mixed else np.full(n, 1024)
    host = rng.integers(0, 256, size=(n, slot), dtype=np.uint8)
    L = lens.astype(np.int64)
    host[:, 12], host[:, 13], host[:, 14], host[:, 15] = 0x08, 0x00, 0x45, 0x00
    host[:, 16], host[:, 17] = (L - 14) >> 8, (L - 14) & 0xFF
    host[:, 22], host[:, 23] = 64, 17
    host[:, 38], host[:, 39] = (L - 34) >> 8, (L - 34) & 0xFF
    host = host.reshape(-1)
    desc = np.zeros(n, dtype=oracle.DESC_DTYPE)
    desc["off16"] = np.arange(n, dtype=np.uint32) * (slot // 16)
    desc["len"] = lens
    ref = host.copy()
    oracle.update_batch(ref, desc, nthreads=8)
    engine.set_slot_bytes(0)
    # a burst is known by (descriptor array, n, arena bytes): a different arena size per case keeps the
    # other case's sample (its descriptors may land at the same address) from being taken for this one's
    # first call; from then on every call re-samples, so the footprint read back is this burst's own
    nbytes = host.nbytes + (4096 if mixed else 0)
    a = engine.alloc(nbytes).upload(host)
    d = engine.alloc(desc.nbytes).upload(desc)
    try:
        for k in range(3):
            engine.update_device(a, nbytes, d, n)
            engine.sync()
            assert np.array_equal(a.download(np.uint8, host.nbytes), ref), k
        fp = engine.launch_footprint(nbytes, d, n)
        if mixed:
            assert 800 <= fp < 1200, fp  # the short shape, by the mean
        else:
            assert fp == 799, fp  # 8-lane rows
    finally:
        a.free()
        d.free()
