"""Host-memory bursts in the forms a NetFlow++ caller holds them (round 5), against the oracle:

* a NIC ring burst that wraps past the ring's end: nfcs_update_host splits it where
  an offset drops below its predecessor's (packet_buffer.hpp:21-31 — separate PacketBuffers never
  constrain their order), in all three host modes;
* frames scattered in host memory, one pointer each (nfcs_update_host_frames: each PacketBuffer's data
  window, packet_buffer.hpp:51-52), at arbitrary byte offsets and in any order, with NULL and empty
  frames, over several staging chunks.

Every byte outside the frames must stay as it was (the reference writes only its 2+2 checksum bytes,
packet.hpp:740, 822, 867-871, 886)."""
import numpy as np
import pytest

import netflow_amd as nf
import oracle

pytestmark = pytest.mark.gpu

SLOT = 2176  # BufferPool's default slot (DPDK mbuf: 2048 data + 128 headroom)


def ring_burst(n_slots: int, first_slot: int, frames: list[bytes], junk_seed: int):
    """A ring of n_slots SLOT-byte slots filled with junk, the burst's frames written into consecutive
    slots from first_slot on, wrapping to slot 0 at the ring's end."""
    rng = np.random.default_rng(junk_seed)
    ring = rng.integers(0, 256, n_slots * SLOT, dtype=np.uint8)
    desc = np.zeros(len(frames), dtype=nf.DESC_DTYPE)
    for j, f in enumerate(frames):
        o = ((first_slot + j) % n_slots) * SLOT
        ring[o: o + len(f)] = np.frombuffer(f, dtype=np.uint8)
        desc[j] = (o // 16, len(f))
    return ring, desc


def short_frames(seed: int, n: int) -> list[bytes]:
    """Fuzz frames (every header kind) that fit one ring slot."""
    out, i = [], 0
    while len(out) < n:
        batch = oracle.fuzz_frames(seed, i, 4096)
        i += 4096
        out += [f for f in batch if len(f) <= SLOT]
    return out[:n]


@pytest.mark.parametrize("mode", ["patch", "frames", "zero_copy"])
def test_ring_burst_that_wraps(engine, mode):
    """200K frames over a 256K-slot ring (557 MB), starting 80K slots before its end: the burst's
    descriptors drop back to offset 0 mid-burst. Bytes and statuses equal the oracle's, per packet;
    the ring's other slots are untouched."""
    n_slots, n = 1 << 18, 200_000
    frames = short_frames(41, n)
    ring, desc = ring_burst(n_slots, n_slots - 80_000, frames, 7)
    assert int(desc["off16"][80_000]) == 0 and int(desc["off16"][79_999]) > 0  # the wrap
    ref = ring.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    if mode == "zero_copy":
        arena = engine.host_array(ring.nbytes)
        try:
            arena[:] = ring
            st = engine.update_host(arena, desc, mode=mode)
            got = arena.copy()
        finally:
            engine.host_free(arena)
    else:
        st = engine.update_host(ring, desc, mode=mode)
        got = ring
    assert np.array_equal(st, rst)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("mode", ["patch", "frames"])
def test_ring_burst_wrapping_several_times_in_short_runs(engine, mode):
    """A burst whose descriptors jump back every few frames (runs of 1..64 ascending frames at random
    places of the ring): a chunk is cut where an offset drops, so chunks' spans interleave — each
    chunk's span can hold frames of the chunks beside it. Every result the oracle's, also with whole
    frames back (only a chunk's own frames are copied back then)."""
    n_slots, n = 1 << 17, 60_000
    frames = short_frames(43, n)
    rng = np.random.default_rng(5)
    ring = rng.integers(0, 256, n_slots * SLOT, dtype=np.uint8)
    desc = np.zeros(n, dtype=nf.DESC_DTYPE)
    j = 0
    used = np.zeros(n_slots, bool)
    while j < n:
        run = int(rng.integers(1, 65))
        start = int(rng.integers(0, n_slots - run))
        while used[start: start + run].any():
            start = int(rng.integers(0, n_slots - run))
        for k in range(min(run, n - j)):
            o = (start + k) * SLOT
            f = frames[j]
            ring[o: o + len(f)] = np.frombuffer(f, dtype=np.uint8)
            desc[j] = (o // 16, len(f))
            used[start + k] = True
            j += 1
    ref = ring.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    st = engine.update_host(ring, desc, mode=mode)
    assert np.array_equal(st, rst)
    assert np.array_equal(ring, ref)


def scattered(frames: list[bytes], seed: int, null_every: int = 0):
    """The frames at random byte offsets of one junk-filled buffer (gaps of 0-300 bytes, any
    alignment), listed in a shuffled order; every null_every-th entry a NULL frame."""
    rng = np.random.default_rng(seed)
    gaps = rng.integers(0, 301, len(frames))
    offs = np.zeros(len(frames), np.int64)
    o = 0
    for i, f in enumerate(frames):
        o += int(gaps[i])
        offs[i] = o
        o += len(f)
    buf = rng.integers(0, 256, o + 64, dtype=np.uint8)
    for i, f in enumerate(frames):
        buf[offs[i]: offs[i] + len(f)] = np.frombuffer(f, dtype=np.uint8)
    lens = np.array([len(f) for f in frames], np.uint32)
    perm = rng.permutation(len(frames))
    offs, lens = offs[perm], lens[perm]
    if null_every:
        offs[::null_every] = -1
    return buf, offs, lens


def expected(buf: np.ndarray, offs: np.ndarray, lens: np.ndarray):
    """The oracle on the same frames, packed, written back into a copy of the scattered buffer."""
    live = offs >= 0
    frames = [bytes(buf[o: o + ln]) if o >= 0 else b"" for o, ln in zip(offs, lens)]
    packed, desc = oracle.pack_frames(frames)
    rst, _ = oracle.update_batch(packed, desc, nthreads=8)
    out = buf.copy()
    for i in np.nonzero(live)[0]:
        o, ln = int(offs[i]), int(lens[i])
        p = int(desc[i]["off16"]) * 16
        out[o: o + ln] = packed[p: p + ln]
    rst = rst.copy()
    rst[~live] = nf.ST_NONE
    return out, rst


def test_scattered_frames_vs_oracle(engine):
    """nfcs_update_host_frames over 150K fuzz frames (every header kind, jumbo frames, runts, empty
    frames) at arbitrary byte offsets in a shuffled order, every 97th entry NULL: several 64 MiB
    staging chunks; bytes and statuses equal the oracle's, bytes between the frames untouched."""
    frames = oracle.fuzz_frames(44, 0, 150_000)
    frames[17] = b""
    buf, offs, lens = scattered(frames, 9, null_every=97)
    want, wst = expected(buf, offs, lens)
    st = engine.update_host_frames(buf, offs, lens)
    assert np.array_equal(st, wst)
    assert np.array_equal(buf, want)


def test_scattered_c1_frames_match_reference_digest(engine):
    """BASELINE C1's first 65,536 frames, each copied to its own place (shuffled, unaligned),
    through nfcs_update_host_frames and gathered back into the generator's layout: byte-equal to
    the oracle's update of the generated batch (the full 1M-frame C1 digest against the reference's
    is bench.py's host_adapter sub-line)."""
    n = 65536
    arena, desc = oracle.gen_config(1, 20250620, 0, n)
    frames = oracle.unpack_frames(arena, desc)
    buf, offs, lens = scattered(frames, 10)
    order = np.argsort(offs)  # entries in buffer order: order[k] is packet k's entry
    st = engine.update_host_frames(buf, offs, lens)
    assert (st == nf.ST_V4_UDP).all()
    out = np.zeros_like(arena)
    for k in range(n):
        i = int(order[k])  # the k-th frame in buffer order is packet k
        o = int(offs[i])
        out[int(desc[k]["off16"]) * 16: int(desc[k]["off16"]) * 16 + int(lens[i])] = buf[o: o + int(lens[i])]
    ref = arena.copy()
    oracle.update_batch(ref, desc, nthreads=8)
    assert oracle.digest(out, desc) == oracle.digest(ref, desc)
    assert np.array_equal(out, ref)


def test_scattered_small_bursts(engine):
    """Bursts of 0, 1 and 3 frames (one chunk, no worker threads) and a burst whose frames are all
    NULL."""
    frames = oracle.fuzz_frames(45, 0, 3)
    for k in (0, 1, 3):
        buf, offs, lens = scattered(frames[:k], 11)
        want, wst = expected(buf, offs, lens)
        st = engine.update_host_frames(buf, offs, lens)
        assert np.array_equal(st, wst) and np.array_equal(buf, want)
    buf, offs, lens = scattered(frames, 12)
    offs[:] = -1
    before = buf.copy()
    st = engine.update_host_frames(buf, offs, lens)
    assert (st == nf.ST_NONE).all() and np.array_equal(buf, before)


def test_scattered_frames_longer_than_a_staging_slot(engine):
    """Data windows longer than NFCS_FRAME_RELEVANT_BYTES (128 KiB) — one of them longer than a 64 MiB
    staging slot, which round 5's ABI 2 refused with NFCS_EINVAL — go as their first
    128 KiB: the reference reads and bounds-tests no offset past 65,613, so bytes and statuses equal
    the oracle's on the whole frames, and nothing past the checksum fields changes."""
    base = oracle.fuzz_frames(46, 0, 64)
    rng = np.random.default_rng(13)
    sizes = [0, 200_000, (64 << 20) + 4096, 131_071, 131_072, 131_073]
    frames = [f + rng.integers(0, 256, max(0, sz - len(f)), dtype=np.uint8).tobytes() if sz else f
              for f, sz in zip(base, sizes * 11)]
    buf, offs, lens = scattered(frames, 14)
    want, wst = expected(buf, offs, lens)
    st = engine.update_host_frames(buf, offs, lens)
    assert np.array_equal(st, wst)
    assert np.array_equal(buf, want)


@pytest.mark.parametrize("mode", ["patch", "frames"])
@pytest.mark.parametrize("shift", [1, 8, 13])
def test_pageable_arena_at_any_address(engine, mode, shift):
    """A pageable arena that starts off a 16-byte boundary (a view `shift` bytes into a larger
    buffer), 20K ring slots (43.5 MB: chunks of a quarter of the span, over 8 MiB, so each staging copy
    splits over the copy threads): the staging copy
    in and, with whole frames back, the copy out store non-temporally only from the first 16-byte
    boundary on (round 5). Results equal the oracle's; the guard bytes around the view stay."""
    n_slots, n = 20_000, 19_000
    frames = short_frames(47 + shift, n)
    ring, desc = ring_burst(n_slots, 3_000, frames, 13 + shift)
    ref = ring.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    big = np.random.default_rng(shift).integers(0, 256, ring.nbytes + 64, dtype=np.uint8)
    guard = big.copy()
    view = big[shift: shift + ring.nbytes]
    view[:] = ring
    assert view.ctypes.data % 16 == shift % 16
    st = engine.update_host(view, desc, mode=mode)
    assert np.array_equal(st, rst)
    assert np.array_equal(view, ref)
    assert np.array_equal(big[:shift], guard[:shift])
    assert np.array_equal(big[shift + ring.nbytes:], guard[shift + ring.nbytes:])


def test_bursts_of_every_size_in_sequence(engine):
    """Round 6: host bursts small enough to run as direct chunks (no DMA; the kernel's last workgroup
    signals through a host-mapped flag, nfcs::DoneReq) alternate with ones that take the copy engines,
    through all three host entry points and both staging slots — 300 calls of 1 to 40,000 frames over a
    pinned arena, a pageable one and scattered frames, each call's bytes and statuses the oracle's, so the
    slots' completion counters and their event / flag waits stay in step across every kind of call."""
    rng = np.random.default_rng(71)
    frames = oracle.fuzz_frames(47, 0, 40_000)
    arena, desc = oracle.pack_frames(frames)
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    pinned = engine.host_array(arena.nbytes)
    try:
        for k in range(300):
            n = int(rng.choice([1, 3, 64, 256, 1000, 4000, 40_000], p=[.1, .1, .3, .2, .15, .1, .05]))
            i = int(rng.integers(0, len(desc) - n + 1))
            sub = np.ascontiguousarray(desc[i: i + n])
            kind = k % 3
            if kind == 0:
                pinned[:] = arena
                st = engine.update_host(pinned, sub)
                got = pinned
            elif kind == 1:
                work = arena.copy()
                st = engine.update_host(work, sub)
                got = work
            else:
                buf = arena.copy()
                offs = sub["off16"].astype(np.int64) * 16
                st = engine.update_host_frames(buf, offs, sub["len"].astype(np.uint32))
                got = buf
            assert np.array_equal(st, rst[i: i + n]), (k, kind, n)
            lo, hi = int(desc[i]["off16"]) * 16, int(desc[i + n - 1]["off16"]) * 16 + int(desc[i + n - 1]["len"])
            assert np.array_equal(got[lo:hi], ref[lo:hi]), (k, kind, n)
            assert np.array_equal(got[:lo], arena[:lo]) and np.array_equal(got[hi:], arena[hi:]), (k, kind, n)
    finally:
        engine.host_free(pinned)


@pytest.mark.parametrize("shift", [16, 4096, 1 << 20, 8, 3])
def test_pinned_arena_at_an_interior_address(engine, shift):
    """Round 6: a pinned burst of up to 32 MiB runs zero-copy by default, the kernel addressing the
    caller's arena through hipHostGetDevicePointer — here an arena that starts inside a pinned
    allocation (a slice of a pinned ring, as a NIC driver hands out), small bursts (direct, completion
    by flag) and one above 2 MiB; bytes and statuses the oracle's, the bytes before the arena untouched.
    An arena that is not 16-byte aligned (shift 8, 3) is staged through the copy engines instead."""
    frames = oracle.fuzz_frames(48, 0, 6000)
    arena, desc = oracle.pack_frames(frames)
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    pinned = engine.host_array(arena.nbytes + shift)
    try:
        junk = np.random.default_rng(shift).integers(0, 256, shift, dtype=np.uint8)
        for lo, hi in ((0, 3), (100, 164), (0, len(desc))):
            pinned[:shift] = junk
            view = pinned[shift:]
            view[:] = arena
            sub = np.ascontiguousarray(desc[lo:hi])
            st = engine.update_host(view, sub)
            assert np.array_equal(st, rst[lo:hi]), (lo, hi)
            a = int(desc[lo]["off16"]) * 16
            b = int(desc[hi - 1]["off16"]) * 16 + int(desc[hi - 1]["len"])
            assert np.array_equal(view[a:b], ref[a:b]), (lo, hi)
            assert np.array_equal(pinned[:shift], junk)
    finally:
        engine.host_free(pinned)
