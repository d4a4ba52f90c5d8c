"""The C ABI's error convention on a GPU (include/nfcs.h): where the reference's
void members return silently, every entry point here returns NFCS_OK or a negative NFCS_E* code
and never touches memory on a rejected call; per-packet problems (a descriptor outside the arena)
are status bytes, not call failures. Called straight through ctypes, as a foreign binding would."""
import ctypes

import numpy as np
import pytest

import netflow_amd as nf
import oracle

pytestmark = pytest.mark.gpu

OK, EINVAL = 0, -1


def _frames(n=64):
    return oracle.fuzz_frames(515, 0, n)


def test_null_and_empty_arguments(engine):
    L = nf.lib()
    d = engine.alloc(4096)
    assert L.nfcs_update_device(None, d.ptr, 4096, d.ptr, 1, None, None, None) == EINVAL
    assert L.nfcs_update_device(engine.ctx, None, 4096, d.ptr, 1, None, None, None) == EINVAL
    assert L.nfcs_update_device(engine.ctx, d.ptr, 4096, None, 1, None, None, None) == EINVAL
    # n = 0 is a no-op whatever the pointers
    assert L.nfcs_update_device(engine.ctx, None, 0, None, 0, None, None, None) == OK
    assert L.nfcs_flow_keys_device(engine.ctx, None, 0, None, 0, None, None, None) == OK
    assert L.nfcs_l3_forward_device(engine.ctx, None, 0, None, None, 0, None, 0, None, None) == OK
    assert L.nfcs_vlan_device(engine.ctx, None, 0, None, 0, None, 0, None, 0, None, None) == OK


def test_misaligned_pointers_are_rejected_untouched(engine):
    L = nf.lib()
    arena, desc = oracle.pack_frames(_frames())
    d_arena = engine.alloc(arena.nbytes + 64).upload(np.concatenate([arena, np.zeros(64, np.uint8)]))
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    n = len(desc)
    before = d_arena.download(np.uint8, arena.nbytes + 64)
    # arena not 16-byte aligned
    assert L.nfcs_update_device(engine.ctx, d_arena.ptr + 8, arena.nbytes, d_desc.ptr, n, None, None, None) == EINVAL
    assert L.nfcs_vlan_device(engine.ctx, d_arena.ptr + 4, arena.nbytes, d_desc.ptr, n, None,
                              nf.VLAN_POP, None, 64, None, None) == EINVAL
    # flow-key records must be 16-byte aligned
    d_keys = engine.alloc(64 * n + 16)
    assert L.nfcs_flow_keys_device(engine.ctx, d_arena.ptr, arena.nbytes, d_desc.ptr, n,
                                   d_keys.ptr + 4, None, None) == EINVAL
    # a next-hop table promised but missing
    d_nh = engine.alloc(4 * n)
    assert L.nfcs_l3_forward_device(engine.ctx, d_arena.ptr, arena.nbytes, d_desc.ptr, d_nh.ptr, n,
                                    None, 3, None, None) == EINVAL
    engine.sync()
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes + 64), before)


def test_host_path_argument_rules(engine):
    L = nf.lib()
    arena, desc = oracle.pack_frames(_frames())
    n = len(desc)
    before = arena.copy()
    # zero-copy needs a pinned arena; this one is pageable
    assert L.nfcs_update_host(engine.ctx, arena.ctypes.data, arena.nbytes, desc.ctypes.data, n, None,
                              nf.HOST_ZERO_COPY) == EINVAL
    assert np.array_equal(arena, before)
    # scattered frames: a NULL pointer array with n > 0, and a non-zero (reserved) flags word
    lens = np.ascontiguousarray(desc["len"])
    assert L.nfcs_update_host_frames(engine.ctx, None, lens.ctypes.data, n, None, 0) == EINVAL
    ptrs = (arena.ctypes.data + desc["off16"].astype(np.uint64) * 16).astype(np.uint64)
    assert L.nfcs_update_host_frames(engine.ctx, ptrs.ctypes.data, lens.ctypes.data, n, None, 1) == EINVAL
    assert np.array_equal(arena, before)


@pytest.mark.parametrize("n", [1, 70_000])
def test_scattered_frames_with_bad_arguments_are_rejected_untouched(engine, n):
    """nfcs_update_host_frames rejects reserved flags and NULL arrays with NFCS_EINVAL before anything
    is staged, and no frame is read or written (the frames here are 64-byte runts of one small
    buffer). A frame longer than a 64 MiB staging slot is no longer an error: since round 6 it goes
    as its first NFCS_FRAME_RELEVANT_BYTES, with the same result (test_gpu_host_ring.py
    test_scattered_frames_longer_than_a_staging_slot)."""
    L = nf.lib()
    buf = np.random.default_rng(n).integers(0, 256, 64 * 16, dtype=np.uint8)
    before = buf.copy()
    ptrs = (buf.ctypes.data + (np.arange(n, dtype=np.uint64) % 16) * 64).astype(np.uint64)
    lens = np.full(n, 64, dtype=np.uint32)
    status = np.full(n, 0xAB, dtype=np.uint8)
    assert L.nfcs_update_host_frames(engine.ctx, ptrs.ctypes.data, lens.ctypes.data, n, status.ctypes.data, 1) == EINVAL
    assert L.nfcs_update_host_frames(engine.ctx, None, lens.ctypes.data, n, status.ctypes.data, 0) == EINVAL
    assert L.nfcs_update_host_frames(engine.ctx, ptrs.ctypes.data, None, n, status.ctypes.data, 0) == EINVAL
    assert np.array_equal(buf, before)
    assert (status == 0xAB).all()


def test_host_path_takes_descriptors_in_any_order(engine):
    """Round 5: nfcs_update_host no longer requires arena order — descriptors
    in reverse order (every frame its own run of ascending offsets) give the oracle's bytes and
    statuses, per descriptor."""
    arena, desc = oracle.pack_frames(_frames())
    rev = np.ascontiguousarray(desc[::-1])
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, rev)
    st = engine.update_host(arena, rev)
    assert np.array_equal(st, rst) and np.array_equal(arena, ref)


def test_descriptor_outside_the_arena_is_a_status_not_an_error(engine):
    frames = _frames()
    arena, desc = oracle.pack_frames(frames)
    desc = desc.copy()
    desc[3]["off16"] = arena.nbytes // 16 + 1          # starts past the arena
    desc[5]["len"] = arena.nbytes                      # runs past the arena
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(desc.nbytes).upload(desc)
    d_st = engine.alloc(len(desc))
    engine.update_device(d_arena, arena.nbytes, d_desc, len(desc), d_st)  # raises on rc != 0
    engine.sync()
    st = d_st.download(np.uint8, len(desc))
    assert st[3] == nf.ST_BAD_DESC and st[5] == nf.ST_BAD_DESC
    assert np.array_equal(st, rst)
    assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)


def test_strerror_covers_every_code():
    L = nf.lib()
    for rc in (0, -1, -2, -3, -4):
        msg = L.nfcs_strerror(rc)
        assert isinstance(msg, bytes) and len(msg) > 0
    assert L.nfcs_abi_version() == 2
    assert isinstance(ctypes.c_int(L.nfcs_last_hip_error()).value, int)


def test_contexts_on_threads_are_independent():
    """One context per host thread on the same device (the documented threading model): four
    threads update their own batches concurrently, each bit-exact with the oracle."""
    import threading
    results = {}

    def work(t):
        frames = oracle.fuzz_frames(700 + t, 0, 20000)
        arena, desc = oracle.pack_frames(frames)
        ref = arena.copy()
        rst, _ = oracle.update_batch(ref, desc)
        with nf.Engine(0) as e:
            d_arena = e.alloc(arena.nbytes).upload(arena)
            d_desc = e.alloc(desc.nbytes).upload(desc)
            d_st = e.alloc(len(desc))
            e.update_device(d_arena, arena.nbytes, d_desc, len(desc), d_st)
            e.sync()
            results[t] = (bool(np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)),
                          bool(np.array_equal(d_st.download(np.uint8, len(desc)), rst)))

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert results == {t: (True, True) for t in range(4)}


def test_stream_read_reference(engine):
    """nfcs_time_stream_read (the bench's read-stream ceiling): every form times a read of a buffer
    and write nothing into it; bad arguments are rejected."""
    L = nf.lib()
    nbytes = 64 << 20
    host = np.random.default_rng(3).integers(0, 256, size=nbytes, dtype=np.uint8)
    d = engine.alloc(nbytes).upload(host)
    for form in (0, 1, 2, 3, 4, 5):
        ms = engine.time_stream_read(d, nbytes, 3, form=form)
        assert ms > 0
    assert np.array_equal(d.download(np.uint8, nbytes), host)
    # the frames-read form: the batch's frames in the read pass's pattern, nothing written
    desc = np.zeros(4097, dtype=nf.DESC_DTYPE)
    desc["off16"] = np.arange(4097, dtype=np.uint32) * 96
    desc["len"] = 1500
    desc["len"][7] = 9000  # a jumbo frame: continuation batches
    dd = engine.alloc(desc.nbytes).upload(desc)
    assert engine.time_frames_read(d, nbytes, dd, len(desc), 3) > 0
    assert np.array_equal(d.download(np.uint8, nbytes), host)
    dd.free()
    ms = ctypes.c_float()
    assert L.nfcs_time_stream_read(engine.ctx, d.ptr + 8, 4096, 0, 1, None, ctypes.byref(ms)) == EINVAL
    assert L.nfcs_time_stream_read(engine.ctx, d.ptr, 4096, 6, 1, None, ctypes.byref(ms)) == EINVAL
    assert L.nfcs_time_stream_read(engine.ctx, d.ptr, 4096, 0, 0, None, ctypes.byref(ms)) == EINVAL
    assert L.nfcs_time_stream_read(engine.ctx, None, 4096, 0, 1, None, ctypes.byref(ms)) == EINVAL


def test_timing_entries_with_no_packets(engine):
    """the time_* entry points reach the launch-shape choice, which divided the arena size
    by n: with n = 0 and no slot hint every one of them is a clean no-op (NFCS_OK, ~0 ms)."""
    L = nf.lib()
    d = engine.alloc(4096)
    ms = ctypes.c_float()
    engine.set_slot_bytes(0)
    assert L.nfcs_time_update_device(engine.ctx, d.ptr, 4096, d.ptr, 0, None, 2, None, ctypes.byref(ms)) == OK
    assert L.nfcs_time_l3_forward_device(engine.ctx, d.ptr, 4096, d.ptr, d.ptr, 0, d.ptr, 1, None, 2, None,
                                         ctypes.byref(ms)) == OK
    assert L.nfcs_time_vlan_device(engine.ctx, d.ptr, 4096, d.ptr, 0, 0, 0, 1536, None, 2, None,
                                   ctypes.byref(ms)) == OK
    assert L.nfcs_time_flow_keys_device(engine.ctx, d.ptr, 4096, d.ptr, 0, d.ptr, None, 2, None,
                                        ctypes.byref(ms)) == OK
    arenas = (ctypes.c_void_p * 1)(d.ptr)
    sizes = (ctypes.c_uint64 * 1)(4096)
    assert L.nfcs_time_update_batches(engine.ctx, 1, arenas, sizes, arenas, 0, 2, None, ctypes.byref(ms)) == OK
    assert engine.launch_footprint(4096, d, 0) == 4096
    # and the rotation's own argument rules
    assert L.nfcs_time_update_batches(engine.ctx, 0, arenas, sizes, arenas, 0, 2, None, ctypes.byref(ms)) == EINVAL
    bad = (ctypes.c_void_p * 1)(d.ptr + 8)
    assert L.nfcs_time_update_batches(engine.ctx, 1, bad, sizes, arenas, 1, 2, None, ctypes.byref(ms)) == EINVAL


def test_rotating_timing_matches_the_reference(engine):
    """nfcs_time_update_batches (the timing of bench.py's headline line and of its c4_shard / c3
    sub-lines): rotating over 3 batches of fuzz frames, every batch ends equal to the oracle's update
    of it."""
    bs, refs = [], []
    for k in range(3):
        arena, desc = oracle.pack_frames(oracle.fuzz_frames(600 + k, 0, 3000))
        ref = arena.copy()
        oracle.update_batch(ref, desc)
        bs.append((engine.alloc(arena.nbytes).upload(arena), arena.nbytes, engine.alloc(desc.nbytes).upload(desc)))
        refs.append(ref)
    n = 3000
    assert engine.time_update_batches(bs, n, 7) > 0
    for (a, nb, _), ref in zip(bs, refs):
        assert np.array_equal(a.download(np.uint8, nb), ref)
