"""The checksum kernel's store forms against the oracle and the reference.

`nfcs_update_device` decides per wave of four packets, from their descriptor lengths alone: frames
averaging at least kDeferMeanBytes (1280) write 8-byte patch records and a second, write-only pass
stores them non-temporally; shorter frames store their bytes inline from the read pass. Covered:
(a) fuzz frames in arena order (a mix of both forms) and sorted by length (long runs that all defer,
short runs that all store inline), byte for byte with statuses and patch records, over two calls;
(b) the same burst placed at the start of a > 2 GiB arena gives the same bytes as in an exact-size
arena (the arena size never changes the result or the form); (c) BASELINE C4 shards (4M x 1500 B =
6.3 GB, every wave deferred) against the reference's digests; (d) two streams sharing one context's
deferred-store workspace; (e) zero-copy over a > 2 GiB pinned host arena (inline stores over PCIe).
"""
import json
import os

import numpy as np
import pytest

import netflow_amd as nf
import oracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEFER_MEAN = 1280  # kDeferMeanBytes (netflow_amd/csrc/nfcs_internal.h)


def deferred_waves(desc):
    """Which groups of 4 packets the kernel defers (its rule, restated for the test)."""
    lens = np.minimum(desc["len"].astype(np.int64), 0xFFFF)
    pad = (-len(lens)) % 4
    g = np.concatenate([lens, np.zeros(pad, np.int64)]).reshape(-1, 4).sum(axis=1)
    return g >= 4 * DEFER_MEAN


def apply_patches(arena, desc, pt):
    re = arena.copy()
    for i in range(len(desc)):
        o = int(desc[i]["off16"]) * 16
        for f in ("ip", "l4"):
            if pt[i][f + "_off"] != 0xFFFF:
                re[o + int(pt[i][f + "_off"]): o + int(pt[i][f + "_off"]) + 2] = pt[i][f]
    return re


@pytest.mark.parametrize("order", ["arena", "by_length"])
def test_store_forms_fuzz_vs_oracle(engine, order):
    frames = oracle.fuzz_frames(30, 0, 90000)  # above kInlineMaxPackets: per-wave forms apply
    if order == "by_length":
        frames = sorted(frames, key=len)
    for align in (16, 128):
        arena, desc = oracle.pack_frames(frames, align=align)
        dw = deferred_waves(desc)
        assert dw.any() and not dw.all()  # both forms in the same launch
        n = len(desc)
        d_arena = engine.alloc(arena.nbytes).upload(arena)
        d_desc = engine.alloc(desc.nbytes).upload(desc)
        d_st = engine.alloc(n)
        d_pt = engine.alloc(8 * n)
        ref = arena.copy()
        for call in range(2):  # the second call runs over the updated frames (IHL < 5 overlaps
            #                    change status on a second pass, in the reference as well)
            rst, _ = oracle.update_batch(ref, desc, nthreads=8)
            before = d_arena.download(np.uint8, arena.nbytes)
            # with caller patch records on the first call, into the workspace on the second
            engine.update_device(d_arena, arena.nbytes, d_desc, n, d_st, d_pt if call == 0 else None)
            engine.sync()
            assert np.array_equal(d_st.download(np.uint8, n), rst)
            assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)
            if call == 0:  # the records reproduce the update on the original frames
                assert np.array_equal(apply_patches(before, desc, d_pt.download(nf.PATCH_DTYPE, n)), ref)
        for b in (d_arena, d_desc, d_st, d_pt):
            b.free()


def test_small_burst_in_large_arena_same_bytes(engine):
    """A short-frame burst at the start of a > 2 GiB arena (the round-1 size rule would have changed
    the store form) and the same burst in its own exact-size arena: identical bytes and statuses,
    both equal to the oracle; likewise a long-frame burst."""
    for frames in (oracle.fuzz_frames(31, 0, 20000), [f for f in oracle.fuzz_frames(32, 0, 40000) if len(f) >= 1200]):
        arena, desc = oracle.pack_frames(frames, align=128)
        n = len(desc)
        ref = arena.copy()
        rst, _ = oracle.update_batch(ref, desc, nthreads=8)
        big = (2 << 30) + 4096
        outs = []
        for nbytes in (arena.nbytes, big):
            d_arena = engine.alloc(nbytes).upload(arena)
            d_desc = engine.alloc(desc.nbytes).upload(desc)
            d_st = engine.alloc(n)
            engine.update_device(d_arena, nbytes, d_desc, n, d_st)
            engine.sync()
            outs.append((d_arena.download(np.uint8, arena.nbytes), d_st.download(np.uint8, n)))
            for b in (d_arena, d_desc, d_st):
                b.free()
        for got, st in outs:
            assert np.array_equal(st, rst)
            assert np.array_equal(got, ref)


@pytest.mark.parametrize("rank", range(8))
def test_c4_shard_digest_large_arena(engine, rank):
    g = json.load(open(os.path.join(GOLD, "configs.json")))
    sh = g["c4_rank_shards"][rank]
    n = sh["n"]
    d_arena, nbytes, d_desc, hdesc = engine.config_batch(1, g["seed"], sh["first"], n, 128)
    assert deferred_waves(hdesc).all()
    assert f"{engine.digest_device(d_arena, nbytes, d_desc, n, sh['first']):016x}" == sh["digest_in"]
    engine.update_device(d_arena, nbytes, d_desc, n)
    engine.sync()
    dout = engine.digest_device(d_arena, nbytes, d_desc, n, sh["first"])
    assert f"{dout:016x}" == sh["digest_out"]
    engine.update_device(d_arena, nbytes, d_desc, n)  # idempotent
    engine.sync()
    assert engine.digest_device(d_arena, nbytes, d_desc, n, sh["first"]) == dout
    d_arena.free()
    d_desc.free()


def test_two_streams_share_the_workspace(engine):
    """Back-to-back calls on one context from two caller streams and the context's own stream, no
    caller patch records: all use the context's deferred-store workspace; each call on another
    stream than the previous one waits for that one's write pass (a caller stream's event is
    recorded by its call; the own stream's only when another stream comes). The streams come from
    the HIP runtime libnfcs.so is bound to: opened by its SONAME, the loader returns the copy
    already in the process."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    g = json.load(open(os.path.join(GOLD, "configs.json")))
    streams = []
    for _ in range(2):
        st = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(st)) == 0
        streams.append(st)

    class _S:
        def __init__(self, st):
            self.cuda_stream = st.value

        def synchronize(self):
            assert hip.hipStreamSynchronize(ctypes.c_void_p(self.cuda_stream)) == 0
    s1, s2 = _S(streams[0]), _S(streams[1])
    b1 = engine.config_batch(1, g["seed"], 0, 1 << 20, 128)
    b2 = engine.config_batch(1, g["seed"], 0, 1 << 20, 128)
    b0 = engine.config_batch(1, g["seed"], 0, 1 << 20, 128)
    b3 = engine.config_batch(1, g["seed"], 0, 1 << 20, 128)
    want = g["configs"]["1"]["digest_out"]
    for order in ((s1, s2), (None, s1, None, s2), (s1, None, s2, None)):
        bs = (b1, b2) if len(order) == 2 else (b0, b1, b3, b2)
        for b in bs:
            engine.gen_config_device(1, g["seed"], 0, 1 << 20, b[0], b[1], b[2])
        engine.sync()
        for b, st in zip(bs, order):  # no host sync between the calls
            engine.update_device(b[0], b[1], b[2], 1 << 20, stream=None if st is None else st.cuda_stream)
        s1.synchronize()
        s2.synchronize()
        engine.sync()
        for b in bs:
            assert f"{engine.digest_device(b[0], b[1], b[2], 1 << 20, 0):016x}" == want
    for b in (b0, b1, b2, b3):
        b[0].free()
        b[2].free()
    for st in streams:
        hip.hipStreamDestroy(st)


def test_zero_copy_large_pinned_arena(engine):
    """nfcs_update_host zero-copy over a pinned host arena of more than 2 GiB (1.4M C1 frames,
    128-byte aligned, 2.15 GB): the kernel reads the frames over PCIe and stores the checksum bytes
    inline (write-through); statuses and every byte against the oracle."""
    n = 1_400_000
    src, desc = oracle.gen_config(1, 20250620, 0, n, 128)
    assert src.nbytes >= 2 << 30
    pinned = engine.host_array(src.nbytes)
    try:
        pinned[:] = src
        rst, _ = oracle.update_batch(src, desc, nthreads=8)
        st = engine.update_host(pinned, desc, mode="zero_copy")
        assert np.array_equal(st, rst)
        assert np.array_equal(pinned, src)
    finally:
        engine.host_free(pinned)


@pytest.mark.parametrize("n", [1_500_000, 2 * 524_288 + 100])
def test_sub_batches_status_patch_and_digest(engine, n):
    """A long-frame batch past kSubBatchAbovePackets (C1-shaped packets from index 12,345: 1.5M =
    sub-batches of 512K, 512K and 476K; 1M + 100 = 512K, 512K and a 100-packet tail that runs as
    one inline kernel): statuses and caller patch records land at their packets' own indices, the
    status histogram and result digest equal the oracle's (pinned to the reference), and every
    record names the bytes now in its frame."""
    g = json.load(open(os.path.join(GOLD, "configs.json")))
    first = 12_345
    d_arena, nbytes, d_desc, hdesc = engine.config_batch(1, g["seed"], first, n, 128)
    din, dout, hist = oracle.config_digest(1, g["seed"], first, n, 8)
    assert engine.digest_device(d_arena, nbytes, d_desc, n, first) == din
    d_st, d_pt = engine.alloc(n), engine.alloc(8 * n)
    engine.update_device(d_arena, nbytes, d_desc, n, d_st, d_pt)
    engine.sync()
    assert engine.digest_device(d_arena, nbytes, d_desc, n, first) == dout
    st = d_st.download(np.uint8, n)
    vals, cnt = np.unique(st, return_counts=True)
    assert {int(v): int(c) for v, c in zip(vals, cnt)} == hist
    pt = d_pt.download(nf.PATCH_DTYPE, n)
    arena = d_arena.download(np.uint8, nbytes)
    base = hdesc["off16"].astype(np.int64) * 16
    for f in ("ip", "l4"):
        off = pt[f + "_off"].astype(np.int64)
        live = off != 0xFFFF
        assert live.all()  # every C1 packet has both fields
        for b in (0, 1):
            assert np.array_equal(arena[base[live] + off[live] + b], pt[f][live, b])
    for b in (d_arena, d_desc, d_st, d_pt):
        b.free()
