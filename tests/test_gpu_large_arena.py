"""The write-back store form of the checksum kernel (variant 30), which `nfcs_update_device`
chooses for arenas of at least 2 GiB (kWriteBackArenaBytes), against the oracle
and the reference: (a) forced on a fresh fuzz batch, byte for byte, status and patch records;
(b) chosen by size on BASELINE C4 shards (4M x 1500 B = 6.3 GB), whose whole-arena digests must
equal the reference's (tests/golden/configs.json, made from the compiled reference). Also split
mode (variant 8) forced on fuzz frames."""
import json
import os

import numpy as np
import pytest

import netflow_amd as nf
import oracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture
def wb_engine(monkeypatch):
    monkeypatch.setenv("NFCS_VARIANT", "30")  # read by nfcs_ctx_create
    e = nf.Engine(0)
    yield e
    e.close()


def test_write_back_form_fuzz_vs_oracle(wb_engine):
    frames = oracle.fuzz_frames(30, 0, 60000)
    for align in (16, 128):
        arena, desc = oracle.pack_frames(frames, align=align)
        ref = arena.copy()
        rst, _ = oracle.update_batch(ref, desc, nthreads=8)
        n = len(desc)
        d_arena = wb_engine.alloc(arena.nbytes).upload(arena)
        d_desc = wb_engine.alloc(desc.nbytes).upload(desc)
        d_st = wb_engine.alloc(n)
        d_pt = wb_engine.alloc(8 * n)
        wb_engine.update_device(d_arena, arena.nbytes, d_desc, n, d_st, d_pt)
        wb_engine.sync()
        assert np.array_equal(d_st.download(np.uint8, n), rst)
        assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)
        pt = d_pt.download(nf.PATCH_DTYPE, n)
        re = arena.copy()  # the patch records reproduce the update on the original frames
        for i in range(n):
            o = int(desc[i]["off16"]) * 16
            for f in ("ip", "l4"):
                if pt[i][f + "_off"] != 0xFFFF:
                    re[o + int(pt[i][f + "_off"]): o + int(pt[i][f + "_off"]) + 2] = pt[i][f]
        assert np.array_equal(re, ref)


@pytest.mark.parametrize("rank", [0, 7])
def test_c4_shard_digest_large_arena(engine, rank):
    g = json.load(open(os.path.join(GOLD, "configs.json")))
    sh = g["c4_rank_shards"][rank]
    n = sh["n"]
    d_arena, nbytes, d_desc, _ = engine.config_batch(1, g["seed"], sh["first"], n, 128)
    assert nbytes >= 2 << 30  # the size that selects the write-back form
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


def test_split_mode_fuzz_vs_oracle(monkeypatch):
    """Split mode forced on fuzz frames (variant 8: the product's form for large frames, chosen
    by size only for C2-like batches, so the fuzz corpus never reaches it on its own), byte for
    byte against the oracle over two successive calls."""
    monkeypatch.setenv("NFCS_VARIANT", "8")
    e = nf.Engine(0)
    try:
        frames = oracle.fuzz_frames(8, 0, 60000)
        for align in (16, 128):
            arena, desc = oracle.pack_frames(frames, align=align)
            n = len(desc)
            d_arena = e.alloc(arena.nbytes).upload(arena)
            d_desc = e.alloc(desc.nbytes).upload(desc)
            d_st = e.alloc(n)
            ref = arena.copy()
            # the second call runs over the updated frames; the oracle follows the same sequence (frames with IHL < 5 overlaps
            # change status on a second pass, in the reference as well)
            for _ in range(2):
                rst, _ = oracle.update_batch(ref, desc, nthreads=8)
                e.update_device(d_arena, arena.nbytes, d_desc, n, d_st)
                e.sync()
                assert np.array_equal(d_st.download(np.uint8, n), rst)
                assert np.array_equal(d_arena.download(np.uint8, arena.nbytes), ref)
    finally:
        e.close()


def test_zero_copy_large_pinned_arena(engine):
    """nfcs_update_host zero-copy over a pinned host arena of more than 2 GiB (1.4M C1 frames,
    128-byte aligned, 2.15 GB): the size rule picks the write-back form for a kernel whose frames
    live in host memory; statuses and every byte against the oracle."""
    n = 1_400_000
    src, desc = oracle.gen_config(1, 20250620, 0, n, 128)
    assert src.nbytes >= 2 << 30 and src.nbytes // n < 2048  # write-back form, not split mode
    pinned = engine.host_array(src.nbytes)
    pinned[:] = src
    rst, _ = oracle.update_batch(src, desc, nthreads=8)
    st = engine.update_host(pinned, desc, mode="zero_copy")
    assert np.array_equal(st, rst)
    assert np.array_equal(pinned, src)
