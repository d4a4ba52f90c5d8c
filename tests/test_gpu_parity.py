"""GPU parity tests (run on the MI355X box: pytest -m gpu).

Every test drives the HIP kernels through the C ABI (netflow_amd -> libnfcs.so) and checks
the bytes against (a) fixtures produced by the REFERENCE implementation (tests/golden/) and
(b) the oracle restatement on the same seeded inputs. Integer work: everything is bit-exact.
"""
import json
import os

import numpy as np
import pytest

import netflow_amd as nf
import oracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
SEED = 20250620


def run_device(engine, arena: np.ndarray, desc: np.ndarray, want_patch=False):
    n = len(desc)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(max(desc.nbytes, 16)).upload(desc)
    d_st = engine.alloc(max(n, 16))
    d_pt = engine.alloc(max(8 * n, 16)) if want_patch else None
    engine.update_device(d_arena, arena.nbytes, d_desc, n, d_st, d_pt)
    engine.sync()
    out = d_arena.download(np.uint8, arena.nbytes)
    st = d_st.download(np.uint8, n)
    pt = d_pt.download(nf.PATCH_DTYPE, n) if want_patch else None
    return out, st, pt


def test_kat_frames_match_reference(engine):
    kat = json.load(open(os.path.join(GOLD, "kat.json")))
    names = sorted(kat)
    frames = [bytes.fromhex(kat[k]["in"]) for k in names]
    arena, desc = oracle.pack_frames(frames)
    out, st, _ = run_device(engine, arena, desc)
    got = oracle.unpack_frames(out, desc)
    for name, g, s in zip(names, got, st):
        assert g.hex() == kat[name]["out"], name
        assert s == kat[name]["status"], name


def test_fuzz_corpus_matches_reference_fixture(engine):
    z = np.load(os.path.join(GOLD, "fuzz_ref.npz"))
    frames = oracle.fuzz_frames(int(z["seed"]), 0, len(z["lens"]))
    arena, desc = oracle.pack_frames(frames)
    orig = arena.copy()
    out, st, _ = run_device(engine, arena, desc)
    assert np.array_equal(st, z["oracle_status"])
    L = oracle.lib()
    h = np.array([L.nfo_frame_hash(oracle._ptr(out[int(d["off16"]) * 16:]), int(d["len"])) for d in desc],
                 dtype=np.uint64)
    dom = (st & 0x3F) != 14
    bad = np.nonzero(h[dom] != z["hash_out"][dom])[0]
    assert len(bad) == 0, f"{len(bad)} frames differ from the reference, first {bad[:5]}"
    for i in np.nonzero(~dom)[0]:  # outside the parity domain: untouched
        o, ln = int(desc[i]["off16"]) * 16, int(desc[i]["len"])
        assert np.array_equal(out[o:o + ln], orig[o:o + ln])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_vs_oracle_fresh_seeds(engine, seed):
    frames = oracle.fuzz_frames(seed, 0, 50000)
    arena, desc = oracle.pack_frames(frames)
    ref = arena.copy()
    rst, rpt = oracle.update_batch(ref, desc, nthreads=8)
    out, st, pt = run_device(engine, arena, desc, want_patch=True)
    assert np.array_equal(st, rst)
    assert np.array_equal(out, ref)
    # patch records reproduce the update when applied to the original frames
    re = arena.copy()
    for i, d in enumerate(desc):
        o = int(d["off16"]) * 16
        if pt[i]["ip_off"] != 0xFFFF:
            re[o + int(pt[i]["ip_off"]): o + int(pt[i]["ip_off"]) + 2] = pt[i]["ip"]
        if pt[i]["l4_off"] != 0xFFFF:
            re[o + int(pt[i]["l4_off"]): o + int(pt[i]["l4_off"]) + 2] = pt[i]["l4"]
    assert np.array_equal(re, ref)


@pytest.mark.parametrize("cfg,align", [(0, 16), (1, 16), (2, 16), (3, 16), (1, 128), (3, 128), (2, 64)])
def test_config_batch_generator_and_update_vs_oracle(engine, cfg, align):
    n = {0: 1024, 1: 8192, 2: 2048, 3: 16384}[cfg]
    d_arena, nbytes, d_desc, hdesc = engine.config_batch(cfg, SEED, 12345, n, align)
    gen = d_arena.download(np.uint8, nbytes)
    o_arena, o_desc = oracle.gen_config(cfg, SEED, 12345, n, align)
    assert np.array_equal(hdesc, o_desc)
    assert np.array_equal(gen, o_arena[:nbytes]), "device generator != oracle generator"
    d_st = engine.alloc(n)
    engine.update_device(d_arena, nbytes, d_desc, n, d_st)
    engine.sync()
    rst, _ = oracle.update_batch(o_arena, o_desc, nthreads=8)
    assert np.array_equal(d_st.download(np.uint8, n), rst)
    assert np.array_equal(d_arena.download(np.uint8, nbytes), o_arena[:nbytes])


@pytest.mark.parametrize("cfg", [0, 1, 3, 2])
def test_full_size_digest_matches_reference(engine, cfg):
    """BASELINE sizes (C1 1M x 1500 B, C2 1M x 9000 B, C3 4M mixed): digest of the whole
    updated arena == the digest of the REFERENCE's output (tests/golden/configs.json)."""
    g = json.load(open(os.path.join(GOLD, "configs.json")))
    c = g["configs"][str(cfg)]
    n = c["n"]
    d_arena, nbytes, d_desc, _ = engine.config_batch(cfg, g["seed"], 0, n, 128 if cfg in (1, 3) else 16)
    din = engine.digest_device(d_arena, nbytes, d_desc, n, 0)
    assert f"{din:016x}" == c["digest_in"]
    d_st = engine.alloc(n)
    engine.update_device(d_arena, nbytes, d_desc, n, d_st)
    engine.sync()
    dout = engine.digest_device(d_arena, nbytes, d_desc, n, 0)
    assert f"{dout:016x}" == c["digest_out"]
    st = d_st.download(np.uint8, n)
    hist = {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}
    assert hist == c["oracle_status_hist"]
    # idempotence: a second pass changes nothing
    engine.update_device(d_arena, nbytes, d_desc, n, None)
    engine.sync()
    assert engine.digest_device(d_arena, nbytes, d_desc, n, 0) == dout
    d_arena.free()


def test_c1_rank_shard_digests(engine):
    """The per-rank shards bench.py uses at N GPUs (weak scaling) are bit-exact too."""
    g = json.load(open(os.path.join(GOLD, "configs.json")))
    for sh in g["c1_rank_shards"][:3]:
        d_arena, nbytes, d_desc, _ = engine.config_batch(1, g["seed"], sh["first"], sh["n"])
        engine.update_device(d_arena, nbytes, d_desc, sh["n"])
        engine.sync()
        assert f"{engine.digest_device(d_arena, nbytes, d_desc, sh['n'], sh['first']):016x}" == sh["digest_out"]
        d_arena.free()


def test_edge_cases(engine):
    frames = []
    kat = json.load(open(os.path.join(GOLD, "kat.json")))
    base = bytearray.fromhex(kat["B_packet_test_udp"]["in"])
    frames.append(b"")                                  # empty frame
    frames.append(bytes(1))
    frames.append(bytes(base[:33]))                      # one byte short of an IPv4 header + eth
    frames.append(bytes(base[:34]))                      # IPv4 header only, UDP header missing
    # maximum-size IPv4/TCP: total_length 65535 -> 65515-byte segment (odd), frame 65549 B
    big = bytearray(os.urandom(65549))
    big[12:14] = b"\x08\x00"; big[14] = 0x45; big[16:18] = b"\xff\xff"; big[23] = 6; big[46] = 0x50
    frames.append(bytes(big))
    # maximum-size UDP: udp.length 65535 inside a larger frame (trailing bytes ignored)
    bigu = bytearray(os.urandom(65535 + 34 + 100))
    bigu[12:14] = b"\x08\x00"; bigu[14] = 0x46; bigu[23] = 17; bigu[16:18] = b"\xff\xff"
    bigu[38 + 4 - 4 + 4:38 + 4 - 4 + 6] = b"\xff\xff"  # l4 = 38 (IHL 6): length at l4+4
    frames.append(bytes(bigu))
    # VLAN-tagged IPv6 UDP with odd payload; IPv6 jumbo TCP
    frames.append(bytes.fromhex(kat["J_ipv6_vlan_tcp"]["in"]))
    frames.append(bytes.fromhex(kat["I_ipv6_udp_data"]["in"]) + b"x")
    # alone (a short burst: one inline kernel) and followed by 70,000 64-byte frames (a batch past
    # kInlineMaxPackets: the waves holding the large frames defer to the write pass)
    filler = [bytes(base[:64])] * 70000
    for align, pad in ((16, False), (64, False), (4096, False), (16, True), (128, True)):
        arena, desc = oracle.pack_frames(frames + (filler if pad else []), align=align)
        ref = arena.copy()
        rst, _ = oracle.update_batch(ref, desc, nthreads=8)
        out, st, _ = run_device(engine, arena, desc)
        assert np.array_equal(st, rst), (align, pad)
        assert np.array_equal(out, ref), (align, pad)
    # descriptors in reverse / random order (device path accepts any order)
    frames = oracle.fuzz_frames(99, 0, 3000)
    arena, desc = oracle.pack_frames(frames)
    perm = np.random.default_rng(0).permutation(len(desc))
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc)
    out, st, _ = run_device(engine, arena, desc[perm])
    assert np.array_equal(out, ref) and np.array_equal(st, rst[perm])


def test_bad_descriptors_and_empty_batch(engine):
    frames = oracle.fuzz_frames(5, 0, 64)
    arena, desc = oracle.pack_frames(frames)
    desc = desc.copy()
    desc[3]["off16"] = arena.nbytes // 16          # starts at the end of the arena
    desc[7]["len"] = arena.nbytes + 1              # reaches past it
    ref = arena.copy()
    out, st, _ = run_device(engine, arena, desc)
    assert st[3] == nf.ST_BAD_DESC and st[7] == nf.ST_BAD_DESC
    # n == 0 is a no-op
    d = engine.alloc(64)
    engine.update_device(d, 64, d, 0)
    engine.sync()


@pytest.mark.parametrize("mode", ["patch", "frames"])
def test_host_path_pipeline(engine, mode):
    """nfcs_update_host: frames in pageable host memory, chunked through the pinned ring."""
    frames = oracle.fuzz_frames(11, 0, 40000)
    arena, desc = oracle.pack_frames(frames)
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    st = engine.update_host(arena, desc, mode=mode)
    assert np.array_equal(st, rst)
    assert np.array_equal(arena, ref)


def test_host_path_config_multi_chunk(engine):
    arena, desc = oracle.gen_config(1, SEED, 0, 120000)   # 180 MB -> several 64 MiB slots
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    st = engine.update_host(arena, desc)
    assert np.array_equal(st, rst) and np.array_equal(arena, ref)


@pytest.mark.parametrize("mode", ["zero_copy", "patch", "frames"])
def test_host_path_pinned(engine, mode):
    """nfcs_update_host on a pinned arena: zero-copy (the kernel reads the frames over PCIe in
    place and writes the checksum bytes back) or staged through the ring; fuzz frames incl. jumbo
    and out-of-arena descriptors."""
    frames = oracle.fuzz_frames(12, 0, 30000)
    packed, desc = oracle.pack_frames(frames)
    arena = engine.host_array(packed.nbytes)
    try:
        arena[:] = packed
        ref = packed.copy()
        rst, _ = oracle.update_batch(ref, desc, nthreads=8)
        st = engine.update_host(arena, desc, mode=mode)
        assert np.array_equal(st, rst)
        assert np.array_equal(arena, ref)
    finally:
        engine.host_free(arena)


def test_host_staging_numa(engine):
    """The staging ring of nfcs_update_host is placed on the GPU's NUMA node when sysfs names one
    (SURVEY.md §8e); a node it reports exists on this host."""
    node, local = engine.host_numa()
    print(f"gpu numa node {node}, staging bound to it: {local}")
    assert node >= -1
    if node >= 0:
        assert os.path.exists(f"/sys/devices/system/node/node{node}")


@pytest.mark.parametrize("mode", ["patch", "frames"])
def test_host_path_out_of_arena_descriptors_multi_chunk(engine, mode):
    """Descriptors reaching past a > 64 MiB arena (len 0xFFFFFFFF; a length past the end) become
    NFCS_ST_BAD_DESC in the middle of a multi-chunk staged call — every other frame as the oracle,
    no error return, nothing left in flight."""
    arena, desc = oracle.gen_config(1, SEED, 0, 50000)
    assert arena.nbytes > 64 << 20
    desc = desc.copy()
    desc[100]["len"] = 0xFFFFFFFF
    desc[30000]["len"] = arena.nbytes
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    assert rst[100] == nf.ST_BAD_DESC and rst[30000] == nf.ST_BAD_DESC
    st = engine.update_host(arena, desc, mode=mode)
    assert np.array_equal(st, rst)
    assert np.array_equal(arena, ref)


@pytest.mark.parametrize("mode", ["patch", "frames", "pinned", "zero_copy"])
def test_host_path_frame_larger_than_a_slot(engine, mode):
    """A frame inside the arena longer than a 64 MiB staging slot (round 6; NFCS_EINVAL before): it is
    staged as its first NFCS_FRAME_RELEVANT_BYTES, which gives the same bytes — the reference reads and
    bounds-tests no offset past 65,613 — so the whole arena, the frames around it and the frame's own
    65 MiB tail equal the oracle's update of the whole frames, in every host mode."""
    arena0, desc0 = oracle.gen_config(1, SEED, 0, 1000)
    frames = oracle.unpack_frames(arena0, desc0)
    rng = np.random.default_rng(5)
    huge = frames[500] + rng.integers(0, 256, (65 << 20) - len(frames[500]), dtype=np.uint8).tobytes()
    arena, desc = oracle.pack_frames(frames[:500] + [huge] + frames[500:])
    ref = arena.copy()
    rst, _ = oracle.update_batch(ref, desc, nthreads=8)
    if mode in ("pinned", "zero_copy"):
        host = engine.host_array(arena.nbytes)
        host[:] = arena
    else:
        host = arena
    try:
        st = engine.update_host(host, desc, mode={"pinned": "patch"}.get(mode, mode))
        assert np.array_equal(st, rst)
        assert np.array_equal(host, ref)
    finally:
        if host is not arena:
            engine.host_free(host)
