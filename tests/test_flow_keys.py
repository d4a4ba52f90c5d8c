"""Flow-key extract + hash (PacketClassifier::extract_flow_key / hash_flow,
packet_classifier.cpp:12-108). CPU: the oracle restatement against the
reference's own output (tests/golden/kat_flow.json, flow_ref.npz: produced by compiling
packet_classifier.cpp from the reference source). GPU: nfcs_flow_keys_device through the C ABI
against the same fixtures and the oracle, byte for byte."""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def record_digests(recs: np.ndarray) -> np.ndarray:
    L = oracle.lib()
    out = np.zeros(len(recs), dtype=np.uint64)
    buf = np.zeros(80, dtype=np.uint8)
    for i, r in enumerate(recs):
        buf[:64] = r
        out[i] = L.nfo_frame_hash(oracle._ptr(buf), 64)
    return out


def test_flow_kat_oracle_matches_reference(oracle_lib):
    kat = json.load(open(os.path.join(GOLD, "kat_flow.json")))
    for name, k in kat.items():
        rec, h = oracle.flow_key(bytes.fromhex(k["in"]))
        assert rec.hex() == k["record"], name
        assert h == k["hash"], name
    # the reference test's expectations (packet_classifier_test.cpp:174-244) hold in the records
    r = {n: np.frombuffer(bytes.fromhex(k["record"]), dtype=np.uint8) for n, k in kat.items()}
    assert r["arp"][6] == 0x06 and r["arp"][7] == 0x08            # ethertype 0x0806
    assert bytes(r["ipv4_proto0"][32:36]) == (0xC0A80101).to_bytes(4, "little")
    assert int.from_bytes(bytes(r["vlan101_ipv4_tcp"][4:6]), "little") == 101


def test_flow_fixture_oracle_matches_reference(oracle_lib):
    z = np.load(os.path.join(GOLD, "flow_ref.npz"))
    frames = oracle.fuzz_frames(int(z["seed"]), 0, len(z["lens"]))
    arena, desc = oracle.pack_frames(frames)
    recs, hashes = oracle.flow_keys_batch(arena, desc)
    assert np.array_equal(hashes, z["hash"])
    assert np.array_equal(record_digests(recs), z["record_digest"])


@pytest.mark.skipif(not oracle.ref_available(), reason="reference shim not built here")
def test_flow_oracle_vs_reference_fresh():
    for f in oracle.fuzz_frames(31, 0, 5000):
        assert oracle.flow_key(f) == oracle.ref_flow_key(f)


def run_flow(engine, arena, desc):
    import netflow_amd as nf
    n = len(desc)
    d_arena = engine.alloc(arena.nbytes).upload(arena)
    d_desc = engine.alloc(max(desc.nbytes, 16)).upload(desc)
    d_keys = engine.alloc(max(64 * n, 16))
    d_hash = engine.alloc(max(4 * n, 16))
    engine.flow_keys_device(d_arena, arena.nbytes, d_desc, n, d_keys, d_hash)
    engine.sync()
    return (d_keys.download(np.uint8, 64 * n).reshape(n, 64), d_hash.download(np.uint32, n))


@pytest.mark.gpu
def test_gpu_flow_kat(engine):
    kat = json.load(open(os.path.join(GOLD, "kat_flow.json")))
    names = sorted(kat)
    arena, desc = oracle.pack_frames([bytes.fromhex(kat[k]["in"]) for k in names])
    recs, hashes = run_flow(engine, arena, desc)
    for i, name in enumerate(names):
        assert bytes(recs[i]).hex() == kat[name]["record"], name
        assert int(hashes[i]) == kat[name]["hash"], name


@pytest.mark.gpu
@pytest.mark.parametrize("align", [16, 128])
def test_gpu_flow_fixture(engine, align):
    z = np.load(os.path.join(GOLD, "flow_ref.npz"))
    frames = oracle.fuzz_frames(int(z["seed"]), 0, len(z["lens"]))
    arena, desc = oracle.pack_frames(frames, align=align)
    recs, hashes = run_flow(engine, arena, desc)
    assert np.array_equal(hashes, z["hash"])
    assert np.array_equal(record_digests(recs), z["record_digest"])


@pytest.mark.gpu
def test_gpu_flow_fresh_and_bad_desc(engine):
    frames = oracle.fuzz_frames(41, 0, 40000)
    arena, desc = oracle.pack_frames(frames)
    desc = desc.copy()
    desc[7]["off16"] = arena.nbytes // 16 + 5   # past the arena: zero record, hash 0
    rrecs, rh = oracle.flow_keys_batch(arena, desc)
    recs, hashes = run_flow(engine, arena, desc)
    assert np.array_equal(hashes, rh) and rh[7] == 0
    assert np.array_equal(recs, rrecs)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 7, 9, 31, 33, 63, 65, 127, 129, 255, 257, 1001])
def test_gpu_flow_ragged_counts(engine, n):
    # a wave takes 64 packets (one lane each; headers loaded 8 per instruction), a workgroup 256:
    # counts that end mid-row, mid-wave and mid-workgroup
    frames = oracle.fuzz_frames(43, 0, n)
    arena, desc = oracle.pack_frames(frames)
    rrecs, rh = oracle.flow_keys_batch(arena, desc)
    recs, hashes = run_flow(engine, arena, desc)
    assert np.array_equal(hashes, rh)
    assert np.array_equal(recs, rrecs)


@pytest.mark.gpu
def test_gpu_flow_config_batch(engine):
    n = 1 << 16
    d_arena, nbytes, d_desc, hdesc = engine.config_batch(3, 20250620, 0, n, 128)
    arena, desc = oracle.gen_config(3, 20250620, 0, n, 128)
    rrecs, rh = oracle.flow_keys_batch(arena, desc)
    d_keys = engine.alloc(64 * n)
    engine.flow_keys_device(d_arena, nbytes, d_desc, n, d_keys, None)
    engine.sync()
    assert np.array_equal(d_keys.download(np.uint8, 64 * n).reshape(n, 64), rrecs)
