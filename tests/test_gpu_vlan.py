"""GPU parity of the VLAN push/pop + checksum path (nfcs_vlan_device) through
the C ABI against the reference's own output (tests/golden/kat_vlan.json, vlan_ref.npz, the C1
digests in configs.json) and against the oracle on fresh seeded inputs, byte for byte: the
frames, the arena bytes around them, the new lengths and the status bytes."""
import json
import os

import numpy as np
import pytest

import netflow_amd as nf
import oracle
from vlan_common import GOLD, random_vlan_case, vlan_fixture, vlan_kats, window_hashes

pytestmark = pytest.mark.gpu


class Batch:
    def __init__(self, engine, arena, desc, ops=None, caps=None):
        self.e, self.n, self.nbytes = engine, len(desc), arena.nbytes
        self.arena = engine.alloc(arena.nbytes).upload(arena)
        self.desc = engine.alloc(max(desc.nbytes, 16)).upload(desc)
        self.ops = None if ops is None else engine.alloc(max(4 * self.n, 16)).upload(
            np.ascontiguousarray(ops, dtype=np.uint32))
        self.caps = None if caps is None else engine.alloc(max(4 * self.n, 16)).upload(
            np.ascontiguousarray(caps, dtype=np.uint32))
        self.st = engine.alloc(max(self.n, 16))

    def run(self, op_all=0, cap_all=0):
        self.e.vlan_device(self.arena, self.nbytes, self.desc, self.n, self.ops, op_all, self.caps,
                           cap_all, self.st)
        self.e.sync()
        return self

    def result(self):
        return (self.arena.download(np.uint8, self.nbytes), self.desc.download(nf.DESC_DTYPE, self.n),
                self.st.download(np.uint8, self.n))


def test_vlan_kat_matches_reference(engine):
    kat = vlan_kats()
    names = sorted(kat)
    frames = [bytes.fromhex(kat[k]["in"]) for k in names]
    caps = np.array([kat[k]["cap"] for k in names], dtype=np.uint32)
    arena, desc = oracle.pack_frames(frames, room=4)
    d0 = desc.copy()
    steps = max(len(kat[k]["ops"]) for k in names)
    sts = []
    b = Batch(engine, arena, desc, np.zeros(len(names), np.uint32), caps)
    for s in range(steps):  # edit sequences: one launch per step (no-op once a sequence ends)
        ops = np.array([kat[k]["ops"][s] if s < len(kat[k]["ops"]) else 0 for k in names], np.uint32)
        b.ops.upload(ops)
        b.run()
        sts.append(b.result()[2])
    out, desc_out, _ = b.result()
    for i, name in enumerate(names):
        o, w = int(d0[i]["off16"]) * 16, oracle.vlan_window(len(frames[i]))
        assert out[o:o + w].tobytes().hex() == kat[name]["out"], name
        assert int(desc_out[i]["len"]) == kat[name]["len_out"], name
        assert [int(sts[s][i]) for s in range(len(kat[name]["ops"]))] == kat[name]["status"], name


@pytest.mark.parametrize("align", [16, 128])
def test_vlan_fixture_matches_reference(engine, align):
    z, frames = vlan_fixture()
    arena, desc = oracle.pack_frames(frames, align=align, room=4)
    d0 = desc.copy()
    out, desc_out, st = Batch(engine, arena, desc, z["ops"], z["caps"]).run().result()
    assert np.array_equal(st, z["oracle_status"])
    dom = (st & 0x1F) != 14
    h = window_hashes(out, d0)
    bad = np.nonzero(h[dom] != z["hash_window"][dom])[0]
    assert len(bad) == 0, f"{len(bad)} frames differ from the reference, first {np.nonzero(dom)[0][bad[:5]]}"
    assert np.array_equal(desc_out["len"][dom], z["len_out"][dom])


@pytest.mark.parametrize("seed", [41, 42, 43])
def test_vlan_fresh_vs_oracle(engine, seed):
    frames, ops, caps = random_vlan_case(seed, 20000)
    arena, desc = oracle.pack_frames(frames, room=4)
    ref, rdesc = arena.copy(), desc.copy()
    rst = oracle.vlan_batch(ref, rdesc, ops, caps)
    out, desc_out, st = Batch(engine, arena, desc, ops, caps).run().result()
    assert np.array_equal(st, rst)
    assert np.array_equal(desc_out, rdesc)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("config,n", [(1, 4096), (2, 2048), (3, 65536)])
def test_vlan_config_push_pop_vs_oracle(engine, config, n):
    """Uniform edits (no ops / caps arrays) on generated batches: push then pop, jumbo frames
    (C2) take the multi-batch path. Slots are 128-byte aligned, capacity = the slot."""
    d_arena, nbytes, d_desc, hdesc = engine.config_batch(config, 20250620, 0, n, 128)
    arena, desc = oracle.gen_config(config, 20250620, 0, n, 128)
    assert np.array_equal(d_arena.download(np.uint8, nbytes), arena[:nbytes])
    slot = {1: 1536, 2: 9088, 3: 128}[config]
    caps = None
    if config == 3:  # per-frame capacity = distance to the next frame (the slot), arena end for the last
        offs = hdesc["off16"].astype(np.int64) * 16
        caps = np.append(offs[1:], nbytes) - offs
    push = nf.vlan_push_op(3000 + config, 5)
    d_st = engine.alloc(n)
    d_caps = None if caps is None else engine.alloc(4 * n).upload(caps.astype(np.uint32))
    for op in (push, nf.VLAN_POP):
        rst = oracle.vlan_batch(arena, desc, None, caps, op_all=op, cap_all=slot)
        engine.vlan_device(d_arena, nbytes, d_desc, n, None, op, d_caps, slot, d_st)
        engine.sync()
        assert np.array_equal(d_st.download(np.uint8, n), rst)
        assert np.array_equal(d_desc.download(nf.DESC_DTYPE, n), desc)
        assert np.array_equal(d_arena.download(np.uint8, nbytes), arena[:nbytes])
        assert ((rst & 0x20) != 0).sum() > n * 0.99 if config != 3 else ((rst & 0x20) != 0).sum() > 0


def test_vlan_c1_digests_match_reference(engine):
    """Full BASELINE C1 size (1M x 1500 B, 1536-byte slots): push_vlan(100, 3) on every frame,
    then pop_vlan(), digests equal the reference's (configs.json vlan_c1); push + pop gives
    back update_checksums() of the original frames (the C1 reference digest)."""
    g = json.load(open(os.path.join(GOLD, "configs.json")))
    v = g["vlan_c1"]
    n = v["n"]
    d_arena, nbytes, d_desc, _ = engine.config_batch(1, 20250620, 0, n, v["align"])
    d_st = engine.alloc(n)
    engine.vlan_device(d_arena, nbytes, d_desc, n, None, nf.vlan_push_op(100, 3), None, v["cap"], d_st)
    engine.sync()
    st = d_st.download(np.uint8, n)
    assert (st == (0x20 | nf.ST_V4_UDP)).all()
    assert f"{engine.digest_device(d_arena, nbytes, d_desc, n, 0):016x}" == v["digest_push"]
    assert (d_desc.download(nf.DESC_DTYPE, n)["len"] == 1504).all()
    engine.vlan_device(d_arena, nbytes, d_desc, n, None, nf.VLAN_POP, None, v["cap"], d_st)
    engine.sync()
    got = f"{engine.digest_device(d_arena, nbytes, d_desc, n, 0):016x}"
    assert got == v["digest_push_pop"] == g["configs"]["1"]["digest_out"]


def test_vlan_bad_descriptor_and_nop(engine):
    frames = [bytes(range(64)), bytes(60)]
    arena, desc = oracle.pack_frames(frames, room=4)
    desc[1]["off16"] = 10_000  # outside the arena
    b = Batch(engine, arena, desc).run(op_all=nf.vlan_push_op(1), cap_all=2048)
    out, dout, st = b.result()
    assert list(st) == [nf.ST_FLAG_VLAN | nf.ST_NONE, nf.ST_BAD_DESC]
    b2 = Batch(engine, arena, oracle.pack_frames(frames, room=4)[1]).run(op_all=nf.VLAN_NOP, cap_all=2048)
    out2, dout2, st2 = b2.result()
    assert list(st2) == [0, 0] and np.array_equal(out2, arena)
