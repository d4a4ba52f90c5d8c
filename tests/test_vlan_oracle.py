"""CPU tests of the VLAN push/pop restatement (oracle nfo_vlan, packet.hpp:655-720) against the
reference's own output: tests/golden/kat_vlan.json and vlan_ref.npz were produced by the
reference's Packet::push_vlan / pop_vlan (tests/golden/make_golden.py, oracle/ref_shim.cpp)."""
import numpy as np
import pytest

import oracle
from vlan_common import random_vlan_case, vlan_fixture, vlan_kats, window_hashes


def run_kat_oracle(k):
    f = bytes.fromhex(k["in"])
    buf = oracle._vlan_buf(f, k["cap"])
    ln = np.array([len(f)], dtype=np.uint32)
    sts = [oracle.lib().nfo_vlan(oracle._ptr(buf), oracle._ptr(ln, oracle._u32p), k["cap"], op)
           for op in k["ops"]]
    return bytes(buf[:oracle.vlan_window(len(f))]), int(ln[0]), sts


def test_vlan_kat_matches_reference(oracle_lib):
    kat = vlan_kats()
    assert len(kat) >= 40
    for name, k in kat.items():
        out, ln, sts = run_kat_oracle(k)
        assert out.hex() == k["out"], name
        assert ln == k["len_out"], name
        assert sts == k["status"], name
        assert [s != 16 for s in sts] == [bool(r) for r in k["ret"]], name


def test_vlan_kat_reference_behaviours():
    """The reference test expectations on the same frames (packet_test.cpp:326-379)."""
    kat = vlan_kats()
    k = kat["C_packet_test_tcp/push_no_tailroom"]  # PushVlanNoHeadroom: false, unchanged
    assert k["ret"] == [0] and k["out"][: 2 * len(bytes.fromhex(k["in"]))] == k["in"]
    k = kat["C_packet_test_tcp/pop_untagged"]      # PopVlanOnNonVlanPacket: false
    assert k["ret"] == [0] and k["len_out"] == len(bytes.fromhex(k["in"]))
    k = kat["B_packet_test_udp/push202p3_pop"]     # phase2_l2_parsing.cpp:114-132
    assert k["ret"] == [1, 1] and k["len_out"] == len(bytes.fromhex(k["in"]))


def test_vlan_fixture_matches_reference(oracle_lib):
    z, frames = vlan_fixture()
    arena, desc = oracle.pack_frames(frames, room=4)
    d0 = desc.copy()
    st = oracle.vlan_batch(arena, desc, z["ops"], z["caps"])
    assert np.array_equal(st, z["oracle_status"])
    dom = (st & 0x1F) != 14
    assert np.array_equal(window_hashes(arena, d0)[dom], z["hash_window"][dom])
    assert np.array_equal(desc["len"][dom], z["len_out"][dom])
    assert np.array_equal((st[dom] != 16), z["ret"][dom] != 0)
    for s in (0, 16, 0x20, 0x22, 0x23, 0x24, 0x27, 0x28, 0x62, 0x63):
        assert (st == s).sum() > 20, hex(s)


@pytest.mark.skipif(not oracle.ref_available(), reason="reference shim not built here")
def test_vlan_oracle_vs_reference_fresh():
    frames, ops, caps = random_vlan_case(31, 3000)
    for i, f in enumerate(frames):
        o, st, win = oracle.vlan_frame(f, int(ops[i]), int(caps[i]))
        if (st & 0x1F) == 14:
            continue
        r, ok, rwin = oracle.ref_vlan_frame(f, int(ops[i]), int(caps[i]))
        assert win == rwin and o == r and (st != 16) == bool(ok or ops[i] == 0), i
