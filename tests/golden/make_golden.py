"""Generate the golden fixtures in tests/golden/ from the REFERENCE implementation.

Run in the build container (needs /root/reference):   python tests/golden/make_golden.py

It compiles the reference checksum path (header-only, include/netflow++/packet.hpp, never
copied) through oracle/ref_shim.cpp into oracle/_ref/libnfref.so and records what the
reference does on:
  kat.json          the SURVEY.md Appendix-B known-answer frames (+ KAT-G/H edge cases and
                    the reference's own tests/packet_test.cpp builder frames), full in/out hex
  fuzz_ref.npz      N fuzz frames (oracle.nfo_fuzz_frame, seed FUZZ_SEED): per frame the
                    length, frame_hash before and after the reference's update_checksums()
  configs.json      digests of the synthetic configs C0..C3 before/after the
                    reference, at full BASELINE sizes, plus per-rank shards for multi-GPU
  l3fwd_ref.npz     the fused L3 forward (switch.hpp:247-294 data path: TTL check/decrement,
  kat_l3.json       MAC rewrite, update_checksums()) through the reference's Packet on fuzz
                    frames with TTL overrides and next-hop indexes, and on the KAT frames
  kat_flow.json     PacketClassifier::extract_flow_key + hash_flow (packet_classifier.cpp,
  flow_ref.npz      compiled from the reference source) on builder-shaped frames and on fuzz
                    frames: 64-byte records (nfcs_flow_key layout) and hashes
  kat_vlan.json     Packet::push_vlan / pop_vlan + update_checksums (packet.hpp:655-720) on
  vlan_ref.npz      edit sequences over KAT frames and on fuzz frames with per-frame edits and
                    buffer capacities: the buffer window after the edit, new length, return
  configs.json      (c4) also the digests of the 8 C4 rank shards (4M x 1500 B each)
The fixtures are data only: frames in, frames/hashes out.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
FUZZ_SEED = 20250620
FUZZ_N = 65536
CONFIG_SEED = 20250620
CHUNK = 1 << 16


def be16(v):
    return bytes([(v >> 8) & 0xFF, v & 0xFF])


def kat_frames():
    k = {}
    k["A_main_cpp_tcp"] = bytes.fromhex(  # src/main.cpp:319-341
        "0000000000aa0000000000bb0800450000281234000040060000c0a80101c0a8010a"
        "3039005000000000000000005000000000000000")
    k["B_packet_test_udp"] = bytes.fromhex(
        "aabbccddeeff0011223344550800450000200001000040110000c0a8010ac0a80114d4310035000c000044415441")
    k["C_packet_test_tcp"] = bytes.fromhex(
        "aabbccddeeff0011223344550800450000280001000040060000c0a8010ac0a801143039005000000000"
        "000000000000000050000000" "54455354")
    k["D_icmp_odd"] = bytes.fromhex(
        "00000000000000000000000008004500001d000000004001000000000000000000000800000000000000ab")
    k["E_udp_odd_ABC"] = bytes.fromhex(
        "aabbccddeeff00112233445508004500001f00010000401100000a0000010a00000204d2162e000b0000414243")
    k["F_vlan_udp"] = bytes.fromhex(
        "aabbccddeeff0011223344558100a0650800450000200001000040110000c0a8010ac0a80114d4310035000c000044415441")
    # G: UDP whose sum folds to 0xFFFF -> checksum 0 -> stored 0xFFFF (packet.hpp:867-871)
    eth = bytes(12) + b"\x08\x00"
    ip = bytes([0x45, 0]) + be16(30) + bytes(4) + bytes([64, 17]) + bytes(2) + bytes([10, 0, 0, 1, 10, 0, 0, 2])
    udp_wo = be16(4660) + be16(53) + be16(10) + bytes(2)
    s = 0x0A00 + 0x0001 + 0x0A00 + 0x0002 + 17 + 10
    s += 4660 + 53 + 10
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    w = 0xFFFF - s
    k["G_udp_zero_to_ffff"] = eth + ip + udp_wo + be16(w)
    # H: ICMP all-zero 8-byte message (exact zero sum -> 0xFFFF) and the 0xFFFF-sum twin (-> 0)
    iph = bytes([0x45, 0]) + be16(28) + bytes(4) + bytes([64, 1]) + bytes(2) + bytes([10, 0, 0, 1, 10, 0, 0, 2])
    k["H1_icmp_all_zero"] = eth + iph + bytes(8)
    k["H2_icmp_sum_ffff"] = eth + iph + bytes(4) + b"\xff\xff" + bytes(2)
    # reference test builder frames (tests/packet_test.cpp:82-138, 140-176)
    k["I_ipv6_udp_data"] = bytes.fromhex(
        "aabbccddeeff001122334455" "86dd" "60000000000c1140"
        "20010db885a3000000008a2e03707334" "20010db885a3000000008a2e03707335"
        "d4310035000c0000" "44415441")
    k["J_ipv6_vlan_tcp"] = bytes.fromhex(
        "aabbccddeeff001122334455" "8100a065" "86dd" "600000000018063f"
        "20010db885a3000000008a2e03707334" "20010db885a3000000008a2e03707335"
        "30390050000000010000000250180100abcd0000" "74657374")
    k["K_ipv4_ihl7_tcp"] = bytes.fromhex(
        "aabbccddeeff001122334455" "0800" "4700003500010000400600000a0000010a000002" "0102030405060708"
        "303900500000000100000002601801001111000000000000" "7a")[:14 + 28 + 24 + 1]
    k["L_short_13B"] = bytes(13)
    k["M_ipv4_ihl2_udp_overlap"] = bytes.fromhex(
        "aabbccddeeff001122334455" "0800" "42000020000100004011aaaa0a0000010a000002" "0004000c0000" "41424344")
    return k


def make_kat(R):
    out = {}
    for name, fr in kat_frames().items():
        o_ref = oracle.ref_update_frame(fr)
        o_orc, st = oracle.update_frame(fr)
        assert o_ref == o_orc, name
        out[name] = {"in": fr.hex(), "out": o_ref.hex(), "status": st}
    with open(os.path.join(OUT, "kat.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("kat.json:", len(out), "frames")


def make_fuzz(R):
    L = oracle.lib()
    frames = oracle.fuzz_frames(FUZZ_SEED, 0, FUZZ_N)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    h_in = np.zeros(FUZZ_N, dtype=np.uint64)
    h_out = np.zeros(FUZZ_N, dtype=np.uint64)
    st = np.zeros(FUZZ_N, dtype=np.uint8)
    for i, f in enumerate(frames):
        b = np.frombuffer(f + bytes(16), dtype=np.uint8).copy()
        h_in[i] = L.nfo_frame_hash(oracle._ptr(b), len(f))
        _, s = oracle.update_frame(f)
        st[i] = s
        if (s & 0x3F) == 14:  # outside the reference's defined domain
            h_out[i] = 0
            continue
        o = oracle.ref_update_frame(f)
        ob = np.frombuffer(o + bytes(16), dtype=np.uint8).copy()
        h_out[i] = L.nfo_frame_hash(oracle._ptr(ob), len(f))
    np.savez_compressed(os.path.join(OUT, "fuzz_ref.npz"), seed=np.uint64(FUZZ_SEED), lens=lens,
                        hash_in=h_in, hash_out=h_out, oracle_status=st)
    print("fuzz_ref.npz:", FUZZ_N, "frames; statuses", np.unique(st, return_counts=True))


L3_SEED = 20250621
L3_N = 32768


def l3_table():
    """8 next hops {dst[6], src[6]} (fixed bytes)."""
    rng = np.random.default_rng(L3_SEED)
    return rng.integers(0, 256, size=(8, 12), dtype=np.uint8)


def l3_inputs(n=L3_N):
    """Fuzz frames (seed L3_SEED) with a TTL override and a next-hop index per frame:
    ttl_set[i] = 255 means no override, else the TTL byte at l2+8 is set to it (frames long
    enough); nh_index = i % 9 (8 = no route)."""
    frames = oracle.fuzz_frames(L3_SEED, 0, n)
    ttl_set = np.full(n, 255, dtype=np.uint8)
    ttl_set[0::5] = 1
    ttl_set[1::7] = 0
    ttl_set[2::11] = 2
    out = []
    for i, f in enumerate(frames):
        b = bytearray(f)
        l2 = 18 if len(b) >= 14 and b[12:14] == b"\x81\x00" else 14
        if ttl_set[i] != 255 and len(b) > l2 + 8:
            b[l2 + 8] = int(ttl_set[i])
        out.append(bytes(b))
    nh_index = (np.arange(n) % 9).astype(np.uint32)
    return out, ttl_set, nh_index


def make_l3(R):
    """Fused L3 forward (switch.hpp:247-294 data path) through the reference's Packet."""
    L = oracle.lib()
    table = l3_table()
    frames, ttl_set, nh_index = l3_inputs()
    n = len(frames)
    h_in = np.zeros(n, dtype=np.uint64)
    h_out = np.zeros(n, dtype=np.uint64)
    fwd = np.zeros(n, dtype=np.uint8)
    st = np.zeros(n, dtype=np.uint8)
    for i, f in enumerate(frames):
        nh = bytes(table[nh_index[i]]) if nh_index[i] < 8 else None
        b = np.frombuffer(f + bytes(16), dtype=np.uint8).copy()
        h_in[i] = L.nfo_frame_hash(oracle._ptr(b), len(f))
        o_orc, s = oracle.l3_forward_frame(f, nh)
        st[i] = s
        if (s & 0x3F) == 14:  # outside the reference's defined domain (IHL past the frame)
            continue
        o, fw = oracle.ref_l3_forward_frame(f, nh)
        assert o == o_orc and fw == (1 if s & 0x80 else 0), i
        fwd[i] = fw
        ob = np.frombuffer(o + bytes(16), dtype=np.uint8).copy()
        h_out[i] = L.nfo_frame_hash(oracle._ptr(ob), len(f))
    np.savez_compressed(os.path.join(OUT, "l3fwd_ref.npz"), seed=np.uint64(L3_SEED),
                        lens=np.array([len(f) for f in frames], dtype=np.uint16), ttl_set=ttl_set,
                        nh_index=nh_index, table=table, hash_in=h_in, hash_out=h_out,
                        forwarded=fwd, oracle_status=st)
    print("l3fwd_ref.npz:", n, "frames; statuses", np.unique(st, return_counts=True))
    # known answers: the KAT frames forwarded through next hop 0, plus drop cases
    kats = {}
    for name, fr in kat_frames().items():
        for tag, nh in (("fwd", bytes(table[0])), ("noroute", None)):
            o, fw = oracle.ref_l3_forward_frame(fr, nh)
            o2, s = oracle.l3_forward_frame(fr, nh)
            assert o == o2
            kats[f"{name}/{tag}"] = {"in": fr.hex(), "nh": None if nh is None else nh.hex(),
                                     "out": o.hex(), "forwarded": fw, "status": s}
    ttl1 = bytearray(kat_frames()["B_packet_test_udp"])
    ttl1[22] = 1
    o, fw = oracle.ref_l3_forward_frame(bytes(ttl1), bytes(table[1]))
    kats["B_packet_test_udp/ttl1"] = {"in": bytes(ttl1).hex(), "nh": bytes(table[1]).hex(),
                                      "out": o.hex(), "forwarded": fw,
                                      "status": oracle.l3_forward_frame(bytes(ttl1), bytes(table[1]))[1]}
    with open(os.path.join(OUT, "kat_l3.json"), "w") as fh:
        json.dump(kats, fh, indent=1, sort_keys=True)
    print("kat_l3.json:", len(kats), "cases")
    # bench workload: C1, one fused forward, next hop i % 9 of l3_table() (8 = no route)
    res = json.load(open(os.path.join(OUT, "configs.json")))
    n = 1 << 20
    M = (1 << 64) - 1
    dout = 0
    tab = np.ascontiguousarray(table.reshape(-1))
    for lo in range(0, n, CHUNK):
        m = min(CHUNK, n - lo)
        arena, desc = oracle.gen_config(1, CONFIG_SEED, lo, m)
        nh = ((np.arange(lo, lo + m)) % 9).astype(np.uint32)
        R.nfref_l3_forward_batch(oracle._ptr(arena), desc.ctypes.data, oracle._ptr(nh, oracle._u32p),
                                 m, oracle._ptr(tab), 8, 8)
        dout = (dout + oracle.digest(arena, desc, lo)) & M
    res["l3fwd_c1"] = {"first": 0, "n": n, "nh": "i % 9 (8 = no route), table = l3_table()",
                       "table": table.tobytes().hex(), "digest_out": f"{dout:016x}"}
    with open(os.path.join(OUT, "configs.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(f"l3fwd C1 digest {dout:016x}")


FLOW_SEED = 20250622
FLOW_N = 32768


def flow_kat_frames():
    """Frames shaped like the reference's packet_classifier_test.cpp builders (Ethernet / VLAN /
    IPv4 / IPv6 / TCP / UDP helpers at :16-146, MACs and IPv6 addresses of its fixture :158-167)."""
    sm, dm = bytes([0, 1, 2, 3, 4, 5]), bytes([0xAA, 0xBB, 0xCC, 0xDD, 0xEE, 0xFF])
    s6 = bytes([0x20, 0x01, 0x0D, 0xB8] + [0] * 11 + [1])
    d6 = bytes([0x20, 0x01, 0x0D, 0xB8] + [0] * 11 + [2])

    def eth(et):
        return dm + sm + be16(et)

    def vlan(vid, prio, et):
        return be16((prio << 13) | vid) + be16(et)

    def ip4(src, dst, proto, tl=20):
        return bytes([0x45, 0]) + be16(tl) + be16(12345) + bytes(2) + bytes([64, proto]) + bytes(2) + \
            src.to_bytes(4, "big") + dst.to_bytes(4, "big")

    def ip6(nh, plen=0):
        return (6 << 28).to_bytes(4, "big") + be16(plen) + bytes([nh, 64]) + s6 + d6

    def tcp(sp, dp):
        return be16(sp) + be16(dp) + (1000).to_bytes(4, "big") + bytes(4) + bytes([0x50, 0]) + \
            be16(8192) + bytes(4)

    def udp(sp, dp):
        return be16(sp) + be16(dp) + be16(8) + bytes(2)

    k = {}
    k["arp"] = eth(0x0806) + bytes(28)
    k["ipv4_proto0"] = eth(0x0800) + ip4(0xC0A80101, 0xC0A80102, 0)
    k["ipv6_nh0"] = eth(0x86DD) + ip6(0)
    k["vlan101_ipv4_tcp"] = eth(0x8100) + vlan(101, 3, 0x0800) + ip4(0x0A000001, 0x0A000002, 6, 40) + tcp(12345, 80)
    k["ipv4_tcp"] = eth(0x0800) + ip4(0xC0A80101, 0xC0A80102, 6, 40) + tcp(1024, 443)
    k["ipv4_udp"] = eth(0x0800) + ip4(0xC0A80101, 0xC0A80102, 17, 28) + udp(5353, 53)
    k["ipv6_tcp"] = eth(0x86DD) + ip6(6, 20) + tcp(40000, 22)
    k["ipv6_udp"] = eth(0x86DD) + ip6(17, 8) + udp(546, 547)
    k["vlan_ipv6_udp"] = eth(0x8100) + vlan(4095, 7, 0x86DD) + ip6(17, 8) + udp(1, 2)
    k["ipv4_tcp_19B_edge"] = (eth(0x0800) + ip4(1, 2, 6, 39) + tcp(7, 9))[:14 + 20 + 19]
    k["ipv4_tcp_18B_short"] = (eth(0x0800) + ip4(1, 2, 6, 38) + tcp(7, 9))[:14 + 20 + 18]
    k["vlan_runt"] = eth(0x8100) + bytes(2)
    k["runt_13"] = eth(0x0800)[:13]
    k["ipv4_ihl7_udp"] = eth(0x0800) + bytes([0x47, 0]) + be16(36) + bytes(4) + bytes([64, 17]) + \
        bytes(2) + bytes([1, 2, 3, 4, 5, 6, 7, 8]) + bytes(8) + udp(11, 22)
    return k


def make_flow(R):
    """Flow key + hash (packet_classifier.cpp:12-108) through the reference's PacketClassifier."""
    L = oracle.lib()
    kats = {}
    for name, fr in flow_kat_frames().items():
        rec, h = oracle.ref_flow_key(fr)
        assert (rec, h) == oracle.flow_key(fr), name
        kats[name] = {"in": fr.hex(), "record": rec.hex(), "hash": h}
    with open(os.path.join(OUT, "kat_flow.json"), "w") as fh:
        json.dump(kats, fh, indent=1, sort_keys=True)
    frames = oracle.fuzz_frames(FLOW_SEED, 0, FLOW_N)
    hashes = np.zeros(FLOW_N, dtype=np.uint32)
    rdig = np.zeros(FLOW_N, dtype=np.uint64)
    for i, f in enumerate(frames):
        rec, h = oracle.ref_flow_key(f)
        assert (rec, h) == oracle.flow_key(f), i
        hashes[i] = h
        rb = np.frombuffer(rec + bytes(16), dtype=np.uint8).copy()
        rdig[i] = L.nfo_frame_hash(oracle._ptr(rb), 64)
    np.savez_compressed(os.path.join(OUT, "flow_ref.npz"), seed=np.uint64(FLOW_SEED),
                        lens=np.array([len(f) for f in frames], dtype=np.uint16), hash=hashes,
                        record_digest=rdig)
    print("kat_flow.json:", len(kats), "frames; flow_ref.npz:", FLOW_N, "frames,",
          len(np.unique(hashes)), "distinct hashes")


VLAN_SEED = 20250623
VLAN_N = 32768


def vlan_inputs(n=VLAN_N, seed=VLAN_SEED):
    """Fuzz frames (25% tagged, IPv6, IHL 0-15, runts, jumbo) with one edit word and one buffer
    capacity each: 40% push (random id / priority), 40% pop, 10% no edit, 10% push into a buffer
    without tailroom; capacities len+4..len+68, exactly len+4, len..len+3 (no room) or 65536."""
    frames = oracle.fuzz_frames(seed, 0, n)
    rng = np.random.default_rng(seed)
    ops = np.zeros(n, dtype=np.uint32)
    caps = np.zeros(n, dtype=np.uint32)
    for i, f in enumerate(frames):
        r, c = rng.random(), rng.random()
        vid, prio = int(rng.integers(0, 8192)), int(rng.integers(0, 8))
        if r < 0.4 or r >= 0.9:
            ops[i] = oracle.vlan_op("push", vid, prio)
        elif r < 0.8:
            ops[i] = oracle.vlan_op("pop")
        ln = len(f)
        if r >= 0.9 or c < 0.15:
            caps[i] = ln + int(rng.integers(0, 4))
        elif c < 0.65:
            caps[i] = ln + 4 + int(rng.integers(0, 65))
        elif c < 0.9:
            caps[i] = ln + 4
        else:
            caps[i] = 65536
    return frames, ops, caps


def vlan_kat_frames():
    """(name -> (frame, [ops], cap)): the reference's own push/pop uses (phase2_l2_parsing.cpp:114
    push_vlan(202, 3) then pop_vlan(); packet_test.cpp:326-379 no tailroom / nothing to pop;
    vlan_manager.cpp:90 ingress push of a native VLAN, :159/:174 egress pops) on the KAT frames,
    plus runts, DEI preservation, IP options and IHL < 5 after the edit, and a jumbo frame."""
    k = kat_frames()
    P = lambda vid, prio=0: oracle.vlan_op("push", vid, prio)
    POP = oracle.vlan_op("pop")
    out = {}
    for name in ("A_main_cpp_tcp", "B_packet_test_udp", "C_packet_test_tcp", "D_icmp_odd",
                 "E_udp_odd_ABC", "G_udp_zero_to_ffff", "H1_icmp_all_zero", "I_ipv6_udp_data",
                 "K_ipv4_ihl7_tcp", "M_ipv4_ihl2_udp_overlap"):
        f = k[name]
        out[f"{name}/push202p3_pop"] = (f, [P(202, 3), POP], len(f) + 4)
        out[f"{name}/push_no_tailroom"] = (f, [P(10)], len(f))
        out[f"{name}/pop_untagged"] = (f, [POP], len(f) + 64)
    for name in ("F_vlan_udp", "J_ipv6_vlan_tcp"):
        f = k[name]
        out[f"{name}/pop"] = (f, [POP], len(f))
        out[f"{name}/retag4095p7"] = (f, [P(4095, 7)], len(f))
        out[f"{name}/pop_push1"] = (f, [POP, P(1, 0)], len(f))
    dei = bytearray(k["F_vlan_udp"])
    dei[14] |= 0x10  # DEI bit set: set_vlan_id / set_priority keep it (packet.hpp:185-190)
    out["F_dei/retag7p2"] = (bytes(dei), [P(7, 2)], len(dei))
    tag = bytes(12) + b"\x81\x00"
    out["tagged_len14/retag"] = (tag, [P(0xABC, 5)], 14)  # writes TCI bytes 14-15 past len
    out["tagged_len15/retag"] = (tag + b"\x42", [P(0x123, 1)], 15)
    out["tagged_len17/pop"] = (tag + b"\x11\x22\x33", [POP], 17)
    out["tagged_len18/pop"] = (tag + bytes.fromhex("e0010800"), [POP], 18)
    out["untagged_len13/push"] = (bytes(12) + b"\x08", [P(5)], 64)
    out["untagged_len14/push"] = (bytes(12) + b"\x08\x00", [P(5)], 18)
    out["untagged_len14/push_cap17"] = (bytes(12) + b"\x08\x00", [P(5)], 17)
    jumbo = oracle.gen_config(2, CONFIG_SEED, 7, 1)[0][:9000].tobytes()
    out["C2_jumbo/push_pop"] = (jumbo, [P(300, 2), POP], 9004)
    out["C2_jumbo/push"] = (jumbo, [P(300, 2)], 9004)
    c1 = oracle.gen_config(1, CONFIG_SEED, 3, 1)[0][:1500].tobytes()
    out["C1/push"] = (c1, [P(100, 6)], 1504)
    odd = oracle.gen_config(3, CONFIG_SEED, 11, 1)
    oddf = odd[0][:int(odd[1][0]["len"])].tobytes()
    out["C3/push_pop"] = (oddf, [P(42), POP], len(oddf) + 4)
    return out


def make_vlan(R):
    """VLAN push / pop + update_checksums (packet.hpp:655-720) through the reference's Packet."""
    L = oracle.lib()
    kats = {}
    for name, (f, ops, cap) in vlan_kat_frames().items():
        cur, rets, sts = f, [], []
        buf_r = oracle._vlan_buf(f, cap)
        buf_o = buf_r.copy()
        ln_r = np.array([len(f)], dtype=np.uint32)
        ln_o = ln_r.copy()
        for op in ops:  # successive edits on the same buffer
            rets.append(int(R.nfref_vlan(oracle._ptr(buf_r), oracle._ptr(ln_r, oracle._u32p), cap, op)))
            sts.append(int(L.nfo_vlan(oracle._ptr(buf_o), oracle._ptr(ln_o, oracle._u32p), cap, op)))
        w = oracle.vlan_window(len(f))
        assert bytes(buf_r[:w]) == bytes(buf_o[:w]) and ln_r[0] == ln_o[0], name
        assert all((s == 16) == (r == 0) for s, r in zip(sts, rets)), name
        kats[name] = {"in": f.hex(), "ops": [int(o) for o in ops], "cap": int(cap),
                      "out": bytes(buf_r[:w]).hex(), "len_out": int(ln_r[0]), "ret": rets,
                      "status": sts}
    with open(os.path.join(OUT, "kat_vlan.json"), "w") as fh:
        json.dump(kats, fh, indent=1, sort_keys=True)
    print("kat_vlan.json:", len(kats), "cases")
    frames, ops, caps = vlan_inputs()
    n = len(frames)
    h_out = np.zeros(n, dtype=np.uint64)
    len_out = np.zeros(n, dtype=np.uint32)
    ret = np.zeros(n, dtype=np.int8)
    st = np.zeros(n, dtype=np.uint8)
    for i, f in enumerate(frames):
        o_orc, s, win_o = oracle.vlan_frame(f, int(ops[i]), int(caps[i]))
        st[i] = s
        if (s & 0x1F) == 14:  # IHL past the edited frame: the reference reads past it
            continue
        o, r, win = oracle.ref_vlan_frame(f, int(ops[i]), int(caps[i]))
        assert win == win_o and o == o_orc and (r == 0) == (s == 16), i
        ret[i] = r
        len_out[i] = len(o)
        wb = np.frombuffer(win, dtype=np.uint8).copy()
        h_out[i] = L.nfo_frame_hash(oracle._ptr(wb), len(win))
    np.savez_compressed(os.path.join(OUT, "vlan_ref.npz"), seed=np.uint64(VLAN_SEED), ops=ops,
                        caps=caps, lens=np.array([len(f) for f in frames], dtype=np.uint16),
                        len_out=len_out, ret=ret, hash_window=h_out, oracle_status=st)
    print("vlan_ref.npz:", n, "frames; statuses", np.unique(st, return_counts=True))
    # bench workload: C1 1M frames in 1536-byte slots, push_vlan(100, 3) then pop_vlan()
    res = json.load(open(os.path.join(OUT, "configs.json")))
    nb = 1 << 20
    M = (1 << 64) - 1
    d1 = d2 = 0
    for lo in range(0, nb, CHUNK):
        m = min(CHUNK, nb - lo)
        arena, desc = oracle.gen_config(1, CONFIG_SEED, lo, m, 128)
        R.nfref_vlan_batch(oracle._ptr(arena), desc.ctypes.data,
                           oracle._ptr(np.full(m, oracle.vlan_op("push", 100, 3), np.uint32), oracle._u32p),
                           m, 1536, 8)
        d1 = (d1 + oracle.digest(arena, desc, lo)) & M
        R.nfref_vlan_batch(oracle._ptr(arena), desc.ctypes.data,
                           oracle._ptr(np.full(m, oracle.vlan_op("pop"), np.uint32), oracle._u32p),
                           m, 1536, 8)
        d2 = (d2 + oracle.digest(arena, desc, lo)) & M
    res["vlan_c1"] = {"first": 0, "n": nb, "align": 128, "cap": 1536, "op_push": "push_vlan(100, 3)",
                      "digest_push": f"{d1:016x}", "digest_push_pop": f"{d2:016x}"}
    with open(os.path.join(OUT, "configs.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(f"vlan C1 digests push {d1:016x} push+pop {d2:016x}")


def ref_config_digest(R, config, seed, first, n, nthreads=8):
    """Digest of config packets [first, first+n) before and after the REFERENCE."""
    din = dout = 0
    M = (1 << 64) - 1
    for lo in range(0, n, CHUNK):
        m = min(CHUNK, n - lo)
        arena, desc = oracle.gen_config(config, seed, first + lo, m)
        din = (din + oracle.digest(arena, desc, first + lo)) & M
        R.nfref_update_batch(oracle._ptr(arena), desc.ctypes.data, m, nthreads)
        dout = (dout + oracle.digest(arena, desc, first + lo)) & M
    return din, dout


def make_configs(R):
    sizes = {0: 1024, 1: 1 << 20, 2: 1 << 20, 3: 1 << 22}
    res = {"seed": CONFIG_SEED, "configs": {}}
    for cfg, n in sizes.items():
        t = time.time()
        din, dout = ref_config_digest(R, cfg, CONFIG_SEED, 0, n)
        _, odout, hist = oracle.config_digest(cfg, CONFIG_SEED, 0, n, 8)
        assert odout == dout, (cfg, hex(odout), hex(dout))
        res["configs"][str(cfg)] = {"first": 0, "n": n, "digest_in": f"{din:016x}",
                                    "digest_out": f"{dout:016x}",
                                    "oracle_status_hist": {str(k): v for k, v in hist.items()}}
        print(f"config C{cfg} n={n}: in {din:016x} out {dout:016x}  ({time.time() - t:.1f}s)")
    # multi-GPU weak-scaling shards of C1: rank r owns packets [r*2^20, (r+1)*2^20)
    shards = []
    for r in range(8):
        t = time.time()
        din, dout = ref_config_digest(R, 1, CONFIG_SEED, r << 20, 1 << 20)
        shards.append({"rank": r, "first": r << 20, "n": 1 << 20, "digest_in": f"{din:016x}",
                       "digest_out": f"{dout:016x}"})
        print(f"C1 shard {r}: {dout:016x} ({time.time() - t:.1f}s)")
    res["c1_rank_shards"] = shards
    with open(os.path.join(OUT, "configs.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)


def make_flowkey_c1(R):
    """Digest of the reference's flow-key records (nfcs_flow_key layout) and hashes for C1 (1M
    packets, 128-byte aligned frames): the records as an arena of 64-byte frames, hashes as
    4-byte frames, each digested with DESIGN.md §6's order-independent digest."""
    res = json.load(open(os.path.join(OUT, "configs.json")))
    n = 1 << 20
    M = (1 << 64) - 1
    dr = dh = 0
    for lo in range(0, n, CHUNK):
        m = min(CHUNK, n - lo)
        arena, desc = oracle.gen_config(1, CONFIG_SEED, lo, m, 128)
        recs = np.zeros((m, 64), dtype=np.uint8)
        hashes = np.zeros(m, dtype=np.uint32)
        R.nfref_flow_keys_batch(oracle._ptr(arena), desc.ctypes.data, m, oracle._ptr(recs),
                                oracle._ptr(hashes, oracle._u32p), 8)
        rdesc = np.zeros(m, dtype=oracle.DESC_DTYPE)
        rdesc["off16"] = np.arange(m, dtype=np.uint32) * 4
        rdesc["len"] = 64
        dr = (dr + oracle.digest(recs.reshape(-1), rdesc, lo)) & M
        hdesc = np.zeros(m, dtype=oracle.DESC_DTYPE)
        hb = np.zeros((m, 16), dtype=np.uint8)
        hb[:, :4] = hashes.view(np.uint8).reshape(m, 4)
        hdesc["off16"] = np.arange(m, dtype=np.uint32)
        hdesc["len"] = 4
        dh = (dh + oracle.digest(hb.reshape(-1), hdesc, lo)) & M
    res["flowkey_c1"] = {"first": 0, "n": n, "align": 128, "digest_records": f"{dr:016x}",
                         "digest_hashes": f"{dh:016x}",
                         "how": "records as 64-byte frames at 64-byte stride; hashes as 4-byte frames at 16-byte stride"}
    with open(os.path.join(OUT, "configs.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(f"flowkey C1 digests records {dr:016x} hashes {dh:016x}")


def make_l3_more(R):
    """The bench's other fused-forward workloads (bench.py --op l3fwd --config 3 / --packets 4M):
    the reference's data path (TTL, MACs, update_checksums) over C3's 4M mixed frames and over 4M
    C1 frames, next hop i % 9 of l3_table() (8 = no route), one forward each."""
    res = json.load(open(os.path.join(OUT, "configs.json")))
    table = l3_table()
    tab = np.ascontiguousarray(table.reshape(-1))
    M = (1 << 64) - 1
    out = []
    for cfg, n in ((3, 1 << 22), (1, 1 << 22)):
        dout = 0
        for lo in range(0, n, CHUNK):
            m = min(CHUNK, n - lo)
            arena, desc = oracle.gen_config(cfg, CONFIG_SEED, lo, m)
            nh = ((np.arange(lo, lo + m)) % 9).astype(np.uint32)
            R.nfref_l3_forward_batch(oracle._ptr(arena), desc.ctypes.data, oracle._ptr(nh, oracle._u32p),
                                     m, oracle._ptr(tab), 8, 8)
            dout = (dout + oracle.digest(arena, desc, lo)) & M
        out.append({"config": cfg, "first": 0, "n": n, "digest_out": f"{dout:016x}"})
        print(f"l3fwd config {cfg} n {n}: {dout:016x}")
    res["l3fwd_more"] = out
    with open(os.path.join(OUT, "configs.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)


def make_c4(R):
    """C4: 32M x 1500 B IPv4+UDP sharded across 8 GPUs, 4M packets per rank (weak scaling at
    1/2/4/8 GPUs): the reference's digest of every rank's shard."""
    res = json.load(open(os.path.join(OUT, "configs.json")))
    shards = []
    for r in range(8):
        t = time.time()
        din, dout = ref_config_digest(R, 1, CONFIG_SEED, r << 22, 1 << 22)
        shards.append({"rank": r, "first": r << 22, "n": 1 << 22, "digest_in": f"{din:016x}",
                       "digest_out": f"{dout:016x}"})
        print(f"C4 shard {r}: {dout:016x} ({time.time() - t:.1f}s)")
    res["c4_rank_shards"] = shards
    with open(os.path.join(OUT, "configs.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    oracle.build(ref=True)
    R = oracle.ref()
    what = sys.argv[1:] or ["kat", "fuzz", "configs", "l3", "flow", "vlan"]
    if "kat" in what:
        make_kat(R)
    if "fuzz" in what:
        make_fuzz(R)
    if "configs" in what:
        make_configs(R)
    if "l3" in what:
        make_l3(R)
    if "flow" in what:
        make_flow(R)
    if "vlan" in what:
        make_vlan(R)
    if "c4" in what:
        make_c4(R)
    if "l3_more" in what:
        make_l3_more(R)
    if "flowkey_c1" in what:
        make_flowkey_c1(R)
