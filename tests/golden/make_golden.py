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


if __name__ == "__main__":
    oracle.build(ref=True)
    R = oracle.ref()
    what = sys.argv[1:] or ["kat", "fuzz", "configs", "l3", "flow"]
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
