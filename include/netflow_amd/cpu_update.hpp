// netflow_amd/cpu_update.hpp — the single-packet path, on the host CPU.
//
// NetFlow++ calls Packet::update_checksums() (include/netflow++/packet.hpp:722-890) and
// push_vlan()/pop_vlan() (packet.hpp:655-720) one packet at a time from its control plane (the ICMP
// processor, icmp_processor.cpp:180,336; the VLAN manager, vlan_manager.cpp:90,159,174). A single
// packet is a latency-bound call that a PCIe round trip to the GPU would only slow down, so the
// single-packet members of netflow_amd::Packet run here, on the CPU, like the reference: void /
// bool, never throwing. Bursts go to the GPU engine (ChecksumEngine, include/netflow_amd/packet.hpp)
// and never fall back to this code.
//
// The arithmetic follows the reference step by step in its write order:
// the IPv4 header checksum is written before the L4 region is read, so an IPv4 header with IHL < 5
// whose L4 region overlaps it gives the reference's bytes too. Bit-exactness with the reference is
// tested in tests/test_netflow_adapter.py (against the reference's own Packet, compiled in).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>

#include "nfcs.h"

namespace netflow_amd {
namespace cpu {

inline uint32_t be16(const unsigned char* f, size_t o) { return (uint32_t(f[o]) << 8) | f[o + 1]; }

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "the sums below read little-endian words");

// calculate_checksum's running sum (packet.hpp:898-905) in the little-endian domain: the reference adds big-endian 16-bit words and an odd trailing byte as the LOW byte of a
// word (its quirk, not RFC 1071's high byte). One's-complement addition commutes with the byte swap
// (RFC 1071 §2(B)), so the sum of the region's little-endian 16-bit words — zero exactly when every
// byte is — folds to the byte swap of the reference's fold (finish below); the odd byte b, a big-endian value b, is b << 8 here.
// (The GPU kernels use the same identity)

// Lanes of four 32-bit words (GCC/Clang vector extension: SSE2 / NEON code at -O2, no intrinsics).
typedef uint32_t le_v4 __attribute__((vector_size(16)));

inline uint64_t le_sum(const unsigned char* p, size_t n) {
    // 16 bytes per step: the low and the high 16-bit words of four dwords added into separate 32-bit
    // lanes; a lane adds at most 0xFFFF per step, so it cannot wrap for regions below 1 MiB (the
    // callers' regions are below 2^16 + 60 bytes)
    le_v4 lo = {0, 0, 0, 0}, hi = {0, 0, 0, 0};
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        le_v4 v;
        std::memcpy(&v, p + i, 16);
        lo += v & 0xFFFFu;
        hi += v >> 16;
    }
    uint64_t s = 0;
    for (int k = 0; k < 4; ++k) s += (uint64_t)lo[k] + hi[k];
    for (; i + 1 < n; i += 2) s += uint32_t(p[i]) | (uint32_t(p[i + 1]) << 8);
    if (n & 1) s += uint32_t(p[n - 1]) << 8;
    return s;
}

// A big-endian-domain 16-bit term (the pseudo-header's protocol and length) in the little-endian domain.
inline uint64_t le_term(uint32_t be) { return ((be & 0xFFu) << 8) | ((be >> 8) & 0xFFu); }

// End-around carry, complement (packet.hpp:907-911) of a little-endian-domain sum: the value the
// reference stores big-endian. A zero sum gives 0xFFFF, any other multiple of 0xFFFF 0x0000, as there.
inline uint32_t finish(uint64_t s) {
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return ~(((s & 0xFFu) << 8) | (s >> 8)) & 0xFFFFu;
}

inline void put_be16(unsigned char* f, size_t o, uint32_t v) {
    f[o] = (unsigned char)(v >> 8);
    f[o + 1] = (unsigned char)v;
}

// Packet::update_checksums() on the frame f[0, len). Returns the NFCS_ST_* status the GPU engine
// reports for the same frame. A frame whose IPv4 IHL reaches past its end (the reference then reads
// past the buffer) is left untouched (NFCS_ST_OOB), as the engine leaves it.
inline uint8_t update_checksums(unsigned char* f, size_t len) noexcept {
    if (!f) return NFCS_ST_NONE;
    const size_t l2 = (len >= 14 && be16(f, 12) == 0x8100u) ? 18 : 14;  // ethernet()
    bool v4 = false;
    uint32_t proto = 0, ihl4 = 0;
    size_t l4 = 0;
    uint8_t st;
    if (l2 + 20 <= len && (f[l2] >> 4) == 4) {  // ipv4(): by version nibble, EtherType not read
        v4 = true;
        ihl4 = (f[l2] & 15u) * 4u;
        proto = f[l2 + 9];
        l4 = l2 + ihl4;
        if (l4 > len) return NFCS_ST_OOB;
        f[l2 + 10] = f[l2 + 11] = 0;
        put_be16(f, l2 + 10, finish(le_sum(f + l2, ihl4)));
        st = NFCS_ST_V4;
    } else {
        uint32_t et = len >= 14 ? be16(f, 12) : 0u;
        if (et == 0x8100u) et = len >= 18 ? be16(f, 16) : 0u;  // one tag only
        if (et != 0x86DDu || l2 + 40 > len || (f[l2] >> 4) != 6) return NFCS_ST_NONE;
        proto = f[l2 + 6];
        l4 = l2 + 40;
        st = NFCS_ST_V6;
    }
    // IHL < 5 with TCP/UDP/ICMP: the L4 region overlaps the IPv4 header (flagged, as the engine does)
    const uint8_t ov = (v4 && ihl4 < 20 && (proto == 6 || proto == 17 || proto == 1)) ? NFCS_ST_FLAG_OVERLAP : 0;
    const uint8_t skip = (v4 ? NFCS_ST_V4_L4SKIP : NFCS_ST_V6_L4SKIP) | ov;
    uint32_t seg;
    size_t field;
    if (proto == 6) {                      // tcp(): the 19-byte packed TcpHeader
        if (l4 + 19 > len) return skip;
        const uint32_t hl = (f[l4 + 12] >> 4) * 4u;
        if (v4) {
            const uint32_t tl = be16(f, l2 + 2);
            if (tl < ihl4) return skip;
            seg = (tl - ihl4) & 0xFFFFu;
        } else {
            seg = be16(f, l2 + 4);
        }
        if (seg < hl || l4 + seg > len) return skip;
        field = l4 + 15;                   // TcpHeader::checksum sits at byte 15 of the struct
        st = v4 ? NFCS_ST_V4_TCP : NFCS_ST_V6_TCP;
    } else if (proto == 17) {              // udp(): covers udp.length bytes
        if (l4 + 8 > len) return skip;
        seg = be16(f, l4 + 4);
        if (seg < 8 || l4 + seg > len) return skip;
        field = l4 + 6;
        st = v4 ? NFCS_ST_V4_UDP : NFCS_ST_V6_UDP;
    } else if (proto == 1 && v4) {         // icmp(): IPv4 only, no pseudo-header
        if (l4 + 8 > len) return skip;
        const uint32_t tl = be16(f, l2 + 2);
        if (tl < ihl4) return skip;
        seg = tl - ihl4;
        if (l4 + seg > len || seg < 8) return skip;
        field = l4 + 2;
        st = NFCS_ST_V4_ICMP;
    } else {
        return st;
    }
    f[field] = f[field + 1] = 0;           // zeroed, then the pseudo-header and the segment read
    uint64_t s = 0;
    if (proto != 1)  // {src, dst, 0, proto, seg} (IPv6: {src16, dst16, seg32, 0, 0, 0, nh}); seg < 2^16
        s = le_sum(f + l2 + (v4 ? 12 : 8), v4 ? 8 : 32) + le_term(proto) + le_term(seg);
    s += le_sum(f + l4, seg);
    uint32_t c = finish(s);
    if (proto == 17 && c == 0) c = 0xFFFFu;  // UDP only (packet.hpp:867-871)
    put_be16(f, field, c);
    return st | ov;
}

// Packet::push_vlan(vid, prio) / pop_vlan() (packet.hpp:655-720) on a frame f[0, *len) whose
// buffer holds `room` bytes from f (PacketBuffer capacity minus headroom), each ending with
// update_checksums(). Returns what the reference returns; *len changes as the reference changes the
// buffer's data length. Where the reference writes past its buffer (a re-tag of a 14- or 15-byte
// frame in a buffer of fewer than 16 bytes; a push into a buffer without tailroom, which it then
// fails) only bytes inside the buffer are written.
inline bool push_vlan(unsigned char* f, size_t* len, size_t room, uint16_t vid, uint8_t prio) noexcept {
    if (!f || !len || *len < 14) return false;
    const size_t n = *len;
    if (be16(f, 12) == 0x8100u) {          // has_vlan(): re-tag in place, DEI kept (185-190)
        const uint32_t old = room >= 16 ? be16(f, 14) : 0u;
        const uint32_t tci = (old & 0x1000u) | ((uint32_t)(prio & 7u) << 13) | (vid & 0x0FFFu);
        if (room > 14) f[14] = (unsigned char)(tci >> 8);
        if (room > 15) f[15] = (unsigned char)tci;
    } else {
        if (n + 4 > room) return false;    // tailroom < 4 (the reference fails, 666-672, 684-686)
        const unsigned char e0 = f[12], e1 = f[13];
        std::memmove(f + 18, f + 14, n - 14);
        const uint32_t tci = ((uint32_t)(prio & 7u) << 13) | (vid & 0x0FFFu);
        f[12] = 0x81;
        f[13] = 0x00;
        f[14] = (unsigned char)(tci >> 8);
        f[15] = (unsigned char)tci;
        f[16] = e0;
        f[17] = e1;
        *len = n + 4;
    }
    update_checksums(f, *len);
    return true;
}

inline bool pop_vlan(unsigned char* f, size_t* len) noexcept {
    if (!f || !len || *len < 14 || be16(f, 12) != 0x8100u) return false;  // has_vlan()
    const size_t n = *len;
    if (n < 18) return false;
    const unsigned char e0 = f[16], e1 = f[17];
    std::memmove(f + 14, f + 18, n - 18);  // the old last 4 bytes stay past the new length
    f[12] = e0;
    f[13] = e1;
    *len = n - 4;
    update_checksums(f, *len);
    return true;
}

}  // namespace cpu
}  // namespace netflow_amd
