// nfcs_kernels.hip — CDNA4 (gfx950) kernels of the batched Internet-checksum engine.
//
// The hot path is NetFlow++'s Packet::update_checksums() (include/netflow++/packet.hpp:722-890)
// with its fold Packet::calculate_checksum() (packet.hpp:894-912), applied to a batch of
// frames in HBM. Design:
//
//  * One wave64 owns one packet at a time; waves grid-stride over the batch. The descriptor
//    is a wave-uniform scalar load; the frame streams in as 16-byte chunks, lane l holding
//    chunks l, l+64, ... (global_load_dwordx4, fully coalesced: 1 KiB per wave-instruction).
//    The next packet's first batch (K0 chunks per lane = 2 KiB) is issued before the current
//    packet is reduced, so every wave keeps a packet in flight while it computes.
//  * The first 96 bytes of the frame (every header field the reference looks at) are copied
//    from the chunk registers of lanes 0..5 into a per-wave LDS slot. The parse — VLAN, IPv4
//    by version nibble, IPv6, TCP/UDP/ICMP bounds rules, the 19-byte TcpHeader's checksum at
//    offset 15 — runs on wave-uniform values (readfirstlane -> SGPRs, scalar branches). The
//    IPv4 header checksum and the pseudo-header sum are finished from LDS on the scalar side.
//  * The L4 region is summed as little-endian dwords into an exact 64-bit per-lane sum. The
//    one's-complement sum is byte-order independent (RFC 1071 §2(B)): the LE-domain fold is
//    bswap16 of the reference's big-endian fold, so one swap at the end replaces the
//    reference's per-word ntohs. Chunks wholly inside the region are added unmasked; the
//    (at most two) boundary chunks per packet are masked per dword. Bytes that the
//    reference zeroes (the checksum field) and the 2 bytes before a region that starts at
//    2 mod 4 are subtracted exactly on the scalar side; the odd trailing byte, which the
//    reference adds as the LOW byte (packet.hpp:903-905), gets +255*b in its lane.
//  * The wave sum is a DPP reduction (4 row-local steps + 4 readlanes); the final fold,
//    complement, UDP 0->0xFFFF (packet.hpp:867-871) and the 2+2 byte stores are wave-uniform.
//  * Packets whose L4 region overlaps the IPv4 header (IHL < 5 with TCP/UDP/ICMP) go through
//    an exact sequential emulation on one lane (same byte order of writes as the reference).
//  * No MFMA and no LDS staging of payload: this is an HBM-read-bound integer fold.
#include "nfcs_internal.h"

namespace nfcs {

#define DEV __device__ __forceinline__

DEV uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
DEV uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// End-around-carry fold of an exact sum to 16 bits (packet.hpp:907-909). Zero stays zero;
// a nonzero multiple of 0xFFFF folds to 0xFFFF, as in the reference.
DEV uint32_t fold64(uint64_t s) {
    s = (s & 0xFFFFFFFFull) + (s >> 32);
    while (s >> 16) s = (s & 0xFFFFull) + (s >> 16);
    return (uint32_t)s;
}

// ---- staged chunk registers ------------------------------------------------------------------
// A batch holds K chunks per lane: chunk cbase + lane + 64*k in slot k.
template <int K>
struct Batch {
    uint4 v[K];
};

__device__ uint4 g_zero16;  // target of the clamped loads of lanes past the frame end

// Component j of a uint4 by mask arithmetic (no indexable temporary, so no scratch).
DEV uint32_t comp(const uint4& v, uint32_t j) {
    const uint32_t m0 = 0u - (uint32_t)(j == 0), m1 = 0u - (uint32_t)(j == 1);
    const uint32_t m2 = 0u - (uint32_t)(j == 2), m3 = 0u - (uint32_t)(j == 3);
    return (v.x & m0) | (v.y & m1) | (v.z & m2) | (v.w & m3);
}

// Frame dword q (wave-uniform) from the registers of batch B whose first chunk is cbase.
// With a compile-time q this folds to a single v_readlane_b32 into an SGPR.
template <int K>
DEV uint32_t batch_dw(const Batch<K>& B, uint32_t q, uint32_t cbase) {
    const uint32_t rc = (q >> 2) - cbase;
    const uint32_t k = rc >> 6, l = rc & 63u, j = q & 3u;
    uint32_t x = 0;
#pragma unroll
    for (int s = 0; s < K; ++s) x |= comp(B.v[s], j) & (0u - (uint32_t)(k == (uint32_t)s));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}

// header accessors: frame bytes [0, 96) live in lanes 0..5 of slot 0 of the staged batch
template <int K>
struct Hdr {
    const Batch<K>& B;
    DEV uint32_t dw(uint32_t q) const { return batch_dw<K>(B, q, 0); }
    DEV uint32_t b(uint32_t o) const { return (dw(o >> 2) >> (8 * (o & 3u))) & 0xFFu; }
    DEV uint32_t le16(uint32_t o) const { return (dw(o >> 2) >> (8 * (o & 2u))) & 0xFFFFu; }  // o even
    DEV uint32_t be16(uint32_t o) const { return bswap16(le16(o)); }
};

// ---- parse: everything update_checksums() decides, on wave-uniform values -------------------
struct Plan {
    uint32_t st;      // NFCS_ST_* (without the overlap flag)
    uint32_t mode;    // 0: write nothing, 1: vector path, 2: sequential path
    uint32_t has_ip;  // IPv4 header checksum to write at ip_off (value ip_val, LE store)
    uint32_t ip_off, ip_val;
    uint32_t has_l4;  // L4 checksum over [rs, re) written at fs, fs+1
    uint32_t rs, re, fs;
    uint32_t udp;     // 0 -> 0xFFFF rule
    uint32_t tailfix; // odd region: trailing byte counts as the low byte
    uint64_t add;     // exact LE-domain constant: pseudo-header
    uint64_t sub;     // exact LE-domain bytes counted by the dword sum but not by the reference
};

DEV Plan plan_none(uint32_t st) {
    Plan P;
    P.st = st; P.mode = 0; P.has_ip = 0; P.ip_off = 0; P.ip_val = 0; P.has_l4 = 0;
    P.rs = P.re = P.fs = 0; P.udp = 0; P.tailfix = 0; P.add = 0; P.sub = 0;
    return P;
}

// L4 decisions of packet.hpp:773-889 for a packet whose L4 header starts at l4. Inlined at
// call sites where l2/l4 are literals, so every header offset is a compile-time constant.
template <int K>
DEV Plan plan_l4(const Hdr<K>& H, Plan P, uint32_t len, uint32_t v4, uint32_t l2,
                 uint32_t ihl4, uint32_t l4, uint32_t proto) {
    const uint32_t skip = v4 ? NFCS_ST_V4_L4SKIP : NFCS_ST_V6_L4SKIP;
    uint32_t L;
    if (proto == 6) {  // 773-823
        if (l4 + 19 > len) { P.st = skip; return P; }  // sizeof(TcpHeader) == 19
        const uint32_t hl = (H.b(l4 + 12) >> 4) * 4u;
        if (v4) {
            const uint32_t tl = H.be16(l2 + 2);
            if (tl < ihl4) { P.st = skip; return P; }
            L = (tl - ihl4) & 0xFFFFu;
        } else {
            L = H.be16(l2 + 4);
        }
        if (L < hl || l4 + L > len) { P.st = skip; return P; }
        P.fs = l4 + 15;  // TcpHeader::checksum sits at offset 15 under #pragma pack(1)
        P.st = v4 ? NFCS_ST_V4_TCP : NFCS_ST_V6_TCP;
    } else if (proto == 17) {  // 824-872
        if (l4 + 8 > len) { P.st = skip; return P; }
        L = H.be16(l4 + 4);
        if (L < 8 || l4 + L > len) { P.st = skip; return P; }
        P.fs = l4 + 6;
        P.udp = 1;
        P.st = v4 ? NFCS_ST_V4_UDP : NFCS_ST_V6_UDP;
    } else if (proto == 1 && v4) {  // 873-889
        if (l4 + 8 > len) { P.st = skip; return P; }
        const uint32_t tl = H.be16(l2 + 2);
        if (tl < ihl4) { P.st = skip; return P; }
        L = tl - ihl4;
        if (l4 + L > len || L < 8) { P.st = skip; return P; }
        P.fs = l4 + 2;
        P.st = NFCS_ST_V4_ICMP;
    } else {
        return P;  // IPv4 header only (v4) / nothing (v6)
    }
    P.mode = 1;
    P.has_l4 = 1;
    P.rs = l4;
    P.re = l4 + L;
    // pseudo-header (797-816 / 840-859) in the LE domain: address words + bswap16(proto word)
    // + bswap16(length word); IPv6's 32-bit length has a zero upper word (L <= 0xFFFF).
    uint64_t add = 0;
    if (proto != 1) {
        add = bswap16(proto) + bswap16(L);
        if (v4) {
#pragma unroll
            for (uint32_t w = 0; w < 8; w += 2) add += H.le16(l2 + 12 + w);
        } else {
#pragma unroll
            for (uint32_t w = 0; w < 32; w += 2) add += H.le16(l2 + 8 + w);
        }
    }
    P.add = add;
    // exact corrections of the dword sum: the region is summed from rs & ~3 (l4 is even, so
    // that may add the LE word at rs-2) and it includes the raw checksum field bytes that the
    // reference zeroes before summing (795 / 838 / 885)
    uint64_t sub = (P.rs & 2u) ? H.le16(P.rs - 2) : 0u;
    if (P.fs >= P.rs && P.fs < P.re) sub += (uint64_t)H.b(P.fs) << ((P.fs & 1u) ? 8 : 0);
    if (P.fs + 1 >= P.rs && P.fs + 1 < P.re) sub += (uint64_t)H.b(P.fs + 1) << (((P.fs + 1) & 1u) ? 8 : 0);
    P.sub = sub;
    // odd region: its trailing byte (even frame offset: the LOW byte of its LE word in the
    // dword sum) counts as the HIGH byte in the reference (903-905): +255*b, unless zeroed
    const uint32_t t = P.re - 1;
    P.tailfix = (L & 1u) && !(t >= P.fs && t < P.fs + 2);
    return P;
}

template <int K>
DEV Plan plan_v4(const Hdr<K>& H, uint32_t len, uint32_t l2, uint32_t ihl4, uint32_t proto) {
    Plan P = plan_none(NFCS_ST_V4);
    // 739-740: checksum over ihl4 bytes with the field at l2+10 zeroed
    uint64_t s = 0;
    for (uint32_t w = 0; w < ihl4; w += 2)
        if (w != 10) s += H.le16(l2 + w);
    P.has_ip = 1;
    P.ip_off = l2 + 10;
    P.ip_val = (~fold64(s)) & 0xFFFFu;
    P.mode = 1;
    return plan_l4<K>(H, P, len, 1u, l2, ihl4, l2 + ihl4, proto);
}

template <int K>
DEV Plan plan_at(const Hdr<K>& H, uint32_t len, uint32_t l2) {
    const uint32_t b0 = (l2 + 20 <= len) ? H.b(l2) : 0u;
    if (l2 + 20 <= len && (b0 >> 4) == 4) {  // 728-734: IPv4 by version nibble
        const uint32_t proto = H.b(l2 + 9);
        const uint32_t ihl4 = (b0 & 15u) * 4u;
        if (l2 + ihl4 > len) return plan_none(NFCS_ST_OOB);  // ref reads past the frame
        if (ihl4 < 20 && (proto == 6 || proto == 17 || proto == 1)) {
            Plan P = plan_none(NFCS_ST_NONE);
            P.mode = 2;  // the L4 region overlaps the IPv4 header: sequential path
            return P;
        }
        if (ihl4 == 20) return plan_v4<K>(H, len, l2, 20u, proto);  // constant offsets
        return plan_v4<K>(H, len, l2, ihl4, proto);                 // IP options
    }
    // 741-765: effective EtherType after one 0x8100 tag; IPv6 needs the nibble too
    uint32_t et = (len >= 14) ? H.be16(12) : 0u;
    if (et == 0x8100u) et = (len >= 18) ? H.be16(16) : 0u;
    if (et != 0x86DDu || !(l2 + 40 <= len && (H.b(l2) >> 4) == 6)) return plan_none(NFCS_ST_NONE);
    Plan P = plan_none(NFCS_ST_V6);
    return plan_l4<K>(H, P, len, 0u, l2, 0u, l2 + 40, H.b(l2 + 6));
}

template <int K>
DEV Plan parse(const Hdr<K>& H, uint32_t len) {
    // ethernet(), packet.hpp:405-418: l2 = 18 after a 0x8100 tag (len < 14 keeps the ctor's 14)
    const bool tagged = (len >= 14) && H.be16(12) == 0x8100u;
    return tagged ? plan_at<K>(H, len, 18u) : plan_at<K>(H, len, 14u);
}

// ---- exact sequential path (IHL < 5 overlap cases), one lane --------------------------------
// Mirrors packet.hpp:722-890 byte by byte on global memory, in the reference's write order.
struct SeqOut { uint32_t st, ip_off, ip_val, l4_off, l4_val; };

__device__ uint32_t g_be16(const uint8_t* f, uint32_t o) { return ((uint32_t)f[o] << 8) | f[o + 1]; }
__device__ uint32_t g_sum(const uint8_t* d, uint32_t len) {  // 898-905, raw sum
    uint32_t s = 0, i = 0;
    for (; len > 1; len -= 2, i += 2) s += g_be16(d, i);
    if (len) s += d[i];
    return s;
}
__device__ uint32_t g_fin(uint32_t s) {  // 907-911: value stored big-endian
    while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
    return (~s) & 0xFFFFu;
}

__device__ __noinline__ SeqOut seq_update(uint8_t* f, uint32_t len) {
    SeqOut o = {NFCS_ST_NONE, NFCS_PATCH_NONE, 0, NFCS_PATCH_NONE, 0};
    uint32_t l2 = 14;
    if (len >= 14) l2 = (g_be16(f, 12) == 0x8100u) ? 18u : 14u;
    uint32_t v4 = 0, proto, ihl4 = 0, l4;
    if (l2 + 20 <= len && (f[l2] >> 4) == 4) {
        v4 = 1;
        proto = f[l2 + 9];
        ihl4 = (f[l2] & 15u) * 4u;
        l4 = l2 + ihl4;
        if (l2 + ihl4 > len) { o.st = NFCS_ST_OOB; return o; }
        f[l2 + 10] = 0;
        f[l2 + 11] = 0;
        uint32_t c = g_fin(g_sum(f + l2, ihl4));
        f[l2 + 10] = (uint8_t)(c >> 8);
        f[l2 + 11] = (uint8_t)c;
        o.ip_off = l2 + 10;
        o.ip_val = bswap16(c);
        o.st = NFCS_ST_V4;
    } else {
        uint32_t et = (len >= 14) ? g_be16(f, 12) : 0;
        if (et == 0x8100u) et = (len >= 18) ? g_be16(f, 16) : 0;
        if (et != 0x86DDu || !(l2 + 40 <= len && (f[l2] >> 4) == 6)) return o;
        proto = f[l2 + 6];
        l4 = l2 + 40;
        o.st = NFCS_ST_V6;
    }
    const uint32_t skip = v4 ? NFCS_ST_V4_L4SKIP : NFCS_ST_V6_L4SKIP;
    uint32_t fs, L, st;
    uint32_t sum = 0;
    if (proto == 6) {
        if (l4 + 19 > len) { o.st = skip; return o; }
        uint32_t hl = (f[l4 + 12] >> 4) * 4u;
        if (v4) {
            uint32_t tl = g_be16(f, l2 + 2);
            if (tl < ihl4) { o.st = skip; return o; }
            L = (tl - ihl4) & 0xFFFFu;
        } else {
            L = g_be16(f, l2 + 4);
        }
        if (L < hl || l4 + L > len) { o.st = skip; return o; }
        fs = l4 + 15;
        st = v4 ? NFCS_ST_V4_TCP : NFCS_ST_V6_TCP;
    } else if (proto == 17) {
        if (l4 + 8 > len) { o.st = skip; return o; }
        L = g_be16(f, l4 + 4);
        if (L < 8 || l4 + L > len) { o.st = skip; return o; }
        fs = l4 + 6;
        st = v4 ? NFCS_ST_V4_UDP : NFCS_ST_V6_UDP;
    } else if (proto == 1 && v4) {
        if (l4 + 8 > len) { o.st = skip; return o; }
        uint32_t tl = g_be16(f, l2 + 2);
        if (tl < ihl4) { o.st = skip; return o; }
        L = tl - ihl4;
        if (l4 + L > len || L < 8) { o.st = skip; return o; }
        fs = l4 + 2;
        st = NFCS_ST_V4_ICMP;
    } else {
        return o;
    }
    f[fs] = 0;  // zero the field, then read pseudo-header and segment (reference order)
    f[fs + 1] = 0;
    if (proto != 1) {
        if (v4) sum = g_sum(f + l2 + 12, 8) + proto + L;
        else sum = g_sum(f + l2 + 8, 32) + (L >> 16) + (L & 0xFFFF) + proto;
    }
    sum += g_sum(f + l4, L);
    uint32_t c = g_fin(sum);
    if (proto == 17 && c == 0) c = 0xFFFF;
    f[fs] = (uint8_t)(c >> 8);
    f[fs + 1] = (uint8_t)c;
    o.l4_off = fs;
    o.l4_val = bswap16(c);
    o.st = st;
    return o;
}

// ---- region accumulation ---------------------------------------------------------------------
// The L4 region [rs, re) is summed as LE dwords starting at lo4 = rs & ~3, in three parts:
//   head: dwords in [lo4, min(lo16, re))   scalar, from the header registers (lo16 <= 80)
//   body: full chunks in [lo16, hi16)      vector, unmasked uint4 adds into a u64 per lane
//   tail: dwords in [hi16, re) if hi16 >= lo16: scalar, readlane of the last partial chunk
// with lo16 = round_up(lo4, 16), hi16 = round_down(re, 16). The odd trailing byte is in the
// head or the tail (re is odd, so never 16-aligned), where it gets its +255*b.
DEV uint64_t masked_dw(uint32_t d, uint32_t q, uint32_t re, uint32_t tailfix) {
    const int n = (int)re - (int)(4u * q);
    const uint32_t m = n >= 4 ? 0xFFFFFFFFu : (n <= 0 ? 0u : ((1u << (8 * n)) - 1u));
    uint64_t a = d & m;
    const uint32_t t = re - 1;
    if (tailfix && (t >> 2) == q) a += 255ull * ((d >> (8 * (t & 3u))) & 0xFFu);
    return a;
}

DEV uint64_t add_chunk(const uint4& v) {
    return ((uint64_t)v.x + v.y) + ((uint64_t)v.z + v.w);
}

DEV uint64_t wave_sum64(uint64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
#define NFCS_DPP_STEP(ctrl)                                                              \
    {                                                                                    \
        uint32_t l2_ = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, ctrl, 0xF, 0xF, true); \
        uint32_t h2_ = (uint32_t)__builtin_amdgcn_mov_dpp((int)hi, ctrl, 0xF, 0xF, true); \
        uint64_t s_ = ((uint64_t)hi << 32 | lo) + ((uint64_t)h2_ << 32 | l2_);           \
        lo = (uint32_t)s_;                                                               \
        hi = (uint32_t)(s_ >> 32);                                                       \
    }
    NFCS_DPP_STEP(0xB1)   // quad_perm [1,0,3,2]
    NFCS_DPP_STEP(0x4E)   // quad_perm [2,3,0,1]
    NFCS_DPP_STEP(0x141)  // row_half_mirror
    NFCS_DPP_STEP(0x140)  // row_mirror: every lane of a 16-lane row now holds the row sum
#undef NFCS_DPP_STEP
    uint64_t s = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        s += ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 16 * r) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)lo, 16 * r);
    return s;
}

// One packet's staged state: descriptor and its first batch of K0 chunks per lane.
template <int K0>
struct Staged {
    uint64_t off;  // byte offset of the frame in the arena (wave-uniform)
    uint32_t len;
    uint32_t bad;
    Batch<K0> b;
};

// Issue the loads of packet p's first K0*64 chunks. Every lane always issues every load
// (lanes past the frame read g_zero16), so the number of loads in flight is the same on
// every path and the compiler can wait with a counted vmcnt instead of vmcnt(0).
template <int K0>
DEV void stage(Staged<K0>& S, const uint8_t* __restrict__ arena, uint64_t arena_bytes,
               const nfcs_desc* __restrict__ desc, uint32_t p, uint32_t base16, uint32_t lane) {
    const nfcs_desc d = desc[p];  // wave-uniform -> s_load_dwordx2
    const uint64_t off = ((uint64_t)d.off16 - base16) * 16u;
    S.off = off;
    S.len = d.len;
    S.bad = (d.off16 < base16) || (off + (((uint64_t)d.len + 15u) & ~15ull) > arena_bytes);
    const uint32_t nch = S.bad ? 0u : (d.len + 15u) >> 4;
    const uint4* src = (const uint4*)(arena + off);
#pragma unroll
    for (int k = 0; k < K0; ++k) {
        const uint32_t c = lane + 64u * k;
        const uint4* a = (c < nch) ? src + c : &g_zero16;
        S.b.v[k] = *a;
    }
}

template <int K0, int K1>
DEV void process(const Staged<K0>& S, uint8_t* arena, uint32_t p, uint32_t lane,
                 uint8_t* status, nfcs_patch* patch) {
    uint32_t st;
    uint32_t ip_off = NFCS_PATCH_NONE, ip_val = 0, l4_off = NFCS_PATCH_NONE, l4_val = 0;
    uint8_t* frame = arena + S.off;
    if (S.bad) {
        st = NFCS_ST_BAD_DESC;
    } else {
        const Hdr<K0> H{S.b};
        const Plan P = parse<K0>(H, S.len);
        st = P.st;
        if (P.mode == 2) {
            SeqOut o = {0, 0, 0, 0, 0};
            if (lane == 0) o = seq_update(frame, S.len);
            st = rfl(o.st) | NFCS_ST_FLAG_OVERLAP;
            ip_off = rfl(o.ip_off); ip_val = rfl(o.ip_val);
            l4_off = rfl(o.l4_off); l4_val = rfl(o.l4_val);
        } else if (P.mode == 1) {
            if (P.has_l4) {
                const uint32_t re = P.re, lo4 = P.rs & ~3u;
                const uint32_t lo16 = (lo4 + 15u) & ~15u, hi16 = re & ~15u;
                const uint32_t c_lo = lo16 >> 4, c_hi = hi16 >> 4;  // body chunks [c_lo, c_hi)
                const uint32_t nre = (re + 15u) >> 4;
                const bool has_tail = (re & 15u) && hi16 >= lo16;  // partial chunk c_hi
                // head, scalar
                uint64_t sc = 0;
                const uint32_t hend = lo16 < re ? lo16 : re;
                for (uint32_t q = lo4 >> 2; 4u * q < hend; ++q)
                    sc += masked_dw(H.dw(q), q, re, P.tailfix);
                // body of the staged batch, vector
                uint64_t acc = 0;
#pragma unroll
                for (int k = 0; k < K0; ++k) {
                    const uint32_t c = lane + 64u * k;
                    if (c >= c_lo && c < c_hi) acc += add_chunk(S.b.v[k]);
                }
                if (has_tail && c_hi < 64u * K0)
                    for (uint32_t q = hi16 >> 2; 4u * q < re; ++q)
                        sc += masked_dw(batch_dw<K0>(S.b, q, 0), q, re, P.tailfix);
                // continuation batches (frames longer than 64*K0 chunks)
                const uint4* src = (const uint4*)frame;
                for (uint32_t cb = 64u * K0; cb < nre; cb += 64u * K1) {
                    Batch<K1> B;
#pragma unroll
                    for (int k = 0; k < K1; ++k) {
                        const uint32_t c = cb + lane + 64u * k;
                        B.v[k] = *((c < nre) ? src + c : &g_zero16);
                    }
#pragma unroll
                    for (int k = 0; k < K1; ++k) {
                        const uint32_t c = cb + lane + 64u * k;
                        if (c >= c_lo && c < c_hi) acc += add_chunk(B.v[k]);
                    }
                    if (has_tail && c_hi >= cb && c_hi < cb + 64u * K1)
                        for (uint32_t q = hi16 >> 2; 4u * q < re; ++q)
                            sc += masked_dw(batch_dw<K1>(B, q, cb), q, re, P.tailfix);
                }
                const uint64_t z = wave_sum64(acc) + sc + P.add - P.sub;
                uint32_t c = (~fold64(z)) & 0xFFFFu;  // LE-domain complement = bswap of ref value
                if (P.udp && c == 0) c = 0xFFFFu;     // 867-871
                l4_off = P.fs;
                l4_val = c;
            }
            if (P.has_ip) {
                ip_off = P.ip_off;
                ip_val = P.ip_val;
            }
            // stores: lanes 0,1 -> IPv4 field bytes, lanes 2,3 -> L4 field bytes
            if (lane < 4) {
                const uint32_t isl4 = lane >> 1;
                const uint32_t ok = isl4 ? P.has_l4 : P.has_ip;
                const uint32_t pos = (isl4 ? l4_off : ip_off) + (lane & 1u);
                const uint32_t val = isl4 ? l4_val : ip_val;
                if (ok) frame[pos] = (uint8_t)(val >> (8 * (lane & 1u)));
            }
        }
    }
    if (lane == 0) {
        if (status) status[p] = (uint8_t)st;
        if (patch) {
            uint2 r;
            r.x = (ip_off & 0xFFFFu) | (l4_off << 16);
            r.y = (ip_val & 0xFFFFu) | (l4_val << 16);
            ((uint2*)patch)[p] = r;
        }
    }
}

template <int K0, int K1>
__global__ __launch_bounds__(kBlock) void update_kernel(uint8_t* __restrict__ arena,
                                                        uint64_t arena_bytes,
                                                        const nfcs_desc* __restrict__ desc,
                                                        uint32_t n, uint32_t base16,
                                                        uint8_t* __restrict__ status,
                                                        nfcs_patch* __restrict__ patch) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    uint32_t p = blockIdx.x * kWavesPerBlock + rfl(threadIdx.x >> 6);
    if (p >= n) return;
    Staged<K0> A;
    stage<K0>(A, arena, arena_bytes, desc, p, base16, lane);
    for (;;) {
        const uint32_t pn = p + nw;
        const bool more = pn < n && pn > p;
        // always issue the next batch (re-read p at the end) so the wait count is static
        Staged<K0> B;
        stage<K0>(B, arena, arena_bytes, desc, more ? pn : p, base16, lane);
        process<K0, K1>(A, arena, p, lane, status, patch);
        if (!more) break;
        A = B;
        p = pn;
    }
}

hipError_t launch_update(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes,
                         const nfcs_desc* desc, uint32_t n, uint32_t base16, uint8_t* status,
                         nfcs_patch* patch, hipStream_t stream, int variant, int grid) {
    if (n == 0) return hipSuccess;
    if (grid <= 0) grid = di.cus * 8;  // 8 blocks (32 waves) per CU, grid-stride beyond
    const uint32_t need = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    if ((uint32_t)grid > need) grid = (int)need;
    switch (variant) {
    default:
    case 0:
        hipLaunchKernelGGL((update_kernel<2, 4>), dim3(grid), dim3(kBlock), 0, stream, arena,
                           arena_bytes, desc, n, base16, status, patch);
        break;
    case 1:
        hipLaunchKernelGGL((update_kernel<1, 4>), dim3(grid), dim3(kBlock), 0, stream, arena,
                           arena_bytes, desc, n, base16, status, patch);
        break;
    case 2:
        hipLaunchKernelGGL((update_kernel<2, 8>), dim3(grid), dim3(kBlock), 0, stream, arena,
                           arena_bytes, desc, n, base16, status, patch);
        break;
    }
    return hipGetLastError();
}

// ---- synthetic config generator (same spec as oracle/nfcs_oracle.c) -----------
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;
__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t pkt_key(uint64_t seed, uint64_t i) { return mix64(seed ^ (i * kGolden)); }
__host__ __device__ inline uint64_t draw(uint64_t key, uint64_t k) { return mix64(key + k * kGolden); }

__host__ __device__ inline uint32_t cfg_len(int config, uint64_t seed, uint64_t index) {
    switch (config) {
    case 0: return 64;
    case 1: return 1500;
    case 2: return 9000;
    case 3: return 64u + (uint32_t)(draw(pkt_key(seed, index), 1) % 1437u);
    default: return 0;
    }
}

uint32_t config_len(int config, uint64_t seed, uint64_t index) { return cfg_len(config, seed, index); }

// header byte override at frame offset o (o < 64), or -1
DEV int hdr_byte(uint32_t o, uint32_t len, uint32_t proto, uint32_t old_ip, uint32_t old_l4) {
    switch (o) {
    case 12: return 0x08;
    case 13: return 0x00;
    case 14: return 0x45;
    case 15: return 0x00;
    case 16: return (int)(((len - 14) >> 8) & 0xFF);
    case 17: return (int)((len - 14) & 0xFF);
    case 22: return 64;
    case 23: return (int)proto;
    case 24: return (int)(old_ip >> 8);
    case 25: return (int)(old_ip & 0xFF);
    default: break;
    }
    if (proto == 17) {
        if (o == 38) return (int)(((len - 34) >> 8) & 0xFF);
        if (o == 39) return (int)((len - 34) & 0xFF);
        if (o == 40) return (int)(old_l4 >> 8);
        if (o == 41) return (int)(old_l4 & 0xFF);
    } else if (proto == 6) {
        if (o == 46) return 0x50;
        if (o == 49) return (int)(old_l4 >> 8);
        if (o == 50) return (int)(old_l4 & 0xFF);
    }
    return -1;
}

__global__ __launch_bounds__(kBlock) void gen_config_kernel(int config, uint64_t seed,
                                                            uint64_t first, uint32_t n,
                                                            uint8_t* __restrict__ arena,
                                                            uint64_t arena_bytes,
                                                            const nfcs_desc* __restrict__ desc) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    for (uint32_t p = blockIdx.x * kWavesPerBlock + rfl(threadIdx.x >> 6); p < n; p += nw) {
        const nfcs_desc d = desc[p];
        const uint64_t off = (uint64_t)d.off16 * 16u;
        const uint32_t len = d.len;
        if (off + (((uint64_t)len + 15) & ~15ull) > arena_bytes) continue;
        const uint64_t key = pkt_key(seed, first + p);
        const uint32_t proto = config == 0 ? 253u : config == 1 ? 17u : config == 2 ? 6u
                             : ((draw(key, 2) & 1u) ? 6u : 17u);
        const uint32_t old_ip = (uint32_t)((draw(key, 3) & 0xFFFFu) | 0x0101u);
        const uint32_t old_l4 = (uint32_t)((draw(key, 4) & 0xFFFFu) | 0x0101u);
        uint4* dst = (uint4*)(arena + off);
        const uint32_t nch = (len + 15u) >> 4;
        for (uint32_t c = lane; c < nch; c += 64u) {
            uint64_t q[2] = {draw(key, 16 + 2 * c), draw(key, 17 + 2 * c)};
            uint8_t* b = (uint8_t*)q;
            for (uint32_t j = 0; j < 16; ++j) {
                const uint32_t o = c * 16u + j;
                if (o >= len) b[j] = 0;
                else if (o < 64) {
                    int hb = hdr_byte(o, len, proto, old_ip, old_l4);
                    if (hb >= 0) b[j] = (uint8_t)hb;
                }
            }
            uint4 v;
            v.x = (uint32_t)q[0]; v.y = (uint32_t)(q[0] >> 32);
            v.z = (uint32_t)q[1]; v.w = (uint32_t)(q[1] >> 32);
            dst[c] = v;
        }
    }
}

hipError_t launch_gen_config(const DevInfo& di, int config, uint64_t seed, uint64_t first,
                             uint32_t n, uint8_t* arena, uint64_t arena_bytes,
                             const nfcs_desc* desc, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    uint32_t grid = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    if (grid > (uint32_t)di.cus * 8u) grid = (uint32_t)di.cus * 8u;
    hipLaunchKernelGGL(gen_config_kernel, dim3(grid), dim3(kBlock), 0, stream, config, seed,
                       first, n, arena, arena_bytes, desc);
    return hipGetLastError();
}

// ---- order-independent frame digest (same as oracle nfo_digest) --------------
__global__ __launch_bounds__(kBlock) void digest_kernel(const uint8_t* __restrict__ arena,
                                                        uint64_t arena_bytes,
                                                        const nfcs_desc* __restrict__ desc,
                                                        uint32_t n, uint64_t first,
                                                        unsigned long long* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    uint64_t wsum = 0;  // uniform
    for (uint32_t p = blockIdx.x * kWavesPerBlock + rfl(threadIdx.x >> 6); p < n; p += nw) {
        const nfcs_desc d = desc[p];
        const uint64_t off = (uint64_t)d.off16 * 16u;
        const uint32_t len = d.len;
        if (off + (((uint64_t)len + 15) & ~15ull) > arena_bytes) continue;
        const uint4* src = (const uint4*)(arena + off);
        const uint32_t nch = (len + 15u) >> 4;
        uint64_t acc = 0;
        for (uint32_t c = lane; c < nch; c += 64u) {
            uint4 v = src[c];
            uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
            const uint32_t o = c * 16u;
            if (o + 16 > len) {  // bytes >= len read as zero
                const uint32_t keep = len - o;  // 1..15
                if (keep < 8) { lo &= (1ull << (8 * keep)) - 1ull; hi = 0; }
                else if (keep == 8) { hi = 0; }
                else { hi &= (1ull << (8 * (keep - 8))) - 1ull; }
            }
            acc += mix64(lo ^ mix64(hi + (uint64_t)(c + 1) * kGolden));
        }
        const uint64_t h = mix64((uint64_t)len * 0xD6E8FEB86659FD93ull + wave_sum64(acc));
        wsum += mix64(h ^ ((first + p) * 0xA0761D6478BD642Full));
    }
    if (lane == 0 && wsum) atomicAdd(out, (unsigned long long)wsum);
}

hipError_t launch_digest(const DevInfo& di, const uint8_t* arena, uint64_t arena_bytes,
                         const nfcs_desc* desc, uint32_t n, uint64_t first, uint64_t* d_out,
                         hipStream_t stream) {
    if (n == 0) return hipSuccess;
    uint32_t grid = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    if (grid > (uint32_t)di.cus * 8u) grid = (uint32_t)di.cus * 8u;
    hipLaunchKernelGGL(digest_kernel, dim3(grid), dim3(kBlock), 0, stream, arena, arena_bytes,
                       desc, n, first, (unsigned long long*)d_out);
    return hipGetLastError();
}

}  // namespace nfcs
