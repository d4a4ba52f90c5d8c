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

constexpr int kHdr = 96;  // header bytes staged in LDS per wave: l4 <= 78, fields <= l4+17

DEV uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
DEV uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// End-around-carry fold of an exact sum to 16 bits (packet.hpp:907-909). Zero stays zero;
// a nonzero multiple of 0xFFFF folds to 0xFFFF, as in the reference.
DEV uint32_t fold64(uint64_t s) {
    s = (s & 0xFFFFFFFFull) + (s >> 32);
    while (s >> 16) s = (s & 0xFFFFull) + (s >> 16);
    return (uint32_t)s;
}

// ---- LDS header accessors (wave-uniform offsets) -------------------------------------------
DEV uint32_t h8(const uint8_t* h, uint32_t o) { return rfl(h[o]); }
DEV uint32_t hbe16(const uint8_t* h, uint32_t o) {  // o even
    return bswap16(rfl(*(const uint16_t*)(h + o)));
}
DEV uint32_t hle16(const uint8_t* h, uint32_t o) {  // o even
    return rfl(*(const uint16_t*)(h + o));
}

// ---- parse: everything update_checksums() decides, on wave-uniform values -------------------
struct Plan {
    uint32_t st;      // NFCS_ST_* (without the overlap flag)
    uint32_t mode;    // 0: write nothing, 1: fast path, 2: sequential path
    uint32_t has_ip;  // IPv4 header checksum to write at ip_off (value ip_val, LE store)
    uint32_t ip_off, ip_val;
    uint32_t has_l4;  // L4 checksum over [rs, re) written at fs, fs+1
    uint32_t rs, re, fs;
    uint32_t udp;     // 0 -> 0xFFFF rule
    uint32_t tailfix; // odd region: trailing byte counts as the low byte
    uint64_t add;     // exact LE-domain constant: pseudo-header
    uint64_t sub;     // exact LE-domain bytes counted by the dword sum but not by the reference
};

DEV Plan parse(const uint8_t* h, uint32_t len) {
    Plan P;
    P.st = NFCS_ST_NONE; P.mode = 0; P.has_ip = 0; P.ip_off = 0; P.ip_val = 0; P.has_l4 = 0;
    P.rs = P.re = P.fs = 0; P.udp = 0; P.tailfix = 0; P.add = 0; P.sub = 0;

    // ethernet(), packet.hpp:405-418 (len < 14 keeps the ctor's 14, 346)
    uint32_t l2 = 14;
    if (len >= 14) l2 = (hbe16(h, 12) == 0x8100u) ? 18u : 14u;
    uint32_t v4 = 0, proto = 0, ihl4 = 0, l4 = 0;
    uint32_t b0 = (l2 + 20 <= len) ? h8(h, l2) : 0;
    if (l2 + 20 <= len && (b0 >> 4) == 4) {  // 728-734: IPv4 by version nibble
        v4 = 1;
        proto = h8(h, l2 + 9);
        ihl4 = (b0 & 15u) * 4u;
        l4 = l2 + ihl4;
        if (l2 + ihl4 > len) { P.st = NFCS_ST_OOB; return P; }  // ref reads past the frame
        if (ihl4 < 20 && (proto == 6 || proto == 17 || proto == 1)) {
            P.mode = 2;  // L4 region overlaps the IPv4 header: sequential path
            return P;
        }
        // 739-740: checksum over ihl4 bytes with the field (l2+10) zeroed
        uint32_t s = 0;
        for (uint32_t w = 0; w < ihl4; w += 2)
            if (w != 10) s += hle16(h, l2 + w);
        P.has_ip = 1;
        P.ip_off = l2 + 10;
        P.ip_val = (~fold64(s)) & 0xFFFFu;
        P.mode = 1;
        P.st = NFCS_ST_V4;
    } else {
        // 741-765: effective EtherType after one 0x8100 tag; IPv6 needs the nibble too
        uint32_t et = (len >= 14) ? hbe16(h, 12) : 0;
        if (et == 0x8100u) et = (len >= 18) ? hbe16(h, 16) : 0;
        if (et != 0x86DDu) return P;
        if (!(l2 + 40 <= len && (h8(h, l2) >> 4) == 6)) return P;
        proto = h8(h, l2 + 6);
        l4 = l2 + 40;
        P.st = NFCS_ST_V6;
    }
    const uint32_t skip = v4 ? NFCS_ST_V4_L4SKIP : NFCS_ST_V6_L4SKIP;
    uint32_t L = 0;
    if (proto == 6) {  // 773-823
        if (l4 + 19 > len) { P.st = skip; return P; }   // sizeof(TcpHeader) == 19
        uint32_t hl = (h8(h, l4 + 12) >> 4) * 4u;
        if (v4) {
            uint32_t tl = hbe16(h, l2 + 2);
            if (tl < ihl4) { P.st = skip; return P; }
            L = (tl - ihl4) & 0xFFFFu;
        } else {
            L = hbe16(h, l2 + 4);
        }
        if (L < hl || l4 + L > len) { P.st = skip; return P; }
        P.fs = l4 + 15;  // TcpHeader::checksum at offset 15 under #pragma pack(1)
        P.st = v4 ? NFCS_ST_V4_TCP : NFCS_ST_V6_TCP;
    } else if (proto == 17) {  // 824-872
        if (l4 + 8 > len) { P.st = skip; return P; }
        L = hbe16(h, l4 + 4);
        if (L < 8 || l4 + L > len) { P.st = skip; return P; }
        P.fs = l4 + 6;
        P.udp = 1;
        P.st = v4 ? NFCS_ST_V4_UDP : NFCS_ST_V6_UDP;
    } else if (proto == 1 && v4) {  // 873-889
        if (l4 + 8 > len) { P.st = skip; return P; }
        uint32_t tl = hbe16(h, l2 + 2);
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
    // + bswap16(length word). IPv6's 32-bit length has a zero upper word (L <= 0xFFFF).
    uint64_t add = bswap16(proto) + bswap16(L);
    if (proto != 1) {
        if (v4) {
            for (uint32_t w = 0; w < 8; w += 2) add += hle16(h, l2 + 12 + w);
        } else {
            for (uint32_t w = 0; w < 32; w += 2) add += hle16(h, l2 + 8 + w);
        }
    } else {
        add = 0;  // ICMP: no pseudo-header
    }
    P.add = add;
    // Exact corrections of the dword sum: the vector pass starts at rs & ~3 (l4 is even,
    // so it may include the two bytes rs-2, rs-1 = one LE word), and it includes the raw
    // checksum field bytes that the reference zeroed first (795 / 838 / 885).
    uint64_t sub = 0;
    if (P.rs & 2u) sub += hle16(h, P.rs - 2);
    for (uint32_t b = P.fs; b < P.fs + 2; ++b)
        if (b >= P.rs && b < P.re) sub += (uint64_t)h8(h, b) << ((b & 1u) ? 8 : 0);
    P.sub = sub;
    // odd region: the trailing byte (at an even frame offset, so the LOW byte of its LE word
    // in the dword sum) must count as the HIGH byte: +255*b, unless it is a zeroed field byte
    uint32_t t = P.re - 1;
    P.tailfix = (L & 1u) && !(t >= P.fs && t < P.fs + 2);
    return P;
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

// ---- vector pass ----------------------------------------------------------------------------
DEV uint32_t lowmask(int n) {  // bytes [0, n) of a dword, n clamped to [0, 4]
    n = n < 0 ? 0 : (n > 4 ? 4 : n);
    return n >= 4 ? 0xFFFFFFFFu : ((1u << (8 * n)) - 1u);
}
DEV uint32_t comp(const uint4& v, uint32_t j) {
    return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// Add chunk (16 bytes at frame offset o) restricted to dwords from lo4 (4-aligned) up to
// byte re, plus the odd-tail fix.
DEV void acc_chunk(uint64_t& acc, const uint4& v, uint32_t o, uint32_t lo4, uint32_t re,
                   uint32_t tailfix) {
    if (o >= re) return;
    if (o >= lo4 && o + 16 <= re) {
        acc += (uint64_t)v.x + v.y + (uint64_t)v.z + v.w;
    } else {
        uint64_t a = 0;
        a += (o + 0 >= lo4) ? (v.x & lowmask((int)re - (int)(o + 0))) : 0u;
        a += (o + 4 >= lo4) ? (v.y & lowmask((int)re - (int)(o + 4))) : 0u;
        a += (o + 8 >= lo4) ? (v.z & lowmask((int)re - (int)(o + 8))) : 0u;
        a += (o + 12 >= lo4) ? (v.w & lowmask((int)re - (int)(o + 12))) : 0u;
        uint32_t t = re - 1;
        if (tailfix && t >= o && t < o + 16) {
            uint32_t d = comp(v, (t - o) >> 2);
            a += 255u * ((d >> (8 * (t & 3u))) & 0xFFu);
        }
        acc += a;
    }
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

template <int K>
struct Batch {
    uint4 v[K];
};

// One packet's staged state: descriptor and its first batch of K0 chunks per lane.
template <int K0>
struct Staged {
    uint64_t off;  // byte offset of the frame in the arena (wave-uniform)
    uint32_t len;
    uint32_t bad;
    Batch<K0> b;
};

template <int K0>
DEV void stage(Staged<K0>& S, const uint8_t* __restrict__ arena, uint64_t arena_bytes,
               const nfcs_desc* __restrict__ desc, uint32_t p, uint32_t base16, uint32_t lane) {
    const nfcs_desc d = desc[p];  // uniform -> s_load_dwordx2
    const uint64_t off = ((uint64_t)d.off16 - base16) * 16u;
    S.off = off;
    S.len = d.len;
    S.bad = (d.off16 < base16) || (off + (((uint64_t)d.len + 15u) & ~15ull) > arena_bytes);
    const uint32_t nch = S.bad ? 0u : (d.len + 15u) >> 4;
    const uint4* src = (const uint4*)(arena + off);
#pragma unroll
    for (int k = 0; k < K0; ++k) {
        const uint32_t c = lane + 64u * k;
        S.b.v[k] = (c < nch) ? src[c] : make_uint4(0, 0, 0, 0);
    }
}

template <int K0, int K1>
DEV void process(const Staged<K0>& S, uint8_t* arena, uint32_t p, uint32_t lane, uint8_t* hdr,
                 uint8_t* status, nfcs_patch* patch) {
    uint32_t st;
    uint32_t ip_off = NFCS_PATCH_NONE, ip_val = 0, l4_off = NFCS_PATCH_NONE, l4_val = 0;
    uint8_t* frame = arena + S.off;
    if (S.bad) {
        st = NFCS_ST_BAD_DESC;
    } else {
        // header bytes [0, 96) from lanes 0..5 into this wave's LDS slot
        if (lane < kHdr / 16) ((uint4*)hdr)[lane] = S.b.v[0];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const Plan P = parse(hdr, S.len);
        st = P.st;
        if (P.mode == 2) {
            SeqOut o = {0, 0, 0, 0, 0};
            if (lane == 0) o = seq_update(frame, S.len);
            st = rfl(o.st) | NFCS_ST_FLAG_OVERLAP;
            ip_off = rfl(o.ip_off); ip_val = rfl(o.ip_val);
            l4_off = rfl(o.l4_off); l4_val = rfl(o.l4_val);
        } else if (P.mode == 1) {
            if (P.has_l4) {
                const uint32_t lo4 = P.rs & ~3u, re = P.re;
                const uint32_t nre = (re + 15u) >> 4;  // chunks that hold region bytes
                uint64_t acc = 0;
#pragma unroll
                for (int k = 0; k < K0; ++k) {
                    const uint32_t c = lane + 64u * k;
                    if (64u * k < nre) acc_chunk(acc, S.b.v[k], c * 16u, lo4, re, P.tailfix);
                }
                // continuation batches (jumbo frames): K1 chunks per lane each
                const uint4* src = (const uint4*)frame;
                for (uint32_t cb = 64u * K0; cb < nre; cb += 64u * K1) {
                    Batch<K1> B;
#pragma unroll
                    for (int k = 0; k < K1; ++k) {
                        const uint32_t c = cb + lane + 64u * k;
                        B.v[k] = (c < nre) ? src[c] : make_uint4(0, 0, 0, 0);
                    }
#pragma unroll
                    for (int k = 0; k < K1; ++k) {
                        const uint32_t c = cb + lane + 64u * k;
                        acc_chunk(acc, B.v[k], c * 16u, lo4, re, P.tailfix);
                    }
                }
                const uint64_t z = wave_sum64(acc) - P.sub + P.add;
                uint32_t c = (~fold64(z)) & 0xFFFFu;  // LE-domain complement = bswap of ref value
                if (P.udp && c == 0) c = 0xFFFFu;
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
    __shared__ __attribute__((aligned(16))) uint8_t s_hdr[kWavesPerBlock][kHdr];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wib = rfl(threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    uint32_t p = blockIdx.x * kWavesPerBlock + wib;
    if (p >= n) return;
    uint8_t* hdr = s_hdr[wib];
    Staged<K0> A;
    stage<K0>(A, arena, arena_bytes, desc, p, base16, lane);
    for (;;) {
        const uint32_t pn = p + nw;
        const bool more = pn < n && pn > p;
        Staged<K0> B;
        if (more) stage<K0>(B, arena, arena_bytes, desc, pn, base16, lane);
        process<K0, K1>(A, arena, p, lane, hdr, status, patch);
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
