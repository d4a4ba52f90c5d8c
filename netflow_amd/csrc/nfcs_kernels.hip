// nfcs_kernels.hip — CDNA4 (gfx950) kernels of the batched Internet-checksum engine.
//
// The hot path is NetFlow++'s Packet::update_checksums() (include/netflow++/packet.hpp:722-890)
// with its fold Packet::calculate_checksum() (packet.hpp:894-912), applied to a batch of
// frames in HBM. Design (every choice below was A/B-measured, profiles/):
//
//  * One 16-lane DPP row per packet, four packets per wave64, 16 packets per 256-thread
//    workgroup, one workgroup per 16 packets (no grid-stride loop). Lane rl of a row loads
//    chunks rl, rl+16, ... of its frame as 16-byte global_load_dwordx4 (a row reads 256
//    contiguous bytes per instruction); K = 6 slots cover a 1536-byte frame in one batch,
//    longer (jumbo) frames continue in further batches of K slots.
//  * The descriptors of a wave's four packets are consecutive: one scalar s_load_dwordx8.
//  * All per-packet decisions run on the VALU, so one instruction serves four packets. (A
//    wave-per-packet kernel with the parse on SGPRs measured 364 SALU + 194 VALU instructions
//    per 1500-byte packet and was bound by the CU's single scalar unit at 1.9 TB/s.)
//  * Header fields reach the whole row by DPP row_newbcast at compile-time offsets: an
//    802.1Q tag is removed once per lane (one row_shl:1 + 4 selects), and the common headers
//    (untagged/tagged x IPv4 IHL 5 / IPv6 / non-IP) are planned at constant offsets. Anything
//    else (IP options, IHL < 5, headers past the frame) is parsed by the row's lane 0 from
//    memory; IHL < 5 overlaps run an exact sequential emulation of the reference.
//  * The L4 region is summed as little-endian dwords into an exact 64-bit per-lane sum. The
//    one's-complement sum is byte-order independent (RFC 1071 §2(B)): the LE-domain fold is
//    bswap16 of the reference's big-endian fold, so one swap at the end replaces the
//    reference's per-word ntohs. Full chunks are added unmasked; at most two boundary chunks
//    per packet are masked. The checksum field bytes (which the reference zeroes) and the 2
//    bytes before a region starting at 2 mod 4 are subtracted exactly; the odd trailing byte,
//    which the reference adds as the LOW byte (packet.hpp:903-905), gets +255*b.
//  * Row sum: four DPP steps. Final fold, complement, UDP 0 -> 0xFFFF (packet.hpp:867-871),
//    then the 2+2 checksum bytes are stored from lanes 0..3 of the row.
//  * Cache policy: the header slot is loaded with the default policy and the payload slots
//    with non-temporal (evict-first) loads (measured best for the 1500-byte config).
//  * No MFMA and no LDS staging: this is an HBM-read-bound integer fold.
#include "nfcs_internal.h"

namespace nfcs {

#define DEV __device__ __forceinline__

DEV uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// XCD-aware block order: workgroups are dealt to the 8 XCDs round-robin; this bijection on
// [0, gridDim.x) gives each XCD one contiguous eighth of the blocks (the tail beyond a
// multiple of 8 keeps its order).
DEV uint32_t xcd_block_n(uint32_t nblocks) {
    const uint32_t b = blockIdx.x, g8 = nblocks / 8u;
    return b < 8u * g8 ? (b % 8u) * g8 + b / 8u : b;
}
DEV uint32_t xcd_block() { return xcd_block_n(gridDim.x); }
DEV uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// The target of every load of a lane past its frame (or, in a line-aligned window, before it): every
// load is issued by every lane, so a wave's compiler-counted vmcnt waits stay static. One zero line,
// aligned to 4 KB, so its page offset never depends on what the linker places before it (round 4's
// 16-byte g_zero16 sat wherever the linker put it). Round 5 measured the alternatives on one box,
// alternating builds (profiles/r05_zero_target_ab.jsonl): one chunk per slot of a pool,
// the same instruction's first in-frame chunk (no extra request, but ~12 more instructions per slot
// ahead of the loads: C1 -2.5%, the C4 shard -2%), the wave's row-0 frame start — none faster; and the
// forward's C3 mix moves by +-3% from run to run in every form, round 4's as well.
__device__ __attribute__((aligned(4096))) uint4 g_zero_line[8];

// Component j of a uint4 by mask arithmetic (no indexable temporary, so no scratch).
DEV uint32_t comp(const uint4& v, uint32_t j) {
    const uint32_t m0 = 0u - (uint32_t)(j == 0), m1 = 0u - (uint32_t)(j == 1);
    const uint32_t m2 = 0u - (uint32_t)(j == 2), m3 = 0u - (uint32_t)(j == 3);
    return (v.x & m0) | (v.y & m1) | (v.z & m2) | (v.w & m3);
}


DEV uint4 put_byte(const uint4& v, uint32_t i, uint32_t b) {
    uint32_t r[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t sh = 8u * (i & 3u);
        const uint32_t m = ((i >> 2) == j) ? (0xFFu << sh) : 0u;
        r[j] = (comp(v, j) & ~m) | ((b << sh) & m);
    }
    return make_uint4(r[0], r[1], r[2], r[3]);
}

// Lane rl's chunk register v (frame bytes 16*rl .. 16*rl+15) with the 2-byte field w patched in
// (w: frame offset in the low half, the byte for that offset in bits 16-23, the next in 24-31;
// offset 0xFFFF = none). A field inside one dword — every fast-path header's — is one masked
// 16-bit insert; one that straddles two dwords goes byte by byte. In the fused L3 forward's
// segment store it took the forward on the C3 mix from 0.511 to 0.536 (its short waves are
// latency-bound and this VALU sits on their path).
DEV uint4 put_field(const uint4& v, uint32_t w, uint32_t rl) {
    const uint32_t pos = w & 0xFFFFu;
    if (pos == NFCS_PATCH_NONE || (pos & 3u) != 3u) {
        const bool mine = pos != NFCS_PATCH_NONE && (pos >> 4) == rl;
        const uint32_t sh = 8u * (pos & 3u), j = (pos >> 2) & 3u;
        const uint32_t m = mine ? (0xFFFFu << sh) : 0u, b = ((w >> 16) << sh) & m;
        return make_uint4(j == 0 ? ((v.x & ~m) | b) : v.x, j == 1 ? ((v.y & ~m) | b) : v.y,
                          j == 2 ? ((v.z & ~m) | b) : v.z, j == 3 ? ((v.w & ~m) | b) : v.w);
    }
    uint4 r = v;
    if ((pos >> 4) == rl) r = put_byte(r, pos & 15u, (w >> 16) & 0xFFu);
    if (((pos + 1u) >> 4) == rl) r = put_byte(r, (pos + 1u) & 15u, (w >> 24) & 0xFFu);
    return r;
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
// The L4 region is summed as 16-bit little-endian words: v_sad_u16(d, 0, acc) adds both
// halves of a dword to a u32 accumulator in one instruction, with no carry chain. The word
// sum is congruent to the dword sum mod 0xFFFF (65536 = 1 mod 0xFFFF) and both are zero
// exactly when every byte is, so they fold to the same checksum; it cannot overflow 32 bits
// (a region ends before l4 + 65,536 < 65,614 bytes: 16,404 dwords x 131,070 < 2^32).
DEV uint32_t wsum(uint32_t d, uint32_t acc) { return __builtin_amdgcn_sad_u16(d, 0u, acc); }

DEV uint32_t add_chunk(const uint4& v, uint32_t acc) {
    return wsum(v.w, wsum(v.z, wsum(v.y, wsum(v.x, acc))));
}

// End-around-carry fold of an exact sum to 16 bits (packet.hpp:907-909), branch-free: two
// steps take any u32 below 0x10000 (a further step on such a value is the identity, so this
// equals the reference's while loop). Zero stays zero; a nonzero multiple of 0xFFFF folds to
// 0xFFFF, as in the reference.
DEV uint32_t fold32(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);  // <= 0x1FFFE
    return (s & 0xFFFFu) + (s >> 16);
}

// =============================================================================================
// v3: one 16-lane DPP row per packet, four packets per wave, all per-packet logic on the VALU.
//
// v2 (one wave per packet, parse on SGPRs) measured 364 SALU + 194 VALU instructions per
// 1500 B packet: the CU's single scalar unit, not HBM, set the rate (profiles/). Here every
// per-packet decision runs once per 16-lane row, so one VALU instruction serves four packets
// and the scalar unit only runs the loop. Lane rl of a row holds chunks rl, rl+16, ... of its
// packet; header dwords reach the whole row by DPP row_newbcast (compile-time offsets) or
// ds_bpermute (runtime offsets: IP options, IPv6); the row sum is four DPP steps.
// =============================================================================================

// Lane L of this lane's packet row. R = 16: one DPP row_newbcast. R = 8 (two packets per DPP
// row): row_newbcast L into banks 0-1 (lanes 0-7), row_newbcast 8+L into banks 2-3 (8-15).
template <int L, int R = 16>
DEV uint32_t row_bcast(uint32_t x) {
    static_assert(R == 16 || R == 8, "row width");
    if (R == 16) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + L, 0xF, 0xF, false);
    const int lo = __builtin_amdgcn_mov_dpp((int)x, 0x150 + (L & 7), 0xF, 0x3, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(lo, (int)x, 0x158 + (L & 7), 0xF, 0xC, false);
}

// Per-lane view of the header bytes [0, 16R) of the row's packet: lane rl of the row holds
// chunk rl (frame bytes 16rl .. 16rl+15) of slot 0. Every header field the plan reads lies
// below byte 128, so R = 8 rows see all of them.
template <int R>
struct RowHdr {
    uint4 c0;
    uint32_t rowbase4;  // byte address of lane 0 of this row, for ds_bpermute
    DEV uint32_t dw(uint32_t q) const {
        const uint32_t x = comp(c0, q & 3u);
        if (__builtin_constant_p(q)) {
            switch ((q >> 2) & (R - 1)) {
            case 0: return row_bcast<0, R>(x);   case 1: return row_bcast<1, R>(x);
            case 2: return row_bcast<2, R>(x);   case 3: return row_bcast<3, R>(x);
            case 4: return row_bcast<4, R>(x);   case 5: return row_bcast<5, R>(x);
            case 6: return row_bcast<6, R>(x);   case 7: return row_bcast<7, R>(x);
            case 8: return row_bcast<8, R>(x);   case 9: return row_bcast<9, R>(x);
            case 10: return row_bcast<10, R>(x); case 11: return row_bcast<11, R>(x);
            case 12: return row_bcast<12, R>(x); case 13: return row_bcast<13, R>(x);
            case 14: return row_bcast<14, R>(x); default: return row_bcast<15, R>(x);
            }
        }
        return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(rowbase4 + ((q >> 2) & (R - 1)) * 4u), (int)x);
    }
    DEV uint32_t b(uint32_t o) const { return (dw(o >> 2) >> (8 * (o & 3u))) & 0xFFu; }
    DEV uint32_t le16(uint32_t o) const { return (dw(o >> 2) >> (8 * (o & 2u))) & 0xFFFFu; }
    DEV uint32_t be16(uint32_t o) const { return bswap16(le16(o)); }
};

// Compact per-lane plan (row-uniform values).
enum : uint32_t { F_IP = 1, F_L4 = 2, F_UDP = 4, F_TAIL = 8, F_SEQ = 16 };
struct RPlan {
    uint32_t st;     // status byte
    uint32_t flags;  // F_*
    uint32_t ipw;    // ip_off | ip_val << 16
    uint32_t rs, re, fs;
    uint32_t corr;   // pseudo-header words minus over-counted bytes (two's complement)
};

DEV RPlan rplan_none(uint32_t st) {
    RPlan P;
    P.st = st; P.flags = 0; P.ipw = 0; P.rs = 0; P.re = 0; P.fs = 0; P.corr = 0;
    return P;
}

// Header bytes with an 802.1Q tag removed: view byte o (o >= 12) is frame byte o + 4*tagged.
// The reference's offsets are all relative to l2 = 14 or 18 (ethernet(), packet.hpp:405-418),
// so one plan written at l2 = 14 serves both framings. Each lane shifts its own chunk by one
// dword (the 4th dword comes from the next lane of the row via DPP row_shl:1), so every
// header access afterwards is a single row broadcast at a compile-time offset.
DEV uint4 strip_tag(const uint4& c, bool tagged) {
    const uint32_t nx = (uint32_t)__builtin_amdgcn_mov_dpp((int)c.x, 0x101, 0xF, 0xF, true);
    const uint32_t m = 0u - (uint32_t)tagged;
    return make_uint4((c.x & ~m) | (c.y & m), (c.y & ~m) | (c.z & m),
                      (c.z & ~m) | (c.w & m), (c.w & ~m) | (nx & m));
}


// L4 branch of packet.hpp:773-889 in view coordinates with compile-time l2 = 14 and l4
// (34 for IPv4 with IHL 5, 54 for IPv6); sh = 4 for tagged frames shifts the frame offsets.
template <int R>
DEV RPlan fast_l4(const RowHdr<R>& V, RPlan P, uint32_t lenv, uint32_t v4, uint32_t l4, uint32_t proto,
                  uint32_t sh) {
    const uint32_t l2 = 14, ihl4 = 20;
    const uint32_t skip = v4 ? NFCS_ST_V4_L4SKIP : NFCS_ST_V6_L4SKIP;
    uint32_t L, fs, st, fl = F_L4;
    if (proto == 6) {
        if (l4 + 19 > lenv) { P.st = skip; return P; }  // sizeof(TcpHeader) == 19
        const uint32_t hl = (V.b(l4 + 12) >> 4) * 4u;
        if (v4) {
            const uint32_t tl = V.be16(l2 + 2);
            if (tl < ihl4) { P.st = skip; return P; }
            L = (tl - ihl4) & 0xFFFFu;
        } else {
            L = V.be16(l2 + 4);
        }
        if (L < hl || l4 + L > lenv) { P.st = skip; return P; }
        fs = l4 + 15;  // TcpHeader::checksum at offset 15 (19-byte packed struct)
        st = v4 ? NFCS_ST_V4_TCP : NFCS_ST_V6_TCP;
    } else if (proto == 17) {
        if (l4 + 8 > lenv) { P.st = skip; return P; }
        L = V.be16(l4 + 4);
        if (L < 8 || l4 + L > lenv) { P.st = skip; return P; }
        fs = l4 + 6;
        fl |= F_UDP;
        st = v4 ? NFCS_ST_V4_UDP : NFCS_ST_V6_UDP;
    } else if (proto == 1 && v4) {
        if (l4 + 8 > lenv) { P.st = skip; return P; }
        const uint32_t tl = V.be16(l2 + 2);
        if (tl < ihl4) { P.st = skip; return P; }
        L = tl - ihl4;
        if (l4 + L > lenv || L < 8) { P.st = skip; return P; }
        fs = l4 + 2;
        st = NFCS_ST_V4_ICMP;
    } else {
        return P;
    }
    uint32_t add = 0;
    if (proto != 1) {  // pseudo-header in the LE domain (797-816 / 840-859)
        add = bswap16(proto) + bswap16(L);
        if (v4) {
#pragma unroll
            for (uint32_t w = 0; w < 8; w += 2) add += V.le16(l2 + 12 + w);
        } else {
#pragma unroll
            for (uint32_t w = 0; w < 32; w += 2) add += V.le16(l2 + 8 + w);
        }
    }
    // over-counted bytes: the LE word before l4 when l4 = 2 mod 4 (sh keeps the parity), and
    // the raw checksum field bytes the reference zeroes first (795 / 838 / 885)
    const uint32_t re = l4 + L;
    uint32_t sub = ((l4 + sh) & 2u) ? V.le16(l4 - 2) : 0u;
    if (fs < re) sub += V.b(fs) << (((fs + sh) & 1u) ? 8 : 0);
    if (fs + 1 < re) sub += V.b(fs + 1) << (((fs + 1 + sh) & 1u) ? 8 : 0);
    const uint32_t t = re - 1;
    if ((L & 1u) && !(t >= fs && t < fs + 2)) fl |= F_TAIL;
    P.st = st;
    P.flags |= fl;
    P.rs = l4 + sh;
    P.re = re + sh;
    P.fs = fs + sh;
    P.corr = add - sub;
    return P;
}

// fast_l4 for IPv4 with IHL 5 (l4 = 34 in view coordinates), its three protocol branches evaluated
// side by side and merged by selects: every field sits at a compile-time offset (one row_newbcast per
// dword), so a wave whose rows carry different protocols (C3 mixes TCP and UDP in most waves) runs one
// pass instead of one per protocol, and the checksum field's bytes are read at their constant offsets
// instead of through two runtime-indexed ds_bpermute round trips. Same conditions and values as
// fast_l4 (packet.hpp:773-889).
template <int R>
DEV RPlan fast_l4_v4(const RowHdr<R>& V, RPlan P, uint32_t lenv, uint32_t proto, uint32_t sh) {
    const bool isT = proto == 6, isU = proto == 17, isI = proto == 1;
    const uint32_t d4 = V.dw(4), d6 = V.dw(6), d7 = V.dw(7), d8 = V.dw(8);
    const uint32_t d9 = V.dw(9), d10 = V.dw(10), d11 = V.dw(11), d12 = V.dw(12);
    const uint32_t tl = bswap16(d4 & 0xFFFFu);  // total length (bytes 16-17)
    const uint32_t lu = bswap16(d9 >> 16);      // udp.length (bytes 38-39)
    const uint32_t hl = (d11 >> 18) & 0x3Cu;    // TCP data offset * 4 (byte 46, high nibble)
    const uint32_t L = isU ? lu : ((tl - 20u) & 0xFFFFu);
    // the conditions combined with non-short-circuit & so they stay selects, not branches
    const bool inl = (34u + L <= lenv) & (42u <= lenv);
    const bool ok = (isT & (53u <= lenv) & (tl >= 20u) & (L >= hl) & inl) |  // sizeof(TcpHeader) == 19
                    (isU & (lu >= 8u) & inl) | (isI & (tl >= 20u) & (L >= 8u) & inl);
    const uint32_t fs = isT ? 49u : (isU ? 40u : 36u), re = 34u + L;
    // the raw field bytes the reference zeroes (LE weights): TCP 49 (high byte of word 48) and 50
    // (low byte of word 50), each only inside the region; UDP 40-41, ICMP 36-37 (always inside: L >= 8)
    const uint32_t ft = (d12 & ((49u < re) ? 0xFF00u : 0u)) + ((d12 >> 16) & ((50u < re) ? 0xFFu : 0u));
    const uint32_t fsub = isT ? ft : ((isU ? d10 : d9) & 0xFFFFu);
    // pseudo-header (src, dst, proto, length) in the LE domain; ICMP has none
    const uint32_t ph = bswap16(proto) + bswap16(L) + (d6 >> 16) + (d7 & 0xFFFFu) + (d7 >> 16) + (d8 & 0xFFFFu);
    const uint32_t add = isI ? 0u : ph;
    // over-counted: the LE word at 32 (l4 = 2 mod 4, sh keeps the parity) and the field bytes
    const uint32_t sub = (d8 & 0xFFFFu) + fsub;
    const uint32_t t = re - 1u;
    const bool tail = (L & 1u) & ((t < fs) | (t >= fs + 2u));
    const uint32_t st = ok ? (isT ? NFCS_ST_V4_TCP : (isU ? NFCS_ST_V4_UDP : NFCS_ST_V4_ICMP)) : NFCS_ST_V4_L4SKIP;
    P.st = (isT | isU | isI) ? st : P.st;
    P.flags |= ok ? (F_L4 | (isU ? F_UDP : 0u) | (tail ? F_TAIL : 0u)) : 0u;
    P.rs = ok ? 34u + sh : P.rs;
    P.re = ok ? re + sh : P.re;
    P.fs = ok ? fs + sh : P.fs;
    P.corr = ok ? add - sub : P.corr;
    return P;
}

// Common headers with compile-time offsets: untagged / 802.1Q; IPv4 with IHL 5; IPv6; non-IP.
// Returns F_SEQ in flags for everything else (IHL != 5: options, IHL < 5, past the frame).
template <int R>
DEV RPlan fast_plan(const uint4& c0, uint32_t rowbase4, uint32_t len) {
    const RowHdr<R> h{c0, rowbase4};
    const bool tagged = (len >= 14) && h.be16(12) == 0x8100u;  // ethernet(): l2 = 18
    const uint32_t sh = tagged ? 4u : 0u;
    const RowHdr<R> V{strip_tag(c0, tagged), rowbase4};
    const uint32_t lenv = len - sh;  // len >= 14 whenever tagged
    const uint32_t b0 = V.b(14);
    if (len >= 14 + sh && lenv >= 34 && (b0 >> 4) == 4) {  // 728-734: IPv4 by nibble
        if ((b0 & 15u) != 5) return rplan_none(NFCS_ST_NONE | (F_SEQ << 8));
        uint32_t s = 0;  // 739-740: header checksum, field zeroed
#pragma unroll
        for (uint32_t w = 0; w < 20; w += 2)
            if (w != 10) s += V.le16(14 + w);
        RPlan P = rplan_none(NFCS_ST_V4);
        P.flags = F_IP;
        P.ipw = (24u + sh) | (((~fold32(s)) & 0xFFFFu) << 16);
        return fast_l4_v4(V, P, lenv, V.b(23), sh);
    }
    // 741-765: effective EtherType (after one tag) must be IPv6 and the nibble 6
    const uint32_t et = (len >= 14 + sh) ? V.be16(12) : 0u;
    if (et != 0x86DDu || !(len >= 14 + sh && lenv >= 54 && (b0 >> 4) == 6))
        return rplan_none(NFCS_ST_NONE);
    return fast_l4(V, rplan_none(NFCS_ST_V6), lenv, 0u, 54u, V.b(20), sh);
}

// Any header, parsed by one lane from global memory (IP options, IHL < 5, past the frame).
__device__ __noinline__ RPlan slow_plan(const uint8_t* f, uint32_t len) {
    uint32_t l2 = 14;
    if (len >= 14) l2 = (g_be16(f, 12) == 0x8100u) ? 18u : 14u;
    RPlan P = rplan_none(NFCS_ST_NONE);
    uint32_t v4 = 0, proto, ihl4 = 0, l4;
    if (l2 + 20 <= len && (f[l2] >> 4) == 4) {
        v4 = 1;
        proto = f[l2 + 9];
        ihl4 = (f[l2] & 15u) * 4u;
        l4 = l2 + ihl4;
        if (l2 + ihl4 > len) return rplan_none(NFCS_ST_OOB);
        if (ihl4 < 20 && (proto == 6 || proto == 17 || proto == 1)) {
            P.flags = F_SEQ;  // overlapping headers: full sequential emulation
            return P;
        }
        uint32_t s = 0;
        for (uint32_t w = 0; w < ihl4; w += 2)
            if (w != 10) s += g_be16(f, l2 + w);
        P.st = NFCS_ST_V4;
        P.flags = F_IP;
        P.ipw = (l2 + 10) | (bswap16(g_fin(s)) << 16);
    } else {
        uint32_t et = (len >= 14) ? g_be16(f, 12) : 0;
        if (et == 0x8100u) et = (len >= 18) ? g_be16(f, 16) : 0;
        if (et != 0x86DDu || !(l2 + 40 <= len && (f[l2] >> 4) == 6)) return P;
        proto = f[l2 + 6];
        l4 = l2 + 40;
        P.st = NFCS_ST_V6;
    }
    const uint32_t skip = v4 ? NFCS_ST_V4_L4SKIP : NFCS_ST_V6_L4SKIP;
    uint32_t L, fs, st, fl = F_L4;
    if (proto == 6) {
        if (l4 + 19 > len) { P.st = skip; return P; }
        const uint32_t hl = (f[l4 + 12] >> 4) * 4u;
        if (v4) {
            const uint32_t tl = g_be16(f, l2 + 2);
            if (tl < ihl4) { P.st = skip; return P; }
            L = (tl - ihl4) & 0xFFFFu;
        } else {
            L = g_be16(f, l2 + 4);
        }
        if (L < hl || l4 + L > len) { P.st = skip; return P; }
        fs = l4 + 15;
        st = v4 ? NFCS_ST_V4_TCP : NFCS_ST_V6_TCP;
    } else if (proto == 17) {
        if (l4 + 8 > len) { P.st = skip; return P; }
        L = g_be16(f, l4 + 4);
        if (L < 8 || l4 + L > len) { P.st = skip; return P; }
        fs = l4 + 6;
        fl |= F_UDP;
        st = v4 ? NFCS_ST_V4_UDP : NFCS_ST_V6_UDP;
    } else if (proto == 1 && v4) {
        if (l4 + 8 > len) { P.st = skip; return P; }
        const uint32_t tl = g_be16(f, l2 + 2);
        if (tl < ihl4) { P.st = skip; return P; }
        L = tl - ihl4;
        if (l4 + L > len || L < 8) { P.st = skip; return P; }
        fs = l4 + 2;
        st = NFCS_ST_V4_ICMP;
    } else {
        return P;
    }
    uint32_t add = 0;
    if (proto != 1) {
        add = bswap16(proto) + bswap16(L);
        const uint32_t a0 = v4 ? l2 + 12 : l2 + 8, an = v4 ? 8u : 32u;
        for (uint32_t w = 0; w < an; w += 2) add += bswap16(g_be16(f, a0 + w));
    }
    const uint32_t re = l4 + L;
    uint32_t sub = (l4 & 2u) ? bswap16(g_be16(f, l4 - 2)) : 0u;
    if (fs < re) sub += (uint32_t)f[fs] << ((fs & 1u) ? 8 : 0);
    if (fs + 1 < re) sub += (uint32_t)f[fs + 1] << (((fs + 1) & 1u) ? 8 : 0);
    const uint32_t t = re - 1;
    if ((L & 1u) && !(t >= fs && t < fs + 2)) fl |= F_TAIL;
    P.st = st;
    P.flags |= fl;
    P.rs = l4;
    P.re = re;
    P.fs = fs;
    P.corr = add - sub;
    return P;
}

// Masked add of one boundary chunk at frame offset o: dwords from lo4 up to byte re, plus the
// odd-tail fix.
DEV uint32_t masked_chunk(const uint4& v, uint32_t o, uint32_t lo4, uint32_t re, uint32_t tailfix,
                          uint32_t acc) {
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t od = o + 4u * j;
        const int nb = (int)re - (int)od;
        uint32_t m = nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
        m = (od >= lo4) ? m : 0u;
        acc = wsum(comp(v, j) & m, acc);
    }
    const uint32_t t = re - 1;
    if (tailfix && t >= o && t < o + 16) acc += 255u * ((comp(v, (t - o) >> 2) >> (8 * (t & 3u))) & 0xFFu);
    return acc;
}

DEV void acc_slot(uint32_t& acc, const uint4& v, uint32_t c, uint32_t lo4, uint32_t re, uint32_t tailfix) {
    const uint32_t o = c * 16u;
    const bool full = (o >= lo4) && (o + 16u <= re);
    const bool part = !full && (o + 16u > lo4) && (o < re);
    if (full) acc = add_chunk(v, acc);
    if (part) acc = masked_chunk(v, o, lo4, re, tailfix, acc);
}

template <int R>
DEV uint32_t row_sum(uint32_t x) {  // every lane of an R-lane row gets the row's sum
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);   // quad_perm 1,0,3,2
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);   // quad_perm 2,3,0,1
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true);  // row_half_mirror
    if (R == 16) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true);  // row_mirror
    return x;
}

template <int R>
DEV uint32_t wave_max_rows(uint32_t x) {  // x row-uniform
    uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)x, 0);
#pragma unroll
    for (int l = R; l < 64; l += R) m = max(m, (uint32_t)__builtin_amdgcn_readlane((int)x, l));
    return m;
}

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
constexpr int kCpolNt = 2;  // buffer-load cache policy bits: nt (the global loads' non-temporal hint)

template <int NT>
DEV uint4 ld16(const uint4* p) {
    if (NT) {
        const u32x4_t t = __builtin_nontemporal_load((const u32x4_t*)p);
        return make_uint4(t.x, t.y, t.z, t.w);
    }
    return *p;
}

// Frame stores. WT: write-through at agent scope (`sc1`): the L2 keeps no dirty copy of the
// frame's line, so the line leaves as a clean eviction and the write goes to memory at once
// instead of as a later write-back in the middle of the read stream (session 3: C1 +2.5%,
// C3 +5% over plain stores; `sc0 sc1` measured the same, `sc0 sc1 nt` 5% worse).

template <bool WT>
DEV void st8(uint8_t* p, uint32_t b) {
    if (WT) __hip_atomic_store(p, (uint8_t)b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = (uint8_t)b;
}
// A byte store that goes to memory past the caches (`sc0 sc1 nt`: system scope, non-temporal).
DEV void st8_nt(uint8_t* p, uint32_t b) {
    asm volatile("global_store_byte %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(b) : "memory");
}
// The same for 16 bytes (the s_nop: see st16 below).
DEV void st16_nt(uint4* p, const uint4& v) {
    const u32x4_t t = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" ::"v"(p), "v"(t) : "memory");
}
template <bool WT>
DEV void st16(uint4* p, const uint4& v) {
    if (WT) {
        // One dwordx4 sc1 store. The s_nop covers the gfx9 hazard of a VALU write to the data
        // VGPRs of a store wider than 8 bytes right after it, which hipcc's hazard recognizer
        // does not see inside inline asm (without it the VLAN kernel stored clobbered dwords).
        // Two 8-byte atomic sc1 stores instead cost 37% on VLAN C1.
        const u32x4_t t = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(t) : "memory");
    } else {
        *p = v;
    }
}

// Descriptors of the wave's four rows: packets w, w+1, w+2, w+3 are consecutive in the
// descriptor array, so one wave-uniform scalar load (s_load_dwordx8) fetches all four; each
// lane picks its row's pair. Counted on lgkmcnt, so prefetching them never holds up a vmcnt
// wait for chunk data.
template <int P>  // packets per wave
struct DescW { uint32_t w[2 * P]; };

template <int P>
DEV DescW<P> load_descw(const nfcs_desc* __restrict__ desc, uint64_t pw, uint32_t n) {
    DescW<P> D;
    if (pw + P <= n) {
        const uint32_t* q = (const uint32_t*)(desc + pw);
#pragma unroll
        for (int i = 0; i < 2 * P; ++i) D.w[i] = q[i];
    } else {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            const bool ok = pw + i < n;
            D.w[2 * i] = ok ? desc[pw + i].off16 : 0u;
            D.w[2 * i + 1] = ok ? desc[pw + i].len : 0u;
        }
    }
    return D;
}

template <int P>
DEV nfcs_desc pick_desc(const DescW<P>& D, uint32_t row) {  // mask selects: no indexable temp
    nfcs_desc d;
    d.off16 = 0;
    d.len = 0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const uint32_t m = 0u - (uint32_t)(row == (uint32_t)i);
        d.off16 |= D.w[2 * i] & m;
        d.len |= D.w[2 * i + 1] & m;
    }
    return d;
}

// The wave's frames as one raw buffer resource (round 4): based at the lowest frame of the wave's
// rows (wave-uniform, from the descriptors in SGPRs), so a lane past its frame (or, in a line-aligned
// window, before it) gives an out-of-range offset and its load returns zeros with no memory request.
// With every such lane aimed at one shared zero chunk instead, up to half the load requests of a
// short-frame batch went to a single 16-byte address, and C3 moved by 3% with the link-time address
// of that chunk (profiles/r04_s2_zero_target_ab.jsonl). Used where it measured faster (rows_body's
// BUF: the plain update's short shape). ok = every row's frame starts within
// kBufSpan16 16-byte units of the base (32-bit offsets, a 64 KB frame on top); else row_stage loads
// through global addresses, lanes past the frame from the wave's zero chunk.
struct WaveBuf {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t lo16;
    bool ok;
};
constexpr uint32_t kBufSpan16 = (1u << 28) - (1u << 13);
constexpr uint32_t kBufOob = 0xFFFFFFF0u;  // num_records, and the offset of a lane past its frame

template <int P>
DEV WaveBuf wave_buf(const DescW<P>& D, uint64_t pw, uint32_t n, uint8_t* arena, uint32_t base16) {
    uint32_t lo = D.w[0], hi = D.w[0];  // row 0 is always a packet (the wave exits when pw >= n)
#pragma unroll
    for (int i = 1; i < P; ++i) {
        const uint32_t o = (pw + (uint64_t)i < n) ? D.w[2 * i] : D.w[0];
        lo = min(lo, o);
        hi = max(hi, o);
    }
    lo = rfl(lo);  // wave-uniform: a scalar branch in row_stage, not an exec-masked one
    hi = rfl(hi);
    WaveBuf b;
    b.lo16 = lo;
    b.ok = hi - lo < kBufSpan16;
    b.rs = __builtin_amdgcn_make_buffer_rsrc(arena + ((int64_t)lo - (int64_t)base16) * 16, (short)0, kBufOob,
                                             0x00020000);
    return b;
}

// One row's packet, staged: frame window and its first K slots of chunks in flight.
template <int K>
struct RowStage {
    uint4 v[K];
    uint8_t* frame;
    uint32_t len;   // 0 unless live
    uint32_t p;
    uint32_t valid, bad;
    uint32_t nh;    // fused L3 forward: next-hop index (row-uniform)
    uint32_t mis;   // 16-byte chunks between the frame start and the 128-byte line below it
};

// Per-launch extras of update_rows_kernel: the fused L3 forward's inputs (unused by the plain
// update) and the footprint observation slot (sample_footprint; null = none).
struct FwdArgs {
    const uint32_t* nh;
    const nfcs_nexthop* table;
    uint32_t table_n;
    ObsReq obs;
    DoneReq done = {};
};

// DoneReq (nfcs_internal.h): every wave releases its own frame / record / status stores at system scope
// (each wave's fence waits for that wave's stores; one lane's fence would not cover the other waves'
// stores still in flight), the barrier then has them all; one lane counts the workgroup (a vector
// atomic), and the workgroup that completes the count publishes it with a system-scope release store
// (a vector store), which the host's acquire load of the flag pairs with. Waves that had no packets reach
// the barrier too (update_rows_kernel returns early only without a DoneReq).
DEV void signal_done(const DoneReq& d, uint32_t nblocks) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t now = __hip_atomic_fetch_add(d.ctr, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1ull;
        if (now == d.base + nblocks) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            __hip_atomic_store(d.flag, now, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// The footprint of a call's frames — 256 descriptors spread evenly over the call's tag & 0xFFFFFFFF
// packets from desc (the whole call, also when it runs as sub-batches: the first sub-batch samples):
// the mean of their lengths rounded up to 128 bytes, how many of the 256 are longer than one 8-lane row
// pass (kTinyRowBytes), whether many start off a 128-byte line (kObsUnaligned), whether their rounded
// lengths vary (kObsMixed) and how many lie between minimum and full size (kObsMidShift) — written to
// *obs (host-mapped, system scope) by one wave of the launch, in one 64-bit store together with the
// burst's generation (tag >> 32), so the host can tell a late sample of an earlier burst from this
// one's: kObsPresent | bits | longs << kObsLongShift | mean (nfcs_internal.h). The
// next call over the same burst (descriptor array, n and arena_bytes) picks its launch shape from it
// when arena_bytes / n cannot tell (a burst inside a larger ring; a densely packed mix whose mean
// alone says 8-lane rows; nfcs_api.hip launch_shape). Speed only.
DEV void sample_footprint(const nfcs_desc* __restrict__ desc, uint64_t tag, uint32_t lane, uint64_t* obs) {
    const uint32_t n = (uint32_t)tag;
    uint32_t s = 0, c = 0, u = 0, md = 0, lo = 0xFFFFFFFFu, hi = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const nfcs_desc d = desc[(uint32_t)(((uint64_t)(4u * lane + k) * n) >> 8)];
        const uint32_t r = ((d.len < 0xFFFFu ? d.len : 0xFFFFu) + 127u) & ~127u;
        s += r;
        c += d.len > kTinyRowBytes ? 1u : 0u;
        u += (d.off16 & 7u) ? 1u : 0u;
        md += (r > 128u && r <= 1408u) ? 1u : 0u;
        lo = min(lo, r);
        hi = max(hi, r);
    }
    s = row_sum<16>(s);
    c = row_sum<16>(c);
    u = row_sum<16>(u);
    md = row_sum<16>(md);
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {  // wave min / max of the rounded lengths (one wave, once per launch)
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, m));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, m));
    }
    auto wave_total = [](uint32_t v) {
        return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
               (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    };
    const uint32_t t = wave_total(s), l = wave_total(c), un = wave_total(u), mid = wave_total(md) >> 5;
    const uint32_t bits = (un > kObsUnalignedMax ? kObsUnaligned : 0u) | (hi - lo > 128u ? kObsMixed : 0u) |
                          ((mid < 7u ? mid : 7u) << kObsMidShift);
    if (lane == 0)
        __hip_atomic_store(obs, (tag & 0xFFFFFFFF00000000ull) | kObsPresent | bits | (l << kObsLongShift) | (t >> 8),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Issue the row's K chunk loads: the header slot with the default cache policy (its lines are
// parsed and, with inline stores, written back while still in L2), payload slots non-temporal
// (evict-first). Every load is always issued — lanes past the frame read zeros: from g_zero_line, or
// in the BUF shape (the update's short shape) through an out-of-range buffer offset with no memory
// request (WaveBuf; g_zero_line again where a wave's frames span more than 4 GB) — so the waits are
// counted vmcnt waits. Line-aligned windows (LA, round 3): lane rl of slot k holds the chunk
// R*k + rl past the 128-byte line in which the frame starts, i.e. frame chunk R*k + rl - mis, so
// each load instruction covers whole lines (2 for 16-lane rows, 1 for 8-lane rows) whatever the
// frame's alignment; lanes before the frame start or past its end read zeros. Frame-relative
// windows on a frame that starts mid-line make every instruction touch one line more (densely
// packed frames: C1 -4.5%, C2 -8%, C3 -15%; 64-byte-aligned starts C1 -5%;
// profiles/r03_s3_ab_align*.jsonl). Without LA, mis = 0 and the windows are frame-relative.
template <int K, int R = 16, bool FWD = false, bool LA = false, bool BUF = false>
DEV void row_stage(RowStage<K>& S, uint8_t* arena, uint64_t arena_bytes, const nfcs_desc& d,
                   uint64_t p64, uint32_t n, uint32_t base16, uint32_t rl, const WaveBuf& wb, uint32_t nh = 0) {
    const bool valid = p64 < n;
    const uint64_t off = ((uint64_t)d.off16 - base16) * 16u;
    const bool bad = valid && ((d.off16 < base16) ||
                               (off + (((uint64_t)d.len + 15u) & ~15ull) > arena_bytes));
    const bool live = valid && !bad;
    S.valid = valid;
    S.bad = bad;
    S.p = (uint32_t)p64;
    S.len = live ? d.len : 0u;
    S.frame = arena + (live ? off : 0);
    S.mis = LA && live ? (uint32_t)(((uintptr_t)S.frame >> 4) & 7u) : 0u;
    const uint32_t nch = (S.len + 15u) >> 4;
    const uint4* src = (const uint4*)S.frame;
    if (FWD) S.nh = nh;  // its MACs arrive as wave-uniform scalars (update_rows_kernel)
    if (BUF && wb.ok) {  // wave-uniform
        const uint32_t rel = (d.off16 - wb.lo16) * 16u;  // the row's frame in the wave's buffer
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = rl + (uint32_t)R * k - S.mis;  // frame chunk (wraps below the frame start)
            const uint32_t vo = (c < nch) ? rel + 16u * c : kBufOob;
            const u32x4_t t = k == 0 ? __builtin_amdgcn_raw_buffer_load_b128(wb.rs, vo, 0, 0)
                                     : __builtin_amdgcn_raw_buffer_load_b128(wb.rs, vo, 0, kCpolNt);
            S.v[k] = make_uint4(t.x, t.y, t.z, t.w);
        }
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = rl + (uint32_t)R * k - S.mis;
            const uint4* a = (c < nch) ? src + c : g_zero_line;
            S.v[k] = k == 0 ? ld16<0>(a) : ld16<1>(a);
        }
    }
    // all K loads issue before any use of the header slot: without this fence the scheduler
    // hoists the forward decision's first DPP read above the last loads of the FWD kernel and
    // waits for the header line (vmcnt) with half the row's loads not yet issued
    if (FWD) __builtin_amdgcn_sched_barrier(0);
}

// How update_rows_kernel's checksum bytes reach the frames:
//   SF_INLINE   the row's lanes 0-3 store the 2+2 bytes as soon as they are known, write-through
//               (sc1) or, in the short-frame shape, past the caches (sc0 sc1 nt): one 64-byte
//               write request per packet inside the read stream;
//   SF_DEFER    per wave, from its four descriptor lengths (SGPRs): a wave whose frames average
//               at least kDeferMeanBytes writes 8-byte patch records instead, and
//               apply_bytes_kernel writes them after the read pass with non-temporal stores (the
//               writes then reach HBM in a write-only pass instead of interleaving with, or being
//               evicted from the memory-side cache into, the read stream); other waves as SF_INLINE;
//   SF_RECORDS  patch records only, frames untouched (nfcs_update_host: only the records cross
//               PCIe back).
// Round 4 measured, under rotating batches, forms storing each frame's first 64 bytes whole (from
// the read pass, or from 64-byte records through a write pass) and write passes of write-back /
// write-through stores: all slower than SF_DEFER's masked `nt` stores (their code is
// in git 2288ac5, tools/r04/fresh_exp.hip variants 4-8, 11-13, 30-34).
enum : int { SF_INLINE = 0, SF_DEFER = 1, SF_RECORDS = 2 };
// The fused forward's deferred record (large bursts, SF_DEFER; the write pass apply_fwd_kernel is
// its only reader), 8 bytes for a forwarded frame with a common header, all offsets below 64:
//   x = ip_off | ttl' << 8 | proto << 16 | l4_off << 24, y = ip checksum bytes | l4 checksum bytes << 16
// ip_off 0xFE: forwarded without an IPv4 checksum field (EtherType IPv4, version nibble != 4:
// update_checksums() is a no-op), the TTL offset then in y's low byte; l4_off 0xFF: no L4 field;
// x = 0xFFFFFFFF: nothing for the write pass (not forwarded, or written by the read pass's cold path).
constexpr uint32_t kFwdNoIp = 0xFEu, kFwdNone = 0xFFu;
DEV uint2 fwd_record(uint32_t ipw, uint32_t l4w, uint32_t ttl_new, uint32_t proto, bool tagged) {
    const bool ip = (ipw & 0xFFFFu) != NFCS_PATCH_NONE, l4 = (l4w & 0xFFFFu) != NFCS_PATCH_NONE;
    const uint32_t ipo = ip ? (ipw & 0xFFu) : kFwdNoIp, l4o = l4 ? (l4w & 0xFFu) : kFwdNone;
    const uint32_t y = (ip ? (ipw >> 16) : (tagged ? 26u : 22u)) | (l4w & 0xFFFF0000u);
    return make_uint2(ipo | ((ttl_new & 0xFFu) << 8) | ((proto & 0xFFu) << 16) | (l4o << 24), y);
}

// SF_DEFER's decision for the P packets pw .. pw+P-1 (lengths 0 past n), shared by the read pass
// and apply_bytes_kernel so both pick the same waves.
DEV bool defer_group(uint32_t lensum, uint32_t P) { return lensum >= P * (uint32_t)kDeferMeanBytes; }
DEV uint32_t defer_len(uint32_t len) { return len < 0xFFFFu ? len : 0xFFFFu; }

// Frame chunk rl (rl < R) of the row's packet from its line-aligned slots 0 and 1: the header
// view the plan, the forward's rewrite and its segment stores work on (lane rl + mis of the row).
template <int K, int R>
DEV uint4 hdr_view(const RowStage<K>& S, uint32_t rowbase4, uint32_t rl) {
    const uint32_t a = rl + S.mis;
    const int sl = (int)(rowbase4 + (a & (R - 1)) * 4u);
    const uint4 v0 = S.v[0], v1 = S.v[1];
    const uint4 r0 = make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v0.x),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v0.y),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v0.z),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v0.w));
    const uint4 r1 = make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v1.x),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v1.y),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v1.z),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v1.w));
    return a < (uint32_t)R ? r0 : r1;
}

// (Round 4's measurement-only knobs — uncommon-header rows deferred to a later pass, fewer
// continuation slots — were measured, not adopted, and dropped from the product; tools/r04/fresh_exp.hip
// builds against the round-4 sources, git 00f5686.)
template <int K, int R = 16, bool FWD = false, bool NT = false, bool DFR = false, bool LA = false>
DEV void row_process(const RowStage<K>& S, uint32_t rl, uint32_t rowbase4, uint8_t* status,
                     nfcs_patch* rec, bool frame_stores, uint32_t table_n = 0,
                     const uint32_t* wmac = nullptr, const nfcs_nexthop* table = nullptr) {
    const uint32_t len = S.len;
    uint8_t* frame = S.frame;
    const uint4* src = (const uint4*)frame;
    const bool live = S.valid && !S.bad;
    static_assert(K >= 2, "the header view reads slots 0 and 1");
    // frame chunk rl in lane rl: slot 0 itself when every row of the wave starts on a line
    uint4 h0 = S.v[0];
    if (LA && __builtin_amdgcn_ballot_w64(S.mis != 0) != 0) h0 = hdr_view<K, R>(S, rowbase4, rl);
    // Fused L3 forward (switch.hpp:247-294): the decision, then the TTL decrement and MAC
    // rewrite applied to the header registers, so the checksums below see the new header.
    bool fwd = false, tagged = false;
    uint32_t fst = NFCS_ST_NONE, ttl = 0, proto = 0;
    if (FWD) {
        const RowHdr<R> h{h0, rowbase4};
        const uint32_t e12 = h.be16(12);
        tagged = e12 == 0x8100u;  // ethernet() l2 = 18 (packet.hpp:410)
        const uint32_t l3t = len < 14 ? 0u : (tagged ? (len >= 18 ? h.be16(16) : e12) : e12);
        const bool v4 = l3t == 0x0800u && (tagged ? 38u : 34u) <= len;  // ipv4() present
        ttl = tagged ? h.b(26) : h.b(22);
        if (DFR) proto = tagged ? h.b(27) : h.b(23);  // the byte beside the TTL (the write pass's TTL short)
        fst = !v4 ? (uint32_t)NFCS_ST_NOT_IPV4
                  : (ttl <= 1 ? (uint32_t)NFCS_ST_TTL_EXPIRED
                              : (S.nh >= table_n ? (uint32_t)NFCS_ST_NO_ROUTE : 0u));
        fwd = live && fst == 0;
        if (fwd && rl == 0 && (!DFR || frame_stores)) {  // dst_mac, src_mac (286-289): the row's pick of the wave's MACs
            constexpr uint32_t PW = 64 / R;
            const uint32_t row = rowbase4 / (4u * R);
            uint32_t m0 = 0, m1 = 0, m2 = 0;
#pragma unroll
            for (uint32_t i = 0; i < PW; ++i) {
                m0 = (row == i) ? wmac[3 * i] : m0;
                m1 = (row == i) ? wmac[3 * i + 1] : m1;
                m2 = (row == i) ? wmac[3 * i + 2] : m2;
            }
            h0.x = m0;
            h0.y = m1;
            h0.z = m2;
        }
        if (fwd && rl == 1) {  // ttl-- (279): byte 22 (dword 1) or 26 (dword 2), never borrows
            if (tagged) h0.z -= 1u << 16;
            else h0.y -= 1u << 16;
        }
    }
    RPlan P = fast_plan<R>(h0, rowbase4, len);
    const bool act = live && (!FWD || fwd);  // rows whose checksums are updated
    // uncommon headers (IP options, IHL < 5, IHL past the frame) take the cold path below,
    // after the chunk registers are dead, so it adds nothing to the kernel's register peak
    const bool slow = act && (P.st >> 8) != 0;
    if (!act || slow)
        P = rplan_none(S.bad ? (uint32_t)NFCS_ST_BAD_DESC
                             : (FWD && live && !fwd) ? fst : (uint32_t)NFCS_ST_NONE);
    const uint32_t st = P.st | ((FWD && fwd) ? (uint32_t)NFCS_ST_FLAG_FWD : 0u);
    const uint32_t ipw = (P.flags & F_IP) ? P.ipw : NFCS_PATCH_NONE;
    uint32_t l4w = NFCS_PATCH_NONE;
    // Region sums without per-slot boundary branches (rows without an L4 region add nothing):
    // chunks below nre are added whole (the region starts below byte 80, in the header view h0,
    // where dwords under lo4 are masked); the last chunk's bytes past re and the odd trailing byte
    // are corrected once per row by the lane that holds it. The header view stands for slot 0:
    // it holds frame chunks 0..R-1 in lanes 0..R-1, so slot 0's own lanes (frame chunks below
    // R - mis) are never summed and slot 1 adds only its chunks from R on; lane rl of slot k >= 1
    // holds frame chunk R*k + rl - mis (row_stage). Frames longer than one batch leave
    // their end to the masked continuation below. rlv is opaque so the per-slot offsets are
    // recomputed rather than hoisted into ~35 long-lived VGPRs.
    const uint32_t re = (P.flags & F_L4) ? P.re : 0u, lo4 = P.rs & ~3u;
    const uint32_t tailfix = P.flags & F_TAIL;
    uint32_t rlv = rl;
    asm volatile("" : "+v"(rlv));
    uint32_t acc = 0;
    const uint32_t nre = (re + 15u) >> 4;
    {
        // la: the last chunk's place in the slots (lane la % R of slot la / R; slot 0 = h0)
        const uint32_t last = nre - 1u, la = (!LA || last < (uint32_t)R) ? last : last + S.mis;
        const uint32_t own = (re != 0) && (la < (uint32_t)R * K) && ((la & (R - 1)) == rl);
        uint4 lc = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint4 v = k == 0 ? h0 : S.v[k];
            const uint32_t c = k == 0 ? rlv : rlv + (uint32_t)R * k - S.mis;
            const uint32_t m = (c < nre && (!LA || k != 1 || c >= (uint32_t)R)) ? 0xFFFFFFFFu : 0u;
            if (k == 0) {
                const uint32_t o = 16u * c;
                acc = wsum(v.x & m & ((o >= lo4) ? 0xFFFFFFFFu : 0u), acc);
                acc = wsum(v.y & m & ((o + 4u >= lo4) ? 0xFFFFFFFFu : 0u), acc);
                acc = wsum(v.z & m & ((o + 8u >= lo4) ? 0xFFFFFFFFu : 0u), acc);
                acc = wsum(v.w & m & ((o + 12u >= lo4) ? 0xFFFFFFFFu : 0u), acc);
            } else {
                acc = wsum(v.w & m, wsum(v.z & m, wsum(v.y & m, wsum(v.x & m, acc))));
            }
            const bool sel = (la >> (R == 16 ? 4 : 3)) == (uint32_t)k;
            lc.x = sel ? v.x : lc.x;
            lc.y = sel ? v.y : lc.y;
            lc.z = sel ? v.z : lc.z;
            lc.w = sel ? v.w : lc.w;
        }
        if (own) {
            // the chunk's bytes at or past re come off again: dword j keeps its low
            // clamp(8 (re - o) - 32 j, 0, 32) bits (one 64-bit shift each). Bytes under lo4 of a one-chunk
            // region were never added, and none of them lies at or past re (re >= rs >= lo4).
            const uint32_t o = 16u * last, kb8 = 8u * (re - o);
            uint32_t ex = 0;
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const int s = min(max((int)kb8 - 32 * (int)j, 0), 32);
                ex = wsum(comp(lc, j) & (uint32_t)(~0ull << s), ex);
            }
            acc -= ex;
            const uint32_t t = re - 1u - o, q = t >> 2;
            const uint32_t dt = q == 0 ? lc.x : (q == 1 ? lc.y : (q == 2 ? lc.z : lc.w));
            if (tailfix) acc += 255u * ((dt >> (8 * (t & 3u))) & 0xFFu);
        }
    }
    // continuation batches for frames longer than R*K chunks (jumbo)
    const uint32_t cmax = wave_max_rows<R>(LA ? nre + S.mis : nre);
    for (uint32_t cb = (uint32_t)R * K; cb < cmax; cb += (uint32_t)R * K) {
        uint4 w[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = cb + rlv + (uint32_t)R * k - S.mis;
            w[k] = ld16<1>((c < nre) ? src + c : g_zero_line);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc_slot(acc, w[k], cb + rlv + (uint32_t)R * k - S.mis, lo4, re, tailfix);
    }
    const uint32_t z = row_sum<R>(acc) + P.corr;
    if (P.flags & F_L4) {
        uint32_t c = (~fold32(z)) & 0xFFFFu;  // LE-domain complement = bswap of ref value
        if ((P.flags & F_UDP) && c == 0) c = 0xFFFFu;  // 867-871
        l4w = P.fs | (c << 16);
    }
    // The (at most 4) checksum bytes from lanes 0..3 of the row, write-through (sc1: the L2
    // keeps no dirty copy of the header line; session 3, C1 +2.5% / C3 +5% over write-back
    // stores; byte stores measured fastest against chunk, dword, whole-line and re-load-then-
    // store forms) or, with NT (the short-frame shape), past the caches (`sc0 sc1 nt`: round 2
    // session 3, C3 +2%, uniform 1024-byte frames +2.7%; in the long shape it cost 64K-packet
    // bursts of 9000-byte frames 3%, in 8-lane rows IMIX ±1%), then the status byte / patch
    // record from lane 0.
    auto emit = [&](bool on, uint32_t st_, uint32_t ipw_, uint32_t l4w_, bool stores, bool recw = true) {
        if (stores && on && rl < 4) {
            const uint32_t w = (rl & 2u) ? l4w_ : ipw_;
            const uint32_t pos = (w & 0xFFFFu) + (rl & 1u);
            if ((w & 0xFFFFu) != NFCS_PATCH_NONE) {
                if (NT) st8_nt(frame + pos, w >> (16 + 8 * (rl & 1u)));
                else st8<true>(frame + pos, w >> (16 + 8 * (rl & 1u)));
            }
        }
        if (on && rl == 0) {
            if (status) status[S.p] = (uint8_t)st_;
            if (rec && recw) {
                uint2 r;
                r.x = (ipw_ & 0xFFFFu) | (l4w_ << 16);
                r.y = (ipw_ >> 16) | (l4w_ & 0xFFFF0000u);
                ((uint2*)rec)[S.p] = r;
            }
        }
    };
    if (FWD) {
        // The fused forward's segment store: one write-through segment per forwarded packet.
        // Lanes 0..c store chunks 0..c of the header (c = the last chunk holding a byte to
        // write) from the header registers with the checksum bytes and the forward's rewrite
        // patched in; unchanged bytes are rewritten with the values just read from them (a frame
        // never shares a 16-byte chunk with another frame). +1.5% over a 16-byte store + byte
        // stores (session 3).
        if (S.valid && !slow && fwd) {
            // IPv4 field first, then L4, as the reference writes them
            const uint4 v = put_field(put_field(h0, ipw, rl), l4w, rl);
            uint32_t last = 1u;
            if ((ipw & 0xFFFFu) != NFCS_PATCH_NONE) last = max(last, ((ipw & 0xFFFFu) + 1u) >> 4);
            if ((l4w & 0xFFFFu) != NFCS_PATCH_NONE) last = max(last, ((l4w & 0xFFFFu) + 1u) >> 4);
            // the short-mix shape (8-lane rows, line-aligned windows) stores past the caches (`sc0 sc1
            // nt`, as the update's short shape does), the others write-through (`sc1`): round 5, calls
            // rotating over fresh C3-mix batches, 0.690-0.710 against 0.719-0.735 ms per call
            // (profiles/r05_fwd_var.jsonl, r05_fwd_store_ab.jsonl; the replayed measurements of rounds
            // 2-3 had seen no gain); 1M x 64-byte frames (the tiny shape) 1% slower with them
            if ((!DFR || frame_stores) && rl <= last && 16u * rl < len) {
                if (R == 8 && LA) st16_nt((uint4*)frame + rl, v);
                else st16<true>((uint4*)frame + rl, v);
            }
        }
        // a deferred wave (large bursts, SF_DEFER) leaves the frame alone here: its forward record
        // (fwd_record) goes to apply_fwd_kernel, which writes the rewritten bytes without reading
        // the frame again
        emit(S.valid && !slow, st, ipw, l4w, false, !DFR);
        if (DFR && rec && S.valid && !slow && rl == 0)
            ((uint2*)rec)[S.p] = (fwd && live) ? fwd_record(ipw, l4w, ttl - 1u, proto, tagged) : make_uint2(0xFFFFFFFFu, 0u);
    } else {
        emit(S.valid && !slow, st, ipw, l4w, frame_stores);
    }
    if (__builtin_amdgcn_ballot_w64(slow) != 0) {  // cold path, wave-uniform branch
        // Uncommon headers, handled last so that only the frame address and length are live
        // across the calls: the row's lane 0 parses from memory (IHL < 5 overlaps run the
        // exact sequential emulation, which writes its own bytes) and the region is re-summed
        // from memory.
        if (FWD && slow && fwd) {
            // segment stores skip uncommon headers: their forward rewrite goes out here, from
            // the next-hop MACs (SGPRs) and the TTL byte in memory (the header registers are
            // dead by now, which keeps the fast path free of spills)
            if (rl == 0) {
                constexpr uint32_t PW = 64 / R;
                const uint32_t row = rowbase4 / (4u * R);
                uint32_t m[3] = {0, 0, 0};
                if (DFR && !frame_stores) {  // a deferring wave loaded no MACs: this row's, from the table
#pragma unroll
                    for (uint32_t j = 0; j < 3; ++j) m[j] = ((const uint32_t*)(table + S.nh))[j];
                } else {
#pragma unroll
                    for (uint32_t i = 0; i < PW; ++i) {
#pragma unroll
                        for (uint32_t j = 0; j < 3; ++j) m[j] = (row == i) ? wmac[3 * i + j] : m[j];
                    }
                }
#pragma unroll
                for (uint32_t j = 0; j < 3; ++j)
                    __hip_atomic_store((uint32_t*)frame + j, m[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (rl == 1) {
                const uint32_t o = tagged ? 26u : 22u;
                st8<true>(frame + o, frame[o] - 1u);
            }
        }
        if (FWD) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // see the header stores
        RPlan Q = rplan_none(0);
        SeqOut o = {0, 0, 0, 0, 0};
        if (slow && rl == 0) {
            Q = slow_plan(frame, len);
            if (Q.flags & F_SEQ) o = seq_update(frame, len);
        }
        Q.st = row_bcast<0, R>(Q.st);
        Q.flags = row_bcast<0, R>(Q.flags);
        Q.ipw = row_bcast<0, R>(Q.ipw);
        Q.rs = row_bcast<0, R>(Q.rs);
        Q.re = row_bcast<0, R>(Q.re);
        Q.fs = row_bcast<0, R>(Q.fs);
        Q.corr = row_bcast<0, R>(Q.corr);
        const uint32_t ost = row_bcast<0, R>(o.st);
        const uint32_t oip = row_bcast<0, R>((o.ip_off & 0xFFFFu) | (o.ip_val << 16));
        const uint32_t ol4 = row_bcast<0, R>((o.l4_off & 0xFFFFu) | (o.l4_val << 16));
        const bool seq = slow && (Q.flags & F_SEQ);
        const uint32_t re2 = (slow && !seq && (Q.flags & F_L4)) ? Q.re : 0u;
        const uint32_t lo42 = Q.rs & ~3u, tf2 = Q.flags & F_TAIL;
        uint32_t acc2 = 0;
        for (uint32_t c = rl; c < ((re2 + 15u) >> 4); c += R) acc_slot(acc2, src[c], c, lo42, re2, tf2);
        const uint32_t z2 = row_sum<R>(acc2) + Q.corr;
        uint32_t st2 = Q.st, ipw2 = (Q.flags & F_IP) ? Q.ipw : NFCS_PATCH_NONE, l4w2 = NFCS_PATCH_NONE;
        if (Q.flags & F_L4) {
            uint32_t c = (~fold32(z2)) & 0xFFFFu;
            if ((Q.flags & F_UDP) && c == 0) c = 0xFFFFu;
            l4w2 = Q.fs | (c << 16);
        }
        if (seq) {
            st2 = ost | NFCS_ST_FLAG_OVERLAP;
            ipw2 = oip;
            l4w2 = ol4;
        }
        if (FWD) st2 |= NFCS_ST_FLAG_FWD;
        // the forward always stores (its header rewrite went out above)
        emit(slow, st2, ipw2, l4w2, !seq && (FWD || frame_stores), !(FWD && DFR));
        // the forward stored everything of an uncommon header here: nothing left for the write pass
        if (FWD && DFR && rec && slow && rl == 0) ((uint2*)rec)[S.p] = make_uint2(0xFFFFFFFFu, 0u);
    }
}

// One wave = 64/R packet rows; one workgroup per BS/R packets, as many workgroups as the batch
// needs (a grid that strides over resident workgroups measured 10-15% slower).
// XCD-aware block order (session 3): workgroups are dealt to the 8 XCDs round-robin; remapped,
// the workgroups one XCD runs take one contiguous eighth of the batch, so each XCD streams its
// own region of HBM and the descriptor lines its workgroups share stay in its L2 (a bijection on
// [0, gridDim.x); the tail beyond a multiple of 8 keeps its order). C1 +1.3%, C3 +0.5%.
// Arguments in the order a wave needs them: the first eight (14 dwords: what every wave reads
// before its frame loads, plus the footprint slot) are preloaded into SGPRs at dispatch
// (-amdgpu-kernarg-preload-count=8, netflow_amd/__init__.py), so a wave's first memory access is
// its descriptor load, with no kernel-argument round trip ahead of it; `nblocks` (= gridDim.x) is
// passed explicitly for the same reason (the grid size is a hidden argument, loaded from memory).
// The rows of one wave from their frame loads on: line-aligned windows of KL slots (LA) or
// frame-relative ones of K slots.
template <int K, int R, int BS, bool FWD, int SF, bool LA, int PW>
DEV void rows_body(const DescW<PW>& D, uint64_t pw, uint32_t n, uint8_t* arena, uint64_t arena_bytes, uint32_t base16,
                   uint32_t rl, uint32_t row, uint32_t rowbase4, bool defer, const uint32_t (&q)[PW],
                   uint8_t* status, nfcs_patch* patch, nfcs_patch* ws, const nfcs_nexthop* table, uint32_t table_n) {
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    const bool frame_stores = SF == SF_INLINE || (SF == SF_DEFER && !defer);
    nfcs_patch* rec = patch ? patch : (defer ? ws : nullptr);
    RowStage<K> S;
    // buffer loads in the plain update's short shape (16-lane rows, frame-relative windows), where
    // most lanes of a wave's later slots are past their frames: C3 0.689-0.692 -> 0.664-0.669 ms per
    // call; the long shape (+0.5%), the C4 shard (+0.8%), the 8-lane tiny shape (+1.2%) and the
    // fused forward's short-mix shape (+4-10%) measured slower with them and keep global loads
    // (profiles/r04_s2_wave_buf_ab.jsonl). (The long shape's frame-relative body is never launched:
    // it runs line-aligned windows, LAM 1.)
    constexpr bool BUF = !FWD && R == 16 && !LA;
    row_stage<K, R, FWD, LA, BUF>(S, arena, arena_bytes, pick_desc<PW>(D, row), pw + row, n, base16, rl,
                                  wave_buf<PW>(D, pw, n, arena, base16), 0u);
    uint32_t wmac[3 * PW];  // the wave's next-hop MACs: scalar loads, selected per row at use
    if (FWD) {
#pragma unroll
        for (uint32_t i = 0; i < PW; ++i) S.nh |= (row == i) ? q[i] : 0u;
        // a deferring wave's MACs are written by apply_fwd_kernel (the checksums do not cover
        // them): only waves that store inline load them
        if (!(SF == SF_DEFER && defer)) {
#pragma unroll
            for (uint32_t i = 0; i < PW; ++i) {
                const cu32* m = (q[i] < table_n) ? (const cu32*)(table + q[i]) : (const cu32*)g_zero_line;
                wmac[3 * i] = m[0];
                wmac[3 * i + 1] = m[1];
                wmac[3 * i + 2] = m[2];
            }
        }
    }
    // inline checksum stores past the caches in the short-frame shape (16-lane rows, frame-relative
    // windows), write-through elsewhere (see row_process)
    row_process<K, R, FWD, !FWD && R == 16 && !LA, FWD && SF == SF_DEFER, LA>(S, rl, rowbase4, status, rec,
                                                                                 frame_stores, table_n, wmac, table);
}

// One wave of update_rows_kernel: its PW packets from the descriptor load on.
template <int K, int R, int BS, bool FWD, int SF, int LAM, int KL>
DEV void rows_wave(const nfcs_desc* __restrict__ desc, uint32_t n, uint8_t* __restrict__ arena, uint64_t arena_bytes,
                   uint32_t base16, const uint32_t* __restrict__ nh, uint64_t* __restrict__ obs,
                   uint8_t* __restrict__ status, nfcs_patch* __restrict__ patch, nfcs_patch* __restrict__ ws,
                   const nfcs_nexthop* __restrict__ table, uint32_t table_n, uint64_t obs_tag, uint32_t lane,
                   uint32_t rl, uint32_t row, uint32_t rowbase4, uint64_t pw) {
    constexpr uint32_t PW = 64 / R;  // packets per wave
    if (blockIdx.x == 0 && threadIdx.x < 64 && obs) sample_footprint(desc, obs_tag, lane, obs);
    // the wave's PW descriptors: one scalar load (s_load_dwordx8 for PW = 4)
    const DescW<PW> D = load_descw<PW>(desc, pw, n);
    // the store form of each aligned group of 4 packets, from their own frame lengths (scalar
    // arithmetic on the descriptors): the whole wave with 16-lane rows, each half of the wave with
    // 8-lane rows; apply_bytes_kernel recomputes the same groups
    bool defer = false;
    if (SF == SF_DEFER) {
        static_assert(PW == 4 || PW == 8, "deferral groups of 4 packets");
        uint32_t s0 = 0, s1 = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) s0 += defer_len(D.w[2 * i + 1]);
#pragma unroll
        for (uint32_t i = 4; i < PW; ++i) s1 += defer_len(D.w[2 * i + 1]);
        defer = (PW == 8 && row >= 4) ? defer_group(s1, 4) : defer_group(s0, 4);
    }
    // Fused L3 forward: the wave's PW next-hop indexes and their table rows are wave-uniform.
    // Read through the constant address space they are scalar loads on lgkmcnt: the indexes are
    // issued with the descriptors, and everything that depends on them (the row's pick, the MAC
    // loads) comes after the frame loads are issued (row_stage's sched_barrier), so no frame load
    // waits for a next-hop round trip (as generic loads the compiler made each index a vector load
    // drained by vmcnt(0) ahead of the frame loads: four serial memory round trips per wave).
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    uint32_t q[PW];
    if (FWD) {
        const cu32* nhp = (const cu32*)nh + pw;
        if (pw + PW <= n) {
#pragma unroll
            for (uint32_t i = 0; i < PW; ++i) q[i] = nhp[i];
        } else {
#pragma unroll
            for (uint32_t i = 0; i < PW; ++i) q[i] = (pw + i < n) ? nhp[i] : NFCS_NH_NONE;
        }
    }
    bool la = LAM == 1;
    if (LAM == 2) {  // any row of the wave starting mid-line (its frame address, as row_stage computes it)
        const nfcs_desc d = pick_desc<PW>(D, row);
        const uint64_t a = (uint64_t)(uintptr_t)arena + ((uint64_t)d.off16 - base16) * 16u;
        la = __builtin_amdgcn_ballot_w64(pw + row < n && d.len != 0 && ((a >> 4) & 7u) != 0) != 0;
    }
    if (la)
        rows_body<KL, R, BS, FWD, SF, true, PW>(D, pw, n, arena, arena_bytes, base16, rl, row, rowbase4, defer, q,
                                                status, patch, ws, table, table_n);
    else
        rows_body<K, R, BS, FWD, SF, false, PW>(D, pw, n, arena, arena_bytes, base16, rl, row, rowbase4, defer, q,
                                                status, patch, ws, table, table_n);
}

// LAM: 0 frame-relative windows of K slots; 1 line-aligned windows of KL slots; 2 per wave, line-
// aligned (KL slots) when a row of the wave starts mid-line, else frame-relative (K slots), so
// line-aligned batches run the frame-relative code unchanged.
template <int K, int R, int OCC, int BS, bool FWD, int SF, int LAM = 0, int KL = K>
__global__ __launch_bounds__(BS, OCC) void update_rows_kernel(const nfcs_desc* __restrict__ desc, uint32_t n,
                                                              uint32_t nblocks, uint8_t* __restrict__ arena,
                                                              uint64_t arena_bytes, uint32_t base16,
                                                              const uint32_t* __restrict__ nh,
                                                              uint64_t* __restrict__ obs,
                                                              uint8_t* __restrict__ status,
                                                              nfcs_patch* __restrict__ patch,
                                                              nfcs_patch* __restrict__ ws,
                                                              const nfcs_nexthop* __restrict__ table,
                                                              uint32_t table_n, uint64_t obs_tag, DoneReq done) {
    constexpr uint32_t PW = 64 / R;  // packets per wave
    const uint32_t lane = threadIdx.x & 63u, rl = lane & (R - 1), row = lane / R;
    const uint32_t rowbase4 = (lane & ~(uint32_t)(R - 1)) * 4u;
    const uint64_t pw = (uint64_t)xcd_block_n(nblocks) * (BS / R) + rfl(threadIdx.x >> 6) * PW;
    // with a DoneReq (a kernel argument: uniform) waves without packets stay for signal_done's barrier
    if (pw >= n && !done.flag) return;
    if (pw < n)
        rows_wave<K, R, BS, FWD, SF, LAM, KL>(desc, n, arena, arena_bytes, base16, nh, obs, status, patch, ws, table,
                                              table_n, obs_tag, lane, rl, row, rowbase4, pw);
    if (done.flag) signal_done(done, nblocks);
}

// SF_DEFER's write pass: the patch records of the waves that deferred, written into the frames
// with ONE store request per packet, non-temporal at system scope (`sc0 sc1 nt`): the writes go to
// HBM during this write-only pass instead of lingering dirty in the memory-side cache and being
// evicted into the next read stream (4M x 1500 B shard: read pass + this pass 0.715-0.718 of 8 TB/s
// against 0.658 for the fused kernel with write-back stores; tools/wr_probe.hip).
// One thread per packet: lane l of a wave loads descriptor p0 + l (one coalesced 512-byte load)
// and, from the lengths of its aligned quad of lanes, recomputes the read pass's decision for that
// group of 4 packets, and loads its record (with the descriptor when EARLY). The stores go out in 4
// rounds of 16 packets: in round k lane l writes byte l % 4 of (ip[0], ip[1], l4[0], l4[1]) of packet 16k + l/4
// (its record and frame offset by ds_bpermute), so the packet's 4 bytes leave in one store
// instruction as one write request with a byte mask. An IPv4 byte that the L4 field overlaps
// (IHL < 5) is left to the L4 lane: the reference writes the L4 field last.
__global__ __launch_bounds__(kBlock) void apply_bytes_kernel(uint8_t* __restrict__ arena,
                                                             const nfcs_desc* __restrict__ desc,
                                                             uint32_t n, uint32_t base16,
                                                             const nfcs_patch* __restrict__ rec) {
    const uint32_t lane = threadIdx.x & 63u;
    // the read pass's XCD-aware order: each XCD writes the eighth of the sub-batch its own read pass
    // covered, whose records and descriptors its L2 still holds (round 5, calls rotating over fresh
    // batches: C1 -0.5%, the C4 shard -0.4% per call; profiles/r05_block_order_ab.jsonl)
    const uint64_t i = (uint64_t)xcd_block() * kBlock + threadIdx.x;
    const nfcs_desc d = i < n ? desc[i] : nfcs_desc{0u, 0u};
    // The record is loaded with the descriptor, before the decision — one memory round trip ahead
    // of the stores instead of two (C1 +1.5%, the 4M shard +0.5%; records of waves that stored
    // inline are stale and ignored). Only the long shape runs this pass (launch_update_one).
    uint2 r0 = make_uint2(0u, 0u);
    if (i < n) r0 = ((const uint2*)rec)[i];
    uint32_t s = defer_len(d.len);
    s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0xB1, 0xF, 0xF, true);  // quad_perm 1,0,3,2
    s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x4E, 0xF, 0xF, true);  // quad_perm 2,3,0,1
    const bool dfr = i < n && defer_group(s, 4);
    const uint64_t mask = __builtin_amdgcn_ballot_w64(dfr);
    if (!mask) return;
    const uint2 r = dfr ? r0 : make_uint2(NFCS_PATCH_NONE | (NFCS_PATCH_NONE << 16), 0u);
    const uint32_t j = lane & 3u;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        if (((mask >> (16u * k)) & 0xFFFFu) == 0) continue;  // wave-uniform
        const int q4 = (int)((16u * k + (lane >> 2)) * 4u);  // source lane, in bytes
        const uint32_t rx = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)r.x);
        const uint32_t ry = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)r.y);
        const uint32_t o16 = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)d.off16);
        const uint32_t ipo = rx & 0xFFFFu, l4o = rx >> 16;
        const uint32_t off = j < 2 ? ipo : l4o;
        const uint32_t a = off + (j & 1u);
        const bool overlap = j < 2 && l4o != NFCS_PATCH_NONE && (a == l4o || a == l4o + 1u);
        if (off != NFCS_PATCH_NONE && !overlap) {
            const uint32_t b = (j < 2 ? (ry >> (8 * j)) : (ry >> (16 + 8 * (j - 2)))) & 0xFFu;
            uint8_t* p = arena + ((uint64_t)o16 - base16) * 16u + a;
            asm volatile("global_store_byte %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(b) : "memory");
        }
    }
}

// A 2-byte store past the caches (`sc0 sc1 nt`), as st8_nt.
DEV void st16b_nt(uint8_t* p, uint32_t v) {
    asm volatile("global_store_short %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}

// The fused L3 forward's write pass (large bursts, SF_DEFER), from the records alone — no frame
// byte is read again. One thread per packet loads its descriptor, record and next hop (coalesced)
// and, for a forwarded packet of a deferring group of 4 (the decision recomputed from the four
// lengths, as in apply_bytes_kernel), its next hop's MACs. Then 16 rounds of 4 packets: in round k
// the 16 lanes of row r write packet 4k + r (its values by ds_bpermute) as ONE instruction of 2-byte
// stores — lanes 0-5 the MACs (switch.hpp:286-289), lane 6 the TTL with the protocol byte beside it
// (279), lane 7 the IPv4 checksum, lane 8 an even-offset L4 checksum — so each packet's bytes leave
// as one write request with a byte mask, past the caches (`sc0 sc1 nt`); an L4 field at an odd
// offset (TCP: l4 + 15, the 19-byte TcpHeader) goes out as two byte stores after it.
__global__ __launch_bounds__(kBlock) void apply_fwd_kernel(uint8_t* __restrict__ arena,
                                                           const nfcs_desc* __restrict__ desc, uint32_t n,
                                                           const uint32_t* __restrict__ nh,
                                                           const nfcs_nexthop* __restrict__ table,
                                                           const nfcs_patch* __restrict__ rec) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t i = (uint64_t)xcd_block() * kBlock + threadIdx.x;  // as apply_bytes_kernel
    const bool in = i < n;
    const nfcs_desc d = in ? desc[i] : nfcs_desc{0u, 0u};
    const uint2 r0 = in ? ((const uint2*)rec)[i] : make_uint2(0xFFFFFFFFu, 0u);
    const uint32_t h = in ? nh[i] : 0u;
    uint32_t s = defer_len(d.len);
    s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0xB1, 0xF, 0xF, true);  // quad_perm 1,0,3,2
    s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x4E, 0xF, 0xF, true);  // quad_perm 2,3,0,1
    // records of groups that stored inline are stale: ignored
    const bool go = in && defer_group(s, 4) && (r0.x & 0xFFu) != kFwdNone;
    const uint64_t mask = __builtin_amdgcn_ballot_w64(go);
    if (!mask) return;
    uint32_t m0 = 0, m1 = 0, m2 = 0;
    if (go) {  // a forwarded packet's next hop is in the table (the read pass checked it)
        const uint32_t* m = (const uint32_t*)(table + h);
        m0 = m[0];
        m1 = m[1];
        m2 = m[2];
    }
    const uint32_t rx = go ? r0.x : 0xFFFFFFFFu, ry = r0.y;
    const uint32_t j = lane & 15u;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        if (((mask >> (4u * k)) & 0xFu) == 0) continue;  // wave-uniform
        const int q4 = (int)((4u * k + (lane >> 4)) * 4u);  // source lane, in bytes
        const uint32_t x = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)rx);
        const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)ry);
        const uint32_t o16 = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)d.off16);
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)m0);
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)m1);
        const uint32_t a2 = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)m2);
        const uint32_t ipo = x & 0xFFu, l4o = x >> 24;
        if (ipo == kFwdNone) continue;
        uint8_t* f = arena + (uint64_t)o16 * 16u;
        const uint32_t mw = j < 2 ? a0 : (j < 4 ? a1 : a2);
        uint32_t off = 0xFFFFu, v = 0;
        if (j < 6) {
            off = 2u * j;
            v = mw >> (16u * (j & 1u));
        } else if (j == 6) {  // TTL and protocol (l2 + 8, l2 + 9)
            off = ipo == kFwdNoIp ? (y & 0xFFu) : ipo - 2u;
            v = ((x >> 8) & 0xFFu) | (((x >> 16) & 0xFFu) << 8);
        } else if (j == 7 && ipo != kFwdNoIp) {
            off = ipo;
            v = y;
        } else if (j == 8 && l4o != kFwdNone && !(l4o & 1u)) {
            off = l4o;
            v = y >> 16;
        }
        if (off != 0xFFFFu) st16b_nt(f + off, v & 0xFFFFu);
        if ((j == 8 || j == 9) && l4o != kFwdNone && (l4o & 1u))
            st8_nt(f + l4o + (j - 8u), (y >> (16u + 8u * (j - 8u))) & 0xFFu);
    }
}

// Workgroup shapes of the checksum read pass, chosen per call from the mean arena footprint per
// packet (speed only: results and store forms never depend on it):
//   kShapeTiny   (< kTinyMeanBytes)  8-lane rows of 6 slots (768 B per row pass), 8 packets per
//                one-wave workgroup: frames this short are packet-rate bound, and twice the packets
//                per wave doubles it (64-256 B frames 1.8-1.9x, IMIX 1.47x, 768 B 1.2x);
//   kShapeShort  (< kSmallMeanBytes) 16-lane rows in 256-thread workgroups at 7 waves/SIMD: mixes of
//                short and long frames (C3), where 8-lane rows would need a second row pass for
//                most waves (C3 -7.5%);
//   kShapeLong   16-lane rows in 256-thread workgroups held at 5 waves/SIMD.
enum : int { kShapeTiny = 0, kShapeShort = 1, kShapeLong = 2 };

// One launch of update_rows_kernel (the grid size passed as `nblocks` too).
template <int K, int R, int OCC, int BS, bool FWD, int SF, int LAM = 0, int KL = K>
static void launch_rows(uint32_t grid, unsigned lds, hipStream_t stream, uint8_t* arena, uint64_t arena_bytes,
                        const nfcs_desc* desc, uint32_t n, uint32_t base16, uint8_t* status, nfcs_patch* patch,
                        nfcs_patch* ws, const FwdArgs& fa) {
    hipLaunchKernelGGL((update_rows_kernel<K, R, OCC, BS, FWD, SF, LAM, KL>), dim3(grid), dim3(BS), lds, stream, desc, n, grid,
                       arena, arena_bytes, base16, fa.nh, fa.obs.slot, status, patch, ws, fa.table, fa.table_n,
                       fa.obs.tag, fa.done);
}

// One launch of the checksum path (its read pass and, for kUpdateAuto, its write pass) over n
// packets, in the shape chosen for the whole call.
static hipError_t launch_update_one(uint8_t* arena, uint64_t arena_bytes, const nfcs_desc* desc, uint32_t n,
                                    uint32_t base16, uint8_t* status, nfcs_patch* patch, nfcs_patch* ws,
                                    int form, int shape, hipStream_t stream, ObsReq obs, DoneReq done = {}) {
    const FwdArgs nofwd = {nullptr, nullptr, 0, obs, done};
    // a burst of at most kInlineMaxPackets packets: one kernel, every wave inline (the write pass's
    // launch would cost more than deferral saves on so few packets)
    if (form == kUpdateAuto && n <= kInlineMaxPackets) form = kUpdateInline;
    const uint32_t g8 = (n + 7u) / 8u, g4 = (n + 15u) / 16u;
#define NFCS_ROWS(OCC, BS, G, SF)                                                                  \
    launch_rows<6, 16, OCC, BS, false, SF, BS == kBlock ? 1 : 0, BS == kBlock ? 7 : 6>(                          \
        G, BS == kBlock ? kRowsLdsPad : 0u, stream, arena, arena_bytes, desc,                                 \
                                           n, base16, status, patch, ws, nofwd)
#define NFCS_ROWS8(SF) \
    launch_rows<6, 8, 8, 64, false, SF>(g8, 0u, stream, arena, arena_bytes, desc, n, base16, status, patch, ws, nofwd)
#define NFCS_SHORT(SF) \
    launch_rows<6, 16, 7, kBlock, false, SF, 0, 6>(g4, 0u, stream, arena, arena_bytes, desc, n, base16, status, patch, ws, nofwd)
#define NFCS_SHAPED(SF)                                                                            \
    do {                                                                                           \
        if (shape == kShapeTiny) NFCS_ROWS8(SF);                                                   \
        else if (shape == kShapeShort) NFCS_SHORT(SF);                                             \
        else NFCS_ROWS(1, kBlock, g4, SF);                                                         \
    } while (0)
    if (form == kUpdateRecords) {
        NFCS_ROWS(1, kBlock, g4, SF_RECORDS);
    } else if (form == kUpdateInline) {
        NFCS_SHAPED(SF_INLINE);
    } else if (shape != kShapeLong) {
        // short and tiny shapes: every wave stores inline and no write pass is launched. The few
        // groups of 4 that average >= kDeferMeanBytes in such batches gain less from deferral than
        // the write pass costs to find them among all the descriptors (round 3, same box: C3 +1.5-2.4%,
        // 1M x 64 B +5.5%, 4M mixes of 64/1500-byte frames with 25/50/75% long frames +2/+1.3/+3.7%;
        // profiles/r03_s3_ab_c3_inline.jsonl, r03_s3_ab_bimodal.jsonl)
        NFCS_SHAPED(SF_INLINE);
    } else {
        NFCS_ROWS(1, kBlock, g4, SF_DEFER);
        hipLaunchKernelGGL(apply_bytes_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream,
                           arena, desc, n, base16, patch ? patch : ws);
    }
#undef NFCS_SHAPED
#undef NFCS_SHORT
#undef NFCS_ROWS8
#undef NFCS_ROWS
    return hipGetLastError();
}

hipError_t launch_update(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes,
                         const nfcs_desc* desc, uint32_t n, uint32_t base16, uint8_t* status,
                         nfcs_patch* patch, nfcs_patch* ws, int form, hipStream_t stream,
                         uint64_t slot_bytes, ObsReq obs, DoneReq done) {
    (void)di;
    if (n == 0) return hipSuccess;
    if (form == kUpdateRecords && !patch) return hipErrorInvalidValue;
    if (done.flag && form == kUpdateAuto) return hipErrorInvalidValue;  // one kernel per call only
    if (form == kUpdateAuto && !patch && !ws) return hipErrorInvalidValue;
    // The short shape at 7 waves/SIMD: __launch_bounds__ 7 caps the kernel at 94 SGPRs (at the
    // compiler's 106 the SGPR file admits only 6 waves/SIMD: C3 +2%). Its workgroups were one wave
    // (round 3, a replayed batch: short-lived waves retire and relaunch with less granularity loss,
    // C3 +2-3%); in the steady state 256-thread workgroups, whose 4 waves on one CU share the
    // descriptor line of their 16 packets, measured 0.3-0.5% faster (round 5, C3 0.662-0.663
    // against 0.665 ms per call; profiles/r05_c3_rows_ab.jsonl). 256-thread workgroups are held at 5 waves/SIMD by kRowsLdsPad
    // bytes of (unused) LDS: at the 8 their 54 VGPRs allow, the read stream runs slower (round 1,
    // one replayed batch: C1 0.768 vs 0.777 at 6). Round 4, calls rotating over fresh batches with
    // 512K-packet sub-batches: 5 waves beat 6 by 1.2-1.5% on C1, 1.6% on the C4 shard, 0.3% on C2
    // (profiles/r04_s2_long_occupancy5_ab.jsonl).
    const uint64_t mean = shape_mean(arena_bytes, n, slot_bytes);
    const int shape = mean < kTinyMeanBytes ? kShapeTiny : (mean < kSmallMeanBytes ? kShapeShort : kShapeLong);
    // Long frames in a batch of more than kSubBatchAbovePackets: read pass and write pass alternate
    // per sub-batch of kSubBatchPackets, so the write pass finds its header lines still in the
    // 256 MB memory-side cache that the read pass just brought them into (the 4M
    // shard 0.683-0.714 -> 0.749-0.755). Sub-batches are multiples of 4 packets, so every wave's
    // deferral group is the same as in one launch; they run in order on the stream and share the
    // workspace.
    if (form == kUpdateAuto && shape == kShapeLong && n > kSubBatchAbovePackets) {
        for (uint32_t i = 0; i < n; i += kSubBatchPackets) {
            const hipError_t e = launch_update_one(arena, arena_bytes, desc + i, std::min(kSubBatchPackets, n - i),
                                                   base16, status ? status + i : nullptr,
                                                   patch ? patch + i : nullptr, ws, form, shape, stream,
                                                   i == 0 ? obs : ObsReq{});
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    return launch_update_one(arena, arena_bytes, desc, n, base16, status, patch, ws, form, shape, stream, obs, done);
}

hipError_t launch_l3_forward(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes,
                             const nfcs_desc* desc, const uint32_t* nh, uint32_t n,
                             const nfcs_nexthop* table, uint32_t table_n, uint8_t* status,
                             nfcs_patch* ws, hipStream_t stream, uint64_t slot_bytes, ObsReq obs) {
    (void)di;
    if (n == 0) return hipSuccess;
    const FwdArgs fa = {nh, table, table_n, obs};
    const uint64_t mean = shape_mean(arena_bytes, n, slot_bytes);
    if (mean < kTinyMeanBytes) {
        // short frames: 8-lane rows, 8 packets per one-wave workgroup (packet-rate bound, §5g)
        launch_rows<6, 8, 8, 64, true, SF_INLINE>((n + 7u) / 8u, 0u, stream, arena, arena_bytes, desc, n, 0u, status,
                                                  nullptr, nullptr, fa);
        return hipGetLastError();
    }
    if (mean < kSmallMeanBytes) {
        // mixes of short and long frames (the C3 mix): 8-lane rows of 12 slots (1536 bytes per row
        // pass, so a 1500-byte frame needs no second pass), 8 packets per wave at 6 waves/SIMD (80
        // VGPRs). The forward's header work (decision, MAC pick, segment) then serves 8 packets per
        // instruction instead of 4; its short waves are latency-bound and every instruction is on
        // their path: C3 mix 0.519 -> 0.587 (round 3, profiles/r03_s1_ab_fwd_c3_rows.jsonl). The plain
        // update keeps 16-lane rows there (8-lane rows of 12 slots: C3 0.569 vs 0.594). 256-thread
        // workgroups (32 packets) since round 5: in the steady state, median 0.6915 against 0.6935 ms
        // per call over 9 alternating processes each (profiles/r05_fwd_wg256_ab.jsonl)
        launch_rows<12, 8, 6, kBlock, true, SF_INLINE, 1, 12>((n + 31u) / 32u, 0u, stream, arena, arena_bytes, desc, n, 0u, status,
                                                   nullptr, nullptr, fa);
        return hipGetLastError();
    }
    if (ws && n > kFwdDeferAbovePackets) {
        // bursts of long frames: per 512K-packet sub-batch, a read pass whose long-frame waves write
        // forward records instead of segments, then apply_fwd_kernel while the header lines are
        // still in the memory-side cache (4M x 1500 B 0.681 -> 0.705; round 4, calls
        // rotating over fresh batches: 1M C1 bursts too; mixes like C3, whose waves rarely defer,
        // lose 10% to the sub-batch launches and take the short-mix shape above). The read pass is
        // held at 6 waves/SIMD by kRowsLdsPad6 (round 4, calls rotating over fresh batches: 4M -0.9%,
        // C1 -0.2% per call against 7; 5 waves, the update's long shape, +1.5-3.5% here;
        // profiles/r04_s2_fwd_occupancy_ab.jsonl)
        for (uint32_t i = 0; i < n; i += kSubBatchPackets) {
            const uint32_t m = std::min(kSubBatchPackets, n - i);
            const FwdArgs fs = {nh + i, table, table_n, i == 0 ? obs : ObsReq{}};
            launch_rows<6, 16, 7, kBlock, true, SF_DEFER, 2, 7>((m + 15u) / 16u, kRowsLdsPad6, stream, arena, arena_bytes, desc + i, m,
                                                          0u, status ? status + i : nullptr, nullptr, ws, fs);
            hipLaunchKernelGGL(apply_fwd_kernel, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, arena,
                               desc + i, m, nh + i, table, (const nfcs_patch*)ws);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    // 7 waves per SIMD (72 VGPRs and 94 SGPRs, no scratch; the compiler alone picks 81 VGPRs
    // and 106 SGPRs = 6 waves and the kernel runs 4-5% slower)
    launch_rows<6, 16, 7, kBlock, true, SF_INLINE, 2, 7>((n + 15u) / 16u, 0u, stream, arena, arena_bytes, desc, n, 0u, status,
                                                   nullptr, nullptr, fa);
    return hipGetLastError();
}

// ---- VLAN push / pop + checksum ----------------------------------------------
// Packet::push_vlan(vid, prio) / pop_vlan() (packet.hpp:655-720) and the update_checksums() they
// end with, in one pass per frame. One 16-lane row per packet as in update_rows_kernel: the row
// loads the frame's chunks (K slots of 16 lanes), builds the EDITED frame's chunks in registers
// (a 4-byte shift is one DPP row_shr:1 / row_shl:1 of a dword plus three register moves per
// chunk; the chunk that crosses a slot boundary takes a row_newbcast from the neighbouring
// slot), plans update_checksums() on the edited header, sums the edited chunks, patches the
// checksum bytes into the chunk registers and stores the edited frame with 16-byte stores. So
// the memmove, the tag and the checksums cost one read and one write of the frame.
//   * frames longer than one batch (K*16 chunks) are processed batch by batch, in ascending
//     order: a push carries the last dword of the previous batch's old chunks in a register
//     (the store of batch b overwrites it), a pop loads the first dword of the next batch;
//     batch 0 is then stored before the loop and the checksum bytes are stored at the end by
//     the lanes that stored their chunks;
//   * bytes of a frame's last chunk past the bytes the reference writes keep their old values
//     (the slot's tail is rewritten with what it held), so the arena matches the reference's
//     memmove byte for byte;
//   * uncommon headers take the same cold path as update_rows_kernel, after the edited frame is
//     in memory.
enum : uint32_t { VM_NONE = 0, VM_FAIL = 1, VM_RETAG = 2, VM_PUSH = 3, VM_POP = 4 };

// Chunk bytes at frame offsets >= wend keep their old values.
DEV uint4 keep_tail(const uint4& nv, const uint4& ov, uint32_t o, uint32_t wend) {
    uint32_t r[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const int nb = (int)wend - (int)(o + 4u * j);
        const uint32_t m = nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
        r[j] = (comp(nv, j) & m) | (comp(ov, j) & ~m);
    }
    return make_uint4(r[0], r[1], r[2], r[3]);
}

// Byte i (0..15) of a chunk register := b.

DEV uint32_t dpp_prev(uint32_t x) {  // lane rl gets lane rl-1 of its row (0 for rl = 0)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xF, 0xF, true);
}
DEV uint32_t dpp_next(uint32_t x) {  // lane rl gets lane rl+1 of its row (0 for rl = 15)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x101, 0xF, 0xF, true);
}

// Edited chunks of one batch. v: old chunks rl + 16k (+ cb) of the row's window, i.e. frame chunks
// rl + 16k + cb - mis (line-aligned windows: the frame's chunk 0 sits in lane mis of slot 0);
// prevw: for a push, the old dword just before this batch (the row's lane 15 of the previous
// batch); nextx: for a pop, the old dword just after it. Batch 0 (first = true) builds the new
// bytes 12-15 in chunk 0. Lanes before the frame start get values that are never stored or summed.
template <int K, int R = 16>
DEV void vlan_edit(uint4 (&nv)[K], const uint4 (&v)[K], uint32_t mode, uint32_t rl, bool first,
                   uint32_t prevw, uint32_t nextx, uint32_t tag_dw, uint32_t cb, uint32_t wend,
                   uint32_t mis = 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint4 e = v[k];
        if (mode == VM_PUSH) {  // new[o] = old[o - 4] for o >= 16
            uint32_t pw = dpp_prev(v[k].w);  // across an 8-lane row's start: replaced below
            const uint32_t lw = (k > 0) ? row_bcast<R - 1, R>(v[k - 1].w) : prevw;
            if (rl == 0) pw = lw;
            e = make_uint4(pw, v[k].x, v[k].y, v[k].z);
            if (first && k == 0 && rl == mis) e = make_uint4(v[0].x, v[0].y, v[0].z, tag_dw);
        } else if (mode == VM_POP) {  // new[o] = old[o + 4] for o >= 12
            uint32_t nx = dpp_next(v[k].x);  // across an 8-lane row's end: replaced below
            const uint32_t fx = (k + 1 < K) ? row_bcast<0, R>(v[k + 1 < K ? k + 1 : k].x) : nextx;
            if (rl == (uint32_t)R - 1u) nx = fx;
            e = make_uint4(v[k].y, v[k].z, v[k].w, nx);
            if (first && k == 0 && rl == mis) e = make_uint4(v[0].x, v[0].y, v[0].z, nx);
        } else if (mode == VM_RETAG) {
            if (first && k == 0 && rl == mis) e.w = tag_dw;
        }
        const uint32_t c = cb + rl + (uint32_t)R * (uint32_t)k - mis;
        nv[k] = (int)c < 0 ? v[k] : keep_tail(e, v[k], 16u * c, wend);
    }
}

// Store policy of the VLAN kernel's frame writes: every write of a frame (its rewritten chunks and,
// after them, its checksum bytes) takes the same path, so same-address writes stay in program order.
enum : int { VST_PLAIN = 0, VST_WT = 1, VST_NT = 2 };
template <int POL>
DEV void vst16(uint4* p, const uint4& v) {
    if (POL == VST_NT) st16_nt(p, v);
    else st16<POL == VST_WT>(p, v);
}
template <int POL>
DEV void vst8(uint8_t* p, uint32_t b) {
    if (POL == VST_NT) st8_nt(p, b);
    else st8<POL == VST_WT>(p, b);
}

// Frame chunk rl (rl < R) of a row whose window is line-aligned (slot 0 lane rl + mis, or slot 1).
template <int K, int R>
DEV uint4 vlan_view(const uint4 (&v)[K], uint32_t rowbase4, uint32_t rl, uint32_t mis) {
    const uint32_t a = rl + mis;
    const int sl = (int)(rowbase4 + (a & (R - 1)) * 4u);
    const uint4 r0 = make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[0].x),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[0].y),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[0].z),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[0].w));
    const uint4 r1 = make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[1].x),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[1].y),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[1].z),
                                (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[1].w));
    return a < (uint32_t)R ? r0 : r1;
}

// LA: line-aligned windows as in the checksum kernel (row_stage): lane rl of slot k holds frame
// chunk 16k + rl - mis, so every load and store instruction covers whole lines whatever the frame's
// line offset; the 4-byte moves are the same lane shifts in these coordinates, and the header views
// the edit and the plan read are rotated into frame order (vlan_view) in waves with a row starting
// mid-line.
template <int K, int K2 = 2, int POL = VST_PLAIN, int R = 16, bool LA = false>
__global__ __launch_bounds__(kBlock) void vlan_rows_kernel(uint8_t* __restrict__ arena,
                                                           uint64_t arena_bytes,
                                                           nfcs_desc* __restrict__ desc, uint32_t n,
                                                           const uint32_t* __restrict__ ops,
                                                           uint32_t op_all,
                                                           const uint32_t* __restrict__ caps,
                                                           uint32_t cap_all,
                                                           uint8_t* __restrict__ status,
                                                           uint64_t* __restrict__ obs, uint64_t obs_tag) {
    static_assert(R == 16 || R == 8, "16- or 8-lane rows");
    constexpr uint32_t PW = 64 / R, KR = (uint32_t)(K * R);
    const uint32_t lane = threadIdx.x & 63u, rl = lane & (R - 1), row = lane / R;
    const uint32_t rowbase4 = (lane & ~(uint32_t)(R - 1)) * 4u;
    const uint64_t pw = (uint64_t)blockIdx.x * (kBlock / R) + rfl(threadIdx.x >> 6) * PW;
    if (pw >= n) return;
    // the footprint sample for the next call's shape (lengths other waves are editing may be read
    // old or new: speed only)
    if (blockIdx.x == 0 && threadIdx.x < 64 && obs) sample_footprint(desc, obs_tag, lane, obs);
    const nfcs_desc d = pick_desc<PW>(load_descw<PW>(desc, pw, n), row);
    uint32_t op = op_all, cap = cap_all;
    {  // the wave's edit words / capacities: scalar loads, like the descriptors
        uint32_t q[PW], r[PW];
#pragma unroll
        for (uint32_t i = 0; i < PW; ++i) {
            q[i] = (ops && pw + i < n) ? ops[pw + i] : op_all;
            r[i] = (caps && pw + i < n) ? caps[pw + i] : cap_all;
        }
        if (ops) { op = 0; for (uint32_t i = 0; i < PW; ++i) op |= (row == i) ? q[i] : 0u; }
        if (caps) { cap = 0; for (uint32_t i = 0; i < PW; ++i) cap |= (row == i) ? r[i] : 0u; }
    }
    const uint64_t p = pw + row;
    const bool valid = p < n;
    const uint32_t kind = op & NFCS_VLAN_OP_MASK;
    const uint64_t off = (uint64_t)d.off16 * 16u;
    const uint64_t need = (uint64_t)d.len + (kind == NFCS_VLAN_PUSH ? 4u : 0u);
    const bool bad = valid && (off + ((need + 15u) & ~15ull) > arena_bytes);
    const bool live = valid && !bad;
    const uint32_t len = live ? d.len : 0u;
    uint8_t* frame = arena + (live ? off : 0);
    const uint4* src = (const uint4*)frame;
    const uint32_t nl = live ? (uint32_t)((need + 15u) >> 4) : 0u;  // old chunks to load
    // a row takes line-aligned windows only where they need no more row passes than frame-relative
    // ones (a 1500-byte frame 48+ bytes into a line would spill into a second pass: 64-byte starts
    // measured 0.47 against 0.71 with it)
    const uint32_t lm = LA && live ? (uint32_t)(((uintptr_t)frame >> 4) & 7u) : 0u;
    const uint32_t mis = (nl + lm <= KR || nl > KR) ? lm : 0u;
    const bool rot = LA && __builtin_amdgcn_ballot_w64(mis != 0) != 0;  // wave-uniform

    const uint4* zl = g_zero_line;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = rl + (uint32_t)R * k - mis;  // frame chunk (wraps below the frame start)
        v[k] = ld16<0>((c < nl) ? src + c : zl);
    }
    // pop: the old dword after batch 0 (first dword of the window's chunk KR)
    const uint32_t nx0 = *(const uint32_t*)((KR - mis < nl) ? src + (KR - mis) : zl);

    // the edit the reference makes (packet.hpp:655-720), decided on the old header
    const RowHdr<R> h{rot ? vlan_view<K, R>(v, rowbase4, rl, mis) : v[0], rowbase4};
    const bool tagged = len >= 14 && h.be16(12) == 0x8100u;  // has_vlan() (603-606)
    uint32_t mode = VM_NONE;
    if (live && kind == NFCS_VLAN_PUSH)
        mode = len < 14 ? VM_FAIL : tagged ? VM_RETAG : (len + 4u > cap ? VM_FAIL : VM_PUSH);
    else if (live && kind == NFCS_VLAN_POP)
        mode = (!tagged || len < 18) ? VM_FAIL : VM_POP;
    const bool act = mode >= VM_RETAG;
    const uint32_t vid = op & 0x0FFFu, prio = (op >> 13) & 7u;
    const uint32_t tci_old = h.be16(14);
    const uint32_t tci = ((mode == VM_RETAG ? tci_old : 0u) & 0x1000u) | (prio << 13) | vid;  // 185-190
    const uint32_t tag_dw = (mode == VM_RETAG) ? ((comp(v[0], 3) & 0xFFFFu) | (bswap16(tci) << 16))
                                               : (0x81u | (bswap16(tci) << 16));
    const uint32_t nlen = mode == VM_PUSH ? len + 4u : mode == VM_POP ? len - 4u : len;
    // bytes the reference writes end at wend: the moved frame, or bytes 14-15 of the tag
    const uint32_t wend = mode == VM_RETAG ? (len > 16u ? len : 16u) : nlen;
    const uint32_t nst = !act ? 0u : mode == VM_RETAG ? 1u : (wend + 15u) >> 4;  // chunks stored

    uint4 nv[K];
    vlan_edit<K, R>(nv, v, mode, rl, true, 0u, nx0, tag_dw, 0u, wend, mis);
    uint32_t carry = row_bcast<R - 1, R>(v[K - 1].w);  // push: old dword before batch 1

    // update_checksums() on the edited frame (690 / 718)
    RPlan P = fast_plan<R>(rot ? vlan_view<K, R>(nv, rowbase4, rl, mis) : nv[0], rowbase4, nlen);
    const bool slow = act && (P.st >> 8) != 0;
    if (!act || slow) P = rplan_none(0);
    const uint32_t re = (P.flags & F_L4) ? P.re : 0u, lo4 = P.rs & ~3u;
    const uint32_t tailfix = P.flags & F_TAIL;
    uint32_t rlv = rl;
    asm volatile("" : "+v"(rlv));
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = rlv + (uint32_t)R * k - mis;
        if ((int)c >= 0) acc_slot(acc, nv[k], c, lo4, re, tailfix);
    }

    // rows whose frame continues past batch 0 (moved chunks or summed chunks)
    const uint32_t nre = (re + 15u) >> 4;
    const uint32_t cm = ((nst > nre) ? nst : nre) + mis;  // window chunks
    const bool multi = __builtin_amdgcn_ballot_w64(cm > KR) != 0;  // wave-uniform
    auto finish = [&](uint32_t a) -> uint32_t {  // l4 field word
        const uint32_t z = row_sum<R>(a) + P.corr;
        uint32_t c = (~fold32(z)) & 0xFFFFu;
        if ((P.flags & F_UDP) && c == 0) c = 0xFFFFu;
        return (P.flags & F_L4) ? (P.fs | (c << 16)) : NFCS_PATCH_NONE;
    };
    const uint32_t ipw = (P.flags & F_IP) ? P.ipw : NFCS_PATCH_NONE;
    uint32_t l4w = NFCS_PATCH_NONE;
    if (!multi) {
        l4w = finish(acc);
        // checksum bytes into the chunk registers (fast-path fields lie below byte 80: slot 0);
        // a re-tag stores chunk 0 and the chunks holding checksum bytes
        // (byte by byte: put_field measured 1.2% slower here, 0.723 against 0.732 on C1)
        // (with line-aligned windows the chunk of byte pos sits in lane (pos/16 + mis) % R of slot
        // (pos/16 + mis) / R: slot 0, or slot 1 of an 8-lane row)
        bool patched0 = false, patched1 = false;
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) {
            const uint32_t w = (t < 2) ? ipw : l4w;
            const uint32_t pos = (w & 0xFFFFu) + (t & 1u);
            const uint32_t a = (pos >> 4) + mis, b = (w >> (16 + 8 * (t & 1u))) & 0xFFu;
            if ((w & 0xFFFFu) != NFCS_PATCH_NONE && (a & (R - 1)) == rl) {
                if (a < (uint32_t)R) {
                    nv[0] = put_byte(nv[0], pos & 15u, b);
                    patched0 = true;
                } else {
                    nv[1] = put_byte(nv[1], pos & 15u, b);
                    patched1 = true;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = rl + (uint32_t)R * k - mis;
            if (c < nst || (k == 0 && patched0) || (k == 1 && patched1)) vst16<POL>((uint4*)frame + c, nv[k]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = rl + (uint32_t)R * k - mis;
            if (c < nst) vst16<POL>((uint4*)frame + c, nv[k]);
        }
        const uint32_t cmax = wave_max_rows<R>(cm);
        // the rest of a long frame in batches of K2 slots (K2 < K saves VGPRs: w and e live
        // together here)
        constexpr uint32_t KR2 = (uint32_t)(K2 * R);
        for (uint32_t cb = KR; cb < cmax; cb += KR2) {
            uint4 w[K2], e[K2];
#pragma unroll
            for (int k = 0; k < K2; ++k) {
                const uint32_t c = cb + rlv + (uint32_t)R * k - mis;
                w[k] = ld16<1>((c < nl) ? src + c : zl);
            }
            const uint32_t nx = *(const uint32_t*)((cb + KR2 - mis < nl) ? src + (cb + KR2 - mis) : zl);
            vlan_edit<K2, R>(e, w, mode, rl, false, carry, nx, 0u, cb, wend, mis);
            carry = row_bcast<R - 1, R>(w[K2 - 1].w);
#pragma unroll
            for (int k = 0; k < K2; ++k) {
                const uint32_t c = cb + rlv + (uint32_t)R * k - mis;
                acc_slot(acc, e[k], c, lo4, re, tailfix);
                if (c < nst) vst16<POL>((uint4*)frame + c, e[k]);
            }
        }
        l4w = finish(acc);
        // the lanes that stored chunk pos/16 store the checksum bytes (program order)
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) {
            const uint32_t w = (t < 2) ? ipw : l4w;
            const uint32_t pos = (w & 0xFFFFu) + (t & 1u);
            if ((w & 0xFFFFu) != NFCS_PATCH_NONE && (((pos >> 4) + mis) & (R - 1)) == rl)
                vst8<POL>(frame + pos, w >> (16 + 8 * (t & 1u)));
        }
    }
    const uint32_t st0 = bad ? (uint32_t)NFCS_ST_BAD_DESC
                       : mode == VM_FAIL ? (uint32_t)NFCS_ST_VLAN_FAIL
                       : act ? (P.st | NFCS_ST_FLAG_VLAN) : (uint32_t)NFCS_ST_NONE;
    if (valid && rl == 0) {
        if (!slow && status) status[p] = (uint8_t)st0;
        if (act) desc[p].len = nlen;
    }
    if (__builtin_amdgcn_ballot_w64(slow) != 0) {  // cold path on the edited frame in memory
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        RPlan Q = rplan_none(0);
        SeqOut o = {0, 0, 0, 0, 0};
        if (slow && rl == 0) {
            Q = slow_plan(frame, nlen);
            if (Q.flags & F_SEQ) o = seq_update(frame, nlen);
        }
        Q.st = row_bcast<0, R>(Q.st);
        Q.flags = row_bcast<0, R>(Q.flags);
        Q.ipw = row_bcast<0, R>(Q.ipw);
        Q.rs = row_bcast<0, R>(Q.rs);
        Q.re = row_bcast<0, R>(Q.re);
        Q.fs = row_bcast<0, R>(Q.fs);
        Q.corr = row_bcast<0, R>(Q.corr);
        const uint32_t ost = row_bcast<0, R>(o.st);
        const bool seq = slow && (Q.flags & F_SEQ);
        const uint32_t re2 = (slow && !seq && (Q.flags & F_L4)) ? Q.re : 0u;
        const uint32_t lo42 = Q.rs & ~3u, tf2 = Q.flags & F_TAIL;
        uint32_t acc2 = 0;
        for (uint32_t c = rl; c < ((re2 + 15u) >> 4); c += R) acc_slot(acc2, src[c], c, lo42, re2, tf2);
        const uint32_t z2 = row_sum<R>(acc2) + Q.corr;
        const uint32_t ipw2 = (Q.flags & F_IP) ? Q.ipw : NFCS_PATCH_NONE;
        uint32_t l4w2 = NFCS_PATCH_NONE;
        if (Q.flags & F_L4) {
            uint32_t c = (~fold32(z2)) & 0xFFFFu;
            if ((Q.flags & F_UDP) && c == 0) c = 0xFFFFu;
            l4w2 = Q.fs | (c << 16);
        }
        if (slow && !seq && rl < 4) {
            const uint32_t w = (rl & 2u) ? l4w2 : ipw2;
            const uint32_t pos = (w & 0xFFFFu) + (rl & 1u);
            if ((w & 0xFFFFu) != NFCS_PATCH_NONE) vst8<POL>(frame + pos, w >> (16 + 8 * (rl & 1u)));
        }
        if (slow && rl == 0 && status)
            status[p] = (uint8_t)((seq ? (ost | NFCS_ST_FLAG_OVERLAP) : Q.st) | NFCS_ST_FLAG_VLAN);
    }
}

hipError_t launch_vlan(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes, nfcs_desc* desc,
                       uint32_t n, const uint32_t* ops, uint32_t op_all, const uint32_t* caps,
                       uint32_t cap_all, uint8_t* status, hipStream_t stream, uint64_t slot_bytes,
                       ObsReq obs, uint32_t sample_bits) {
    (void)di;
    if (n == 0) return hipSuccess;
    // Long frames continue in batches of 6 slots (128 VGPRs, 4 waves/SIMD); batches of 2 slots
    // (94 VGPRs, 5 waves/SIMD) measured 6% slower on C1 push/pop, capping the occupancy lower
    // slower still (profiles/r01_s2_occupancy.md); dispatch order (the XCD-aware order measured 2%
    // slower here). Frame stores past the caches (`sc0 sc1 nt`, round 2 session 3): C1 push/pop
    // +4.5%, 1M 256 / 512-byte frames +2-5% against write-through `sc1` (itself +1.2% over plain
    // stores); frames in slots under 256 B keep `sc1` (64-byte frames: 177 vs 181 µs per 1M).
    // Short frames (mean footprint < kTinyMeanBytes): 8-lane rows, 8 packets per wave (§5g), their
    // stores write-through also when the burst's sample found frames off their lines or of varying
    // lengths (sample_bits; nfcs_internal.h kVlanWtMeanBytes).
    const uint64_t mean = shape_mean(arena_bytes, n, slot_bytes);
    const dim3 g8((n + 31u) / 32u), g16((n + 15u) / 16u);
    if (mean < kVlanWtMeanBytes || (mean < kTinyMeanBytes && (sample_bits & (kObsUnaligned | kObsMixed))))
        hipLaunchKernelGGL((vlan_rows_kernel<6, 6, VST_WT, 8>), g8, dim3(kBlock), 0, stream, arena, arena_bytes,
                           desc, n, ops, op_all, caps, cap_all, status, obs.slot, obs.tag);
    else if (mean < kTinyMeanBytes)
        hipLaunchKernelGGL((vlan_rows_kernel<6, 6, VST_NT, 8>), g8, dim3(kBlock), 0, stream, arena, arena_bytes,
                           desc, n, ops, op_all, caps, cap_all, status, obs.slot, obs.tag);
    else  // 4 rows per wave, 4 waves per workgroup
        hipLaunchKernelGGL((vlan_rows_kernel<6, 6, VST_NT, 16, true>), g16, dim3(kBlock), 0, stream, arena, arena_bytes,
                           desc, n, ops, op_all, caps, cap_all, status, obs.slot, obs.tag);
    return hipGetLastError();
}

// ---- flow-key extract + hash -----------------------------------------------
// PacketClassifier::extract_flow_key + hash_flow (packet_classifier.cpp:12-108) on the first 96
// bytes of each frame (every field the key reads lies below byte 82: l2 18 + IHL 60 + 4 port bytes).
// hash_flow's byte-wise XOR at shift (i % 4) * 8 is the XOR of little-endian dwords.
static_assert(sizeof(nfcs_flow_key) == 64, "nfcs_flow_key is a 64-byte record");

// A wave takes 64 packets. Their header bytes 0..95 are loaded in 8-lane rows — one coalesced
// 128-byte line per packet, 8 packets per instruction, 8 instructions in flight — and written to
// LDS (96 bytes per packet); then lane l parses packet l on its own, reading the fields at their
// (802.1Q- and IHL-dependent) byte offsets from LDS, so one VALU instruction serves 64 packets and
// no DPP broadcast is needed (round 2's form parsed in 8-lane rows: 909 VALU + 539 SALU per 32
// packets, 0.77 against 0.82 now); the 64-byte records go back through LDS so each global store
// writes 1 KB of consecutive records.
DEV uint32_t lds_u8(const uint8_t* b, uint32_t o) { return b[o]; }
DEV uint32_t lds_be16(const uint8_t* b, uint32_t o) { return ((uint32_t)b[o] << 8) | b[o + 1]; }
DEV uint32_t lds_le32(const uint8_t* b, uint32_t o) {  // any alignment, 2-byte pieces where it can
    if ((o & 1u) == 0) return (uint32_t)*(const uint16_t*)(b + o) | ((uint32_t)*(const uint16_t*)(b + o + 2) << 16);
    return (uint32_t)b[o] | ((uint32_t)b[o + 1] << 8) | ((uint32_t)b[o + 2] << 16) | ((uint32_t)b[o + 3] << 24);
}

constexpr uint32_t kFkRow = 96;  // LDS bytes per packet: header bytes 0..95

__global__ __launch_bounds__(kBlock) void flow_keys_lanes_kernel(const nfcs_desc* __restrict__ desc, uint32_t n,
                                                                 uint32_t nblocks, const uint8_t* __restrict__ arena,
                                                                 uint64_t arena_bytes, nfcs_flow_key* __restrict__ keys,
                                                                 uint32_t* __restrict__ hashes) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerBlock * 64 * kFkRow];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t p0 = ((uint64_t)xcd_block_n(nblocks) * kWavesPerBlock + rfl(wave)) * 64u;
    if (p0 >= n) return;
    uint8_t* rows = lds + wave * 64u * kFkRow;
    // lane l: descriptor of packet p0 + l (one coalesced load); dead packets read as length 0
    const uint64_t p = p0 + lane;
    uint2 dl = make_uint2(0u, 0u);
    if (p < n) dl = ((const uint2*)desc)[p];
    const uint64_t off = (uint64_t)dl.x * 16u;
    const bool live = p < n && off + (((uint64_t)dl.y + 15u) & ~15ull) <= arena_bytes;
    const uint32_t len = live ? dl.y : 0u;
    // Header bytes 0..47 (every field of an IPv4 header without options, tagged or not, and its
    // ports) in 8-lane rows: instruction k, row r -> packet 8k + r, lane rl -> chunk rl (0..2). A
    // frame starting up to 80 bytes into a 128-byte line reads that one line (64-byte starts: one
    // line instead of two; round 3). Headers reaching past byte 47 (IPv6, IPv4 options) load chunks
    // 3..5 afterwards, lane by lane. The header lines load non-temporally (round 5, calls rotating
    // over fresh batches, same box: 0.0385-0.0390 against 0.0411-0.0414 ms per 1M C1 frames; `sc1` /
    // `sc0 sc1` loads measured as the default; profiles/r05_flowkey_load_policy_ab.jsonl).
    const uint32_t rl = lane & 7u, r = lane >> 3;
    const uint4* zl = g_zero_line;
    uint4 c[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t q = 8u * k + r;
        const uint32_t qo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(q * 4u), (int)dl.x);
        const uint32_t ql = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(q * 4u), (int)len);
        const uint4* src = (const uint4*)(arena + (uint64_t)qo * 16u);
        c[k] = ld16<1>((rl < 3u && rl * 16u < ql) ? src + rl : zl);
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k)
        if (rl < 3u) *(uint4*)(rows + (8u * k + r) * kFkRow + 16u * rl) = c[k];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done
    __builtin_amdgcn_wave_barrier();
    // lane l parses packet l (extract_flow_key + hash_flow, packet_classifier.cpp:12-108)
    uint8_t* b = rows + lane * kFkRow;
    {  // the bytes the key reads end at the ports (IPv4: l2 + IHL*4 + 4; IPv6: l2 + 44)
        const uint32_t f12 = lds_be16(b, 12), ft = f12 == 0x8100u ? 4u : 0u;
        const uint32_t fet = (f12 == 0x8100u && len >= 18) ? lds_be16(b, 16) : f12;
        const uint32_t need = (fet == 0x0800u && 34u + ft <= len) ? 18u + ft + (lds_u8(b, 14u + ft) & 15u) * 4u
                            : (fet == 0x86DDu && 54u + ft <= len) ? 58u + ft : 0u;
        const bool more = len >= 14 && need > 48u && len > 48u;
        if (__builtin_amdgcn_ballot_w64(more) != 0) {
            if (more) {
                const uint4* src = (const uint4*)(arena + off);
#pragma unroll
                for (uint32_t j = 3; j < 6; ++j) *(uint4*)(b + 16u * j) = ld16<0>(16u * j < len ? src + j : zl);
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
        }
    }
    const bool eth = len >= 14;
    const uint32_t m0 = eth ? *(const uint32_t*)b : 0u, m1 = eth ? *(const uint32_t*)(b + 4) : 0u;
    const uint32_t m2 = eth ? *(const uint32_t*)(b + 8) : 0u;
    const uint32_t e12 = lds_be16(b, 12);
    const bool tagged = e12 == 0x8100u;
    uint32_t et = eth ? e12 : 0u, vlan = 0;
    if (eth && tagged && len >= 18) {  // has_vlan / vlan_id / vlan() (packet.hpp:603-618)
        vlan = lds_be16(b, 14) & 0x0FFFu;
        et = lds_be16(b, 16);
    }
    const uint32_t sh = tagged ? 4u : 0u;  // l2 = 18 after a tag (ethernet(), packet.hpp:410)
    const bool v4 = et == 0x0800u, v6 = et == 0x86DDu;
    uint32_t proto = 0, sp = 0, dp = 0, s4 = 0, d4 = 0, l4 = 0;
    uint32_t s6[4] = {0, 0, 0, 0}, d6[4] = {0, 0, 0, 0};
    bool hdr = false;
    if (v4 && 34u + sh <= len) {  // ipv4() present
        s4 = __builtin_bswap32(lds_le32(b, 26u + sh));
        d4 = __builtin_bswap32(lds_le32(b, 30u + sh));
        proto = lds_u8(b, 23u + sh);
        l4 = 14u + (lds_u8(b, 14u + sh) & 15u) * 4u;
        hdr = true;
    } else if (v6 && 54u + sh <= len) {  // ipv6() present
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            s6[j] = lds_le32(b, 22u + sh + 4u * j);
            d6[j] = lds_le32(b, 38u + sh + 4u * j);
        }
        proto = lds_u8(b, 20u + sh);
        l4 = 54u;
        hdr = true;
    }
    // tcp() needs l4 + 19 <= len (19-byte TcpHeader), udp() l4 + 8 (packet.hpp:473-535)
    if (hdr && ((proto == 6 && l4 + sh + 19u <= len) || (proto == 17 && l4 + sh + 8u <= len))) {
        sp = lds_be16(b, l4 + sh);
        dp = lds_be16(b, l4 + sh + 2u);
    }
    uint32_t hv = m0 ^ (m1 & 0xFFFFu) ^ ((m1 >> 16) | (m2 << 16)) ^ (m2 >> 16);
    hv ^= vlan ^ (et << 16);
    if (v6) hv ^= s6[0] ^ s6[1] ^ s6[2] ^ s6[3] ^ d6[0] ^ d6[1] ^ d6[2] ^ d6[3];
    else hv ^= s4 ^ d4;
    hv ^= proto ^ (sp << 16) ^ dp;
    if (!live) hv = 0;
    if (hashes && p < n) hashes[p] = hv;
    if (!keys) return;
    // the record (nfcs_flow_key: hash, vlan, ethertype, MACs, ports, addresses) into this lane's LDS row, then 1 KB of
    // consecutive records per store instruction
    uint4* rec = (uint4*)(rows + lane * kFkRow);
    __builtin_amdgcn_wave_barrier();
    rec[0] = make_uint4(hv, vlan | (et << 16), (m1 >> 16) | (m2 << 16), (m2 >> 16) | (m0 << 16));
    rec[1] = make_uint4((m0 >> 16) | (m1 << 16), proto | ((v6 ? 1u : 0u) << 8) | (sp << 16), dp, 0u);
    rec[2] = v6 ? make_uint4(s6[0], s6[1], s6[2], s6[3]) : make_uint4(s4, 0u, 0u, 0u);
    rec[3] = v6 ? make_uint4(d6[0], d6[1], d6[2], d6[3]) : make_uint4(d4, 0u, 0u, 0u);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t q = 16u * j + (lane >> 2);  // packet of this 16-byte piece
        const uint4 v = *(const uint4*)(rows + q * kFkRow + 16u * (lane & 3u));
        // plain (write-back) stores: the L2 merges each 1 KB into whole lines (round 5, calls
        // rotating over fresh batches, same box: 0.0352-0.0355 against 0.0387-0.0392 ms per 1M C1
        // frames with non-temporal ones; profiles/r05_store_policy_ab.jsonl)
        if (p0 + q < n) *((uint4*)(keys + p0 + q) + (lane & 3u)) = v;
    }
}

hipError_t launch_flow_keys(const DevInfo& di, const uint8_t* arena, uint64_t arena_bytes,
                            const nfcs_desc* desc, uint32_t n, nfcs_flow_key* keys,
                            uint32_t* hashes, hipStream_t stream) {
    (void)di;
    if (n == 0) return hipSuccess;
    // 64 packets per wave, one lane each (round 3: C1 0.77 -> 0.82 against round 2's 8-lane rows of
    // 4 slots; profiles/r03_s2_ab_flowkey_lanes.jsonl); write-back record stores, XCD-aware order
    const uint32_t g = (n + 255u) / 256u;
    hipLaunchKernelGGL(flow_keys_lanes_kernel, dim3(g), dim3(kBlock), 0, stream, desc, n, g, arena, arena_bytes, keys,
                       hashes);
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

// ---- read-stream reference (bench support; SURVEY.md §8d "achieved fraction of a measured
// read-only stream kernel on the same box") -------------------------------------------------------
// Pure reads of `bytes` (16-byte multiple), summed into a value that is stored only if it equals an
// impossible constant (the loads stay live, nothing is written). The bench times every form over the
// batch's own arena and takes the fastest as the ceiling:
//   form 0  the checksum read pass's own shape: 256-thread workgroups in the XCD-aware order held at
//           6 waves/SIMD, each wave reading 6 KiB as 6 wave-wide 1 KiB loads in flight (lane l:
//           chunks l + 64k), the first with the default policy and the rest non-temporal;
//   form 2  the same, every load non-temporal;
//   form 3  8 loads per lane (8 KiB per wave), all non-temporal, no occupancy cap;
//   form 4  16 loads per lane (16 KiB per wave), all non-temporal, no occupancy cap;
//   form 5  4 loads per lane (4 KiB per wave), all non-temporal, no occupancy cap;
//   form 1  round 1's microbenchmark (tools/stream_read.hip): 512 workgroups striding over the
//           buffer, 4 non-temporal loads per lane in flight.
template <uint32_t K, bool MIX>  // MIX: the first load of each wave with the default policy
__global__ __launch_bounds__(kBlock) void stream_read_kernel(const uint4* __restrict__ p, uint64_t n16,
                                                             unsigned long long* __restrict__ sink) {
    const uint64_t w = (uint64_t)xcd_block() * kWavesPerBlock + (threadIdx.x >> 6);
    const uint64_t base = w * 64u * K + (threadIdx.x & 63u);
    uint4 v[K];
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) {
        const uint64_t i = base + 64u * k;
        const uint4* a = i < n16 ? p + i : g_zero_line;
        v[k] = (MIX && k == 0) ? ld16<0>(a) : ld16<1>(a);
    }
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) acc += v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (acc == 0x9E3779B9u && sink) *sink = acc;
}

__global__ __launch_bounds__(kBlock) void stream_read_strided_kernel(const uint4* __restrict__ p, uint64_t n16,
                                                                     unsigned long long* __restrict__ sink) {
    constexpr uint32_t U = 4;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t acc = 0;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        uint4 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = ld16<1>(p + i + u * stride);
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) {
        const uint4 v = ld16<1>(p + i);
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u && sink) *sink = acc;
}

hipError_t launch_stream_read(const uint8_t* buf, uint64_t bytes, int form, unsigned long long* sink,
                              hipStream_t stream) {
    const uint64_t n16 = bytes / 16u;
    if (n16 == 0) return hipSuccess;
    const uint4* q = (const uint4*)buf;
    auto grid = [&](uint32_t k) { return dim3((uint32_t)((n16 + 64u * k * kWavesPerBlock - 1) / (64u * k * kWavesPerBlock))); };
    switch (form) {
    case 1: hipLaunchKernelGGL(stream_read_strided_kernel, dim3(512), dim3(kBlock), 0, stream, q, n16, sink); break;
    // forms 0 and 2 are held at 6 waves/SIMD (the round-1 read stream's best)
    case 0: hipLaunchKernelGGL((stream_read_kernel<6, true>), grid(6), dim3(kBlock), kRowsLdsPad6, stream, q, n16, sink); break;
    case 2: hipLaunchKernelGGL((stream_read_kernel<6, false>), grid(6), dim3(kBlock), kRowsLdsPad6, stream, q, n16, sink); break;
    case 3: hipLaunchKernelGGL((stream_read_kernel<8, false>), grid(8), dim3(kBlock), 0, stream, q, n16, sink); break;
    case 4: hipLaunchKernelGGL((stream_read_kernel<16, false>), grid(16), dim3(kBlock), 0, stream, q, n16, sink); break;
    default: hipLaunchKernelGGL((stream_read_kernel<4, false>), grid(4), dim3(kBlock), 0, stream, q, n16, sink); break;
    }
    return hipGetLastError();
}

// The read-only floor of the checksum read pass's own access pattern (bench `stream_ceiling`): the
// batch's frames read exactly as update_rows_kernel reads them — 16-lane rows, 6 slots, four packets
// per wave, 256-thread workgroups held at 5 waves/SIMD, XCD-aware order, the header slot with the
// default policy and the rest non-temporal, jumbo frames continued in batches of 6 slots — with
// nothing computed or written (the chunks are XOR-ed into a value stored only if it equals an
// impossible constant). A buffer stream reads the arena contiguously; this form reads what the
// product reads, in its order, so it bounds the product on every layout (C2's 9.5 GB arena: a
// contiguous stream measured below the product on some boxes).
__global__ __launch_bounds__(kBlock) void frames_read_kernel(const nfcs_desc* __restrict__ desc, uint32_t n,
                                                             uint32_t nblocks, const uint8_t* __restrict__ arena,
                                                             uint64_t arena_bytes, unsigned long long* __restrict__ sink) {
    constexpr int K = 6, R = 16, PW = 4;
    const uint32_t lane = threadIdx.x & 63u, rl = lane & (R - 1), row = lane / R;
    const uint64_t pw = (uint64_t)xcd_block_n(nblocks) * (kBlock / R) + rfl(threadIdx.x >> 6) * PW;
    if (pw >= n) return;
    const nfcs_desc d = pick_desc<PW>(load_descw<PW>(desc, pw, n), row);
    const uint64_t off = (uint64_t)d.off16 * 16u;
    const bool live = pw + row < n && off + (((uint64_t)d.len + 15u) & ~15ull) <= arena_bytes;
    const uint32_t nch = live ? (d.len + 15u) >> 4 : 0u;
    const uint4* src = (const uint4*)(arena + (live ? off : 0));
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = rl + (uint32_t)R * k;
        const uint4* a = (c < nch) ? src + c : g_zero_line;
        v[k] = k == 0 ? ld16<0>(a) : ld16<1>(a);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    const uint32_t cmax = wave_max_rows<R>(nch);
    for (uint32_t cb = (uint32_t)R * K; cb < cmax; cb += (uint32_t)R * K) {
        uint4 w[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = cb + rl + (uint32_t)R * k;
            w[k] = ld16<1>((c < nch) ? src + c : g_zero_line);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc ^= w[k].x ^ w[k].y ^ w[k].z ^ w[k].w;
    }
    if (acc == 0x9E3779B9u && sink) *sink = acc;
}

hipError_t launch_frames_read(const uint8_t* arena, uint64_t arena_bytes, const nfcs_desc* desc, uint32_t n,
                              unsigned long long* sink, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t grid = (n + 15u) / 16u;
    hipLaunchKernelGGL(frames_read_kernel, dim3(grid), dim3(kBlock), kRowsLdsPad, stream, desc, n, grid, arena,
                       arena_bytes, sink);
    return hipGetLastError();
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
