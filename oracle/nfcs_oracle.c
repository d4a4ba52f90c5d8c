/*
 * nfcs_oracle.c — TEST INFRASTRUCTURE ONLY (see nfcs_oracle.h).
 *
 * A plain-C restatement of NetFlow++'s checksum path, kept deliberately sequential and
 * byte-level so that it reproduces the reference's behaviour exactly, including:
 *   - the 19-byte TcpHeader whose checksum sits at TCP offset 15 (packet.hpp:258-270);
 *   - the odd trailing byte added as the LOW byte (packet.hpp:903-905);
 *   - UDP coverage = udp.length, TCP/ICMP coverage = total_length - IHL*4;
 *   - UDP 0 -> 0xFFFF only (packet.hpp:867-871);
 *   - IPv4 selected by the version nibble, IPv6 by EtherType + nibble (packet.hpp:728-752);
 *   - writes happen in the reference's order (IPv4 checksum first, then the L4 field is
 *     zeroed before the pseudo-header and segment are read), which matters only when
 *     IHL < 5 makes the L4 region overlap the IPv4 header.
 * Each function cites the reference lines it follows.
 */
#include "nfcs_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define GOLDEN 0x9E3779B97F4A7C15ULL

static inline unsigned be16(const uint8_t* f, size_t o) { return ((unsigned)f[o] << 8) | f[o + 1]; }

/* Raw one's-complement accumulation of packet.hpp:898-905 (before the fold):
 * big-endian 16-bit words, odd trailing byte added as its raw value (the low byte). */
static uint32_t sum_words(const uint8_t* d, size_t len) {
    uint32_t sum = 0;
    size_t i = 0;
    while (len > 1) {           /* packet.hpp:898-901 */
        sum += be16(d, i);
        i += 2;
        len -= 2;
    }
    if (len > 0) sum += d[i];   /* packet.hpp:903-905: ntohs((uint16_t)b << 8) == b */
    return sum;
}

/* packet.hpp:907-911: end-around-carry fold, complement. Returns the host value whose
 * big-endian bytes the reference stores (it returns htons(~sum) and stores it raw). */
static uint16_t finish(uint32_t sum) {
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    return (uint16_t)~sum;
}

uint16_t nfo_calculate_checksum(const uint8_t* data, size_t len) {
    return finish(sum_words(data, len));
}

static inline void store_be16(uint8_t* f, size_t o, uint16_t v) {
    f[o] = (uint8_t)(v >> 8);
    f[o + 1] = (uint8_t)v;
}

/* Packet::update_checksums(), packet.hpp:722-890, on frame bytes [0, len). */
int nfo_update(uint8_t* f, size_t len) {
    /* ethernet() 405-418: l2 is 18 after a 0x8100 tag; with len < 14 it keeps the ctor's 14 (346) */
    size_t l2 = 14;
    if (len >= 14) l2 = (be16(f, 12) == 0x8100) ? 18 : 14;

    int v4 = 0;
    unsigned proto;
    size_t ihl4 = 0, l4;
    int overlap = 0;

    /* 728-740: IPv4 when get_header<IPv4Header>(l2) fits (l2+20 <= len) and nibble == 4 */
    if (l2 + 20 <= len && (f[l2] >> 4) == 4) {
        v4 = 1;
        proto = f[l2 + 9];
        ihl4 = (size_t)(f[l2] & 15) * 4;
        l4 = l2 + ihl4;
        /* 740 sums ihl4 bytes with no bound check: past the frame it reads foreign memory.
         * Outside the parity domain: leave the frame untouched. */
        if (l2 + ihl4 > len) return NFO_ST_OOB;
        overlap = (ihl4 < 20) && (proto == 6 || proto == 17 || proto == 1);
        f[l2 + 10] = 0; /* 739 */
        f[l2 + 11] = 0;
        store_be16(f, l2 + 10, nfo_calculate_checksum(f + l2, ihl4)); /* 740 */
    } else {
        /* 741-765: effective EtherType after at most one 0x8100 tag */
        unsigned et = (len >= 14) ? be16(f, 12) : 0;
        if (et == 0x8100) et = (len >= 18) ? be16(f, 16) : 0;
        if (et != 0x86DD) return NFO_ST_NONE;
        if (!(l2 + 40 <= len && (f[l2] >> 4) == 6)) return NFO_ST_NONE; /* 750-759 */
        proto = f[l2 + 6];
        l4 = l2 + 40;
    }
    const int ov = overlap ? NFO_ST_FLAG_OVERLAP : 0;
    const int skip = (v4 ? NFO_ST_V4_L4SKIP : NFO_ST_V6_L4SKIP) | ov;

    if (proto == 6) {
        /* 773-823 */
        if (l4 + 19 > len) return skip;                /* get_header<TcpHeader>: sizeof 19 */
        size_t hl = (size_t)(f[l4 + 12] >> 4) * 4;     /* get_header_length(): byte 12 */
        unsigned seg;
        if (v4) {
            unsigned tl = be16(f, l2 + 2);
            if (tl < ihl4) return skip;                /* 780 */
            seg = (unsigned)((tl - ihl4) & 0xFFFF);     /* 781: uint16_t */
        } else {
            seg = be16(f, l2 + 4);                     /* 783 */
        }
        if (seg < hl) return skip;                     /* 786 */
        if (l4 + seg > len) return skip;               /* 791-793 */
        f[l4 + 15] = 0;                                /* 795: checksum at offset 15 */
        f[l4 + 16] = 0;
        /* 797-822: pseudo-header (12 or 40 bytes, even) ++ segment, one fold */
        uint32_t sum;
        if (v4) {
            sum = sum_words(f + l2 + 12, 8) + 6 + seg;            /* src, dst, 0, 6, len */
        } else {
            sum = sum_words(f + l2 + 8, 32) + (seg >> 16) + (seg & 0xFFFF) + 6;
        }
        sum += sum_words(f + l4, seg);
        store_be16(f, l4 + 15, finish(sum));           /* 822 */
        return (v4 ? NFO_ST_V4_TCP : NFO_ST_V6_TCP) | ov;
    }
    if (proto == 17) {
        /* 824-872 */
        if (l4 + 8 > len) return skip;
        unsigned ul = be16(f, l4 + 4);
        if (ul < 8) return skip;                       /* 830 */
        if (l4 + ul > len) return skip;                /* 834-836 */
        f[l4 + 6] = 0;                                 /* 838 */
        f[l4 + 7] = 0;
        uint32_t sum;
        if (v4) {
            sum = sum_words(f + l2 + 12, 8) + 17 + ul;
        } else {
            sum = sum_words(f + l2 + 8, 32) + (ul >> 16) + (ul & 0xFFFF) + 17;
        }
        sum += sum_words(f + l4, ul);
        uint16_t c = finish(sum);
        store_be16(f, l4 + 6, c == 0 ? 0xFFFF : c);    /* 867-871 */
        return (v4 ? NFO_ST_V4_UDP : NFO_ST_V6_UDP) | ov;
    }
    if (proto == 1 && v4) {
        /* 873-889 */
        if (l4 + 8 > len) return skip;                 /* get_header<IcmpHeader>: 8 bytes */
        unsigned tl = be16(f, l2 + 2);
        if (tl < ihl4) return skip;                    /* 877 */
        size_t m = tl - ihl4;
        if (l4 + m > len) return skip;                 /* 880-882 */
        if (m < 8) return skip;                        /* 883 */
        f[l4 + 2] = 0;                                 /* 885 */
        f[l4 + 3] = 0;
        store_be16(f, l4 + 2, nfo_calculate_checksum(f + l4, m)); /* 886 */
        return NFO_ST_V4_ICMP | ov;
    }
    return (v4 ? NFO_ST_V4 : NFO_ST_V6) | ov;
}

/* Switch::process_received_packet, transit IPv4 (switch.hpp:247-294), restricted to the data
 * path: the control-plane steps (ACL, classification, is_my_ip, route + ARP lookup) are the
 * caller's and arrive as nh (NULL = no route / ARP miss). */
int nfo_l3_forward(uint8_t* f, size_t len, const uint8_t* nh) {
    if (len < 14) return NFO_ST_NOT_IPV4;            /* 248: ethernet() null -> L3 type 0 */
    unsigned l3t = be16(f, 12);                      /* 257 */
    size_t l2 = 14;
    if (l3t == 0x8100) {                             /* 259-262: one tag; vlan() null keeps 0x8100 */
        l2 = 18;                                     /* ethernet() set l2_header_size_ (packet.hpp:410) */
        if (len >= 18) l3t = be16(f, 16);
    }
    if (l3t != 0x0800) return NFO_ST_NOT_IPV4;       /* 265 */
    if (l2 + 20 > len) return NFO_ST_NOT_IPV4;       /* 266-267: ipv4() (packet.hpp:432-451) null */
    if (f[l2 + 8] <= 1) return NFO_ST_TTL_EXPIRED;   /* 278: ICMP time exceeded, drop */
    if (!nh) return NFO_ST_NO_ROUTE;                 /* 282-294: no route / ARP miss, drop */
    f[l2 + 8]--;                                     /* 279 */
    memcpy(f, nh, 12);                               /* 287-289: dst_mac, src_mac */
    return nfo_update(f, len) | NFO_ST_FLAG_FWD;     /* 290 */
}

int nfo_l3_forward_batch(uint8_t* arena, uint64_t arena_bytes, const nfo_desc* desc,
                         const uint32_t* nh_index, uint32_t n, const uint8_t* table,
                         uint32_t table_n, uint8_t* status) {
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t off = (uint64_t)desc[i].off16 * 16;
        int st;
        if (off + (((uint64_t)desc[i].len + 15) & ~15ull) > arena_bytes) {
            st = NFO_ST_BAD_DESC;
        } else {
            const uint8_t* nh = nh_index[i] < table_n ? table + (size_t)nh_index[i] * 12 : NULL;
            st = nfo_l3_forward(arena + off, desc[i].len, nh);
        }
        if (status) status[i] = (uint8_t)st;
    }
    return 0;
}

/* ---- VLAN push / pop + checksum -------------------------------------------- */
/* VlanHeader::set_vlan_id then set_priority (packet.hpp:185-190) on the TCI at bytes 14-15. */
static void set_tci(uint8_t* f, unsigned vid, unsigned prio) {
    unsigned tci = be16(f, 14);
    tci = (tci & 0xF000u) | (vid & 0x0FFFu);
    tci = (tci & 0x1FFFu) | ((prio & 7u) << 13);
    store_be16(f, 14, (uint16_t)tci);
}

/* Packet::push_vlan(vid, prio) (packet.hpp:655-692) and pop_vlan() (694-720) on a frame whose
 * buffer holds `cap` bytes from the frame start (the PacketBuffer's capacity minus headroom, so
 * tailroom = cap - len). Frame bytes past the new length are left as the reference's memmove
 * leaves them. */
int nfo_vlan(uint8_t* f, uint32_t* len_io, uint32_t cap, uint32_t op) {
    const uint32_t kind = op & NFO_VLAN_OP_MASK, vid = op & 0x0FFFu, prio = (op >> 13) & 7u;
    uint32_t len = *len_io;
    if (kind == NFO_VLAN_PUSH) {
        if (len < 14) return NFO_ST_VLAN_FAIL;                         /* 656 */
        if (be16(f, 12) == 0x8100) {                                   /* 661: has_vlan() */
            set_tci(f, vid, prio);                                     /* 662-664: no bounds check */
        } else {
            if (len + 4 > cap) return NFO_ST_VLAN_FAIL;                /* 666-670 (headroom 0) */
            memmove(f + 18, f + 14, len - 14);                         /* 673-676 */
            f[16] = f[12];                                             /* 681: inner = original */
            f[17] = f[13];
            f[14] = 0;                                                 /* 679: tci = 0 */
            f[15] = 0;
            set_tci(f, vid, prio);                                     /* 679-680 */
            f[12] = 0x81;                                              /* 683 */
            f[13] = 0x00;
            len += 4;                                                  /* 685 */
        }
    } else if (kind == NFO_VLAN_POP) {
        if (len < 14 || be16(f, 12) != 0x8100) return NFO_ST_VLAN_FAIL; /* 695 */
        if (len < 18) return NFO_ST_VLAN_FAIL;                          /* 698 */
        const uint8_t e0 = f[16], e1 = f[17];                           /* 703 */
        memmove(f + 14, f + 18, len - 18);                              /* 705-709 */
        f[12] = e0;                                                     /* 711 */
        f[13] = e1;
        len -= 4;                                                       /* 713 */
    } else {
        return NFO_ST_NONE;                                             /* no edit requested */
    }
    *len_io = len;
    return nfo_update(f, len) | NFO_ST_FLAG_VLAN;                       /* 690 / 718 */
}

int nfo_vlan_batch(uint8_t* arena, uint64_t arena_bytes, nfo_desc* desc, const uint32_t* ops,
                   uint32_t op_all, const uint32_t* caps, uint32_t cap_all, uint32_t n,
                   uint8_t* status) {
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t off = (uint64_t)desc[i].off16 * 16;
        uint32_t len = desc[i].len;
        const uint32_t op = ops ? ops[i] : op_all;
        const uint32_t kind = op & NFO_VLAN_OP_MASK;
        const uint64_t need = (uint64_t)len + (kind == NFO_VLAN_PUSH ? 4u : 0u);
        int st;
        if (off + ((need + 15) & ~15ull) > arena_bytes) {
            st = NFO_ST_BAD_DESC;
        } else {
            st = nfo_vlan(arena + off, &len, caps ? caps[i] : cap_all, op);
            desc[i].len = len;
        }
        if (status) status[i] = (uint8_t)st;
    }
    return 0;
}

/* ---- flow key ----------------------------------------------------------- */
static inline void put16le(uint8_t* p, unsigned v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
static inline void put32le(uint8_t* p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
static inline uint32_t be32(const uint8_t* f, size_t o) {
    return ((uint32_t)f[o] << 24) | ((uint32_t)f[o + 1] << 16) | ((uint32_t)f[o + 2] << 8) | f[o + 3];
}
static inline uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* extract_flow_key (packet_classifier.cpp:12-80) with the Packet accessors it calls:
 * ethernet()/src_mac()/dst_mac() need len >= 14; has_vlan()/vlan_id()/vlan() need the tag and
 * len >= 18 (get_header<VlanHeader>(14)); ipv4()/ipv6() need the effective EtherType and
 * l2 + 20 / l2 + 40 <= len (packet.hpp:432-470); tcp()/udp() need the IPv4 protocol / IPv6
 * next header and l4 + 19 (the 19-byte TcpHeader) / l4 + 8 <= len, l4 = l2 + IHL*4 or l2 + 40
 * (packet.hpp:473-535). hash_flow (82-108) XORs byte i of each MAC / IPv6 address at shift
 * (i % 4) * 8, i.e. the little-endian dwords. */
uint32_t nfo_flow_key(const uint8_t* f, size_t len, uint8_t* rec) {
    uint8_t src_mac[6] = {0}, dst_mac[6] = {0}, src6[16] = {0}, dst6[16] = {0};
    unsigned vlan = 0, et = 0, proto = 0, sp = 0, dp = 0;
    int is6 = 0;
    uint32_t sip = 0, dip = 0;
    size_t l2 = 14;
    if (len >= 14) {
        memcpy(dst_mac, f, 6);
        memcpy(src_mac, f + 6, 6);
        et = be16(f, 12);
        if (et == 0x8100) {
            l2 = 18;
            if (len >= 18) {
                vlan = be16(f, 14) & 0x0FFF;
                et = be16(f, 16);
            }
        }
    }
    if (et == 0x0800) {
        if (l2 + 20 <= len) {
            sip = be32(f, l2 + 12);
            dip = be32(f, l2 + 16);
            proto = f[l2 + 9];
            const size_t l4 = l2 + (size_t)(f[l2] & 15) * 4;
            if (proto == 6 && l4 + 19 <= len) { sp = be16(f, l4); dp = be16(f, l4 + 2); }
            if (proto == 17 && l4 + 8 <= len) { sp = be16(f, l4); dp = be16(f, l4 + 2); }
        }
    } else if (et == 0x86DD) {
        is6 = 1;
        if (l2 + 40 <= len) {
            memcpy(src6, f + l2 + 8, 16);
            memcpy(dst6, f + l2 + 24, 16);
            proto = f[l2 + 6];
            const size_t l4 = l2 + 40;
            if (proto == 6 && l4 + 19 <= len) { sp = be16(f, l4); dp = be16(f, l4 + 2); }
            if (proto == 17 && l4 + 8 <= len) { sp = be16(f, l4); dp = be16(f, l4 + 2); }
        }
    }
    uint32_t h = 0;
    for (int i = 0; i < 6; ++i) {
        h ^= (uint32_t)src_mac[i] << (i % 4 * 8);
        h ^= (uint32_t)dst_mac[i] << (i % 4 * 8);
    }
    h ^= vlan;
    h ^= (uint32_t)et << 16;
    if (is6) {
        for (int i = 0; i < 16; ++i) {
            h ^= (uint32_t)src6[i] << ((i % 4) * 8);
            h ^= (uint32_t)dst6[i] << ((i % 4) * 8);
        }
    } else {
        h ^= sip;
        h ^= dip;
    }
    h ^= proto;
    h ^= (uint32_t)sp << 16;
    h ^= dp;
    if (rec) {
        memset(rec, 0, 64);
        put32le(rec, h);
        put16le(rec + 4, vlan);
        put16le(rec + 6, et);
        memcpy(rec + 8, src_mac, 6);
        memcpy(rec + 14, dst_mac, 6);
        rec[20] = (uint8_t)proto;
        rec[21] = (uint8_t)is6;
        put16le(rec + 22, sp);
        put16le(rec + 24, dp);
        if (is6) {
            memcpy(rec + 32, src6, 16);
            memcpy(rec + 48, dst6, 16);
        } else {
            put32le(rec + 32, sip);
            put32le(rec + 48, dip);
        }
    }
    (void)le32;
    return h;
}

void nfo_flow_keys_batch(const uint8_t* arena, uint64_t arena_bytes, const nfo_desc* desc,
                         uint32_t n, uint8_t* recs, uint32_t* hashes) {
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t off = (uint64_t)desc[i].off16 * 16;
        uint8_t* r = recs ? recs + (size_t)i * 64 : NULL;
        uint32_t h = 0;
        if (off + (((uint64_t)desc[i].len + 15) & ~15ull) <= arena_bytes) {
            h = nfo_flow_key(arena + off, desc[i].len, r);
        } else if (r) {
            memset(r, 0, 64);
        }
        if (hashes) hashes[i] = h;
    }
}

/* result word as documented in nfcs.h: (ipv4 csum << 16) | l4 csum, 0 where not written */
static uint32_t result_word(const uint8_t* f, size_t len, int st) {
    int base = st & 0x3F;
    if (base == NFO_ST_NONE || base == NFO_ST_V6 || base == NFO_ST_V6_L4SKIP || base >= NFO_ST_OOB)
        return 0;
    size_t l2 = (len >= 14 && be16(f, 12) == 0x8100) ? 18 : 14;
    uint32_t ip = 0, l4c = 0;
    size_t l4 = 0;
    if (base <= NFO_ST_V4_L4SKIP) {
        ip = be16(f, l2 + 10);
        l4 = l2 + (size_t)(f[l2] & 15) * 4;
    } else {
        l4 = l2 + 40;
    }
    switch (base) {
    case NFO_ST_V4_TCP: case NFO_ST_V6_TCP: l4c = be16(f, l4 + 15); break;
    case NFO_ST_V4_UDP: case NFO_ST_V6_UDP: l4c = be16(f, l4 + 6); break;
    case NFO_ST_V4_ICMP: l4c = be16(f, l4 + 2); break;
    default: break;
    }
    return (ip << 16) | l4c;
}

typedef struct {
    uint8_t* arena;
    uint64_t arena_bytes;
    const nfo_desc* desc;
    uint8_t* status;
    uint32_t* result;
    uint32_t lo, hi;
} batch_job;

static void* batch_worker(void* p) {
    batch_job* j = (batch_job*)p;
    for (uint32_t i = j->lo; i < j->hi; ++i) {
        uint64_t off = (uint64_t)j->desc[i].off16 * 16;
        uint32_t len = j->desc[i].len;
        int st;
        uint32_t r = 0;
        if (off + (((uint64_t)len + 15) & ~15ULL) > j->arena_bytes) {
            st = NFO_ST_BAD_DESC;
        } else {
            st = nfo_update(j->arena + off, len);
            if (j->result) r = result_word(j->arena + off, len, st);
        }
        if (j->status) j->status[i] = (uint8_t)st;
        if (j->result) j->result[i] = r;
    }
    return NULL;
}

int nfo_update_batch(uint8_t* arena, uint64_t arena_bytes, const nfo_desc* desc, uint32_t n,
                     uint8_t* status, uint32_t* result, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
    batch_job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (batch_job){arena, arena_bytes, desc, status, result,
                              (uint32_t)((uint64_t)n * t / nthreads),
                              (uint32_t)((uint64_t)n * (t + 1) / nthreads)};
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    batch_worker(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

/* ---- synthetic configs --------------------------------------------------- */

uint64_t nfo_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline uint64_t pkt_key(uint64_t seed, uint64_t index) { return nfo_mix64(seed ^ (index * GOLDEN)); }
static inline uint64_t draw(uint64_t key, uint64_t k) { return nfo_mix64(key + k * GOLDEN); }

uint32_t nfo_config_len(int config, uint64_t seed, uint64_t index) {
    switch (config) {
    case 0: return 64;
    case 1: return 1500;
    case 2: return 9000;
    case 3: return 64 + (uint32_t)(draw(pkt_key(seed, index), 1) % 1437);
    default: return 0;
    }
}

void nfo_config_frame(int config, uint64_t seed, uint64_t index, uint8_t* f) {
    const uint64_t key = pkt_key(seed, index);
    const uint32_t len = nfo_config_len(config, seed, index);
    unsigned proto = config == 0 ? 253 : config == 1 ? 17 : config == 2 ? 6
                   : ((draw(key, 2) & 1) ? 6 : 17);
    /* random fill: byte o = byte (o % 8) of draw(key, 16 + o / 8), little-endian */
    for (uint32_t o = 0; o < len; o += 8) {
        uint64_t r = draw(key, 16 + o / 8);
        for (uint32_t b = 0; b < 8 && o + b < len; ++b) f[o + b] = (uint8_t)(r >> (8 * b));
    }
    f[12] = 0x08; f[13] = 0x00;                 /* EtherType IPv4, untagged */
    f[14] = 0x45; f[15] = 0x00;                 /* version 4, IHL 5 */
    store_be16(f, 16, (uint16_t)(len - 14));    /* total_length */
    f[22] = 64;                                 /* TTL */
    f[23] = (uint8_t)proto;
    store_be16(f, 24, (uint16_t)((draw(key, 3) & 0xFFFF) | 0x0101)); /* stale, nonzero */
    if (proto == 17) {
        store_be16(f, 38, (uint16_t)(len - 34));                        /* udp.length */
        store_be16(f, 40, (uint16_t)((draw(key, 4) & 0xFFFF) | 0x0101));
    } else if (proto == 6) {
        f[46] = 0x50;                                                   /* data offset 5 */
        store_be16(f, 49, (uint16_t)((draw(key, 4) & 0xFFFF) | 0x0101)); /* field @ l4+15 */
    }
}

uint64_t nfo_layout_config(int config, uint64_t seed, uint64_t first, uint32_t n, uint32_t align,
                           nfo_desc* desc) {
    if (align < 16) align = 16;
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t len = nfo_config_len(config, seed, first + i);
        if (desc) {
            desc[i].off16 = (uint32_t)(off >> 4);
            desc[i].len = len;
        }
        off += ((uint64_t)len + align - 1) / align * align;
    }
    return off;
}

void nfo_gen_config(int config, uint64_t seed, uint64_t first, uint32_t n, uint8_t* arena,
                    const nfo_desc* desc) {
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t* f = arena + (uint64_t)desc[i].off16 * 16;
        nfo_config_frame(config, seed, first + i, f);
        uint32_t len = desc[i].len, pad = ((len + 15) & ~15u) - len;
        memset(f + len, 0, pad);
    }
}

/* ---- fuzz corpus ------------------------------------------------------------------------ */

typedef struct { uint64_t s; } rng_t;
static inline uint64_t rnext(rng_t* r) { r->s += GOLDEN; return nfo_mix64(r->s); }
static inline uint32_t rint_(rng_t* r, uint32_t n) { return (uint32_t)(rnext(r) % n); }

uint32_t nfo_fuzz_frame(uint64_t seed, uint64_t index, uint8_t* f) {
    rng_t r = {nfo_mix64(seed ^ (index * GOLDEN) ^ 0xF022F022F022F022ULL)};
    uint32_t len, u = rint_(&r, 100);
    if (u < 3) len = rint_(&r, 80);              /* short / runt frames, 0..79 */
    else if (u < 8) len = 9000 - rint_(&r, 8);   /* jumbo */
    else len = 14 + rint_(&r, 1600);
    for (uint32_t o = 0; o < len; ++o) f[o] = (uint8_t)rnext(&r);
    if (len < 14) return len;

    size_t l2 = 14;
    if (rint_(&r, 4) == 0) { f[12] = 0x81; f[13] = 0x00; l2 = 18; }
    uint32_t kind = rint_(&r, 100);
    if (kind < 62) {
        /* IPv4 (EtherType usually 0x0800; sometimes something else: the nibble decides) */
        if (l2 + 2 <= len) {
            if (rint_(&r, 10) != 0) { f[l2 - 2] = 0x08; f[l2 - 1] = 0x00; }
        }
        if (l2 + 20 > len) return len;
        uint32_t ihl, iu = rint_(&r, 100);
        if (iu < 82) ihl = 5;
        else if (iu < 94) ihl = 6 + rint_(&r, 10);
        else ihl = rint_(&r, 5);
        f[l2] = (uint8_t)(0x40 | ihl);
        uint32_t pu = rint_(&r, 100);
        unsigned proto = pu < 34 ? 6 : pu < 68 ? 17 : pu < 84 ? 1 : (unsigned)(rnext(&r) & 0xFF);
        f[l2 + 9] = (uint8_t)proto;
        size_t ihl4 = ihl * 4, l4 = l2 + ihl4;
        if (l2 + ihl4 > len) return len; /* OOB case stays in the corpus (status OOB) */
        /* total length: consistent, or off */
        uint32_t tl = (uint32_t)(len - l2);
        uint32_t tu = rint_(&r, 12);
        if (tu == 0) tl = (uint32_t)(rnext(&r) & 0xFFFF);
        else if (tu == 1) tl = tl - rint_(&r, 16);
        else if (tu == 2) tl = tl + 1 + rint_(&r, 8);
        else if (tu == 3) tl = (uint32_t)ihl4 + rint_(&r, 12);
        tl &= 0xFFFF;
        store_be16(f, l2 + 2, (uint16_t)tl);
        if (proto == 6 && l4 + 13 <= len) {
            f[l4 + 12] = rint_(&r, 5) ? 0x50 : (uint8_t)rnext(&r);
        } else if (proto == 17 && l4 + 6 <= len) {
            uint32_t ul = (uint32_t)(len - l4), uu = rint_(&r, 10);
            if (uu == 0) ul = (uint32_t)(rnext(&r) & 0xFFFF);
            else if (uu == 1) ul = rint_(&r, 12);
            else if (uu == 2) ul = ul - rint_(&r, (uint32_t)(ul < 40 ? ul + 1 : 40));
            else if (uu == 3) ul = ul + 1;
            store_be16(f, l4 + 4, (uint16_t)ul);
        } else if (proto == 1 && l4 + 4 <= len && rint_(&r, 6) == 0) {
            /* all-zero ICMP message sometimes (exact-zero sum -> 0xFFFF) */
            size_t m = tl >= ihl4 ? tl - ihl4 : 0;
            for (size_t k = 0; k < m && l4 + k < len; ++k) f[l4 + k] = 0;
        }
        /* sometimes truncate after building the headers */
        if (rint_(&r, 10) == 0) len -= rint_(&r, (uint32_t)(len - l2 < 64 ? len - l2 : 64) + 1);
        return len;
    } else if (kind < 84) {
        /* IPv6 */
        if (l2 + 2 <= len) { f[l2 - 2] = 0x86; f[l2 - 1] = 0xDD; }
        if (l2 + 40 > len) return len;
        f[l2] = (uint8_t)((rint_(&r, 10) ? 0x60 : (rnext(&r) & 0xF0)) | (f[l2] & 0x0F));
        uint32_t pu = rint_(&r, 100);
        unsigned nh = pu < 42 ? 6 : pu < 84 ? 17 : pu < 92 ? 1 : (unsigned)(rnext(&r) & 0xFF);
        f[l2 + 6] = (uint8_t)nh;
        size_t l4 = l2 + 40;
        uint32_t pl = (uint32_t)(len - l4), pv = rint_(&r, 10);
        if (pv == 0) pl = (uint32_t)(rnext(&r) & 0xFFFF);
        else if (pv == 1) pl = pl + 1 + rint_(&r, 4);
        store_be16(f, l2 + 4, (uint16_t)pl);
        if (nh == 6 && l4 + 13 <= len) f[l4 + 12] = rint_(&r, 5) ? 0x50 : (uint8_t)rnext(&r);
        if (nh == 17 && l4 + 6 <= len) {
            uint32_t ul = (uint32_t)(len - l4);
            if (rint_(&r, 8) == 0) ul = (uint32_t)(rnext(&r) & 0xFFFF);
            store_be16(f, l4 + 4, (uint16_t)ul);
        }
        if (rint_(&r, 10) == 0) len -= rint_(&r, (uint32_t)(len - l2 < 64 ? len - l2 : 64) + 1);
        return len;
    }
    /* anything else: random EtherType, random bytes (version nibble may still say 4/6) */
    return len;
}

/* ---- digests ------------------------------------------------------------------------------ */

static inline uint64_t ld64(const uint8_t* p, uint32_t avail) {
    uint64_t v = 0;
    for (uint32_t b = 0; b < 8 && b < avail; ++b) v |= (uint64_t)p[b] << (8 * b);
    return v;
}

uint64_t nfo_frame_hash(const uint8_t* f, uint32_t len) {
    uint64_t acc = 0;
    for (uint32_t c = 0; c * 16 < len; ++c) {
        uint32_t o = c * 16;
        uint64_t lo = ld64(f + o, len - o);
        uint64_t hi = (o + 8 < len) ? ld64(f + o + 8, len - o - 8) : 0;
        acc += nfo_mix64(lo ^ nfo_mix64(hi + (uint64_t)(c + 1) * GOLDEN));
    }
    return nfo_mix64((uint64_t)len * 0xD6E8FEB86659FD93ULL + acc);
}

static inline uint64_t digest_term(uint64_t h, uint64_t index) {
    return nfo_mix64(h ^ (index * 0xA0761D6478BD642FULL));
}

uint64_t nfo_digest(const uint8_t* arena, const nfo_desc* desc, uint32_t n, uint64_t first) {
    uint64_t d = 0;
    for (uint32_t i = 0; i < n; ++i)
        d += digest_term(nfo_frame_hash(arena + (uint64_t)desc[i].off16 * 16, desc[i].len), first + i);
    return d;
}

typedef struct {
    int config;
    uint64_t seed, lo, hi;
    uint64_t din, dout;
    uint64_t hist[256];
} cfg_job;

static void* cfg_worker(void* p) {
    cfg_job* j = (cfg_job*)p;
    uint8_t* buf = (uint8_t*)malloc(9024);
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        uint32_t len = nfo_config_len(j->config, j->seed, i);
        nfo_config_frame(j->config, j->seed, i, buf);
        j->din += digest_term(nfo_frame_hash(buf, len), i);
        int st = nfo_update(buf, len);
        j->hist[st & 0xFF]++;
        j->dout += digest_term(nfo_frame_hash(buf, len), i);
    }
    free(buf);
    return NULL;
}

void nfo_config_digest(int config, uint64_t seed, uint64_t first, uint64_t n, int nthreads,
                       uint64_t* digest_in, uint64_t* digest_out, uint64_t* status_hist) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 128) nthreads = 128;
    cfg_job* jobs = (cfg_job*)calloc((size_t)nthreads, sizeof(cfg_job));
    pthread_t th[128];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].config = config;
        jobs[t].seed = seed;
        jobs[t].lo = first + n * t / nthreads;
        jobs[t].hi = first + n * (t + 1) / nthreads;
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, cfg_worker, &jobs[t]);
    cfg_worker(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    uint64_t din = 0, dout = 0;
    for (int t = 0; t < nthreads; ++t) {
        din += jobs[t].din;
        dout += jobs[t].dout;
        if (status_hist)
            for (int s = 0; s < 256; ++s) status_hist[s] += jobs[t].hist[s];
    }
    if (digest_in) *digest_in = din;
    if (digest_out) *digest_out = dout;
    free(jobs);
}
