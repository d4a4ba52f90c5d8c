/*
 * nfcs_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of NetFlow++'s Packet::update_checksums() (packet.hpp:722-912) used as the
 * parity checker for the HIP engine. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (netflow_amd / libnfcs.so) never links it.
 *
 * Parity pinning: this restatement is checked against the reference itself — the
 * reference header compiled from /root/reference by oracle/Makefile into oracle/_ref/ —
 * on the Appendix-B known-answer frames and on a fuzz corpus; the committed fixtures in
 * tests/golden/ were produced by the compiled reference (tests/golden/make_golden.py).
 */
#ifndef NFCS_ORACLE_H
#define NFCS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: identical values to include/nfcs.h NFCS_ST_* (checked by tests) */
enum {
    NFO_ST_NONE = 0, NFO_ST_V4 = 1, NFO_ST_V4_TCP = 2, NFO_ST_V4_UDP = 3, NFO_ST_V4_ICMP = 4,
    NFO_ST_V4_L4SKIP = 5, NFO_ST_V6 = 6, NFO_ST_V6_TCP = 7, NFO_ST_V6_UDP = 8,
    NFO_ST_V6_L4SKIP = 9, NFO_ST_NO_ROUTE = 11, NFO_ST_NOT_IPV4 = 12, NFO_ST_TTL_EXPIRED = 13,
    NFO_ST_OOB = 14, NFO_ST_BAD_DESC = 15, NFO_ST_VLAN_FAIL = 16, NFO_ST_FLAG_VLAN = 0x20,
    NFO_ST_FLAG_OVERLAP = 0x40, NFO_ST_FLAG_FWD = 0x80
};

/* VLAN edit word (identical to include/nfcs.h NFCS_VLAN_*): op | prio << 13 | vid */
#define NFO_VLAN_PUSH 0x40000000u
#define NFO_VLAN_POP 0x80000000u
#define NFO_VLAN_OP_MASK 0xC0000000u

typedef struct nfo_desc { uint32_t off16; uint32_t len; } nfo_desc;

/* one frame, in place; returns the status byte */
int nfo_update(uint8_t* frame, size_t len);
/* Packet::calculate_checksum (packet.hpp:894-912): returns the 16-bit value that the
 * reference stores big-endian (i.e. ntohs of the stored field) */
uint16_t nfo_calculate_checksum(const uint8_t* data, size_t len);
/* batch over an arena; status may be NULL; returns 0 */
int nfo_update_batch(uint8_t* arena, uint64_t arena_bytes, const nfo_desc* desc, uint32_t n,
                     uint8_t* status, uint32_t* result, int nthreads);

/* Transit-IPv4 L3 forward of one frame as Switch::process_received_packet does it
 * (switch.hpp:247-294): L3 EtherType after one tag, ipv4() present, TTL <= 1 -> dropped,
 * TTL--, destination/source MAC rewrite, update_checksums(). nh = 12 bytes {dst[6], src[6]}
 * of the resolved next hop, or NULL when the route / ARP lookup failed. Frames that are not
 * forwarded are left untouched. Returns NFO_ST_NOT_IPV4 / TTL_EXPIRED / NO_ROUTE, or the
 * update_checksums() status | NFO_ST_FLAG_FWD. */
int nfo_l3_forward(uint8_t* frame, size_t len, const uint8_t* nh);
/* batch: next hop of packet i = table[nh_index[i]] (12 bytes each), none if >= table_n */
int nfo_l3_forward_batch(uint8_t* arena, uint64_t arena_bytes, const nfo_desc* desc,
                         const uint32_t* nh_index, uint32_t n, const uint8_t* table,
                         uint32_t table_n, uint8_t* status);

/* Packet::push_vlan(vid, prio) / pop_vlan() (packet.hpp:655-720) + their update_checksums()
 * on one frame whose buffer holds cap bytes from the frame start. op = NFO_VLAN_PUSH | prio << 13
 * | vid, NFO_VLAN_POP, or 0 (no edit). *len is updated. Returns NFO_ST_VLAN_FAIL when the
 * reference returns false (frame untouched), NFO_ST_NONE for no edit, else the
 * update_checksums() status | NFO_ST_FLAG_VLAN. The buffer must hold max(len + 4, 16) bytes. */
int nfo_vlan(uint8_t* frame, uint32_t* len, uint32_t cap, uint32_t op);
/* batch (the nfcs_vlan_device contract): op / cap of frame i = ops[i] / caps[i], or op_all /
 * cap_all when the array is NULL; desc[i].len updated in place */
int nfo_vlan_batch(uint8_t* arena, uint64_t arena_bytes, nfo_desc* desc, const uint32_t* ops,
                   uint32_t op_all, const uint32_t* caps, uint32_t cap_all, uint32_t n,
                   uint8_t* status);

/* PacketClassifier::extract_flow_key + hash_flow (packet_classifier.cpp:12-108) of one frame,
 * written as the 64-byte nfcs_flow_key record of include/nfcs.h; returns the hash. */
uint32_t nfo_flow_key(const uint8_t* frame, size_t len, uint8_t* rec /* 64 bytes */);
void nfo_flow_keys_batch(const uint8_t* arena, uint64_t arena_bytes, const nfo_desc* desc,
                         uint32_t n, uint8_t* recs /* n x 64, may be NULL */, uint32_t* hashes);

/* synthetic configs (spec in DESIGN.md §6) */
uint32_t nfo_config_len(int config, uint64_t seed, uint64_t index);
void nfo_config_frame(int config, uint64_t seed, uint64_t index, uint8_t* out /* >= len */);
uint64_t nfo_layout_config(int config, uint64_t seed, uint64_t first, uint32_t n, uint32_t align,
                           nfo_desc* desc);
void nfo_gen_config(int config, uint64_t seed, uint64_t first, uint32_t n, uint8_t* arena,
                    const nfo_desc* desc);

/* fuzz corpus frames (edge cases: VLAN, IHL 0-15, IPv6, ICMP, truncation, bad lengths,
 * odd lengths, jumbo). Returns len (<= 9000); out must hold 9016 bytes. */
uint32_t nfo_fuzz_frame(uint64_t seed, uint64_t index, uint8_t* out);

/* digests (order-independent) */
uint64_t nfo_mix64(uint64_t z);
uint64_t nfo_frame_hash(const uint8_t* frame, uint32_t len);
uint64_t nfo_digest(const uint8_t* arena, const nfo_desc* desc, uint32_t n, uint64_t first);
/* streaming: generate packets [first, first+n) of a config, digest them before and after
 * nfo_update, count statuses; multi-threaded; O(1) memory per thread */
void nfo_config_digest(int config, uint64_t seed, uint64_t first, uint64_t n, int nthreads,
                       uint64_t* digest_in, uint64_t* digest_out, uint64_t* status_hist /*[256]*/);

#ifdef __cplusplus
}
#endif
#endif
