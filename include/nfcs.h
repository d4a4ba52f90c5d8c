/*
 * nfcs.h — C ABI of the MI355X batched Internet-checksum engine.
 *
 * This is the drop-in boundary for NetFlow++'s checksum path:
 *
 *   netflow::Packet::update_checksums()      include/netflow++/packet.hpp:722-890
 *   netflow::Packet::calculate_checksum()    include/netflow++/packet.hpp:894-912
 *
 * The reference exposes the path as a non-virtual inline C++ member that works on ONE
 * packet in a PacketBuffer (packet_buffer.hpp:10-111). This ABI exposes the same
 * computation over a BATCH of frames laid out in one arena (device or pinned host memory)
 * and described by 8-byte descriptors. Every function returns an int status (0 = OK,
 * < 0 = error; see nfcs_strerror) and never throws across the ABI. Per-packet results are
 * written in place into the frames exactly as the reference writes them (bit-exact,
 * including its quirks — SURVEY.md Appendix A), plus an optional per-packet status byte
 * that records which branch of update_checksums() ran (the reference returns void and
 * silently skips malformed packets: packet.hpp:758,763,780,784,786,791-793,830,834-836).
 *
 * No torch / HIP types appear in the signatures: streams are passed as void* (a
 * hipStream_t, or NULL for the context's own stream).
 */
#ifndef NFCS_H
#define NFCS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define NFCS_API __attribute__((visibility("default")))
#else
#define NFCS_API
#endif

/* ABI versions: 1 = rounds 1-4; 2 = round 5 on: nfcs_update_host_frames, and nfcs_update_host accepts
 * descriptors in any order (an ABI-1 library returns NFCS_EINVAL for a burst that is not one ascending
 * run). A caller that needs either checks nfcs_abi_version() >= 2. */
#define NFCS_ABI_VERSION 2

/* ---- data layout ------------------------------------------------------------------ */

/* One frame inside an arena: bytes arena[off16*16, off16*16 + len).
 * Replaces PacketBuffer's data window [get_data_start_ptr(), +get_data_length())
 * (packet_buffer.hpp:51-52). Frames start on 16-byte boundaries; the arena must cover
 * off16*16 + round_up(len, 16) bytes for every descriptor (the kernel reads whole 16-byte
 * chunks; a descriptor outside the arena is rejected per packet with NFCS_ST_BAD_DESC).
 * Frames of one batch must not overlap (as separate PacketBuffers never do): the kernels may
 * rewrite a frame's own 16-byte chunks whole, with the values they read from them. */
typedef struct nfcs_desc {
    uint32_t off16; /* frame start, in 16-byte units from the arena base */
    uint32_t len;   /* frame length in bytes (PacketBuffer::data_len_)     */
} nfcs_desc;

/* What update_checksums() wrote into one frame: at most two 2-byte fields. Applying
 * ip then l4 to the original frame reproduces the updated frame exactly (also when the two
 * fields overlap, IHL < 5). Offsets are frame offsets; 0xFFFF = field not written. */
typedef struct nfcs_patch {
    uint16_t ip_off;  /* IPv4 header checksum field: l2 + 10                         */
    uint16_t l4_off;  /* L4 checksum field: TCP l4+15 (sic), UDP l4+6, ICMP l4+2     */
    uint8_t ip[2];    /* bytes written at ip_off (big-endian checksum)               */
    uint8_t l4[2];    /* bytes written at l4_off                                     */
} nfcs_patch;

#define NFCS_PATCH_NONE 0xFFFFu

/* ---- per-packet status (which branch of update_checksums() ran) -------------------- */
enum {
    NFCS_ST_NONE = 0,       /* neither IPv4 (by version nibble) nor IPv6: untouched (packet.hpp:761-765) */
    NFCS_ST_V4 = 1,         /* IPv4 header checksum written; protocol not TCP/UDP/ICMP              */
    NFCS_ST_V4_TCP = 2,     /* IPv4 header + TCP checksum (TCP field at l4+15, packet.hpp:258-270)  */
    NFCS_ST_V4_UDP = 3,     /* IPv4 header + UDP checksum                                            */
    NFCS_ST_V4_ICMP = 4,    /* IPv4 header + ICMP checksum                                           */
    NFCS_ST_V4_L4SKIP = 5,  /* IPv4 header written; TCP/UDP/ICMP branch returned early (bounds)    */
    NFCS_ST_V6 = 6,         /* IPv6 detected, next header neither TCP nor UDP: untouched            */
    NFCS_ST_V6_TCP = 7,     /* IPv6 TCP checksum                                                     */
    NFCS_ST_V6_UDP = 8,     /* IPv6 UDP checksum                                                     */
    NFCS_ST_V6_L4SKIP = 9,  /* IPv6 TCP/UDP branch returned early (bounds): untouched                */
    /* nfcs_l3_forward_device only (switch.hpp:247-294); such frames are left untouched:    */
    NFCS_ST_NO_ROUTE = 11,  /* next-hop index >= table size: no route / ARP miss (282-294)       */
    NFCS_ST_NOT_IPV4 = 12,  /* L3 EtherType (after one tag) not IPv4, or ipv4() absent (265-267) */
    NFCS_ST_TTL_EXPIRED = 13, /* TTL <= 1: the switch sends ICMP time exceeded and drops (278)   */
    NFCS_ST_OOB = 14,       /* IPv4 with l2 + IHL*4 > len: the reference reads past the frame (UB);
                               outside the parity domain, frame left untouched                      */
    NFCS_ST_BAD_DESC = 15,  /* descriptor reaches past arena_bytes: frame not touched                */
    NFCS_ST_VLAN_FAIL = 16, /* nfcs_vlan_device: push_vlan / pop_vlan returned false (no tag to pop,
                               runt frame, no tailroom): frame and length untouched                 */
    NFCS_ST_FLAG_VLAN = 0x20, /* OR-ed in by nfcs_vlan_device: the tag was pushed / re-written /
                                 popped, then the update_checksums() status in the low bits      */
    NFCS_ST_FLAG_OVERLAP = 0x40, /* OR-ed in: IPv4 IHL < 5 with TCP/UDP/ICMP, so the L4 region
                                   overlaps the IPv4 header; handled by the exact sequential path */
    NFCS_ST_FLAG_FWD = 0x80     /* OR-ed in by nfcs_l3_forward_device: TTL decremented, MACs
                                   rewritten, then the update_checksums() status in the low bits */
};

/* ---- error codes -------------------------------------------------------------------- */
enum {
    NFCS_OK = 0,
    NFCS_EINVAL = -1,   /* bad argument (null pointer with n > 0, misaligned arena, ...) */
    NFCS_EHIP = -2,     /* a HIP runtime call failed; nfcs_last_hip_error() has the code  */
    NFCS_ENOMEM = -3,   /* allocation failed                                              */
    NFCS_ENODEV = -4    /* no such device / no gfx950 device                              */
};

/* Synthetic workload configurations (BASELINE.json "configs"). */
enum {
    NFCS_CFG_C0_64B_V4 = 0,   /* 64 B IPv4, protocol 253 (header checksum only)   */
    NFCS_CFG_C1_1500B_UDP = 1,/* 1500 B IPv4 + UDP                                 */
    NFCS_CFG_C2_9000B_TCP = 2,/* 9000 B IPv4 + TCP                                 */
    NFCS_CFG_C3_MIXED = 3     /* U{64..1500} B, 50/50 IPv4 TCP/UDP                 */
};

typedef struct nfcs_ctx nfcs_ctx;

/* ---- library / context ---------------------------------------------------------------- */
NFCS_API int nfcs_abi_version(void);
NFCS_API const char* nfcs_strerror(int err);
NFCS_API int nfcs_last_hip_error(void);

/* Threads: any entry point may be called from any host thread; it makes the context's device
 * current for its duration and restores the caller's device on return. Calls on ONE context are
 * serialised by the caller (or ordered by a stream); different contexts run concurrently
 * (netflow_amd::MultiGpu, include/netflow_amd/multi_gpu.hpp: one thread per GPU). */

/* One context per device: owns a stream, events and the pinned staging ring used by
 * nfcs_update_host. Calls on one context must be serialised by the caller. */
NFCS_API int nfcs_ctx_create(int device, nfcs_ctx** out);
NFCS_API int nfcs_ctx_destroy(nfcs_ctx* ctx);
NFCS_API void* nfcs_ctx_stream(nfcs_ctx* ctx); /* the context's own hipStream_t */
/* Launch shapes (speed only; the bytes written never depend on them) follow the mean footprint per
 * packet: 8-lane rows for short frames, 16-lane rows for long ones, long-frame sub-batches. Without
 * a hint it is arena_bytes / n, which is exact for a batch that fills its arena and otherwise only
 * over-estimates; when that estimate says "long" or "8-lane rows", the update, the L3 forward and
 * VLAN also sample the frames on the device (256 descriptors, one wave, no host sync: the mean of their
 * lengths rounded up to 128 and how many exceed one 8-lane row pass), and the next call over the same
 * burst (descriptor array, n and arena_bytes) launches in the shape the sample calls for — a burst
 * inside a larger ring (a NIC ring reusing its descriptor array) adapts after one call,
 * and so does a densely packed mix of short and long frames (§5e). A caller may
 * instead state its frames' mean slot size, e.g. 128 for 64-byte frames in 128-byte slots; 0 (the
 * default) restores the automatic choice. Applies to the device-path calls that follow on ctx
 * (update, L3 forward, VLAN; nfcs_update_host measures each staged chunk itself). */
NFCS_API int nfcs_ctx_set_slot_bytes(nfcs_ctx* ctx, uint32_t bytes);
/* The mean footprint per packet (bytes) that the next device-path call on ctx over this burst
 * (d_arena of arena_bytes, d_desc, n) picks its launch shape from: the slot-size hint, arena_bytes / n,
 * or the footprint the previous call over the same burst sampled (once that call has finished).
 * No side effect; speed only (the bytes written never depend on it). */
NFCS_API int nfcs_ctx_launch_footprint(nfcs_ctx* ctx, uint64_t arena_bytes, const nfcs_desc* d_desc,
                                       uint32_t n, uint64_t* mean);
/* The host staging ring of nfcs_update_host (allocated by this call if not yet): *node = the GPU's
 * NUMA node (-1 if unknown), *local = 1 when the ring's pinned memory is bound to that node (its
 * copy threads then run on that node's CPUs). SURVEY.md §8e: one GPU per host thread, staging
 * NUMA-local to each GPU. */
NFCS_API int nfcs_ctx_host_numa(nfcs_ctx* ctx, int* node, int* local);

/* ---- the hot path --------------------------------------------------------------------- */

/* Batched Packet::update_checksums() on device-resident frames (packet.hpp:722-890).
 *   d_arena      device pointer, 16-byte aligned, frames mutated in place
 *   arena_bytes  size of the arena in bytes (descriptors are checked against it)
 *   d_desc       n device-resident descriptors
 *   d_status     optional (NULL) n status bytes, NFCS_ST_*
 *   d_patch      optional (NULL) n nfcs_patch records describing the bytes written
 *   stream       hipStream_t or NULL (context stream). Asynchronous: completion is
 *                observed by synchronising the stream.
 * Launches (speed only; the bytes written never depend on them): a call of at most 65,536
 * packets is one kernel; waves of long frames write their checksum bytes in a second, write-only
 * pass; a long-frame call of more than 1M packets runs as consecutive 512K-packet sub-batches. */
NFCS_API int nfcs_update_device(nfcs_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes,
                                const nfcs_desc* d_desc, uint32_t n, uint8_t* d_status,
                                nfcs_patch* d_patch, void* stream);

/* Same on host memory (NIC / socket buffers). Synchronous. Descriptors may come in any order;
 * each run of ascending offsets is staged as a contiguous span (a NIC ring burst that wraps past
 * the ring's end is two runs; ABI 1 required one ascending run). Frames go H2D in
 * chunks on two streams (from a pageable arena through the context's pinned ring, copied by host
 * threads; a pinned arena — nfcs_host_alloc — is copied from directly), the kernel runs per
 * chunk, and only the 8-byte nfcs_patch records come back and are applied on the host. A frame
 * inside the arena longer than NFCS_FRAME_RELEVANT_BYTES is staged as its first
 * NFCS_FRAME_RELEVANT_BYTES bytes, with the same result (see nfcs_update_host_frames); before round 6
 * a frame larger than one 64 MiB staging slot was NFCS_EINVAL. Pinned bursts of up to 32 MiB run
 * zero-copy (below).
 * flags:
 *   NFCS_HOST_FRAMES     copy whole frames back instead of patch records (same bytes, slower;
 *                        each chunk's span goes back whole, so bytes between the burst's frames
 *                        are rewritten with the values read: not for a ring whose other slots
 *                        are being filled meanwhile — the default writes only checksum bytes)
 *   NFCS_HOST_ZERO_COPY  pinned arenas only: the kernel reads the frames over PCIe in place and
 *                        writes the checksum bytes straight back (no staging copies); the default
 *                        form for pinned bursts of up to 32 MiB (round 6: one launch, no DMA)
 *   NFCS_HOST_PATCH_ONLY the default since ABI 1 session 2; accepted and ignored
 * Rates: DESIGN.md §7. */
/* A pinned burst whose frames (its runs of ascending offsets, gaps included) span at most this many bytes
 * runs zero-copy unless NFCS_HOST_FRAMES is given (round 6): one kernel launch and no DMA, the kernel
 * reading only the frames' own bytes; larger bursts go through the copy engines. */
#define NFCS_HOST_ZERO_COPY_AUTO_BYTES (32u << 20)
#define NFCS_HOST_PATCH_ONLY 1u
#define NFCS_HOST_ZERO_COPY 2u
#define NFCS_HOST_FRAMES 4u
NFCS_API int nfcs_update_host(nfcs_ctx* ctx, uint8_t* h_arena, uint64_t arena_bytes,
                              const nfcs_desc* h_desc, uint32_t n, uint8_t* h_status,
                              uint32_t flags);

/* Batched Packet::update_checksums() over n frames scattered in host memory, one pointer each —
 * the form a NetFlow++ caller holds them in: frames[i] / lens[i] = the i-th packet's
 * PacketBuffer::get_data_start_ptr() / get_data_length() (packet_buffer.hpp:21-31, 51-52: one
 * `new[]` per buffer, BufferPool::allocate_buffer, buffer_pool.hpp:57-94). Synchronous. The frames
 * are gathered in chunks (16-byte aligned, back to back) into the context's NUMA-local pinned ring
 * by its copy threads, moved H2D, checksummed on the GPU in the records-only form, and the 2+2
 * checksum bytes written back into each frame in place (ip field first, then l4, the reference's
 * write order); the gather, the transfers, the kernel and the write-back of successive chunks
 * overlap on two streams. Only the bytes the reference writes are written. frames[i] == NULL or
 * lens[i] == 0: nothing read or written, status NFCS_ST_NONE. A frame longer than
 * NFCS_FRAME_RELEVANT_BYTES is processed as its first NFCS_FRAME_RELEVANT_BYTES bytes, with the same
 * result: update_checksums() reads, and compares with data_len, no offset past 65,613 (l2 18 + IHL 60
 * + a 16-bit length; packet.hpp:728-889), so any longer length passes each of its bounds tests alike
 * (ABI 2 as first shipped returned NFCS_EINVAL above 64 MiB). Frames must not overlap.
 *   h_status  optional (NULL) n status bytes, NFCS_ST_*
 *   flags     0 (reserved) */
#define NFCS_FRAME_RELEVANT_BYTES 131072u
NFCS_API int nfcs_update_host_frames(nfcs_ctx* ctx, uint8_t* const* frames, const uint32_t* lens, uint32_t n,
                                     uint8_t* h_status, uint32_t flags);

/* ---- fused L3 forward ------------------------------------------------- */

/* One next hop: the MACs Switch::process_received_packet writes (switch.hpp:286-289). */
typedef struct nfcs_nexthop {
    uint8_t dst_mac[6]; /* ARP-resolved next-hop MAC (arp_processor_.lookup_mac)      */
    uint8_t src_mac[6]; /* egress interface MAC (interface_manager_.get_interface_mac) */
} nfcs_nexthop;
#define NFCS_NH_NONE 0xFFFFFFFFu

/* Batched data path of the switch's transit-IPv4 forward (switch.hpp:247-294) in one HBM read pass:
 * for packet i with L3 EtherType IPv4 and an IPv4 header, TTL <= 1 -> NFCS_ST_TTL_EXPIRED;
 * d_nh[i] >= table_n -> NFCS_ST_NO_ROUTE; else TTL--, dst/src MAC = d_table[d_nh[i]], then
 * Packet::update_checksums(), status = its status | NFCS_ST_FLAG_FWD. Frames that are not
 * forwarded are untouched. The control-plane steps (ACL, classification, is_my_ip, route and
 * ARP lookup) stay with the caller and arrive as next-hop indexes.
 *   d_nh     n device-resident u32 next-hop indexes (NFCS_NH_NONE = no route)
 *   d_table  table_n device-resident next hops
 * Launches (speed only): one kernel; a burst of more than 1M long frames runs as 512K-packet
 * sub-batches whose long-frame waves write their header rewrites in a second pass.
 * Asynchronous on the stream; d_nh and d_table must stay valid until it completes. */
NFCS_API int nfcs_l3_forward_device(nfcs_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes,
                                    const nfcs_desc* d_desc, const uint32_t* d_nh, uint32_t n,
                                    const nfcs_nexthop* d_table, uint32_t table_n,
                                    uint8_t* d_status, void* stream);

/* ---- VLAN push / pop + checksum ---------------------------------------- */

/* One VLAN edit per packet as a u32: the operation in bits 30-31, the priority in bits 13-15
 * and the VLAN id in bits 0-11 (the arguments of Packet::push_vlan, masked as
 * VlanHeader::set_vlan_id / set_priority mask them, packet.hpp:185-190). */
#define NFCS_VLAN_NOP 0x00000000u
#define NFCS_VLAN_PUSH 0x40000000u /* Packet::push_vlan(vid, prio)  packet.hpp:655-692 */
#define NFCS_VLAN_POP 0x80000000u  /* Packet::pop_vlan()            packet.hpp:694-720 */
#define NFCS_VLAN_OP_MASK 0xC0000000u
#define NFCS_VLAN_PUSH_OP(vid, prio) \
    (NFCS_VLAN_PUSH | (((uint32_t)(prio) & 7u) << 13) | ((uint32_t)(vid) & 0xFFFu))

/* Batched Packet::push_vlan / pop_vlan, each followed by the update_checksums() it ends with, on
 * device-resident frames in one HBM pass (VlanManager::process_ingress / process_egress call
 * them per packet, vlan_manager.cpp:90,159,174). Per packet i with edit op_i (d_ops[i], or
 * op_all when d_ops is NULL) and buffer capacity cap_i (d_caps[i], or cap_all; the bytes the
 * frame's buffer holds from the frame start, i.e. PacketBuffer capacity minus headroom):
 *   push, frame already tagged   -> TCI id/priority rewritten in place (DEI kept), checksums
 *   push, untagged, len+4 <= cap -> bytes [14, len) move up by 4, 0x8100 + TCI inserted at 12,
 *                                   len += 4, checksums
 *   pop, tagged and len >= 18    -> bytes [18, len) move down by 4, inner EtherType at 12,
 *                                   len -= 4, checksums
 *   anything else                -> untouched: NFCS_ST_VLAN_FAIL (the reference returns false)
 *                                   or NFCS_ST_NONE (NFCS_VLAN_NOP).
 * d_desc[i].len is updated in place. Frame bytes past the new length keep the values the
 * reference's memmove leaves. A push needs the 16-byte chunks up to len + 4 inside the arena
 * (else NFCS_ST_BAD_DESC) and cap_i must not reach into another frame.
 *   d_status  optional (NULL) n status bytes: NFCS_ST_FLAG_VLAN | update_checksums() status,
 *             NFCS_ST_VLAN_FAIL, NFCS_ST_NONE or NFCS_ST_BAD_DESC */
NFCS_API int nfcs_vlan_device(nfcs_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes,
                              nfcs_desc* d_desc, uint32_t n, const uint32_t* d_ops,
                              uint32_t op_all, const uint32_t* d_caps, uint32_t cap_all,
                              uint8_t* d_status, void* stream);

/* ---- flow-key extract + hash -------------------------------------------- */

/* PacketClassifier::FlowKey + hash_flow (packet_classifier.hpp:15-56, packet_classifier.cpp:12-108)
 * as one 64-byte record per packet. Integers little-endian in host order (the reference stores
 * ntohs/ntohl values); an IPv4 address is the host-order u32 key.src_ip/dst_ip in bytes 0-3 of
 * its 16-byte field (the rest zero), an IPv6 address its 16 bytes. */
typedef struct nfcs_flow_key {
    uint32_t hash;        /* PacketClassifier::hash_flow(key)                          */
    uint16_t vlan_id;     /* key.vlan_id (TCI & 0xFFF of the first tag, 0 if none)      */
    uint16_t ethertype;   /* key.ethertype (inner EtherType after one tag)             */
    uint8_t src_mac[6];
    uint8_t dst_mac[6];
    uint8_t protocol;     /* IPv4 protocol / IPv6 next header                          */
    uint8_t is_ipv6;
    uint16_t src_port;
    uint16_t dst_port;
    uint8_t reserved[6];  /* zero */
    uint8_t src_ip[16];
    uint8_t dst_ip[16];
} nfcs_flow_key;

/* Batched PacketClassifier::extract_flow_key + hash_flow over device-resident frames (read
 * only: the first 128 bytes of each frame at most). d_keys (n records) and d_hash (n u32) are
 * each optional; a descriptor outside the arena yields a zero record and hash 0. */
NFCS_API int nfcs_flow_keys_device(nfcs_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes,
                                   const nfcs_desc* d_desc, uint32_t n, nfcs_flow_key* d_keys,
                                   uint32_t* d_hash, void* stream);

/* ---- multi-GPU partition ----------------------------------------------- */

/* Split a batch into `parts` contiguous packet ranges balanced by frame bytes: part p owns packets
 * [bounds[p], bounds[p+1]) (bounds has parts + 1 entries, bounds[0] = 0, bounds[parts] = n), and
 * its frame bytes (sum of len) differ from total / parts by less than one frame. Packets are
 * independent (packet.hpp:722-890 reads only its own frame), so each part goes to its own GPU with
 * its own context and no collective. Pure host code. */
NFCS_API int nfcs_shard_bytes(const nfcs_desc* h_desc, uint32_t n, uint32_t parts, uint32_t* bounds);

/* ---- synthetic batches and digests (bench / parity support; not on the hot path) ------ */

/* Lay out n frames of a config (packet indices first_index .. first_index+n-1), frame starts
 * aligned to `align` bytes (a multiple of 16: 16 packs frames densely, 64 matches NIC
 * buffer rings); fills h_desc (may be NULL) and returns the arena bytes needed through
 * *arena_bytes. Pure host code. */
NFCS_API int nfcs_layout_config(int config, uint64_t seed, uint64_t first_index, uint32_t n,
                                uint32_t align, nfcs_desc* h_desc, uint64_t* arena_bytes);

/* Fill the frames of a laid-out config batch on the device (d_desc from nfcs_layout_config);
 * the whole arena is zeroed first, so padding between aligned frames is defined. */
NFCS_API int nfcs_gen_config_device(nfcs_ctx* ctx, int config, uint64_t seed,
                                    uint64_t first_index, uint32_t n, uint8_t* d_arena,
                                    uint64_t arena_bytes, const nfcs_desc* d_desc, void* stream);

/* Order-independent 64-bit digest of the n frames (packet index first_index + i):
 *   digest = sum_i mix64(frame_hash(frame_i) ^ ((first_index + i) * 0xA0761D6478BD642F))
 * (DESIGN.md §6 gives frame_hash). Synchronous; result in *h_digest. */
NFCS_API int nfcs_digest_device(nfcs_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes,
                                const nfcs_desc* d_desc, uint32_t n, uint64_t first_index,
                                uint64_t* h_digest, void* stream);

/* ---- memory helpers for callers without their own HIP runtime ------------------------- */
NFCS_API int nfcs_device_alloc(nfcs_ctx* ctx, size_t bytes, void** out);
NFCS_API int nfcs_device_free(nfcs_ctx* ctx, void* p);
NFCS_API int nfcs_host_alloc(nfcs_ctx* ctx, size_t bytes, void** out); /* pinned */
NFCS_API int nfcs_host_free(nfcs_ctx* ctx, void* p);
NFCS_API int nfcs_memcpy_h2d(nfcs_ctx* ctx, void* dst, const void* src, size_t bytes);
NFCS_API int nfcs_memcpy_d2h(nfcs_ctx* ctx, void* dst, const void* src, size_t bytes);
NFCS_API int nfcs_stream_sync(nfcs_ctx* ctx, void* stream);

/* ---- timing (bench support): HIP events on the given stream ---------------------------- */
/* Time `iters` back-to-back nfcs_update_device launches on `stream` with HIP events recorded
 * on that same stream; returns total milliseconds in *ms. */
NFCS_API int nfcs_time_update_device(nfcs_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes,
                                     const nfcs_desc* d_desc, uint32_t n, uint8_t* d_status,
                                     int iters, void* stream, float* ms);
/* The steady state of a NIC ring: `iters` back-to-back nfcs_update_device calls rotating over
 * `batches` separate batches (call i runs batch i % batches: d_arenas[b], arena_bytes[b],
 * d_descs[b], n packets each), so no call re-processes the frames the previous call wrote; HIP
 * events on `stream` around all of them. Total milliseconds in *ms. */
NFCS_API int nfcs_time_update_batches(nfcs_ctx* ctx, uint32_t batches, uint8_t* const* d_arenas,
                                      const uint64_t* arena_bytes, const nfcs_desc* const* d_descs,
                                      uint32_t n, int iters, void* stream, float* ms);
/* Same for nfcs_flow_keys_device. */
NFCS_API int nfcs_time_flow_keys_device(nfcs_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes,
                                        const nfcs_desc* d_desc, uint32_t n, nfcs_flow_key* d_keys,
                                        uint32_t* d_hash, int iters, void* stream, float* ms);
/* Same for nfcs_l3_forward_device (after the first launch every TTL has been decremented
 * again, so repeated launches keep forwarding until TTLs reach 1: the bench restores them). */
NFCS_API int nfcs_time_l3_forward_device(nfcs_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes,
                                         const nfcs_desc* d_desc, const uint32_t* d_nh,
                                         uint32_t n, const nfcs_nexthop* d_table, uint32_t table_n,
                                         uint8_t* d_status, int iters, void* stream, float* ms);

/* The read-stream reference the bench compares its kernels with: `iters` pure
 * non-temporal reads of the first `bytes` (16-byte multiple, 16-byte aligned) of d_buf, nothing
 * written; form 0 = the checksum read pass's shape and load policies (6 KiB per wave, 6 loads in
 * flight, XCD-aware order, the first load default-policy and the rest non-temporal), 1 = 512
 * workgroups striding with 4 non-temporal loads per lane in flight, 2 = form 0 with every load
 * non-temporal, 3 / 4 / 5 = 8 / 16 / 4 non-temporal loads per lane (8 / 16 / 4 KiB per wave) with
 * no occupancy cap. Total milliseconds in *ms. */
NFCS_API int nfcs_time_stream_read(nfcs_ctx* ctx, const uint8_t* d_buf, uint64_t bytes, int form,
                                   int iters, void* stream, float* ms);
/* The read-only floor of the checksum read pass's own access pattern: `iters` launches that read the
 * n frames of d_desc in d_arena exactly as nfcs_update_device's read pass does (16-lane rows, 6
 * slots, the same load policies, order and occupancy), computing and writing nothing. Total
 * milliseconds in *ms. */
NFCS_API int nfcs_time_frames_read(nfcs_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes,
                                   const nfcs_desc* d_desc, uint32_t n, int iters, void* stream, float* ms);
/* Same for nfcs_vlan_device with a uniform edit: launches alternate between op_all (even
 * iterations) and op_alt (odd), so a push / pop pair leaves every frame as it was. */
NFCS_API int nfcs_time_vlan_device(nfcs_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes,
                                   nfcs_desc* d_desc, uint32_t n, uint32_t op_all,
                                   uint32_t op_alt, uint32_t cap_all, uint8_t* d_status, int iters,
                                   void* stream, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* NFCS_H */
