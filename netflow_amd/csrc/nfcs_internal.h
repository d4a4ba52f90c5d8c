// nfcs_internal.h — shared between the HIP kernels (nfcs_kernels.hip) and the C-ABI /
// context code (nfcs_api.hip). Not installed; the public boundary is include/nfcs.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nfcs.h"

namespace nfcs {

// Workgroup geometry: 256-thread blocks = 4 waves of 64 lanes.
constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

// per-device properties cached in the context
struct DevInfo {
    int device = 0;
    int cus = 256;
    char arch[64] = {0};
};

// Forms of launch_update (how the checksum bytes reach the frames; nfcs_kernels.hip SF_*):
enum : int {
    kUpdateAuto = 0,     // per wave from its frame lengths: inline stores, or patch records and a
                         // non-temporal write pass (needs patch or ws: n records)
    kUpdateRecords = 1,  // patch records only, frames untouched (needs patch)
    kUpdateInline = 2    // every wave stores inline (the zero-copy host path: frames over PCIe)
};

// In the long shape (mean footprint >= kSmallMeanBytes) a wave whose four frames average at least
// this many bytes defers its checksum stores to the write pass (kUpdateAuto); the short and tiny
// shapes store every wave inline (round 3: no write pass for them, launch_update_one). Uniform-length sweeps (round 2, tools/exp/len_sweep.sh in git b164560^; 1M frames, DESIGN.md
// §5e): at 1024 B inline stores win (0.661 vs 0.635), at 1280 B deferral wins (replayed 0.782 vs
// 0.768, fresh 0.760 vs 0.624), at 1500 B too (0.759 / 0.745 vs 0.757 / 0.653). Short frames' reads
// are latency-bound and hide the inline stores; a mixed batch like C3 (U{64..1500}) lost 3.5% when
// its waves of mean >= 1024 B (12%) deferred, and defers < 1% of its waves at 1280.
constexpr uint32_t kDeferMeanBytes = 1280;
// kUpdateAuto on a burst of at most this many packets stores every wave inline from one kernel:
// the write pass's launch (~3 µs) outweighs what deferral saves on so few packets (burst sweep,
// round 2, tools/exp/ab.py c<k>n<N> in git b164560^; DESIGN.md §5e: 1K-64K C1 packets 13-35% faster, 64K C3 16%; 64K C2
// jumbo frames 5% slower; 128K C1 even). The packet count alone decides: the arena size never
// changes the form.
constexpr uint32_t kInlineMaxPackets = 65536;
// update_checksums() reads and tests against data_len no offset past 65,613 (nfcs.h)
constexpr uint32_t kFrameRelevantBytes = NFCS_FRAME_RELEVANT_BYTES;
// kUpdateAuto on long frames processes a batch of more than kSubBatchAbovePackets as sub-batches
// of kSubBatchPackets (read pass, then write pass, per sub-batch): 512K header lines (64 MB,
// 128 MB when frames straddle lines) stay in the 256 MB memory-side cache between the two passes.
// On the 4M shard 512K and 1M sub-batches measured alike (0.749-0.755 / 0.749 against 0.683-0.714
// in one launch), 2M 0.710. Round 4, calls rotating over fresh batches (the steady state): C1 as two
// 512K sub-batches 0.2591-0.2604 ms per call against 0.2596-0.2669 in one launch pair on two boxes
// (rocprofv3: 2 x (116.8 + 13.1) against 231.0 + 30.0 us), and on the boxes where C1 in one pair ran
// 2-3% below the 4M shard's 512K sub-batches in the same run, those held their rate: so every batch
// above 512K long-frame packets is split (profiles/r04_s2_c1_sub_batches.jsonl).
constexpr uint32_t kSubBatchPackets = 1u << 19;
constexpr uint32_t kSubBatchAbovePackets = 1u << 19;
// The fused L3 forward on long frames defers its stores (read pass writing 8-byte forward records,
// then apply_fwd_kernel per kSubBatchPackets sub-batch) for bursts of more than this many packets;
// smaller bursts store their segments inline from one kernel. Round 4: in the steady state (calls
// rotating over fresh batches) the inline write-through segments cost 1M-packet C1 bursts as much as
// the update's inline stores do.
constexpr uint32_t kFwdDeferAbovePackets = kInlineMaxPackets;
// Below this mean arena footprint per packet the checksum kernel runs the short shape (16-lane rows,
// frame-relative windows, buffer loads, 7 waves/SIMD); the shape changes speed only, never the
// store form.
constexpr uint64_t kSmallMeanBytes = 1200;
// Below this one it runs 8-lane rows, 8 packets per wave (short frames are packet-rate bound:
// uniform 64-256 B frames 1.8-1.9x, IMIX 7:4:1 of 64/570/1500 B 1.47x, 768 B 1.2x; the C3 mix,
// 870 B of footprint per packet, stays on 16-lane rows, where 8-lane rows lose 7.5%).
constexpr uint64_t kTinyMeanBytes = 800;
// One row pass of those 8-lane rows (6 slots of 8 x 16 bytes); a wave with a longer frame makes a
// second one. So a mix whose mean alone says 8-lane rows but whose frames often exceed this (C3's
// U{64..1500} packed at 16-byte starts: 782 B of footprint, half the frames longer) runs 16-lane rows
// once its footprint sample (sample_footprint) finds more than kTinyLongMax of 256 sampled frames
// longer than this: round 6, packed C3 0.787-0.818 ms per call in 8-lane rows against 0.655 in the
// 16-lane short shape (profiles/r06_c3_packed_shapes.jsonl). A wave of 8 frames of which a fraction
// p is long continues with probability 1 - (1 - p)^8; with a continued 8-lane wave costing about
// 1.2x two 16-lane waves (the packed C3 figures) and an uncontinued one 0.6x, they break even near
// p = 1/8 (32 of 256): IMIX 7:4:1 (64/570/1500 B, p = 1/12) stays on 8-lane rows. The model holds
// only where the short frames are not packet-rate bound themselves: the round-6 shape audit
// (tools/r06/shape_audit.py, profiles/r06_y_shape_audit_threshold.jsonl) found 64-byte frames mixed
// with 20-40% of 1024- or 1500-byte ones 4-27% faster in 8-lane rows, U{64..1000} and 64/1500 mixes
// from 35% long frames 1-16% faster in 16-lane rows; the mean footprint splits them: below
// kTinyMixMeanBytes a mix stays on 8-lane rows whatever its long frames.
constexpr uint32_t kTinyRowBytes = 768;
constexpr uint32_t kTinyLongMax = 32;
constexpr uint64_t kTinyMixMeanBytes = 512;
// A burst inside a larger ring whose sample finds frames of one length (rounded to 128 bytes), each
// starting on a line, with a footprint between kTinyMeanBytes and kSmallMeanBytes runs 8-lane rows
// rather than the short shape (nfcs_api.hip peek_shape; the update and the forward, not VLAN): round 6
// audit, 832-1216-byte frames in 2 KiB ring slots 11-16% faster (update) and 8-13% (forward), in 4 KiB
// slots within 3% either way (profiles/r06_y_shape_audit_threshold.jsonl, r06_an_fwd_threshold.jsonl).
// Packed layouts of such frames: the update does not sample them (their estimate is exact) and keeps the
// short shape, where 8-lane rows measured -5% to +11% depending on the batch; the forward samples them
// and takes its 8-lane rows of 6 slots (uniform 896-1152-byte frames packed on their lines -0.5% to +12%
// against its short-mix rows; 832-byte frames at alternating 64-byte offsets, whose sample finds them off
// their lines, 13% slower there and keep the short-mix rows).
// The footprint sample's 32-bit word (sample_footprint; the burst's generation in the other 32 bits).
constexpr uint32_t kObsPresent = 0x80000000u;
constexpr uint32_t kObsLongShift = 20;  // bits 20-28: sampled frames longer than kTinyRowBytes (0-256)
constexpr uint32_t kObsMeanMask = 0x1FFFFu;  // bits 0-16: the mean of the lengths rounded up to 128
// bits 17-19: how many sampled frames have a rounded length above 128 and at most 1408 bytes (neither
// minimum-size nor full-size), in 32s, at most 7; a mix with fewer than kObsMidMin8 such 32s is
// bimodal (64 / 1500-byte traffic). The fused forward keeps such mixes on 8-lane rows of 6 slots at any
// mean below kTinyMeanBytes: round 6 audit, 64/1500 mixes with 35-50% full-size frames packed at 16-byte
// starts 24-34% faster there than in its 12-slot short-mix rows, at 128-byte starts within 3%; U{64..hi}
// mixes and packed C3, whose frames fill the middle, keep the short-mix rows (1-14% faster in them;
// profiles/r06_an_fwd_threshold.jsonl, r06_y_shape_audit_l3fwd.jsonl).
constexpr uint32_t kObsMidShift = 17;
constexpr uint32_t kObsMidMin8 = 2;
// bit 29: more than kObsUnalignedMax of the sampled frames start off a 128-byte line (they share lines
// with their neighbours); bit 30: the sampled lengths, rounded up to 128, span more than 128 bytes
constexpr uint32_t kObsUnaligned = 1u << 29;
constexpr uint32_t kObsMixed = 1u << 30;
constexpr uint32_t kObsUnalignedMax = 32;
// VLAN push/pop below this mean footprint writes its frames write-through (`sc1`), at or above it
// past the caches (`sc0 sc1 nt`): 1M frames in 128-byte slots 177 vs 181 µs, in 384 / 640-byte
// slots 212-216 vs 208 / 258 vs 245 µs, C1 0.698-0.704 vs 0.728-0.731. In 8-lane
// rows that holds only for frames of one length starting on lines: a sample that finds frames off
// their lines or lengths that vary (kObsUnaligned / kObsMixed) writes write-through at any mean below
// kTinyMeanBytes — round 6 shape audit (profiles/r06_ak_vlan_audit2.jsonl): packed 384-768-byte frames
// 14-43% faster write-through, IMIX 15-31%, 64/1500 mixes 28-47%; uniform 384-640-byte frames at
// 128-byte starts 1-21% faster past the caches.
constexpr uint64_t kVlanWtMeanBytes = 256;
// VLAN's kTinyMixMeanBytes: its write-through 8-lane rows keep mixes with many long frames up to a higher
// mean than the checksum kernel's (same audit: U{64..1000} and 64/1500 with 30% long frames, 540-550 B,
// 17-24% faster in them than in 16-lane rows; 64/1500 half and half and packed C3, 782-784 B, 16-22%
// slower).
constexpr uint64_t kVlanMixMeanBytes = 640;
// Dynamic LDS per 256-thread checksum workgroup (unused): 5 workgroups = 5 waves/SIMD per CU.
constexpr unsigned kRowsLdsPad = 30720;
// The same for 6 workgroups = 6 waves/SIMD: the forward's deferred read pass, the stream-read forms.
constexpr unsigned kRowsLdsPad6 = 24576;

// The mean arena bytes per packet that pick a launch shape (speed only): the context's slot-size
// hint (nfcs_ctx_set_slot_bytes) when set, else arena_bytes / n.
inline uint64_t shape_mean(uint64_t arena_bytes, uint32_t n, uint64_t slot_bytes) {
    return slot_bytes ? slot_bytes : arena_bytes / n;
}

// A footprint observation request (sample_footprint in nfcs_kernels.hip, for the next call's launch
// shape): the host-mapped 64-bit slot the launch writes its sample to (null: none) and its tag — the
// burst's generation in the high 32 bits (written back with the sample, so a late sample of an
// earlier burst is told apart) and in the low 32 the packets to sample over: the whole call's n,
// also when the call runs as sub-batches (the first one samples for all).
struct ObsReq {
    uint64_t* slot = nullptr;
    uint64_t tag = 0;
};

// A completion request (round 6, the host path's small chunks): every workgroup counts itself in *ctr
// (device memory) once its stores have been released at system scope; the one that brings the count to
// base + gridDim.x (base: the count before this launch, which the host tracks) stores that count into
// *flag (host-mapped) with a system-scope release, and the host spins on *flag instead of waiting for the
// stream's event. The count only grows, so a flag above base means this launch is done, and no reset
// (no extra launch) is needed between launches. Only for launches of kUpdateRecords / kUpdateInline (one
// kernel per call). flag null: none.
struct DoneReq {
    uint64_t* flag = nullptr;
    uint64_t* ctr = nullptr;
    uint64_t base = 0;
};

hipError_t launch_update(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes,
                         const nfcs_desc* desc, uint32_t n, uint32_t base16, uint8_t* status,
                         nfcs_patch* patch, nfcs_patch* ws, int form, hipStream_t stream,
                         uint64_t slot_bytes = 0, ObsReq obs = {}, DoneReq done = {});

hipError_t launch_l3_forward(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes,
                             const nfcs_desc* desc, const uint32_t* nh, uint32_t n,
                             const nfcs_nexthop* table, uint32_t table_n, uint8_t* status,
                             nfcs_patch* ws, hipStream_t stream, uint64_t slot_bytes = 0,
                             ObsReq obs = {});

hipError_t launch_vlan(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes, nfcs_desc* desc,
                       uint32_t n, const uint32_t* ops, uint32_t op_all, const uint32_t* caps,
                       uint32_t cap_all, uint8_t* status, hipStream_t stream, uint64_t slot_bytes = 0,
                       ObsReq obs = {}, uint32_t sample_bits = 0);

hipError_t launch_flow_keys(const DevInfo& di, const uint8_t* arena, uint64_t arena_bytes,
                            const nfcs_desc* desc, uint32_t n, nfcs_flow_key* keys,
                            uint32_t* hashes, hipStream_t stream);

hipError_t launch_gen_config(const DevInfo& di, int config, uint64_t seed, uint64_t first,
                             uint32_t n, uint8_t* arena, uint64_t arena_bytes,
                             const nfcs_desc* desc, hipStream_t stream);

hipError_t launch_digest(const DevInfo& di, const uint8_t* arena, uint64_t arena_bytes,
                         const nfcs_desc* desc, uint32_t n, uint64_t first, uint64_t* d_out,
                         hipStream_t stream);

hipError_t launch_stream_read(const uint8_t* buf, uint64_t bytes, int form, unsigned long long* sink,
                              hipStream_t stream);

hipError_t launch_frames_read(const uint8_t* arena, uint64_t arena_bytes, const nfcs_desc* desc, uint32_t n,
                              unsigned long long* sink, hipStream_t stream);

// host-side synthetic layout (same spec as the device generator)
uint32_t config_len(int config, uint64_t seed, uint64_t index);

}  // namespace nfcs
