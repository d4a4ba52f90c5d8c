// nfcs_internal.h — shared between the HIP kernels (nfcs_kernels.hip) and the C-ABI /
// context code (nfcs_api.hip). Not installed; the public boundary is include/nfcs.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nfcs.h"

namespace nfcs {

// Launch geometry of the checksum kernel: 256-thread blocks = 4 waves; one wave owns one
// packet at a time (grid-stride over packets), with the next packet's first batch in flight.
constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

struct LaunchCfg {
    int grid;    // blocks
    int variant; // kernel variant (see nfcs_kernels.hip)
};

// per-device properties cached in the context
struct DevInfo {
    int device = 0;
    int cus = 256;
    char arch[64] = {0};
    // measurement knob (env NFCS_LDS_PAD): dynamic LDS bytes per workgroup, which caps the
    // workgroups per CU and so the waves per SIMD; 0 in production
    unsigned lds_pad = 0;
};

// Per-context device workspace handed to the checksum launch.
struct Work {
    nfcs_patch* patch = nullptr;  // split mode: patch records of the checksum pass
};

hipError_t launch_update(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes,
                         const nfcs_desc* desc, uint32_t n, uint32_t base16, uint8_t* status,
                         nfcs_patch* patch, hipStream_t stream, int variant, int grid,
                         const Work& work);

// Split mode (checksum pass without frame stores, then a patch-apply pass) beats the fused
// kernel once frames are large: a store in the middle of a long read stream costs more than
// the same store in its own pass. The default variant picks it when the mean
// arena footprint per packet is at least kSplitMeanBytes.
constexpr uint64_t kSplitMeanBytes = 2048;
// Below this mean footprint per packet the default kernel runs in one-wave workgroups: short
// frames make short-lived waves, and single-wave workgroups retire and relaunch them with less
// granularity loss (C3 +2-3%, profiles/r01_s2_variants.md run bs1/bs2).
constexpr uint64_t kSmallMeanBytes = 1200;
// At or above this arena size the C1-form kernel stores its checksum bytes write-back instead
// of write-through: over a batch too large to stay partly cached between launches (the C4
// shard, 6.3 GB) write-back measured 0.657 vs 0.632; re-processing a 1.5 GB batch, write-through
// 0.765 vs 0.743 (profiles/r01_s4_batch_footprint.jsonl).
constexpr uint64_t kWriteBackArenaBytes = 2ull << 30;
inline bool use_split(int variant, uint64_t arena_bytes, uint32_t n) {
    return variant == 8 || (variant >= 9 && variant <= 14) || variant == 22 ||
           variant == 23 ||  // 9-14, 22, 23: experiments build only
           (variant == 0 && n > 0 && arena_bytes / n >= kSplitMeanBytes);
}
// variants that stage patch records in a context workspace (split mode)
inline bool variant_needs_ws(int variant, uint64_t arena_bytes, uint32_t n) {
    return use_split(variant, arena_bytes, n);
}

hipError_t launch_l3_forward(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes,
                             const nfcs_desc* desc, const uint32_t* nh, uint32_t n,
                             const nfcs_nexthop* table, uint32_t table_n, uint8_t* status,
                             hipStream_t stream, int grid, int variant = 0);

hipError_t launch_vlan(const DevInfo& di, uint8_t* arena, uint64_t arena_bytes, nfcs_desc* desc,
                       uint32_t n, const uint32_t* ops, uint32_t op_all, const uint32_t* caps,
                       uint32_t cap_all, uint8_t* status, hipStream_t stream, int variant = 0);

hipError_t launch_flow_keys(const DevInfo& di, const uint8_t* arena, uint64_t arena_bytes,
                            const nfcs_desc* desc, uint32_t n, nfcs_flow_key* keys,
                            uint32_t* hashes, hipStream_t stream, int variant = 0);

hipError_t launch_gen_config(const DevInfo& di, int config, uint64_t seed, uint64_t first,
                             uint32_t n, uint8_t* arena, uint64_t arena_bytes,
                             const nfcs_desc* desc, hipStream_t stream);

hipError_t launch_digest(const DevInfo& di, const uint8_t* arena, uint64_t arena_bytes,
                         const nfcs_desc* desc, uint32_t n, uint64_t first, uint64_t* d_out,
                         hipStream_t stream);

// host-side synthetic layout (same spec as the device generator)
uint32_t config_len(int config, uint64_t seed, uint64_t index);

}  // namespace nfcs
