// nfcs_exp.hip — measurement translation unit (not product). Built with nfcs_api.hip into
// tools/exp/libnfcs_exp.so by tools/exp/build.sh; the product library never contains it.
//
// It compiles the product kernels (the text of netflow_amd/csrc/nfcs_kernels.hip) and adds
// launch forms that the product does not ship, so A/B runs time the product's own templates with
// other shapes, store forms or occupancy caps. One C entry times `iters` launches of a variant with
// HIP events on the given stream:
//   variant 0   the product (kUpdateAuto)
//           1   every wave inline (SF_INLINE, 256-thread workgroups) — the round-1 fused form
//           2   every wave inline, one-wave workgroups at 7 waves/SIMD (round-1 short-frame form)
//           3   SF_DEFER in one-wave workgroups whatever the footprint
//           4   SF_DEFER in 256-thread workgroups whatever the footprint
//           5   the read pass only, records for every packet (SF_RECORDS) — no frame writes
// lds_pad: dynamic LDS bytes per workgroup, to cap the waves per SIMD (occupancy sweeps).
#include "../../netflow_amd/csrc/nfcs_kernels.hip"

namespace nfcs {

static hipError_t exp_launch(int variant, uint8_t* arena, uint64_t arena_bytes, const nfcs_desc* desc,
                             uint32_t n, nfcs_patch* ws, unsigned lds_pad, hipStream_t st) {
    const FwdArgs nofwd = {nullptr, nullptr, 0};
    const dim3 g1((n + 3u) / 4u), g4((n + 15u) / 16u);
    const dim3 ga((n + kBlock - 1) / kBlock);
#define NFCS_X(OCC, BS, G, SF)                                                                     \
    hipLaunchKernelGGL((update_rows_kernel<6, 16, OCC, BS, false, SF>), G, dim3(BS), lds_pad, st, \
                       arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws, nofwd)
    switch (variant) {
    case 0: return launch_update(DevInfo{}, arena, arena_bytes, desc, n, 0u, nullptr, nullptr, ws,
                                 kUpdateAuto, st);
    case 1: NFCS_X(1, kBlock, g4, SF_INLINE); break;
    case 2: NFCS_X(7, 64, g1, SF_INLINE); break;
    case 3:
        NFCS_X(7, 64, g1, SF_DEFER);
        hipLaunchKernelGGL(apply_bytes_kernel, ga, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    case 4:
        NFCS_X(1, kBlock, g4, SF_DEFER);
        hipLaunchKernelGGL(apply_bytes_kernel, ga, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    case 5:
        hipLaunchKernelGGL((update_rows_kernel<6, 16, 1, kBlock, false, SF_RECORDS>), g4, dim3(kBlock),
                           lds_pad, st, arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, ws,
                           (nfcs_patch*)nullptr, nofwd);
        break;
    default: return hipErrorInvalidValue;
    }
#undef NFCS_X
    return hipGetLastError();
}

}  // namespace nfcs

// ws: n device records (the deferred-store workspace). Returns 0 or the hipError_t.
extern "C" NFCS_API int nfcs_exp_time_update(int variant, uint8_t* d_arena, uint64_t arena_bytes,
                                            const nfcs_desc* d_desc, uint32_t n, nfcs_patch* ws,
                                            unsigned lds_pad, int iters, void* stream, float* ms) {
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1;
    hipError_t e = hipEventRecord(e0, st);
    for (int it = 0; it < iters && e == hipSuccess; ++it)
        e = nfcs::exp_launch(variant, d_arena, arena_bytes, d_desc, n, ws, lds_pad, st);
    if (e == hipSuccess) e = hipEventRecord(e1, st);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return (int)e;
}
