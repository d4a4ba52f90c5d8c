// fwd_bound.hip — round-6 measurement translation unit (not product). Built with nfcs_api.hip into
// tools/r06/libnfcs_fwdb.so by tools/r06/build_fwdb.sh; the product library never contains it.
//
// the bound of the fused L3 forward on BASELINE C3's mix, as DESIGN.md §5c bounds the
// update's C3. The product runs that mix in its short-mix shape (update_rows_kernel<12, 8, 6, 256, true,
// SF_INLINE, 1, 12>: 8-lane rows of 12 slots, line-aligned windows, 8 packets per wave, 256-thread
// workgroups at 6 waves/SIMD, one 16-byte store per header chunk past the caches). fwd_rw_kernel reads
// every frame in exactly that pattern (the same loads, policies, block order and occupancy), computes
// nothing but an xor, and then:
//   MODE 0  writes nothing                                    (the read floor of the forward's pattern)
//   MODE 1  stores the frame's first 64 bytes back as 4 chunk stores past the caches once its loads have
//           returned (the values read: the forward's segment store without its arithmetic)
//   MODE 2  stores the same 4 chunks with no loads at all (the writes alone into lines no one has read;
//           the frames' first 64 bytes are zeroed: timing only)
// Variants of nfcs_r6_fwd_time: 0 the product forward (nfcs_l3_forward_device), 1/2/3 = MODE 0/1/2, 4 the
// product update (nfcs_update_device) on the same batches, 5 the update's frames_read floor.
#include "../../netflow_amd/csrc/nfcs_kernels.hip"

namespace nfcs {

template <int MODE>
__global__ __launch_bounds__(kBlock, 6) void fwd_rw_kernel(const nfcs_desc* __restrict__ desc, uint32_t n,
                                                           uint32_t nblocks, uint8_t* __restrict__ arena,
                                                           uint64_t arena_bytes) {
    constexpr int K = 12, R = 8, PW = 8;
    const uint32_t lane = threadIdx.x & 63u, rl = lane & (R - 1), row = lane / R;
    const uint64_t pw = (uint64_t)xcd_block_n(nblocks) * (kBlock / R) + rfl(threadIdx.x >> 6) * PW;
    if (pw >= n) return;
    const nfcs_desc d = pick_desc<PW>(load_descw<PW>(desc, pw, n), row);
    const uint64_t off = (uint64_t)d.off16 * 16u;
    const bool live = pw + row < n && off + (((uint64_t)d.len + 15u) & ~15ull) <= arena_bytes;
    const uint32_t nch = live ? (d.len + 15u) >> 4 : 0u;
    uint8_t* f = arena + (live ? off : 0);
    uint4* src = (uint4*)f;
    if (MODE == 2) {
        if (live && rl < 4 && rl < nch) st16_nt(src + rl, make_uint4(0u, 0u, 0u, 0u));
        return;
    }
    const uint32_t mis = live ? (uint32_t)(((uintptr_t)f >> 4) & 7u) : 0u;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = rl + (uint32_t)R * k - mis;
        const uint4* a = (c < nch) ? src + c : g_zero_line;
        v[k] = k == 0 ? ld16<0>(a) : ld16<1>(a);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    const uint32_t cmax = wave_max_rows<R>(nch + mis);
    for (uint32_t cb = (uint32_t)R * K; cb < cmax; cb += (uint32_t)R * K) {
        uint4 w[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = cb + rl + (uint32_t)R * k - mis;
            w[k] = ld16<1>((c < nch) ? src + c : g_zero_line);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc ^= w[k].x ^ w[k].y ^ w[k].z ^ w[k].w;
    }
    acc = row_sum<R>(acc);
    if (MODE == 0) {
        if (acc == 0x9E3779B9u) f[0] = 0;  // keeps the loads (never true on the bench's frames)
        return;
    }
    // frame chunks 0..3 from the lanes that hold them (slot 0 lanes mis.., slot 1 lanes ..mis-5), stored
    // once every load of the row has returned (the xor feeds the value: never changes it here)
    const uint32_t flip = acc == 0x9E3779B9u ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t c = rl + (uint32_t)R * k - mis;
        if (live && c < 4u && c < nch) st16_nt(src + c, make_uint4(v[k].x ^ flip, v[k].y, v[k].z, v[k].w));
    }
}

template <int MODE>
static void launch_fwd_rw(uint8_t* arena, uint64_t bytes, const nfcs_desc* desc, uint32_t n, hipStream_t st) {
    const uint32_t grid = (uint32_t)(((uint64_t)n + 31u) / 32u);
    // held at 6 waves/SIMD (24 KiB of unused LDS per workgroup), the product shape's occupancy (80 VGPRs)
    hipLaunchKernelGGL((fwd_rw_kernel<MODE>), dim3(grid), dim3(kBlock), kRowsLdsPad6, st, desc, n, grid, arena, bytes);
}

}  // namespace nfcs

extern "C" NFCS_API int nfcs_r6_fwd_time(nfcs_ctx* ctx, int v, uint32_t batches, uint8_t* const* arenas,
                                         const uint64_t* bytes, const nfcs_desc* const* descs, uint32_t n, int iters,
                                         const uint32_t* nh, const nfcs_nexthop* table, uint32_t table_n,
                                         void* sink, float* ms) {
    hipStream_t st = (hipStream_t)nfcs_ctx_stream(ctx);
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return NFCS_EHIP;
    int rc = NFCS_OK;
    (void)hipEventRecord(e0, st);
    for (int it = 0; it < iters && rc == NFCS_OK; ++it) {
        const uint32_t b = (uint32_t)it % batches;
        hipError_t e = hipSuccess;
        switch (v) {
        case 0: rc = nfcs_l3_forward_device(ctx, arenas[b], bytes[b], descs[b], nh, n, table, table_n, nullptr, st); break;
        case 1: nfcs::launch_fwd_rw<0>(arenas[b], bytes[b], descs[b], n, st); break;
        case 2: nfcs::launch_fwd_rw<1>(arenas[b], bytes[b], descs[b], n, st); break;
        case 3: nfcs::launch_fwd_rw<2>(arenas[b], bytes[b], descs[b], n, st); break;
        case 4: rc = nfcs_update_device(ctx, arenas[b], bytes[b], descs[b], n, nullptr, nullptr, st); break;
        case 5: e = nfcs::launch_frames_read(arenas[b], bytes[b], descs[b], n, (unsigned long long*)sink, st); break;
        default: rc = NFCS_EINVAL;
        }
        if (e == hipSuccess) e = hipGetLastError();
        if (e != hipSuccess) rc = NFCS_EHIP;
    }
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}
