// c3_exp.hip — round-5 measurement translation unit (not product): one more write schedule for
// BASELINE C3 (4M x U{64..1500} B), VERDICT r4 item 5. Built with the product C ABI into
// tools/r05/libnfcs_c3x.so by tools/r05/build_c3x.sh; the product library never contains it.
//
// C3's product (the short shape: 16-lane rows in one-wave workgroups, inline `nt` byte stores) runs at
// the time of a kernel that only reads the frames plus the time of its 4.19M in-place writes
// (DESIGN.md §5c): the writes interleave with the read stream. Here the reads and the writes of a
// sub-batch are decoupled in time but not in launches: the call runs as sub-batches of S packets, and
// the launch of sub-batch j is the short shape's read pass over j writing 8-byte patch records, with
// one write-only workgroup after every 16 read workgroups (in dispatch order) applying sub-batch j-1's
// records (64 packets each, one masked `sc0 sc1 nt` byte store request per packet, as
// apply_bytes_kernel). The writes of j-1 land while j's reads stream, from a separate set of waves,
// in address order, into header lines sub-batch j-1 has just brought into the memory-side cache. The
// last sub-batch's records go out in a write-only launch at the end.
//   v 0   the product (launch_update, kUpdateAuto: the short shape, inline stores)
//   v 1   write workgroups interleaved, S = 512K      v 2   S = 256K      v 3   S = 1M
//   v 4   records only in the same launches (no frame write: the floor of this read pass; no parity)
//   v 5   S = 512K, the write workgroups of j-1 first in the launch (dispatched before j's reads)
#include "../../netflow_amd/csrc/nfcs_kernels.hip"

namespace nfcs {

// One wave applies the patch records of packets p0 .. p0+63 (apply_bytes_kernel's stores without its
// deferral decision: every packet of the sub-batch has a record).
DEV void apply_records_wave(uint8_t* arena, const nfcs_desc* desc, uint32_t n, const nfcs_patch* rec, uint64_t p0,
                            uint32_t lane) {
    const uint64_t i = p0 + lane;
    const bool in = i < n;
    const nfcs_desc d = in ? desc[i] : nfcs_desc{0u, 0u};
    const uint2 r = in ? ((const uint2*)rec)[i] : make_uint2(NFCS_PATCH_NONE | (NFCS_PATCH_NONE << 16), 0u);
    const uint32_t j = lane & 3u;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const int q4 = (int)((16u * k + (lane >> 2)) * 4u);
        const uint32_t rx = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)r.x);
        const uint32_t ry = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)r.y);
        const uint32_t o16 = (uint32_t)__builtin_amdgcn_ds_bpermute(q4, (int)d.off16);
        const uint32_t ipo = rx & 0xFFFFu, l4o = rx >> 16;
        const uint32_t off = j < 2 ? ipo : l4o;
        const uint32_t a = off + (j & 1u);
        const bool overlap = j < 2 && l4o != NFCS_PATCH_NONE && (a == l4o || a == l4o + 1u);
        if (off != NFCS_PATCH_NONE && !overlap) {
            const uint32_t b = (j < 2 ? (ry >> (8 * j)) : (ry >> (16 + 8 * (j - 2)))) & 0xFFu;
            uint8_t* p = arena + (uint64_t)o16 * 16u + a;
            asm volatile("global_store_byte %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(b) : "memory");
        }
    }
}

// Read workgroups of sub-batch j (the short shape's body, records only) and write workgroups of
// sub-batch j-1, dispatched in the order FIRST ? (all writes, then reads) : (16 reads, 1 write, ...).
template <bool FIRST, bool WRITES>
__global__ __launch_bounds__(64, 7) void c3_fused_kernel(const nfcs_desc* __restrict__ desc, uint32_t m,
                                                         uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                         nfcs_patch* __restrict__ rec_out,
                                                         const nfcs_desc* __restrict__ pdesc, uint32_t pm,
                                                         const nfcs_patch* __restrict__ rec_in,
                                                         uint32_t wblocks, uint32_t nblocks) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t b = xcd_block_n(nblocks);
    bool wr;
    uint32_t idx;
    if (FIRST) {
        wr = b < wblocks;
        idx = wr ? b : b - wblocks;
    } else if (b / 17u < wblocks) {
        wr = b % 17u == 16u;
        idx = wr ? b / 17u : (b / 17u) * 16u + b % 17u;
    } else {
        wr = false;
        idx = 16u * wblocks + (b - 17u * wblocks);
    }
    if (wr) {
        if (WRITES) apply_records_wave(arena, pdesc, pm, rec_in, (uint64_t)idx * 64u, lane);
        return;
    }
    constexpr uint32_t PW = 4;
    const uint32_t rl = lane & 15u, row = lane / 16u;
    const uint32_t rowbase4 = (lane & ~15u) * 4u;
    const uint64_t pw = (uint64_t)idx * PW;
    if (pw >= m) return;
    const DescW<PW> D = load_descw<PW>(desc, pw, m);
    uint32_t q[PW] = {0, 0, 0, 0};
    rows_body<6, 16, 64, false, SF_RECORDS, false, PW>(D, pw, m, arena, arena_bytes, 0u, rl, row, rowbase4, false, q,
                                                      nullptr, rec_out, nullptr, nullptr, 0u);
}

__global__ __launch_bounds__(kBlock) void apply_records_kernel(uint8_t* __restrict__ arena,
                                                               const nfcs_desc* __restrict__ desc, uint32_t n,
                                                               const nfcs_patch* __restrict__ rec) {
    apply_records_wave(arena, desc, n, rec, ((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 64u,
                       threadIdx.x & 63u);
}

static hipError_t c3_call(int v, uint8_t* arena, uint64_t bytes, const nfcs_desc* desc, uint32_t n, nfcs_patch* ws,
                          hipStream_t st) {
    const uint32_t S = v == 2 ? (1u << 18) : v == 3 ? (1u << 20) : (1u << 19);
    const bool writes = v != 4, first = v == 5;
    nfcs_patch* rec[2] = {ws, ws + S};
    uint32_t prev_i = 0, prev_m = 0;
    int k = 0;
    for (uint32_t i = 0; i < n; i += S, k ^= 1) {
        const uint32_t m = std::min(S, n - i);
        const uint32_t rblocks = (m + 3u) / 4u, wblocks = (prev_m + 63u) / 64u;
        const uint32_t nblocks = first ? rblocks + wblocks : std::max(rblocks + wblocks, 17u * wblocks);
        if (first)
            hipLaunchKernelGGL((c3_fused_kernel<true, true>), dim3(nblocks), dim3(64), 0, st, desc + i, m, arena, bytes,
                               rec[k], desc + prev_i, prev_m, rec[k ^ 1], wblocks, nblocks);
        else if (writes)
            hipLaunchKernelGGL((c3_fused_kernel<false, true>), dim3(nblocks), dim3(64), 0, st, desc + i, m, arena,
                               bytes, rec[k], desc + prev_i, prev_m, rec[k ^ 1], wblocks, nblocks);
        else
            hipLaunchKernelGGL((c3_fused_kernel<false, false>), dim3(nblocks), dim3(64), 0, st, desc + i, m, arena,
                               bytes, rec[k], desc + prev_i, prev_m, rec[k ^ 1], wblocks, nblocks);
        prev_i = i;
        prev_m = m;
    }
    if (writes && prev_m)
        hipLaunchKernelGGL(apply_records_kernel, dim3((prev_m + kBlock - 1) / kBlock), dim3(kBlock), 0, st, arena,
                           desc + prev_i, prev_m, (const nfcs_patch*)rec[k ^ 1]);
    return hipGetLastError();
}

}  // namespace nfcs

// v 0: the product; v >= 1: c3_call. Rotation over `batches` batches, HIP events around `iters` calls
// on the context's stream; ws: 2 x 1M patch records (8 MB x 2).
extern "C" NFCS_API int nfcs_r5_c3_time(nfcs_ctx* ctx, int v, uint32_t batches, uint8_t* const* arenas,
                                        const uint64_t* bytes, const nfcs_desc* const* descs, uint32_t n, int iters,
                                        void* ws, float* ms) {
    hipStream_t st = (hipStream_t)nfcs_ctx_stream(ctx);
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return NFCS_EHIP;
    int rc = NFCS_OK;
    (void)hipEventRecord(e0, st);
    for (int it = 0; it < iters && rc == NFCS_OK; ++it) {
        const uint32_t b = (uint32_t)it % batches;
        if (v == 0) rc = nfcs_update_device(ctx, arenas[b], bytes[b], descs[b], n, nullptr, nullptr, st);
        else if (nfcs::c3_call(v, arenas[b], bytes[b], descs[b], n, (nfcs_patch*)ws, st) != hipSuccess) rc = NFCS_EHIP;
    }
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}
