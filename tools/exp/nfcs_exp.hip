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
//           6   two row groups per wave, the second landing in LDS (8 packets per wave), 1-wave WGs
//           7   the same in 256-thread workgroups
//           9   variant 6's kernel writing patch records only;  10  the same with no writes at all
//          11   the product's one-wave row kernel with no writes at all
//          12   every packet deferred: records-only read pass + a write pass over every packet
//          13   that write pass alone (run after 12: it re-applies 12's records)
//       14/15   the product's read pass + a write pass of whole 16-byte chunks re-read from the frame
//               (default-policy / non-temporal re-read)
//    16/17/18   the product form over consecutive sub-batches of 1M / 512K / 2M packets (the
//               product itself uses 512K, kSubBatchPackets);  19  one launch pair, no sub-batches
//       20/21   256K / 512K sub-batches with write pass i on a second stream, overlapping read pass i+1
//       22/23   the product's launches (long-frame shape) with the write pass's stores plain / sc1
//    24/25/26   8-lane rows (8 packets per wave) with 2 / 4 / 6 slots, inline, one-wave workgroups
//       27/28   8-lane rows with 6 / 2 slots, per-group deferral + write pass
//    40/41/42   C3 floors (timing only): the short shape's reads with no parse and no writes / with
//               4 bytes written per packet / with the first 64 bytes written back
// lds_pad: dynamic LDS bytes per workgroup, to cap the waves per SIMD (occupancy sweeps).
#include "../../netflow_amd/csrc/nfcs_kernels.hip"

namespace nfcs {

// Two row groups per wave, the second landing in LDS (variants 6/7): group B's six chunk slots
// are LDS-DMA loads (global_load_lds_dwordx4: no VGPR destination), so a wave carries 8 packets
// with the VGPR footprint of 4. Issued B first, then A; A is processed from registers, then B's
// chunks are read back from LDS (each lane reads the 16 bytes it loaded: no bank conflicts).
typedef __attribute__((address_space(3))) void lds_void_t;

template <int K>
DEV void row_stage_lds(RowStage<K>& S, uint8_t* arena, uint64_t arena_bytes, const nfcs_desc& d,
                       uint64_t p64, uint32_t n, uint32_t base16, uint32_t rl, uint4* wbuf) {
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
    const uint32_t nch = (S.len + 15u) >> 4;
    const uint4* src = (const uint4*)S.frame;
    __builtin_amdgcn_global_load_lds((const void*)(rl < nch ? src + rl : &g_zero16), (lds_void_t*)wbuf, 16, 0, 0);
#pragma unroll
    for (int k = 1; k < K; ++k) {
        const uint32_t c = rl + 16u * k;
        const uint4* a = (c < nch) ? src + c : &g_zero16;
        __builtin_amdgcn_global_load_lds((const void*)a, (lds_void_t*)(wbuf + 64 * k), 16, 0, 2);
    }
}

template <int K, int BS, int SF>
__global__ __launch_bounds__(BS) void update_rows2_kernel(uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                          const nfcs_desc* __restrict__ desc, uint32_t n,
                                                          uint32_t base16, uint8_t* __restrict__ status,
                                                          nfcs_patch* __restrict__ patch,
                                                          nfcs_patch* __restrict__ ws) {
    extern __shared__ uint4 lbuf[];
    const uint32_t lane = threadIdx.x & 63u, rl = lane & 15u, row = lane >> 4;
    const uint32_t rowbase4 = (lane & ~15u) * 4u;
    const uint32_t wv = rfl(threadIdx.x >> 6);
    const uint64_t pw = (uint64_t)xcd_block() * (BS / 64 * 8) + wv * 8u;
    if (pw >= n) return;
    const DescW<8> D = load_descw<8>(desc, pw, n);
    DescW<4> DA, DB;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        DA.w[i] = D.w[i];
        DB.w[i] = D.w[8 + i];
    }
    bool dA = false, dB = false;
    if (SF == SF_DEFER) {
        uint32_t sa = 0, sb = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            sa += defer_len(DA.w[2 * i + 1]);
            sb += defer_len(DB.w[2 * i + 1]);
        }
        dA = defer_group(sa, 4);
        dB = defer_group(sb, 4);
    }
    uint4* wbuf = lbuf + wv * (64u * K);
    RowStage<K> A, B;
    row_stage_lds<K>(B, arena, arena_bytes, pick_desc<4>(DB, row), pw + 4 + row, n, base16, rl, wbuf);
    row_stage<K, 16, false>(A, arena, arena_bytes, pick_desc<4>(DA, row), pw + row, n, base16, rl);
    nfcs_patch* recA = SF == 3 ? nullptr : (patch ? patch : (dA ? ws : nullptr));
    nfcs_patch* recB = SF == 3 ? nullptr : (patch ? patch : (dB ? ws : nullptr));
    row_process<K, 16, false>(A, rl, rowbase4, status, recA, SF == SF_INLINE || (SF == SF_DEFER && !dA));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < K; ++k) B.v[k] = wbuf[64 * k + lane];
    row_process<K, 16, false>(B, rl, rowbase4, status, recB, SF == SF_INLINE || (SF == SF_DEFER && !dB));
}

// apply_bytes_kernel for every packet (no deferral decision): the write pass of variant 12, where
// the read pass wrote records for every packet (SF_RECORDS) whatever the frame lengths.
__global__ __launch_bounds__(kBlock) void apply_all_kernel(uint8_t* __restrict__ arena,
                                                           const nfcs_desc* __restrict__ desc, uint32_t n,
                                                           const nfcs_patch* __restrict__ rec) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool live = i < n;
    const nfcs_desc d = live ? desc[i] : nfcs_desc{0u, 0u};
    const uint2 r = live ? ((const uint2*)rec)[i] : make_uint2(NFCS_PATCH_NONE | (NFCS_PATCH_NONE << 16), 0u);
    const uint64_t mask = __builtin_amdgcn_ballot_w64(live);
    const uint32_t j = lane & 3u;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        if (((mask >> (16u * k)) & 0xFFFFu) == 0) continue;
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

// Write pass with whole 16-byte chunks (variants 14/15): 4 lanes per deferred packet re-read the
// frame's first 64 bytes (chunk j by lane j; LD: 0 default policy, 1 non-temporal), patch the
// checksum bytes in and store the chunks back (`sc0 sc1 nt`), so a 64-byte-aligned frame's write
// is one whole 64-byte segment instead of a byte-masked partial write. Frames whose fields lie past
// byte 63, or shorter than 49 bytes, take the byte stores of apply_bytes_kernel.
template <int LD>
__global__ __launch_bounds__(kBlock) void apply_seg_kernel(uint8_t* __restrict__ arena,
                                                           const nfcs_desc* __restrict__ desc, uint32_t n,
                                                           uint32_t base16, const nfcs_patch* __restrict__ rec) {
    const uint32_t lane = threadIdx.x & 63u, j = lane & 3u;
    const uint64_t p = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 2;
    const bool live = p < n;
    const nfcs_desc d = live ? desc[p] : nfcs_desc{0u, 0u};
    const uint2 r = live ? ((const uint2*)rec)[p] : make_uint2(0u, 0u);
    const uint32_t s = row_sum<16>(j == 0 ? defer_len(d.len) : 0u);  // the aligned quad's lengths
    const bool dfr = live && defer_group(s, 4);
    if (!dfr) return;
    const uint32_t ipo = r.x & 0xFFFFu, l4o = r.x >> 16;
    uint8_t* f = arena + ((uint64_t)d.off16 - base16) * 16u;
    const bool seg = d.len > 48u && (ipo == NFCS_PATCH_NONE || ipo + 1u < 64u) &&
                     (l4o == NFCS_PATCH_NONE || l4o + 1u < 64u);
    if (seg) {
        uint4* q = (uint4*)f + j;
        uint4 v = LD ? ld16<1>(q) : *q;
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) {  // IPv4 bytes first, L4 bytes last (as the reference)
            const uint32_t off = t < 2 ? ipo : l4o;
            const uint32_t a = off + (t & 1u);
            const uint32_t b = (r.y >> (8u * t)) & 0xFFu;
            if (off != NFCS_PATCH_NONE && (a >> 4) == j) v = put_byte(v, a & 15u, b);
        }
        const u32x4_t w = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" ::"v"(q), "v"(w) : "memory");
    } else {
        const uint32_t off = j < 2 ? ipo : l4o;
        const uint32_t a = off + (j & 1u);
        const bool overlap = j < 2 && l4o != NFCS_PATCH_NONE && (a == l4o || a == l4o + 1u);
        if (off != NFCS_PATCH_NONE && !overlap) {
            const uint32_t b = (r.y >> (8u * j)) & 0xFFu;
            asm volatile("global_store_byte %0, %1, off sc0 sc1 nt" ::"v"(f + a), "v"(b) : "memory");
        }
    }
}

// apply_bytes_kernel<true> with another store policy (variants 22/23): POL 0 plain (write-back),
// 1 `sc1` (agent-scope write-through). The product stores `sc0 sc1 nt`.
template <int POL>
__global__ __launch_bounds__(kBlock) void apply_pol_kernel(uint8_t* __restrict__ arena,
                                                           const nfcs_desc* __restrict__ desc, uint32_t n,
                                                           const nfcs_patch* __restrict__ rec) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const nfcs_desc d = i < n ? desc[i] : nfcs_desc{0u, 0u};
    const uint2 r0 = i < n ? ((const uint2*)rec)[i] : make_uint2(0u, 0u);
    uint32_t s = defer_len(d.len);
    s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0xB1, 0xF, 0xF, true);
    s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x4E, 0xF, 0xF, true);
    const bool dfr = i < n && defer_group(s, 4);
    const uint64_t mask = __builtin_amdgcn_ballot_w64(dfr);
    if (!mask) return;
    const uint2 r = dfr ? r0 : make_uint2(NFCS_PATCH_NONE | (NFCS_PATCH_NONE << 16), 0u);
    const uint32_t j = lane & 3u;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        if (((mask >> (16u * k)) & 0xFFFFu) == 0) continue;
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
            if (POL == 1) st8<true>(p, b);
            else *p = (uint8_t)b;
        }
    }
}

// Write-pass probes (variants 33/34). MODE 0: apply_bytes_kernel<true>'s loads and decision only, no
// stores (the pass's launch + load round trip). MODE 1: 4 lanes per packet (lane j of the quad
// loads the packet's descriptor and record itself and writes byte j): no cross-lane permutes,
// 4x the threads.
template <int MODE>
__global__ __launch_bounds__(kBlock) void apply_probe_kernel(uint8_t* __restrict__ arena,
                                                             const nfcs_desc* __restrict__ desc, uint32_t n,
                                                             const nfcs_patch* __restrict__ rec, uint32_t* sink) {
    const uint32_t lane = threadIdx.x & 63u;
    if (MODE == 0) {
        const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        const nfcs_desc d = i < n ? desc[i] : nfcs_desc{0u, 0u};
        const uint2 r0 = i < n ? ((const uint2*)rec)[i] : make_uint2(0u, 0u);
        uint32_t s = defer_len(d.len);
        s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0xB1, 0xF, 0xF, true);
        s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x4E, 0xF, 0xF, true);
        const bool dfr = i < n && defer_group(s, 4);
        const uint32_t v = dfr ? (r0.x ^ r0.y ^ d.off16) : 0u;
        if (v == 0x9E3779B9u && lane == 7u) sink[0] = v;  // never true on real records
        return;
    }
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t p = t >> 2;
    const uint32_t j = lane & 3u;
    const nfcs_desc d = p < n ? desc[p] : nfcs_desc{0u, 0u};
    const uint2 r = p < n ? ((const uint2*)rec)[p] : make_uint2(0u, 0u);
    const uint32_t s = row_sum<16>(j == 0 ? defer_len(d.len) : 0u);
    if (!(p < n && defer_group(s, 4))) return;
    const uint32_t ipo = r.x & 0xFFFFu, l4o = r.x >> 16;
    const uint32_t off = j < 2 ? ipo : l4o;
    const uint32_t a = off + (j & 1u);
    const bool overlap = j < 2 && l4o != NFCS_PATCH_NONE && (a == l4o || a == l4o + 1u);
    if (off != NFCS_PATCH_NONE && !overlap) {
        const uint32_t b = (r.y >> (8u * j)) & 0xFFu;
        uint8_t* q = arena + (uint64_t)d.off16 * 16u + a;
        asm volatile("global_store_byte %0, %1, off sc0 sc1 nt" ::"v"(q), "v"(b) : "memory");
    }
}

// Floors of C3's time without the checksum computation (variants 40-42; timing only, the frames
// are not updated correctly): the product's short shape (16-lane rows, 6 slots, one-wave
// workgroups at 7 waves/SIMD, the same load policies and XCD order) reads every frame and XORs
// its chunks — no header parse, no checksum plan — and then WR 0 writes nothing, WR 1 writes
// 4 bytes per packet at frame offsets 24, 25, 40, 41 as the product's inline checksum bytes go
// (one `sc0 sc1 nt` byte store per lane 0-3, one write request per packet), WR 2 writes the
// frame's first 64 bytes back as one segment (lanes 0-3, 16 bytes each, `sc0 sc1 nt`).
template <int WR>
__global__ __launch_bounds__(64, 7) void floor_rows_kernel(uint8_t* __restrict__ arena,
                                                           const nfcs_desc* __restrict__ desc, uint32_t n,
                                                           uint32_t* __restrict__ sink) {
    constexpr int K = 6, R = 16, PW = 4;
    const uint32_t lane = threadIdx.x & 63u, rl = lane & (R - 1), row = lane / R;
    const uint64_t pw = (uint64_t)xcd_block() * PW;
    if (pw >= n) return;
    const DescW<PW> D = load_descw<PW>(desc, pw, n);
    const nfcs_desc d = pick_desc<PW>(D, row);
    const bool valid = pw + row < n;
    const uint32_t len = valid ? d.len : 0u, nch = (len + 15u) >> 4;
    uint8_t* frame = arena + (uint64_t)d.off16 * 16u;
    const uint4* src = (const uint4*)frame;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = rl + (uint32_t)R * k;
        const uint4* a = c < nch ? src + c : &g_zero16;
        v[k] = k == 0 ? ld16<0>(a) : ld16<1>(a);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) acc += v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    acc = row_sum<R>(acc);
    if (acc == 0x9E3779B9u && sink) sink[0] = acc;  // keeps every load live
    if (WR == 1 && valid && rl < 4 && len >= 42) st8_nt(frame + (rl < 2 ? 24u + rl : 38u + rl), acc >> (8u * rl));
    if (WR == 2 && valid && rl < 4 && 16u * rl < len) {
        st16_nt((uint4*)frame + rl, v[0]);  // the values read
    }
}

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
        hipLaunchKernelGGL(apply_bytes_kernel<true>, ga, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    case 4:
        NFCS_X(1, kBlock, g4, SF_DEFER);
        hipLaunchKernelGGL(apply_bytes_kernel<true>, ga, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    case 5:
        hipLaunchKernelGGL((update_rows_kernel<6, 16, 1, kBlock, false, SF_RECORDS>), g4, dim3(kBlock),
                           lds_pad, st, arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, ws,
                           (nfcs_patch*)nullptr, nofwd);
        break;
    case 6:
        hipLaunchKernelGGL((update_rows2_kernel<6, 64, SF_DEFER>), dim3((n + 7u) / 8u), dim3(64), 6 * 1024, st,
                           arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws);
        hipLaunchKernelGGL(apply_bytes_kernel<true>, ga, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    case 7:
        hipLaunchKernelGGL((update_rows2_kernel<6, 256, SF_DEFER>), dim3((n + 31u) / 32u), dim3(256), 24 * 1024,
                           st, arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws);
        hipLaunchKernelGGL(apply_bytes_kernel<true>, ga, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    case 9:  // two-group LDS kernel, records only (frames untouched)
        hipLaunchKernelGGL((update_rows2_kernel<6, 64, SF_RECORDS>), dim3((n + 7u) / 8u), dim3(64), 6 * 1024, st,
                           arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, ws, (nfcs_patch*)nullptr);
        break;
    case 10:  // two-group LDS kernel, no writes at all (bound for full-line record writes)
        hipLaunchKernelGGL((update_rows2_kernel<6, 64, 3>), dim3((n + 7u) / 8u), dim3(64), 6 * 1024, st,
                           arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, ws, (nfcs_patch*)nullptr);
        break;
    case 11:  // product row kernel (one-wave workgroups), no writes at all
        hipLaunchKernelGGL((update_rows_kernel<6, 16, 7, 64, false, SF_RECORDS>), g1, dim3(64), lds_pad, st,
                           arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr,
                           (nfcs_patch*)nullptr, nofwd);
        break;
    case 12:  // every packet deferred: records-only read pass (one-wave WGs) + apply_all_kernel
        hipLaunchKernelGGL((update_rows_kernel<6, 16, 7, 64, false, SF_RECORDS>), g1, dim3(64), lds_pad, st,
                           arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, ws, (nfcs_patch*)nullptr, nofwd);
        hipLaunchKernelGGL(apply_all_kernel, ga, dim3(kBlock), 0, st, arena, desc, n, ws);
        break;
    case 13:  // the write pass alone (records from the last variant-12 call)
        hipLaunchKernelGGL(apply_all_kernel, ga, dim3(kBlock), 0, st, arena, desc, n, ws);
        break;
    case 14:
    case 15: {
        if (arena_bytes / n < kSmallMeanBytes) NFCS_X(7, 64, g1, SF_DEFER);
        else hipLaunchKernelGGL((update_rows_kernel<6, 16, 1, kBlock, false, SF_DEFER>), g4, dim3(kBlock),
                                kRowsLdsPad, st, arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr,
                                (nfcs_patch*)nullptr, ws, nofwd);
        const dim3 gs((uint32_t)(((uint64_t)n * 4u + kBlock - 1) / kBlock));
        if (variant == 14) hipLaunchKernelGGL(apply_seg_kernel<0>, gs, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        else hipLaunchKernelGGL(apply_seg_kernel<1>, gs, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    }
    case 16:
    case 17:
    case 18: {  // the product form over consecutive sub-batches of 1M / 512K / 2M packets
        const uint32_t S = variant == 16 ? (1u << 20) : (variant == 17 ? (1u << 19) : (1u << 21));
        for (uint32_t i = 0; i < n; i += S) {
            const hipError_t e = launch_update_one(arena, arena_bytes, desc + i, std::min(S, n - i), 0u, nullptr,
                                                   nullptr, ws, kUpdateAuto, kShapeLong, st);
            if (e != hipSuccess) return e;
        }
        break;
    }
    case 19:  // the product form in ONE launch pair (no sub-batches), the round-2 session-1/2 form
        return launch_update_one(arena, arena_bytes, desc, n, 0u, nullptr, nullptr, ws, kUpdateAuto,
                                 arena_bytes / n < kTinyMeanBytes ? kShapeTiny
                                 : (arena_bytes / n < kSmallMeanBytes ? kShapeShort : kShapeLong), st);
    case 20:
    case 21: {  // sub-batches of 256K (20) / 512K (21): read pass i+1 overlaps write pass i on a second stream
        static hipStream_t s2 = nullptr;
        static hipEvent_t ev[64];
        if (!s2) {
            if (hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess) return hipErrorInvalidValue;
            for (auto& x : ev) (void)hipEventCreateWithFlags(&x, hipEventDisableTiming);
        }
        const uint32_t S = variant == 20 ? (1u << 18) : (1u << 19);
        const bool small = arena_bytes / n < kSmallMeanBytes;
        int k = 0;
        for (uint32_t i = 0; i < n && k < 63; i += S, ++k) {
            const uint32_t m = std::min(S, n - i);
            if (small) hipLaunchKernelGGL((update_rows_kernel<6, 16, 7, 64, false, SF_DEFER>), dim3((m + 3u) / 4u),
                                          dim3(64), 0u, st, arena, arena_bytes, desc + i, m, 0u, (uint8_t*)nullptr,
                                          (nfcs_patch*)nullptr, ws + i, nofwd);
            else hipLaunchKernelGGL((update_rows_kernel<6, 16, 1, kBlock, false, SF_DEFER>), dim3((m + 15u) / 16u),
                                    dim3(kBlock), kRowsLdsPad, st, arena, arena_bytes, desc + i, m, 0u,
                                    (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws + i, nofwd);
            (void)hipEventRecord(ev[k], st);
            (void)hipStreamWaitEvent(s2, ev[k], 0);
            hipLaunchKernelGGL(apply_bytes_kernel<true>, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, s2,
                               arena, desc + i, m, 0u, ws + i);
        }
        (void)hipEventRecord(ev[63], s2);
        (void)hipStreamWaitEvent(st, ev[63], 0);  // the call ends when its last write pass has
        break;
    }
    case 22:
    case 23: {  // the product's sub-batched launches with the write pass's stores plain (22) / sc1 (23)
        const uint32_t S = n > kSubBatchAbovePackets ? kSubBatchPackets : n;
        for (uint32_t i = 0; i < n; i += S) {
            const uint32_t m = std::min(S, n - i);
            hipLaunchKernelGGL((update_rows_kernel<6, 16, 1, kBlock, false, SF_DEFER>), dim3((m + 15u) / 16u),
                               dim3(kBlock), kRowsLdsPad, st, arena, arena_bytes, desc + i, m, 0u, (uint8_t*)nullptr,
                               (nfcs_patch*)nullptr, ws, nofwd);
            if (variant == 22)
                hipLaunchKernelGGL(apply_pol_kernel<0>, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, st, arena,
                                   desc + i, m, ws);
            else
                hipLaunchKernelGGL(apply_pol_kernel<1>, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, st, arena,
                                   desc + i, m, ws);
        }
        break;
    }
    case 24:  // 8-lane rows, 2 slots (256 B per row batch), 8 packets per wave, one-wave workgroups, inline
        hipLaunchKernelGGL((update_rows_kernel<2, 8, 8, 64, false, SF_INLINE>), dim3((n + 7u) / 8u), dim3(64), 0u, st,
                           arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr,
                           (nfcs_patch*)nullptr, nofwd);
        break;
    case 25:  // 8-lane rows, 4 slots (512 B per row batch)
        hipLaunchKernelGGL((update_rows_kernel<4, 8, 8, 64, false, SF_INLINE>), dim3((n + 7u) / 8u), dim3(64), 0u, st,
                           arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr,
                           (nfcs_patch*)nullptr, nofwd);
        break;
    case 26:  // 8-lane rows, 6 slots (768 B per row batch)
        hipLaunchKernelGGL((update_rows_kernel<6, 8, 8, 64, false, SF_INLINE>), dim3((n + 7u) / 8u), dim3(64), 0u, st,
                           arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr,
                           (nfcs_patch*)nullptr, nofwd);
        break;
    case 27:
    case 28: {  // 8-lane rows with 6 (27) / 2 (28) slots, SF_DEFER (per group of 4) + write pass
        if (variant == 27)
            hipLaunchKernelGGL((update_rows_kernel<6, 8, 8, 64, false, SF_DEFER>), dim3((n + 7u) / 8u), dim3(64), 0u,
                               st, arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws,
                               nofwd);
        else
            hipLaunchKernelGGL((update_rows_kernel<2, 8, 8, 64, false, SF_DEFER>), dim3((n + 7u) / 8u), dim3(64), 0u,
                               st, arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws,
                               nofwd);
        hipLaunchKernelGGL(apply_bytes_kernel<false>, ga, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    }
    case 29:
    case 30: {  // the product form over consecutive sub-batches of 256K (29) / 128K (30) packets
        const uint32_t S = variant == 29 ? (1u << 18) : (1u << 17);
        for (uint32_t i = 0; i < n; i += S) {
            const hipError_t e = launch_update_one(arena, arena_bytes, desc + i, std::min(S, n - i), 0u, nullptr,
                                                   nullptr, ws, kUpdateAuto, kShapeLong, st);
            if (e != hipSuccess) return e;
        }
        break;
    }
    case 31:  // the write pass alone, over the records of the last call
        hipLaunchKernelGGL(apply_bytes_kernel<true>, ga, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    case 32:  // the long-shape read pass alone (records for deferred waves, no write pass)
        hipLaunchKernelGGL((update_rows_kernel<6, 16, 1, kBlock, false, SF_DEFER>), g4, dim3(kBlock), kRowsLdsPad,
                           st, arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws, nofwd);
        break;
    case 33:  // the write pass's loads and decision only
        hipLaunchKernelGGL(apply_probe_kernel<0>, ga, dim3(kBlock), 0, st, arena, desc, n, ws, (uint32_t*)ws);
        break;
    case 34:  // the product read pass + the 4-lanes-per-packet write pass
    case 35: {  // that write pass alone
        if (variant == 34)
            hipLaunchKernelGGL((update_rows_kernel<6, 16, 1, kBlock, false, SF_DEFER>), g4, dim3(kBlock), kRowsLdsPad,
                               st, arena, arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws, nofwd);
        const dim3 gq((uint32_t)(((uint64_t)n * 4u + kBlock - 1) / kBlock));
        hipLaunchKernelGGL(apply_probe_kernel<1>, gq, dim3(kBlock), 0, st, arena, desc, n, ws, (uint32_t*)ws);
        break;
    }
    case 40:
        hipLaunchKernelGGL(floor_rows_kernel<0>, g1, dim3(64), 0, st, arena, desc, n, (uint32_t*)ws);
        break;
    case 41:
        hipLaunchKernelGGL(floor_rows_kernel<1>, g1, dim3(64), 0, st, arena, desc, n, (uint32_t*)ws);
        break;
    case 42:
        hipLaunchKernelGGL(floor_rows_kernel<2>, g1, dim3(64), 0, st, arena, desc, n, (uint32_t*)ws);
        break;
    case 36:
    case 37:
    case 38:
    case 39: {  // 8-lane rows with more slots (8 packets per wave, one-wave workgroups), SF_DEFER + write pass:
        //        12 slots (1536 B per row pass) at 5 (36) / 4 (37) waves/SIMD, 8 slots (38, 6 waves), 10 (39, 5)
        const dim3 g8((n + 7u) / 8u);
        if (variant == 36)
            hipLaunchKernelGGL((update_rows_kernel<12, 8, 5, 64, false, SF_DEFER>), g8, dim3(64), 0u, st, arena,
                               arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws, nofwd);
        else if (variant == 37)
            hipLaunchKernelGGL((update_rows_kernel<12, 8, 4, 64, false, SF_DEFER>), g8, dim3(64), 0u, st, arena,
                               arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws, nofwd);
        else if (variant == 38)
            hipLaunchKernelGGL((update_rows_kernel<8, 8, 6, 64, false, SF_DEFER>), g8, dim3(64), 0u, st, arena,
                               arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws, nofwd);
        else
            hipLaunchKernelGGL((update_rows_kernel<10, 8, 5, 64, false, SF_DEFER>), g8, dim3(64), 0u, st, arena,
                               arena_bytes, desc, n, 0u, (uint8_t*)nullptr, (nfcs_patch*)nullptr, ws, nofwd);
        hipLaunchKernelGGL(apply_bytes_kernel<false>, ga, dim3(kBlock), 0, st, arena, desc, n, 0u, ws);
        break;
    }
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

// ---- flow keys: launch forms (nfcs_exp_time_flow) -------------------------------------------
//   variant 0   the product (launch_flow_keys: one wave per 32 packets, XCD-aware block order)
//           1/2 a persistent grid (1/2: CUs x 8 / CUs x 16 workgroups of 256 threads) striding over
//               the same 32-packet wave groups, so the launch has no ramp-up / drain of short waves
namespace nfcs {
template <int K>
__global__ __launch_bounds__(kBlock) void flow_keys_loop_kernel(const uint8_t* __restrict__ arena,
                                                                uint64_t arena_bytes,
                                                                const nfcs_desc* __restrict__ desc, uint32_t n,
                                                                nfcs_flow_key* __restrict__ keys,
                                                                uint32_t* __restrict__ hashes) {
    constexpr int R = 8;
    constexpr uint32_t PR = 64 / R, PW = PR * K;
    const uint32_t lane = threadIdx.x & 63u, rl = lane & (R - 1), row = lane / R;
    const uint32_t rowbase4 = (lane & ~(uint32_t)(R - 1)) * 4u;
    const uint64_t groups = ((uint64_t)n + PW - 1) / PW;
    const uint64_t stride = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t w = (uint64_t)blockIdx.x * (kBlock / 64) + rfl(threadIdx.x >> 6); w < groups; w += stride) {
        const uint64_t pw = w * PW;
        uint2 dl = make_uint2(0u, 0u);
        if (lane < PW && pw + lane < n) dl = ((const uint2*)desc)[pw + lane];
        uint4 c[K];
        uint32_t L[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t sl = (uint32_t)k * PR + row;
            const uint32_t off16 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(sl * 4u), (int)dl.x);
            const uint32_t dlen = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(sl * 4u), (int)dl.y);
            const uint64_t off = (uint64_t)off16 * 16u;
            const bool live = pw + sl < n && off + (((uint64_t)dlen + 15u) & ~15ull) <= arena_bytes;
            L[k] = live ? dlen : 0u;
            const uint4* src = (const uint4*)(arena + (live ? off : 0));
            c[k] = ld16<0>((rl * 16u < L[k]) ? src + rl : &g_zero16);
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            flow_key_row(c[k], L[k], pw + (uint32_t)k * PR + row, n, rl, rowbase4, keys, hashes);
    }
}
}  // namespace nfcs

extern "C" NFCS_API int nfcs_exp_time_flow(int variant, const uint8_t* d_arena, uint64_t arena_bytes,
                                          const nfcs_desc* d_desc, uint32_t n, nfcs_flow_key* d_keys,
                                          uint32_t* d_hash, int iters, void* stream, float* ms) {
    hipStream_t st = (hipStream_t)stream;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return -1;
    const unsigned cus = (unsigned)prop.multiProcessorCount;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1;
    hipError_t e = hipEventRecord(e0, st);
    for (int it = 0; it < iters && e == hipSuccess; ++it) {
        if (variant == 0) {
            e = nfcs::launch_flow_keys(nfcs::DevInfo{}, d_arena, arena_bytes, d_desc, n, d_keys, d_hash, st);
        } else {
            const unsigned g = cus * (variant == 1 ? 8u : 16u);
            hipLaunchKernelGGL((nfcs::flow_keys_loop_kernel<4>), dim3(g), dim3(nfcs::kBlock), 0, st, d_arena,
                               arena_bytes, d_desc, n, d_keys, d_hash);
            e = hipGetLastError();
        }
    }
    if (e == hipSuccess) e = hipEventRecord(e1, st);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return (int)e;
}
