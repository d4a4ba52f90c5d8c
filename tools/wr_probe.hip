// wr_probe.hip — measurement tool (not product): what does a store cost inside the checksum
// kernel's read stream, and why more on a large (fresh) batch than on a re-processed 1.5 GB one?
//
// The read side mirrors update_rows_kernel: 256-thread workgroups, one 16-lane row per 1536-byte
// frame (4 frames per wave, 16 per workgroup), 6 slots of global_load_dwordx4 per lane (slot 0
// default policy, slots 1-5 non-temporal), v_sad_u16 word sums, XCD-aware block order. Only the
// store differs by mode:
//   0 none                          1 8 B per packet, dense array, plain (split mode's records)
//   2 8 B per packet into a 4 KiB array (L2-resident: no DRAM write traffic), plain
//   3 4 B in place at frame+24, plain      4 the same, write-through (sc1)
//   5 dense 8 B, sc1                       6 dense 8 B, nt
//   7 4 KiB array, sc1                     8 dense, one 16-byte store per wave (4 packets)
//   9 in place, 1 in 16 packets            10 dense 8 B, 1 in 16 packets
//  11 the frame's first 64 bytes in place from lanes 0-3 (16 B each), plain
//  12 the same, write-through (sc1)        13 the same, nt        14 the same, sc0 sc1 nt
// Prints one JSON line per (packets, mode): average and best kernel time of 10 launches (HIP events).
//   hipcc --offload-arch=gfx950 -O3 tools/wr_probe.hip -o tools/wr_probe && tools/wr_probe [M ...]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
constexpr uint32_t kStride = 1536;

__device__ __forceinline__ uint4 ld(const uint4* p, bool nt) {
    if (nt) {
        const u32x4_t t = __builtin_nontemporal_load((const u32x4_t*)p);
        return make_uint4(t.x, t.y, t.z, t.w);
    }
    return *p;
}
__device__ __forceinline__ uint32_t ws(uint32_t d, uint32_t a) { return __builtin_amdgcn_sad_u16(d, 0u, a); }

template <int MODE>
__global__ __launch_bounds__(256) void probe(uint8_t* __restrict__ arena, uint32_t n,
                                             uint64_t* __restrict__ dense, uint64_t* __restrict__ tiny) {
    uint32_t bid = blockIdx.x;
    const uint32_t g8 = gridDim.x / 8u;
    if (bid < 8u * g8) bid = (bid % 8u) * g8 + bid / 8u;
    const uint32_t lane = threadIdx.x & 63u, rl = lane & 15u, row = lane >> 4;
    const uint32_t p = bid * 16u + (threadIdx.x >> 6) * 4u + row;
    if (p >= n) return;
    uint8_t* f = arena + (uint64_t)p * kStride;
    const uint4* src = (const uint4*)f;
    uint4 v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = ld(src + rl + 16 * k, k != 0);
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) acc = ws(v[k].w, ws(v[k].z, ws(v[k].y, ws(v[k].x, acc))));
    // row sum (4 DPP steps), as the checksum kernel
    acc += (uint32_t)__builtin_amdgcn_mov_dpp((int)acc, 0xB1, 0xF, 0xF, true);
    acc += (uint32_t)__builtin_amdgcn_mov_dpp((int)acc, 0x4E, 0xF, 0xF, true);
    acc += (uint32_t)__builtin_amdgcn_mov_dpp((int)acc, 0x141, 0xF, 0xF, true);
    acc += (uint32_t)__builtin_amdgcn_mov_dpp((int)acc, 0x140, 0xF, 0xF, true);
    const uint64_t r = ((uint64_t)p << 32) | acc;
    if (MODE == 0) {
        asm volatile("" ::"v"(acc));
    } else if (MODE == 1 || MODE == 5 || MODE == 6 || MODE == 10) {
        if (rl == 0 && (MODE != 10 || (p & 15u) == 0)) {
            if (MODE == 5) __hip_atomic_store(dense + p, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (MODE == 6) __builtin_nontemporal_store(r, dense + p);
            else dense[p] = r;
        }
    } else if (MODE == 2 || MODE == 7) {
        if (rl == 0) {
            if (MODE == 7) __hip_atomic_store(tiny + (p & 511u), r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else tiny[p & 511u] = r;
        }
    } else if (MODE == 3 || MODE == 4 || MODE == 9) {
        if (rl == 1 && (MODE != 9 || (p & 15u) == 0)) {
            uint32_t* q = (uint32_t*)(f + 24);
            if (MODE == 4) __hip_atomic_store(q, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else *q = acc;
        }
    } else if (MODE >= 11 && MODE <= 14) {
        if (rl < 4) {  // the header slot's chunk rl, one byte changed: a full 64-byte segment
            uint4 v0 = v[0];
            v0.x ^= acc & 0xFFu;
            const u32x4_t t = {v0.x, v0.y, v0.z, v0.w};
            u32x4_t* q = (u32x4_t*)f + rl;
            if (MODE == 12) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(q), "v"(t) : "memory");
            else if (MODE == 13) __builtin_nontemporal_store(t, q);
            else if (MODE == 14) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" ::"v"(q), "v"(t) : "memory");
            else *q = t;
        }
    } else if (MODE == 8) {
        // the wave's four row sums in lane 0 as one 16-byte store
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)acc, 16);
        const uint32_t a2 = (uint32_t)__builtin_amdgcn_readlane((int)acc, 32);
        const uint32_t a3 = (uint32_t)__builtin_amdgcn_readlane((int)acc, 48);
        if (lane == 0) ((uint4*)dense)[p >> 2] = make_uint4(acc, a1, a2, a3);
    }
}

// Split-mode write pass: one write per frame at frame+24 (or a 64-byte segment at frame+0), by
// cache policy: 0 plain, 1 sc1, 2 nt, 3 sc0 sc1, 4 sc0 sc1 nt, 5 64 B plain, 6 64 B nt, 7 64 B sc0 sc1 nt;
// 8: the 64-byte segment re-read (default policy) then written back whole, nt; 9: as 8 in reverse
// frame order (the header lines read last by the read pass first)
template <int POL>
__global__ __launch_bounds__(256) void apply(uint8_t* __restrict__ arena, uint32_t n,
                                             const uint64_t* __restrict__ dense) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (POL >= 5) {  // 4 lanes x 16 B per frame
        uint32_t p = t >> 2;
        const uint32_t l = t & 3u;
        if (p >= n) return;
        if (POL == 9) p = n - 1 - p;
        const uint64_t r = dense[p];
        u32x4_t v = {(uint32_t)r, (uint32_t)(r >> 32), p, l};
        u32x4_t* q = (u32x4_t*)(arena + (uint64_t)p * kStride) + l;
        if (POL >= 8) {
            v = *q;
            v.x ^= (uint32_t)r & 0xFFFFu;
            __builtin_nontemporal_store(v, q);
        } else if (POL == 6) __builtin_nontemporal_store(v, q);
        else if (POL == 7) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" ::"v"(q), "v"(v) : "memory");
        else *q = v;
        return;
    }
    const uint32_t p = t;
    if (p >= n) return;
    const uint32_t val = (uint32_t)dense[p];
    uint32_t* q = (uint32_t*)(arena + (uint64_t)p * kStride + 24);
    if (POL == 1) __hip_atomic_store(q, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (POL == 2) __builtin_nontemporal_store(val, q);
    else if (POL == 3) __hip_atomic_store(q, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else if (POL == 4) asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(q), "v"(val) : "memory");
    else *q = val;
}

template <int POL>
void run_split(uint8_t* arena, uint32_t n, uint64_t* dense, uint64_t* tiny) {
    hipEvent_t e0, e1, e2;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventCreate(&e2);
    float sr = 0, sa = 0;
    const int warm = 3, iters = 10;
    const uint32_t ga = POL >= 5 ? (4 * n + 255) / 256 : (n + 255) / 256;
    for (int it = 0; it < warm + iters; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((probe<1>), dim3((n + 15) / 16), dim3(256), 0, 0, arena, n, dense, tiny);
        (void)hipEventRecord(e1);
        hipLaunchKernelGGL((apply<POL>), dim3(ga), dim3(256), 0, 0, arena, n, dense);
        (void)hipEventRecord(e2);
        (void)hipEventSynchronize(e2);
        float m1, m2;
        (void)hipEventElapsedTime(&m1, e0, e1);
        (void)hipEventElapsedTime(&m2, e1, e2);
        if (it >= warm) { sr += m1; sa += m2; }
    }
    const double bytes = (double)n * (1500.0 + 12.0);
    printf("{\"packets\": %u, \"split_policy\": %d, \"read_us\": %.1f, \"apply_us\": %.1f, \"algo_frac\": %.4f}\n",
           n, POL, 1e3f * sr / iters, 1e3f * sa / iters, bytes / ((sr + sa) / iters * 1e-3) / 8e12);
    fflush(stdout);
}

template <int MODE>
void run(uint8_t* arena, uint32_t n, uint64_t* dense, uint64_t* tiny) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float sum = 0, best = 1e30f;
    const int warm = 3, iters = 10;
    for (int it = 0; it < warm + iters; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((probe<MODE>), dim3((n + 15) / 16), dim3(256), 0, 0, arena, n, dense, tiny);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (it >= warm) {
            sum += ms;
            if (ms < best) best = ms;
        }
    }
    const double bytes = (double)n * (1500.0 + 12.0);
    printf("{\"packets\": %u, \"mode\": %d, \"avg_us\": %.1f, \"best_us\": %.1f, \"algo_frac_avg\": %.4f}\n",
           n, MODE, 1e3f * sum / iters, 1e3f * best, bytes / (sum / iters * 1e-3) / 8e12);
    fflush(stdout);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main(int argc, char** argv) {
    for (int a = 1; a < (argc > 1 ? argc : 2); ++a) {
        const uint32_t n = (uint32_t)(argc > 1 ? atoi(argv[a]) : 4) << 20;
        uint8_t* arena;
        uint64_t *dense, *tiny;
        if (hipMalloc(&arena, (size_t)n * kStride) != hipSuccess) return 1;
        if (hipMalloc(&dense, (size_t)n * 8) != hipSuccess) return 1;
        if (hipMalloc(&tiny, 4096) != hipSuccess) return 1;
        (void)hipMemset(arena, 0x5A, (size_t)n * kStride);
        (void)hipMemset(dense, 0, (size_t)n * 8);
        (void)hipDeviceSynchronize();
        if (getenv("WRP_SPLIT")) {
            run_split<0>(arena, n, dense, tiny);
            run_split<1>(arena, n, dense, tiny);
            run_split<2>(arena, n, dense, tiny);
            run_split<3>(arena, n, dense, tiny);
            run_split<4>(arena, n, dense, tiny);
            run_split<5>(arena, n, dense, tiny);
            run_split<6>(arena, n, dense, tiny);
            run_split<7>(arena, n, dense, tiny);
            run_split<8>(arena, n, dense, tiny);
            run_split<9>(arena, n, dense, tiny);
            run_split<0>(arena, n, dense, tiny);
            (void)hipFree(arena); (void)hipFree(dense); (void)hipFree(tiny);
            continue;
        }
        run<0>(arena, n, dense, tiny);
        run<1>(arena, n, dense, tiny);
        run<2>(arena, n, dense, tiny);
        run<3>(arena, n, dense, tiny);
        run<4>(arena, n, dense, tiny);
        run<5>(arena, n, dense, tiny);
        run<6>(arena, n, dense, tiny);
        run<7>(arena, n, dense, tiny);
        run<8>(arena, n, dense, tiny);
        run<9>(arena, n, dense, tiny);
        run<10>(arena, n, dense, tiny);
        run<11>(arena, n, dense, tiny);
        run<12>(arena, n, dense, tiny);
        run<13>(arena, n, dense, tiny);
        run<14>(arena, n, dense, tiny);
        run<0>(arena, n, dense, tiny);
        (void)hipFree(arena);
        (void)hipFree(dense);
        (void)hipFree(tiny);
    }
    return 0;
}
