// stream_copy.hip — measurement tool (not product): read + write stream ceilings on one MI355X,
// the reference point for kernels that rewrite whole frames (VLAN push/pop, §11 of DESIGN.md).
//   mode 0: in-place rewrite — every 16-byte chunk is read and written back to its address
//   mode 1: copy — read buffer A, write buffer B
//   mode 2: in-place rewrite with 4 chunks per lane in flight (loads first, then stores)
//   mode 3: copy with 4 chunks per lane in flight
//   mode 4: as 2 with write-through (sc1) stores;  mode 5: as 2 with non-temporal stores
// GB/s = (bytes read + bytes written) / kernel time, best of 10 launches (HIP events).
//   hipcc --offload-arch=gfx950 -O3 tools/stream_copy.hip -o tools/stream_copy && tools/stream_copy
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// MODE 4: in-place rewrite, 4 in flight, write-through (sc1) dwordx4 stores (+ s_nop for the
// wide-store data hazard); MODE 5: the same with non-temporal stores
template <int MODE>
__device__ __forceinline__ void put(uint4* p, const uint4& v) {
    if (MODE == 4) {
        const u32x4_t t = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(t) : "memory");
    } else if (MODE == 5) {
        __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, (u32x4_t*)p);
    } else {
        *p = v;
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void rw(uint4* __restrict__ a, uint4* __restrict__ b, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    uint4* dst = (MODE == 1 || MODE == 3) ? b : a;  // 4, 5: in place
    if (MODE <= 1) {  // 0, 1: one chunk per lane at a time
        for (; i < n16; i += stride) {
            uint4 v = a[i];
            asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));  // opaque: not a dead store
            dst[i] = v;
        }
    } else {
        for (; i < n16; i += 4 * stride) {
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = (i + k * stride < n16) ? a[i + k * stride] : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                asm volatile("" : "+v"(v[k].x), "+v"(v[k].y), "+v"(v[k].z), "+v"(v[k].w));
                if (i + k * stride < n16) put<MODE>(dst + i + k * stride, v[k]);
            }
        }
    }
}

template <int MODE>
float run(uint4* a, uint4* b, size_t n16, int grid) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int it = 0; it < 12; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(rw<MODE>, dim3(grid), dim3(256), 0, 0, a, b, n16);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (it >= 2 && ms < best) best = ms;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return best;
}

int main() {
    const size_t bytes = (size_t)1504 << 20;  // 1.5 GB per buffer, past the 256 MB MALL
    const size_t n16 = bytes / 16;
    uint4 *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 2, bytes);
    printf("| grid | in-place rewrite | copy | in-place, 4 in flight | copy, 4 in flight | in-place, 4 in flight, sc1 stores | ... nt stores |\n");
    printf("|---|---|---|---|---|---|---|\n");
    for (int grid : {512, 1024, 2048, 4096, 8192}) {
        const double gb = 2.0 * bytes / 1e9;
        printf("| %d | %.0f | %.0f | %.0f | %.0f | %.0f | %.0f |\n", grid, gb / (run<0>(a, b, n16, grid) * 1e-3),
               gb / (run<1>(a, b, n16, grid) * 1e-3), gb / (run<2>(a, b, n16, grid) * 1e-3),
               gb / (run<3>(a, b, n16, grid) * 1e-3), gb / (run<4>(a, b, n16, grid) * 1e-3),
               gb / (run<5>(a, b, n16, grid) * 1e-3));
    }
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
}
