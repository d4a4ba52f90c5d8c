// stride_read.hip — measurement tool (not product): the rate of isolated line reads, the access
// pattern of the flow-key kernel (one 128-byte header line per 1536-byte frame)
// and of the checksum stores (one line per frame).
//   8 lanes read one 128-B line (16 B each); lines lie STRIDE bytes apart over a 1.5 GB buffer;
//   K lines per 8-lane row in flight (all loads issued, then summed). Best of 10 launches.
//   hipcc --offload-arch=gfx950 -O3 tools/stride_read.hip -o tools/stride_read && tools/stride_read
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int K>
__global__ __launch_bounds__(256) void rd(const uint4* __restrict__ a, uint64_t lines, uint64_t stride16,
                                          uint32_t* __restrict__ out) {
    const uint32_t rl = threadIdx.x & 7u;
    const uint64_t row = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 3;  // 32 rows per block
    const uint64_t rows = (uint64_t)gridDim.x * 32;
    uint32_t acc = 0;
    for (uint64_t l0 = row; l0 < lines; l0 += rows * K) {
        u32x4_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t l = l0 + (uint64_t)k * rows;
            v[k] = (l < lines) ? __builtin_nontemporal_load((const u32x4_t*)(a + l * stride16 + rl))
                               : u32x4_t{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc += v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;  // keeps the loads live
}

template <int K>
float run(const uint4* a, uint64_t lines, uint64_t stride16, uint32_t* out, int grid) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int it = 0; it < 12; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(rd<K>, dim3(grid), dim3(256), 0, 0, a, lines, stride16, out);
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
    const size_t bytes = (size_t)1536 << 20;  // 1.5 GiB, past the 256 MB MALL
    uint4* a;
    uint32_t* out;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    printf("| stride B | grid | G lines/s K=1 | K=2 | K=4 | GB/s of lines (best) |\n|---|---|---|---|---|---|\n");
    for (uint64_t stride : {128ull, 256ull, 512ull, 1024ull, 1536ull, 3072ull, 9216ull}) {
        const uint64_t lines = bytes / stride;
        for (int grid : {2048, 8192, 32768}) {
            const float t1 = run<1>(a, lines, stride / 16, out, grid);
            const float t2 = run<2>(a, lines, stride / 16, out, grid);
            const float t4 = run<4>(a, lines, stride / 16, out, grid);
            float tb = t1 < t2 ? t1 : t2;
            tb = tb < t4 ? tb : t4;
            printf("| %llu | %d | %.1f | %.1f | %.1f | %.0f |\n", (unsigned long long)stride, grid,
                   lines / (t1 * 1e6), lines / (t2 * 1e6), lines / (t4 * 1e6), lines * 128.0 / (tb * 1e6));
        }
    }
    (void)hipFree(a);
    (void)hipFree(out);
    return 0;
}
