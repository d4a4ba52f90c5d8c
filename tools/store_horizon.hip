// store_horizon.hip — measurement tool (not product): how long after a line is read can it
// be written in place without slowing the read stream? 1536-byte frames; every chunk is read
// and summed; one dword (or byte) per frame is written D grid-strides after it was read.
//   hipcc --offload-arch=gfx950 -O3 tools/store_horizon.hip -o tools/store_horizon
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int D, int W>  // W: 0 none, 1 byte, 4 dword, 5 re-load + dependent dword
__global__ __launch_bounds__(256) void rw(uint4* __restrict__ p, size_t n16, unsigned long long* out) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    uint64_t acc = 0;
    for (; i < n16; i += stride) {
        const uint4 v = p[i];
        acc += (uint64_t)v.x + v.y + v.z + v.w;
        if (W != 0 && i >= (size_t)D * stride) {
            const size_t j = i - (size_t)D * stride;
            if (j % 96 == 1) {
                if (W == 4) ((uint32_t*)(p + j))[2] = 0x01010101u;
                if (W == 1) ((uint8_t*)(p + j))[8] = 0x01u;
                if (W == 5) {  // re-load the chunk, then a dependent dword store
                    const uint4 r = p[j];
                    ((uint32_t*)(p + j))[2] = r.z | 0x01010101u;
                }
            }
        }
    }
    if (acc == 0x123456789ull) *out = acc;
}

template <int D, int W>
float run(uint4* p, size_t n16, int grid, unsigned long long* o) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) rw<D, W><<<grid, 256>>>(p, n16, o);
    float best = 1e9;
    for (int r = 0; r < 10; ++r) {
        (void)hipEventRecord(a);
        rw<D, W><<<grid, 256>>>(p, n16, o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best;
}

int main() {
    const size_t bytes = 1536ull * 1048576ull;
    uint4* p;
    unsigned long long* o;
    (void)hipMalloc(&p, bytes);
    (void)hipMalloc(&o, 8);
    (void)hipMemset(p, 1, bytes);
    const size_t n16 = bytes / 16;
    for (int g : {1024, 2048}) {
        const double mb = g * 256.0 * 16 / 1048576.0;
        printf("{\"grid\": %d, \"stride_MiB\": %.0f, \"none\": %.0f", g, mb, bytes / run<0, 0>(p, n16, g, o) / 1e6);
#define NFCS_H(D)                                                                              \
        printf(", \"dw_d%d\": %.0f, \"b_d%d\": %.0f, \"reld_d%d\": %.0f", D,                  \
               bytes / run<D, 4>(p, n16, g, o) / 1e6, D, bytes / run<D, 1>(p, n16, g, o) / 1e6, D, \
               bytes / run<D, 5>(p, n16, g, o) / 1e6);
        NFCS_H(0) NFCS_H(1) NFCS_H(2) NFCS_H(3) NFCS_H(4) NFCS_H(6) NFCS_H(8) NFCS_H(16)
        printf("}\n");
    }
    return 0;
}
