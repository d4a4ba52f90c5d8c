// stream_rw.hip — measurement tool (not product): cost of in-place writes inside an HBM read
// stream. 1536-byte "frames" (128-B aligned); every chunk is read and summed; the first W
// bytes of each frame are written back in place (rewriting the bytes just read), with plain,
// non-temporal (nt) or write-through (sc1) stores, as 1-, 2- or 16-byte stores.
//   hipcc --offload-arch=gfx950 -O3 tools/stream_rw.hip -o tools/stream_rw && tools/stream_rw
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// MODE: 0 none; 1 byte @24; 2 two bytes @24,@40 (separate stores); 3 16-B chunk 1;
//       4 64-B (chunks 0..3); 5 128-B (chunks 0..7); 6 16-B chunk 1 nt; 7 64-B nt; 8 128-B nt;
//       9 16-B chunk 1 sc1 (write-through)
template <int MODE>
__global__ __launch_bounds__(256) void rw(uint4* __restrict__ p, size_t n16, unsigned long long* out) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    uint64_t acc = 0;
    for (; i < n16; i += stride) {
        const uint4 v0 = p[i];
        acc += (uint64_t)v0.x + v0.y + v0.z + v0.w;
        // opaque copy: a store of the just-loaded value back to its own address is otherwise
        // removed as a dead store by the compiler (an earlier version measured exactly that)
        uint4 v = v0;
        asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
        const uint32_t c = (uint32_t)(i % 96);  // chunk within the 1536-B frame
        if (MODE == 1 && c == 1) ((uint8_t*)(p + i))[8] = (uint8_t)v.z;
        if (MODE == 2 && c == 1) ((uint8_t*)(p + i))[8] = (uint8_t)v.z;
        if (MODE == 2 && c == 2) ((uint8_t*)(p + i))[8] = (uint8_t)v.z;
        if (MODE == 3 && c == 1) p[i] = v;
        if (MODE == 4 && c < 4) p[i] = v;
        if (MODE == 5 && c < 8) p[i] = v;
        if ((MODE == 6 && c == 1) || (MODE == 7 && c < 4) || (MODE == 8 && c < 8)) {
            u32x4 t = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(t, (u32x4*)(p + i));
        }
        if (MODE == 10 && c == 1) ((uint32_t*)(p + i))[2] = v.z;                  // 4-B dword
        if (MODE == 11 && c == 1) ((uint16_t*)(p + i))[4] = (uint16_t)v.z;        // 2-B short
        // delayed by 8 iterations (~the frame read 8 grid strides ago): value rewritten as memset
        if (MODE == 12 && c == 1 && i >= 8 * stride) p[i - 8 * stride] = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
        if (MODE == 13 && c == 1 && i >= 8 * stride) ((uint32_t*)(p + i - 8 * stride))[2] = 0x01010101u;
        if (MODE == 14 && c == 1 && i >= 8 * stride) ((uint8_t*)(p + i - 8 * stride))[8] = 0x01u;
        if (MODE == 15 && c < 4 && i >= 8 * stride) p[i - 8 * stride] = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
        if (MODE == 16 && c < 8 && i >= 8 * stride) p[i - 8 * stride] = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
        if (MODE == 17 && c < 8 && i >= 64 * stride) p[i - 64 * stride] = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
        if (MODE == 18 && c == 1 && i >= 64 * stride) p[i - 64 * stride] = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
        if (MODE == 9 && c == 1) {
            __hip_atomic_store((unsigned long long*)(p + i), ((unsigned long long)v.y << 32) | v.x,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store((unsigned long long*)(p + i) + 1, ((unsigned long long)v.w << 32) | v.z,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (acc == 0x123456789ull) *out = acc;
}

template <int MODE>
float run(uint4* p, size_t n16, int grid, unsigned long long* o) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) rw<MODE><<<grid, 256>>>(p, n16, o);
    float best = 1e9;
    for (int r = 0; r < 10; ++r) {
        (void)hipEventRecord(a);
        rw<MODE><<<grid, 256>>>(p, n16, o);
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
    const char* names[] = {"none", "1B", "2x1B", "16B", "64B", "128B", "16B_nt", "64B_nt", "128B_nt", "16B_sc1",
                           "4B", "2B", "16B_late", "4B_late", "1B_late", "64B_late", "128B_late",
                           "128B_later64", "16B_later64"};
    for (int g : {2048, 8192}) {
        float t[19] = {run<0>(p, n16, g, o), run<1>(p, n16, g, o), run<2>(p, n16, g, o), run<3>(p, n16, g, o),
                       run<4>(p, n16, g, o), run<5>(p, n16, g, o), run<6>(p, n16, g, o), run<7>(p, n16, g, o),
                       run<8>(p, n16, g, o), run<9>(p, n16, g, o), run<10>(p, n16, g, o), run<11>(p, n16, g, o),
                       run<12>(p, n16, g, o), run<13>(p, n16, g, o), run<14>(p, n16, g, o),
                       run<15>(p, n16, g, o), run<16>(p, n16, g, o), run<17>(p, n16, g, o), run<18>(p, n16, g, o)};
        printf("{\"grid\": %d", g);
        for (int m = 0; m < 19; ++m) printf(", \"%s\": %.0f", names[m], bytes / t[m] / 1e6);
        printf("}\n");
    }
    return 0;
}
