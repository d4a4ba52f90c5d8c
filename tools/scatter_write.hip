// scatter_write.hip — measurement tool (not product): the cost of isolated writes, one per
// 1536-byte frame over a 1.5 GiB buffer (the checksum write-back pattern of C1), by size and
// cache policy: a pure write pass like split mode's patch pass.
//   W =   4: one dword at frame offset 24          (partial line)
//   W =  64: 4 lanes x 16 B at frame offset 0       (a full 64-byte half line)
//   W = 128: 8 lanes x 16 B at frame offset 0       (a full 128-byte line)
// policy: 0 plain (write-back), 1 sc1 (write-through), 2 nt. Best of 10 launches.
//   hipcc --offload-arch=gfx950 -O3 tools/scatter_write.hip -o tools/scatter_write && tools/scatter_write
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int W, int POL>
__global__ __launch_bounds__(256) void wr(uint8_t* __restrict__ buf, uint32_t frames, uint32_t val,
                                          uint32_t stride) {
    constexpr uint32_t LPF = W >= 16 ? W / 16 : 1;  // lanes per frame
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    const uint32_t f = t / LPF, l = t % LPF;
    if (f >= frames) return;
    uint8_t* p = buf + (uint64_t)f * stride;
    if (W == 4) {
        uint32_t* q = (uint32_t*)(p + 24);
        if (POL == 1) __hip_atomic_store(q, val + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (POL == 2) __builtin_nontemporal_store(val + f, q);
        else *q = val + f;
    } else {
        u32x4_t v = {val + f, val, f, l};
        u32x4_t* q = (u32x4_t*)(p + 16u * l);
        if (POL == 1) {
            uint64_t* q2 = (uint64_t*)q;
            __hip_atomic_store(q2, ((uint64_t)v.y << 32) | v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(q2 + 1, ((uint64_t)v.w << 32) | v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (POL == 2) {
            __builtin_nontemporal_store(v, q);
        } else {
            *q = v;
        }
    }
}

template <int W, int POL>
float run(uint8_t* buf, uint32_t frames, uint32_t stride = 1536u) {
    constexpr uint32_t LPF = W >= 16 ? W / 16 : 1;
    const uint32_t grid = (frames * LPF + 255) / 256;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int it = 0; it < 12; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((wr<W, POL>), dim3(grid), dim3(256), 0, 0, buf, frames, (uint32_t)it, stride);
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

int main(int argc, char** argv) {
    if (argc > 2) {  // session 4: scatter_write <M frames> <stride> [stride ...]: W = 4 by stride
        const uint32_t fr = (uint32_t)atoi(argv[1]) << 20;
        for (int a = 2; a < argc; ++a) {
            const uint32_t st = (uint32_t)atoi(argv[a]);
            uint8_t* b;
            if (hipMalloc(&b, (size_t)fr * st) != hipSuccess) return 1;
            (void)hipMemset(b, 1, (size_t)fr * st);
            const float t0 = run<4, 0>(b, fr, st), t1 = run<4, 1>(b, fr, st), t2 = run<64, 0>(b, fr, st);
            printf("{\"frames\": %u, \"stride\": %u, \"dword_plain_us\": %.1f, \"dword_sc1_us\": %.1f, "
                   "\"seg64_plain_us\": %.1f}\n", fr, st, 1e3f * t0, 1e3f * t1, 1e3f * t2);
            (void)hipFree(b);
        }
        return 0;
    }
    const uint32_t frames = 1u << 20;  // C1: 1M frames of 1536 bytes
    uint8_t* buf;
    if (hipMalloc(&buf, (size_t)frames * 1536u) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, (size_t)frames * 1536u);
    printf("| write per frame | plain us | sc1 (write-through) us | nt us |\n|---|---|---|---|\n");
    printf("| 4 B (dword at 24) | %.1f | %.1f | %.1f |\n", 1e3f * run<4, 0>(buf, frames),
           1e3f * run<4, 1>(buf, frames), 1e3f * run<4, 2>(buf, frames));
    printf("| 64 B (full half line) | %.1f | %.1f | %.1f |\n", 1e3f * run<64, 0>(buf, frames),
           1e3f * run<64, 1>(buf, frames), 1e3f * run<64, 2>(buf, frames));
    printf("| 128 B (full line) | %.1f | %.1f | %.1f |\n", 1e3f * run<128, 0>(buf, frames),
           1e3f * run<128, 1>(buf, frames), 1e3f * run<128, 2>(buf, frames));
    (void)hipFree(buf);
    return 0;
}
