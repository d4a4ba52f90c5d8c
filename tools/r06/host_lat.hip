// host_lat.hip — measurement tool (not product): where a per-RX-burst call's ~20 µs go.
// Times, median of 2000 repetitions each, on one stream:
//   launch_sync    an empty kernel, hipStreamSynchronize
//   launch_event   an empty kernel, hipEventRecord, hipEventSynchronize (what nfcs_update_host waits on)
//   launch_flag    a one-wave kernel that stores a sequence number into host-mapped pinned memory with a
//                  system-scope release (a vector store); the host spins on that word, no HIP call
//   read_flag      the same kernel after reading 64 descriptors' worth (512 B) of pinned host memory first
//   update_host    nfcs_update_host on 64 / 256 C1 frames of a pinned arena (direct chunks)
//   update_zc      the same with NFCS_HOST_ZERO_COPY
// Prints one JSON line. Built by hipcc against the product library (tools/r06/build_host_lat.sh).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "nfcs.h"

__global__ void empty_kernel() {}

__global__ void flag_kernel(uint64_t* flag, uint64_t seq, const uint4* host_src, uint32_t n16) {
    uint32_t x = 0;
    for (uint32_t i = threadIdx.x; i < n16; i += 64) x ^= host_src[i].x;
    if (x == 0x9E3779B9u) seq = 0;  // keeps the reads
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double med(std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    using clk = std::chrono::steady_clock;
    constexpr int R = 2000;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    uint64_t* flag = nullptr;
    uint4* src = nullptr;
    (void)hipHostMalloc((void**)&flag, 4096, hipHostMallocMapped);
    (void)hipHostMalloc((void**)&src, 1 << 20, hipHostMallocMapped);
    uint64_t* dflag = nullptr;
    uint4* dsrc = nullptr;
    (void)hipHostGetDevicePointer((void**)&dflag, flag, 0);
    (void)hipHostGetDevicePointer((void**)&dsrc, src, 0);
    *(volatile uint64_t*)flag = 0;
    auto time = [&](auto&& body) {
        std::vector<double> us;
        for (int i = 0; i < 50; ++i) body(i);
        for (int i = 0; i < R; ++i) {
            auto t0 = clk::now();
            body(i);
            us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
        }
        return med(us);
    };
    const double launch_sync = time([&](int) {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
        (void)hipStreamSynchronize(st);
    });
    const double launch_event = time([&](int) {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
        (void)hipEventRecord(ev, st);
        (void)hipEventSynchronize(ev);
    });
    uint64_t seq = 1;
    const double launch_flag = time([&](int) {
        const uint64_t s = ++seq;
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, st, dflag, s, dsrc, 0u);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != s) __builtin_ia32_pause();
    });
    const double read_flag = time([&](int) {
        const uint64_t s = ++seq;
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, st, dflag, s, dsrc, 32u);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != s) __builtin_ia32_pause();
    });
    (void)hipStreamSynchronize(st);

    // nfcs_update_host on C1 frames in a pinned arena (128-byte aligned 1536-byte slots)
    nfcs_ctx* c = nullptr;
    if (nfcs_ctx_create(0, &c)) return 1;
    const uint32_t n = 4096;
    std::vector<nfcs_desc> desc(n);
    uint64_t bytes = 0;
    nfcs_layout_config(NFCS_CFG_C1_1500B_UDP, 20250620ull, 0, n, 128, desc.data(), &bytes);
    void *d_arena = nullptr, *d_desc = nullptr, *h_arena = nullptr;
    nfcs_device_alloc(c, bytes, &d_arena);
    nfcs_device_alloc(c, n * sizeof(nfcs_desc), &d_desc);
    nfcs_host_alloc(c, bytes, &h_arena);
    nfcs_memcpy_h2d(c, d_desc, desc.data(), n * sizeof(nfcs_desc));
    nfcs_gen_config_device(c, NFCS_CFG_C1_1500B_UDP, 20250620ull, 0, n, (uint8_t*)d_arena, bytes, (nfcs_desc*)d_desc, nullptr);
    nfcs_stream_sync(c, nullptr);
    nfcs_memcpy_d2h(c, h_arena, d_arena, bytes);
    double uh[2], uz[2];
    const uint32_t sizes[2] = {64, 256};
    for (int k = 0; k < 2; ++k) {
        const uint32_t b = sizes[k];
        uh[k] = time([&](int i) {
            nfcs_update_host(c, (uint8_t*)h_arena, bytes, desc.data() + (size_t)(i % (n / b)) * b, b, nullptr, 0);
        });
        uz[k] = time([&](int i) {
            nfcs_update_host(c, (uint8_t*)h_arena, bytes, desc.data() + (size_t)(i % (n / b)) * b, b, nullptr,
                             NFCS_HOST_ZERO_COPY);
        });
    }
    std::printf("{\"reps\": %d, \"launch_sync_us\": %.2f, \"launch_event_us\": %.2f, \"launch_flag_us\": %.2f, "
                "\"read512_flag_us\": %.2f, \"update_host_64_us\": %.2f, \"update_host_256_us\": %.2f, "
                "\"update_zc_64_us\": %.2f, \"update_zc_256_us\": %.2f}\n",
                R, launch_sync, launch_event, launch_flag, read_flag, uh[0], uh[1], uz[0], uz[1]);
    nfcs_host_free(c, h_arena);
    nfcs_device_free(c, d_arena);
    nfcs_device_free(c, d_desc);
    nfcs_ctx_destroy(c);
    return 0;
}
