// exit_probe.hip — measurement tool (not product): what a launch costs whose workgroups read a
// device flag and exit at once, by grid shape; and a one-workgroup descriptor-sample prepass.
// Decides whether kUpdateAuto can pick its launch shape on the device.
//   hipcc --offload-arch=gfx950 -O3 tools/r03/exit_probe.hip -o tools/r03/exit_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct Desc { uint32_t off16, len; };

__global__ void exit_kernel(const int* flag, int me, const Desc* d, uint32_t n, uint8_t* out) {
    typedef const __attribute__((address_space(4))) int ci;
    const int f = *(ci*)flag;
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const Desc x = d[w < n ? w : 0];
    if (f != me) return;
    if (threadIdx.x == 0 && x.len == 0xFFFFFFFFu) out[0] = 1;
}

// one workgroup: lengths of a strided sample of `samples` descriptors -> mean -> shape flag
__global__ __launch_bounds__(256) void sample_kernel(const Desc* d, uint32_t n, uint32_t samples, int* flag) {
    __shared__ uint64_t part[256];
    uint64_t s = 0;
    const uint64_t step = n > samples ? n / samples : 1;
    const uint32_t m = n < samples ? n : samples;
    for (uint32_t i = threadIdx.x; i < m; i += 256) s += d[i * step].len;
    part[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) part[threadIdx.x] += part[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const uint64_t mean = part[0] / (m ? m : 1);
        *flag = mean < 800 ? 0 : (mean < 1200 ? 1 : 2);
    }
}

int main() {
    const uint32_t n = 1u << 20;
    Desc* d; int* flag; uint8_t* out;
    CK(hipMalloc(&d, n * sizeof(Desc)));
    CK(hipMalloc(&flag, 4));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(d, 0, n * sizeof(Desc)));
    CK(hipMemset(flag, 0, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    struct Shape { const char* name; uint32_t grid, block; } shapes[] = {
        {"tiny n/8 x 64", n / 8, 64}, {"short n/4 x 64", n / 4, 64}, {"long n/16 x 256", n / 16, 256},
        {"tiny4M n/8 x 64", 4 * n / 8, 64}, {"long4M n/16 x 256", 4 * n / 16, 256}};
    for (int rep = 0; rep < 2; ++rep) {
        for (auto& s : shapes) {
            const int it = 50;
            for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(exit_kernel, dim3(s.grid), dim3(s.block), 0, 0, flag, 9, d, n, out);
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < it; ++i) hipLaunchKernelGGL(exit_kernel, dim3(s.grid), dim3(s.block), 0, 0, flag, 9, d, n, out);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            printf("{\"probe\": \"exit\", \"shape\": \"%s\", \"us_per_launch\": %.2f}\n", s.name, ms * 1e3 / it);
        }
        for (uint32_t samples : {1024u, 4096u, 16384u}) {
            const int it = 50;
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < it; ++i) hipLaunchKernelGGL(sample_kernel, dim3(1), dim3(256), 0, 0, d, n, samples, flag);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            printf("{\"probe\": \"sample\", \"samples\": %u, \"us_per_launch\": %.2f}\n", samples, ms * 1e3 / it);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
