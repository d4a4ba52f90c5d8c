// host_pipe — measurement tool (not product): does the scattered-frame gather overlap the H2D copy?
// host_phases measured, for BASELINE C1's 1M frames in one heap buffer each, the product call at
// 51.5 ms = gather alone (22.0 ms, 8 threads) + H2D alone (27.6 ms) + write-back (1.5 ms): no
// overlap. This replays the product's pipeline without the kernel: two 64 MiB pinned slots; for
// chunk k: wait for the H2D of chunk k-2, gather chunk k (8 workers + the caller, non-temporal
// stores), then queue its H2D on stream k % 2. Variants (wall clock, best of R, frames restored
// before each):
//   gather     the gathers alone           h2d        the H2D copies alone
//   pipe       the pipeline                pipe_pin   the pipeline, workers pinned to the GPU's node
//   pipe_loc   the pipeline, pinned workers, frames first touched on the GPU's node
//   pipe_sdma  as pipe, one stream for every copy (a single copy queue)
// Build: tools/r05/build_host_pipe.sh (hipcc, host code only). One JSON line.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static void copy_nt(uint8_t* dst, const uint8_t* src, uint64_t len) {
    uint64_t k = 0;
    for (; k + 64 <= len; k += 64) {
        u32x4 a, b, c, d;
        memcpy(&a, src + k, 16); memcpy(&b, src + k + 16, 16);
        memcpy(&c, src + k + 32, 16); memcpy(&d, src + k + 48, 16);
        __builtin_nontemporal_store(a, (u32x4*)(dst + k));
        __builtin_nontemporal_store(b, (u32x4*)(dst + k + 16));
        __builtin_nontemporal_store(c, (u32x4*)(dst + k + 32));
        __builtin_nontemporal_store(d, (u32x4*)(dst + k + 48));
    }
    for (; k + 16 <= len; k += 16) {
        u32x4 a;
        memcpy(&a, src + k, 16);
        __builtin_nontemporal_store(a, (u32x4*)(dst + k));
    }
    if (k < len) {
        u32x4 t = {0u, 0u, 0u, 0u};
        memcpy(&t, src + k, len - k);
        __builtin_nontemporal_store(t, (u32x4*)(dst + k));
    }
}

// a persistent pool: run(k, fn) runs fn(0..k-1) over the workers and the caller
class Pool {
public:
    void start(int n, const cpu_set_t* cpus) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this, cpus] { loop(cpus); });
    }
    void stop() {
        {
            std::lock_guard<std::mutex> l(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
        th_.clear();
        quit_ = false;
    }
    int size() const { return (int)th_.size(); }
    template <class F>
    void run(int k, const F& fn) {
        std::unique_lock<std::mutex> l(mu_);
        call_ = [](const void* f, int i) { (*(const F*)f)(i); };
        job_ = &fn;
        parts_ = k;
        next_ = 0;
        pending_ = k;
        ++gen_;
        cv_.notify_all();
        take(l);
        done_.wait(l, [&] { return pending_ == 0; });
    }

private:
    void take(std::unique_lock<std::mutex>& l) {
        while (next_ < parts_) {
            const int i = next_++;
            auto c = call_;
            auto f = job_;
            l.unlock();
            c(f, i);
            l.lock();
            if (--pending_ == 0) done_.notify_all();
        }
    }
    void loop(const cpu_set_t* cpus) {
        if (cpus) pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), cpus);
        std::unique_lock<std::mutex> l(mu_);
        uint64_t seen = 0;
        for (;;) {
            cv_.wait(l, [&] { return quit_ || (gen_ != seen && next_ < parts_); });
            if (quit_) return;
            take(l);
            seen = gen_;
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    void (*call_)(const void*, int) = nullptr;
    const void* job_ = nullptr;
    int parts_ = 0, next_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

static bool gpu_node_cpus(cpu_set_t* set, int* node_out) {
    char bus[64];
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), 0) != hipSuccess) return false;
    for (char* p = bus; *p; ++p) *p = (char)tolower(*p);
    char path[256];
    std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE* f = std::fopen(path, "r");
    if (!f) return false;
    int node = -1;
    if (std::fscanf(f, "%d", &node) != 1) node = -1;
    std::fclose(f);
    *node_out = node;
    if (node < 0) return false;
    std::snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
    f = std::fopen(path, "r");
    if (!f) return false;
    CPU_ZERO(set);
    long a, b;
    char sep;
    while (std::fscanf(f, "%ld", &a) == 1) {
        b = a;
        if (std::fscanf(f, "%c", &sep) == 1 && sep == '-') {
            if (std::fscanf(f, "%ld", &b) != 1) break;
            if (std::fscanf(f, "%c", &sep) != 1) sep = 0;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET((int)c, set);
        if (sep != ',') break;
    }
    std::fclose(f);
    // keep only CPUs this process may run on
    cpu_set_t mine;
    if (sched_getaffinity(0, sizeof(mine), &mine) == 0) CPU_AND(set, set, &mine);
    return CPU_COUNT(set) > 0;
}

int main(int argc, char** argv) {
    using clk = std::chrono::steady_clock;
    const size_t n = argc > 1 ? std::stoul(argv[1]) : (1u << 20);
    const size_t reps = argc > 2 ? std::stoul(argv[2]) : 5;
    const int workers = argc > 3 ? std::stoi(argv[3]) : 8;
    const uint32_t L = 1500;
    CK(hipSetDevice(0));
    cpu_set_t node_set;
    int node = -1;
    const bool have_node = gpu_node_cpus(&node_set, &node);

    std::vector<uint8_t> pristine(L);
    for (uint32_t i = 0; i < L; ++i) pristine[i] = (uint8_t)(i * 7 + 1);
    std::vector<uint8_t*> frames(n);
    auto alloc_frames = [&](Pool& pool, int k) {
        for (auto*& f : frames) f = new uint8_t[32 + 1536];
        pool.run(k, [&](int t) {  // first touch by the pool's threads
            for (size_t i = n * t / k; i < n * (t + 1) / k; ++i) memset(frames[i], 0, 32 + 1536);
        });
    };
    auto free_frames = [&] {
        for (auto*& f : frames) delete[] f;
    };

    const size_t slot = 64u << 20, per = slot / 1504;
    uint8_t* stage = nullptr;
    CK(hipHostMalloc((void**)&stage, 2 * slot, hipHostMallocDefault));
    memset(stage, 0, 2 * slot);
    void* dev = nullptr;
    CK(hipMalloc(&dev, (n + per) * 1504));
    hipStream_t st[2];
    hipEvent_t ev[2];
    for (int i = 0; i < 2; ++i) {
        CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }

    std::string out = "{";
    char tmp[256];
    std::snprintf(tmp, sizeof(tmp), "\"gpu_node\": %d, \"node_cpus\": %d, \"workers\": %d", node,
                  have_node ? CPU_COUNT(&node_set) : 0, workers);
    out += tmp;
    auto put = [&](const char* k, double s) {
        std::snprintf(tmp, sizeof(tmp), ", \"%s\": {\"ms\": %.3f, \"GBps\": %.2f}", k, s * 1e3, (double)n * L / s / 1e9);
        out += tmp;
    };

    for (int variant = 0; variant < 3; ++variant) {
        // 0: unpinned pool, frames touched by it; 1: pinned pool, frames touched by an unpinned pool;
        // 2: pinned pool, frames touched by it (on the GPU's node)
        Pool pool, toucher;
        pool.start(workers, (variant >= 1 && have_node) ? &node_set : nullptr);
        toucher.start(workers, nullptr);
        alloc_frames(variant == 1 ? toucher : pool, workers + 1);
        const int parts = workers + 1;
        auto restore = [&] {
            pool.run(parts, [&](int t) {
                for (size_t i = n * t / parts; i < n * (t + 1) / parts; ++i) memcpy(frames[i] + 32, pristine.data(), L);
            });
        };
        auto gather = [&](size_t i0, size_t m, uint8_t* d) {
            pool.run(parts, [&](int t) {
                const size_t j0 = m * t / parts, j1 = m * (t + 1) / parts;
                for (size_t j = j0; j < j1; ++j) {
                    if (j + 4 < j1) {
                        __builtin_prefetch(frames[i0 + j + 4] + 32, 0, 0);
                        __builtin_prefetch(frames[i0 + j + 4] + 96, 0, 0);
                        __builtin_prefetch(frames[i0 + j + 4] + 160, 0, 0);
                    }
                    copy_nt(d + j * 1504, frames[i0 + j] + 32, L);
                }
                __builtin_ia32_sfence();
            });
        };
        auto best = [&](auto&& fn) {
            double b = 1e30;
            for (size_t r = 0; r < reps; ++r) {
                restore();
                const auto t0 = clk::now();
                fn();
                b = std::min(b, std::chrono::duration<double>(clk::now() - t0).count());
            }
            return b;
        };
        auto pipe = [&](bool one_stream) {
            bool used[2] = {false, false};
            for (size_t i0 = 0, k = 0; i0 < n; i0 += per, ++k) {
                const int s = (int)(k & 1);
                if (used[s]) CK(hipEventSynchronize(ev[s]));
                const size_t m = std::min(per, n - i0);
                gather(i0, m, stage + s * slot);
                hipStream_t q = one_stream ? st[0] : st[s];
                CK(hipMemcpyAsync((uint8_t*)dev + i0 * 1504, stage + s * slot, m * 1504, hipMemcpyHostToDevice, q));
                CK(hipEventRecord(ev[s], q));
                used[s] = true;
            }
            CK(hipStreamSynchronize(st[0]));
            CK(hipStreamSynchronize(st[1]));
        };
        if (variant == 0) {
            put("gather", best([&] {
                for (size_t i0 = 0, k = 0; i0 < n; i0 += per, ++k) gather(i0, std::min(per, n - i0), stage + (k & 1) * slot);
            }));
            put("h2d", best([&] {
                for (size_t i0 = 0, k = 0; i0 < n; i0 += per, ++k)
                    CK(hipMemcpyAsync((uint8_t*)dev + i0 * 1504, stage + (k & 1) * slot, std::min(per, n - i0) * 1504,
                                      hipMemcpyHostToDevice, st[k & 1]));
                CK(hipStreamSynchronize(st[0]));
                CK(hipStreamSynchronize(st[1]));
            }));
            pipe(false);  // warm
            put("pipe", best([&] { pipe(false); }));
            put("pipe_sdma", best([&] { pipe(true); }));
        } else if (variant == 1) {
            put("pipe_pin", best([&] { pipe(false); }));
        } else {
            put("gather_loc", best([&] {
                for (size_t i0 = 0, k = 0; i0 < n; i0 += per, ++k) gather(i0, std::min(per, n - i0), stage + (k & 1) * slot);
            }));
            put("pipe_loc", best([&] { pipe(false); }));
        }
        pool.stop();
        toucher.stop();
        free_frames();
    }
    out += "}";
    std::printf("%s\n", out.c_str());
    return 0;
}
