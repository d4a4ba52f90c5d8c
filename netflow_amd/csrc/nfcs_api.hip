// nfcs_api.hip — the C ABI (include/nfcs.h) over the gfx950 kernels: per-device context,
// argument checking, the device-resident entry point, the host-memory pipeline (pinned
// staging ring, H2D / kernel / D2H overlapped on two streams), synthetic batches, digests.
//
// Boundary being replaced: netflow::Packet::update_checksums() (packet.hpp:722-890), a void
// member that never throws and silently skips malformed packets. Here every entry point returns
// an int (0 or a negative NFCS_E*), never throws, and reports per-packet outcomes as status bytes.
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "nfcs_internal.h"

// Pinned host memory for the staging ring, on the GPU's NUMA node when that is known: mmap'd,
// bound to the node (mbind, MPOL_PREFERRED), faulted in there, then registered with HIP; else
// hipHostMalloc.
struct HostBlock {
    void* p = nullptr;
    size_t bytes = 0;
    bool mapped = false;  // mmap + hipHostRegister (free with hipHostUnregister + munmap)
};

// A fixed set of host threads for the host path's staging copies, gathers and checksum write-back,
// pinned to the GPU's NUMA node (round 5: started once with the staging ring, instead of threads
// spawned per copy). run(k, fn) runs fn(0) .. fn(k-1) over the workers and the calling thread and
// returns when all are done; with no worker (none could be started) the caller runs them all.
// Never throws: a thread that cannot be started is simply not there.
class Workers {
public:
    ~Workers() { stop(); }
    void start(int n, const cpu_set_t* cpus) noexcept {
        for (int i = 0; i < n; ++i) {
            try {
                th_.emplace_back([this, cpus] { loop(cpus); });
            } catch (...) {
                break;
            }
        }
    }
    void stop() noexcept {
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
    // fn is called by reference, never copied (no allocation: nothing here can throw)
    template <class F>
    void run(int k, const F& fn) noexcept {
        if (k <= 1 || th_.empty()) {
            for (int i = 0; i < k; ++i) fn(i);
            return;
        }
        run_erased(k, [](const void* f, int i) { (*(const F*)f)(i); }, &fn);
    }

private:
    void run_erased(int k, void (*call)(const void*, int), const void* fn) noexcept {
        std::unique_lock<std::mutex> l(mu_);
        call_ = call;
        job_ = fn;
        parts_ = k;
        next_ = 0;
        pending_ = k;
        ++gen_;
        cv_.notify_all();
        take(l);  // the caller works too
        done_.wait(l, [&] { return pending_ == 0; });
        job_ = nullptr;
    }
    void take(std::unique_lock<std::mutex>& l) {
        while (next_ < parts_) {
            const int i = next_++;
            void (*const call)(const void*, int) = call_;
            const void* const f = job_;
            l.unlock();
            call(f, i);
            l.lock();
            if (--pending_ == 0) done_.notify_all();
        }
    }
    void loop(const cpu_set_t* cpus) {
        if (cpus) (void)pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), cpus);
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

struct nfcs_ctx {
    nfcs::DevInfo di;
    int numa_node = -1;     // the GPU's NUMA node (sysfs), -1 if unknown
    bool numa_local = false;  // staging memory bound to it
    bool have_cpus = false;   // copy threads pinned to its CPUs
    cpu_set_t node_cpus;
    HostBlock hb[2];
    hipStream_t stream = nullptr;
    // host pipeline (nfcs_update_host)
    static constexpr int kSlots = 2;
    static constexpr size_t kStageBytes = size_t(64) << 20;  // arena bytes per staging slot
    bool host_ready = false;  // every staging slot allocated (ensure_host_pipeline)
    hipStream_t hs[kSlots] = {nullptr, nullptr};
    hipEvent_t done[kSlots] = {nullptr, nullptr};    // a slot's chunk finished (records / frames back)
    hipEvent_t staged[kSlots] = {nullptr, nullptr};  // a slot's host arena and descriptors copied in
    size_t stage_bytes = 0;   // arena bytes per slot
    uint32_t stage_pkts = 0;  // descriptors per slot
    int copy_threads = 8;     // host threads for pageable <-> pinned staging copies
    Workers workers;          // copy_threads - 1 of them (the calling thread is the last)
    uint8_t* d_arena[kSlots] = {nullptr, nullptr};
    nfcs_desc* d_desc[kSlots] = {nullptr, nullptr};
    uint8_t* d_status[kSlots] = {nullptr, nullptr};
    nfcs_patch* d_patch[kSlots] = {nullptr, nullptr};
    // direct chunks' completion flags (nfcs::DoneReq): per slot a host-mapped word on its own 64-byte
    // line (done_host[8 s]), a device counter of finished workgroups, and the count the slot's next
    // launch starts from; wait_for[s] != 0: the chunk in slot s signals through its flag
    uint64_t* done_host = nullptr;
    uint64_t* done_dev = nullptr;
    uint64_t* done_ctr = nullptr;
    uint64_t done_base[kSlots] = {0, 0};
    int slot_wait[kSlots] = {0, 0};  // 0: the slot's chunk is waited for on its event; 1: on its flag; 2: flag seen
    uint8_t* z_block[kSlots] = {nullptr, nullptr};  // the pinned block of each slot as the GPU addresses it
                                                    // (direct chunks; null: not mapped, DMA only)
    uint8_t* h_arena[kSlots] = {nullptr, nullptr};  // pinned
    nfcs_desc* h_desc[kSlots] = {nullptr, nullptr};
    uint8_t* h_status[kSlots] = {nullptr, nullptr};
    nfcs_patch* h_patch[kSlots] = {nullptr, nullptr};
    uint64_t* d_digest = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // patch records of the waves that defer their stores (kUpdateAuto without a caller d_patch),
    // grown on demand; its last user ran on ws_stream (ws_own: the context's own stream). ws_ev
    // marks that user's write pass: recorded by the call itself on a caller's stream, and only when
    // another stream comes along on the context's own one (acquire_ws)
    nfcs_patch* ws = nullptr;
    size_t ws_cap = 0;  // records
    hipEvent_t ws_ev = nullptr;
    hipStream_t ws_stream = nullptr;
    bool ws_used = false;
    bool ws_own = false;
    uint32_t slot_bytes = 0;  // launch-shape hint (nfcs_ctx_set_slot_bytes); 0 = arena_bytes / n
    // the footprint observations (launch_shape): kObsSlots host-mapped 64-bit slots the kernels
    // write ({generation, mean}), one per recently seen burst (descriptor array, n, arena bytes),
    // least recently used replaced; so calls rotating over a few bursts (a ring's descriptor arrays,
    // the bench's batches) each adapt, and a late sample of a replaced burst is ignored
    static constexpr int kObsSlots = 8;
    uint64_t* obs_host = nullptr;
    uint64_t* obs_dev = nullptr;
    struct ObsBurst { const void* desc; uint32_t n; uint64_t bytes; uint32_t gen; uint64_t used; };
    ObsBurst obs_burst[kObsSlots] = {};
    uint32_t obs_gen = 0;   // the last generation handed out (0: never; slots start empty)
    uint64_t obs_clock = 0;
};

namespace {

thread_local int g_last_hip = 0;

// The deferred-store workspace for a launch of n packets on `st`. A launch on another stream
// than the previous user first waits (on the device) for that user's write pass, so calls on one
// context from several streams never overwrite each other's records; growing it waits on the host.
// A previous user on the context's own stream gets its event here, when it is needed: that stream
// lives as long as the context, and an event recorded now follows all its work. So back-to-back
// calls on one stream queue nothing between their kernels (an event per call cost C1 ~6 µs of idle
// GPU between calls, 1.5-2%; round 3, profiles/r03_s3_ab_ws_event.jsonl).
hipError_t wait_ws_user(nfcs_ctx* c, hipStream_t st) {
    if (c->ws_own) {
        hipError_t e = hipEventRecord(c->ws_ev, c->stream);
        if (e != hipSuccess) return e;
    }
    return st ? hipStreamWaitEvent(st, c->ws_ev, 0) : hipEventSynchronize(c->ws_ev);
}

hipError_t acquire_ws(nfcs_ctx* c, size_t n, hipStream_t st) {
    if (n > c->ws_cap) {
        if (c->ws_used) {
            hipError_t e = wait_ws_user(c, nullptr);  // on the host: the buffer is freed next
            if (e != hipSuccess) return e;
        }
        if (c->ws) (void)hipFree(c->ws);
        c->ws = nullptr;
        c->ws_cap = 0;
        c->ws_used = false;
        const size_t cap = n < (1u << 20) ? (1u << 20) : n;
        hipError_t e = hipMalloc(&c->ws, cap * sizeof(nfcs_patch));
        if (e != hipSuccess) return e;
        c->ws_cap = cap;
    } else if (c->ws_used && c->ws_stream != st) {
        hipError_t e = wait_ws_user(c, st);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
hipError_t release_ws(nfcs_ctx* c, hipStream_t st) {
    c->ws_stream = st;
    c->ws_used = true;
    c->ws_own = st == c->stream;
    // a caller's stream may be gone by the time another stream comes: its event is recorded now
    return c->ws_own ? hipSuccess : hipEventRecord(c->ws_ev, st);
}

int hip_fail(hipError_t e) {
    g_last_hip = (int)e;
    return NFCS_EHIP;
}
#define NFCS_HIP(x)                              \
    do {                                         \
        hipError_t e_ = (x);                     \
        if (e_ != hipSuccess) return hip_fail(e_); \
    } while (0)

hipStream_t pick(nfcs_ctx* ctx, void* s) { return s ? (hipStream_t)s : ctx->stream; }

// Makes `device` current on the calling thread for one entry point and restores the caller's
// device on return: a context may be driven from any host thread (netflow_amd::MultiGpu runs one
// thread per GPU), and allocations / copies must land on the context's device.
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int device) {
        err = hipGetDevice(&prev);
        if (err == hipSuccess && prev != device) err = hipSetDevice(device);
        else prev = -1;  // nothing to restore
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// The GPU's NUMA node from sysfs (PCI bus id -> /sys/bus/pci/devices/<id>/numa_node), -1 if unknown.
int gpu_numa_node(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    for (char* q = bus; *q; ++q) *q = (char)((*q >= 'A' && *q <= 'F') ? *q - 'A' + 'a' : *q);
    char path[160];
    snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    int node = -1;
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
    return node;
}

// The CPUs of a NUMA node (/sys/devices/system/node/node<N>/cpulist, e.g. "0-31,128-159").
bool node_cpus(int node, cpu_set_t* set) {
    char path[96];
    snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
    FILE* f = fopen(path, "r");
    if (!f) return false;
    char buf[4096] = {0};
    const bool ok = fgets(buf, sizeof(buf), f) != nullptr;
    fclose(f);
    if (!ok) return false;
    CPU_ZERO(set);
    int n = 0;
    for (char* q = buf; *q && *q != '\n';) {
        char* e;
        const long a = strtol(q, &e, 10);
        if (e == q) break;
        long b = a;
        if (*e == '-') b = strtol(e + 1, &e, 10);
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c, ++n) CPU_SET((int)c, set);
        q = (*e == ',') ? e + 1 : e;
    }
    return n > 0;
}

hipError_t host_block_alloc(HostBlock& b, size_t bytes, int node, bool* local) {
    b.bytes = bytes;
    *local = false;
    if (node >= 0 && node < 1024) {
        void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p != MAP_FAILED) {
            unsigned long mask[16] = {0};
            mask[node / 64] |= 1ul << (node % 64);
            // MPOL_PREFERRED (1): the node's memory while it has free pages, never a failure
            const bool bound = syscall(SYS_mbind, p, bytes, 1, mask, 16 * 64 + 1, 0) == 0;
            memset(p, 0, bytes);  // fault the pages in on the node
            if (hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess) {
                b.p = p;
                b.mapped = true;
                *local = bound;
                return hipSuccess;
            }
            (void)hipGetLastError();
            munmap(p, bytes);
        }
    }
    return hipHostMalloc(&b.p, bytes, hipHostMallocDefault);
}

void host_block_free(HostBlock& b) {
    if (!b.p) return;
    if (b.mapped) {
        (void)hipHostUnregister(b.p);
        munmap(b.p, b.bytes);
    } else {
        (void)hipHostFree(b.p);
    }
    b = HostBlock{};
}

// A pointer into slot s's pinned block, as the GPU addresses it.
template <class T>
T* zdev(const nfcs_ctx* c, int s, T* host) {
    return host ? reinterpret_cast<T*>(c->z_block[s] + (reinterpret_cast<const uint8_t*>(host) -
                                                        static_cast<const uint8_t*>(c->hb[s].p)))
                : nullptr;
}

// Direct chunks (round 6, VERDICT r5 item 2: the per-RX-burst operating point). A chunk of at most
// kDirectChunkBytes of frames moves no DMA at all: the kernel reads its descriptors and frames where
// the host left them (the slot's pinned block, or a pinned caller arena in place) and writes its patch
// records and statuses straight into the slot's pinned block; the host waits for one event. At these
// sizes a call is bound by fixed costs, and the three copy-engine transfers it saves (descriptors,
// frames in, records out: each a queued DMA with its own setup latency) were most of them: 256 C1
// frames through nfcs_update_host 49.5 µs per call with copies, 26.4 in the zero-copy form
// (profiles/r06_host_bursts_*.json). Larger chunks keep the copy engines, which move bytes over PCIe
// faster than kernel loads do (1M C1 frames: 51.7 against 43 GB/s zero-copy).
#ifndef NFCS_DIRECT_CHUNK_BYTES
#define NFCS_DIRECT_CHUNK_BYTES (2u << 20)
#endif
constexpr uint64_t kDirectChunkBytes = NFCS_DIRECT_CHUNK_BYTES;
constexpr uint64_t kZeroCopyAutoBytes = NFCS_HOST_ZERO_COPY_AUTO_BYTES;  // nfcs.h
// The staged chunk size of a host burst of `total` bytes: about total / kChunksPerBurst (at least
// kMinChunkBytes, at most a staging slot), so that the host copies, the transfers, the kernel and the
// write-back of successive chunks overlap across the two slots even when the burst would fit one slot
// (round 2: 16K C1 frames pinned 583 -> 559 µs, pageable 979 -> 710 µs in 4 chunks of >= 4 MiB).
#ifndef NFCS_MIN_CHUNK_BYTES
#define NFCS_MIN_CHUNK_BYTES (4ull << 20)
#endif
#ifndef NFCS_CHUNKS_PER_BURST
#define NFCS_CHUNKS_PER_BURST 4
#endif
constexpr uint64_t kMinChunkBytes = NFCS_MIN_CHUNK_BYTES;
constexpr uint64_t kChunksPerBurst = NFCS_CHUNKS_PER_BURST;
inline uint64_t chunk_bytes(uint64_t total) {
    return std::min<uint64_t>(nfcs_ctx::kStageBytes, std::max<uint64_t>(kMinChunkBytes, total / kChunksPerBurst));
}
// Host copy work per thread before a copy is split over the workers (a worker's wake-up costs ~10 µs;
// one thread stages ~15 GB/s): gathers and staging copies from 512 KiB, write-backs from 2048 frames.
#ifndef NFCS_COPY_BYTES_PER_THREAD
#define NFCS_COPY_BYTES_PER_THREAD (512u << 10)
#endif
constexpr uint64_t kCopyBytesPerThread = NFCS_COPY_BYTES_PER_THREAD;
constexpr uint32_t kPatchFramesPerThread = 2048;

// Host copies whose destination this CPU does not read again (the staging slots, which the copy
// engine reads next; frames copied back into a caller's arena): 16-byte non-temporal stores, so a
// destination line is written once instead of first being read for ownership (a plain memcpy of a
// 1500-byte frame moves 3 bytes over the memory bus per byte copied, this 2). Bytes before dst's
// first 16-byte boundary and after its last go through plain stores; with zero_pad the last partial
// chunk is instead stored whole, its bytes past len zeroed (the staged frames' 16-byte padding, which
// the kernels read). Every worker that streamed calls nt_fence() before its part counts as done.
typedef uint32_t host_u32x4 __attribute__((ext_vector_type(4)));
static inline void stream_copy(uint8_t* dst, const uint8_t* src, uint64_t len, bool zero_pad) {
    uint64_t k = std::min<uint64_t>(len, (16u - ((uintptr_t)dst & 15u)) & 15u);
    if (k) memcpy(dst, src, k);
    for (; k + 64 <= len; k += 64) {
        host_u32x4 a, b, c, d;
        memcpy(&a, src + k, 16); memcpy(&b, src + k + 16, 16);
        memcpy(&c, src + k + 32, 16); memcpy(&d, src + k + 48, 16);
        __builtin_nontemporal_store(a, (host_u32x4*)(dst + k));
        __builtin_nontemporal_store(b, (host_u32x4*)(dst + k + 16));
        __builtin_nontemporal_store(c, (host_u32x4*)(dst + k + 32));
        __builtin_nontemporal_store(d, (host_u32x4*)(dst + k + 48));
    }
    for (; k + 16 <= len; k += 16) {
        host_u32x4 a;
        memcpy(&a, src + k, 16);
        __builtin_nontemporal_store(a, (host_u32x4*)(dst + k));
    }
    if (k < len) {
        if (zero_pad && !((uintptr_t)(dst + k) & 15u)) {
            host_u32x4 t = {0u, 0u, 0u, 0u};
            memcpy(&t, src + k, len - k);
            __builtin_nontemporal_store(t, (host_u32x4*)(dst + k));
        } else {
            memcpy(dst + k, src + k, len - k);
        }
    }
}
static inline void nt_fence() { __builtin_ia32_sfence(); }  // the non-temporal stores drained

// Copy split across the context's workers: one host thread copies pageable memory at ~15-25 GB/s,
// below what PCIe moves (e2e: pageable staging 27 GB/s single-threaded vs 54 GB/s pinned). The
// workers run on the GPU's NUMA node, next to the staging memory.
void par_memcpy(nfcs_ctx* c, void* dst, const void* src, size_t bytes) {
    const size_t kMin = kCopyBytesPerThread;
    if (bytes < 2 * kMin || c->workers.size() == 0) {
        stream_copy((uint8_t*)dst, (const uint8_t*)src, bytes, false);
        nt_fence();
        return;
    }
    const size_t t = std::min<size_t>((size_t)c->workers.size() + 1, bytes / kMin);
    const size_t per = (bytes / t + 4095) & ~size_t(4095);
    c->workers.run((int)t, [&](int i) {
        const size_t o = (size_t)i * per;
        if (o < bytes) stream_copy((uint8_t*)dst + o, (const uint8_t*)src + o, std::min(per, bytes - o), false);
        nt_fence();
    });
}

// Frees the host pipeline's streams, events and buffers (also a partly built one).
void free_host_pipeline(nfcs_ctx* c) {
    c->host_ready = false;
    c->workers.stop();
    if (c->done_host) {
        for (int s = 0; s < nfcs_ctx::kSlots; ++s)
            if (c->hs[s]) (void)hipStreamSynchronize(c->hs[s]);  // no launch still counting into them
        (void)hipHostFree(c->done_host);
    }
    if (c->done_ctr) (void)hipFree(c->done_ctr);
    c->done_host = nullptr;
    c->done_dev = nullptr;
    c->done_ctr = nullptr;
    for (int s = 0; s < nfcs_ctx::kSlots; ++s) {
        if (c->hs[s]) { (void)hipStreamSynchronize(c->hs[s]); (void)hipStreamDestroy(c->hs[s]); }
        if (c->done[s]) (void)hipEventDestroy(c->done[s]);
        if (c->staged[s]) (void)hipEventDestroy(c->staged[s]);
        (void)hipFree(c->d_arena[s]);
        (void)hipFree(c->d_desc[s]);
        (void)hipFree(c->d_status[s]);
        (void)hipFree(c->d_patch[s]);
        host_block_free(c->hb[s]);
        c->hs[s] = nullptr;
        c->done[s] = nullptr;
        c->staged[s] = nullptr;
        c->d_arena[s] = nullptr;
        c->d_desc[s] = nullptr;
        c->d_status[s] = nullptr;
        c->d_patch[s] = nullptr;
        c->h_arena[s] = nullptr;
        c->z_block[s] = nullptr;
        c->h_desc[s] = nullptr;
        c->h_status[s] = nullptr;
        c->h_patch[s] = nullptr;
    }
}

int build_host_pipeline(nfcs_ctx* ctx);

// A direct chunk's completion request for slot s (nfcs::DoneReq), or none where the context has no flags.
nfcs::DoneReq done_req(nfcs_ctx* c, int s) {
    c->slot_wait[s] = c->done_host ? 1 : 0;
    if (!c->done_host) return {};
    return {c->done_dev + 8 * s, c->done_ctr + s, c->done_base[s]};
}
// The chunk launched in slot s is waited for on its events.
void event_wait(nfcs_ctx* c, int s) { c->slot_wait[s] = 0; }

// Waits for the chunk in slot s: on its completion flag when it has one (a direct chunk: the kernel's
// last workgroup publishes the count; once seen, later waits for the same chunk return at once), else
// — or after kFlagSpinNs without the flag, e.g. a launch that failed — on the event.
hipError_t wait_slot(nfcs_ctx* c, int s, hipEvent_t ev) {
    constexpr int64_t kFlagSpinNs = 20000000;
    if (c->slot_wait[s] == 2) return hipSuccess;
    if (c->slot_wait[s] == 1) {
        const uint64_t base = c->done_base[s];
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t k = 1;; ++k) {
            const uint64_t v = __atomic_load_n(c->done_host + 8 * s, __ATOMIC_ACQUIRE);
            if (v > base) {
                c->done_base[s] = v;
                c->slot_wait[s] = 2;
                return hipSuccess;
            }
            if ((k & 1023u) == 0 &&
                std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() > kFlagSpinNs)
                break;
            __builtin_ia32_pause();
        }
        const hipError_t e = hipEventSynchronize(ev);
        c->done_base[s] = std::max(c->done_base[s], __atomic_load_n(c->done_host + 8 * s, __ATOMIC_ACQUIRE));
        c->slot_wait[s] = 0;
        return e;
    }
    return hipEventSynchronize(ev);
}

// The host pipeline, built on first use on the context's device (the caller holds a DeviceGuard).
// A build that fails part-way is torn down, so the next call retries it instead of using half of it.
int ensure_host_pipeline(nfcs_ctx* ctx) {
    if (ctx->host_ready) return NFCS_OK;
    const int rc = build_host_pipeline(ctx);
    if (rc != NFCS_OK) {
        free_host_pipeline(ctx);
        return rc;
    }
    ctx->host_ready = true;
    return NFCS_OK;
}

int build_host_pipeline(nfcs_ctx* ctx) {
    // host threads for the staging copies, gathers and write-back: 8, or NFCS_HOST_THREADS (1-64) —
    // a caller that shares the host's cores with other work, or has more to give, sets it
    ctx->copy_threads = 8;
    if (const char* e = getenv("NFCS_HOST_THREADS")) {
        const int t = atoi(e);
        if (t >= 1 && t <= 64) ctx->copy_threads = t;
    }
    ctx->stage_bytes = nfcs_ctx::kStageBytes;
    ctx->stage_pkts = (uint32_t)(ctx->stage_bytes / 64);
    // staging ring on the GPU's NUMA node, copy threads on its CPUs
    ctx->numa_node = gpu_numa_node(ctx->di.device);
    ctx->have_cpus = ctx->numa_node >= 0 && node_cpus(ctx->numa_node, &ctx->node_cpus);
    const size_t a_desc = (size_t)ctx->stage_pkts * sizeof(nfcs_desc);
    const size_t a_patch = (size_t)ctx->stage_pkts * sizeof(nfcs_patch);
    const size_t a_status = ((size_t)ctx->stage_pkts + 4095) & ~size_t(4095);
    bool local = true;
    for (int s = 0; s < nfcs_ctx::kSlots; ++s) {
        NFCS_HIP(hipStreamCreateWithFlags(&ctx->hs[s], hipStreamNonBlocking));
        NFCS_HIP(hipEventCreateWithFlags(&ctx->done[s], hipEventDisableTiming));
        NFCS_HIP(hipEventCreateWithFlags(&ctx->staged[s], hipEventDisableTiming));
        NFCS_HIP(hipMalloc(&ctx->d_arena[s], ctx->stage_bytes));
        NFCS_HIP(hipMalloc(&ctx->d_desc[s], a_desc));
        NFCS_HIP(hipMalloc(&ctx->d_status[s], ctx->stage_pkts));
        NFCS_HIP(hipMalloc(&ctx->d_patch[s], a_patch));
        // one pinned block per slot: arena | descriptors | patch records | statuses
        bool l = false;
        NFCS_HIP(host_block_alloc(ctx->hb[s], ctx->stage_bytes + a_desc + a_patch + a_status,
                                  ctx->numa_node, &l));
        local = local && l;
        uint8_t* p = static_cast<uint8_t*>(ctx->hb[s].p);
        ctx->h_arena[s] = p;
        ctx->h_desc[s] = reinterpret_cast<nfcs_desc*>(p + ctx->stage_bytes);
        ctx->h_patch[s] = reinterpret_cast<nfcs_patch*>(p + ctx->stage_bytes + a_desc);
        ctx->h_status[s] = p + ctx->stage_bytes + a_desc + a_patch;
        // the block as the GPU addresses it (registered and hipHostMalloc'd memory is mapped): direct
        // chunks read their frames and descriptors and write their records and statuses here
        void* zp = nullptr;
        if (hipHostGetDevicePointer(&zp, p, 0) == hipSuccess) ctx->z_block[s] = static_cast<uint8_t*>(zp);
        else (void)hipGetLastError();
    }
    ctx->numa_local = local;
    // completion flags of direct chunks: optional (without them the chunks wait on their events)
    if (hipHostMalloc((void**)&ctx->done_host, nfcs_ctx::kSlots * 64, hipHostMallocMapped) == hipSuccess &&
        hipHostGetDevicePointer((void**)&ctx->done_dev, ctx->done_host, 0) == hipSuccess &&
        hipMalloc((void**)&ctx->done_ctr, nfcs_ctx::kSlots * sizeof(uint64_t)) == hipSuccess &&
        hipMemset(ctx->done_ctr, 0, nfcs_ctx::kSlots * sizeof(uint64_t)) == hipSuccess) {
        memset(ctx->done_host, 0, nfcs_ctx::kSlots * 64);
    } else {
        (void)hipGetLastError();
        if (ctx->done_host) (void)hipHostFree(ctx->done_host);
        if (ctx->done_ctr) (void)hipFree(ctx->done_ctr);
        ctx->done_host = nullptr;
        ctx->done_dev = nullptr;
        ctx->done_ctr = nullptr;
    }
    for (int s = 0; s < nfcs_ctx::kSlots; ++s) {
        ctx->done_base[s] = 0;
        ctx->slot_wait[s] = 0;
    }
    ctx->workers.start(ctx->copy_threads - 1, ctx->have_cpus ? &ctx->node_cpus : nullptr);
    return NFCS_OK;
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// A caller's descriptor as the host path stages it: a frame inside the arena that is longer than
// kFrameRelevantBytes goes as its first kFrameRelevantBytes — the same result (nfcs.h), and no frame
// outgrows a staging slot; others unchanged (a frame reaching past the arena stays NFCS_ST_BAD_DESC).
inline nfcs_desc staged_desc(const nfcs_desc& d, uint64_t arena_bytes) {
    const uint64_t o = (uint64_t)d.off16 * 16u;
    if (d.len > nfcs::kFrameRelevantBytes && o + (((uint64_t)d.len + 15u) & ~15ull) <= arena_bytes)
        return nfcs_desc{d.off16, nfcs::kFrameRelevantBytes};
    return d;
}
// Descriptors [i, i + m) into a staging slot, as staged_desc stages them (a plain copy when the burst
// has no frame longer than kFrameRelevantBytes).
void stage_descs(nfcs_desc* dst, const nfcs_desc* src, uint32_t m, uint64_t arena_bytes, bool any_long) {
    if (!any_long) {
        memcpy(dst, src, (size_t)m * sizeof(nfcs_desc));
        return;
    }
    for (uint32_t j = 0; j < m; ++j) dst[j] = staged_desc(src[j], arena_bytes);
}

// The arena bytes that descriptors [i0, i1) span, summed over their runs of ascending offsets: a NIC
// ring burst that wraps past the ring's end is two runs, each from its first frame's start to the end
// of its furthest frame (frames outside the arena count nothing). The launch shape's footprint.
uint64_t run_span(const nfcs_desc* d, uint32_t i0, uint32_t i1, uint64_t arena_bytes) {
    uint64_t total = 0, lo = 0, hi = 0;
    for (uint32_t i = i0; i < i1; ++i) {
        const nfcs_desc sd = staged_desc(d[i], arena_bytes);
        const uint64_t o = (uint64_t)sd.off16 * 16u, e = o + (((uint64_t)sd.len + 15u) & ~15ull);
        if (i == i0 || d[i].off16 < d[i - 1].off16) {  // a new run
            total += hi - lo;
            lo = hi = std::min(o, arena_bytes);
        }
        if (e <= arena_bytes) hi = std::max(hi, e);
    }
    return total + (hi - lo);
}

// Pinned host arena: the kernel reads the frames over PCIe where they are and writes the 2+2
// checksum bytes straight back (host memory from hipHostMalloc is mapped into the GPU's address
// space), inline from the read pass (kUpdateInline: a deferred write pass would cross the link
// again). The descriptors (8 B/packet) are copied into a staging slot's pinned block, where the kernel
// reads them, and the statuses (1 B/packet) come back there (round 6; copied H2D / D2H by DMA before),
// in chunks on the two pipeline streams; frames cross the link once, in one direction. On an error both
// slots are drained before returning, so nothing is left in flight on the caller's memory. Also the
// default form of nfcs_update_host for pinned bursts of up to kZeroCopyAutoBytes.
int update_host_zero_copy(nfcs_ctx* c, uint8_t* h_arena, uint64_t arena_bytes,
                          const nfcs_desc* h_desc, uint32_t n, uint8_t* h_status, bool any_long) {
    void* dptr = nullptr;
    NFCS_HIP(hipHostGetDevicePointer(&dptr, h_arena, 0));
    uint8_t* d_arena = static_cast<uint8_t*>(dptr);
    uint32_t cnt[nfcs_ctx::kSlots] = {0, 0}, first[nfcs_ctx::kSlots] = {0, 0};
    hipError_t e = hipSuccess;
    // wait for slot s; its statuses are copied out only while no error has occurred
    auto finish = [&](int s) {
        if (!cnt[s]) return;
        const hipError_t f = wait_slot(c, s, c->done[s]);
        if (e == hipSuccess) e = f;
        if (e == hipSuccess && h_status) memcpy(h_status + first[s], c->h_status[s], cnt[s]);
        cnt[s] = 0;
    };
    int s = 0;
    for (uint32_t i = 0; i < n && e == hipSuccess; s ^= 1) {
        finish(s);
        if (e != hipSuccess) break;
        const uint32_t m = std::min<uint32_t>(n - i, c->stage_pkts);
        hipStream_t st = c->hs[s];
        stage_descs(c->h_desc[s], h_desc + i, m, arena_bytes, any_long);
        // the launch shape follows this chunk's own frames (their span per packet, over the runs of
        // a burst that wraps its ring), not the caller's whole arena, unless the context has a hint
        const uint64_t span = run_span(h_desc, i, i + m, arena_bytes);
        uint64_t shape = c->slot_bytes;
        if (!shape) shape = std::max<uint64_t>(1, span / m);
        if (c->z_block[s]) {
            // round 6: the kernel reads the chunk's descriptors from the slot's pinned block and writes
            // its statuses there (no DMA at all: burst sizes where the call is bound by fixed costs); a
            // small chunk signals its completion through the slot's flag (nfcs::DoneReq)
            const nfcs::DoneReq dr = span <= kDirectChunkBytes ? done_req(c, s) : nfcs::DoneReq{};
            if (!dr.flag) event_wait(c, s);
            e = nfcs::launch_update(c->di, d_arena, arena_bytes, zdev(c, s, c->h_desc[s]), m, 0u,
                                    h_status ? zdev(c, s, c->h_status[s]) : nullptr, nullptr, nullptr,
                                    nfcs::kUpdateInline, st, shape, {}, dr);
        } else {
            event_wait(c, s);
            e = hipMemcpyAsync(c->d_desc[s], c->h_desc[s], (size_t)m * sizeof(nfcs_desc),
                               hipMemcpyHostToDevice, st);
            if (e == hipSuccess)
                e = nfcs::launch_update(c->di, d_arena, arena_bytes, c->d_desc[s], m, 0u,
                                        h_status ? c->d_status[s] : nullptr, nullptr, nullptr,
                                        nfcs::kUpdateInline, st, shape);
            if (e == hipSuccess && h_status)
                e = hipMemcpyAsync(c->h_status[s], c->d_status[s], m, hipMemcpyDeviceToHost, st);
        }
        if (e == hipSuccess) e = hipEventRecord(c->done[s], st);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(st);  // whatever was queued on this slot has finished
            break;
        }
        first[s] = i;
        cnt[s] = m;
        i += m;
    }
    finish(s);  // drain both slots, also after an error
    finish(s ^ 1);
    if (e != hipSuccess) return hip_fail(e);
    return NFCS_OK;
}

// The launch shape's mean footprint per packet for a device call (speed only; the bytes written
// never depend on it): the context's slot-size hint when set; else arena_bytes / n, which is exact
// for a batch that fills its arena and can only over-estimate (frames never overlap). So a short
// estimate is right, and only a long one can be wrong — a burst inside a larger ring. Then the call
// also has its launch sample the frames' real footprint (sample_footprint, one wave, host-mapped
// result), and the next call on the same burst (descriptor array, n and arena_bytes; up to kObsSlots
// bursts tracked, least recently used replaced) launches in the shape that sample says: a NIC ring
// reusing its descriptor arrays adapts after one call, with no hint and no host sync.
struct Shape { uint64_t mean; nfcs::ObsReq obs; uint32_t bits = 0; };  // bits: the sample's kObsUnaligned / kObsMixed
// The burst's observation slot, or -1 (no side effects).
int find_burst(const nfcs_ctx* c, uint64_t arena_bytes, const nfcs_desc* d_desc, uint32_t n) {
    for (int k = 0; k < nfcs_ctx::kObsSlots; ++k) {
        const nfcs_ctx::ObsBurst& b = c->obs_burst[k];
        if (b.gen && b.desc == d_desc && b.n == n && b.bytes == arena_bytes) return k;
    }
    return -1;
}
// The shape a call over this burst launches in, without side effects (nfcs_ctx_launch_footprint):
// *slot = the burst's observation slot, -1 when it has none yet (the call then takes one).
// Estimates that a sample can correct: "long" (a burst inside a larger ring), and "8-lane rows" (a
// densely packed mix whose frames often need a second 8-lane row pass; round 6).
// (the forward samples mid-size estimates too: ShapeRule::packed_rows8)
bool sampled_estimate(uint64_t est, bool mid = false) {
    return mid || est >= nfcs::kSmallMeanBytes || est < nfcs::kTinyMeanBytes;
}
// Each op's use of the sample (nfcs_internal.h, after kTinyMixMeanBytes): the mean from which a mix with
// many long frames leaves 8-lane rows, whether mid-size frames of one length in a ring take 8-lane rows,
// whether a mix with hardly any mid-length frames (64 / 1500-byte traffic) stays on them, and whether
// densely packed mid-size frames of one length on their own lines take them too (sampled for it).
struct ShapeRule { uint64_t mix_mean; bool ring_rows8; bool bimodal_rows8; bool packed_rows8; };
constexpr ShapeRule kUpdateRule = {nfcs::kTinyMixMeanBytes, true, false, false};
constexpr ShapeRule kFwdRule = {nfcs::kTinyMixMeanBytes, true, true, true};
constexpr ShapeRule kVlanRule = {nfcs::kVlanMixMeanBytes, false, false, false};
Shape peek_shape(const nfcs_ctx* c, uint64_t arena_bytes, const nfcs_desc* d_desc, uint32_t n, int* slot,
                 const ShapeRule& rule = kUpdateRule) {
    *slot = -1;
    if (c->slot_bytes) return {c->slot_bytes, {}};
    if (n == 0) return {arena_bytes, {}};  // nothing is launched; never divide by zero
    const uint64_t est = arena_bytes / n;
    if (!sampled_estimate(est, rule.packed_rows8) || !c->obs_host) return {est, {}};
    const int k = find_burst(c, arena_bytes, d_desc, n);
    if (k < 0) return {est, {}};
    *slot = k;
    // the latest sample of this burst's generation (a late one of an earlier burst has another)
    const uint64_t o = __atomic_load_n(c->obs_host + k, __ATOMIC_RELAXED);
    const uint32_t gen = c->obs_burst[k].gen;
    const nfcs::ObsReq req = {c->obs_dev + k, ((uint64_t)gen << 32) | n};
    if ((uint32_t)(o >> 32) != gen || !((uint32_t)o & nfcs::kObsPresent)) return {est, req};
    uint64_t mean = std::min<uint64_t>((uint32_t)o & nfcs::kObsMeanMask, est);
    // 8-lane rows only for frames that mostly fit their one row pass, or short enough on average that
    // the packet rate bounds them (nfcs_internal.h kTinyLongMax, kTinyMixMeanBytes), or — the forward —
    // a mix of short and full-size frames with hardly any in between (kObsMidShift)
    const bool bimodal = rule.bimodal_rows8 && (((uint32_t)o >> nfcs::kObsMidShift) & 7u) < nfcs::kObsMidMin8;
    if (mean < nfcs::kTinyMeanBytes && mean >= rule.mix_mean && !bimodal &&
        (((uint32_t)o >> nfcs::kObsLongShift) & 0x1FFu) > nfcs::kTinyLongMax)
        mean = nfcs::kTinyMeanBytes;
    const uint32_t bits = (uint32_t)o & (nfcs::kObsUnaligned | nfcs::kObsMixed);
    // a ring (the sample corrected a "long" estimate) of mid-size frames of one length, each on its own
    // lines — or, for the forward, such frames packed: 8-lane rows (nfcs_internal.h, after
    // kTinyMixMeanBytes)
    if (rule.ring_rows8 && !bits && (est >= nfcs::kSmallMeanBytes || rule.packed_rows8) &&
        mean >= nfcs::kTinyMeanBytes && mean < nfcs::kSmallMeanBytes)
        mean = nfcs::kTinyMeanBytes - 1;
    return {mean, req, bits};
}
Shape launch_shape(nfcs_ctx* c, uint64_t arena_bytes, const nfcs_desc* d_desc, uint32_t n,
                   const ShapeRule& rule = kUpdateRule) {
    int k = -1;
    Shape sh = peek_shape(c, arena_bytes, d_desc, n, &k, rule);
    if (sh.obs.slot == nullptr && k < 0 && !c->slot_bytes && n && c->obs_host &&
        sampled_estimate(arena_bytes / n, rule.packed_rows8)) {
        // a burst not seen lately: the least recently used slot, under a new generation
        k = 0;
        for (int j = 1; j < nfcs_ctx::kObsSlots; ++j)
            if (c->obs_burst[j].used < c->obs_burst[k].used) k = j;
        if (++c->obs_gen == 0) c->obs_gen = 1;
        c->obs_burst[k] = {d_desc, n, arena_bytes, c->obs_gen, 0};
        sh.obs = {c->obs_dev + k, ((uint64_t)c->obs_gen << 32) | n};
    }
    if (k >= 0) c->obs_burst[k].used = ++c->obs_clock;
    return sh;
}

// The device-resident update on stream st: kUpdateAuto, deferred records into the caller's
// d_patch when given, else into the context workspace.
int update_device(nfcs_ctx* c, uint8_t* d_arena, uint64_t arena_bytes, const nfcs_desc* d_desc,
                  uint32_t n, uint8_t* d_status, nfcs_patch* d_patch, hipStream_t st) {
    if (!d_patch) NFCS_HIP(acquire_ws(c, n, st));
    const Shape sh = launch_shape(c, arena_bytes, d_desc, n);
    NFCS_HIP(nfcs::launch_update(c->di, d_arena, arena_bytes, d_desc, n, 0u, d_status, d_patch,
                                 d_patch ? nullptr : c->ws, nfcs::kUpdateAuto, st, sh.mean, sh.obs));
    if (!d_patch) NFCS_HIP(release_ws(c, st));
    return NFCS_OK;
}

// The fused L3 forward on stream st; a burst above kFwdDeferAbovePackets defers the stores of its
// long-frame waves through forward records in the context workspace (one per packet of a sub-batch).
int l3_forward_device(nfcs_ctx* c, uint8_t* d_arena, uint64_t arena_bytes, const nfcs_desc* d_desc,
                      const uint32_t* d_nh, uint32_t n, const nfcs_nexthop* d_table, uint32_t table_n,
                      uint8_t* d_status, hipStream_t st) {
    const bool dfr = n > nfcs::kFwdDeferAbovePackets;
    if (dfr) NFCS_HIP(acquire_ws(c, nfcs::kSubBatchPackets, st));
    const Shape sh = launch_shape(c, arena_bytes, d_desc, n, kFwdRule);
    NFCS_HIP(nfcs::launch_l3_forward(c->di, d_arena, arena_bytes, d_desc, d_nh, n, d_table, table_n,
                                     d_status, dfr ? c->ws : nullptr, st, sh.mean, sh.obs));
    if (dfr) NFCS_HIP(release_ws(c, st));
    return NFCS_OK;
}

}  // namespace

extern "C" {

NFCS_API int nfcs_abi_version(void) { return NFCS_ABI_VERSION; }

NFCS_API const char* nfcs_strerror(int err) {
    switch (err) {
    case NFCS_OK: return "ok";
    case NFCS_EINVAL: return "invalid argument";
    case NFCS_EHIP: return "HIP runtime error";
    case NFCS_ENOMEM: return "out of memory";
    case NFCS_ENODEV: return "no gfx950 device";
    default: return "unknown error";
    }
}

NFCS_API int nfcs_last_hip_error(void) { return g_last_hip; }

NFCS_API int nfcs_ctx_create(int device, nfcs_ctx** out) {
    if (!out) return NFCS_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        (void)hipGetLastError();
        return NFCS_ENODEV;
    }
    DeviceGuard dg_(device);  // the new context's device while it is set up; the caller's after
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipDeviceProp_t prop;
    NFCS_HIP(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return NFCS_ENODEV;
    nfcs_ctx* c = new (std::nothrow) nfcs_ctx();
    if (!c) return NFCS_ENOMEM;
    c->di.device = device;
    c->di.cus = prop.multiProcessorCount;
    strncpy(c->di.arch, prop.gcnArchName, sizeof(c->di.arch) - 1);
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&c->d_digest, sizeof(uint64_t));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ws_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreate(&c->ev0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev1);
    if (e == hipSuccess) e = hipHostMalloc((void**)&c->obs_host, nfcs_ctx::kObsSlots * sizeof(uint64_t), hipHostMallocMapped);
    if (e == hipSuccess) {
        for (int k = 0; k < nfcs_ctx::kObsSlots; ++k) c->obs_host[k] = 0;
        e = hipHostGetDevicePointer((void**)&c->obs_dev, c->obs_host, 0);
    }
    if (e != hipSuccess) {
        nfcs_ctx_destroy(c);
        return hip_fail(e);
    }
    *out = c;
    return NFCS_OK;
}

NFCS_API int nfcs_ctx_destroy(nfcs_ctx* c) {
    if (!c) return NFCS_OK;
    DeviceGuard dg_(c->di.device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->ws_used && !c->ws_own && c->ws_ev) (void)hipEventSynchronize(c->ws_ev);  // a caller stream's last write pass
    free_host_pipeline(c);
    if (c->d_digest) (void)hipFree(c->d_digest);
    if (c->ws) (void)hipFree(c->ws);
    if (c->ws_ev) (void)hipEventDestroy(c->ws_ev);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->obs_host) (void)hipHostFree(c->obs_host);
    delete c;
    return NFCS_OK;
}

NFCS_API void* nfcs_ctx_stream(nfcs_ctx* c) { return c ? (void*)c->stream : nullptr; }

NFCS_API int nfcs_ctx_set_slot_bytes(nfcs_ctx* c, uint32_t bytes) {
    if (!c) return NFCS_EINVAL;
    c->slot_bytes = bytes;
    return NFCS_OK;
}

NFCS_API int nfcs_ctx_launch_footprint(nfcs_ctx* c, uint64_t arena_bytes, const nfcs_desc* d_desc,
                                       uint32_t n, uint64_t* mean) {
    if (!c || !mean) return NFCS_EINVAL;
    int slot = -1;
    *mean = peek_shape(c, arena_bytes, d_desc, n, &slot).mean;
    return NFCS_OK;
}

NFCS_API int nfcs_ctx_host_numa(nfcs_ctx* c, int* node, int* local) {
    if (!c || !node || !local) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the pipeline is built on the context's device
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    const int rc = ensure_host_pipeline(c);
    if (rc) return rc;
    *node = c->numa_node;
    *local = c->numa_local ? 1 : 0;
    return NFCS_OK;
}

NFCS_API int nfcs_update_device(nfcs_ctx* c, uint8_t* d_arena, uint64_t arena_bytes,
                                const nfcs_desc* d_desc, uint32_t n, uint8_t* d_status,
                                nfcs_patch* d_patch, void* stream) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    if (n == 0) return NFCS_OK;
    if (!d_arena || !d_desc || ((uintptr_t)d_arena & 15u)) return NFCS_EINVAL;
    return update_device(c, d_arena, arena_bytes, d_desc, n, d_status, d_patch, pick(c, stream));
}

NFCS_API int nfcs_l3_forward_device(nfcs_ctx* c, uint8_t* d_arena, uint64_t arena_bytes,
                                    const nfcs_desc* d_desc, const uint32_t* d_nh, uint32_t n,
                                    const nfcs_nexthop* d_table, uint32_t table_n,
                                    uint8_t* d_status, void* stream) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    if (n == 0) return NFCS_OK;
    if (!d_arena || !d_desc || !d_nh || ((uintptr_t)d_arena & 15u)) return NFCS_EINVAL;
    if (table_n > 0 && (!d_table || ((uintptr_t)d_table & 3u))) return NFCS_EINVAL;
    return l3_forward_device(c, d_arena, arena_bytes, d_desc, d_nh, n, d_table, table_n, d_status,
                             pick(c, stream));
}

NFCS_API int nfcs_vlan_device(nfcs_ctx* c, uint8_t* d_arena, uint64_t arena_bytes,
                              nfcs_desc* d_desc, uint32_t n, const uint32_t* d_ops,
                              uint32_t op_all, const uint32_t* d_caps, uint32_t cap_all,
                              uint8_t* d_status, void* stream) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    if (n == 0) return NFCS_OK;
    if (!d_arena || !d_desc || ((uintptr_t)d_arena & 15u)) return NFCS_EINVAL;
    if (((uintptr_t)d_ops & 3u) || ((uintptr_t)d_caps & 3u)) return NFCS_EINVAL;
    const Shape sh = launch_shape(c, arena_bytes, d_desc, n, kVlanRule);
    NFCS_HIP(nfcs::launch_vlan(c->di, d_arena, arena_bytes, d_desc, n, d_ops, op_all, d_caps,
                               cap_all, d_status, pick(c, stream), sh.mean, sh.obs, sh.bits));
    return NFCS_OK;
}

NFCS_API int nfcs_flow_keys_device(nfcs_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes,
                                   const nfcs_desc* d_desc, uint32_t n, nfcs_flow_key* d_keys,
                                   uint32_t* d_hash, void* stream) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    if (n == 0) return NFCS_OK;
    if (!d_arena || !d_desc || ((uintptr_t)d_arena & 15u) || ((uintptr_t)d_keys & 15u))
        return NFCS_EINVAL;
    NFCS_HIP(nfcs::launch_flow_keys(c->di, d_arena, arena_bytes, d_desc, n, d_keys, d_hash,
                                    pick(c, stream)));
    return NFCS_OK;
}

NFCS_API int nfcs_update_host(nfcs_ctx* c, uint8_t* h_arena, uint64_t arena_bytes,
                              const nfcs_desc* h_desc, uint32_t n, uint8_t* h_status,
                              uint32_t flags) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    if (n == 0) return NFCS_OK;
    if (!h_arena || !h_desc) return NFCS_EINVAL;
    // Every frame inside the arena fits one staging slot as staged (staged_desc: a frame longer than
    // kFrameRelevantBytes goes as its first kFrameRelevantBytes, round 6; NFCS_EINVAL above 64 MiB
    // before). A frame reaching past the arena is staged as nothing and becomes NFCS_ST_BAD_DESC (the
    // kernel checks it against its chunk), as on the device path. Frames come in any order: a chunk
    // is a run of ascending offsets, so a burst that wraps past its ring's end (round 5; VERDICT r4
    // item 4) is split where an offset drops below its predecessor's, as separate PacketBuffers
    // (packet_buffer.hpp:21-31) never constrain their order either.
    auto frame_end = [&](uint32_t i) -> uint64_t {  // 0: outside the arena; as staged (staged_desc)
        const nfcs_desc d = staged_desc(h_desc[i], arena_bytes);
        const uint64_t o = (uint64_t)d.off16 * 16u;
        const uint64_t e = o + (((uint64_t)d.len + 15u) & ~15ull);
        return e <= arena_bytes ? e : 0;
    };
    bool ordered = true;  // ascending offsets: the chunks' spans are disjoint
    bool any_long = false;  // a frame inside the arena longer than kFrameRelevantBytes (staged_desc)
    for (uint32_t i = 0; i < n; ++i) {
        any_long = any_long || h_desc[i].len > nfcs::kFrameRelevantBytes;
        ordered = ordered && (i == 0 || h_desc[i].off16 >= h_desc[i - 1].off16);
    }
    const uint64_t span = run_span(h_desc, 0, n, arena_bytes);
    int rc = ensure_host_pipeline(c);
    if (rc) return rc;
    const bool pinned = is_pinned(h_arena);
    if (flags & NFCS_HOST_ZERO_COPY) {
        if (!pinned) return NFCS_EINVAL;
        return update_host_zero_copy(c, h_arena, arena_bytes, h_desc, n, h_status, any_long);
    }
    // A pinned arena's burst of at most kZeroCopyAutoBytes of frames (the default, records form) runs
    // zero-copy: the kernel reads its frames in place and stores the checksum bytes straight back,
    // the same bytes the records would carry (round 6, profiles/r06_host_bursts_ab.jsonl: 64 to 16K C1
    // frames 2-18% faster zero-copy than through the copy engines, 64K 3-5% slower)
    // (a 16-byte aligned arena only: the kernel's 16-byte loads address the frames in place)
    const bool aligned = ((uintptr_t)h_arena & 15u) == 0;
    if (pinned && aligned && !(flags & NFCS_HOST_FRAMES) && span <= kZeroCopyAutoBytes)
        return update_host_zero_copy(c, h_arena, arena_bytes, h_desc, n, h_status, any_long);
    // default: frames H2D and only the 8-byte patch records D2H (kUpdateRecords: the staged
    // frames are not written), applied here; whole frames back only on request (NFCS_HOST_FRAMES:
    // kUpdateAuto on the staged frames, the slot's patch buffer as the deferred-store workspace)
    const bool patch_only = !(flags & NFCS_HOST_FRAMES);
    // Chunk size: a burst is cut into ~4 chunks (at least kMinChunk bytes, at most a staging slot)
    // so that its host copy, H2D copy, kernel, D2H copy and patch application overlap across the
    // two slots even when it would fit one slot (16K C1 frames: pinned 583 -> 559 µs, pageable
    // 979 -> 710 µs; 64K: 2267 -> 1992 / 3133 -> 2273 µs). Whole frames back from a pinned arena
    // keep slot-sized chunks (4 chunks measured slower there: 64K 3.13 -> 3.59 ms).
    const uint64_t chunk_target = (!patch_only && pinned) ? nfcs_ctx::kStageBytes : chunk_bytes(span);

    struct Chunk { uint32_t i0, i1; uint64_t base, bytes; bool used; };
    Chunk slot[nfcs_ctx::kSlots] = {};
    hipError_t e = hipSuccess;
    // finish a slot: wait for its D2H, then apply patches / copy frames / copy statuses (only
    // while no error has occurred; after one the slot is only drained)
    auto finish = [&](int s) {
        Chunk& k = slot[s];
        if (!k.used) return;
        k.used = false;
        const hipError_t f = wait_slot(c, s, c->done[s]);
        if (e == hipSuccess) e = f;
        if (e != hipSuccess) return;
        const uint32_t m = k.i1 - k.i0;
        if (patch_only) {
            // each record writes into another frame's header line, which the DMA read but the
            // CPU has not cached: prefetch the line kPf packets ahead so the misses overlap; large
            // chunks over the workers
            const nfcs_patch* pq = c->h_patch[s];
            const int np = std::min<int>(c->workers.size() + 1, std::max<uint32_t>(1, m / kPatchFramesPerThread));
            c->workers.run(np, [&](int t) {
                const uint32_t j0 = (uint32_t)((uint64_t)m * t / np), j1 = (uint32_t)((uint64_t)m * (t + 1) / np);
                constexpr uint32_t kPf = 16;
                for (uint32_t j = j0; j < j1; ++j) {
                    if (j + kPf < j1) {
                        const nfcs_patch& q = pq[j + kPf];
                        const uint32_t o = q.ip_off != NFCS_PATCH_NONE ? q.ip_off : q.l4_off;
                        const uint64_t a = (uint64_t)h_desc[k.i0 + j + kPf].off16 * 16u + (o & 0xFFC0u);
                        if (a < arena_bytes) __builtin_prefetch(h_arena + a, 1, 0);
                    }
                    const nfcs_patch& pt = pq[j];
                    if (!frame_end(k.i0 + j)) continue;
                    uint8_t* f = h_arena + (uint64_t)h_desc[k.i0 + j].off16 * 16u;
                    if (pt.ip_off != NFCS_PATCH_NONE) { f[pt.ip_off] = pt.ip[0]; f[pt.ip_off + 1] = pt.ip[1]; }
                    if (pt.l4_off != NFCS_PATCH_NONE) { f[pt.l4_off] = pt.l4[0]; f[pt.l4_off + 1] = pt.l4[1]; }
                }
            });
        } else if (ordered && !pinned) {
            par_memcpy(c, h_arena + k.base, c->h_arena[s], k.bytes);
        } else if (!ordered) {
            // Frames in any order: a chunk's span can hold frames of other chunks, staged before an
            // earlier chunk wrote them back, so only the chunk's own frames are copied back (from
            // the slot, where the frames came back also for a pinned arena)
            const int np = m >= 16384 ? c->workers.size() + 1 : 1;
            c->workers.run(np, [&](int t) {
                for (uint32_t j = (uint32_t)((uint64_t)m * t / np); j < (uint32_t)((uint64_t)m * (t + 1) / np); ++j) {
                    const uint32_t q = k.i0 + j;
                    if (!frame_end(q)) continue;
                    const uint64_t o = (uint64_t)h_desc[q].off16 * 16u;
                    memcpy(h_arena + o, c->h_arena[s] + (o - k.base), staged_desc(h_desc[q], arena_bytes).len);
                }
            });
        }
        if (h_status) memcpy(h_status + k.i0, c->h_status[s], m);
    };

    uint32_t i = 0;
    int s = 0;
    while (i < n && e == hipSuccess) {
        // next chunk: packets [i, i1) in ascending arena order whose in-arena frames fit one
        // staging slot (a ring wrap closes the chunk: the next one starts at the lower offset)
        const uint64_t base = std::min<uint64_t>((uint64_t)h_desc[i].off16 * 16u, arena_bytes);
        uint32_t i1 = i;
        uint64_t end = base;
        while (i1 < n && i1 - i < c->stage_pkts) {
            if (i1 > i && h_desc[i1].off16 < h_desc[i1 - 1].off16) break;
            const uint64_t fe = frame_end(i1);
            const uint64_t ne = std::max(end, fe);
            if (ne - base > c->stage_bytes) break;  // i1 > i: a single frame always fits (above)
            if (i1 > i && ne - base > chunk_target) break;
            end = ne;
            ++i1;
        }
        // With patch records back, the slot's host arena and descriptors are free again once chunk
        // k-2 has been copied in (`staged`), so chunk k's staging copy runs before chunk k-2's
        // patches are applied and beside chunk k-1's transfer (round 5); with whole frames back the
        // slot's arena receives them, and chunk k-2 is finished first
        if (!patch_only) {
            finish(s);
        } else if (slot[s].used) {
            e = wait_slot(c, s, c->staged[s]);
        }
        if (e != hipSuccess) break;
        const uint32_t m = i1 - i;
        const uint64_t bytes = end - base;
        const uint8_t* src = h_arena + base;
        // a direct chunk (records back, small): no DMA; the kernel reads a pinned arena in place
        uint8_t* zsrc = nullptr;
        if (patch_only && c->z_block[s] && bytes <= kDirectChunkBytes && (!pinned || aligned)) {
            if (pinned) {
                void* dp = nullptr;
                if (hipHostGetDevicePointer(&dp, h_arena, 0) == hipSuccess) zsrc = static_cast<uint8_t*>(dp) + base;
                else (void)hipGetLastError();
            } else {
                zsrc = zdev(c, s, c->h_arena[s]);
            }
        }
        if (!pinned) {
            par_memcpy(c, c->h_arena[s], src, bytes);
            src = c->h_arena[s];
        }
        stage_descs(c->h_desc[s], h_desc + i, m, arena_bytes, any_long);
        if (patch_only) {
            finish(s);  // chunk k-2's records and statuses are read out before chunk k's land
            if (e != hipSuccess) break;
        }
        hipStream_t st = c->hs[s];
        if (zsrc) {
            e = nfcs::launch_update(c->di, zsrc, bytes ? bytes : 16, zdev(c, s, c->h_desc[s]), m, (uint32_t)(base >> 4),
                                    h_status ? zdev(c, s, c->h_status[s]) : nullptr, zdev(c, s, c->h_patch[s]),
                                    nullptr, nfcs::kUpdateRecords, st, 0, {}, done_req(c, s));
            if (e == hipSuccess) e = hipEventRecord(c->staged[s], st);  // the kernel read the slot
            if (e == hipSuccess) e = hipEventRecord(c->done[s], st);
            if (e != hipSuccess) {
                (void)hipStreamSynchronize(st);
                break;
            }
            slot[s] = {i, i1, base, bytes, true};
            i = i1;
            s ^= 1;
            continue;
        }
        event_wait(c, s);
        e = hipMemcpyAsync(c->d_desc[s], c->h_desc[s], (size_t)m * sizeof(nfcs_desc),
                           hipMemcpyHostToDevice, st);
        if (e == hipSuccess && bytes)
            e = hipMemcpyAsync(c->d_arena[s], src, bytes, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipEventRecord(c->staged[s], st);
        if (e == hipSuccess)
            e = nfcs::launch_update(c->di, c->d_arena[s], bytes, c->d_desc[s], m, (uint32_t)(base >> 4),
                                    c->d_status[s], patch_only ? c->d_patch[s] : nullptr,
                                    patch_only ? nullptr : c->d_patch[s],
                                    patch_only ? nfcs::kUpdateRecords : nfcs::kUpdateAuto, st);
        if (e == hipSuccess) {
            if (patch_only)
                e = hipMemcpyAsync(c->h_patch[s], c->d_patch[s], (size_t)m * sizeof(nfcs_patch),
                                   hipMemcpyDeviceToHost, st);
            else if (bytes)
                e = hipMemcpyAsync(pinned && ordered ? h_arena + base : c->h_arena[s], c->d_arena[s], bytes,
                                   hipMemcpyDeviceToHost, st);
        }
        if (e == hipSuccess && h_status)
            e = hipMemcpyAsync(c->h_status[s], c->d_status[s], m, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipEventRecord(c->done[s], st);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(st);  // whatever was queued on this slot has finished
            break;
        }
        slot[s] = {i, i1, base, bytes, true};
        i = i1;
        s ^= 1;
    }
    finish(s);  // drain both slots, also after an error
    finish(s ^ 1);
    if (e != hipSuccess) return hip_fail(e);
    return NFCS_OK;
}

NFCS_API int nfcs_update_host_frames(nfcs_ctx* c, uint8_t* const* frames, const uint32_t* lens, uint32_t n,
                                     uint8_t* h_status, uint32_t flags) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    if (n == 0) return NFCS_OK;
    if (!frames || !lens || flags != 0) return NFCS_EINVAL;
    int rc = ensure_host_pipeline(c);
    if (rc) return rc;
    // a NULL frame is empty; a frame longer than kFrameRelevantBytes is staged as its first
    // kFrameRelevantBytes bytes, which changes nothing (nfcs.h): so no frame outgrows a staging slot
    auto flen = [&](uint32_t i) -> uint64_t { return frames[i] ? std::min(lens[i], nfcs::kFrameRelevantBytes) : 0u; };
    auto pad = [](uint64_t len) { return (len + 15u) & ~15ull; };
    const int parts = c->workers.size() + 1;
    // the burst's padded bytes (every frame fits one staging slot: checked anyway), over the workers
    // for large bursts (no serial pass over the burst on the caller's thread)
    uint64_t chunk_target = 0;
    {
        constexpr int kMaxParts = 65;
        uint64_t tot[kMaxParts] = {};
        bool bad[kMaxParts] = {};
        const int np = n >= 65536 ? std::min(parts, kMaxParts) : 1;
        c->workers.run(np, [&](int t) {
            const uint32_t j0 = (uint32_t)((uint64_t)n * t / np), j1 = (uint32_t)((uint64_t)n * (t + 1) / np);
            uint64_t sum = 0;
            bool b = false;
            for (uint32_t j = j0; j < j1; ++j) {
                const uint64_t l = flen(j);
                b |= l > nfcs_ctx::kStageBytes;
                sum += pad(l);
            }
            tot[t] = sum;
            bad[t] = b;
        });
        uint64_t total = 0;
        for (int t = 0; t < np; ++t) {
            if (bad[t]) return NFCS_EINVAL;
            total += tot[t];
        }
        // chunks of ~a quarter of the burst (at least 4 MiB, at most a staging slot), as
        // nfcs_update_host cuts them
        chunk_target = chunk_bytes(total);
    }

    // The pipeline over the two slots, per chunk k in slot s: wait until chunk k-2's frames and
    // descriptors have been copied in (`staged`: the slot's host arena is free again — not for its
    // kernel and records, round 5), lay out chunk k's descriptors, gather its frames (the workers),
    // then finish chunk k-2 (its records: checksum bytes written into the frames) and queue chunk
    // k's copies, kernel and record copy. So the gather of chunk k runs beside the copy of chunk k-1.
    struct Chunk { uint32_t i0, i1; bool used; };
    Chunk slot[nfcs_ctx::kSlots] = {};
    hipError_t e = hipSuccess;
    // finish a slot: wait for its records, then write each frame's checksum bytes in place (ip
    // field first, then l4: the reference's order, which also reproduces IHL < 5 overlaps) and copy
    // its statuses; after an error the slot is only drained
    auto finish = [&](int s) {
        Chunk& k = slot[s];
        if (!k.used) return;
        k.used = false;
        const hipError_t f = wait_slot(c, s, c->done[s]);
        if (e == hipSuccess) e = f;
        if (e != hipSuccess) return;
        const uint32_t m = k.i1 - k.i0;
        const nfcs_patch* pt = c->h_patch[s];
        const int np = std::min<int>(parts, std::max<uint32_t>(1, m / kPatchFramesPerThread));
        c->workers.run(np, [&](int t) {
            const uint32_t j0 = (uint32_t)((uint64_t)m * t / np), j1 = (uint32_t)((uint64_t)m * (t + 1) / np);
            constexpr uint32_t kPf = 16;  // the header lines of frames kPf ahead: their misses overlap
            for (uint32_t j = j0; j < j1; ++j) {
                if (j + kPf < j1 && frames[k.i0 + j + kPf]) __builtin_prefetch(frames[k.i0 + j + kPf] + 32, 1, 0);
                uint8_t* fr = frames[k.i0 + j];
                if (!fr) continue;
                if (pt[j].ip_off != NFCS_PATCH_NONE) { fr[pt[j].ip_off] = pt[j].ip[0]; fr[pt[j].ip_off + 1] = pt[j].ip[1]; }
                if (pt[j].l4_off != NFCS_PATCH_NONE) { fr[pt[j].l4_off] = pt[j].l4[0]; fr[pt[j].l4_off + 1] = pt[j].l4[1]; }
            }
        });
        if (h_status) memcpy(h_status + k.i0, c->h_status[s], m);
    };

    uint32_t i = 0;
    int s = 0;
    while (i < n && e == hipSuccess) {
        if (slot[s].used) {  // chunk k-2's copies in are done: its arena and descriptors are free
            e = wait_slot(c, s, c->staged[s]);
            if (e != hipSuccess) break;
        }
        // next chunk: packets [i, i1), their 16-byte padded frames within chunk_target bytes (at
        // least one) and the slot's descriptor room, laid out back to back in the slot
        nfcs_desc* hd = c->h_desc[s];
        uint32_t i1 = i;
        uint64_t bytes = 0;
        while (i1 < n && i1 - i < c->stage_pkts) {
            const uint64_t l = flen(i1), b = bytes + pad(l);
            if (i1 > i && b > chunk_target) break;
            hd[i1 - i] = nfcs_desc{(uint32_t)(bytes >> 4), (uint32_t)l};
            bytes = b;
            ++i1;
        }
        const uint32_t m = i1 - i;
        uint8_t* dst = c->h_arena[s];
        const int ng = (int)std::min<uint64_t>(parts, std::max<uint64_t>(1, bytes / kCopyBytesPerThread));
        c->workers.run(ng, [&](int t) {
            const uint32_t j0 = (uint32_t)((uint64_t)m * t / ng), j1 = (uint32_t)((uint64_t)m * (t + 1) / ng);
            constexpr uint32_t kPf = 4;  // the first lines of the frame kPf ahead: its misses overlap this copy
            for (uint32_t j = j0; j < j1; ++j) {
                if (j + kPf < j1 && frames[i + j + kPf]) {
                    __builtin_prefetch(frames[i + j + kPf], 0, 0);
                    __builtin_prefetch(frames[i + j + kPf] + 64, 0, 0);
                    __builtin_prefetch(frames[i + j + kPf] + 128, 0, 0);
                }
                const uint64_t len = hd[j].len, o = (uint64_t)hd[j].off16 * 16u;
                // the slot's 16-byte padding zeroed: the kernel reads whole 16-byte chunks
                if (len) stream_copy(dst + o, frames[i + j], len, true);
            }
            nt_fence();
        });
        finish(s);  // chunk k-2: its records and statuses are read out of the slot before chunk k's land
        if (e != hipSuccess) break;
        hipStream_t st = c->hs[s];
        if (c->z_block[s] && bytes <= kDirectChunkBytes) {
            // a direct chunk: the kernel reads the gathered frames and descriptors in the pinned slot
            // and writes records and statuses there; no DMA (kDirectChunkBytes)
            e = nfcs::launch_update(c->di, zdev(c, s, dst), bytes ? bytes : 16, zdev(c, s, hd), m, 0u,
                                    h_status ? zdev(c, s, c->h_status[s]) : nullptr, zdev(c, s, c->h_patch[s]),
                                    nullptr, nfcs::kUpdateRecords, st, 0, {}, done_req(c, s));
            if (e == hipSuccess) e = hipEventRecord(c->staged[s], st);
        } else {
            event_wait(c, s);
            e = hipMemcpyAsync(c->d_desc[s], hd, (size_t)m * sizeof(nfcs_desc), hipMemcpyHostToDevice, st);
            if (e == hipSuccess && bytes) e = hipMemcpyAsync(c->d_arena[s], dst, bytes, hipMemcpyHostToDevice, st);
            if (e == hipSuccess) e = hipEventRecord(c->staged[s], st);
            if (e == hipSuccess)
                e = nfcs::launch_update(c->di, c->d_arena[s], bytes ? bytes : 16, c->d_desc[s], m, 0u, c->d_status[s],
                                        c->d_patch[s], nullptr, nfcs::kUpdateRecords, st);
            if (e == hipSuccess)
                e = hipMemcpyAsync(c->h_patch[s], c->d_patch[s], (size_t)m * sizeof(nfcs_patch), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess && h_status) e = hipMemcpyAsync(c->h_status[s], c->d_status[s], m, hipMemcpyDeviceToHost, st);
        }
        if (e == hipSuccess) e = hipEventRecord(c->done[s], st);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(st);  // whatever was queued on this slot has finished
            break;
        }
        slot[s] = {i, i1, true};
        i = i1;
        s ^= 1;
    }
    finish(s);  // drain both slots, also after an error
    finish(s ^ 1);
    if (e != hipSuccess) return hip_fail(e);
    return NFCS_OK;
}

NFCS_API int nfcs_shard_bytes(const nfcs_desc* h_desc, uint32_t n, uint32_t parts, uint32_t* bounds) {
    if (!bounds || parts == 0 || (n && !h_desc)) return NFCS_EINVAL;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += h_desc[i].len;
    // bounds[p] = the first packet at which the running byte count reaches p * total / parts, so
    // every boundary lies within one frame of its ideal position
    uint32_t i = 0;
    uint64_t run = 0;
    bounds[0] = 0;
    for (uint32_t p = 1; p < parts; ++p) {
        const unsigned __int128 t = (unsigned __int128)total * p;
        const uint64_t target = (uint64_t)(t / parts) + (t % parts != 0);
        while (i < n && run < target) run += h_desc[i++].len;
        bounds[p] = i;
    }
    bounds[parts] = n;
    return NFCS_OK;
}

NFCS_API int nfcs_layout_config(int config, uint64_t seed, uint64_t first_index, uint32_t n,
                                uint32_t align, nfcs_desc* h_desc, uint64_t* arena_bytes) {
    if (config < 0 || config > 3 || align < 16 || (align & 15u)) return NFCS_EINVAL;
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t len = nfcs::config_len(config, seed, first_index + i);
        if ((off >> 4) > 0xFFFFFFFFull) return NFCS_EINVAL;
        if (h_desc) h_desc[i] = nfcs_desc{(uint32_t)(off >> 4), len};
        off += ((uint64_t)len + align - 1) / align * align;
    }
    if (arena_bytes) *arena_bytes = off;
    return NFCS_OK;
}

NFCS_API int nfcs_gen_config_device(nfcs_ctx* c, int config, uint64_t seed, uint64_t first,
                                    uint32_t n, uint8_t* d_arena, uint64_t arena_bytes,
                                    const nfcs_desc* d_desc, void* stream) {
    if (!c || config < 0 || config > 3) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    if (n == 0) return NFCS_OK;
    if (!d_arena || !d_desc) return NFCS_EINVAL;
    // padding between aligned frame starts is zeroed too, so the arena is fully defined
    NFCS_HIP(hipMemsetAsync(d_arena, 0, arena_bytes, pick(c, stream)));
    NFCS_HIP(nfcs::launch_gen_config(c->di, config, seed, first, n, d_arena, arena_bytes, d_desc,
                                     pick(c, stream)));
    return NFCS_OK;
}

NFCS_API int nfcs_digest_device(nfcs_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes,
                                const nfcs_desc* d_desc, uint32_t n, uint64_t first,
                                uint64_t* h_digest, void* stream) {
    if (!c || !h_digest) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipStream_t st = pick(c, stream);
    NFCS_HIP(hipMemsetAsync(c->d_digest, 0, sizeof(uint64_t), st));
    if (n) {
        if (!d_arena || !d_desc) return NFCS_EINVAL;
        NFCS_HIP(nfcs::launch_digest(c->di, d_arena, arena_bytes, d_desc, n, first, c->d_digest, st));
    }
    NFCS_HIP(hipMemcpyAsync(h_digest, c->d_digest, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    NFCS_HIP(hipStreamSynchronize(st));
    return NFCS_OK;
}

NFCS_API int nfcs_device_alloc(nfcs_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipError_t e = hipMalloc(out, bytes ? bytes : 16);
    if (e == hipErrorOutOfMemory) { (void)hipGetLastError(); return NFCS_ENOMEM; }
    NFCS_HIP(e);
    return NFCS_OK;
}
NFCS_API int nfcs_device_free(nfcs_ctx* c, void* p) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    NFCS_HIP(hipFree(p));
    return NFCS_OK;
}
NFCS_API int nfcs_host_alloc(nfcs_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipError_t e = hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault);
    if (e == hipErrorOutOfMemory) { (void)hipGetLastError(); return NFCS_ENOMEM; }
    NFCS_HIP(e);
    return NFCS_OK;
}
NFCS_API int nfcs_host_free(nfcs_ctx* c, void* p) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    NFCS_HIP(hipHostFree(p));
    return NFCS_OK;
}
NFCS_API int nfcs_memcpy_h2d(nfcs_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    NFCS_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    NFCS_HIP(hipStreamSynchronize(c->stream));
    return NFCS_OK;
}
NFCS_API int nfcs_memcpy_d2h(nfcs_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    NFCS_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    NFCS_HIP(hipStreamSynchronize(c->stream));
    return NFCS_OK;
}
NFCS_API int nfcs_stream_sync(nfcs_ctx* c, void* stream) {
    if (!c) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    NFCS_HIP(hipStreamSynchronize(pick(c, stream)));
    return NFCS_OK;
}


NFCS_API int nfcs_time_update_device(nfcs_ctx* c, uint8_t* d_arena, uint64_t arena_bytes,
                                     const nfcs_desc* d_desc, uint32_t n, uint8_t* d_status,
                                     int iters, void* stream, float* ms) {
    if (!c || !ms || iters <= 0) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipStream_t st = pick(c, stream);
    if (!d_arena || !d_desc || ((uintptr_t)d_arena & 15u)) return NFCS_EINVAL;
    NFCS_HIP(hipEventRecord(c->ev0, st));
    for (int it = 0; it < iters; ++it) {
        const int rc = update_device(c, d_arena, arena_bytes, d_desc, n, d_status, nullptr, st);
        if (rc) return rc;
    }
    NFCS_HIP(hipEventRecord(c->ev1, st));
    NFCS_HIP(hipEventSynchronize(c->ev1));
    NFCS_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return NFCS_OK;
}

NFCS_API int nfcs_time_update_batches(nfcs_ctx* c, uint32_t batches, uint8_t* const* d_arenas,
                                      const uint64_t* arena_bytes, const nfcs_desc* const* d_descs,
                                      uint32_t n, int iters, void* stream, float* ms) {
    if (!c || !ms || iters <= 0 || batches == 0 || !d_arenas || !arena_bytes || !d_descs) return NFCS_EINVAL;
    for (uint32_t b = 0; b < batches; ++b)
        if (!d_arenas[b] || !d_descs[b] || ((uintptr_t)d_arenas[b] & 15u)) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipStream_t st = pick(c, stream);
    NFCS_HIP(hipEventRecord(c->ev0, st));
    for (int it = 0; it < iters; ++it) {
        const uint32_t b = (uint32_t)it % batches;
        const int rc = update_device(c, d_arenas[b], arena_bytes[b], d_descs[b], n, nullptr, nullptr, st);
        if (rc) return rc;
    }
    NFCS_HIP(hipEventRecord(c->ev1, st));
    NFCS_HIP(hipEventSynchronize(c->ev1));
    NFCS_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return NFCS_OK;
}

NFCS_API int nfcs_time_l3_forward_device(nfcs_ctx* c, uint8_t* d_arena, uint64_t arena_bytes,
                                         const nfcs_desc* d_desc, const uint32_t* d_nh,
                                         uint32_t n, const nfcs_nexthop* d_table, uint32_t table_n,
                                         uint8_t* d_status, int iters, void* stream, float* ms) {
    if (!c || !ms || iters <= 0 || !d_arena || !d_desc || !d_nh) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipStream_t st = pick(c, stream);
    NFCS_HIP(hipEventRecord(c->ev0, st));
    for (int it = 0; it < iters; ++it) {
        const int rc = l3_forward_device(c, d_arena, arena_bytes, d_desc, d_nh, n, d_table, table_n,
                                         d_status, st);
        if (rc) return rc;
    }
    NFCS_HIP(hipEventRecord(c->ev1, st));
    NFCS_HIP(hipEventSynchronize(c->ev1));
    NFCS_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return NFCS_OK;
}

NFCS_API int nfcs_time_vlan_device(nfcs_ctx* c, uint8_t* d_arena, uint64_t arena_bytes,
                                   nfcs_desc* d_desc, uint32_t n, uint32_t op_all,
                                   uint32_t op_alt, uint32_t cap_all, uint8_t* d_status, int iters,
                                   void* stream, float* ms) {
    if (!c || !ms || iters <= 0 || !d_arena || !d_desc) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipStream_t st = pick(c, stream);
    NFCS_HIP(hipEventRecord(c->ev0, st));
    for (int it = 0; it < iters; ++it) {
        const Shape sh = launch_shape(c, arena_bytes, d_desc, n, kVlanRule);
        NFCS_HIP(nfcs::launch_vlan(c->di, d_arena, arena_bytes, d_desc, n, nullptr,
                                   (it & 1) ? op_alt : op_all, nullptr, cap_all, d_status, st,
                                   sh.mean, sh.obs, sh.bits));
    }
    NFCS_HIP(hipEventRecord(c->ev1, st));
    NFCS_HIP(hipEventSynchronize(c->ev1));
    NFCS_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return NFCS_OK;
}

NFCS_API int nfcs_time_flow_keys_device(nfcs_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes,
                                        const nfcs_desc* d_desc, uint32_t n, nfcs_flow_key* d_keys,
                                        uint32_t* d_hash, int iters, void* stream, float* ms) {
    if (!c || !ms || iters <= 0 || !d_arena || !d_desc) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipStream_t st = pick(c, stream);
    NFCS_HIP(hipEventRecord(c->ev0, st));
    for (int it = 0; it < iters; ++it)
        NFCS_HIP(nfcs::launch_flow_keys(c->di, d_arena, arena_bytes, d_desc, n, d_keys, d_hash, st));
    NFCS_HIP(hipEventRecord(c->ev1, st));
    NFCS_HIP(hipEventSynchronize(c->ev1));
    NFCS_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return NFCS_OK;
}

NFCS_API int nfcs_time_stream_read(nfcs_ctx* c, const uint8_t* d_buf, uint64_t bytes, int form, int iters,
                                   void* stream, float* ms) {
    if (!c || !ms || iters <= 0 || !d_buf || form < 0 || form > 5 || ((uintptr_t)d_buf & 15u))
        return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipStream_t st = pick(c, stream);
    unsigned long long* sink = reinterpret_cast<unsigned long long*>(c->d_digest);
    NFCS_HIP(hipEventRecord(c->ev0, st));
    for (int it = 0; it < iters; ++it) NFCS_HIP(nfcs::launch_stream_read(d_buf, bytes, form, sink, st));
    NFCS_HIP(hipEventRecord(c->ev1, st));
    NFCS_HIP(hipEventSynchronize(c->ev1));
    NFCS_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return NFCS_OK;
}

NFCS_API int nfcs_time_frames_read(nfcs_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes,
                                   const nfcs_desc* d_desc, uint32_t n, int iters, void* stream, float* ms) {
    if (!c || !ms || iters <= 0 || !d_arena || !d_desc || ((uintptr_t)d_arena & 15u)) return NFCS_EINVAL;
    DeviceGuard dg_(c->di.device);  // the context's device on this thread, restored on return
    if (dg_.err != hipSuccess) return hip_fail(dg_.err);
    hipStream_t st = pick(c, stream);
    unsigned long long* sink = reinterpret_cast<unsigned long long*>(c->d_digest);
    NFCS_HIP(hipEventRecord(c->ev0, st));
    for (int it = 0; it < iters; ++it) NFCS_HIP(nfcs::launch_frames_read(d_arena, arena_bytes, d_desc, n, sink, st));
    NFCS_HIP(hipEventRecord(c->ev1, st));
    NFCS_HIP(hipEventSynchronize(c->ev1));
    NFCS_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return NFCS_OK;
}

}  // extern "C"
