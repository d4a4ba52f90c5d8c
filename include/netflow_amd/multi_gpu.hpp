// multi_gpu.hpp — one host-memory burst over several GPUs, header-only over the C ABI.
//
// Packets are independent (packet.hpp:722-890 reads only its own frame), so a burst is split into
// contiguous ranges balanced by frame bytes (nfcs_shard_bytes) and each range goes to its own GPU
// context, driven by its own host thread: nfcs_update_host stages the range through that context's
// pinned ring, which sits on its GPU's NUMA node, with copy threads on that node's CPUs. No
// collective, no cross-GPU traffic. The ranges are disjoint sets of frames in one arena, so the
// contexts write disjoint bytes. Errors are return codes (never exceptions), as in the reference's
// void / silent-skip contract (packet.hpp:722-723).
//
//   int rc = 0;
//   netflow_amd::MultiGpu mg({0, 1, 2, 3, 4, 5, 6, 7}, std::nothrow, &rc);
//   if (rc == NFCS_OK) rc = mg.update_host(arena, arena_bytes, desc, n, status);
#pragma once

#include <new>
#include <thread>
#include <vector>

#include "nfcs.h"

namespace netflow_amd {

class MultiGpu {
public:
    // One context per listed device (a device may repeat: several contexts on one GPU). *rc is
    // NFCS_OK, or the first context's error (then no context is kept).
    MultiGpu(const std::vector<int>& devices, std::nothrow_t, int* rc) {
        int e = devices.empty() ? NFCS_EINVAL : NFCS_OK;
        try {
            ctx_.reserve(devices.size());  // push_back below then never allocates
        } catch (...) {
            e = NFCS_ENOMEM;
        }
        for (size_t i = 0; i < devices.size() && e == NFCS_OK; ++i) {
            nfcs_ctx* c = nullptr;
            e = nfcs_ctx_create(devices[i], &c);
            if (e == NFCS_OK) ctx_.push_back(c);
        }
        if (e != NFCS_OK) release();
        if (rc) *rc = e;
    }
    ~MultiGpu() { release(); }
    MultiGpu(const MultiGpu&) = delete;
    MultiGpu& operator=(const MultiGpu&) = delete;

    size_t size() const { return ctx_.size(); }
    nfcs_ctx* context(size_t i) const { return ctx_[i]; }

    // nfcs_update_host over the contexts: descriptors in any order (ABI 2: each context stages its
    // range's runs of ascending offsets as spans, so a range in arena order stages as one span);
    // status (optional) receives every packet's NFCS_ST_* byte at its own index. bounds (optional,
    // size() + 1 entries) receives the ranges used: context p took packets [bounds[p], bounds[p+1]).
    // Returns NFCS_OK or the first negative error of any range (every range has finished by then).
    int update_host(uint8_t* h_arena, uint64_t arena_bytes, const nfcs_desc* h_desc, uint32_t n,
                    uint8_t* h_status = nullptr, uint32_t flags = 0, uint32_t* bounds = nullptr) {
        if (ctx_.empty()) return NFCS_EINVAL;
        if (n == 0) return NFCS_OK;
        const uint32_t parts = (uint32_t)ctx_.size();
        // the per-call bookkeeping, allocated up front: bad_alloc becomes NFCS_ENOMEM (never throw)
        std::vector<uint32_t> b;
        std::vector<int> res;
        std::vector<std::thread> th;
        try {
            b.resize(parts + 1);
            res.assign(parts, NFCS_OK);
            th.reserve(parts);
        } catch (...) {
            return NFCS_ENOMEM;
        }
        int rc = nfcs_shard_bytes(h_desc, n, parts, b.data());
        if (rc != NFCS_OK) return rc;
        for (uint32_t p = 1; p < parts; ++p) {
            try {
                th.emplace_back([&, p] { res[p] = run(p, b, h_arena, arena_bytes, h_desc, h_status, flags); });
            } catch (...) {  // no thread to be had: run that range here, in turn (never throw)
                res[p] = run(p, b, h_arena, arena_bytes, h_desc, h_status, flags);
            }
        }
        res[0] = run(0, b, h_arena, arena_bytes, h_desc, h_status, flags);
        for (auto& t : th) t.join();
        if (bounds)
            for (uint32_t p = 0; p <= parts; ++p) bounds[p] = b[p];
        for (int r : res)
            if (r != NFCS_OK) return r;
        return NFCS_OK;
    }

private:
    int run(uint32_t p, const std::vector<uint32_t>& b, uint8_t* h_arena, uint64_t arena_bytes,
            const nfcs_desc* h_desc, uint8_t* h_status, uint32_t flags) {
        const uint32_t first = b[p], m = b[p + 1] - b[p];
        if (m == 0) return NFCS_OK;
        return nfcs_update_host(ctx_[p], h_arena, arena_bytes, h_desc + first, m,
                                h_status ? h_status + first : nullptr, flags);
    }
    void release() {
        for (nfcs_ctx* c : ctx_) nfcs_ctx_destroy(c);
        ctx_.clear();
    }
    std::vector<nfcs_ctx*> ctx_;
};

}  // namespace netflow_amd
