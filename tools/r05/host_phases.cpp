// host_phases — measurement tool (not product): where the time of nfcs_update_host_frames goes for
// BASELINE C1's 1M frames held one heap buffer each (as the reference's PacketBuffers are), on the
// GPU box. Times, wall clock, best of R after restoring the frames:
//   call         the product call (gather -> H2D -> kernel -> records D2H -> checksum bytes written back)
//   gather_nt/T  the gather alone into two 64 MiB pinned slots, non-temporal stores (the product's
//                copy loop), T threads
//   gather_mc/T  the same with plain memcpy
//   h2d          1.57 GB pinned -> device in 64 MiB copies (nfcs_memcpy_h2d, synchronous)
//   scatter/T    4 bytes written into every frame's header (the write-back), T threads
// Build: tools/r05/build_host_phases.sh. Run: host_phases [n] [reps]. One JSON line.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "nfcs.h"

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

template <class F>
static void par(size_t threads, size_t n, const F& f) {  // f(i0, i1) over contiguous slices
    std::vector<std::thread> th;
    for (size_t t = 1; t < threads; ++t) th.emplace_back([&, t] { f(n * t / threads, n * (t + 1) / threads); });
    f(0, n / threads);
    for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
    using clk = std::chrono::steady_clock;
    const size_t n = argc > 1 ? std::stoul(argv[1]) : (1u << 20);
    const size_t reps = argc > 2 ? std::stoul(argv[2]) : 5;
    nfcs_ctx* c = nullptr;
    if (nfcs_ctx_create(0, &c)) return 1;
    std::vector<nfcs_desc> desc(n);
    uint64_t bytes = 0;
    if (nfcs_layout_config(NFCS_CFG_C1_1500B_UDP, 20250620ull, 0, (uint32_t)n, 16, desc.data(), &bytes)) return 1;
    void *d_arena = nullptr, *d_desc = nullptr;
    if (nfcs_device_alloc(c, bytes, &d_arena) || nfcs_device_alloc(c, n * sizeof(nfcs_desc), &d_desc)) return 1;
    if (nfcs_memcpy_h2d(c, d_desc, desc.data(), n * sizeof(nfcs_desc))) return 1;
    if (nfcs_gen_config_device(c, NFCS_CFG_C1_1500B_UDP, 20250620ull, 0, (uint32_t)n, (uint8_t*)d_arena, bytes,
                               (nfcs_desc*)d_desc, nullptr) || nfcs_stream_sync(c, nullptr))
        return 1;
    std::vector<uint8_t> pristine(bytes);
    if (nfcs_memcpy_d2h(c, pristine.data(), d_arena, bytes)) return 1;
    double frame_bytes = 0;
    for (size_t i = 0; i < n; ++i) frame_bytes += desc[i].len;

    // one heap buffer per frame, 32 bytes of headroom (netflow::PacketBuffer's layout)
    std::vector<uint8_t*> buf(n), frames(n);
    std::vector<uint32_t> lens(n);
    for (size_t i = 0; i < n; ++i) {
        buf[i] = new uint8_t[32 + 1536];
        frames[i] = buf[i] + 32;
        lens[i] = desc[i].len;
    }
    auto restore = [&] {
        par(16, n, [&](size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; ++i) memcpy(frames[i], pristine.data() + (size_t)desc[i].off16 * 16, lens[i]);
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
    std::string out = "{";
    auto put = [&](const char* k, double s) {
        char t[128];
        std::snprintf(t, sizeof(t), "%s\"%s\": {\"ms\": %.3f, \"GBps\": %.2f}", out.size() > 1 ? ", " : "", k, s * 1e3,
                      frame_bytes / s / 1e9);
        out += t;
    };

    int rc = 0;
    nfcs_update_host_frames(c, frames.data(), lens.data(), (uint32_t)n, nullptr, 0);  // warm the pipeline
    put("call", best([&] { rc |= nfcs_update_host_frames(c, frames.data(), lens.data(), (uint32_t)n, nullptr, 0); }));

    const size_t slot = 64u << 20;
    void* pin = nullptr;
    if (nfcs_host_alloc(c, 2 * slot, &pin)) return 1;
    uint8_t* ps = (uint8_t*)pin;
    memset(ps, 0, 2 * slot);
    const size_t per = slot / 1504;
    for (size_t T : {4, 8, 9, 12, 16}) {
        for (int nt = 1; nt >= 0; --nt) {
            const double s = best([&] {
                for (size_t i0 = 0, k = 0; i0 < n; i0 += per, ++k) {
                    const size_t m = std::min(per, n - i0);
                    uint8_t* d = ps + (k & 1) * slot;
                    par(T, m, [&](size_t j0, size_t j1) {
                        for (size_t j = j0; j < j1; ++j) {
                            if (j + 4 < j1) {
                                __builtin_prefetch(frames[i0 + j + 4], 0, 0);
                                __builtin_prefetch(frames[i0 + j + 4] + 64, 0, 0);
                                __builtin_prefetch(frames[i0 + j + 4] + 128, 0, 0);
                            }
                            if (nt) copy_nt(d + j * 1504, frames[i0 + j], lens[i0 + j]);
                            else memcpy(d + j * 1504, frames[i0 + j], lens[i0 + j]);
                        }
                        __builtin_ia32_sfence();
                    });
                }
            });
            const std::string k = std::string(nt ? "gather_nt/" : "gather_mc/") + std::to_string(T);
            put(k.c_str(), s);
        }
    }
    // H2D of the whole burst in 64 MiB copies from the two pinned slots (the slots' bytes, any)
    put("h2d", best([&] {
        for (uint64_t o = 0, k = 0; o < bytes; o += slot, ++k)
            rc |= nfcs_memcpy_h2d(c, (uint8_t*)d_arena + o, ps + (k & 1) * slot, std::min<uint64_t>(slot, bytes - o));
    }));
    for (size_t T : {1, 8, 9, 16}) {
        const double s = best([&] {
            par(T, n, [&](size_t j0, size_t j1) {
                for (size_t j = j0; j < j1; ++j) {
                    if (j + 16 < j1) __builtin_prefetch(frames[j + 16] + 16, 1, 0);
                    uint8_t* f = frames[j];
                    f[24] ^= 1; f[25] ^= 1; f[40] ^= 1; f[41] ^= 1;
                }
            });
        });
        const std::string k = "scatter/" + std::to_string(T);
        put(k.c_str(), s);
    }
    out += "}";
    std::printf("%s\n", out.c_str());
    nfcs_host_free(c, pin);
    nfcs_device_free(c, d_arena);
    nfcs_device_free(c, d_desc);
    for (auto* b : buf) delete[] b;
    nfcs_ctx_destroy(c);
    return rc ? 1 : 0;
}
