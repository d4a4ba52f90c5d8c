// netflow_amd/packet.hpp — C++ host API for NetFlow++ callers of the checksum path.
//
// Mirrors the reference types a caller of Packet::update_checksums() holds:
//   netflow::PacketBuffer   include/netflow++/packet_buffer.hpp:10-111
//   netflow::Packet         include/netflow++/packet.hpp:344-918 (ctor/dtor 346-357,
//                           get_buffer 379, update_checksums 722-890)
// with the same member names, argument meaning and error behaviour, and adds the batched
// entry point that the reference lacks:
//   netflow_amd::update_checksums_batch(Packet* const*, size_t)
// which hands each PacketBuffer's data window to nfcs_update_host_frames (include/nfcs.h): the
// frames are gathered chunk by chunk into a pinned, NUMA-local ring, checksummed on the gfx950
// engine, and the 2+2 checksum bytes written back into each PacketBuffer in place, the chunks
// pipelined — bit-exact with the reference; and
// the batched form of Packet::push_vlan / pop_vlan (packet.hpp:655-720)
//   netflow_amd::vlan_batch(Packet* const*, const uint32_t* ops, size_t, bool* ok)
// (nfcs_vlan_device: tag insert / strip / re-tag and the checksums in one pass); the switch's
// transit-IPv4 forward (switch.hpp:247-294) for a burst
//   netflow_amd::l3_forward_batch(Packet* const*, const uint32_t* next_hop, size_t, table, ...)
// (nfcs_l3_forward_device: TTL--, MAC rewrite and the checksums in one pass); and
// PacketClassifier::extract_flow_key + hash_flow (packet_classifier.cpp:12-108) for a burst
//   netflow_amd::flow_keys_batch(Packet* const*, size_t, nfcs_flow_key*, uint32_t* hashes)
// (nfcs_flow_keys_device: 64-byte FlowKey records in host order + hash_flow values).
//
// The batch entry points are templates over the packet type: they take this header's Packet or
// the reference's own netflow::Packet (include/netflow_amd/netflow_adapter.hpp), whose buffers
// offer the same PacketBuffer members. Bursts run on the GPU only — there is no CPU fallback, and
// constructing the engine without a gfx950 device throws std::runtime_error ("fail loudly"). The
// single-packet members (Packet::update_checksums, push_vlan, pop_vlan) run on the host CPU like
// the reference's (include/netflow_amd/cpu_update.hpp): void / bool, never throwing.
// Header-only; link with -lnfcs (netflow_amd/libnfcs.so).
#pragma once

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "nfcs.h"
#include "netflow_amd/cpu_update.hpp"

namespace netflow_amd {

namespace detail {
// f(i0, i1) over [0, n) split across up to 8 threads for big bursts (the per-packet Packet ->
// PacketBuffer loads of a burst of a million scattered objects take ~10 ms on one core); never throws:
// a thread that cannot be started runs its range here.
template <class F>
void parallel_ranges(size_t n, F&& f) {
    const size_t nt = n >= (size_t(1) << 16) ? 8 : 1;
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; ++t) {
        try {
            th.emplace_back([&f, n, t, nt] { f(n * t / nt, n * (t + 1) / nt); });
        } catch (...) {
            f(n * t / nt, n * (t + 1) / nt);
        }
    }
    f(size_t(0), n / nt);
    for (auto& x : th) x.join();
}
}  // namespace detail

// The caller-facing contract of netflow::PacketBuffer (packet_buffer.hpp:10-111): the same
// constructor arguments, accessors, ref_count and refcount calls, bool results of the window edits,
// and exception types (std::invalid_argument from the constructor, std::out_of_range from
// reset_offsets_and_len). Held here as a window [head_, head_ + len_) into cap_ bytes of storage
// that the buffer owns, or, built External, borrows (a BufferPool's pinned arena slot).
class PacketBuffer {
public:
    std::atomic<int> ref_count{1};

    PacketBuffer(size_t capacity, size_t initial_headroom = 0, size_t initial_data_len = 0)
        : owned_(window_fits(capacity, initial_headroom, initial_data_len, "PacketBuffer")
                     ? new unsigned char[capacity] : nullptr),
          base_(owned_.get()), cap_(capacity), head_(initial_headroom), len_(initial_data_len) {}
    struct External {};
    PacketBuffer(External, unsigned char* storage, size_t capacity, size_t initial_headroom = 0,
                 size_t initial_data_len = 0)
        : base_(window_fits(capacity, initial_headroom, initial_data_len, "PacketBuffer(External)")
                    ? storage : nullptr),
          cap_(capacity), head_(initial_headroom), len_(initial_data_len) {}
    PacketBuffer(const PacketBuffer&) = delete;
    PacketBuffer& operator=(const PacketBuffer&) = delete;

    void increment_ref() { ref_count.fetch_add(1, std::memory_order_relaxed); }
    // true when this call dropped the last reference
    bool decrement_ref() { return ref_count.fetch_sub(1, std::memory_order_acq_rel) == 1; }

    unsigned char* get_data_start_ptr() const { return base_ + head_; }
    size_t get_data_length() const { return len_; }
    size_t get_capacity() const { return cap_; }
    size_t get_headroom() const { return head_; }
    size_t get_tailroom() const { return cap_ - head_ - len_; }
    unsigned char* storage() const { return base_; }  // byte 0 of the capacity

    // Window edits: false (and no change) when the new window would leave [0, capacity).
    bool set_data_len(size_t n) { return place(head_, n); }
    bool append_data(size_t n) { return n <= get_tailroom() && place(head_, len_ + n); }
    bool prepend_data(size_t n) { return n <= head_ && place(head_ - n, len_ + n); }
    bool consume_data_front(size_t n) { return n <= len_ && place(head_ + n, len_ - n); }
    bool consume_data_end(size_t n) { return n <= len_ && place(head_, len_ - n); }
    void reset_offsets_and_len(size_t new_offset, size_t new_len) {
        if (!place(new_offset, new_len))
            throw std::out_of_range("netflow_amd::PacketBuffer::reset_offsets_and_len: window past capacity");
    }

private:
    static bool window_fits(size_t cap, size_t head, size_t len, const char* who) {
        if (len > cap || head > cap - len)
            throw std::invalid_argument(std::string("netflow_amd::") + who + ": headroom + data length > capacity");
        return true;
    }
    bool place(size_t head, size_t len) {
        if (len > cap_ || head > cap_ - len) return false;
        head_ = head;
        len_ = len;
        return true;
    }

    std::unique_ptr<unsigned char[]> owned_;
    unsigned char* base_;
    size_t cap_, head_, len_;
};

class Packet;

// One engine per device: owns the nfcs context plus reusable pinned/device staging. Calls
// on one engine are serialised by an internal mutex.
class ChecksumEngine {
public:
    explicit ChecksumEngine(int device = 0) {
        nfcs_ctx* c = nullptr;
        const int rc = nfcs_ctx_create(device, &c);
        if (rc != NFCS_OK)
            throw std::runtime_error(std::string("netflow_amd: no gfx950 engine on device ") +
                                     std::to_string(device) + ": " + nfcs_strerror(rc));
        ctx_ = c;
    }
    // Non-throwing form: *rc receives nfcs_ctx_create's result; the engine is usable iff it is 0.
    ChecksumEngine(int device, std::nothrow_t, int* rc) noexcept {
        nfcs_ctx* c = nullptr;
        const int r = nfcs_ctx_create(device, &c);
        if (rc) *rc = r;
        ctx_ = r == NFCS_OK ? c : nullptr;
    }
    ~ChecksumEngine() {
        if (!ctx_) return;
        release();
        nfcs_ctx_destroy(ctx_);
    }
    ChecksumEngine(const ChecksumEngine&) = delete;
    ChecksumEngine& operator=(const ChecksumEngine&) = delete;

    // Process-wide engine on device 0 (created on first use); throws if there is none.
    static ChecksumEngine& instance() {
        ChecksumEngine* e = try_instance();
        if (!e) throw std::runtime_error("netflow_amd: no gfx950 engine on device 0");
        return *e;
    }
    // The same engine, or nullptr when none could be created (*rc: the nfcs error code). The batch
    // free functions use this and return the code instead of throwing.
    static ChecksumEngine* try_instance(int* rc = nullptr) noexcept {
        static int err = NFCS_OK;
        static ChecksumEngine e(0, std::nothrow, &err);
        if (rc) *rc = err;
        return err == NFCS_OK ? &e : nullptr;
    }

    // Batched Packet::update_checksums(): frames updated in place in their PacketBuffers.
    // status (optional) receives one NFCS_ST_* byte per packet. Returns 0 or an NFCS_E* code.
    // Pkt: netflow_amd::Packet or netflow::Packet (anything whose get_buffer() has the
    // PacketBuffer window members).
    template <class Pkt>
    int update_checksums_batch(Pkt* const* pkts, size_t n, uint8_t* status = nullptr);

    // Batched Packet::push_vlan(vid, prio) / pop_vlan() (packet.hpp:655-720), each with the
    // update_checksums() it ends with. ops[i] is an NFCS_VLAN_* edit word (NFCS_VLAN_PUSH_OP(vid,
    // prio), NFCS_VLAN_POP or NFCS_VLAN_NOP); ok[i] (optional) receives what the reference call
    // returns; each PacketBuffer's data length changes as the reference changes it. The buffer's
    // room for a push is its capacity minus headroom (tailroom = that minus the length).
    template <class Pkt>
    int vlan_batch(Pkt* const* pkts, const uint32_t* ops, size_t n, bool* ok = nullptr,
                   uint8_t* status = nullptr);

    // Batched data path of the switch's transit-IPv4 forward (switch.hpp:247-294): for packet i
    // with an IPv4 header, TTL <= 1 -> NFCS_ST_TTL_EXPIRED and next_hop[i] >= table_n ->
    // NFCS_ST_NO_ROUTE (frame untouched, as the switch drops or punts it); otherwise TTL--,
    // dst/src MAC = table[next_hop[i]] and update_checksums(), status | NFCS_ST_FLAG_FWD. The
    // route and ARP lookups stay with the caller (next_hop indexes; NFCS_NH_NONE = no route).
    template <class Pkt>
    int l3_forward_batch(Pkt* const* pkts, const uint32_t* next_hop, size_t n,
                         const nfcs_nexthop* table, uint32_t table_n, uint8_t* status = nullptr);

    // PacketClassifier::extract_flow_key(pkt) and hash_flow(key) (packet_classifier.cpp:12-108)
    // for a batch: keys[i] (optional) = the FlowKey fields in host order (nfcs_flow_key, with
    // the hash in .hash), hashes[i] (optional) = hash_flow(key).
    template <class Pkt>
    int flow_keys_batch(Pkt* const* pkts, size_t n, nfcs_flow_key* keys, uint32_t* hashes = nullptr);

    nfcs_ctx* ctx() const { return ctx_; }

    // nfcs_update_host on this engine's context, serialised with its other calls.
    int update_host(uint8_t* h_arena, uint64_t arena_bytes, const nfcs_desc* h_desc, uint32_t n,
                    uint8_t* h_status, uint32_t flags) {
        std::lock_guard<std::mutex> lock(mu_);
        return nfcs_update_host(ctx_, h_arena, arena_bytes, h_desc, n, h_status, flags);
    }
    // nfcs_update_host_frames on this engine's context, serialised with its other calls.
    int update_host_frames(uint8_t* const* frames, const uint32_t* lens, uint32_t n, uint8_t* h_status) {
        std::lock_guard<std::mutex> lock(mu_);
        return nfcs_update_host_frames(ctx_, frames, lens, n, h_status, 0);
    }

private:
    // A device buffer for one call (next-hop tables, flow-key records).
    struct DevTmp {
        nfcs_ctx* c;
        void* p = nullptr;
        DevTmp(nfcs_ctx* c_, size_t bytes, int& rc) : c(c_) {
            if (!rc) rc = nfcs_device_alloc(c, bytes ? bytes : 16, &p);
        }
        ~DevTmp() { if (p) nfcs_device_free(c, p); }
    };
    // Gather each packet's first min(len, limit) bytes (limit 0: all) into 16-byte aligned
    // slots of the pinned arena; returns the arena bytes used.
    template <class Pkt>
    size_t gather(Pkt* const* pkts, size_t n, size_t limit);

    void release() {
        if (h_arena_) nfcs_host_free(ctx_, h_arena_);
        if (h_desc_) nfcs_host_free(ctx_, h_desc_);
        if (h_patch_) nfcs_host_free(ctx_, h_patch_);
        if (d_arena_) nfcs_device_free(ctx_, d_arena_);
        if (d_desc_) nfcs_device_free(ctx_, d_desc_);
        if (d_patch_) nfcs_device_free(ctx_, d_patch_);
        if (d_status_) nfcs_device_free(ctx_, d_status_);
        if (h_ops_) nfcs_host_free(ctx_, h_ops_);
        if (d_ops_) nfcs_device_free(ctx_, d_ops_);
        h_arena_ = h_desc_ = h_patch_ = d_arena_ = d_desc_ = d_patch_ = d_status_ = nullptr;
        h_ops_ = d_ops_ = nullptr;
        arena_cap_ = pkt_cap_ = 0;
    }
    int reserve(size_t arena_bytes, size_t n) {
        if (arena_bytes <= arena_cap_ && n <= pkt_cap_) return NFCS_OK;
        release();
        arena_cap_ = arena_bytes < (1u << 20) ? (1u << 20) : arena_bytes;
        pkt_cap_ = n < 4096 ? 4096 : n;
        int rc = NFCS_OK;
        if (!rc) rc = nfcs_host_alloc(ctx_, arena_cap_, &h_arena_);
        if (!rc) rc = nfcs_host_alloc(ctx_, pkt_cap_ * sizeof(nfcs_desc), &h_desc_);
        if (!rc) rc = nfcs_host_alloc(ctx_, pkt_cap_ * sizeof(nfcs_patch), &h_patch_);
        if (!rc) rc = nfcs_device_alloc(ctx_, arena_cap_, &d_arena_);
        if (!rc) rc = nfcs_device_alloc(ctx_, pkt_cap_ * sizeof(nfcs_desc), &d_desc_);
        if (!rc) rc = nfcs_device_alloc(ctx_, pkt_cap_ * sizeof(nfcs_patch), &d_patch_);
        if (!rc) rc = nfcs_device_alloc(ctx_, pkt_cap_, &d_status_);
        if (!rc) rc = nfcs_host_alloc(ctx_, pkt_cap_ * 2 * sizeof(uint32_t), &h_ops_);  // ops, caps
        if (!rc) rc = nfcs_device_alloc(ctx_, pkt_cap_ * 2 * sizeof(uint32_t), &d_ops_);
        if (rc) release();
        return rc;
    }

    nfcs_ctx* ctx_ = nullptr;
    std::mutex mu_;
    void *h_arena_ = nullptr, *h_desc_ = nullptr, *h_patch_ = nullptr;
    void *d_arena_ = nullptr, *d_desc_ = nullptr, *d_patch_ = nullptr, *d_status_ = nullptr;
    void *h_ops_ = nullptr, *d_ops_ = nullptr;
    size_t arena_cap_ = 0, pkt_cap_ = 0;
    std::vector<uint8_t*> frames_;  // update_checksums_batch's frame pointers and lengths
    std::vector<uint32_t> lens_;
};

// Same interface as netflow::Packet for what the checksum path touches.
class Packet {
public:
    explicit Packet(PacketBuffer* buf) : buffer_(buf) {
        if (!buffer_) throw std::invalid_argument("PacketBuffer cannot be null.");
        buffer_->increment_ref();
    }
    ~Packet() {
        if (buffer_) buffer_->decrement_ref();
    }
    Packet(const Packet&) = delete;
    Packet& operator=(const Packet&) = delete;
    Packet(Packet&& o) noexcept : buffer_(o.buffer_) { o.buffer_ = nullptr; }
    Packet& operator=(Packet&& o) noexcept {
        if (this != &o) {
            if (buffer_) buffer_->decrement_ref();
            buffer_ = o.buffer_;
            o.buffer_ = nullptr;
        }
        return *this;
    }

    PacketBuffer* get_buffer() const { return buffer_; }

    // packet.hpp:655 / 694 on one packet, on the host CPU (cpu_update.hpp), each ending with
    // update_checksums() like the reference; returns what the reference returns, never throws.
    // Bursts: vlan_batch (GPU).
    bool push_vlan(uint16_t vlan_id_val, uint8_t priority = 0) noexcept {
        if (!buffer_) return false;
        size_t len = buffer_->get_data_length();
        const size_t room = buffer_->get_capacity() - buffer_->get_headroom();
        if (!cpu::push_vlan(buffer_->get_data_start_ptr(), &len, room, vlan_id_val, priority)) return false;
        return buffer_->set_data_len(len);
    }
    bool pop_vlan() noexcept {
        if (!buffer_) return false;
        size_t len = buffer_->get_data_length();
        if (!cpu::pop_vlan(buffer_->get_data_start_ptr(), &len)) return false;
        return buffer_->set_data_len(len);
    }

    // packet.hpp:722 on one packet, on the host CPU (cpu_update.hpp): void, never throws, like
    // the reference. A single packet would only pay a PCIe round trip on the GPU; bursts go to
    // update_checksums_batch (GPU).
    void update_checksums() noexcept {
        if (buffer_) cpu::update_checksums(buffer_->get_data_start_ptr(), buffer_->get_data_length());
    }

private:
    PacketBuffer* buffer_;
};

template <class Pkt>
int ChecksumEngine::update_checksums_batch(Pkt* const* pkts, size_t n, uint8_t* status) {
    if (n == 0) return NFCS_OK;
    if (!pkts || n > 0xFFFFFFFFu) return NFCS_EINVAL;
    std::lock_guard<std::mutex> lock(mu_);
    // each packet's data window as the C ABI's (pointer, length) pair: nfcs_update_host_frames
    // gathers the frames chunk by chunk into the context's pinned ring, checksums them on the GPU and
    // writes the 2+2 checksum bytes back into each PacketBuffer in place, the chunks' gather,
    // transfers, kernel and write-back overlapped (round 5; before, one gather of the whole burst,
    // then the transfers, then one scatter, one after the other)
    frames_.resize(n);
    lens_.resize(n);
    // a data window longer than NFCS_FRAME_RELEVANT_BYTES goes as its first NFCS_FRAME_RELEVANT_BYTES
    // bytes: update_checksums() gives the same result (nfcs.h), so no PacketBuffer size is refused
    detail::parallel_ranges(n, [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            auto* b = pkts[i] ? pkts[i]->get_buffer() : nullptr;
            const size_t len = b ? b->get_data_length() : 0;
            frames_[i] = b ? b->get_data_start_ptr() : nullptr;
            lens_[i] = static_cast<uint32_t>(std::min<size_t>(len, NFCS_FRAME_RELEVANT_BYTES));
        }
    });
    return nfcs_update_host_frames(ctx_, frames_.data(), lens_.data(), static_cast<uint32_t>(n), status, 0);
}

template <class Pkt>
int ChecksumEngine::vlan_batch(Pkt* const* pkts, const uint32_t* ops, size_t n, bool* ok,
                               uint8_t* status) {
    if (n == 0) return NFCS_OK;
    if (!pkts || !ops || n > 0xFFFFFFFFu) return NFCS_EINVAL;
    std::lock_guard<std::mutex> lock(mu_);
    // gather: each frame in a slot of round_up(len + 4, 16) bytes (room for a pushed tag)
    auto slot = [](size_t len) { return (len + 4 + 15) & ~size_t(15); };
    size_t bytes = 0;
    for (size_t i = 0; i < n; ++i) {
        auto* b = pkts[i] ? pkts[i]->get_buffer() : nullptr;
        bytes += slot(b ? b->get_data_length() : 0);
    }
    if (bytes / 16 > 0xFFFFFFFFu) return NFCS_EINVAL;
    int rc = reserve(bytes + 16, n);
    if (rc) return rc;
    uint8_t* arena = static_cast<uint8_t*>(h_arena_);
    nfcs_desc* desc = static_cast<nfcs_desc*>(h_desc_);
    uint32_t* hops = static_cast<uint32_t*>(h_ops_);
    uint32_t* hcaps = hops + pkt_cap_;
    size_t off = 0;
    for (size_t i = 0; i < n; ++i) {
        auto* b = pkts[i] ? pkts[i]->get_buffer() : nullptr;
        const size_t len = b ? b->get_data_length() : 0;
        if (len) std::memcpy(arena + off, b->get_data_start_ptr(), len);
        // bytes past the frame: the buffer's own bytes where it has them (a re-tag of a runt
        // writes bytes 14-15 past len, a pop leaves its last 4 bytes), zeros otherwise
        const size_t have = b ? b->get_capacity() - b->get_headroom() : 0;
        const size_t tail = slot(len) - len, keep = have > len ? (have - len < tail ? have - len : tail) : 0;
        if (keep) std::memcpy(arena + off + len, b->get_data_start_ptr() + len, keep);
        std::memset(arena + off + len + keep, 0, tail - keep);
        desc[i] = nfcs_desc{static_cast<uint32_t>(off >> 4), static_cast<uint32_t>(len)};
        hops[i] = b ? ops[i] : NFCS_VLAN_NOP;
        hcaps[i] = static_cast<uint32_t>(have < 0xFFFFFFFFu ? have : 0xFFFFFFFFu);
        off += slot(len);
    }
    const uint32_t m = static_cast<uint32_t>(n);
    uint32_t* dops = static_cast<uint32_t*>(d_ops_);
    if ((rc = nfcs_memcpy_h2d(ctx_, d_arena_, arena, off))) return rc;
    if ((rc = nfcs_memcpy_h2d(ctx_, d_desc_, desc, n * sizeof(nfcs_desc)))) return rc;
    if ((rc = nfcs_memcpy_h2d(ctx_, dops, hops, n * sizeof(uint32_t)))) return rc;
    if ((rc = nfcs_memcpy_h2d(ctx_, dops + pkt_cap_, hcaps, n * sizeof(uint32_t)))) return rc;
    if ((rc = nfcs_vlan_device(ctx_, static_cast<uint8_t*>(d_arena_), off,
                               static_cast<nfcs_desc*>(d_desc_), m, dops, 0, dops + pkt_cap_, 0,
                               static_cast<uint8_t*>(d_status_), nullptr)))
        return rc;
    if ((rc = nfcs_memcpy_d2h(ctx_, arena, d_arena_, off))) return rc;
    std::vector<nfcs_desc> nd(n);
    if ((rc = nfcs_memcpy_d2h(ctx_, nd.data(), d_desc_, n * sizeof(nfcs_desc)))) return rc;
    std::vector<uint8_t> st(n);
    if ((rc = nfcs_memcpy_d2h(ctx_, st.data(), d_status_, n))) return rc;
    // scatter: the edited window back into each PacketBuffer and its new data length
    for (size_t i = 0; i < n; ++i) {
        auto* b = pkts[i] ? pkts[i]->get_buffer() : nullptr;
        const bool done = (st[i] & NFCS_ST_FLAG_VLAN) != 0;
        if (ok) ok[i] = done;
        if (status) status[i] = st[i];
        if (!b || !done) continue;
        const size_t len = desc[i].len, nlen = nd[i].len;
        const size_t have = b->get_capacity() - b->get_headroom();
        size_t w = len > nlen ? len : nlen;
        if (w < 16 && have >= 16) w = 16;  // re-tag of a runt: TCI bytes 14-15
        std::memcpy(b->get_data_start_ptr(), arena + (size_t)desc[i].off16 * 16, w < have ? w : have);
        b->set_data_len(nlen);
    }
    return NFCS_OK;
}

template <class Pkt>
size_t ChecksumEngine::gather(Pkt* const* pkts, size_t n, size_t limit) {
    uint8_t* arena = static_cast<uint8_t*>(h_arena_);
    nfcs_desc* desc = static_cast<nfcs_desc*>(h_desc_);
    size_t off = 0;
    for (size_t i = 0; i < n; ++i) {  // layout first
        auto* b = pkts[i] ? pkts[i]->get_buffer() : nullptr;
        size_t len = b ? b->get_data_length() : 0;
        if (limit && len > limit) len = limit;
        desc[i] = nfcs_desc{static_cast<uint32_t>(off >> 4), static_cast<uint32_t>(len)};
        off += (len + 15) & ~size_t(15);
    }
    // then the copies, by up to 8 host threads over disjoint packet ranges (one thread copies
    // ~10 GB/s, well under the PCIe rate the batch then moves at)
    auto copy = [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            const size_t len = desc[i].len, o = (size_t)desc[i].off16 * 16;
            if (len) std::memcpy(arena + o, pkts[i]->get_buffer()->get_data_start_ptr(), len);
            std::memset(arena + o + len, 0, ((len + 15) & ~size_t(15)) - len);
        }
    };
    const size_t nt = off >= (size_t(32) << 20) ? 8 : 1;
    if (nt == 1) {
        copy(0, n);
    } else {
        std::vector<std::thread> th;
        th.reserve(nt);
        for (size_t t = 0; t < nt; ++t) {
            try {
                th.emplace_back(copy, n * t / nt, n * (t + 1) / nt);
            } catch (...) {  // no thread to be had: copy that range here (never throw)
                copy(n * t / nt, n * (t + 1) / nt);
            }
        }
        for (auto& t : th) t.join();
    }
    return off;
}

template <class Pkt>
int ChecksumEngine::l3_forward_batch(Pkt* const* pkts, const uint32_t* next_hop, size_t n,
                                     const nfcs_nexthop* table, uint32_t table_n, uint8_t* status) {
    if (n == 0) return NFCS_OK;
    if (!pkts || !next_hop || (table_n && !table) || n > 0xFFFFFFFFu) return NFCS_EINVAL;
    std::lock_guard<std::mutex> lock(mu_);
    size_t bytes = 0;
    for (size_t i = 0; i < n; ++i) {
        auto* b = pkts[i] ? pkts[i]->get_buffer() : nullptr;
        bytes += ((b ? b->get_data_length() : 0) + 15) & ~size_t(15);
    }
    if (bytes / 16 > 0xFFFFFFFFu) return NFCS_EINVAL;
    int rc = reserve(bytes + 16, n);
    if (rc) return rc;
    const size_t off = gather(pkts, n, 0);
    uint8_t* arena = static_cast<uint8_t*>(h_arena_);
    const nfcs_desc* desc = static_cast<const nfcs_desc*>(h_desc_);
    uint32_t* hnh = static_cast<uint32_t*>(h_ops_);
    for (size_t i = 0; i < n; ++i) hnh[i] = next_hop[i];
    DevTmp dtab(ctx_, table_n * sizeof(nfcs_nexthop), rc);
    if (rc) return rc;
    const uint32_t m = static_cast<uint32_t>(n);
    if ((rc = nfcs_memcpy_h2d(ctx_, d_arena_, arena, off ? off : 16))) return rc;
    if ((rc = nfcs_memcpy_h2d(ctx_, d_desc_, desc, n * sizeof(nfcs_desc)))) return rc;
    if ((rc = nfcs_memcpy_h2d(ctx_, d_ops_, hnh, n * sizeof(uint32_t)))) return rc;
    if (table_n && (rc = nfcs_memcpy_h2d(ctx_, dtab.p, table, table_n * sizeof(nfcs_nexthop)))) return rc;
    if ((rc = nfcs_l3_forward_device(ctx_, static_cast<uint8_t*>(d_arena_), off ? off : 16,
                                     static_cast<nfcs_desc*>(d_desc_), static_cast<uint32_t*>(d_ops_),
                                     m, static_cast<nfcs_nexthop*>(dtab.p), table_n,
                                     static_cast<uint8_t*>(d_status_), nullptr)))
        return rc;
    if ((rc = nfcs_memcpy_d2h(ctx_, arena, d_arena_, off ? off : 16))) return rc;
    std::vector<uint8_t> st(n);
    if ((rc = nfcs_memcpy_d2h(ctx_, st.data(), d_status_, n))) return rc;
    // scatter: every byte the forward writes lies below byte 128 (MACs, TTL, the IPv4 checksum,
    // the L4 checksum at most at l2 18 + IHL 60 + 16)
    for (size_t i = 0; i < n; ++i) {
        if (status) status[i] = st[i];
        auto* b = pkts[i] ? pkts[i]->get_buffer() : nullptr;
        if (!b || !(st[i] & NFCS_ST_FLAG_FWD)) continue;
        const size_t len = desc[i].len, w = len < 128 ? len : 128;
        std::memcpy(b->get_data_start_ptr(), arena + (size_t)desc[i].off16 * 16, w);
    }
    return NFCS_OK;
}

template <class Pkt>
int ChecksumEngine::flow_keys_batch(Pkt* const* pkts, size_t n, nfcs_flow_key* keys, uint32_t* hashes) {
    if (n == 0) return NFCS_OK;
    if (!pkts || n > 0xFFFFFFFFu) return NFCS_EINVAL;
    std::lock_guard<std::mutex> lock(mu_);
    // every field the key reads lies below byte 98 (l2 18 + IHL 60 + the 19-byte TcpHeader's
    // bounds check), so the first 128 bytes with len clamped to 128 give the same key
    int rc = reserve(n * 128 + 16, n);
    if (rc) return rc;
    const size_t off = gather(pkts, n, 128);
    DevTmp dkeys(ctx_, n * sizeof(nfcs_flow_key), rc);
    DevTmp dhash(ctx_, n * sizeof(uint32_t), rc);
    if (rc) return rc;
    const uint32_t m = static_cast<uint32_t>(n);
    if ((rc = nfcs_memcpy_h2d(ctx_, d_arena_, h_arena_, off ? off : 16))) return rc;
    if ((rc = nfcs_memcpy_h2d(ctx_, d_desc_, h_desc_, n * sizeof(nfcs_desc)))) return rc;
    if ((rc = nfcs_flow_keys_device(ctx_, static_cast<uint8_t*>(d_arena_), off ? off : 16,
                                    static_cast<nfcs_desc*>(d_desc_), m,
                                    static_cast<nfcs_flow_key*>(dkeys.p),
                                    static_cast<uint32_t*>(dhash.p), nullptr)))
        return rc;
    if (keys && (rc = nfcs_memcpy_d2h(ctx_, keys, dkeys.p, n * sizeof(nfcs_flow_key)))) return rc;
    if (hashes && (rc = nfcs_memcpy_d2h(ctx_, hashes, dhash.p, n * sizeof(uint32_t)))) return rc;
    return NFCS_OK;
}

// Same interface as netflow::BufferPool (buffer_pool.hpp:57-123: allocate_buffer(payload,
// headroom), free_buffer(buffer) with the PacketBuffer reference count), except that every
// buffer up to slot_bytes is a slot of ONE pinned arena (nfcs_host_alloc). update_checksums_batch
// builds the descriptors straight from the slots: frames that fill most of their slots go as spans
// DMA'd from the pinned arena (nfcs_update_host, patch records back; or, with NFCS_HOST_ZERO_COPY,
// read by the kernel over PCIe in place); frames that fill less than 85% of them are gathered by the
// library's copy threads first (nfcs_update_host_frames), so the slots' unused bytes do not cross PCIe.
// Buffers larger than a slot are heap PacketBuffers, as the reference allocates them.
// The default slot is 2176 bytes (a 2048-byte data room + 128 bytes of headroom, DPDK's mbuf
// layout): power-of-two slots alias on MI355X — C1's frames in 2048-byte slots checksum at 0.716 of
// 8 TB/s (read pass 232 µs, write pass 41.7 µs) against 0.781 in 2176-byte slots (222 / 28.5 µs;
// round 3, profiles/r03_stride_*.json).
class BufferPool {
public:
    explicit BufferPool(size_t slots = 65536, size_t slot_bytes = 2176,
                        ChecksumEngine& engine = ChecksumEngine::instance())
        : eng_(engine), slots_(slots), slot_bytes_((slot_bytes + 15) & ~size_t(15)) {
        if (slots_ == 0 || slots_ * slot_bytes_ / 16 > 0xFFFFFFFFull)
            throw std::invalid_argument("BufferPool: slots x slot_bytes must address < 64 GiB");
        void* p = nullptr;
        const int rc = nfcs_host_alloc(eng_.ctx(), slots_ * slot_bytes_, &p);
        if (rc != NFCS_OK) throw std::bad_alloc();
        arena_ = static_cast<unsigned char*>(p);
        bufs_.reserve(slots_);
        free_.reserve(slots_);
        for (size_t i = 0; i < slots_; ++i) {
            bufs_.emplace_back(new PacketBuffer(PacketBuffer::External{}, arena_ + i * slot_bytes_, slot_bytes_));
            free_.push_back(static_cast<uint32_t>(slots_ - 1 - i));  // allocate in arena order
        }
    }
    ~BufferPool() {
        std::lock_guard<std::mutex> lock(mu_);
        for (PacketBuffer* b : heap_free_) delete b;
        bufs_.clear();
        nfcs_host_free(eng_.ctx(), arena_);
    }
    BufferPool(const BufferPool&) = delete;
    BufferPool& operator=(const BufferPool&) = delete;

    // buffer_pool.hpp:66-103: data length 0, the given headroom, reference count 1.
    PacketBuffer* allocate_buffer(size_t required_data_payload_size, size_t required_headroom = 32) {
        std::lock_guard<std::mutex> lock(mu_);
        const size_t need = required_data_payload_size + required_headroom;
        if (need <= slot_bytes_ && !free_.empty()) {
            PacketBuffer* b = bufs_[free_.back()].get();
            free_.pop_back();
            b->ref_count.store(1, std::memory_order_relaxed);
            b->reset_offsets_and_len(required_headroom, 0);
            return b;
        }
        for (auto it = heap_free_.begin(); it != heap_free_.end(); ++it) {
            if ((*it)->get_capacity() >= need) {
                PacketBuffer* b = *it;
                heap_free_.erase(it);
                b->ref_count.store(1, std::memory_order_relaxed);
                b->reset_offsets_and_len(required_headroom, 0);
                return b;
            }
        }
        return new PacketBuffer(need, required_headroom, 0);
    }

    // buffer_pool.hpp:106-123: back to the pool when the last reference is released.
    void free_buffer(PacketBuffer* buffer) {
        if (!buffer || !buffer->decrement_ref()) return;
        std::lock_guard<std::mutex> lock(mu_);
        if (in_arena(buffer)) free_.push_back(slot_of(buffer));
        else heap_free_.push_back(buffer);
    }

    bool in_arena(const PacketBuffer* b) const {
        return b && b->storage() >= arena_ && b->storage() < arena_ + slots_ * slot_bytes_;
    }
    size_t available() {
        std::lock_guard<std::mutex> lock(mu_);
        return free_.size();
    }
    unsigned char* arena() const { return arena_; }

    // Batched Packet::update_checksums() on packets whose buffers are pool slots with 16-byte
    // aligned data starts (the default headroom of 32 keeps them aligned): no gather or scatter
    // copies. Other packets make the call fall back to ChecksumEngine::update_checksums_batch.
    // flags: 0 (frames DMA'd from the pinned arena) or NFCS_HOST_ZERO_COPY.
    int update_checksums_batch(Packet* const* pkts, size_t n, uint8_t* status = nullptr,
                               uint32_t flags = 0);

private:
    uint32_t slot_of(const PacketBuffer* b) const {
        return static_cast<uint32_t>((b->storage() - arena_) / slot_bytes_);
    }

    ChecksumEngine& eng_;
    size_t slots_, slot_bytes_;
    unsigned char* arena_ = nullptr;
    std::vector<std::unique_ptr<PacketBuffer>> bufs_;
    std::vector<uint32_t> free_;
    std::vector<PacketBuffer*> heap_free_;
    std::mutex mu_;
};

inline int BufferPool::update_checksums_batch(Packet* const* pkts, size_t n, uint8_t* status,
                                              uint32_t flags) {
    if (n == 0) return NFCS_OK;
    if (!pkts || n > 0xFFFFFFFFu) return NFCS_EINVAL;
    std::vector<nfcs_desc> desc(n);
    std::atomic<bool> foreign{false};  // a packet whose buffer is not a 16-byte aligned slot of the pool
    detail::parallel_ranges(n, [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            PacketBuffer* b = pkts[i] ? pkts[i]->get_buffer() : nullptr;
            const unsigned char* d = b ? b->get_data_start_ptr() : nullptr;
            if (!b || !in_arena(b) || ((d - arena_) & 15)) {
                foreign.store(true, std::memory_order_relaxed);
                break;
            }
            desc[i] = nfcs_desc{static_cast<uint32_t>((d - arena_) >> 4), static_cast<uint32_t>(b->get_data_length())};
        }
    });
    if (foreign.load()) return eng_.update_checksums_batch(pkts, n, status);
    size_t drops = 0;  // places where the burst's arena offsets go down (a wrap of the pool's slots)
    uint64_t frame_bytes = 0, span = 0, lo = 0, hi = 0;  // span: the runs' bytes, as nfcs_update_host stages them
    for (size_t i = 0; i < n; ++i) {
        const uint64_t o = (uint64_t)desc[i].off16 * 16, e = o + ((desc[i].len + 15u) & ~15u);
        if (i && desc[i].off16 < desc[i - 1].off16) {
            ++drops;
            span += hi - lo;
            lo = hi = o;
        } else if (i == 0) {
            lo = hi = o;
        }
        hi = std::max(hi, e);
        frame_bytes += desc[i].len;
    }
    span += hi - lo;
    // Frames that fill less than 85% of their slots: DMA'd as spans, the slots' unused bytes would
    // cross PCIe too (C1's 1500-byte frames in 2176-byte slots: 33 GB/s of frames); gathered by the
    // library's copy threads first, only frame bytes do (49 GB/s; round 5, profiles/r05_b_adapter_t8.json).
    // A burst spanning at most NFCS_HOST_ZERO_COPY_AUTO_BYTES runs zero-copy in nfcs_update_host, where the
    // kernel reads only the frames' bytes in place: no gather then (round 6). NFCS_HOST_ZERO_COPY stays a
    // span read in place.
    if (flags == 0 && frame_bytes < n * slot_bytes_ * 85 / 100 && span > NFCS_HOST_ZERO_COPY_AUTO_BYTES) {
        std::vector<uint8_t*> fr(n);
        std::vector<uint32_t> ln(n);
        for (size_t i = 0; i < n; ++i) {
            fr[i] = arena_ + (size_t)desc[i].off16 * 16;
            ln[i] = desc[i].len;
        }
        return eng_.update_host_frames(fr.data(), ln.data(), static_cast<uint32_t>(n), status);
    }
    // nfcs_update_host stages each run of ascending offsets as one span: a burst in allocation order
    // (the pool hands slots out in arena order) or wrapping once goes as it is; a burst in an order
    // the pool's reuse has scrambled is sorted first, so its spans stay long. A wrap is one drop whose
    // second run ends at or before the first run's first frame ([100..199, 0, 9000] also
    // has one drop, but staged as is its second span would carry every slot from 0 to 9000)
    const bool wrap = drops == 1 && (uint64_t)desc[n - 1].off16 * 16 + desc[n - 1].len <= (uint64_t)desc[0].off16 * 16;
    if (drops == 0 || wrap) {
        return eng_.update_host(arena_, slots_ * slot_bytes_, desc.data(), static_cast<uint32_t>(n), status, flags);
    }
    std::vector<uint32_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = static_cast<uint32_t>(i);
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return desc[a].off16 < desc[b].off16; });
    std::vector<nfcs_desc> sorted(n);
    for (size_t j = 0; j < n; ++j) sorted[j] = desc[order[j]];
    std::vector<uint8_t> st(status ? n : 0);
    const int rc = eng_.update_host(arena_, slots_ * slot_bytes_, sorted.data(), static_cast<uint32_t>(n),
                                    status ? st.data() : nullptr, flags);
    if (rc) return rc;
    if (status)
        for (size_t j = 0; j < n; ++j) status[order[j]] = st[j];
    return NFCS_OK;
}

// Free-function forms on the process-wide engine: they return NFCS_ENODEV (or the error
// nfcs_ctx_create reported) instead of throwing when no gfx950 engine exists.
namespace detail {
template <class F>
int on_default_engine(F&& f) noexcept {
    int rc = NFCS_OK;
    ChecksumEngine* e = ChecksumEngine::try_instance(&rc);
    if (!e) return rc ? rc : NFCS_ENODEV;
    try {
        return f(*e);
    } catch (...) {  // std::bad_alloc from the host-side gather: the reference's only escape too
        return NFCS_ENOMEM;
    }
}
}  // namespace detail

inline int update_checksums_batch(Packet* const* pkts, size_t n, uint8_t* status = nullptr) {
    return detail::on_default_engine([&](ChecksumEngine& e) { return e.update_checksums_batch(pkts, n, status); });
}
inline int update_checksums_batch(const std::vector<Packet*>& pkts, uint8_t* status = nullptr) {
    return update_checksums_batch(pkts.data(), pkts.size(), status);
}
inline int vlan_batch(Packet* const* pkts, const uint32_t* ops, size_t n, bool* ok = nullptr,
                      uint8_t* status = nullptr) {
    return detail::on_default_engine([&](ChecksumEngine& e) { return e.vlan_batch(pkts, ops, n, ok, status); });
}
inline int l3_forward_batch(Packet* const* pkts, const uint32_t* next_hop, size_t n,
                            const nfcs_nexthop* table, uint32_t table_n, uint8_t* status = nullptr) {
    return detail::on_default_engine(
        [&](ChecksumEngine& e) { return e.l3_forward_batch(pkts, next_hop, n, table, table_n, status); });
}
inline int flow_keys_batch(Packet* const* pkts, size_t n, nfcs_flow_key* keys,
                           uint32_t* hashes = nullptr) {
    return detail::on_default_engine([&](ChecksumEngine& e) { return e.flow_keys_batch(pkts, n, keys, hashes); });
}

}  // namespace netflow_amd
