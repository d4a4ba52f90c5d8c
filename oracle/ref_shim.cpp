// ref_shim.cpp — TEST INFRASTRUCTURE ONLY.
//
// Exposes the REFERENCE implementation of the checksum path through a C ABI so that tests
// and the golden-fixture script can run it. The reference source is NOT copied: this file
// is compiled against /root/reference/include by oracle/Makefile (target `ref`), and the
// result goes to oracle/_ref/libnfref.so (git-ignored). The path is header-only
// (include/netflow++/packet.hpp + packet_buffer.hpp) and needs nothing but libc/libstdc++.
//
// Calls netflow::Packet::update_checksums() (packet.hpp:722-890) on a PacketBuffer
// (packet_buffer.hpp:10-111) whose data window is pointed at the caller's frame, so the
// reference mutates the caller's bytes in place exactly as it would its own buffer.
#include <netflow++/packet.hpp>
#include <netflow++/packet_classifier.hpp>

#include <pthread.h>
#include <sched.h>

#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct Window {
    netflow::PacketBuffer pb;
    unsigned char* own;
    Window() : pb(16, 0, 0), own(pb.raw_data_ptr_) {}
    ~Window() { pb.raw_data_ptr_ = own; }  // the PacketBuffer dtor deletes its own bytes
    void point(uint8_t* frame, size_t len) {
        pb.raw_data_ptr_ = frame;
        pb.capacity_ = len;
        pb.data_offset_ = 0;
        pb.data_len_ = len;
    }
};

struct Desc { uint32_t off16; uint32_t len; };

}  // namespace

extern "C" {

// One frame, in place. The caller guarantees the frame is in the reference's defined
// domain (an IPv4 header whose IHL*4 reaches past len makes the reference read past it).
__attribute__((visibility("default"))) void nfref_update(uint8_t* frame, size_t len) {
    Window w;
    w.point(frame, len);
    netflow::Packet pkt(&w.pb);  // increments the refcount like every reference caller
    pkt.update_checksums();
}

// Batch over an arena: one Packet per frame on `nthreads` std::threads (contiguous static
// slices). This is the reference's own per-packet code path and cost structure (per-call
// std::vector pseudo-header+segment copy, scalar ntohs fold), used as the CPU baseline.
__attribute__((visibility("default"))) void nfref_update_batch(uint8_t* arena, const void* desc_v,
                                                               uint32_t n, int nthreads) {
    const Desc* desc = static_cast<const Desc*>(desc_v);
    if (nthreads < 1) nthreads = 1;
    auto work = [&](uint32_t lo, uint32_t hi) {
        Window w;
        for (uint32_t i = lo; i < hi; ++i) {
            w.point(arena + (uint64_t)desc[i].off16 * 16, desc[i].len);
            netflow::Packet pkt(&w.pb);
            pkt.update_checksums();
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t)
        th.emplace_back(work, (uint32_t)((uint64_t)n * t / nthreads),
                        (uint32_t)((uint64_t)n * (t + 1) / nthreads));
    work(0, (uint32_t)((uint64_t)n / nthreads));
    for (auto& t : th) t.join();
}

// The same batch with thread t pinned to cpus[t % ncpus] (the bench's CPU baseline: every allotted
// host CPU, the list interleaved across NUMA nodes by the caller).
__attribute__((visibility("default"))) void nfref_update_batch_on(uint8_t* arena, const void* desc_v,
                                                                  uint32_t n, int nthreads,
                                                                  const int* cpus, int ncpus) {
    const Desc* desc = static_cast<const Desc*>(desc_v);
    if (nthreads < 1) nthreads = 1;
    auto work = [&](int t) {
        if (cpus && ncpus > 0) {
            cpu_set_t set;
            CPU_ZERO(&set);
            CPU_SET(cpus[t % ncpus], &set);
            (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
        }
        const uint32_t lo = (uint32_t)((uint64_t)n * t / nthreads), hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        Window w;
        for (uint32_t i = lo; i < hi; ++i) {
            w.point(arena + (uint64_t)desc[i].off16 * 16, desc[i].len);
            netflow::Packet pkt(&w.pb);
            pkt.update_checksums();
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
    cpu_set_t saved;
    const bool restore = pthread_getaffinity_np(pthread_self(), sizeof(saved), &saved) == 0;
    work(0);
    if (restore) (void)pthread_setaffinity_np(pthread_self(), sizeof(saved), &saved);
    for (auto& t : th) t.join();
}

// The data-path part of Switch::process_received_packet for a transit IPv4 packet
// (switch.hpp:247-294), driven through the reference's own Packet accessors: ethernet(),
// vlan(), ipv4(), the TTL check/decrement, the MAC rewrite and update_checksums(). The
// control-plane lookups are replaced by nh (12 bytes {dst, src}, or NULL for no route / ARP
// miss). Returns 1 if forwarded, 0 if the switch would have dropped or diverted the packet
// (untouched, as the caller sees it here).
__attribute__((visibility("default"))) int nfref_l3_forward(uint8_t* frame, size_t len,
                                                            const uint8_t* nh) {
    Window w;
    w.point(frame, len);
    netflow::Packet pkt(&w.pb);
    netflow::EthernetHeader* eth_hdr = pkt.ethernet();
    uint16_t l2_type = eth_hdr ? ntohs(eth_hdr->ethertype) : 0;
    uint16_t l3_type = l2_type;
    if (l2_type == netflow::ETHERTYPE_VLAN) {
        netflow::VlanHeader* vlan_hdr = pkt.vlan();
        if (vlan_hdr) l3_type = ntohs(vlan_hdr->ethertype);
    }
    if (l3_type != netflow::ETHERTYPE_IPV4) return 0;
    netflow::IPv4Header* ip_hdr = pkt.ipv4();
    if (!ip_hdr) return 0;
    if (ip_hdr->ttl <= 1) return 0;
    if (!nh) return 0;
    ip_hdr->ttl--;
    eth_hdr->dst_mac = netflow::MacAddress(nh);
    eth_hdr->src_mac = netflow::MacAddress(nh + 6);
    pkt.update_checksums();
    return 1;
}

// Batch of the above over an arena (next hop i = table[nh[i]], none if >= table_n) on
// `nthreads` std::threads: the CPU baseline of the fused forward.
__attribute__((visibility("default"))) void nfref_l3_forward_batch(uint8_t* arena, const void* desc_v,
                                                                   const uint32_t* nh, uint32_t n,
                                                                   const uint8_t* table,
                                                                   uint32_t table_n, int nthreads) {
    const Desc* desc = static_cast<const Desc*>(desc_v);
    if (nthreads < 1) nthreads = 1;
    auto work = [&](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i)
            nfref_l3_forward(arena + (uint64_t)desc[i].off16 * 16, desc[i].len,
                             nh[i] < table_n ? table + (size_t)nh[i] * 12 : nullptr);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t)
        th.emplace_back(work, (uint32_t)((uint64_t)n * t / nthreads),
                        (uint32_t)((uint64_t)n * (t + 1) / nthreads));
    work(0, (uint32_t)((uint64_t)n / nthreads));
    for (auto& t : th) t.join();
}

// PacketClassifier::extract_flow_key + hash_flow (src/netflow++/packet_classifier.cpp:12-108,
// compiled from the reference source by oracle/Makefile), serialised into the 64-byte record
// of include/nfcs.h (nfcs_flow_key). Returns the hash.
static void put16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
static void put32(uint8_t* p, uint32_t v) { for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i)); }

__attribute__((visibility("default"))) uint32_t nfref_flow_key(uint8_t* frame, size_t len,
                                                               uint8_t* rec /* 64 bytes */) {
    Window w;
    w.point(frame, len);
    netflow::Packet pkt(&w.pb);
    netflow::PacketClassifier pc;
    const netflow::PacketClassifier::FlowKey k = pc.extract_flow_key(pkt);
    const uint32_t h = netflow::PacketClassifier::hash_flow(k);
    std::memset(rec, 0, 64);
    put32(rec + 0, h);
    put16(rec + 4, k.vlan_id);
    put16(rec + 6, k.ethertype);
    std::memcpy(rec + 8, k.src_mac.bytes, 6);
    std::memcpy(rec + 14, k.dst_mac.bytes, 6);
    rec[20] = k.protocol;
    rec[21] = k.is_ipv6 ? 1 : 0;
    put16(rec + 22, k.src_port);
    put16(rec + 24, k.dst_port);
    if (k.is_ipv6) {
        std::memcpy(rec + 32, k.src_ipv6.data(), 16);
        std::memcpy(rec + 48, k.dst_ipv6.data(), 16);
    } else {
        put32(rec + 32, k.src_ip);
        put32(rec + 48, k.dst_ip);
    }
    return h;
}

// Batch of the above on `nthreads` std::threads (records may be NULL): the CPU baseline.
__attribute__((visibility("default"))) void nfref_flow_keys_batch(uint8_t* arena, const void* desc_v,
                                                                  uint32_t n, uint8_t* recs,
                                                                  uint32_t* hashes, int nthreads) {
    const Desc* desc = static_cast<const Desc*>(desc_v);
    if (nthreads < 1) nthreads = 1;
    auto work = [&](uint32_t lo, uint32_t hi) {
        uint8_t tmp[64];
        for (uint32_t i = lo; i < hi; ++i) {
            const uint32_t h = nfref_flow_key(arena + (uint64_t)desc[i].off16 * 16, desc[i].len,
                                              recs ? recs + (size_t)i * 64 : tmp);
            if (hashes) hashes[i] = h;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t)
        th.emplace_back(work, (uint32_t)((uint64_t)n * t / nthreads),
                        (uint32_t)((uint64_t)n * (t + 1) / nthreads));
    work(0, (uint32_t)((uint64_t)n / nthreads));
    for (auto& t : th) t.join();
}

// Packet::push_vlan(vid, prio) / pop_vlan() (packet.hpp:655-720), which end in
// update_checksums(), on a frame whose PacketBuffer has `cap` bytes of capacity and no headroom
// (tailroom = cap - len). op: bits 30-31 = 1 push / 2 pop, bits 13-15 priority, 0-11 VLAN id
// (include/nfcs.h NFCS_VLAN_*). *len gets the buffer's new data length. Returns the reference's
// bool (1 / 0), or -1 for no edit.
__attribute__((visibility("default"))) int nfref_vlan(uint8_t* frame, uint32_t* len, uint32_t cap,
                                                      uint32_t op) {
    const uint32_t kind = op >> 30;
    if (kind != 1 && kind != 2) return -1;
    Window w;
    w.point(frame, *len);
    w.pb.capacity_ = cap;
    netflow::Packet pkt(&w.pb);
    const bool ok = kind == 1 ? pkt.push_vlan((uint16_t)(op & 0x0FFF), (uint8_t)((op >> 13) & 7))
                              : pkt.pop_vlan();
    *len = (uint32_t)w.pb.get_data_length();
    return ok ? 1 : 0;
}

// Batch of the above over an arena (desc lengths updated) on `nthreads` std::threads: the CPU
// baseline of the VLAN edit path.
__attribute__((visibility("default"))) void nfref_vlan_batch(uint8_t* arena, void* desc_v,
                                                             const uint32_t* ops, uint32_t n,
                                                             uint32_t cap, int nthreads) {
    Desc* desc = static_cast<Desc*>(desc_v);
    if (nthreads < 1) nthreads = 1;
    auto work = [&](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i)
            nfref_vlan(arena + (uint64_t)desc[i].off16 * 16, &desc[i].len, cap, ops[i]);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t)
        th.emplace_back(work, (uint32_t)((uint64_t)n * t / nthreads),
                        (uint32_t)((uint64_t)n * (t + 1) / nthreads));
    work(0, (uint32_t)((uint64_t)n / nthreads));
    for (auto& t : th) t.join();
}

__attribute__((visibility("default"))) int nfref_struct_sizes(int which) {
    switch (which) {
    case 0: return (int)sizeof(netflow::EthernetHeader);
    case 1: return (int)sizeof(netflow::VlanHeader);
    case 2: return (int)sizeof(netflow::IPv4Header);
    case 3: return (int)sizeof(netflow::IPv6Header);
    case 4: return (int)sizeof(netflow::TcpHeader);
    case 5: return (int)sizeof(netflow::UdpHeader);
    case 6: return (int)sizeof(netflow::IcmpHeader);
    case 7: return (int)offsetof(netflow::TcpHeader, checksum);
    default: return -1;
    }
}

}  // extern "C"
