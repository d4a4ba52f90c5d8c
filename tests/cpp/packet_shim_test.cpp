// packet_shim_test.cpp — drives include/netflow_amd/packet.hpp the way NetFlow++ code drives
// netflow::Packet (tests/packet_test.cpp style), reading frames as hex lines on stdin.
//   cpu     : PacketBuffer / Packet semantics; engine construction must fail loudly w/o GPU
//   batch   : update_checksums_batch over all frames; prints "<status> <hex>" per frame
//   single  : Packet::update_checksums() per frame (host CPU); prints "<hex>" per frame
//   vlan    : lines "<op> <room> <hex>"; vlan_batch over all frames in zero-filled buffers with
//             `room` bytes from the data start; prints "<ok> <status> <new len> <hex of room
//             bytes from the data start>" per frame
//   vlan1   : same through Packet::push_vlan / pop_vlan one packet at a time (host CPU)
//   multi K : the frames packed into one host arena (128-byte slots) and updated by
//             netflow_amd::MultiGpu over K contexts on device 0 (one host thread each); prints
//             "<status> <hex>" per frame, then "bounds b0 b1 ... bK" on stderr
#include <netflow_amd/multi_gpu.hpp>
#include <netflow_amd/packet.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

static std::vector<uint8_t> unhex(const std::string& s) {
    std::vector<uint8_t> v;
    for (size_t i = 0; i + 1 < s.size(); i += 2) v.push_back((uint8_t)std::stoul(s.substr(i, 2), nullptr, 16));
    return v;
}
static std::string hex(const unsigned char* p, size_t n) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) { s += d[p[i] >> 4]; s += d[p[i] & 15]; }
    return s;
}

static int cpu_checks() {
    using namespace netflow_amd;
    int bad = 0;
    PacketBuffer pb(128, 32, 0);
    bad += pb.get_headroom() != 32 || pb.get_tailroom() != 96 || pb.ref_count != 1;
    bad += !pb.set_data_len(96) || pb.set_data_len(97);
    bad += !pb.prepend_data(4) || pb.get_data_length() != 100 || pb.get_headroom() != 28;
    bad += !pb.consume_data_front(4) || !pb.consume_data_end(4) || pb.get_data_length() != 92;
    bad += pb.append_data(5) || !pb.append_data(4) || pb.get_tailroom() != 0 || pb.prepend_data(33);
    bad += pb.consume_data_front(97) || pb.consume_data_end(~size_t(0)) || pb.append_data(~size_t(0));
    bad += !pb.consume_data_end(4) || pb.get_data_length() != 92 || pb.get_headroom() != 32;
    try { pb.reset_offsets_and_len(100, 29); bad += 1; } catch (const std::out_of_range&) {}
    pb.reset_offsets_and_len(100, 28);
    bad += pb.get_headroom() != 100 || pb.get_tailroom() != 0 || pb.get_data_start_ptr() != pb.storage() + 100;
    pb.reset_offsets_and_len(32, 92);
    {
        Packet p(&pb);
        bad += pb.ref_count != 2 || p.get_buffer() != &pb;
        Packet q(std::move(p));
        bad += pb.ref_count != 2 || q.get_buffer() != &pb || p.get_buffer() != nullptr;
    }
    bad += pb.ref_count != 1;
    try { Packet nullp(nullptr); bad += 1; } catch (const std::invalid_argument&) {}
    try { PacketBuffer over(8, 4, 8); bad += 1; } catch (const std::invalid_argument&) {}
    bool threw = false;
    try { ChecksumEngine e(0); } catch (const std::runtime_error&) { threw = true; }
    std::printf("engine_without_gpu_throws=%d\n", threw ? 1 : 0);
    {   // the batch free functions return a code instead (the reference's calls never throw)
        PacketBuffer b(128, 32, 60);
        std::memset(b.get_data_start_ptr(), 0, 60);
        Packet p(&b);
        std::vector<Packet*> v{&p};
        std::printf("batch_rc=%d\n", update_checksums_batch(v));
        uint32_t op = NFCS_VLAN_POP;
        bool ok = true;
        std::printf("vlan_batch_rc=%d\n", vlan_batch(v.data(), &op, 1, &ok));
        // single-packet members: host CPU, no engine needed, no throw
        bad += p.pop_vlan() != false;                       // untagged: the reference returns false
        bad += !p.push_vlan(5, 1) || b.get_data_length() != 64;
        bad += !p.pop_vlan() || b.get_data_length() != 60;
        p.update_checksums();
    }
    std::printf("api_failures=%d\n", bad);
    return bad;
}

static int vlan_mode(bool single) {
    std::vector<std::unique_ptr<netflow_amd::PacketBuffer>> bufs;
    std::vector<std::unique_ptr<netflow_amd::Packet>> pkts;
    std::vector<uint32_t> ops, room;
    std::string line;
    while (std::getline(std::cin, line)) {
        const size_t a = line.find(' '), b = line.find(' ', a + 1);
        ops.push_back((uint32_t)std::stoul(line.substr(0, a)));
        room.push_back((uint32_t)std::stoul(line.substr(a + 1, b - a - 1)));
        std::vector<uint8_t> f = unhex(line.substr(b + 1));
        // headroom 32 as the reference's BufferPool allocates (buffer_pool.hpp:57)
        bufs.emplace_back(new netflow_amd::PacketBuffer(room.back() + 32, 32, f.size()));
        std::memset(bufs.back()->storage(), 0, room.back() + 32);
        if (!f.empty()) std::memcpy(bufs.back()->get_data_start_ptr(), f.data(), f.size());
        pkts.emplace_back(new netflow_amd::Packet(bufs.back().get()));
    }
    const size_t n = pkts.size();
    std::vector<netflow_amd::Packet*> raw;
    for (auto& p : pkts) raw.push_back(p.get());
    std::unique_ptr<bool[]> ok(new bool[n ? n : 1]);
    std::vector<uint8_t> st(n, 0xEE);
    if (!single) {
        int rc = netflow_amd::vlan_batch(raw.data(), ops.data(), n, ok.get(), st.data());
        if (rc) { std::fprintf(stderr, "rc=%d\n", rc); return 2; }
    } else {
        for (size_t i = 0; i < n; ++i) {
            const uint32_t kind = ops[i] & NFCS_VLAN_OP_MASK;
            ok[i] = kind == NFCS_VLAN_PUSH ? raw[i]->push_vlan(ops[i] & 0xFFF, (ops[i] >> 13) & 7)
                  : kind == NFCS_VLAN_POP ? raw[i]->pop_vlan() : false;
        }
    }
    for (size_t i = 0; i < n; ++i) {
        auto* b = raw[i]->get_buffer();
        std::printf("%d %d %zu %s\n", ok[i] ? 1 : 0, (int)st[i], b->get_data_length(),
                    hex(b->get_data_start_ptr(), room[i]).c_str());
    }
    return 0;
}

// Input: first line = the next-hop table (hex, 12 bytes per entry), then "nh hexframe" lines.
// Output per packet: "status hex(frame)".
static int l3_mode() {
    std::string line;
    if (!std::getline(std::cin, line)) return 2;
    const std::vector<uint8_t> t = unhex(line);
    std::vector<nfcs_nexthop> table(t.size() / sizeof(nfcs_nexthop));
    if (!table.empty()) std::memcpy(table.data(), t.data(), table.size() * sizeof(nfcs_nexthop));
    std::vector<std::unique_ptr<netflow_amd::PacketBuffer>> bufs;
    std::vector<std::unique_ptr<netflow_amd::Packet>> pkts;
    std::vector<uint32_t> nh;
    while (std::getline(std::cin, line)) {
        const size_t a = line.find(' ');
        nh.push_back((uint32_t)std::stoul(line.substr(0, a)));
        std::vector<uint8_t> f = unhex(line.substr(a + 1));
        bufs.emplace_back(new netflow_amd::PacketBuffer(f.size() + 96, 32, f.size()));
        if (!f.empty()) std::memcpy(bufs.back()->get_data_start_ptr(), f.data(), f.size());
        pkts.emplace_back(new netflow_amd::Packet(bufs.back().get()));
    }
    std::vector<netflow_amd::Packet*> raw;
    for (auto& p : pkts) raw.push_back(p.get());
    std::vector<uint8_t> st(raw.size(), 0xEE);
    int rc = netflow_amd::l3_forward_batch(raw.data(), nh.data(), raw.size(), table.data(),
                                           (uint32_t)table.size(), st.data());
    if (rc) { std::fprintf(stderr, "rc=%d\n", rc); return 2; }
    for (size_t i = 0; i < raw.size(); ++i) {
        auto* b = raw[i]->get_buffer();
        std::printf("%d %s\n", (int)st[i], hex(b->get_data_start_ptr(), b->get_data_length()).c_str());
    }
    return 0;
}

// Input: one hex frame per line. Output per packet: "hash hex(64-byte record)".
static int flow_mode() {
    std::vector<std::unique_ptr<netflow_amd::PacketBuffer>> bufs;
    std::vector<std::unique_ptr<netflow_amd::Packet>> pkts;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::vector<uint8_t> f = unhex(line);
        bufs.emplace_back(new netflow_amd::PacketBuffer(f.size() + 96, 32, f.size()));
        if (!f.empty()) std::memcpy(bufs.back()->get_data_start_ptr(), f.data(), f.size());
        pkts.emplace_back(new netflow_amd::Packet(bufs.back().get()));
    }
    std::vector<netflow_amd::Packet*> raw;
    for (auto& p : pkts) raw.push_back(p.get());
    std::vector<nfcs_flow_key> keys(raw.size());
    std::vector<uint32_t> hashes(raw.size(), 0xEEEEEEEEu);
    int rc = netflow_amd::flow_keys_batch(raw.data(), raw.size(), keys.data(), hashes.data());
    if (rc) { std::fprintf(stderr, "rc=%d\n", rc); return 2; }
    for (size_t i = 0; i < raw.size(); ++i)
        std::printf("%u %s\n", hashes[i], hex(reinterpret_cast<const uint8_t*>(&keys[i]), sizeof(nfcs_flow_key)).c_str());
    return 0;
}

// Frames in BufferPool slots (pinned arena), one batch without gather copies; plus the
// pool's allocate / free / reference-count behaviour. Output per packet: "status hex(frame)".
static int pool_mode(uint32_t flags) {
    netflow_amd::BufferPool pool(4096, 9216);  // jumbo frames fit a slot
    int bad = 0;
    {   // buffer_pool.hpp semantics: headroom, empty data, refcount, reuse, heap overflow
        netflow_amd::PacketBuffer* a = pool.allocate_buffer(100, 32);
        bad += !pool.in_arena(a) || a->get_headroom() != 32 || a->get_data_length() != 0 || a->ref_count != 1;
        const size_t before = pool.available();
        a->increment_ref();
        pool.free_buffer(a);                       // still referenced: stays out
        bad += pool.available() != before;
        pool.free_buffer(a);                       // last reference: back to the pool
        bad += pool.available() != before + 1;
        netflow_amd::PacketBuffer* big = pool.allocate_buffer(12000, 32);  // larger than a slot
        bad += pool.in_arena(big) || big->get_capacity() < 12032;
        pool.free_buffer(big);
        bad += pool.allocate_buffer(10000, 32) != big;  // the heap buffer is reused
        pool.free_buffer(big);
    }
    std::vector<netflow_amd::PacketBuffer*> bufs;
    std::vector<std::unique_ptr<netflow_amd::Packet>> pkts;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::vector<uint8_t> f = unhex(line);
        netflow_amd::PacketBuffer* b = pool.allocate_buffer(f.size(), 32);
        b->set_data_len(f.size());
        if (!f.empty()) std::memcpy(b->get_data_start_ptr(), f.data(), f.size());
        bufs.push_back(b);
        pkts.emplace_back(new netflow_amd::Packet(b));
    }
    std::vector<netflow_amd::Packet*> raw;
    for (auto& p : pkts) raw.push_back(p.get());
    // a burst in arbitrary order (the pool sorts it into arena order)
    for (size_t i = 0; i + 1 < raw.size(); i += 7) std::swap(raw[i], raw[i + 1]);
    std::vector<uint8_t> st(raw.size(), 0xEE);
    int rc = pool.update_checksums_batch(raw.data(), raw.size(), st.data(), flags);
    if (rc) { std::fprintf(stderr, "rc=%d\n", rc); return 2; }
    std::vector<uint8_t> st_by_buf(raw.size());
    for (size_t i = 0; i < raw.size(); ++i) {
        const size_t k = std::find(bufs.begin(), bufs.end(), raw[i]->get_buffer()) - bufs.begin();
        st_by_buf[k] = st[i];
    }
    for (size_t k = 0; k < bufs.size(); ++k)
        std::printf("%d %s\n", (int)st_by_buf[k], hex(bufs[k]->get_data_start_ptr(), bufs[k]->get_data_length()).c_str());
    std::fprintf(stderr, "pool_failures=%d\n", bad);
    pkts.clear();
    for (auto* b : bufs) pool.free_buffer(b);
    return bad ? 3 : 0;
}

// Throughput of the pool path vs the gather path: 256K random 1500-byte UDP-sized frames
// (content irrelevant to the rate), GB/s of frames per batch call, best of 5.
static int pool_bench() {
    const size_t n = 262144, len = 1500;
    netflow_amd::BufferPool pool(n, 1536 + 32);
    std::vector<netflow_amd::PacketBuffer*> bufs;
    std::vector<std::unique_ptr<netflow_amd::Packet>> pkts;
    std::vector<netflow_amd::Packet*> raw;
    uint64_t x = 12345;
    for (size_t i = 0; i < n; ++i) {
        netflow_amd::PacketBuffer* b = pool.allocate_buffer(len, 32);
        b->set_data_len(len);
        for (size_t j = 0; j < len; ++j) { x = x * 6364136223846793005ull + 1442695040888963407ull; b->get_data_start_ptr()[j] = (uint8_t)(x >> 56); }
        bufs.push_back(b);
        pkts.emplace_back(new netflow_amd::Packet(b));
        raw.push_back(pkts.back().get());
    }
    auto rate = [&](auto&& call) {
        double best = 1e30;
        for (int r = 0; r < 6; ++r) {
            const auto t0 = std::chrono::steady_clock::now();
            if (call()) return -1.0;
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (r > 0 && s < best) best = s;
        }
        return n * len / best / 1e9;
    };
    const double g = rate([&] { return netflow_amd::update_checksums_batch(raw.data(), n); });
    const double p = rate([&] { return pool.update_checksums_batch(raw.data(), n); });
    const double z = rate([&] { return pool.update_checksums_batch(raw.data(), n, nullptr, NFCS_HOST_ZERO_COPY); });
    std::printf("gather_GBps=%.1f pool_GBps=%.1f pool_zero_copy_GBps=%.1f\n", g, p, z);
    pkts.clear();
    for (auto* b : bufs) pool.free_buffer(b);
    return 0;
}

// MultiGpu over K contexts (all on device 0 here: the one-GPU box rehearses the per-GPU threads,
// staging rings and byte-balanced ranges of an 8-GPU node).
static int multi_mode(int k) {
    std::vector<std::vector<uint8_t>> fr;
    std::string line;
    while (std::getline(std::cin, line)) fr.push_back(unhex(line));
    std::vector<nfcs_desc> desc(fr.size());
    uint64_t off = 0;
    for (size_t i = 0; i < fr.size(); ++i) {
        desc[i].off16 = (uint32_t)(off / 16);
        desc[i].len = (uint32_t)fr[i].size();
        off += (fr[i].size() + 127) / 128 * 128;
    }
    std::vector<uint8_t> arena(off + 16, 0);
    for (size_t i = 0; i < fr.size(); ++i)
        if (!fr[i].empty()) std::memcpy(arena.data() + (uint64_t)desc[i].off16 * 16, fr[i].data(), fr[i].size());
    int rc = 0;
    netflow_amd::MultiGpu mg(std::vector<int>(k, 0), std::nothrow, &rc);
    if (rc) { std::fprintf(stderr, "ctx rc=%d\n", rc); return 2; }
    std::vector<uint8_t> st(fr.size(), 0xEE);
    std::vector<uint32_t> b(k + 1);
    rc = mg.update_host(arena.data(), arena.size(), desc.data(), (uint32_t)fr.size(), st.data(), 0, b.data());
    if (rc) { std::fprintf(stderr, "rc=%d\n", rc); return 3; }
    for (size_t i = 0; i < fr.size(); ++i)
        std::printf("%d %s\n", (int)st[i], hex(arena.data() + (uint64_t)desc[i].off16 * 16, fr[i].size()).c_str());
    std::fprintf(stderr, "bounds");
    for (uint32_t x : b) std::fprintf(stderr, " %u", x);
    std::fprintf(stderr, "\n");
    return 0;
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    if (mode == "poolbench") return pool_bench();
    if (mode == "pool") return pool_mode(0);
    if (mode == "poolzc") return pool_mode(NFCS_HOST_ZERO_COPY);
    if (mode == "cpu") return cpu_checks();
    if (mode == "vlan" || mode == "vlan1") return vlan_mode(mode == "vlan1");
    if (mode == "l3") return l3_mode();
    if (mode == "flow") return flow_mode();
    if (mode == "multi") return multi_mode(argc > 2 ? std::atoi(argv[2]) : 2);
    std::vector<std::unique_ptr<netflow_amd::PacketBuffer>> bufs;
    std::vector<std::unique_ptr<netflow_amd::Packet>> pkts;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::vector<uint8_t> f = unhex(line);
        // data window inside a larger buffer with headroom, as the reference's pools allocate
        bufs.emplace_back(new netflow_amd::PacketBuffer(f.size() + 96, 32, f.size()));
        if (!f.empty()) std::memcpy(bufs.back()->get_data_start_ptr(), f.data(), f.size());
        pkts.emplace_back(new netflow_amd::Packet(bufs.back().get()));
    }
    std::vector<netflow_amd::Packet*> raw;
    for (auto& p : pkts) raw.push_back(p.get());
    std::vector<uint8_t> st(raw.size(), 0xEE);
    if (mode == "batch") {
        int rc = netflow_amd::update_checksums_batch(raw, st.data());
        if (rc) { std::fprintf(stderr, "rc=%d\n", rc); return 2; }
    } else {
        for (auto* p : raw) p->update_checksums();
    }
    for (size_t i = 0; i < raw.size(); ++i) {
        auto* b = raw[i]->get_buffer();
        std::printf("%d %s\n", (int)st[i], hex(b->get_data_start_ptr(), b->get_data_length()).c_str());
    }
    return 0;
}
