// netflow_adapter_test.cpp — include/netflow_amd/netflow_adapter.hpp over NetFlow++'s OWN
// netflow::Packet / netflow::PacketBuffer, compiled against the reference's headers
// (/root/reference/include, by tests/cpp/Makefile into tests/cpp/_ref/, never copied into the repo).
// The reference's own Packet::update_checksums / push_vlan / pop_vlan run in this process as the
// checker. Frames arrive as hex lines on stdin.
//   cpu   lines "<hex>": netflow_amd::Packet::update_checksums() (the single-packet CPU path of
//         include/netflow_amd/cpu_update.hpp) against the reference's, per frame; then the batch
//         free function without a GPU must return an error code, not throw.
//         Prints "frames=N mismatches=M skipped=S adapter_rc=R".
//   vcpu  lines "<op> <room> <hex>": netflow_amd::Packet::push_vlan / pop_vlan (CPU) against the
//         reference's on identical buffers (return value, data length, every buffer byte).
//         Prints "frames=N mismatches=M skipped=S".
//   gpu   lines "<hex>": a std::vector<netflow::Packet*> burst through
//         netflow_amd::update_checksums_batch (gfx950) against the reference's per-packet calls.
//         Prints "frames=N mismatches=M skipped=S rc=R", then one "<status>" line per frame.
//   vgpu  lines "<op> <room> <hex>": netflow_amd::vlan_batch over netflow::Packet against the
//         reference's push_vlan / pop_vlan. Prints "frames=N mismatches=M skipped=S rc=R".
//   path-gpu / path-cpu  (no input) the reference's own test scenario of the path,
//         PacketTest.UpdateChecksumsAfterModification (tests/packet_test.cpp:202-293): frames from
//         its builder (packet_test.cpp:82-138), update, rewrite src_ip / the TCP source port,
//         update again, with its EXPECT_NE conditions — on a burst of netflow::Packet through
//         netflow_amd::update_checksums_batch (gpu), or through the single-packet CPU members of
//         netflow_amd::Packet (cpu); the reference's per-packet calls on copies are the checker at
//         each step. Prints "frames=N steps=2 mismatches=M expect_ne_failed=F rc=R".
// Frames where the reference itself reads or writes outside its buffer (IHL past the frame; a push
// without tailroom into a buffer whose capacity holds len + 4; a re-tag of a runt in a buffer of
// fewer than 16 bytes) are skipped: there the reference is undefined.
#include <netflow++/packet.hpp>

#include <cstdio>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include "netflow_amd/netflow_adapter.hpp"

namespace {

std::vector<uint8_t> unhex(const std::string& s) {
    std::vector<uint8_t> v;
    for (size_t i = 0; i + 1 < s.size(); i += 2) v.push_back((uint8_t)std::stoul(s.substr(i, 2), nullptr, 16));
    return v;
}

constexpr size_t kHeadroom = 32;

// A reference PacketBuffer holding `f` after kHeadroom bytes, `room` bytes of buffer from the data
// start, zero-filled past the frame.
std::unique_ptr<netflow::PacketBuffer> ref_buffer(const std::vector<uint8_t>& f, size_t room) {
    std::unique_ptr<netflow::PacketBuffer> b(new netflow::PacketBuffer(kHeadroom + room, kHeadroom, f.size()));
    std::memset(b->get_data_start_ptr() - kHeadroom, 0, kHeadroom + room);
    if (!f.empty()) std::memcpy(b->get_data_start_ptr(), f.data(), f.size());
    return b;
}

// The reference reads past its buffer when an IPv4 header's IHL reaches past the frame.
bool ihl_past_frame(const std::vector<uint8_t>& f) {
    const size_t n = f.size();
    if (n < 14) return false;
    const size_t l2 = (f[12] == 0x81 && f[13] == 0x00) ? 18 : 14;
    return l2 + 20 <= n && (f[l2] >> 4) == 4 && l2 + (f[l2] & 15u) * 4u > n;
}

bool vlan_undefined(const std::vector<uint8_t>& f, uint32_t op, size_t room) {
    const size_t n = f.size();
    const bool tagged = n >= 14 && f[12] == 0x81 && f[13] == 0x00;
    if ((op & NFCS_VLAN_OP_MASK) == NFCS_VLAN_PUSH && n >= 14) {
        if (tagged && room < 16) return true;                       // re-tag writes bytes 14-15
        if (!tagged && n + 4 > room && n + 4 <= kHeadroom + room) return true;  // memmove past the end
    }
    // the edited frame then goes through update_checksums()
    std::vector<uint8_t> g(f);
    if ((op & NFCS_VLAN_OP_MASK) == NFCS_VLAN_PUSH && !tagged && n >= 14 && n + 4 <= room) {
        g.insert(g.begin() + 12, {0x81, 0x00, 0x00, 0x00});
    } else if ((op & NFCS_VLAN_OP_MASK) == NFCS_VLAN_POP && tagged && n >= 18) {
        g.erase(g.begin() + 12, g.begin() + 16);
    }
    return ihl_past_frame(g);
}

bool ref_vlan(netflow::Packet& p, uint32_t op) {
    const uint32_t kind = op & NFCS_VLAN_OP_MASK;
    if (kind == NFCS_VLAN_PUSH) return p.push_vlan(op & 0xFFFu, (op >> 13) & 7u);
    if (kind == NFCS_VLAN_POP) return p.pop_vlan();
    return false;
}

int cpu_mode() {
    std::string line;
    size_t n = 0, bad = 0, skipped = 0;
    while (std::getline(std::cin, line)) {
        const std::vector<uint8_t> f = unhex(line);
        ++n;
        if (ihl_past_frame(f)) { ++skipped; continue; }
        auto rb = ref_buffer(f, f.size() + 64);
        netflow::Packet rp(rb.get());
        rp.update_checksums();
        netflow_amd::PacketBuffer mb(kHeadroom + f.size() + 64, kHeadroom, f.size());
        if (!f.empty()) std::memcpy(mb.get_data_start_ptr(), f.data(), f.size());
        netflow_amd::Packet mp(&mb);
        mp.update_checksums();
        bad += f.size() && std::memcmp(rb->get_data_start_ptr(), mb.get_data_start_ptr(), f.size()) != 0;
    }
    // without a device the batch entry returns an error code instead of throwing
    int rc = 0;
    {
        auto rb = ref_buffer(std::vector<uint8_t>(60, 0), 64);
        netflow::Packet rp(rb.get());
        std::vector<netflow::Packet*> v{&rp};
        rc = netflow_amd::update_checksums_batch(v);
    }
    std::printf("frames=%zu mismatches=%zu skipped=%zu adapter_rc=%d\n", n, bad, skipped, rc);
    return bad ? 1 : 0;
}

struct VlanCase {
    uint32_t op;
    size_t room;
    std::vector<uint8_t> f;
};

std::vector<VlanCase> read_vlan_cases() {
    std::vector<VlanCase> cs;
    std::string line;
    while (std::getline(std::cin, line)) {
        const size_t a = line.find(' '), b = line.find(' ', a + 1);
        cs.push_back({(uint32_t)std::stoul(line.substr(0, a)), (size_t)std::stoul(line.substr(a + 1, b - a - 1)),
                      unhex(line.substr(b + 1))});
    }
    return cs;
}

int vcpu_mode() {
    size_t bad = 0, skipped = 0;
    const std::vector<VlanCase> cs = read_vlan_cases();
    for (const VlanCase& c : cs) {
        if (vlan_undefined(c.f, c.op, c.room)) { ++skipped; continue; }
        auto rb = ref_buffer(c.f, c.room);
        netflow::Packet rp(rb.get());
        const bool rok = ref_vlan(rp, c.op);
        netflow_amd::PacketBuffer mb(kHeadroom + c.room, kHeadroom, c.f.size());
        std::memset(mb.get_data_start_ptr() - kHeadroom, 0, kHeadroom + c.room);
        if (!c.f.empty()) std::memcpy(mb.get_data_start_ptr(), c.f.data(), c.f.size());
        netflow_amd::Packet mp(&mb);
        const uint32_t kind = c.op & NFCS_VLAN_OP_MASK;
        const bool mok = kind == NFCS_VLAN_PUSH ? mp.push_vlan(c.op & 0xFFFu, (c.op >> 13) & 7u)
                       : kind == NFCS_VLAN_POP ? mp.pop_vlan() : false;
        bad += rok != mok || rb->get_data_length() != mb.get_data_length() ||
               std::memcmp(rb->get_data_start_ptr(), mb.get_data_start_ptr(), c.room) != 0;
    }
    std::printf("frames=%zu mismatches=%zu skipped=%zu\n", cs.size(), bad, skipped);
    return bad ? 1 : 0;
}

int gpu_mode() {
    std::vector<std::vector<uint8_t>> fs;
    std::string line;
    while (std::getline(std::cin, line)) fs.push_back(unhex(line));
    const size_t n = fs.size();
    std::vector<std::unique_ptr<netflow::PacketBuffer>> gb, rb;
    std::vector<std::unique_ptr<netflow::Packet>> gp, rp;
    std::vector<netflow::Packet*> burst;
    for (const auto& f : fs) {
        gb.push_back(ref_buffer(f, f.size() + 64));
        rb.push_back(ref_buffer(f, f.size() + 64));
        gp.emplace_back(new netflow::Packet(gb.back().get()));
        rp.emplace_back(new netflow::Packet(rb.back().get()));
        burst.push_back(gp.back().get());
    }
    std::vector<uint8_t> st(n, 0xEE);
    const int rc = netflow_amd::update_checksums_batch(burst, st.data());
    size_t bad = 0, skipped = 0;
    for (size_t i = 0; i < n; ++i) {
        if (ihl_past_frame(fs[i])) {  // the engine leaves these untouched (NFCS_ST_OOB)
            ++skipped;
            bad += st[i] != NFCS_ST_OOB || (fs[i].size() && std::memcmp(gb[i]->get_data_start_ptr(), fs[i].data(), fs[i].size()));
            continue;
        }
        rp[i]->update_checksums();  // the reference, one packet at a time
        bad += fs[i].size() && std::memcmp(gb[i]->get_data_start_ptr(), rb[i]->get_data_start_ptr(), fs[i].size()) != 0;
    }
    std::printf("frames=%zu mismatches=%zu skipped=%zu rc=%d\n", n, bad, skipped, rc);
    for (size_t i = 0; i < n; ++i) std::printf("%d\n", (int)st[i]);
    return bad || rc ? 1 : 0;
}

int vgpu_mode() {
    const std::vector<VlanCase> cs = read_vlan_cases();
    const size_t n = cs.size();
    std::vector<std::unique_ptr<netflow::PacketBuffer>> gb, rb;
    std::vector<std::unique_ptr<netflow::Packet>> gp, rp;
    std::vector<netflow::Packet*> burst;
    std::vector<uint32_t> ops;
    for (const VlanCase& c : cs) {
        gb.push_back(ref_buffer(c.f, c.room));
        rb.push_back(ref_buffer(c.f, c.room));
        gp.emplace_back(new netflow::Packet(gb.back().get()));
        rp.emplace_back(new netflow::Packet(rb.back().get()));
        burst.push_back(gp.back().get());
        ops.push_back(c.op);
    }
    std::unique_ptr<bool[]> ok(new bool[n ? n : 1]);
    const int rc = netflow_amd::vlan_batch(burst, ops.data(), ok.get());
    size_t bad = 0, skipped = 0;
    for (size_t i = 0; i < n; ++i) {
        if (vlan_undefined(cs[i].f, cs[i].op, cs[i].room)) { ++skipped; continue; }
        const bool rok = ref_vlan(*rp[i], cs[i].op);
        bad += rok != ok[i] || rb[i]->get_data_length() != gb[i]->get_data_length() ||
               std::memcmp(rb[i]->get_data_start_ptr(), gb[i]->get_data_start_ptr(), cs[i].room) != 0;
    }
    std::printf("frames=%zu mismatches=%zu skipped=%zu rc=%d\n", n, bad, skipped, rc);
    return bad || rc ? 1 : 0;
}

// PacketTest::build_raw_packet (tests/packet_test.cpp:82-138) for the three frames of
// UpdateChecksumsAfterModification: Ethernet II untagged, IPv4 IHL 5, TTL 64, a 20-byte TCP header
// (data offset byte at l4 + 16) or an 8-byte UDP header, then the payload. `salt` > 0 varies the
// source address and payload so a burst holds distinct frames; salt 0 is the test's frame.
std::vector<uint8_t> test_builder_frame(uint8_t proto, uint16_t sp, uint16_t dp, const char* payload,
                                        uint32_t salt) {
    const uint8_t dst_mac[6] = {0xAA, 0xBB, 0xCC, 0xDD, 0xEE, 0xFF};
    const uint8_t src_mac[6] = {0x00, 0x11, 0x22, 0x33, 0x44, 0x55};
    std::vector<uint8_t> pl(payload, payload + std::strlen(payload));
    for (size_t i = 0; i < pl.size() && salt; ++i) pl[i] = (uint8_t)(pl[i] + salt * (i + 1));
    std::vector<uint8_t> d(dst_mac, dst_mac + 6);
    d.insert(d.end(), src_mac, src_mac + 6);
    d.push_back(0x08); d.push_back(0x00);
    const size_t l4_len = proto == 6 ? 20 : 8 + pl.size();
    const uint16_t tl = (uint16_t)(20 + l4_len);
    const uint8_t ip[20] = {0x45, 0x00, (uint8_t)(tl >> 8), (uint8_t)tl, 0x00, 0x01, 0x00, 0x00, 0x40, proto,
                            0x00, 0x00, 192, 168, (uint8_t)(1 + (salt >> 8)), (uint8_t)(10 + salt), 192, 168, 1, 20};
    d.insert(d.end(), ip, ip + 20);
    d.push_back((uint8_t)(sp >> 8)); d.push_back((uint8_t)sp);
    d.push_back((uint8_t)(dp >> 8)); d.push_back((uint8_t)dp);
    if (proto == 6) {
        for (int i = 0; i < 12; ++i) d.push_back(0x00);
        d.push_back(0x50); d.push_back(0x00);
        d.push_back(0x00); d.push_back(0x00);
    } else {
        const uint16_t ul = (uint16_t)(8 + pl.size());
        d.push_back((uint8_t)(ul >> 8)); d.push_back((uint8_t)ul);
        d.push_back(0x00); d.push_back(0x00);
    }
    d.insert(d.end(), pl.begin(), pl.end());
    return d;
}

// The reference's own scenario, packet_test.cpp:202-293, over a burst: per repetition the test's
// three packets — (1) IPv4/TCP with its header checksum zeroed (210-213), (2) IPv4/TCP with the bytes
// it zeroes at l4 + 16..17 (245-248), (3) IPv4/UDP with its checksum zeroed (275-278).
int path_mode(bool gpu) {
    const size_t reps = gpu ? 1024 : 1;
    std::vector<std::vector<uint8_t>> fs;
    for (size_t r = 0; r < reps; ++r) {
        std::vector<uint8_t> a = test_builder_frame(6, 12345, 80, "TEST", (uint32_t)r);
        a[14 + 10] = a[14 + 11] = 0;
        std::vector<uint8_t> b = test_builder_frame(6, 12345, 80, "TEST", (uint32_t)r);
        b[14 + 20 + 16] = b[14 + 20 + 17] = 0;
        std::vector<uint8_t> c = test_builder_frame(17, 54321, 53, "DATA", (uint32_t)r);
        c[14 + 20 + 6] = c[14 + 20 + 7] = 0;
        fs.push_back(a); fs.push_back(b); fs.push_back(c);
    }
    const size_t n = fs.size();
    std::vector<std::unique_ptr<netflow::PacketBuffer>> gb, rb;
    std::vector<std::unique_ptr<netflow::Packet>> gp, rp;
    std::vector<netflow::Packet*> burst;
    for (const auto& f : fs) {
        gb.push_back(ref_buffer(f, f.size()));
        rb.push_back(ref_buffer(f, f.size()));
        gp.emplace_back(new netflow::Packet(gb.back().get()));
        rp.emplace_back(new netflow::Packet(rb.back().get()));
        burst.push_back(gp.back().get());
    }
    int rc = 0;
    size_t bad = 0, ne_failed = 0;
    auto engine_update = [&]() {
        if (gpu) {
            const int r = netflow_amd::update_checksums_batch(burst);
            if (r) rc = r;
            return;
        }
        for (size_t i = 0; i < n; ++i) {  // the single-packet CPU members of netflow_amd::Packet
            netflow_amd::PacketBuffer mb(kHeadroom + fs[i].size(), kHeadroom, fs[i].size());
            std::memcpy(mb.get_data_start_ptr(), gb[i]->get_data_start_ptr(), fs[i].size());
            netflow_amd::Packet mp(&mb);
            mp.update_checksums();
            std::memcpy(gb[i]->get_data_start_ptr(), mb.get_data_start_ptr(), fs[i].size());
        }
    };
    auto check_bytes = [&]() {
        for (size_t i = 0; i < n; ++i) {
            rp[i]->update_checksums();  // the reference, one packet at a time
            bad += std::memcmp(gb[i]->get_data_start_ptr(), rb[i]->get_data_start_ptr(), fs[i].size()) != 0;
        }
    };
    // step 1: update (221, 255, 285), then the EXPECT_NEs on the engine's packets (225, 259, 290)
    engine_update();
    check_bytes();
    std::vector<uint16_t> ip0(reps), tcp0(reps);
    for (size_t r = 0; r < reps; ++r) {
        netflow::Packet& a = *gp[3 * r];
        netflow::Packet& b = *gp[3 * r + 1];
        netflow::Packet& c = *gp[3 * r + 2];
        if (!a.ipv4() || !b.tcp() || !c.udp()) { ++ne_failed; continue; }  // the ASSERT_NEs
        ip0[r] = a.ipv4()->header_checksum;
        tcp0[r] = b.tcp()->checksum;
        ne_failed += ip0[r] == 0;
        ne_failed += tcp0[r] == 0;
        ne_failed += c.udp()->checksum == 0;
        // the modifications (231, 263), on the engine's and the reference's copies alike
        const_cast<netflow::IPv4Header*>(a.ipv4())->src_ip = htonl(0x01020304);
        const_cast<netflow::IPv4Header*>(rp[3 * r]->ipv4())->src_ip = htonl(0x01020304);
        const_cast<netflow::TcpHeader*>(b.tcp())->src_port = htons(54321);
        const_cast<netflow::TcpHeader*>(rp[3 * r + 1]->tcp())->src_port = htons(54321);
    }
    // step 2: update again (233, 265), the EXPECT_NEs of 234-235 and 266-267
    engine_update();
    check_bytes();
    for (size_t r = 0; r < reps; ++r) {
        netflow::Packet& a = *gp[3 * r];
        netflow::Packet& b = *gp[3 * r + 1];
        if (!a.ipv4() || !b.tcp()) { ++ne_failed; continue; }
        ne_failed += a.ipv4()->header_checksum == ip0[r];
        ne_failed += a.ipv4()->header_checksum == 0;
        ne_failed += b.tcp()->checksum == tcp0[r];
        ne_failed += b.tcp()->checksum == 0;
    }
    std::printf("frames=%zu steps=2 mismatches=%zu expect_ne_failed=%zu rc=%d\n", n, bad, ne_failed, rc);
    return bad || ne_failed || rc ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    if (mode == "cpu") return cpu_mode();
    if (mode == "vcpu") return vcpu_mode();
    if (mode == "gpu") return gpu_mode();
    if (mode == "vgpu") return vgpu_mode();
    if (mode == "path-gpu") return path_mode(true);
    if (mode == "path-cpu") return path_mode(false);
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
}
