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
//   icmp-gpu / icmp-cpu  (no input) IcmpProcessorTest's scenarios (tests/icmp_processor_test.cpp:
//         278-407) and the packets IcmpProcessor builds from them (icmp_processor.cpp:96-180,
//         255-336), in two stages of update_checksums() over bursts (see icmp_mode).
//   adapterbench [n reps threads want]  the reference's call convention end to end, timed (bench.py's
//         host_adapter sub-line; see adapterbench_mode). Prints one JSON line.
// Frames where the reference itself reads or writes outside its buffer (IHL past the frame; a push
// without tailroom into a buffer whose capacity holds len + 4; a re-tag of a runt in a buffer of
// fewer than 16 bytes) are skipped: there the reference is undefined.
#include <netflow++/packet.hpp>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <functional>
#include <iostream>
#include <memory>
#include <string>
#include <thread>
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

// One update_checksums() over every packet of `burst` by the engine: the GPU batch entry, or the
// single-packet CPU members of netflow_amd::Packet on a copy of each frame. Returns the batch rc.
int engine_update(bool gpu, std::vector<netflow::Packet*>& burst) {
    if (gpu) return netflow_amd::update_checksums_batch(burst);
    for (netflow::Packet* p : burst) {
        netflow::PacketBuffer* b = p->get_buffer();
        const size_t len = b->get_data_length();
        netflow_amd::PacketBuffer mb(kHeadroom + len, kHeadroom, len);
        if (len) std::memcpy(mb.get_data_start_ptr(), b->get_data_start_ptr(), len);
        netflow_amd::Packet mp(&mb);
        mp.update_checksums();
        if (len) std::memcpy(b->get_data_start_ptr(), mb.get_data_start_ptr(), len);
    }
    return 0;
}

// The reference's sum (packet.hpp:894-912: big-endian words, an odd last byte added as the LOW
// byte, end-around carry) over `n` bytes: a message whose checksum field holds what
// update_checksums() wrote sums to 0xFFFF under it, odd lengths included.
uint32_t ref_sum(const uint8_t* p, size_t n) {
    uint32_t s = 0;
    for (size_t i = 0; i + 1 < n; i += 2) s += (uint32_t)p[i] << 8 | p[i + 1];
    if (n & 1) s += p[n - 1];
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return s;
}

void put16(std::vector<uint8_t>& d, uint16_t v) { d.push_back((uint8_t)(v >> 8)); d.push_back((uint8_t)v); }
void put_bytes(std::vector<uint8_t>& d, const uint8_t* p, size_t n) { d.insert(d.end(), p, p + n); }

// Ethernet II (IPv4) + a 20-byte IPv4 header with a zero checksum, as the ICMP test's builders
// (icmp_processor_test.cpp:103-124, 153-174) and IcmpProcessor (icmp_processor.cpp:142-158,
// 296-311) lay them out. Addresses are given as the four bytes in wire order.
std::vector<uint8_t> eth_ipv4(const uint8_t* dst_mac, const uint8_t* src_mac, uint16_t id, uint8_t ttl,
                              uint8_t proto, const uint8_t* sip, const uint8_t* dip, size_t l4_bytes) {
    std::vector<uint8_t> d;
    put_bytes(d, dst_mac, 6);
    put_bytes(d, src_mac, 6);
    put16(d, 0x0800);
    d.push_back(0x45); d.push_back(0x00);
    put16(d, (uint16_t)(20 + l4_bytes));
    put16(d, id);
    put16(d, 0x0000);
    d.push_back(ttl); d.push_back(proto);
    put16(d, 0x0000);
    put_bytes(d, sip, 4);
    put_bytes(d, dip, 4);
    return d;
}

// IcmpProcessorTest's scenarios (tests/icmp_processor_test.cpp:278-407) on a burst of `reps`
// repetitions (repetition 0 = the test's exact frames; later ones vary ids, sequence numbers,
// payloads and addresses). Stage 1: the test's builders finish with update_checksums()
// (create_icmp_echo_request_packet, 193; create_ipv4_packet_for_icmp_test, 133 — UDP whose 8-byte
// "payload" is the UDP header, length 0xCAFE, so only the IPv4 checksum is written). Stage 2: from
// the ENGINE's stage-1 packets, the packets IcmpProcessor builds — the echo reply
// (send_icmp_echo_reply, icmp_processor.cpp:96-180) and the Time Exceeded / Destination
// Unreachable messages (send_icmp_error_packet_base, 255-336; the random IP id is made
// deterministic) — then update_checksums() (180, 336). At both stages the reference's per-packet
// calls on copies are the checker; then the test's EXPECTs on the reply (313-338), and on every
// packet: IPv4 header and ICMP message sum to 0xFFFF under the reference's own sum.
// Prints "frames=N stages=2 mismatches=M expect_failed=F rc=R".
int icmp_mode(bool gpu) {
    const size_t reps = gpu ? 1024 : 4;
    const uint8_t my_mac[6] = {0x00, 0xAA, 0xBB, 0xCC, 0xDD, 0xEE};
    const uint8_t req_mac[6] = {0x11, 0x22, 0x33, 0x44, 0x55, 0x66};
    const uint8_t my_ip[4] = {192, 168, 0, 1};
    const uint8_t orig_src_mac[6] = {0xDE, 0xAD, 0xBE, 0xEF, 0x00, 0x01};
    const uint8_t orig_dst_mac[6] = {0xDE, 0xAD, 0xBE, 0xEF, 0x00, 0x02};
    const uint8_t orig_src_ip[4] = {192, 168, 1, 100};
    const uint8_t te_dst_ip[4] = {172, 16, 1, 100};
    const uint8_t nu_dst_ip[4] = {203, 0, 113, 5};
    const uint8_t err_src_mac[6] = {0x0A, 0x00, 0x00, 0x00, 0x00, 0x01};
    const uint8_t nh_mac[6] = {0x0A, 0x00, 0x00, 0x00, 0x00, 0x02};
    const uint8_t err_src_ip[4] = {10, 0, 0, 1};
    const uint8_t l4_payload[8] = {0xDE, 0xAD, 0xBE, 0xEF, 0xCA, 0xFE, 0xBA, 0xBE};

    struct Req { uint16_t id, seq; std::vector<uint8_t> payload; uint8_t req_ip[4]; };
    std::vector<Req> reqs(reps);
    std::vector<std::vector<uint8_t>> s1;  // per repetition: echo request, TE original, NU original
    for (size_t r = 0; r < reps; ++r) {
        Req& q = reqs[r];
        q.id = (uint16_t)(1234 + r);
        q.seq = (uint16_t)(1 + r);
        q.payload = {'h', 'e', 'l', 'l', 'o'};
        for (size_t i = 0; i < r % 64; ++i) q.payload.push_back((uint8_t)(r * 31 + i));  // odd and even sizes
        const uint8_t rip[4] = {192, 168, 0, (uint8_t)(100 + r % 100)};
        std::memcpy(q.req_ip, rip, 4);
        std::vector<uint8_t> e = eth_ipv4(my_mac, req_mac, 54321, 64, 1, q.req_ip, my_ip, 8 + q.payload.size());
        e.push_back(8); e.push_back(0);  // TYPE_ECHO_REQUEST, code 0
        put16(e, 0x0000);
        put16(e, q.id);
        put16(e, q.seq);
        put_bytes(e, q.payload.data(), q.payload.size());
        std::vector<uint8_t> te = eth_ipv4(orig_dst_mac, orig_src_mac, 12345, 1, 17, orig_src_ip, te_dst_ip, 8);
        put_bytes(te, l4_payload, 8);
        std::vector<uint8_t> nu = eth_ipv4(orig_dst_mac, orig_src_mac, 12345, 64, 17, orig_src_ip, nu_dst_ip, 8);
        put_bytes(nu, l4_payload, 8);
        s1.push_back(e); s1.push_back(te); s1.push_back(nu);
    }

    int rc = 0;
    size_t bad = 0, failed = 0, frames = 0;
    // one stage: buffers for the engine and the reference, the engine's burst, the reference's calls
    auto stage = [&](const std::vector<std::vector<uint8_t>>& fs, std::vector<std::unique_ptr<netflow::PacketBuffer>>& gb,
                     std::vector<std::unique_ptr<netflow::Packet>>& gp) {
        std::vector<std::unique_ptr<netflow::PacketBuffer>> rb;
        std::vector<std::unique_ptr<netflow::Packet>> rp;
        std::vector<netflow::Packet*> burst;
        for (const auto& f : fs) {
            gb.push_back(ref_buffer(f, f.size()));
            rb.push_back(ref_buffer(f, f.size()));
            gp.emplace_back(new netflow::Packet(gb.back().get()));
            rp.emplace_back(new netflow::Packet(rb.back().get()));
            burst.push_back(gp.back().get());
        }
        const int r = engine_update(gpu, burst);
        if (r) rc = r;
        for (size_t i = 0; i < fs.size(); ++i) {
            rp[i]->update_checksums();
            bad += std::memcmp(gb[i]->get_data_start_ptr(), rb[i]->get_data_start_ptr(), fs[i].size()) != 0;
            const uint8_t* f = gb[i]->get_data_start_ptr();
            failed += ref_sum(f + 14, 20) != 0xFFFFu;                                   // IPv4 header
            if (f[23] == 1) failed += ref_sum(f + 34, fs[i].size() - 34) != 0xFFFFu;    // ICMP message
        }
        frames += fs.size();
    };
    std::vector<std::unique_ptr<netflow::PacketBuffer>> b1, b2;
    std::vector<std::unique_ptr<netflow::Packet>> p1, p2;
    stage(s1, b1, p1);

    std::vector<std::vector<uint8_t>> s2;  // per repetition: echo reply, Time Exceeded, Unreachable
    for (size_t r = 0; r < reps; ++r) {
        // the echo reply from the engine's request (icmp_processor.cpp:96-173)
        const netflow::Packet& rq = *p1[3 * r];
        const netflow::IPv4Header* ip = rq.ipv4();
        const netflow::IcmpHeader* ic = rq.icmp();
        if (!ip || !ic) { ++failed; continue; }
        const uint8_t* q = rq.get_buffer()->get_data_start_ptr();
        const size_t ihl = (size_t)(q[14] & 15u) * 4u;
        size_t pay = ntohs(ip->total_length) - ihl - 8;
        const size_t pay_off = 14 + ihl + 8;
        if (pay_off + pay > rq.get_buffer()->get_data_length()) pay = 0;
        std::vector<uint8_t> e = eth_ipv4(q + 6, my_mac, 0, 64, 1, q + 14 + 16, q + 14 + 12, 8 + pay);
        e.push_back(0); e.push_back(0);  // TYPE_ECHO_REPLY, code 0
        put16(e, 0x0000);
        put_bytes(e, q + 14 + ihl + 4, 4);  // identifier and sequence number as they were
        put_bytes(e, q + pay_off, pay);
        s2.push_back(e);
        // Time Exceeded (11/0) and Destination Unreachable (3/0) from the engine's originals
        // (icmp_processor.cpp:255-327): the original IPv4 header and up to 8 bytes after it
        for (int k = 0; k < 2; ++k) {
            const netflow::Packet& o = *p1[3 * r + 1 + k];
            const uint8_t* g = o.get_buffer()->get_data_start_ptr();
            const size_t olen = o.get_buffer()->get_data_length();
            const size_t oihl = (size_t)(g[14] & 15u) * 4u;
            const size_t l4 = std::min<size_t>(8, olen > 14 + oihl ? olen - 14 - oihl : 0);
            std::vector<uint8_t> m = eth_ipv4(nh_mac, err_src_mac, (uint16_t)(0x1234 + 2 * r + k), 64, 1, err_src_ip,
                                              g + 14 + 12, 8 + oihl + l4);
            m.push_back(k == 0 ? 11 : 3); m.push_back(0);
            put16(m, 0x0000);
            put16(m, 0x0000);
            put16(m, 0x0000);
            put_bytes(m, g + 14, oihl + l4);
            s2.push_back(m);
        }
    }
    stage(s2, b2, p2);

    // ReceiveEchoRequestAndSendReply's EXPECTs (icmp_processor_test.cpp:313-338) on the engine's reply
    for (size_t r = 0; r < reps && 3 * r < p2.size(); ++r) {
        const netflow::Packet& rp = *p2[3 * r];
        const netflow::EthernetHeader* eh = rp.ethernet();
        const netflow::IPv4Header* ih = rp.ipv4();
        const netflow::IcmpHeader* ch = rp.icmp();
        if (!eh || !ih || !ch) { ++failed; continue; }
        netflow::IpAddress mine, theirs;
        std::memcpy(&mine, my_ip, 4);
        std::memcpy(&theirs, reqs[r].req_ip, 4);
        failed += !(eh->dst_mac == netflow::MacAddress(req_mac));
        failed += !(eh->src_mac == netflow::MacAddress(my_mac));
        failed += ntohs(eh->ethertype) != netflow::ETHERTYPE_IPV4;
        failed += ih->src_ip != mine || ih->dst_ip != theirs || ih->protocol != netflow::IPPROTO_ICMP;
        failed += ch->type != netflow::IcmpHeader::TYPE_ECHO_REPLY || ch->code != 0;
        failed += ntohs(ch->identifier) != reqs[r].id || ntohs(ch->sequence_number) != reqs[r].seq;
        const size_t po = 14 + 20 + 8;
        const std::vector<uint8_t>& pl = reqs[r].payload;
        failed += rp.get_buffer()->get_data_length() < po + pl.size() ||
                  std::memcmp(rp.get_buffer()->get_data_start_ptr() + po, pl.data(), pl.size()) != 0;
        // the error messages carry type/code and the original header + 8 bytes
        for (int k = 0; k < 2; ++k) {
            const netflow::Packet& m = *p2[3 * r + 1 + k];
            const uint8_t* g = m.get_buffer()->get_data_start_ptr();
            const uint8_t* o = p1[3 * r + 1 + k]->get_buffer()->get_data_start_ptr();
            failed += g[34] != (k == 0 ? 11 : 3) || g[35] != 0;
            failed += m.get_buffer()->get_data_length() != 14 + 20 + 8 + 28 || std::memcmp(g + 42, o + 14, 28) != 0;
        }
    }
    std::printf("frames=%zu stages=2 mismatches=%zu expect_failed=%zu rc=%d\n", frames, bad, failed, rc);
    return bad || failed || rc ? 1 : 0;
}

// The single-packet CPU path against the reference's on one core: `n` IPv4/UDP frames of `len` bytes
// (random payload, stale checksums), each updated in place `reps` times by the reference's
// Packet::update_checksums() and by netflow_amd::Packet::update_checksums() (cpu_update.hpp), the
// two interleaved per pass so both see the same cache state; then the two arenas compared.
// Prints "frames=N len=L ref_ns=… engine_ns=… speedup=… mismatches=M" (ns per packet).
int cpubench_mode(size_t len, size_t n, size_t reps) {
    if (len < 42) len = 42;
    uint64_t x = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint8_t)x; };
    std::vector<std::unique_ptr<netflow::PacketBuffer>> rb;
    std::vector<std::unique_ptr<netflow::Packet>> rp;
    std::vector<std::unique_ptr<netflow_amd::PacketBuffer>> mb;
    std::vector<std::unique_ptr<netflow_amd::Packet>> mp;
    for (size_t i = 0; i < n; ++i) {
        std::vector<uint8_t> f(len);
        for (auto& b : f) b = rnd();
        f[12] = 0x08; f[13] = 0x00; f[14] = 0x45; f[15] = 0;
        f[16] = (uint8_t)((len - 14) >> 8); f[17] = (uint8_t)(len - 14);
        f[22] = 64; f[23] = 17;
        f[38] = (uint8_t)((len - 34) >> 8); f[39] = (uint8_t)(len - 34);
        rb.push_back(ref_buffer(f, len));
        rp.emplace_back(new netflow::Packet(rb.back().get()));
        mb.emplace_back(new netflow_amd::PacketBuffer(kHeadroom + len, kHeadroom, len));
        std::memcpy(mb.back()->get_data_start_ptr(), f.data(), len);
        mp.emplace_back(new netflow_amd::Packet(mb.back().get()));
    }
    double t_ref = 0, t_eng = 0;
    for (size_t r = 0; r < reps; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < n; ++i) rp[i]->update_checksums();
        auto t1 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < n; ++i) mp[i]->update_checksums();
        auto t2 = std::chrono::steady_clock::now();
        t_ref += std::chrono::duration<double>(t1 - t0).count();
        t_eng += std::chrono::duration<double>(t2 - t1).count();
    }
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i)
        bad += std::memcmp(rb[i]->get_data_start_ptr(), mb[i]->get_data_start_ptr(), len) != 0;
    const double k = 1e9 / (double)(n * reps);
    std::printf("frames=%zu len=%zu ref_ns=%.1f engine_ns=%.1f speedup=%.2f mismatches=%zu\n", n, len, t_ref * k,
                t_eng * k, t_ref / t_eng, bad);
    return bad ? 1 : 0;
}

// The reference's own call convention, end to end: n BASELINE C1 frames (the
// seeded generator, nfcs_gen_config_device) in n separately allocated netflow::PacketBuffers — one
// `new[]` each, 32 bytes of headroom, as BufferPool::allocate_buffer hands them out
// (packet_buffer.hpp:21-31, buffer_pool.hpp:57-94) — checksummed as one burst of netflow::Packet* by
// netflow_amd::update_checksums_batch (netflow_adapter.hpp: frames gathered into the pinned ring, H2D,
// GPU, checksum bytes written back in place; what a caller of switch.hpp:294 that batches its burst
// runs); the same frames in netflow_amd::BufferPool slots of one pinned arena (no gather); and the
// reference's per-packet Packet::update_checksums() over the same PacketBuffers on 1 and on `threads`
// host threads. Wall clock per call, frames restored before each; best and median of `reps`. Each
// result's order-independent digest is compared with `want` (the reference's digest
// of C1, tests/golden/configs.json). Prints one JSON line.
int adapterbench_mode(size_t n, size_t reps, size_t threads, const std::string& want) {
    using clk = std::chrono::steady_clock;
    if (threads < 1) threads = 1;
    int rc = NFCS_OK;
    netflow_amd::ChecksumEngine* eng = netflow_amd::ChecksumEngine::try_instance(&rc);
    if (!eng) {
        std::printf("{\"error\": \"no engine: %s\"}\n", nfcs_strerror(rc));
        return 1;
    }
    nfcs_ctx* c = eng->ctx();
    // the frames: BASELINE C1, 16-byte aligned back to back, generated on the device
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

    auto parallel = [&](size_t k, const std::function<void(size_t, size_t)>& f) {  // f(i0, i1) over k threads
        std::vector<std::thread> th;
        for (size_t t = 1; t < k; ++t) th.emplace_back(f, n * t / k, n * (t + 1) / k);
        f(0, n / k);
        for (auto& x : th) x.join();
    };
    // digest of the frames as they are now in their buffers: gathered into the generator's layout
    std::vector<uint8_t> img(bytes);
    auto digest = [&](const std::function<const uint8_t*(size_t)>& data) -> std::string {
        parallel(threads, [&](size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; ++i) std::memcpy(img.data() + (size_t)desc[i].off16 * 16, data(i), desc[i].len);
        });
        uint64_t d = 0;
        if (nfcs_memcpy_h2d(c, d_arena, img.data(), bytes) ||
            nfcs_digest_device(c, (uint8_t*)d_arena, bytes, (nfcs_desc*)d_desc, (uint32_t)n, 0, &d, nullptr))
            return "error";
        char s[32];
        std::snprintf(s, sizeof(s), "%016llx", (unsigned long long)d);
        return s;
    };
    struct Timing { std::vector<double> s; std::string digest; };
    auto stats = [&](const Timing& t) {
        std::vector<double> v = t.s;
        std::sort(v.begin(), v.end());
        char o[320];
        std::snprintf(o, sizeof(o), "{\"GBps\": %.2f, \"GBps_median\": %.2f, \"ms_per_call\": %.3f, \"digest\": \"%s\", \"match\": %s}",
                      frame_bytes / v[0] / 1e9, frame_bytes / v[v.size() / 2] / 1e9, v[0] * 1e3, t.digest.c_str(),
                      t.digest == want ? "true" : "false");
        return std::string(o);
    };

    // the reference's PacketBuffers and Packets, one heap buffer each
    std::vector<std::unique_ptr<netflow::PacketBuffer>> rb(n);
    std::vector<std::unique_ptr<netflow::Packet>> rp(n);
    std::vector<netflow::Packet*> ptrs(n);
    for (size_t i = 0; i < n; ++i) {
        rb[i].reset(new netflow::PacketBuffer(kHeadroom + 1536, kHeadroom, desc[i].len));
        rp[i].reset(new netflow::Packet(rb[i].get()));
        ptrs[i] = rp[i].get();
    }
    auto restore_ref = [&] {
        parallel(threads, [&](size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; ++i)
                std::memcpy(rb[i]->get_data_start_ptr(), pristine.data() + (size_t)desc[i].off16 * 16, desc[i].len);
        });
    };
    auto ref_data = [&](size_t i) -> const uint8_t* { return rb[i]->get_data_start_ptr(); };
    auto time_reps = [&](const std::function<void()>& restore, const std::function<int()>& call, Timing& t) -> int {
        restore();
        int r = call();  // warm: staging ring, pinned buffers, code
        for (size_t k = 0; k < reps && r == NFCS_OK; ++k) {
            restore();
            const auto t0 = clk::now();
            r = call();
            t.s.push_back(std::chrono::duration<double>(clk::now() - t0).count());
        }
        return r;
    };

    Timing gpu, pool, pool_zc, pool_gather, ref1, refn;
    rc = time_reps(restore_ref, [&] { return netflow_amd::update_checksums_batch(ptrs.data(), n); }, gpu);
    if (rc) { std::printf("{\"error\": \"update_checksums_batch: %s\"}\n", nfcs_strerror(rc)); return 1; }
    gpu.digest = digest(ref_data);

    time_reps(restore_ref, [&] { for (size_t i = 0; i < n; ++i) ptrs[i]->update_checksums(); return 0; }, ref1);
    ref1.digest = digest(ref_data);
    time_reps(restore_ref, [&] {
        parallel(threads, [&](size_t i0, size_t i1) { for (size_t i = i0; i < i1; ++i) ptrs[i]->update_checksums(); });
        return 0;
    }, refn);
    refn.digest = digest(ref_data);
    rp.clear();  // the reference's Packets release their buffers' references first (packet.hpp:352-356)
    rb.clear();

    // the same frames in BufferPool slots (one pinned arena, 2176-byte slots, 32 bytes of headroom)
    {
        netflow_amd::BufferPool bp(n, 2176, *eng);
        std::vector<netflow_amd::PacketBuffer*> pb(n);
        std::vector<std::unique_ptr<netflow_amd::Packet>> pp(n);
        std::vector<netflow_amd::Packet*> pptr(n);
        for (size_t i = 0; i < n; ++i) {
            pb[i] = bp.allocate_buffer(desc[i].len);
            pb[i]->set_data_len(desc[i].len);
            pp[i].reset(new netflow_amd::Packet(pb[i]));
            pptr[i] = pp[i].get();
        }
        auto restore_pool = [&] {
            parallel(threads, [&](size_t i0, size_t i1) {
                for (size_t i = i0; i < i1; ++i)
                    std::memcpy(pb[i]->get_data_start_ptr(), pristine.data() + (size_t)desc[i].off16 * 16, desc[i].len);
            });
        };
        auto pool_data = [&](size_t i) -> const uint8_t* { return pb[i]->get_data_start_ptr(); };
        rc = time_reps(restore_pool, [&] { return bp.update_checksums_batch(pptr.data(), n); }, pool);
        if (rc) { std::printf("{\"error\": \"BufferPool::update_checksums_batch: %s\"}\n", nfcs_strerror(rc)); return 1; }
        pool.digest = digest(pool_data);
        // the same pool buffers read by the kernel over PCIe in place (NFCS_HOST_ZERO_COPY), and
        // gathered by nfcs_update_host_frames (frame bytes only over PCIe, not the slots' gaps)
        rc = time_reps(restore_pool, [&] { return bp.update_checksums_batch(pptr.data(), n, nullptr, NFCS_HOST_ZERO_COPY); },
                       pool_zc);
        if (rc) { std::printf("{\"error\": \"zero-copy: %s\"}\n", nfcs_strerror(rc)); return 1; }
        pool_zc.digest = digest(pool_data);
        std::vector<uint8_t*> fp(n);
        std::vector<uint32_t> fl(n);
        for (size_t i = 0; i < n; ++i) {
            fp[i] = pb[i]->get_data_start_ptr();
            fl[i] = (uint32_t)desc[i].len;
        }
        rc = time_reps(restore_pool, [&] { return nfcs_update_host_frames(c, fp.data(), fl.data(), (uint32_t)n, nullptr, 0); },
                       pool_gather);
        if (rc) { std::printf("{\"error\": \"gather: %s\"}\n", nfcs_strerror(rc)); return 1; }
        pool_gather.digest = digest(pool_data);
        pp.clear();
        for (auto* b : pb) bp.free_buffer(b);
    }
    nfcs_device_free(c, d_arena);
    nfcs_device_free(c, d_desc);
    std::printf("{\"packets\": %zu, \"frame_bytes\": %.0f, \"reps\": %zu, \"threads\": %zu, \"reference_digest\": \"%s\", "
                "\"adapter\": %s, \"buffer_pool\": %s, \"buffer_pool_zero_copy\": %s, \"buffer_pool_gather\": %s, "
                "\"reference_1_thread\": %s, \"reference_threads\": %s}\n",
                n, frame_bytes, reps, threads, want.c_str(), stats(gpu).c_str(), stats(pool).c_str(),
                stats(pool_zc).c_str(), stats(pool_gather).c_str(), stats(ref1).c_str(), stats(refn).c_str());
    for (const Timing* t : {&gpu, &pool, &pool_zc, &pool_gather, &ref1, &refn})
        if (t->digest != want) return 1;
    return 0;
}

// The reference's per-packet calls spread over k threads the way a switch that splits its RX bursts
// over cores would: workers started once, spinning on a generation counter between bursts (a thread
// spawned per burst would cost more than a 256-packet burst's checksums).
class SpinPool {
public:
    explicit SpinPool(size_t k) : k_(std::max<size_t>(1, k)) {
        for (size_t t = 1; t < k_; ++t) th_.emplace_back([this, t] { loop(t); });
    }
    ~SpinPool() {
        quit_.store(true);
        gen_.fetch_add(1, std::memory_order_release);
        for (auto& x : th_) x.join();
    }
    // f(i0, i1) over [0, n), split into k contiguous slices; the caller runs slice 0
    void run(size_t n, const std::function<void(size_t, size_t)>& f) {
        f_ = &f;
        n_ = n;
        left_.store(k_ - 1, std::memory_order_relaxed);
        gen_.fetch_add(1, std::memory_order_release);
        f(0, n / k_);
        while (left_.load(std::memory_order_acquire)) __builtin_ia32_pause();
    }

private:
    void loop(size_t t) {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g;
            while ((g = gen_.load(std::memory_order_acquire)) == seen) __builtin_ia32_pause();
            seen = g;
            if (quit_.load()) return;
            (*f_)(n_ * t / k_, n_ * (t + 1) / k_);
            left_.fetch_sub(1, std::memory_order_release);
        }
    }
    size_t k_;
    std::vector<std::thread> th_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<size_t> left_{0};
    std::atomic<bool> quit_{false};
    const std::function<void(size_t, size_t)>* f_ = nullptr;
    size_t n_ = 0;
};

// The per-RX-burst operating point of INTEGRATION.md §2: a ring of `ring` BASELINE
// C1 frames (1500 B IPv4+UDP, the seeded generator) checksummed burst by burst, consecutive bursts of b
// packets walking the ring (wrapping), for every b in `sizes`, through
//   adapter      netflow_amd::update_checksums_batch over the reference's own netflow::Packet /
//                PacketBuffer objects (one `new[]` each; nfcs_update_host_frames: gather, H2D, GPU,
//                checksum bytes written back);
//   pinned_ring  nfcs_update_host over the same frames in one pinned arena, 1536-byte slots (a NIC
//                ring's DMA area; zero-copy up to 32 MiB, frames H2D and patch records back above), its
//                NFCS_HOST_ZERO_COPY form, and pageable_ring: the same ring in pageable memory (staged
//                by the copy threads);
//   buffer_pool  netflow_amd::BufferPool::update_checksums_batch over the frames in 2176-byte slots of
//                one pinned arena (netflow_amd::Packet, the mirror of the reference's classes);
//   reference_1_thread / reference_threads  the reference's per-packet Packet::update_checksums() over
//                the burst's PacketBuffers, on one thread (the switch's own loop, switch.hpp:213-294) and
//                on `threads` threads (a SpinPool).
// Each call is timed alone (steady clock); a leg runs for `seconds` and at least 20 calls; reported: the
// median and 10th percentile µs per call and GB/s of frames at the median. update_checksums() is
// idempotent, so calls over frames an earlier leg updated cost the same. Parity per path: from the
// pristine frames, every leg, then one more pass over the whole ring, then the ring's digest against
// `want` (the reference's digest of these frames, tests/golden/configs.json). Prints one JSON line.
int burstbench_mode(const std::vector<size_t>& sizes, size_t ring, double seconds, size_t threads,
                    const std::string& want) {
    using clk = std::chrono::steady_clock;
    int rc = NFCS_OK;
    netflow_amd::ChecksumEngine* eng = netflow_amd::ChecksumEngine::try_instance(&rc);
    if (!eng) {
        std::printf("{\"error\": \"no engine: %s\"}\n", nfcs_strerror(rc));
        return 1;
    }
    nfcs_ctx* c = eng->ctx();
    const size_t n = ring;
    std::vector<nfcs_desc> desc(n);
    uint64_t bytes = 0;
    if (nfcs_layout_config(NFCS_CFG_C1_1500B_UDP, 20250620ull, 0, (uint32_t)n, 128, desc.data(), &bytes)) return 1;
    void *d_arena = nullptr, *d_desc = nullptr, *h_ring = nullptr;
    if (nfcs_device_alloc(c, bytes, &d_arena) || nfcs_device_alloc(c, n * sizeof(nfcs_desc), &d_desc) ||
        nfcs_host_alloc(c, bytes, &h_ring))
        return 1;
    if (nfcs_memcpy_h2d(c, d_desc, desc.data(), n * sizeof(nfcs_desc))) return 1;
    if (nfcs_gen_config_device(c, NFCS_CFG_C1_1500B_UDP, 20250620ull, 0, (uint32_t)n, (uint8_t*)d_arena, bytes,
                               (nfcs_desc*)d_desc, nullptr) || nfcs_stream_sync(c, nullptr))
        return 1;
    std::vector<uint8_t> pristine(bytes);
    if (nfcs_memcpy_d2h(c, pristine.data(), d_arena, bytes)) return 1;
    uint8_t* pr = static_cast<uint8_t*>(h_ring);
    std::vector<uint8_t> pageable(bytes);  // the same ring in pageable memory (staged by the copy threads)
    SpinPool copier(std::max<size_t>(1, std::min<size_t>(threads, 8)));  // restores and digests only, untimed

    std::vector<std::unique_ptr<netflow::PacketBuffer>> rb(n);
    std::vector<std::unique_ptr<netflow::Packet>> rp(n);
    std::vector<netflow::Packet*> ptrs(n);
    for (size_t i = 0; i < n; ++i) {
        rb[i].reset(new netflow::PacketBuffer(kHeadroom + 1536, kHeadroom, desc[i].len));
        rp[i].reset(new netflow::Packet(rb[i].get()));
        ptrs[i] = rp[i].get();
    }
    auto frame = [&](size_t i) -> const uint8_t* { return pristine.data() + (size_t)desc[i].off16 * 16; };
    // netflow_amd::BufferPool slots of one pinned arena (2176-byte slots: the frames fill 69% of them)
    netflow_amd::BufferPool bp(n, 2176, *eng);
    std::vector<netflow_amd::PacketBuffer*> pb(n);
    std::vector<std::unique_ptr<netflow_amd::Packet>> pp(n);
    std::vector<netflow_amd::Packet*> pptr(n);
    for (size_t i = 0; i < n; ++i) {
        pb[i] = bp.allocate_buffer(desc[i].len);
        pb[i]->set_data_len(desc[i].len);
        pp[i].reset(new netflow_amd::Packet(pb[i]));
        pptr[i] = pp[i].get();
    }
    // arena kinds: 0 the reference's PacketBuffers, 1 the pinned ring, 2 the pageable ring, 3 the pool
    auto ring_of = [&](int kind) { return kind == 1 ? pr : pageable.data(); };
    auto data_of = [&](int kind, size_t i) -> uint8_t* {
        if (kind == 0) return rb[i]->get_data_start_ptr();
        if (kind == 3) return pb[i]->get_data_start_ptr();
        return ring_of(kind) + (size_t)desc[i].off16 * 16;
    };
    auto restore = [&](int kind) {
        copier.run(n, [&](size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; ++i) std::memcpy(data_of(kind, i), frame(i), desc[i].len);
        });
    };
    std::vector<uint8_t> img(bytes);
    auto digest = [&](int kind) -> std::string {
        const bool ring = kind == 1 || kind == 2;
        if (!ring)
            copier.run(n, [&](size_t i0, size_t i1) {
                for (size_t i = i0; i < i1; ++i)
                    std::memcpy(img.data() + (size_t)desc[i].off16 * 16, data_of(kind, i), desc[i].len);
            });
        uint64_t d = 0;
        if (nfcs_memcpy_h2d(c, d_arena, ring ? ring_of(kind) : img.data(), bytes) ||
            nfcs_digest_device(c, (uint8_t*)d_arena, bytes, (nfcs_desc*)d_desc, (uint32_t)n, 0, &d, nullptr))
            return "error";
        char s[32];
        std::snprintf(s, sizeof(s), "%016llx", (unsigned long long)d);
        return s;
    };
    double frame_len = desc[0].len;

    // one path: call(off, b) checksums packets [off, off + b) of the ring
    std::string out;
    bool all_match = true;
    auto path = [&](const char* name, int kind, const std::function<int(size_t, size_t)>& call) -> int {
        std::fprintf(stderr, "burstbench: %s\n", name);
        restore(kind);
        std::string legs;
        for (size_t b : sizes) {
            if (b == 0 || n % b) return NFCS_EINVAL;
            size_t off = 0;  // bursts of b packets at multiples of b: never past the ring's end
            std::vector<double> us;
            int r = call(off, b);  // warm: staging ring, pinned buffers, code, the workers
            off = (off + b) % n;
            const auto t_end = clk::now() + std::chrono::duration<double>(seconds);
            while (r == NFCS_OK && (us.size() < 20 || clk::now() < t_end)) {
                const auto t0 = clk::now();
                r = call(off, b);
                us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
                off = (off + b) % n;
            }
            if (r) return r;
            std::sort(us.begin(), us.end());
            const double med = us[us.size() / 2], p10 = us[us.size() / 10];
            char o[256];
            std::snprintf(o, sizeof(o), "%s\"%zu\": {\"us_per_call\": %.2f, \"us_p10\": %.2f, \"GBps\": %.3f, \"calls\": %zu}",
                          legs.empty() ? "" : ", ", b, med, p10, b * frame_len / (med * 1e-6) / 1e9, us.size());
            legs += o;
        }
        const size_t big = sizes.back();
        for (size_t k = 0; k < n / big; ++k) {  // one whole pass, untimed: every frame updated
            const int r = call(k * big, big);
            if (r) return r;
        }
        const std::string d = digest(kind);
        all_match = all_match && d == want;
        char o[160];
        std::snprintf(o, sizeof(o), "}, \"digest\": \"%s\", \"match\": %s}", d.c_str(), d == want ? "true" : "false");
        out += std::string(out.empty() ? "" : ", ") + "\"" + name + "\": {\"bursts\": {" + legs + o;
        return NFCS_OK;
    };

    rc = path("adapter", 0, [&](size_t off, size_t b) { return netflow_amd::update_checksums_batch(ptrs.data() + off, b); });
    if (!rc)
        rc = path("pinned_ring", 1, [&](size_t off, size_t b) {
            return nfcs_update_host(c, pr, bytes, desc.data() + off, (uint32_t)b, nullptr, 0);
        });
    if (!rc)
        rc = path("pinned_ring_zero_copy", 1, [&](size_t off, size_t b) {
            return nfcs_update_host(c, pr, bytes, desc.data() + off, (uint32_t)b, nullptr, NFCS_HOST_ZERO_COPY);
        });
    if (!rc)
        rc = path("pageable_ring", 2, [&](size_t off, size_t b) {
            return nfcs_update_host(c, pageable.data(), bytes, desc.data() + off, (uint32_t)b, nullptr, 0);
        });
    if (!rc)
        rc = path("buffer_pool", 3, [&](size_t off, size_t b) { return bp.update_checksums_batch(pptr.data() + off, b); });
    if (!rc)
        rc = path("reference_1_thread", 0, [&](size_t off, size_t b) {
            for (size_t i = off; i < off + b; ++i) ptrs[i]->update_checksums();
            return 0;
        });
    if (!rc) {
        SpinPool pool(threads);
        rc = path("reference_threads", 0, [&](size_t off, size_t b) {
            pool.run(b, [&](size_t i0, size_t i1) { for (size_t i = off + i0; i < off + i1; ++i) ptrs[i]->update_checksums(); });
            return 0;
        });
    }
    if (rc) {
        std::printf("{\"error\": \"%s\"}\n", nfcs_strerror(rc));
        return 1;
    }
    rp.clear();
    rb.clear();
    pp.clear();
    for (auto* b : pb) bp.free_buffer(b);
    nfcs_device_free(c, d_arena);
    nfcs_device_free(c, d_desc);
    nfcs_host_free(c, h_ring);
    std::printf("{\"ring_packets\": %zu, \"frame_bytes\": %.0f, \"threads\": %zu, \"seconds_per_leg\": %.2f, "
                "\"reference_digest\": \"%s\", %s}\n",
                n, frame_len, threads, seconds, want.c_str(), out.c_str());
    return all_match ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    if (mode == "burstbench") {  // burstbench [sizes ring seconds threads want]
        signal(SIGSEGV, [](int) {  // a host-side fault: its stack to stderr (diagnostics only)
            void* bt[64];
            backtrace_symbols_fd(bt, backtrace(bt, 64), 2);
            _exit(139);
        });
        std::vector<size_t> sizes;
        const std::string s = argc > 2 ? argv[2] : "64,256,1024,4096,16384,65536";
        for (size_t p = 0; p < s.size();) {
            const size_t q = s.find(',', p);
            sizes.push_back(std::stoul(s.substr(p, q == std::string::npos ? std::string::npos : q - p)));
            p = q == std::string::npos ? s.size() : q + 1;
        }
        return burstbench_mode(sizes, argc > 3 ? std::stoul(argv[3]) : (1u << 20), argc > 4 ? std::stod(argv[4]) : 0.4,
                               argc > 5 ? std::stoul(argv[5]) : 16, argc > 6 ? argv[6] : "");
    }
    if (mode == "adapterbench")
        return adapterbench_mode(argc > 2 ? std::stoul(argv[2]) : (1u << 20), argc > 3 ? std::stoul(argv[3]) : 3,
                                 argc > 4 ? std::stoul(argv[4]) : 16, argc > 5 ? argv[5] : "");
    if (mode == "cpubench")
        return cpubench_mode(argc > 2 ? std::stoul(argv[2]) : 1500, argc > 3 ? std::stoul(argv[3]) : 4096,
                             argc > 4 ? std::stoul(argv[4]) : 50);
    if (mode == "cpu") return cpu_mode();
    if (mode == "vcpu") return vcpu_mode();
    if (mode == "gpu") return gpu_mode();
    if (mode == "vgpu") return vgpu_mode();
    if (mode == "path-gpu") return path_mode(true);
    if (mode == "path-cpu") return path_mode(false);
    if (mode == "icmp-gpu") return icmp_mode(true);
    if (mode == "icmp-cpu") return icmp_mode(false);
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
}
