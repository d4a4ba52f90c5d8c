// netflow_amd/netflow_adapter.hpp — the GPU batch entry points over NetFlow++'s OWN types.
//
// A NetFlow++ caller holds netflow::Packet (include/netflow++/packet.hpp:344-357) over
// netflow::PacketBuffer (packet_buffer.hpp:10-111): the switch's transit forward
// (switch.hpp:279-294), the VLAN manager (vlan_manager.cpp:90,159,174), the ICMP processor
// (icmp_processor.cpp:180,336). Including this header in such a translation unit (with NetFlow++'s
// include/ on the include path, as its own sources have it) gives it the batched forms of the
// reference's per-packet calls on those very objects, run on the gfx950 engine through the C ABI
// (include/nfcs.h); no change to the Packet type:
//
//   reference, per packet                     here, per burst (std::vector<netflow::Packet*> or ptr + n)
//   pkt.update_checksums()  packet.hpp:722    netflow_amd::update_checksums_batch(pkts[, status])
//   pkt.push_vlan(v, p) / pkt.pop_vlan()      netflow_amd::vlan_batch(pkts, ops, ok[, status])
//        packet.hpp:655-720                   (ops[i] = NFCS_VLAN_PUSH_OP(v, p) / NFCS_VLAN_POP / NOP)
//   the switch's TTL--, MAC rewrite and       netflow_amd::l3_forward_batch(pkts, next_hop, table,
//   update_checksums() switch.hpp:279-294     table_n[, status])
//   extract_flow_key + hash_flow              netflow_amd::flow_keys_batch(pkts, keys[, hashes])
//        packet_classifier.cpp:12-108
//
// Every entry returns 0 or a negative NFCS_E* code and never throws (the reference's calls are
// void / bool and never throw); per-packet outcomes are the NFCS_ST_* status bytes. The bytes
// written into each PacketBuffer are the reference's, bit for bit. A VLAN edit changes the buffer's
// data length as push_vlan / pop_vlan do; the Packet's cached l2_header_size_ (packet.hpp:916) is
// not touched — every reference accessor recomputes it through ethernet() before use.
//
// Single packets stay where the reference has them: call pkt.update_checksums() on the CPU, as
// before. Link with -lnfcs (netflow_amd/libnfcs.so); the engine is the process-wide one on device 0
// unless one is passed (ChecksumEngine(device) per GPU for multi-GPU hosts).
#pragma once

#include <netflow++/packet.hpp>

#include <vector>

#include "netflow_amd/packet.hpp"

namespace netflow_amd {

// On the process-wide engine (device 0): NFCS_ENODEV instead of an exception when there is none.
inline int update_checksums_batch(netflow::Packet* const* pkts, size_t n, uint8_t* status = nullptr) {
    return detail::on_default_engine([&](ChecksumEngine& e) { return e.update_checksums_batch(pkts, n, status); });
}
inline int update_checksums_batch(const std::vector<netflow::Packet*>& pkts, uint8_t* status = nullptr) {
    return update_checksums_batch(pkts.data(), pkts.size(), status);
}
inline int vlan_batch(netflow::Packet* const* pkts, const uint32_t* ops, size_t n, bool* ok = nullptr,
                      uint8_t* status = nullptr) {
    return detail::on_default_engine([&](ChecksumEngine& e) { return e.vlan_batch(pkts, ops, n, ok, status); });
}
inline int vlan_batch(const std::vector<netflow::Packet*>& pkts, const uint32_t* ops, bool* ok = nullptr,
                      uint8_t* status = nullptr) {
    return vlan_batch(pkts.data(), ops, pkts.size(), ok, status);
}
inline int l3_forward_batch(netflow::Packet* const* pkts, const uint32_t* next_hop, size_t n,
                            const nfcs_nexthop* table, uint32_t table_n, uint8_t* status = nullptr) {
    return detail::on_default_engine(
        [&](ChecksumEngine& e) { return e.l3_forward_batch(pkts, next_hop, n, table, table_n, status); });
}
inline int l3_forward_batch(const std::vector<netflow::Packet*>& pkts, const uint32_t* next_hop,
                            const nfcs_nexthop* table, uint32_t table_n, uint8_t* status = nullptr) {
    return l3_forward_batch(pkts.data(), next_hop, pkts.size(), table, table_n, status);
}
inline int flow_keys_batch(netflow::Packet* const* pkts, size_t n, nfcs_flow_key* keys,
                           uint32_t* hashes = nullptr) {
    return detail::on_default_engine([&](ChecksumEngine& e) { return e.flow_keys_batch(pkts, n, keys, hashes); });
}
inline int flow_keys_batch(const std::vector<netflow::Packet*>& pkts, nfcs_flow_key* keys,
                           uint32_t* hashes = nullptr) {
    return flow_keys_batch(pkts.data(), pkts.size(), keys, hashes);
}

// On an engine of the caller's (another device; one engine per GPU, one host thread each).
inline int update_checksums_batch(ChecksumEngine& eng, netflow::Packet* const* pkts, size_t n,
                                  uint8_t* status = nullptr) {
    return eng.update_checksums_batch(pkts, n, status);
}

}  // namespace netflow_amd
