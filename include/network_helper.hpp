// network_helper.hpp — C++ host facade with the reference's configuration
// surface, lowered onto the C ABI in bcsim.h.
//
// Mirrors, name for name:
//   NetworkHelper(uint32_t)            network-helper/network-helper.h:17
//   m_nodesConnectionsIps              network-helper/network-helper.h:19
//   ApplicationContainer Install(...)  network-helper/network-helper.h:21
//   NodeContainer / PointToPointHelper / Simulator::Run / Destroy as used by
//   blockchain-simulator.cc:12-59.
// Node "addresses" are node ids (the reference only uses an Ipv4Address to
// look a peer's socket up); the peer order of m_nodesConnectionsIps[i] is the
// order the app iterates, exactly as in the reference.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "bcsim.h"

namespace bcsim {

using Ipv4Address = uint32_t;  // peer node id

class NodeContainer {
 public:
  void Create(uint32_t n) { n_ = n; }
  uint32_t GetN() const { return n_; }

 private:
  uint32_t n_ = 0;
};

// "3Mbps" / "3ms" style attribute strings (ns-3 DataRate / Time syntax subset)
uint64_t ParseDataRate(const std::string& s);
int64_t ParseTimeNs(const std::string& s);

class PointToPointHelper {
 public:
  void SetDeviceAttribute(const std::string& name, const std::string& value);
  void SetChannelAttribute(const std::string& name, const std::string& value);
  // one link i<->j; returns the link index (the device pair of the reference)
  uint32_t Install(uint32_t i, uint32_t j);
  uint64_t rate_bps() const { return rate_bps_; }
  int64_t delay_ns() const { return delay_ns_; }
  // per installed link: (i, j, delay)
  struct Link {
    uint32_t a, b;
    int64_t delay_ns;
  };
  const std::vector<Link>& links() const { return links_; }

 private:
  uint64_t rate_bps_ = 32768;     // ns-3 PointToPointNetDevice default "32768b/s"
  int64_t delay_ns_ = 0;          // PointToPointChannel default 0s
  std::vector<Link> links_;
};

class Simulation;  // owns a bcsim_sim

class ApplicationContainer {
 public:
  ApplicationContainer() = default;
  explicit ApplicationContainer(Simulation* sim) : sim_(sim) {}
  void Start(int64_t t_ns);  // only 0 is supported (all apps start together)
  void Stop(int64_t t_ns);
  Simulation* simulation() const { return sim_; }

 private:
  Simulation* sim_ = nullptr;
};

class NetworkHelper {
 public:
  // protocol replaces the compile-time edit of network-helper.cc:11,17,28
  explicit NetworkHelper(uint32_t totalNoNodes, uint32_t protocol = BCSIM_PBFT);
  ~NetworkHelper();
  NetworkHelper(const NetworkHelper&) = delete;
  NetworkHelper& operator=(const NetworkHelper&) = delete;

  std::map<uint32_t, std::vector<Ipv4Address>> m_nodesConnectionsIps;

  // engine configuration (defaults: reference values for the protocol)
  bcsim_config& config() { return cfg_; }
  // link parameters used by Install (set from the PointToPointHelper)
  void SetLinks(const PointToPointHelper& p2p);

  ApplicationContainer Install(const NodeContainer& c);

 private:
  bcsim_config cfg_{};
  int m_nodeNo;
  std::map<uint64_t, int64_t> link_delay_;  // (a,b) -> delay from SetLinks
  Simulation* sim_ = nullptr;
};

// The installed applications; the engine is created on the first Run so that
// ApplicationContainer::Start/Stop (called after Install in the reference,
// blockchain-simulator.cc:54-55) still configure it.
class Simulation {
 public:
  Simulation(const bcsim_config& cfg, std::vector<uint32_t> row, std::vector<uint32_t> col,
             std::vector<int64_t> prop)
      : cfg_(cfg), row_(std::move(row)), col_(std::move(col)), prop_(std::move(prop)) {}
  ~Simulation();
  bcsim_config& config() { return cfg_; }
  bcsim_sim* handle() const { return h_; }
  int Run(int64_t t_until_ns);  // returns a BCSIM_* code
  std::vector<bcsim_trace_rec> Trace() const;
  bcsim_counters Counters() const;

 private:
  bcsim_config cfg_;
  std::vector<uint32_t> row_, col_;
  std::vector<int64_t> prop_;
  bcsim_sim* h_ = nullptr;
};

// ns-3 style singletons over the most recently installed simulation
struct Simulator {
  static int Run();        // blockchain-simulator.cc:57
  static void Destroy();   // blockchain-simulator.cc:58
  static Simulation* Current();
  static void SetCurrent(Simulation* s);
};

// The reference's NS_LOG_INFO text of one trace record, byte for byte (pbft-node.cc:259,
// 278,387,408; raft-node.cc:122-123,212,246,249,342,362,399; paxos-node.cc:339,518): the
// original strings, GetSeconds() at the default ostream precision, embedded "\n" kept;
// NS_LOG adds the final newline.  cfg (may be NULL) supplies the encoding and the Raft
// proposal limit.  Same as bcsim_format_trace_line.
std::string FormatTraceLine(const bcsim_trace_rec& r, const bcsim_config* cfg = nullptr);

}  // namespace bcsim
