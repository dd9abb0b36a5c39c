// blockchain_simulator_main.cpp — the drop-in driver: blockchain-simulator.cc
// (startSimulator + main, :12-77) written against the bcsim facade.  The
// protocol, N and link parameters are command-line options instead of source
// edits (blockchain-simulator.cc:67,72; network-helper.cc:11,17,28).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/network_helper.hpp"

using namespace bcsim;

static int startSimulator(int N, uint32_t protocol, const std::string& rate, const std::string& delay,
                          int64_t app_delay_ns, bool fixed, int rounds, bool quiet, int spread_us) {
  NodeContainer nodes;
  nodes.Create(N);
  NetworkHelper networkHelper(N, protocol);
  PointToPointHelper pointToPoint;
  pointToPoint.SetDeviceAttribute("DataRate", rate);   // :23
  pointToPoint.SetChannelAttribute("Delay", delay);    // :24
  const int64_t base_ns = ParseTimeNs(delay);
  for (int i = 0; i < N; i++) {                         // :34-51 (j < i pairs)
    for (int j = 0; j < N && j != i; j++) {
      if (spread_us > 0)  // heterogeneous links: the helper's Delay attribute changed per link
        pointToPoint.SetChannelAttribute(
            "Delay", std::to_string(base_ns + 1000ll * ((i * 7 + j * 3) % (spread_us + 1))) + "ns");
      pointToPoint.Install(i, j);
      networkHelper.m_nodesConnectionsIps[i].push_back(j);
      networkHelper.m_nodesConnectionsIps[j].push_back(i);
    }
  }
  networkHelper.SetLinks(pointToPoint);
  bcsim_config& cfg = networkHelper.config();
  if (fixed) {
    cfg.delay_mode = BCSIM_DELAY_FIXED;
    cfg.app_delay_ns = app_delay_ns;
  }
  if (rounds > 0) cfg.pbft_rounds = rounds;
  if (protocol == BCSIM_RAFT && cfg.t_end_ns <= 0) cfg.t_end_ns = 20000000000ll;
  ApplicationContainer nodeApp = networkHelper.Install(nodes);
  nodeApp.Start(0);
  nodeApp.Stop(10000000000ll);                          // :55
  int rc = Simulator::Run();                            // :57
  if (rc) {
    std::fprintf(stderr, "bcsim: %s (%s)\n", bcsim_strerror(rc), bcsim_last_error_detail());
    return 1;
  }
  if (!quiet)
    for (const auto& r : Simulator::Current()->Trace())  // NS_LOG_INFO(msg) prints msg + newline
      std::printf("%s\n", FormatTraceLine(r, &cfg).c_str());
  bcsim_counters c = Simulator::Current()->Counters();
  std::printf("delivered=%llu echoes=%llu sends=%llu t_last_ns=%lld\n",
              static_cast<unsigned long long>(c.delivered_total), static_cast<unsigned long long>(c.echoes),
              static_cast<unsigned long long>(c.sends), static_cast<long long>(c.t_last_ns));
  Simulator::Destroy();                                 // :58
  return 0;
}

int main(int argc, char* argv[]) {
  int N = 8;                                            // :67
  uint32_t protocol = BCSIM_PBFT;
  std::string rate = "3Mbps", delay = "3ms";
  int64_t app_delay = 3000000;
  bool fixed = false, quiet = false;
  int rounds = 0, spread_us = 0;
  for (int k = 1; k < argc; ++k) {
    std::string a = argv[k];
    auto val = [&]() { return k + 1 < argc ? std::string(argv[++k]) : std::string(); };
    if (a == "--nodes") N = std::atoi(val().c_str());
    else if (a == "--protocol") {
      std::string p = val();
      protocol = p == "raft" ? BCSIM_RAFT : p == "paxos" ? BCSIM_PAXOS : p == "gossip" ? BCSIM_GOSSIP : BCSIM_PBFT;
    } else if (a == "--rate") rate = val();
    else if (a == "--delay") delay = val();
    else if (a == "--fixed-app-delay-ns") { fixed = true; app_delay = std::atoll(val().c_str()); }
    else if (a == "--rounds") rounds = std::atoi(val().c_str());
    else if (a == "--quiet") quiet = true;
    else if (a == "--delay-spread-us") spread_us = std::atoi(val().c_str());
    else {
      std::fprintf(stderr, "usage: %s [--nodes N] [--protocol pbft|raft|paxos|gossip] [--rate 3Mbps] [--delay 3ms]\n"
                           "          [--fixed-app-delay-ns NS] [--rounds R] [--quiet] [--delay-spread-us K]\n", argv[0]);
      return 2;
    }
  }
  return startSimulator(N, protocol, rate, delay, app_delay, fixed, rounds, quiet, spread_us);
}
