// network_helper.cpp — see include/network_helper.hpp.
#include "../../include/network_helper.hpp"

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

namespace bcsim {

static double parse_number(const std::string& s, size_t* pos) {
  size_t k = 0;
  while (k < s.size() && (std::isdigit(static_cast<unsigned char>(s[k])) || s[k] == '.' || s[k] == 'e' ||
                          s[k] == 'E' || s[k] == '-' || s[k] == '+')) {
    if ((s[k] == 'e' || s[k] == 'E') && (k + 1 >= s.size() || !std::isdigit(static_cast<unsigned char>(s[k + 1]))))
      break;
    ++k;
  }
  *pos = k;
  return std::strtod(s.substr(0, k).c_str(), nullptr);
}

uint64_t ParseDataRate(const std::string& s) {  // ns-3 DataRate strings
  size_t k = 0;
  const double v = parse_number(s, &k);
  const std::string u = s.substr(k);
  double mul = 1;
  if (u == "bps" || u == "b/s") mul = 1;
  else if (u == "kbps" || u == "kb/s") mul = 1e3;
  else if (u == "Mbps" || u == "Mb/s") mul = 1e6;
  else if (u == "Gbps" || u == "Gb/s") mul = 1e9;
  else if (u == "KiBps") mul = 8.0 * 1024;
  else if (u == "MiBps") mul = 8.0 * 1024 * 1024;
  else if (u == "kBps" || u == "KBps") mul = 8e3;
  else if (u == "MBps") mul = 8e6;
  else throw std::invalid_argument("unsupported DataRate unit: " + s);
  return static_cast<uint64_t>(v * mul + 0.5);
}

int64_t ParseTimeNs(const std::string& s) {  // ns-3 Time strings
  size_t k = 0;
  const double v = parse_number(s, &k);
  const std::string u = s.substr(k);
  double mul = 1e9;
  if (u == "s" || u.empty()) mul = 1e9;
  else if (u == "ms") mul = 1e6;
  else if (u == "us") mul = 1e3;
  else if (u == "ns") mul = 1;
  else throw std::invalid_argument("unsupported Time unit: " + s);
  return static_cast<int64_t>(v * mul + 0.5);
}

void PointToPointHelper::SetDeviceAttribute(const std::string& name, const std::string& value) {
  if (name == "DataRate") rate_bps_ = ParseDataRate(value);
}
void PointToPointHelper::SetChannelAttribute(const std::string& name, const std::string& value) {
  if (name == "Delay") delay_ns_ = ParseTimeNs(value);
}
uint32_t PointToPointHelper::Install(uint32_t i, uint32_t j) {
  links_.push_back({i, j, delay_ns_});
  return static_cast<uint32_t>(links_.size() - 1);
}

void ApplicationContainer::Start(int64_t t_ns) {
  if (t_ns != 0) throw std::invalid_argument("only Start(Seconds(0)) is supported");
}
void ApplicationContainer::Stop(int64_t t_ns) {
  if (sim_) sim_->config().stop_ns = t_ns;
}

NetworkHelper::NetworkHelper(uint32_t totalNoNodes, uint32_t protocol) : m_nodeNo(static_cast<int>(totalNoNodes)) {
  bcsim_config_default(&cfg_, protocol, totalNoNodes);
}

NetworkHelper::~NetworkHelper() {
  if (Simulator::Current() == sim_) Simulator::SetCurrent(nullptr);
  delete sim_;
}

void NetworkHelper::SetLinks(const PointToPointHelper& p2p) {
  cfg_.link_rate_bps = p2p.rate_bps();
  cfg_.link_delay_ns = p2p.delay_ns();
  for (const auto& l : p2p.links()) {
    link_delay_[(static_cast<uint64_t>(l.a) << 32) | l.b] = l.delay_ns;
    link_delay_[(static_cast<uint64_t>(l.b) << 32) | l.a] = l.delay_ns;
  }
}

ApplicationContainer NetworkHelper::Install(const NodeContainer& c) {  // network-helper.cc:21-37
  const uint32_t N = c.GetN();
  if (N != static_cast<uint32_t>(m_nodeNo)) throw std::invalid_argument("node count mismatch");
  std::vector<uint32_t> row(N + 1, 0), col;
  std::vector<int64_t> prop;
  for (uint32_t i = 0; i < N; ++i) {
    row[i] = static_cast<uint32_t>(col.size());
    auto it = m_nodesConnectionsIps.find(i);
    if (it == m_nodesConnectionsIps.end()) continue;
    for (Ipv4Address peer : it->second) {  // app->m_peersAddresses, iteration order kept
      col.push_back(peer);
      auto d = link_delay_.find((static_cast<uint64_t>(i) << 32) | peer);
      prop.push_back(d == link_delay_.end() ? cfg_.link_delay_ns : d->second);
    }
  }
  row[N] = static_cast<uint32_t>(col.size());
  delete sim_;
  sim_ = new Simulation(cfg_, std::move(row), std::move(col), std::move(prop));
  Simulator::SetCurrent(sim_);
  return ApplicationContainer(sim_);
}

Simulation::~Simulation() {
  if (h_) bcsim_destroy(h_);
}

int Simulation::Run(int64_t t_until_ns) {
  if (!h_) {
    int rc = bcsim_create(&cfg_, &h_);
    if (rc) return rc;
    rc = bcsim_set_topology_csr(h_, cfg_.n_nodes, row_.data(), col_.data(), prop_.data());
    if (rc) return rc;
  }
  return bcsim_run(h_, t_until_ns);
}

std::vector<bcsim_trace_rec> Simulation::Trace() const {
  std::vector<bcsim_trace_rec> out;
  if (!h_) return out;
  uint64_t n = 0;
  if (bcsim_read_trace(h_, nullptr, 0, &n)) return out;
  out.resize(n);
  bcsim_read_trace(h_, out.data(), n, &n);
  return out;
}

bcsim_counters Simulation::Counters() const {
  bcsim_counters c{};
  if (h_) bcsim_read_counters(h_, &c);
  return c;
}

static Simulation* g_current = nullptr;
Simulation* Simulator::Current() { return g_current; }
void Simulator::SetCurrent(Simulation* s) { g_current = s; }
int Simulator::Run() { return g_current ? g_current->Run(INT64_MAX) : BCSIM_E_STATE; }
void Simulator::Destroy() { g_current = nullptr; }

std::string FormatTraceLine(const bcsim_trace_rec& r) {
  char buf[256];
  const double t = static_cast<double>(r.t_ns) / 1e9;
  switch (r.kind) {
    case BCSIM_TR_PBFT_COMMIT:
      std::snprintf(buf, sizeof buf, "node %u in view %d committed #%d at %.9fs, value is %d", r.node, r.a, r.b, t, r.c);
      break;
    case BCSIM_TR_PBFT_BLOCK:
      std::snprintf(buf, sizeof buf, "leader node%u broadcasts block n=%d at %.9fs", r.node, r.a, t);
      break;
    case BCSIM_TR_PBFT_STOP:
      std::snprintf(buf, sizeof buf, " sent block %d at time: %.9fs (node %u stops)", r.a, t, r.node);
      break;
    case BCSIM_TR_PBFT_VIEW:
      std::snprintf(buf, sizeof buf, "view-change done, leader is %d view is %d", r.b, r.a);
      break;
    case BCSIM_TR_RAFT_ELECTION:
      std::snprintf(buf, sizeof buf, "node%u start election at time: %.9fs", r.node, t);
      break;
    case BCSIM_TR_RAFT_LEADER:
      std::snprintf(buf, sizeof buf, "Node %u become leader! at time %.9fs", r.node, t);
      break;
    case BCSIM_TR_RAFT_BLOCK:
      std::snprintf(buf, sizeof buf, "At time %.9f leader finished block %d", t, r.a);
      break;
    case BCSIM_TR_RAFT_DONE:
      std::snprintf(buf, sizeof buf, "node%u finished %d blocks at time: %.9fs", r.node, r.a, t);
      break;
    case BCSIM_TR_RAFT_PROPOSAL:
      std::snprintf(buf, sizeof buf, "broadcast block: %d, time: %.9f s", r.a, t);
      break;
    case BCSIM_TR_RAFT_STOP:
      std::snprintf(buf, sizeof buf, "Blocks:%d Rounds:%d / At time %.9f Stop", r.a, r.b, t);
      break;
    case BCSIM_TR_PAXOS_COMMIT:
      std::snprintf(buf, sizeof buf, "CLIENT COMMIT SUCCESS ##clinet ticket##: %d id: %u at time: %.9fs", r.a, r.node, t);
      break;
    case BCSIM_TR_PAXOS_TICKET:
      std::snprintf(buf, sizeof buf, "node%u require_ticket %d at %.9fs", r.node, r.a, t);
      break;
    case BCSIM_TR_GOSSIP_BLOCK:
      std::snprintf(buf, sizeof buf, "node%u gossips block %d at %.9fs", r.node, r.a, t);
      break;
    case BCSIM_TR_GOSSIP_DELIVER:
      std::snprintf(buf, sizeof buf, "node%u received block %d from node%d after %d hops at %.9fs", r.node, r.a, r.c,
                    r.b, t);
      break;
    default:
      std::snprintf(buf, sizeof buf, "kind %u node %u t=%.9f a=%d b=%d c=%d", r.kind, r.node, t, r.a, r.b, r.c);
  }
  return buf;
}

}  // namespace bcsim
