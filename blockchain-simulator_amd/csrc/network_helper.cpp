// network_helper.cpp — see include/network_helper.hpp.
#include "../../include/network_helper.hpp"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
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

// Simulator::Now().GetSeconds() streamed with the default ostream format (6 significant
// digits, trailing zeros dropped), as every NS_LOG_INFO line of the reference prints it
static std::string secs(int64_t t_ns) {
  std::ostringstream o;
  o << static_cast<double>(t_ns) / 1e9;
  return o.str();
}
// a uint8_t data[3] payload streamed as a C string (raft-node.cc:399, paxos-node.cc:518):
// data[0], intToChar(x), then the uninitialised data[2], read as NUL
static std::string payload2(int c0, int32_t x, uint32_t encoding) {
  std::string d(1, static_cast<char>(c0));
  int32_t c1 = x + '0';
  if (encoding == BCSIM_ENC_COMPAT) c1 = static_cast<int8_t>(static_cast<uint8_t>(c1));
  const char b = static_cast<char>(static_cast<uint8_t>(c1 & 0xFF));
  if (b != 0) d.push_back(b);
  return d;
}

std::string FormatTraceLine(const bcsim_trace_rec& r, const bcsim_config* cfg) {
  std::ostringstream o;
  const std::string t = secs(r.t_ns);
  const uint32_t enc = cfg ? cfg->encoding : BCSIM_ENC_EXTENDED;
  switch (r.kind) {
    case BCSIM_TR_PBFT_COMMIT:  // pbft-node.cc:259
      o << "node " << r.node << " 在视图 " << r.a << " 中完成了第 " << r.b << " 次提交, 时间为 " << t
        << "s, value is " << r.c << "\n";
      break;
    case BCSIM_TR_PBFT_BLOCK:  // pbft-node.cc:387
      o << "主节点 node" << r.node << "开始广播区块, 时间为" << t << "s\n";
      break;
    case BCSIM_TR_PBFT_STOP:  // pbft-node.cc:408
      o << " 已经发送了第 " << r.a << "个区块 at time: " << t << "s";
      break;
    case BCSIM_TR_PBFT_VIEW:  // pbft-node.cc:278 (a = v, b = leader)
      o << "view-change完成, 当前主节点为 " << r.b << "视图为 " << r.a;
      break;
    case BCSIM_TR_RAFT_ELECTION:  // raft-node.cc:399
      o << "node" << r.node << " start election: " << payload2('2', static_cast<int32_t>(r.node), enc)
        << " at time: " << t << "s";
      break;
    case BCSIM_TR_RAFT_LEADER:  // raft-node.cc:212
      o << "Node " << r.node << " become leader! at time " << t << "s";
      break;
    case BCSIM_TR_RAFT_BLOCK:  // raft-node.cc:246 (a = blockNum before the increment)
      o << "At time " << t << " leader处理完一个区块 " << r.a;
      break;
    case BCSIM_TR_RAFT_DONE:  // raft-node.cc:249
      o << "node" << r.node << " 已经处理完 " << r.a << "个区块 at time: " << t << "s";
      break;
    case BCSIM_TR_RAFT_PROPOSAL: {  // raft-node.cc:342, and :362 once round reaches the limit
      o << "广播区块: " << r.a << ", time: " << t << " s";
      const int32_t lim = cfg ? static_cast<int32_t>(cfg->raft_proposal_rounds) : 50;
      if (r.a + 1 == lim) o << "\n" << "node" << r.node << " 已经发送了 " << lim << "个区块 at time: " << t << "s";
      break;
    }
    case BCSIM_TR_RAFT_STOP:  // raft-node.cc:122-123 (two NS_LOG_INFO lines)
      o << "Blocks:" << r.a << " Rounds:" << r.b << "\n" << "At time " << t << " Stop";
      break;
    case BCSIM_TR_PAXOS_COMMIT:  // paxos-node.cc:339
      o << "CLIENT COMMIT SUCCESS\n   ##clinet ticket##: " << r.a << " id: " << r.node << " at time: " << t << "s";
      break;
    case BCSIM_TR_PAXOS_TICKET:  // paxos-node.cc:518
      o << "node" << r.node << " require_data: " << payload2('0', r.a, enc);
      break;
    case BCSIM_TR_GOSSIP_BLOCK:  // build extension (no reference line)
      o << "node" << r.node << " gossips block " << r.a << " at time: " << t << "s";
      break;
    case BCSIM_TR_GOSSIP_DELIVER:
      o << "node" << r.node << " received block " << r.a << " from node" << r.c << " after " << r.b
        << " hops at time: " << t << "s";
      break;
    default:
      o << "kind " << r.kind << " node " << r.node << " at time: " << t << "s a=" << r.a << " b=" << r.b
        << " c=" << r.c;
  }
  return o.str();
}

}  // namespace bcsim

extern "C" int bcsim_format_trace_line(const bcsim_trace_rec* r, const bcsim_config* cfg, char* buf, uint64_t cap,
                                       uint64_t* n_out) {
  if (!r) return BCSIM_E_INVAL;
  const std::string line = bcsim::FormatTraceLine(*r, cfg);
  if (n_out) *n_out = line.size();
  if (buf && cap) {
    const size_t n = std::min<size_t>(line.size(), cap - 1);
    std::memcpy(buf, line.data(), n);
    buf[n] = 0;
  }
  return BCSIM_OK;
}
