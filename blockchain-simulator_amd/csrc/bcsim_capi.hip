// bcsim_capi.hip — host orchestration of the windowed engine + the C ABI
// declared in include/bcsim.h.  One translation unit with the kernels.
#include "engine.hip"

#include <hip/hip_ext.h>

#include <chrono>
#include <cstdlib>

namespace bcsim {

static thread_local std::string g_detail;

#define HIPCHK(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      g_detail = std::string(#x) + ": " + hipGetErrorString(e_);                       \
      return BCSIM_E_HIP;                                                              \
    }                                                                                  \
  } while (0)

}  // namespace bcsim
#include "transport.h"
namespace bcsim {

static uint32_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return static_cast<uint32_t>(p);
}

// control block read back once per cell
struct Ctl {
  int32_t err;
  uint32_t trace_cnt, vlog_cnt, dreq_cnt, ov_cnt;
  int32_t dbg;
  long long scal[6];  // next_local, ov_min_cell, n_alive_ticks, next timer, min shipped cell, (pad)
  long long pred[4];  // k_next's prediction of the next window: valid, cell, lo, hi (engine.hip k_next)
  long long win[kWinWords];  // device-chained windows (engine.hip k_win): the chain's state after its last k_next
  // followed by bucket_cnt[B] and x_cnt[B]
};

struct Sim {
  bcsim_config cfg{};
  uint32_t N = 0, R = 0, NT = 0, E = 0, deg_max = 0, B = 0;
  std::vector<uint32_t> row, col, rev;
  std::vector<int64_t> prop;
  bool started = false;
  // the node-partitioned kernels (P > 1, or forced at one rank with BCSIM_PDES_KERNELS=1 under a
  // transport: the partitioned path, k_link_mesh<XR> -> exchange -> k_import, on one GPU)
  bool pdes = false;
  bool topo_ready = false;  // CSR set by bcsim_set_topology_csr, else the full mesh at first run
  int32_t err = 0;
  int64_t L = 0;
  int64_t t_done = 0;
  long long grouped_cell = -1;
  long long last_full = -1;  // last cell processed to its end (hi == ce)
  int64_t next_tick = INT64_MAX;  // PBFT
  bool start_pending = true;
  bool stop_pending = true;   // Application::Stop at cfg.stop_ns (if >= 0)
  hipStream_t stream = nullptr;
  KP kp{};
  KP* kp_dev = nullptr;  // device copy of kp passed to every kernel
  // PBFT, dense: kp with a doubled k_scan staging window, for launches of few nodes (the
  // leader's oversized cells: one window instead of several, occupancy is moot there)
  KP* kp_dev_big = nullptr;
  size_t lds_big = 0;
  std::vector<void*> allocs;
  // host mirrors
  Ctl* ctl_h = nullptr;  // pinned
  uint32_t* act_h = nullptr;  // pinned: the window's active-list lengths (k_scan, k_link); [4..5] LLONG_MAX
  uint32_t* bcnt_h = nullptr;
  uint32_t* xcnt_h = nullptr;
  void* ctl_d = nullptr;
  void* ctl_m = nullptr;  // host-mapped mirror of the control block (k_next writes it)
  uint32_t* act_m = nullptr;  // host-mapped mirror of the active-list lengths (k_active writes it)
  uint32_t mseq = 0;          // sequence number of the last k_active / k_next launch (mirror words)
  uint32_t next_seq = 0;      // ... of the last k_next
  uint32_t spec_seq = 0;      // ... of a speculative k_active not consumed yet (0: none)
  bool spec_on = false;       // speculative k_active behind k_next (BCSIM_SPEC=0: off)
  bool fuse_act = false;      // ... built by k_next itself (BCSIM_FUSE_ACT=1; measured slower: one workgroup)
  uint64_t spec_hits = 0;
  std::vector<uint32_t> bcnt;  // bucket counts (host view)
  std::vector<uint32_t> xcnt;  // extras counts (host view)
  int x_active = 0;            // extras of the grouped cell are in xgrp
  uint32_t bs_scan = 64, bs_link = 64;
  long long dbg_fail_cell = -1;  // test hook (BCSIM_DBG_FAIL_CELL): this rank fails at that cell
  long long dbg_dev_err = -1;  // test hook (BCSIM_DBG_DEV_ERR): a device error flag raised before that cell's k_next
  long long dbg_fail_import = -1;  // test hook (BCSIM_DBG_FAIL_IMPORT): ... after that cell's exchange
  bool sparse = false;
  uint32_t grid_scan = 0, grid_link = 0;  // k_scan / k_link workgroups (walking the active lists)
  uint32_t gossip_g = 0;  // dense gossip: lanes per node of k_gossip_scan (0 = generic k_scan only)
  bool gossip_link = false;
  bool mesh_link = false;  // full mesh, fixed delay: k_link_mesh first, k_link over list 3
  bool scan_fast = false;  // dense PBFT, fixed delay, reply slots: k_scan_pbft first, k_scan over list 2
  bool mesh_pf = true;     // k_link_mesh parks the node's link words in LDS first (BCSIM_MESH_PF=0: off)
  // one rank: k_link_mesh<TILE> leaves the simple nodes' edges to k_mesh_tile (BCSIM_MESH_TILE=0: off)
  // in launches of at least tile_min nodes (BCSIM_TILE_MIN)
  bool mesh_tile = false;
  uint32_t tile_min = 1, mesh_epoch = 0;
  // the list-2 overlap (BCSIM_L2_OVERLAP=0: off): k_scan_pbft's leftover nodes are scanned and
  // linked by the generic kernels on stream2 (parameter block kp_dev2: list 2, its own staging
  // area) while stream runs everyone else's link stage; joined before the link class ends
  bool l2_overlap = false;
  bool l2_all = false;  // ... in every window with a list 2, not only the few-node scans (BCSIM_L2_OVERLAP=1)
  uint32_t win_epoch = 0, l2_pending = 0;
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  KP* kp_dev2 = nullptr;
  // summary mode: a link stage of at most link_few senders and no scan in the window (the
  // leader's block windows) runs the looped generic kernel over list 1 alone -- one dispatch
  // instead of k_mesh_prep + k_mesh_row + the looped kernel (BCSIM_LINK_FEW=0: off)
  KP* kp_dev_l1 = nullptr;
  uint32_t link_few = 1;
  bool px_cap4 = false;  // sparse Paxos: k_paxos_link<4> (BCSIM_PX_CAP=4) instead of <kPxCap>
  bool gossip_frontier = true;  // dense gossip: k_gossip_cell over the window's frontier (BCSIM_GOSSIP_FRONTIER=0: all)
  uint32_t few_scan = 64;  // k_scan launches of at most this many nodes use kp_dev_big (BCSIM_FEW_SCAN)
  bool sum = false;  // heavy-wave record summaries (BCSIM_SUM=0: off)
  uint32_t row_split_max = 64;  // k_mesh_row: launches of at most this many senders split rows (BCSIM_ROW_SPLIT)
  // summary mode, opt-in (BCSIM_ACT_RB=0): the window's kernels sized on the device, no read-back
  // of k_active's list lengths (measured slower: 0.73 vs 0.53 ms per step)
  bool dev_sized = false;
  uint64_t idle_parts = 0;  // part cells cut by a run limit skipped as idle
  // device-chained windows (dense gossip, one rank; BCSIM_CHAIN=0: off): k_win decides up to
  // chain_k windows on the device per host sync
  bool chain_on = false;
  uint32_t chain_k = 4;
  uint32_t chain_l3_grid = 16;  // chained windows: the looped generic link grid (list 3 is almost always empty; BCSIM_CHAIN_L3)
  uint64_t chains = 0, chain_windows = 0, chain_fr_hits = 0;
  uint64_t host_syncs = 0;  // times the cell loop waited on the GPU (spins, stream syncs, blocking collectives)
  uint64_t link_few_windows = 0;  // windows linked by the generic kernel alone (link_few)
  double host_launch_us = 0, host_wait_us = 0;  // host time inside kernel launches / mirror waits
  uint64_t host_launches = 0;
  bool check_idle = false;
  uint64_t idle_checked = 0;  // idle parts verified by check_idle_part  // debug (BCSIM_CHECK_IDLE=1): k_active verifies every skipped idle part is empty
  uint32_t gossip_l3_grid = 256;  // dense gossip: workgroups of the looped list-3 link grid (BCSIM_GL3; x8)
  uint32_t rt_min = 0;     // summary mode: k_scan_rt takes windows of at least this many scanned nodes (BCSIM_RT_MIN)
  long long next_timer = LLONG_MIN;  // earliest node timer after the last cell (k_next), unknown at start
  bool paxos_fast = false;  // sparse Paxos: k_paxos_scan first (BCSIM_NO_PXFAST=1: off)  // dense gossip: k_gossip_link first (not the full mesh, fixed delay, infinite queues, 1 rank)
  uint32_t* seg_part = nullptr;  // multi-block segment scan partials
  long long next_local = LLONG_MAX, ov_min = LLONG_MAX;
  long long n_alive = 0;
  uint64_t cells = 0;
  uint64_t tag_zeroes = 0;  // bucket zeroings of the slot-tag invariant (zero_tag_buckets)
  std::vector<long long> zeroed_turn;  // per bucket: the ring turn after which it was last zeroed
  // timing
  double us[4] = {0, 0, 0, 0};
  uint64_t launches[4] = {0, 0, 0, 0};
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  std::vector<int> ev_class;
  size_t ev_used = 0;
  // hipExtLaunchKernel timing (BCSIM_EXT_EVENTS=0: marker packets): the pending start event of the
  // open class (recorded by its next launch on ev_start_stream), and the last launch's stop
  bool ext_events = true;
  hipEvent_t ev_start_pend = nullptr;
  hipStream_t ev_start_stream = nullptr;
  bool ev_stop_attach = false, ev_stop_done = false;
  // trace cache
  std::vector<bcsim_trace_rec> trace;
  bool trace_valid = false;
  int dev = 0;
  unsigned long long* trail_h = nullptr;  // checked builds: host view of breadcrumbs
  // multi-GPU node partition
  uint32_t P = 1, prank = 0, nlo = 0, nloc = 0;
  Xport* xp = nullptr;
  uint32_t* scnt_h = nullptr;  // host view of the per-rank send counts (control block)
  // node-partitioned over RCCL: the control words of the window's exchange on the device
  // ([2][P][kCtlWords] int64: this rank's, then the received ones; opt-in, BCSIM_CTL_DEV=1)
  int64_t* ctlw_d = nullptr;
  int64_t* ctlw_h = nullptr;  // pinned
  XRec* recvbuf = nullptr;
  uint64_t cap_recv = 0;
  uint32_t vsync = 0;          // v-log entries already exchanged
  long long next_cell = 0;     // node-partitioned: the next cell of the whole system, agreed by the
  bool next_known = false;     // last cell's control exchange (no separate all-reduce needed)
  uint64_t ctl_collectives = 0;  // collectives + host syncs of the cell loop (engine counters)
  uint64_t last_import = 0;      // records k_import placed at the last exchange
  int carry_err = 0;             // device control words: a failure found after k_ctl sent "fine"
  std::vector<int64_t> lead_w; // leader flags packed for the all-reduce
};

static bool sync_each();

static std::string trail_dump(const Sim& s) {
  std::string out;
  if (!s.trail_h) return out;
  int shown = 0;
  for (uint32_t g = 0; g < s.NT && shown < 64; ++g) {
    const unsigned long long v = s.trail_h[g];
    if (!v) continue;
    out += " [g" + std::to_string(g) + ":L" + std::to_string(v & 0xFFFFFFFFull) + "]";
    ++shown;
  }
  return out;
}

// k_scan dynamic LDS: akey u64 | asec u32 | arec Rec | acls u32 per staged arrival + timers
static size_t scan_lds_bytes(const KP& p) {
  return static_cast<size_t>(p.cap_arr) * (8 + 4 + 4) + p.cap_timers * sizeof(TimerEnt);
}
// k_link dynamic LDS: ecnt[deg+1] | eidx[cap_eidx]
static size_t link_lds_bytes(const KP& p) { return (static_cast<size_t>(p.deg_max) + 1 + p.cap_eidx) * 4; }
// k_link: at most this much dynamic LDS, so that two 512-lane workgroups share a CU
constexpr size_t kLinkLdsTarget = 72 * 1024;

template <typename T>
static int dalloc(Sim& s, T** p, size_t count) {
  if (count == 0) count = 1;
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, count * sizeof(T));
  if (e != hipSuccess) {
    g_detail = std::string("hipMalloc ") + std::to_string(count * sizeof(T)) + " bytes: " +
               hipGetErrorString(e);
    return BCSIM_E_NOMEM;
  }
  s.allocs.push_back(q);
  *p = (T*)q  /* (device pass: T may carry address space 1) */;
  return BCSIM_OK;
}

static int ev_begin(Sim& s, int cls) {
  if (s.ev_used == s.ev_pool.size()) {
    hipEvent_t a, b;
    // timing only: no system-scope fence (an L2 writeback + invalidate at every record cost
    // ~10 us of dispatch gap per event on the MI355X, the gossip step 20 %)
    HIPCHK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
    HIPCHK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
    s.ev_pool.push_back({a, b});
    s.ev_class.push_back(cls);
  }
  s.ev_class[s.ev_used] = cls;
  if (s.ext_events) {  // (recorded by the next launch's own dispatch: no marker packet)
    s.ev_start_pend = s.ev_pool[s.ev_used].first;
    s.ev_start_stream = s.stream;
  } else {
    HIPCHK(hipEventRecord(s.ev_pool[s.ev_used].first, s.stream));
  }
  return BCSIM_OK;
}
static int ev_end(Sim& s) {
  if (s.ev_start_pend) {  // (nothing was launched in between)
    HIPCHK(hipEventRecord(s.ev_start_pend, s.ev_start_stream));
    s.ev_start_pend = nullptr;
  }
  s.ev_stop_attach = false;
  if (s.ev_stop_done)
    s.ev_stop_done = false;  // (the last launch of the class recorded it)
  else
    HIPCHK(hipEventRecord(s.ev_pool[s.ev_used].second, s.stream));
  s.launches[s.ev_class[s.ev_used]]++;
  ++s.ev_used;
  return BCSIM_OK;
}
// (called with the stream drained -- or it drains it: the end-of-window read-back spins on the
// control mirror, which k_next writes before the stream's completion is signalled)
constexpr size_t kEvBatch = 256;  // timing events read back per batch
static int ev_collect(Sim& s) {
  if (s.ev_used) HIPCHK(hipStreamSynchronize(s.stream));
  for (size_t k = 0; k < s.ev_used; ++k) {
    if (s.ev_class[k] < 0) continue;  // (a chained window that did not run)
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, s.ev_pool[k].first, s.ev_pool[k].second));
    s.us[s.ev_class[k]] += 1000.0 * ms;
  }
  s.ev_used = 0;
  return BCSIM_OK;
}

static int mirror_wait(Sim& s, const uint32_t* w, uint32_t seq);  // (below, with readback)
static int readback_apply(Sim& s);
static int readback(Sim& s, bool after_next = false);

static int validate(const bcsim_config& c) {
  if (c.abi_version != BCSIM_ABI_VERSION) return BCSIM_E_INVAL;
  if (c.protocol > BCSIM_GOSSIP || c.n_nodes < 2 || c.link_rate_bps == 0) return BCSIM_E_INVAL;
  if (c.mtu < 68) return BCSIM_E_INVAL;
  if (c.queue_model > BCSIM_QUEUE_FQCODEL) return BCSIM_E_INVAL;
  if (c.queue_model == BCSIM_QUEUE_FQCODEL && (c.queue_dev_pkts == 0 || c.queue_dev_pkts > 4096)) return BCSIM_E_INVAL;
  if (c.queue_model == BCSIM_QUEUE_DROPTAIL && c.queue_dev_pkts + c.queue_disc_pkts == 0) return BCSIM_E_INVAL;
  if (c.delay_mode == BCSIM_DELAY_RANDOM && c.rng_mode == BCSIM_RNG_GLIBC) {
    // the global glibc stream is consumed at every send in event order; only
    // the oracle replays that serially
    return BCSIM_E_UNSUPPORTED;
  }
  return BCSIM_OK;
}

static int build_mesh(Sim& s) {
  if (static_cast<uint64_t>(s.N) * (s.N - 1) >= 0xFFFFFFFFull) {
    g_detail = "full mesh over 2^32 directed edges: pass a topology (bcsim_set_topology_csr)";
    return BCSIM_E_UNSUPPORTED;
  }
  s.row.assign(s.N + 1, 0);
  s.col.clear();
  s.col.reserve(static_cast<size_t>(s.N) * (s.N - 1));
  for (uint32_t i = 0; i < s.N; ++i) {  // blockchain-simulator.cc:34-51 peer order
    s.row[i] = static_cast<uint32_t>(s.col.size());
    for (uint32_t j = 0; j < s.N; ++j)
      if (j != i) s.col.push_back(j);
  }
  s.row[s.N] = static_cast<uint32_t>(s.col.size());
  s.prop.assign(s.col.size(), s.cfg.link_delay_ns);
  return BCSIM_OK;
}

static int build_rev(Sim& s) {
  const uint32_t E = s.row[s.N];
  s.rev.assign(E, kInvalid);
  std::vector<uint64_t> keys(E);
  std::vector<uint32_t> idx(E);
  for (uint32_t a = 0; a < s.N; ++a)
    for (uint32_t e = s.row[a]; e < s.row[a + 1]; ++e) {
      if (s.col[e] >= s.N || s.col[e] == a) return BCSIM_E_INVAL;
      // rows list peers in ascending id order (the reference's peer order,
      // blockchain-simulator.cc:34-51): a receiver's inbox row is then in
      // canonical origin order
      if (e > s.row[a] && s.col[e] <= s.col[e - 1]) {
        g_detail = "CSR rows must list peers in ascending id order";
        return BCSIM_E_INVAL;
      }
      keys[e] = (static_cast<uint64_t>(a) << 32) | s.col[e];
      idx[e] = e;
    }
  std::sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return keys[x] < keys[y]; });
  for (uint32_t k = 1; k < E; ++k)
    if (keys[idx[k]] == keys[idx[k - 1]]) return BCSIM_E_INVAL;  // duplicate edge
  for (uint32_t e = 0; e < E; ++e) {
    const uint64_t want = (static_cast<uint64_t>(keys[e] & 0xFFFFFFFFu) << 32) | (keys[e] >> 32);
    auto it = std::lower_bound(idx.begin(), idx.end(), want,
                               [&](uint32_t x, uint64_t v) { return keys[x] < v; });
    if (it == idx.end() || keys[*it] != want) return BCSIM_E_INVAL;  // asymmetric
    s.rev[e] = *it;
  }
  return BCSIM_OK;
}

// allocate + initialise device state (first run)
static int setup_device(Sim& s) {
  bcsim_config& c = s.cfg;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    g_detail = "no HIP device";
    return BCSIM_E_NODEVICE;
  }
  s.dev = static_cast<int>(c.device) % ndev;
  HIPCHK(hipSetDevice(s.dev));
  HIPCHK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  KP& p = s.kp;
  const uint32_t tr = c.time_round;
  p.N = s.N;
  p.R = s.R;
  p.NT = s.NT;
  p.E = s.E;
  p.protocol = c.protocol;
  p.delay_mode = c.delay_mode;
  p.rng_mode = c.rng_mode;
  p.encoding = c.encoding;
  p.echo = c.echo;
  p.deg_max = s.deg_max;
  {  // a regular topology with row[i] = i * degree: the dense-gossip kernels skip the row loads
    bool reg = s.deg_max > 0 && s.row.size() == static_cast<size_t>(s.N) + 1;
    for (uint32_t i = 0; reg && i <= s.N; ++i) reg = s.row[i] == static_cast<uint64_t>(i) * s.deg_max;
    p.deg_reg = reg ? s.deg_max : 0u;
    if (const char* e = std::getenv("BCSIM_NO_DEGREG"); e && *e == '1') p.deg_reg = 0;
  }
  p.app_delay = c.app_delay_ns;
  // message sizes
  uint32_t small = 3, big = 3;
  if (c.protocol == BCSIM_PBFT) {
    small = 4;  // Create<Packet>(data, 4)
    big = c.pbft_block_bytes;
    if (big == 0) {  // tx_size * (tx_speed / (1000 / (timeout * 1000))) pbft-node.cc:377-380
      const float tmo = c.pbft_timeout_s;
      const int num = static_cast<int>(1000 / (1000 / (tmo * 1000)));
      big = static_cast<uint32_t>(1000 * num);
    }
  } else if (c.protocol == BCSIM_RAFT) {
    big = c.raft_proposal_bytes;
    if (big == 0) {  // raft-node.cc:409 with tx_size 200, tx_speed 2000
      const float hb = c.raft_heartbeat_s;
      const int num = static_cast<int>(2000 / (1000 / (hb * 1000)));
      big = static_cast<uint32_t>(200 * num);
    }
  } else if (c.protocol == BCSIM_GOSSIP) {  // every gossip message carries the block
    big = c.pbft_block_bytes ? c.pbft_block_bytes : 50000;
    small = big;
  }
  const MsgTx ms = message_tx(small, c.mtu, c.link_rate_bps, tr);
  const MsgTx mb = message_tx(big, c.mtu, c.link_rate_bps, tr);
  p.tx_tot[0] = ms.total;
  p.tx_last[0] = ms.last;
  p.tx_tot[1] = mb.total;
  p.tx_last[1] = mb.last;
  const MsgTx* mt[2] = {&ms, &mb};
  for (int k = 0; k < 2; ++k) {  // DROPTAIL frame model: F frames, full fragments of equal time
    p.nfr[k] = mt[k]->frames;
    p.tx_full[k] = mt[k]->frames > 1 ? (mt[k]->total - mt[k]->last) / (mt[k]->frames - 1) : mt[k]->total;
  }
  p.qmodel = c.queue_model == BCSIM_QUEUE_DROPTAIL ? 1u : c.queue_model == BCSIM_QUEUE_FQCODEL ? 2u : 0u;
  {  // FQCODEL: ns-3 attribute defaults for 0
    const uint32_t frag = (c.mtu - 20) & ~7u;
    const uint32_t bytes[2] = {small, big};
    for (int k = 0; k < 2; ++k) {
      p.ip_full[k] = frag + 20;
      p.ip_last[k] = bytes[k] + 8 - frag * (p.nfr[k] - 1) + 20;
    }
    p.fq_limit = c.fq_limit_pkts ? c.fq_limit_pkts : 10240;
    p.fq_quantum = c.fq_quantum ? c.fq_quantum : c.mtu;
    p.fq_batch = c.fq_drop_batch ? c.fq_drop_batch : 64;
    p.fq_min_bytes = c.fq_min_bytes ? c.fq_min_bytes : 1500;
    p.fq_target_c = static_cast<uint32_t>(static_cast<uint64_t>(c.fq_target_ns > 0 ? c.fq_target_ns : 5000000) >> 10);
    p.fq_interval_c = static_cast<uint32_t>(static_cast<uint64_t>(c.fq_interval_ns > 0 ? c.fq_interval_ns : 100000000) >> 10);
    p.fq_devcap = c.queue_dev_pkts;
  }
  p.qcap_frames = c.queue_dev_pkts + c.queue_disc_pkts;
  p.cap_q = c.cap_queue_msgs ? c.cap_queue_msgs : 256;
  p.pbft_period = fsec_to_ns(c.pbft_timeout_s, tr);
  p.raft_hb = fsec_to_ns(c.raft_heartbeat_s, tr);
  p.raft_prop_delay = c.raft_proposal_delay_ns;
  p.stop_ns = c.stop_ns;
  p.pbft_rounds = c.pbft_rounds;
  p.pbft_seq_cap = c.pbft_seq_cap ? c.pbft_seq_cap : 1000;
  if (p.pbft_seq_cap >= (1u << 21)) {  // k_scan's class word holds the sequence index in 21 bits
    g_detail = "pbft_seq_cap must be < 2^21";
    return BCSIM_E_INVAL;
  }
  p.pbft_view_change = c.pbft_view_change;
  p.raft_blocks = c.raft_blocks;
  p.raft_prop_rounds = c.raft_proposal_rounds;
  p.paxos_proposers = c.paxos_proposers;
  p.seed = c.seed;
  int64_t pmin = INT64_MAX;
  for (int64_t v : s.prop) pmin = std::min(pmin, v);
  if (pmin < 0) return BCSIM_E_INVAL;
  s.L = pmin + ms.total;  // lookahead: nothing arrives sooner than this after its send
  if (p.qmodel == 2) {  // FQCODEL: a message is emitted when its last fragment enters the device
    int64_t fmin = std::min(ms.last, mb.last);  // queue, at most one frame before it arrives
    if (mb.frames > 1) fmin = std::min<int64_t>(fmin, p.tx_full[1]);
    if (ms.frames > 1) fmin = std::min<int64_t>(fmin, p.tx_full[0]);
    s.L = pmin + fmin;
  }
  // (L >= 2: the reciprocal ceil(2^64 / L) below wraps to 0 at L == 1; a 1 ns lookahead means a
  // zero propagation delay and a 1 ns frame, far outside anything the reference configures)
  if (s.L < 2 || s.L >= (1ll << 32)) {
    g_detail = "lookahead out of range (2 ns .. 2^32 ns)";
    return BCSIM_E_UNSUPPORTED;
  }
  if ((c.protocol == BCSIM_PBFT || c.protocol == BCSIM_GOSSIP) && p.pbft_period <= 0) return BCSIM_E_INVAL;
  p.L = s.L;
  // ceil(2^64 / L) (L >= 2, checked above)
  p.L_magic = static_cast<uint64_t>(~0ull / static_cast<uint64_t>(s.L)) + 1ull;
  // delay tables (float seconds -> ns), pbft-node.cc:68, raft-node.cc:65,71, paxos-node.cc:399
  std::vector<int64_t> dpb(3), drf(3), del(150), dpx(50);
  for (int k = 0; k < 3; ++k) {
    dpb[k] = fsec_to_ns(static_cast<float>((k * 1.0 + 3) / 1000), tr);
    drf[k] = fsec_to_ns(static_cast<float>(k * 1.0 / 1000), tr);
  }
  for (int k = 0; k < 150; ++k) del[k] = fsec_to_ns(static_cast<float>((k + 150) * 1.0 / 1000), tr);
  for (int k = 0; k < 50; ++k) dpx[k] = fsec_to_ns(static_cast<float>(k * 1.0 / 1000), tr);
  int64_t* tables = nullptr;
  int rc;
  if ((rc = dalloc(s, &tables, 256))) return rc;
  std::vector<int64_t> tab(256, 0);
  std::copy(dpb.begin(), dpb.end(), tab.begin());
  std::copy(drf.begin(), drf.end(), tab.begin() + 4);
  std::copy(del.begin(), del.end(), tab.begin() + 8);
  std::copy(dpx.begin(), dpx.end(), tab.begin() + 160);
  HIPCHK(hipMemcpy(tables, tab.data(), 256 * sizeof(int64_t), hipMemcpyHostToDevice));
  p.pbft_delay = (decltype(p.pbft_delay))(tables);
  p.raft_delay = (decltype(p.raft_delay))(tables + 4);
  p.raft_elec = (decltype(p.raft_elec))(tables + 8);
  p.paxos_delay = (decltype(p.paxos_delay))(tables + 160);
  p.jit_delay = (c.protocol == BCSIM_PBFT || c.protocol == BCSIM_GOSSIP) ? p.pbft_delay : c.protocol == BCSIM_RAFT ? p.raft_delay : p.paxos_delay;
  p.jit_mod = c.protocol == BCSIM_PAXOS ? 50 : 3;
  const int64_t* tab_jit = tab.data() + (p.jit_delay - tables);

  // topology
  uint32_t *row, *col, *rev;
  int64_t *prop, *prop_in;
  if ((rc = dalloc(s, &row, s.N + 1)) || (rc = dalloc(s, &col, s.E)) || (rc = dalloc(s, &rev, s.E)) ||
      (rc = dalloc(s, &prop, s.E)) || (rc = dalloc(s, &prop_in, s.E)))
    return rc;
  std::vector<int64_t> pin(s.E);
  int64_t dt_max = 0;
  for (uint32_t q = 0; q < s.E; ++q) {
    pin[q] = s.prop[s.rev[q]];  // arrival at in-slot q travelled edge rev[q]
    dt_max = std::max(dt_max, pin[q] + std::max(p.tx_last[0], p.tx_last[1]));
  }
  if (dt_max >= (1ll << 32)) {
    g_detail = "propagation + frame time must be < 2^32 ns";
    return BCSIM_E_UNSUPPORTED;
  }
  HIPCHK(hipMemcpy(row, s.row.data(), (s.N + 1) * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(col, s.col.data(), static_cast<size_t>(s.E) * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(rev, s.rev.data(), static_cast<size_t>(s.E) * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(prop, s.prop.data(), static_cast<size_t>(s.E) * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(prop_in, pin.data(), static_cast<size_t>(s.E) * 8, hipMemcpyHostToDevice));
  p.row = (decltype(p.row))(row);
  p.col = (decltype(p.col))(col);
  p.rev = (decltype(p.rev))(rev);
  p.prop = (decltype(p.prop))(prop);
  p.prop_in = (decltype(p.prop_in))(prop_in);
  p.prop_const = s.E ? s.prop[0] : 0;  // uniform links: k_link skips the per-edge loads
  for (uint32_t e = 1; e < s.E && p.prop_const >= 0; ++e)
    if (s.prop[e] != s.prop[0]) p.prop_const = -1;

  // capacities
  const uint64_t NT = s.NT;
  // k_scan stages up to cap_arr arrivals per window in LDS (32 B each); a
  // cell with more is split into windows, so cap_arr only bounds one instant
  p.cap_arr = static_cast<uint32_t>(std::min<uint64_t>(kScanMaxArr, next_pow2(std::max<uint64_t>(64, s.deg_max + 64))));
  if (const char* ca = std::getenv("BCSIM_CAP_ARR"); ca && *ca) {  // testing aid: smaller windows (>= 64)
    const uint32_t v = static_cast<uint32_t>(next_pow2(std::max<uint64_t>(64, std::strtoull(ca, nullptr, 0))));
    if (v < p.cap_arr) p.cap_arr = v;
  }
  if (s.deg_max >= (1u << (32 - kSlotShift))) {  // staged arrival ids carry the in-slot in 18 bits
    g_detail = "node degree above 2^18";
    return BCSIM_E_UNSUPPORTED;
  }
  if (p.cap_arr <= s.deg_max && s.deg_max >= kScanMaxArr) {
    g_detail = "node degree exceeds the k_scan LDS window";
    return BCSIM_E_UNSUPPORTED;
  }
  p.cap_timers = c.cap_timers_per_node ? c.cap_timers_per_node : 8;
  if (p.cap_timers > 64) p.cap_timers = 64;
  p.cap_ops = c.cap_ops_per_node ? c.cap_ops_per_node
                                 : static_cast<uint32_t>(std::max<uint64_t>(1024, 4ull * s.deg_max + 256));
  // engine layout: the dense per-edge state of every replica (8 buckets
  // of inbox slots, link word, reply slots) or the sparse list-only layout
  {
    const double dense_bytes = static_cast<double>(s.R) * s.E * (8.0 * sizeof(Rec) + 8.0 + kOpRing * 16.0);
    s.sparse = c.engine_mode == BCSIM_ENGINE_SPARSE || (c.engine_mode == BCSIM_ENGINE_AUTO && dense_bytes > 96e9);
  }
  p.sparse = s.sparse ? 1u : 0u;
  if (s.sparse && p.qmodel == 2) {
    g_detail = "the FQCODEL queue model needs the dense layout";
    return BCSIM_E_UNSUPPORTED;
  }
  p.n_heavy = s.N;
  p.cap_ops_light = p.cap_ops;
  s.bs_scan = static_cast<uint32_t>(std::min<uint64_t>(1024, std::max<uint64_t>(64, next_pow2(s.deg_max + 1))));
  // k_scan: two 512-lane workgroups per CU when their LDS fits (16 B per staged arrival):
  // 11 % faster than one 1024-lane group at N=4096
  if (s.bs_scan == 1024 && 2 * (scan_lds_bytes(p) + sizeof(ScanShared)) <= 160 * 1024) s.bs_scan = 512;
  // k_link: several smaller workgroups per CU (LDS sized to fit, below) overlap one another's
  // barrier phases: at N=4096 one 1024-lane group per CU was 15 % slower than two 512-lane
  // ones, and four 256-lane ones are another 4 % faster
  s.bs_link = std::min<uint32_t>(s.bs_scan, 256);
  // workgroup size caps (powers of two >= 64; tuning knobs, results do not depend on them)
  auto bs_cap = [](const char* name, uint32_t bs) {
    const char* v = std::getenv(name);
    const uint32_t cap = v ? static_cast<uint32_t>(std::atoi(v)) : 0;
    return (cap >= 64 && cap <= 1024 && (cap & (cap - 1)) == 0) ? std::min(bs, cap) : bs;
  };
  s.bs_scan = bs_cap("BCSIM_BS_SCAN", s.bs_scan);
  s.bs_link = bs_cap("BCSIM_BS_LINK", s.bs_link);
  if (p.qmodel != 0) s.bs_link = std::min<uint32_t>(s.bs_link, 256);  // (k_link<1|2>'s launch bound)
  if (c.protocol != BCSIM_PBFT) s.bs_scan = std::min<uint32_t>(s.bs_scan, 256);  // (k_scan's launch bound)
  {  // k_link dynamic LDS: as many workgroups per CU as 1024 lanes make (1024 / bs_link)
    const size_t target = std::max<size_t>(16 * 1024, kLinkLdsTarget * s.bs_link / 512 - (s.bs_link < 512 ? 4096 : 0));
    const size_t room = target / 4 > s.deg_max + 1 + 1024 ? target / 4 - (s.deg_max + 1) : 1024;
    p.cap_eidx = static_cast<uint32_t>(std::min<size_t>(p.cap_ops, room));
  }
  if (link_lds_bytes(p) > 150 * 1024) {
    g_detail = "node degree / op capacity exceed the LDS budget of k_link";
    return BCSIM_E_UNSUPPORTED;
  }
  // inbox ring: one 16-byte slot per (bucket, replica, edge); as many buckets
  // as ~8 GiB allows, 8..64
  // full mesh (blockchain-simulator.cc:34-51): records are staged sender-major
  // and moved to the receivers by the tiled transpose (k_transpose)
  bool mesh = s.E == static_cast<uint64_t>(s.N) * (s.N - 1) && s.N >= 2;
  for (uint32_t i = 0; mesh && i <= s.N; ++i) mesh = s.row[i] == static_cast<uint64_t>(i) * (s.N - 1);
  if (const char* nm = std::getenv("BCSIM_NO_MESH"); nm && *nm == '1') mesh = false;  // debugging aid
  p.mesh = mesh ? 1u : 0u;
  p.n_tiles = (s.N + kTile - 1) / kTile;
  const uint64_t per_bucket = s.sparse ? 0 : static_cast<uint64_t>(s.R) * s.E * sizeof(Rec);
  s.B = c.n_buckets ? c.n_buckets : 0;
  if (s.B == 0 && s.sparse) {  // list-only buckets: enough cells for the longest send-to-arrival delay
    int64_t dmax = c.delay_mode == BCSIM_DELAY_FIXED ? c.app_delay_ns : 0;
    for (uint32_t k = 0; k < p.jit_mod && c.delay_mode != BCSIM_DELAY_FIXED; ++k)
      dmax = std::max<int64_t>(dmax, tab_jit[k]);
    int64_t pmax = 0;
    for (int64_t v : s.prop) pmax = std::max(pmax, v);
    const uint64_t cells = static_cast<uint64_t>((dmax + std::max(p.tx_tot[0], p.tx_tot[1]) + pmax) / s.L) + 3;
    s.B = static_cast<uint32_t>(std::max<uint64_t>(8, std::min<uint64_t>(kMaxBuckets, cells)));
  }
  if (s.B == 0) {
    const uint64_t nb = per_bucket ? (8ull << 30) / per_bucket : kMaxBuckets;
    s.B = static_cast<uint32_t>(std::max<uint64_t>(8, std::min<uint64_t>(kMaxBuckets, nb)));
  }
  if (s.B < 2 || s.B > static_cast<uint32_t>(kMaxBuckets)) {
    g_detail = "n_buckets must be in [2, 64]";
    return BCSIM_E_INVAL;
  }
  p.n_buckets = s.B;
  uint64_t cap_x = c.cap_bucket_records;
  if (cap_x == 0) cap_x = s.sparse ? std::min<uint64_t>(1ull << 25, std::max<uint64_t>({65536, NT * 2, static_cast<uint64_t>(s.R) * s.E}))
                                   : std::max<uint64_t>({65536, NT * 8,
                                                         // jittered sends: several records per edge and cell
                                                         c.delay_mode == BCSIM_DELAY_RANDOM ? static_cast<uint64_t>(s.R) * s.E / 4 : 0});
  p.cap_x = static_cast<uint32_t>(std::min<uint64_t>(cap_x, 1ull << 26));
  p.cap_stage = static_cast<uint32_t>(2ull * s.deg_max + 256);  // k_link staging per workgroup
  if (s.sparse) {
    // hub-compact link state: Paxos on the full mesh (only proposers broadcast; every
    // reply and echo travels a proposer edge)
    const bool mesh_topo = s.E == static_cast<uint64_t>(s.N) * (s.N - 1);
    p.hubs = (c.protocol == BCSIM_PAXOS && mesh_topo && c.queue_model == BCSIM_QUEUE_INFINITE)
                 ? std::min<uint32_t>(c.paxos_proposers, s.N) : 0u;
    if (p.hubs) {  // proposers hold broadcast expansions and reply waves; acceptors a few ops
      p.n_heavy = p.hubs;
      p.cap_ops_light = std::min<uint32_t>(p.cap_ops, c.cap_ops_per_node ? p.cap_ops : 32);
      if (!c.cap_timers_per_node) p.cap_timers = 4;  // Paxos: the t=0 ticket timer only
    }

    // small workgroups over many nodes: k_scan windows of <= 512 arrivals (split by
    // time), 256 lanes; k_link_sparse has no per-edge LDS arrays
    if (c.delay_mode == BCSIM_DELAY_RANDOM) p.cap_arr = std::min<uint32_t>(p.cap_arr, 512);  // spread arrivals
    s.bs_scan = std::min<uint32_t>(s.bs_scan, 256);
    s.bs_link = 256;
  }
  p.cap_ov = static_cast<uint32_t>(std::min<uint64_t>(std::max<uint64_t>(1ull << 20, NT * 256), 1ull << 26));
  p.cap_trace = static_cast<uint32_t>(std::min<uint64_t>(1ull << 26, std::max<uint64_t>(1u << 20, NT * 256)));
  p.cap_vlog = 1u << 20;
  const bool glibc_draws = c.protocol == BCSIM_RAFT && c.rng_mode == BCSIM_RNG_GLIBC;
  p.cap_dreq = glibc_draws ? static_cast<uint32_t>(std::max<uint64_t>(4096, 4 * NT)) : 1;
  p.cap_E = static_cast<uint64_t>(s.R) * s.E;
  p.cap_inbox = s.sparse ? 1 : static_cast<uint64_t>(s.B) * s.R * s.E;
  p.cap_xbuf = static_cast<uint64_t>(s.B) * p.cap_x;

  // dynamic LDS above the 64 KiB default needs an explicit opt-in (160 KiB per CU on gfx950)
  {
    const size_t lds_scan = scan_lds_bytes(p);
    if (lds_scan + sizeof(ScanShared) > 160 * 1024) {
      g_detail = "k_scan LDS request too large";
      return BCSIM_E_UNSUPPORTED;
    }
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_PBFT, false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_PBFT, false, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_PBFT, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_RAFT, false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_RAFT, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_PAXOS, false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_PAXOS, true, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_PAXOS, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_GOSSIP, false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_GOSSIP, false, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_GOSSIP, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_scan)));
    for (const void* f : {reinterpret_cast<const void*>(k_link<false, false>), reinterpret_cast<const void*>(k_link<false, true>),
                          reinterpret_cast<const void*>(k_link<false, false, true>),
                          reinterpret_cast<const void*>(k_link<false, true, true>),
                          reinterpret_cast<const void*>(k_link<true, false>), reinterpret_cast<const void*>(k_link<true, true>),
                          reinterpret_cast<const void*>(k_link<2, false>), reinterpret_cast<const void*>(k_link<2, true>)})
      HIPCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(link_lds_bytes(p))));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_pbft_tick),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(s.N)));
  }
  if (c.protocol == BCSIM_PBFT && s.N > 60 * 1024) return BCSIM_E_UNSUPPORTED;  // k_pbft_tick: one LDS flag per node

  // node partition: rank prank owns [nlo, nlo + nloc) of every replica
  {
    const char* pk = std::getenv("BCSIM_PDES_KERNELS");
    s.pdes = s.P > 1 || (s.xp && pk && *pk == '1');
  }
  if (s.P > 1) {
    if (s.P > static_cast<uint32_t>(kMaxRanks) || s.N < s.P) return BCSIM_E_INVAL;
    if (c.protocol == BCSIM_RAFT && c.rng_mode == BCSIM_RNG_GLIBC) {
      g_detail = "Raft with the global glibc stream is single-GPU only (draws in global order)";
      return BCSIM_E_UNSUPPORTED;
    }
  }
  s.nlo = static_cast<uint32_t>(static_cast<uint64_t>(s.prank) * s.N / s.P);
  s.nloc = static_cast<uint32_t>(static_cast<uint64_t>(s.prank + 1) * s.N / s.P) - s.nlo;
  p.nlo = s.nlo;
  p.nloc = s.nloc;
  p.rank = s.prank;
  p.nranks = s.P;
  // rank-local per-edge state: the edges of this rank's rows
  p.e_lo = static_cast<uint32_t>(s.row[s.nlo]);
  p.E_loc = static_cast<uint64_t>(s.row[s.nlo + s.nloc]) - s.row[s.nlo];
  p.cap_inbox = s.sparse ? 1 : static_cast<uint64_t>(s.B) * s.R * p.E_loc;
  {
    std::vector<uint16_t> own(s.N);
    for (uint32_t r = 0; r < s.P; ++r)
      for (uint64_t i = static_cast<uint64_t>(r) * s.N / s.P; i < static_cast<uint64_t>(r + 1) * s.N / s.P; ++i)
        own[i] = static_cast<uint16_t>(r);
    uint16_t* own_d = nullptr;
    if ((rc = dalloc(s, &own_d, s.N))) return rc;
    HIPCHK(hipMemcpy(own_d, own.data(), s.N * 2ull, hipMemcpyHostToDevice));
    p.owner = (decltype(p.owner))(own_d);
    // per destination rank: at most one record per (local sender, remote
    // receiver) edge per cell, plus second records and broadcasts
    const uint64_t cs = std::max<uint64_t>(65536, 2ull * s.R * s.nloc * std::min<uint64_t>(s.deg_max, s.N) + 4096);
    p.cap_send = s.xp ? static_cast<uint32_t>(std::min<uint64_t>(cs, 1ull << 28)) : 1;
    s.cap_recv = static_cast<uint64_t>(p.cap_send) * s.P;
    uint8_t *la = nullptr, *ll = nullptr;
    if ((rc = dalloc(s, &p.sendbuf, static_cast<size_t>(p.cap_send) * s.P)) ||
        (rc = dalloc(s, &s.recvbuf, s.xp ? s.cap_recv : 1)) || (rc = dalloc(s, &la, NT + 8)) ||
        (rc = dalloc(s, &ll, NT + 8)))
      return rc;
    HIPCHK(hipMemset(la, 0, NT + 8));
    HIPCHK(hipMemset(ll, 0, NT + 8));
    p.lead_all = (decltype(p.lead_all))(la);
    p.lead_loc = (decltype(p.lead_loc))(ll);
    s.lead_w.assign((NT + 7) / 8, 0);
  }

  // state
  if ((rc = dalloc(s, &p.sub, NT)) || (rc = dalloc(s, &p.draws, NT))) return rc;
  if ((rc = dalloc(s, &p.leader, NT)) || (rc = dalloc(s, &p.block_num, NT)) ||
      (rc = dalloc(s, &p.tick_alive, NT)) || (rc = dalloc(s, &p.tick_sub, NT)) ||
      (rc = dalloc(s, &p.g_n, s.R)) || (rc = dalloc(s, &p.g_nround, s.R)))
    return rc;
  const size_t txn = c.protocol == BCSIM_PBFT ? NT * p.pbft_seq_cap : 1;
  const size_t gsn = c.protocol == BCSIM_GOSSIP ? NT * p.pbft_seq_cap : 1;
  if ((rc = dalloc(s, &p.gseen, gsn))) return rc;
  HIPCHK(hipMemset(p.gseen, 0, gsn));
  p.cap_txn = txn;
  if ((rc = dalloc(s, &p.tx_val, txn)) || (rc = dalloc(s, &p.tx_pv, txn)) || (rc = dalloc(s, &p.tx_cv, txn)))
    return rc;
  int32_t* ibuf = nullptr;
  const size_t nint = 14;
  if ((rc = dalloc(s, &ibuf, NT * nint))) return rc;
  p.is_leader = (decltype(p.is_leader))(ibuf);
  p.has_voted = (decltype(p.has_voted))(ibuf + NT);
  p.m_value = (decltype(p.m_value))(ibuf + 2 * NT);
  p.vote_s = (decltype(p.vote_s))(ibuf + 3 * NT);
  p.vote_f = (decltype(p.vote_f))(ibuf + 4 * NT);
  p.acv = (decltype(p.acv))(ibuf + 5 * NT);
  p.blockNum = (decltype(p.blockNum))(ibuf + 6 * NT);
  p.round = (decltype(p.round))(ibuf + 7 * NT);
  p.decree = (decltype(p.decree))(ibuf + 8 * NT);
  p.ticket = (decltype(p.ticket))(ibuf + 11 * NT);
  p.proposal = (decltype(p.proposal))(ibuf + 13 * NT);
  p.K = c.paxos_decrees ? c.paxos_decrees : 1;
  {  // Paxos acceptor state per decree (START initialises it)
    const size_t npx = c.protocol == BCSIM_PAXOS ? static_cast<size_t>(NT) * p.K * 4 : 4;
    if ((rc = dalloc(s, &p.px, npx))) return rc;
    HIPCHK(hipMemset(p.px, 0, npx * 4));
  }
  if ((rc = dalloc(s, &p.next_election, NT)) || (rc = dalloc(s, &p.next_heartbeat, NT))) return rc;
  const size_t n_ops_total = static_cast<size_t>(s.R) * (static_cast<size_t>(p.n_heavy) * p.cap_ops +
                                                         static_cast<size_t>(s.N - p.n_heavy) * p.cap_ops_light);
  if ((rc = dalloc(s, &p.timers, NT * p.cap_timers)) || (rc = dalloc(s, &p.ops, n_ops_total)) ||
      (rc = dalloc(s, &p.n_ops, NT)))
    return rc;
  if (!s.sparse && p.cap_eidx < p.cap_ops) {  // k_link index area of nodes with > cap_eidx due ops
    // (per workgroup; the looped grids of the list-2 overlap use rows [kLoopGrid, 2 kLoopGrid))
    const size_t rows = std::max<size_t>(static_cast<size_t>(s.R) * s.N, 2 * kLoopGrid);
    if ((rc = dalloc(s, &p.eidx_g, rows * p.cap_ops))) return rc;
  } else {
    p.eidx_g = nullptr;
  }
  // per-edge reply slots of main-slot arrivals (kOpRing cells) and implicit
  // echoes; slots off beyond a 16 GiB budget, both off with BCSIM_NO_SLOTS=1 (A/B aid)
  {
    const uint64_t ne = static_cast<uint64_t>(kOpRing) * s.R * p.E_loc;
    const char* ns = std::getenv("BCSIM_NO_SLOTS");
    const bool off = ns && *ns == '1';
    p.impl = (off || s.sparse) ? 0u : 1u;  // sparse: no slots, echoes listed by k_scan
    // dense gossip of degree <= 64: k_gossip_scan takes the simple nodes (BCSIM_NO_GFAST=1: off)
    const char* nf = std::getenv("BCSIM_NO_GFAST");
    s.gossip_g = (c.protocol == BCSIM_GOSSIP && p.impl && s.deg_max <= 64 && !(nf && *nf == '1'))
                     ? static_cast<uint32_t>(next_pow2(std::max<uint64_t>(1, s.deg_max))) : 0u;
    {
      const char* px = std::getenv("BCSIM_NO_PXFAST");
      s.paxos_fast = s.sparse && c.protocol == BCSIM_PAXOS && !(px && *px == '1');
    }
    s.gossip_link = s.gossip_g && !p.mesh && !s.pdes && c.delay_mode == BCSIM_DELAY_FIXED &&
                    c.queue_model == BCSIM_QUEUE_INFINITE;
    // full mesh, fixed app delay: k_link_mesh takes the nodes whose due ops are all broadcasts
    // (BCSIM_NO_MFAST=1: off)
    {
      const char* mf = std::getenv("BCSIM_NO_MFAST");
      s.mesh_link = p.mesh && !s.sparse && c.delay_mode == BCSIM_DELAY_FIXED &&
                    c.queue_model == BCSIM_QUEUE_INFINITE && !(mf && *mf == '1');
    }
    // PBFT replies with a fixed app delay < L (due in the arrival cell or the next)
    const bool on = ne * 16 <= (16ull << 30) && !off && !s.sparse && c.protocol == BCSIM_PBFT &&
                    c.delay_mode == BCSIM_DELAY_FIXED && c.app_delay_ns < s.L;
    p.cap_eslot = on ? ne : 1;
    {  // BCSIM_NO_SFAST=1: off (A/B aid)
      const char* sf = std::getenv("BCSIM_NO_SFAST");
      s.scan_fast = on && p.impl && s.deg_max <= kFastLanes * kFastRPL && !(sf && *sf == '1');
      // testing aid: BCSIM_FEW_SCAN=0 sends small launches (every launch of a small parity case)
      // through k_scan_pbft too
      if (const char* fs = std::getenv("BCSIM_FEW_SCAN"); fs && *fs) s.few_scan = static_cast<uint32_t>(std::atoi(fs));
      if (const char* gf = std::getenv("BCSIM_GOSSIP_FRONTIER"); gf && *gf == '0') s.gossip_frontier = false;
      if (const char* pf = std::getenv("BCSIM_MESH_PF"); pf && *pf == '0') s.mesh_pf = false;
      if (static_cast<size_t>(s.deg_max) * 8 > 64 * 1024) s.mesh_pf = false;  // (dynamic LDS without an opt-in)
    }
    if ((rc = dalloc(s, &p.eslot, p.cap_eslot)) || (rc = dalloc(s, &p.sflag, static_cast<size_t>(kOpRing) * NT)))
      return rc;
    HIPCHK(hipMemset(p.eslot, 0xFF, p.cap_eslot * 16));  // due t = -1: no live reply
    HIPCHK(hipMemset(p.sflag, 0, static_cast<size_t>(kOpRing) * NT));
    if (!on) p.eslot = nullptr;
    // k_scan_pbft -> k_link_mesh reply / echo descriptors (BCSIM_NO_DESC=1: off)
    const char* nd = std::getenv("BCSIM_NO_DESC");
    // (k_link_mesh applies pending echoes to its LDS-parked link words: the PF variant, which
    // the node-partitioned engine does not launch)
    p.desc = (s.scan_fast && s.mesh_link && s.mesh_pf && !s.pdes && s.deg_max <= 32 * kDescWords && !(nd && *nd == '1')) ? 1u : 0u;
    p.dwords = p.desc ? static_cast<uint32_t>((s.deg_max + 31) / 32) : 1u;
    const size_t nrb = p.desc ? static_cast<size_t>(kOpRing) * NT * p.dwords : 1;
    const size_t neb = p.desc ? static_cast<size_t>(NT) * kEDesc * p.dwords : 1;
    if ((rc = dalloc(s, &p.rdesc, p.desc ? static_cast<size_t>(kOpRing) * NT : 1)) || (rc = dalloc(s, &p.rbits, nrb)) ||
        (rc = dalloc(s, &p.edesc, p.desc ? static_cast<size_t>(NT) * kEDesc : 1)) || (rc = dalloc(s, &p.ebits, neb)) ||
        (rc = dalloc(s, &p.en, p.desc ? NT : 1)))
      return rc;
    HIPCHK(hipMemset(p.rdesc, 0xFF, (p.desc ? static_cast<size_t>(kOpRing) * NT : 1) * 16));  // due -1: sent
    HIPCHK(hipMemset(p.en, 0, p.desc ? NT : 1));
    // the tiled mesh link stage: one rank, degree <= 4096 (the descriptor bitmaps)
    {
      const char* mt = std::getenv("BCSIM_MESH_TILE");
      s.mesh_tile = s.mesh_link && s.mesh_pf && !s.pdes && s.deg_max <= 32 * kDescWords && !(mt && *mt == '0');
      if (const char* tm = std::getenv("BCSIM_TILE_MIN"); tm && *tm) s.tile_min = static_cast<uint32_t>(std::atoi(tm));
    }
    p.n_stiles = (s.N + kTS - 1) / kTS;
    const size_t njob = s.mesh_tile ? NT : 1;
    if ((rc = dalloc(s, &p.mjob, njob * 4)) || (rc = dalloc(s, &p.mbc, njob * kMeshBc * 2)) ||
        (rc = dalloc(s, &p.mtb, njob * p.n_tiles * 2)) || (rc = dalloc(s, &p.mte, njob * p.n_tiles * kEDesc)) ||
        (rc = dalloc(s, &p.mtile, s.mesh_tile ? static_cast<size_t>(s.R) * p.n_stiles : 1)))
      return rc;
    HIPCHK(hipMemset(p.mjob, 0, njob * 4 * 16));  // epoch 0: no job (launch epochs start at 1)
    HIPCHK(hipMemset(p.mtile, 0, (s.mesh_tile ? static_cast<size_t>(s.R) * p.n_stiles : 1) * 4));
    {
      const char* lo = std::getenv("BCSIM_L2_OVERLAP");
      const bool dbg = std::getenv("BCSIM_FDBG") || std::getenv("BCSIM_WGT") || sync_each();
      s.l2_overlap = s.mesh_tile && s.scan_fast && !dbg && !(lo && *lo == '0');
      // (the summary / k_scan_pbft windows' list 2 is the leader's few-us scan: the fork and join
      // cost more than the overlap wins there -- 0.49 vs 0.50-0.52 ms per step -- so by default
      // only the few-node windows (the leader's 8190-arrival scan beside the row stage) fork)
      s.l2_all = s.l2_overlap && lo && *lo == '1';
    }
    if ((rc = dalloc(s, &p.l2mark, s.l2_overlap ? NT : 1))) return rc;
    HIPCHK(hipMemset(p.l2mark, 0, (s.l2_overlap ? NT : 1) * 4));
    // heavy-wave record summaries: the tiled link stage writes them, k_scan_rt
    // reads them (BCSIM_SUM=0: off); 33 B per (bucket, receiver tile, sender) within 8 GB
    {
      const char* sm = std::getenv("BCSIM_SUM");
      const size_t nsum = static_cast<size_t>(s.B) * s.R * p.n_tiles * s.N;
      s.sum = s.mesh_tile && s.scan_fast && p.desc && !s.pdes && c.protocol == BCSIM_PBFT && p.prop_const >= 0 &&
              nsum * 33 <= (8ull << 30) && !(sm && *sm == '0');
      p.sum = s.sum ? 1u : 0u;
      if ((rc = dalloc(s, &p.msum, s.sum ? nsum * 2 : 1)) || (rc = dalloc(s, &p.xsum, s.sum ? nsum : 1)) ||
          (rc = dalloc(s, &p.rul, s.sum ? NT : 1)) || (rc = dalloc(s, &p.rex, s.sum ? static_cast<size_t>(NT) * p.n_tiles : 1)))
        return rc;
      HIPCHK(hipMemset(p.rul, 0, (s.sum ? NT : 1) * 8));  // (no row-uniform state: every word its own)
      HIPCHK(hipMemset(p.rex, 0, (s.sum ? static_cast<size_t>(NT) * p.n_tiles : 1) * 8));
      HIPCHK(hipMemset(p.msum, 0, (s.sum ? nsum * 2 : 1) * 16));
      HIPCHK(hipMemset(p.xsum, 0, s.sum ? nsum : 1));
      if (const char* rm = std::getenv("BCSIM_RT_MIN"); rm && *rm) s.rt_min = static_cast<uint32_t>(std::atoi(rm));
    }
    p.loop_list = 3;
  }
  const size_t n_link = p.hubs ? static_cast<size_t>(s.R) * (static_cast<size_t>(p.hubs) * (s.N - 1) +
                                                              static_cast<size_t>(s.N - p.hubs) * p.hubs)
                               : static_cast<size_t>(s.R) * p.E_loc;
  if ((rc = dalloc(s, &p.link, n_link))) return rc;
  {  // DROPTAIL link queues: ring of cap_q message entries per edge
    const size_t ne = p.qmodel ? static_cast<size_t>(s.R) * p.E_loc : 1;
    if (p.cap_q > 65535) {
      g_detail = "cap_queue_msgs must be < 65536";
      return BCSIM_E_INVAL;
    }
    if ((rc = dalloc(s, &p.qmeta, ne)) || (rc = dalloc(s, &p.qring, ne * (p.qmodel == 1 ? p.cap_q : 1)))) return rc;
    HIPCHK(hipMemset(p.qmeta, 0, ne * 8));
  }
  {  // FQCODEL link queues: header, device-queue ring, packet rings, message table per edge
    const bool fq = p.qmodel == 2;
    const size_t ne = fq ? static_cast<size_t>(s.R) * p.E_loc : 1;
    p.cap_fqm = c.cap_queue_msgs ? std::min<uint32_t>(c.cap_queue_msgs, kFqMaxMsgs) : kFqMaxMsgs;
    p.cap_fqm = (p.cap_fqm + 31) / 32 * 32;
    // per-flow packet rings.  A saturated link's disc holds up to MaxSize packets (the PBFT
    // leader's block links and the echo links back to it run at 2.7x capacity), so the edges
    // of the hub nodes -- PBFT / gossip node 0, the Paxos proposers -- get MaxSize + 1 packets
    // per flow; every other edge gets MaxSize + 1 (at most 4096) when that fits the link-state
    // budget (below), else the largest ring that does (>= 64).  A flow that outgrows its ring
    // fails the run (BCSIM_E_OVERFLOW), never drops silently.
    const uint32_t cap_hi = static_cast<uint32_t>(std::min<uint64_t>(p.fq_limit + 1ull, 65535));
    uint32_t cap_lo = static_cast<uint32_t>(std::min<uint64_t>(p.fq_limit + 1ull, 4096));
    auto hub = [&](uint32_t i) {
      return c.protocol == BCSIM_PAXOS ? i < p.paxos_proposers : (c.protocol == BCSIM_RAFT ? false : i == 0);
    };
    std::vector<uint64_t> poff(fq ? ne : 0);
    size_t n_hub = 0;
    if (fq)
      for (uint32_t i = p.nlo; i < p.nlo + s.nloc; ++i)
        for (uint32_t e = s.row[i]; e < s.row[i + 1]; ++e)
          if (hub(i) || hub(s.col[e])) ++n_hub;
    n_hub *= s.R;
    const double fixed_b = kFqH * 4.0 + p.fq_devcap * 8.0 + p.cap_fqm * 16.0 + 16.0 + 8.0 + 8.0;
    // (per rank: 150 GB or 60 % of the free device memory, divided among the ranks only when
    // they may share the GPU -- the host-callback transport; RCCL runs one rank per device)
    double dev_b = 150e9;
    if (fq) {
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) == hipSuccess) dev_b = std::min(dev_b, 0.6 * static_cast<double>(fr));
    }
    const uint32_t share = (s.P > 1 && s.xp && s.xp->shares_device()) ? s.P : 1u;
    const double budget = dev_b / share - static_cast<double>(n_hub) * 48.0 * cap_hi;
    if (fq && static_cast<double>(ne) * fixed_b + static_cast<double>(ne - n_hub) * 48.0 * cap_lo > budget) {
      const double fit = ((budget - static_cast<double>(ne) * fixed_b) / std::max<double>(1.0, static_cast<double>(ne - n_hub))) / 48.0;
      cap_lo = fit >= 64.0 ? static_cast<uint32_t>(std::min<double>(fit, cap_lo)) : 0u;
      if (cap_lo < 64) {
        g_detail = "FQCODEL link state exceeds its memory budget even with 64-packet flow rings";
        return BCSIM_E_UNSUPPORTED;
      }
    }
    size_t npk = 0;
    if (fq)
      for (uint32_t rep = 0; rep < s.R; ++rep)
        for (uint32_t i = p.nlo; i < p.nlo + s.nloc; ++i)
          for (uint32_t e = s.row[i]; e < s.row[i + 1]; ++e) {
            const uint32_t cap = (hub(i) || hub(s.col[e])) ? cap_hi : cap_lo;
            poff[static_cast<size_t>(rep) * p.E_loc + (e - p.e_lo)] = npk | (static_cast<uint64_t>(cap) << 48);
            npk += 3ull * cap;
          }
    p.cap_fqp = cap_lo;
    uint32_t* fqlnk = nullptr;
    const size_t nt = fq ? s.NT : 1;
    if ((rc = dalloc(s, &p.fqh, ne * kFqH)) || (rc = dalloc(s, &p.fqdev, fq ? ne * p.fq_devcap : 1)) ||
        (rc = dalloc(s, &p.fqpk, fq ? npk : 1)) || (rc = dalloc(s, &p.fqpoff, ne)) ||
        (rc = dalloc(s, &p.fqmsg, fq ? ne * p.cap_fqm : 1)) ||
        (rc = dalloc(s, &fqlnk, fq ? s.E : 1)) || (rc = dalloc(s, &p.fqport, ne)) || (rc = dalloc(s, &p.fqpeer, ne)) ||
        (rc = dalloc(s, &p.fqkey, ne)) || (rc = dalloc(s, &p.fqnport, nt)) || (rc = dalloc(s, &p.fqphant, nt)))
      return rc;
    p.fqlnk = (decltype(p.fqlnk))(fqlnk);
    p.fq_flows = c.fq_flows ? c.fq_flows : 1024;
    p.fq_pert = c.fq_perturbation;
    if (fq) {
      hipLaunchKernelGGL(k_fq_init, dim3(4096), dim3(256), 0, s.stream, p.fqh, p.fqkey, static_cast<uint64_t>(ne));
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(s.stream));
      const std::vector<uint32_t> lnk = fq_link_numbers(s.N, s.row, s.col, s.rev);
      HIPCHK(hipMemcpy(fqlnk, lnk.data(), s.E * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(const_cast<uint64_t*>(p.fqpoff), poff.data(), ne * 8, hipMemcpyHostToDevice));
      // sockets unbound (port 0), no first-send keys pending (all ones)
      HIPCHK(hipMemset(p.fqport, 0, ne * 4));
      HIPCHK(hipMemset(p.fqpeer, 0, ne * 4));
      HIPCHK(hipMemset(p.fqnport, 0, nt * 4));
      HIPCHK(hipMemset(p.fqphant, 0, nt * 4));
    }
  }
  // k_scan / k_link grids (multiples of 8: one list chunk per XCD).  Dense layout: one
  // workgroup per possible list entry (an inactive node's workgroup exits at once); sparse
  // layout: a fixed grid strides over lists of up to millions of gnodes
  {
    const uint64_t nl = (static_cast<uint64_t>(s.R) * s.nloc + 7) / 8 * 8;
    s.grid_scan = s.grid_link = static_cast<uint32_t>(s.sparse ? std::min<uint64_t>(nl, 4096) : nl);
  }
  const size_t n_rtile = p.mesh ? static_cast<size_t>(s.B) * s.R * p.n_tiles * kRtPad : 1;  // (one flag per 128-byte line)
  if ((rc = dalloc(s, &p.rtile, n_rtile))) return rc;
  if ((rc = dalloc(s, &p.bmin, s.B))) return rc;
  if ((rc = dalloc(s, &p.inbox, p.cap_inbox)) || (rc = dalloc(s, &p.iflag, static_cast<size_t>(s.B) * NT)) ||
      (rc = dalloc(s, &p.xbuf, p.cap_xbuf)) || (rc = dalloc(s, &p.xgrp, p.cap_x)) ||
      (rc = dalloc(s, &p.xstage, (static_cast<size_t>(s.grid_link) + (s.l2_overlap ? kLoopGrid : 0)) * p.cap_stage)) ||
      (rc = dalloc(s, &p.xmeta, (static_cast<size_t>(s.grid_link) + (s.l2_overlap ? kLoopGrid : 0)) * p.cap_stage)) ||
      (rc = dalloc(s, &p.ov, p.cap_ov)))
    return rc;
  // (dense layout: the overflow list is compacted at every rebin -- k_rebin / k_ov_back)
  if (!s.sparse) {
    if ((rc = dalloc(s, &p.ov_tmp, p.cap_ov)) || (rc = dalloc(s, &p.rb_n, 2))) return rc;
    HIPCHK(hipMemset((void*)p.rb_n, 0, 8));
  }
  // active lists of k_scan / k_link (k_active; emptied by k_next / k_pbft_tick)
  if ((rc = dalloc(s, &p.act, 4 * NT)) || (rc = dalloc(s, &p.act_n, 4))) return rc;
  HIPCHK(hipMemset(p.act_n, 0, 16));
  if ((rc = dalloc(s, &s.seg_part, (NT + kSegChunk - 1) / kSegChunk + 1))) return rc;
  if ((rc = dalloc(s, &p.seg_cnt, NT)) || (rc = dalloc(s, &p.seg_off, NT + 1)) ||
      (rc = dalloc(s, &p.cursor, NT)))
    return rc;
  if ((rc = dalloc(s, &p.trace, p.cap_trace)) || (rc = dalloc(s, &p.vlog, p.cap_vlog)) ||
      (rc = dalloc(s, &p.dreq, p.cap_dreq)))
    return rc;
  p.cnt_stripes = 64;  // per-workgroup counter stripes (engine.hip cnt_stripe), <= 32 MiB in total
  while (p.cnt_stripes > 1 && static_cast<uint64_t>(p.cnt_stripes) * s.R * CNT_N * 8 > (32ull << 20)) p.cnt_stripes >>= 1;
  if ((rc = dalloc(s, &p.counters, static_cast<size_t>(p.cnt_stripes) * s.R * CNT_N)) ||
      (rc = dalloc(s, &p.kstat, 8 * kKstStripes)))
    return rc;
  if ((rc = dalloc(s, &p.node_tnext, NT)) || (rc = dalloc(s, &p.node_onext, NT)) || (rc = dalloc(s, &p.eapp, NT)))
    return rc;
  // control block: Ctl + bucket counts + extras counts, contiguous for one read-back
  const size_t ctl_bytes = sizeof(Ctl) + 8ull * s.B + 4ull * kMaxRanks;
  char* ctl = nullptr;
  if ((rc = dalloc(s, &ctl, ctl_bytes))) return rc;
  s.ctl_d = ctl;
  Ctl* cd = reinterpret_cast<Ctl*>(ctl);
  p.err = (decltype(p.err))(&cd->err);
  p.dbg = (decltype(p.dbg))(&cd->dbg);
  p.trace_cnt = (decltype(p.trace_cnt))(&cd->trace_cnt);
  p.vlog_cnt = (decltype(p.vlog_cnt))(&cd->vlog_cnt);
  p.dreq_cnt = (decltype(p.dreq_cnt))(&cd->dreq_cnt);
  p.ov_cnt = (decltype(p.ov_cnt))(&cd->ov_cnt);
  p.scal = (decltype(p.scal))(cd->scal);
  p.pred = (decltype(p.pred))(cd->pred);
  p.win = (decltype(p.win))(cd->win);
  if ((rc = dalloc(s, &p.nxt_part, 2 * kNextBlocks)) || (rc = dalloc(s, &p.nxt_done, 1))) return rc;
  HIPCHK(hipMemset(p.nxt_done, 0, 4));
  if ((rc = dalloc(s, &p.rb_acc, 1)) || (rc = dalloc(s, &p.rb_done, 1))) return rc;
  {
    const long long mx = LLONG_MAX;
    HIPCHK(hipMemcpy((void*)p.rb_acc, &mx, 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemset((void*)p.rb_done, 0, 4));
  }
  p.bucket_cnt = (decltype(p.bucket_cnt))(reinterpret_cast<uint32_t*>(ctl + sizeof(Ctl)));
  p.x_cnt = p.bucket_cnt + s.B;
  p.send_cnt = p.x_cnt + s.B;
  HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&s.ctl_h), ctl_bytes));
#ifndef BCSIM_CHECKED
  {  // the control block's host-mapped mirror (k_next publishes it; BCSIM_CTL_MIRROR=0: off)
    const char* cm = std::getenv("BCSIM_CTL_MIRROR");
    if (!(cm && *cm == '0')) {
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&s.ctl_m), ctl_bytes + 4, hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(s.ctl_m, 0, ctl_bytes + 4);
      void* dm = nullptr;
      HIPCHK(hipHostGetDevicePointer(&dm, s.ctl_m, 0));
      p.ctl_mirror = reinterpret_cast<uint32_t*>(dm);
      p.ctl_words = static_cast<uint32_t>(ctl_bytes / 4);
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&s.act_m), 16, hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(s.act_m, 0, 16);
      HIPCHK(hipHostGetDevicePointer(&dm, s.act_m, 0));
      p.act_mirror = reinterpret_cast<uint32_t*>(dm);
      uint32_t* ad = nullptr;
      if ((rc = dalloc(s, &ad, 1))) return rc;
      HIPCHK(hipMemset(ad, 0, 4));
      p.act_done = (decltype(p.act_done))(ad);
    }
  }
#endif
  HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&s.act_h), 32));  // (+ a pinned LLONG_MAX word at [4])
  *reinterpret_cast<long long*>(s.act_h + 4) = LLONG_MAX;
  s.bcnt_h = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(s.ctl_h) + sizeof(Ctl));
  s.xcnt_h = s.bcnt_h + s.B;
  s.scnt_h = s.xcnt_h + s.B;
  if (s.xp && s.xp->device_ctl()) {
    const char* cd = std::getenv("BCSIM_CTL_DEV");
    if (cd && *cd == '1') {  // (opt-in: gossip --pdes1 measured 0.99 against 0.88 ms per step without)
      if ((rc = dalloc(s, &s.ctlw_d, 2ull * s.P * Xport::kCtlWords))) return rc;
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&s.ctlw_h), 2ull * s.P * Xport::kCtlWords * 8));
    }
  }

  // glibc stream tables
  const bool need_glibc = c.rng_mode == BCSIM_RNG_GLIBC &&
                          (c.protocol == BCSIM_RAFT || (c.protocol == BCSIM_PBFT && c.pbft_view_change));
  p.glibc_len = need_glibc ? (1u << 20) : 1;
  int32_t* gl = nullptr;
  if ((rc = dalloc(s, &gl, static_cast<size_t>(s.R) * p.glibc_len)) || (rc = dalloc(s, &p.glibc_pos, s.R)))
    return rc;
  p.glibc = (decltype(p.glibc))(gl);
  p.cap_glibc = static_cast<uint64_t>(s.R) * p.glibc_len;
  if (need_glibc) {
    if (s.R > 64) return BCSIM_E_UNSUPPORTED;
    for (uint32_t r = 0; r < s.R; ++r) {
      std::vector<int32_t> st = glibc_stream(static_cast<uint32_t>(c.seed + r), p.glibc_len);
      HIPCHK(hipMemcpy(gl + static_cast<size_t>(r) * p.glibc_len, st.data(), 4ull * p.glibc_len,
                       hipMemcpyHostToDevice));
    }
  }
  std::vector<uint32_t> gpos(s.R, c.protocol == BCSIM_RAFT ? s.N : 0);
  HIPCHK(hipMemcpy(p.glibc_pos, gpos.data(), 4ull * s.R, hipMemcpyHostToDevice));

  // zero / initial values
  HIPCHK(hipMemset(ibuf, 0, NT * nint * 4));
  std::vector<uint32_t> sub0(NT, 2);  // 0 = START, 1 = STOP
  HIPCHK(hipMemcpy(p.sub, sub0.data(), NT * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(p.draws, 0, NT * 8));
  HIPCHK(hipMemset(p.leader, 0, NT * 4));
  HIPCHK(hipMemset(p.block_num, 0, NT * 4));
  HIPCHK(hipMemset(p.tick_alive, 0, NT));
  HIPCHK(hipMemset(p.tick_sub, 0, NT * 4));
  HIPCHK(hipMemset(p.g_n, 0, s.R * 4));
  HIPCHK(hipMemset(p.g_nround, 0, s.R * 4));
  HIPCHK(hipMemset(p.tx_val, 0, txn * 4));
  HIPCHK(hipMemset(p.tx_pv, 0, txn * 4));
  HIPCHK(hipMemset(p.tx_cv, 0, txn * 4));
  HIPCHK(hipMemset(p.next_election, 0, NT * 4));
  HIPCHK(hipMemset(p.next_heartbeat, 0, NT * 4));
  HIPCHK(hipMemset(p.timers, 0, NT * p.cap_timers * sizeof(TimerEnt)));
  HIPCHK(hipMemset(p.n_ops, 0, NT * 4));
  {  // busy_until 0, no record yet (cell tag 0xFFFF)
    std::vector<uint64_t> l0(n_link, 0xFFFFull);
    HIPCHK(hipMemcpy(p.link, l0.data(), l0.size() * 8, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemset(p.inbox, 0, p.cap_inbox * sizeof(Rec)));
  HIPCHK(hipMemset(p.rtile, 0, n_rtile));
  HIPCHK(hipMemset(p.iflag, 0, static_cast<size_t>(s.B) * NT));
  {
    const std::vector<long long> none(s.B, LLONG_MAX);  // every bucket empty
    HIPCHK(hipMemcpy(p.bmin, none.data(), s.B * sizeof(long long), hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemset(p.seg_cnt, 0, NT * 4));
  HIPCHK(hipMemset(p.seg_off, 0, (NT + 1) * 4));
  HIPCHK(hipMemset(p.cursor, 0, NT * 4));
  HIPCHK(hipMemset(p.counters, 0, static_cast<size_t>(p.cnt_stripes) * s.R * CNT_N * 8));
  HIPCHK(hipMemset(p.kstat, 0, 64 * kKstStripes));
#ifdef BCSIM_CHECKED
  {
    const char* tv = std::getenv("BCSIM_TRAIL");
    if (tv && *tv && *tv != '0') {
      void* hp = nullptr;
      HIPCHK(hipHostMalloc(&hp, NT * 8, hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(hp, 0, NT * 8);
      void* dp = nullptr;
      HIPCHK(hipHostGetDevicePointer(&dp, hp, 0));
      s.trail_h = static_cast<unsigned long long*>(hp);
      p.trail = static_cast<unsigned long long*>(dp);
    }
  }
#endif
  if (const char* fv = std::getenv("BCSIM_FDBG"); fv && *fv == '1') {  // debug: fast-kernel leave reasons
    if ((rc = dalloc(s, &p.fdbg, 16))) return rc;
    HIPCHK(hipMemset(p.fdbg, 0, 16 * 8));
  }
  p.fqlog = nullptr;
  p.fqlog_n = nullptr;
  if (const char* fl = std::getenv("BCSIM_FQLOG"); fl && *fl && p.qmodel == 2) {  // debug: FQCODEL link events
    p.cap_fqlog = 1u << 22;
    const char* a = std::getenv("BCSIM_FQLOG_T0");
    const char* b = std::getenv("BCSIM_FQLOG_T1");
    p.fqlog_t0 = a ? std::atoll(a) : 0;
    p.fqlog_t1 = b ? std::atoll(b) : LLONG_MAX;
    if ((rc = dalloc(s, &p.fqlog, 2ull * p.cap_fqlog)) || (rc = dalloc(s, &p.fqlog_n, 1))) return rc;
    HIPCHK(hipMemset(p.fqlog_n, 0, 4));
  }
  if (const char* wv = std::getenv("BCSIM_WGT"); wv && *wv == '1') {  // debug: k_link per-WG timing
    if ((rc = dalloc(s, &p.wgt, NT * 8)) || (rc = dalloc(s, &p.wgs, NT * 8))) return rc;
    const size_t ntw = static_cast<size_t>(s.R) * p.n_stiles * p.n_tiles;
    if ((rc = dalloc(s, &p.wgtt, ntw * 8))) return rc;
    HIPCHK(hipMemset(p.wgtt, 0, ntw * 64));
    HIPCHK(hipMemset(p.wgt, 0, NT * 64));
    HIPCHK(hipMemset(p.wgs, 0, NT * 64));
  }
  p.dbg_tmax = LLONG_MIN;
  if (const char* xv = std::getenv("BCSIM_EXP"); xv && *xv) p.exp = static_cast<uint32_t>(std::strtol(xv, nullptr, 0));
  {
    const char* pf = std::getenv("BCSIM_PX_FAST");
    p.paxos_fast_win = (pf && *pf == '0') ? 0u : 1u;
  }
  if (const char* fv = std::getenv("BCSIM_DBG_FAIL_CELL"); fv && *fv) s.dbg_fail_cell = std::atoll(fv);
  if (const char* fv = std::getenv("BCSIM_DBG_FAIL_IMPORT"); fv && *fv) s.dbg_fail_import = std::atoll(fv);
  if (const char* fv = std::getenv("BCSIM_DBG_DEV_ERR"); fv && *fv) s.dbg_dev_err = std::atoll(fv);
  if (const char* rs = std::getenv("BCSIM_ROW_SPLIT"); rs && *rs) s.row_split_max = static_cast<uint32_t>(std::atoi(rs));
  if (const char* ab = std::getenv("BCSIM_ACT_RB"); ab && *ab == '0') s.dev_sized = true;
  if (const char* ci = std::getenv("BCSIM_CHECK_IDLE"); ci && *ci == '1') s.check_idle = true;
  if (const char* fa = std::getenv("BCSIM_FUSE_ACT"); fa && *fa == '1') s.fuse_act = true;
  if (const char* xe = std::getenv("BCSIM_EXT_EVENTS"); xe && *xe == '0') s.ext_events = false;
  if (const char* pc = std::getenv("BCSIM_PX_CAP"); pc && *pc == '4') s.px_cap4 = true;
  if (const char* cl = std::getenv("BCSIM_CHAIN_L3"); cl && *cl) s.chain_l3_grid = std::max<uint32_t>(8, static_cast<uint32_t>(std::atoi(cl)) / 8 * 8);
  if (const char* g3 = std::getenv("BCSIM_GL3"); g3 && *g3) s.gossip_l3_grid = std::max<uint32_t>(8, static_cast<uint32_t>(std::atoi(g3)) / 8 * 8);
  {
    const char* sp = std::getenv("BCSIM_SPEC");
    s.spec_on = !(sp && *sp == '0') && !s.sparse && !s.pdes && !s.xp && s.cfg.protocol == BCSIM_PBFT && s.act_m != nullptr &&
                s.ctl_m != nullptr;
  }
  if (const char* dv = std::getenv("BCSIM_DBG_EVENTS"); dv && *dv) p.dbg_tmax = std::atoll(dv);  // debug event log
  {
    const char* ch = std::getenv("BCSIM_CHAIN");
    s.chain_on = !(ch && *ch == '0') && s.gossip_link && s.gossip_frontier && !s.xp && !s.pdes && !s.sparse &&
                 s.kp.dbg_tmax == LLONG_MIN && s.dbg_fail_cell < 0 && s.dbg_dev_err < 0 &&
                 s.dbg_fail_import < 0;
  }
  std::vector<long long> big_ll(NT, LLONG_MAX);
  HIPCHK(hipMemcpy(p.node_tnext, big_ll.data(), NT * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(p.node_onext, big_ll.data(), NT * 8, hipMemcpyHostToDevice));
  {
    const std::vector<long long> never(NT, LLONG_MIN);
    HIPCHK(hipMemcpy(p.eapp, never.data(), NT * 8, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemset(s.ctl_d, 0, ctl_bytes));
  long long sc0[6] = {LLONG_MAX, LLONG_MAX, 0, 0, LLONG_MAX, 0};
  HIPCHK(hipMemcpy(p.scal, sc0, sizeof sc0, hipMemcpyHostToDevice));
  // counters' t_last slot starts at 0 (max)
  HIPCHK(hipDeviceSynchronize());
  if ((rc = dalloc(s, &s.kp_dev, 1))) return rc;
  HIPCHK(hipMemcpy(s.kp_dev, &s.kp, sizeof(KP), hipMemcpyHostToDevice));
  if (s.l2_overlap) {  // the second stream's link stage: list 2, staging rows past the first grids
    KP k2 = s.kp;
    k2.loop_list = 2;
    k2.xstage += static_cast<size_t>(s.grid_link) * p.cap_stage;
    k2.xmeta += static_cast<size_t>(s.grid_link) * p.cap_stage;
    if (k2.eidx_g) k2.eidx_g += static_cast<size_t>(kLoopGrid) * p.cap_ops;
    if ((rc = dalloc(s, &s.kp_dev2, 1))) return rc;
    HIPCHK(hipMemcpy(s.kp_dev2, &k2, sizeof(KP), hipMemcpyHostToDevice));
    HIPCHK(hipStreamCreateWithFlags(&s.stream2, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&s.ev_fork, hipEventDisableTiming | hipEventDisableSystemFence));
    HIPCHK(hipEventCreateWithFlags(&s.ev_join, hipEventDisableTiming | hipEventDisableSystemFence));
  }
  if (s.sum) {  // (summary mode) the looped generic link stage over list 1: windows of few senders
    KP k1 = s.kp;
    k1.loop_list = 1;
    if ((rc = dalloc(s, &s.kp_dev_l1, 1))) return rc;
    HIPCHK(hipMemcpy(s.kp_dev_l1, &k1, sizeof(KP), hipMemcpyHostToDevice));
    if (const char* lf = std::getenv("BCSIM_LINK_FEW"); lf && *lf) s.link_few = static_cast<uint32_t>(std::atoi(lf));
  }
  if (!s.sparse && !s.pdes && c.protocol == BCSIM_PBFT) {
    KP kb = s.kp;
    kb.cap_arr = 2 * s.kp.cap_arr;
    const size_t lb = scan_lds_bytes(kb);
    if (lb + sizeof(ScanShared) <= 160 * 1024) {
      // (sort_window's merge area: one per workgroup of these launches -- at most kLoopGrid)
      if ((rc = dalloc(s, &kb.sortbuf, static_cast<size_t>(std::max<uint32_t>(kLoopGrid, s.few_scan)) * kb.cap_arr))) return rc;
      if ((rc = dalloc(s, &s.kp_dev_big, 1))) return rc;
      HIPCHK(hipMemcpy(s.kp_dev_big, &kb, sizeof(KP), hipMemcpyHostToDevice));
      HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_PBFT, false>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lb)));
      HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_scan<BCSIM_PBFT, false, true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lb)));
      s.lds_big = lb;
    }
  }
  s.bcnt.assign(s.B, 0);
  s.xcnt.assign(s.B, 0);
  s.zeroed_turn.assign(s.B, -1);  // hipMemset above: every bucket is clean before turn 0
  s.next_tick = (c.protocol == BCSIM_PBFT) ? p.pbft_period : INT64_MAX;
  s.n_alive = (c.protocol == BCSIM_PBFT) ? 1 : 0;  // STARTs arm the ticks
  return BCSIM_OK;
}

static bool sync_each() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("BCSIM_SYNC_EACH");
    v = (e && *e && *e != '0') ? 1 : 0;
  }
  return v == 1;
}

// Kernel-class timing (bcsim_read_kernel_stats): HIP events around the launches of the
// classes in BCSIM_KSTATS (bit mask over KS_*, default all, read at every launch).  An event
// pair costs a few microseconds of dispatch per launch (bench.py times the k_link class only).
static uint32_t kstat_mask() {
  const char* e = std::getenv("BCSIM_KSTATS");
  return e && *e ? static_cast<uint32_t>(std::strtol(e, nullptr, 0)) & 15u : 15u;
}
template <typename K, typename... Args>
static int launch_named(Sim& s, const char* name, int cls, K kernel, dim3 grid, dim3 block, size_t lds,
                        Args... args) {
  const auto h0 = std::chrono::steady_clock::now();
  struct HostClock {  // (host time spent launching: bcsim_read_host_stats)
    Sim& s;
    std::chrono::steady_clock::time_point t0;
    ~HostClock() {
      s.host_launch_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      ++s.host_launches;
    }
  } hclock{s, h0};
  const bool timed = cls >= 0 && ((kstat_mask() >> cls) & 1u);
  int rc = timed ? ev_begin(s, cls) : BCSIM_OK;
  if (rc) return rc;
  if (timed && s.ext_events) s.ev_stop_attach = true;
  // timing events of a class are recorded by its first / last launch's dispatch (hipExtLaunchKernel:
  // the kernel's own start / end timestamps) instead of separate marker packets, each of which
  // cost a few us of dispatch gap
  hipEvent_t st = nullptr, sp = nullptr;
  if (s.ev_start_pend) {
    if (s.stream == s.ev_start_stream)
      st = s.ev_start_pend;
    else
      HIPCHK(hipEventRecord(s.ev_start_pend, s.ev_start_stream));  // (a launch on the other stream first)
    s.ev_start_pend = nullptr;
  }
  if (s.ev_stop_attach) {
    sp = s.ev_pool[s.ev_used].second;
    s.ev_stop_attach = false;
    s.ev_stop_done = true;
  }
  if (st || sp)
    hipExtLaunchKernelGGL(kernel, grid, block, static_cast<uint32_t>(lds), s.stream, st, sp, 0u, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, lds, s.stream, args...);
  HIPCHK(hipGetLastError());
  if (timed) {
    rc = ev_end(s);
    if (rc) return rc;
  } else if (cls >= 0) {
    s.launches[cls]++;
  }
  if (sync_each()) {  // debugging aid: pin a failure to one launch
    hipError_t e = hipStreamSynchronize(s.stream);
    if (e != hipSuccess) {
      g_detail = std::string(name) + " cell " + std::to_string(s.cells) + ": " + hipGetErrorString(e) +
                 " trail:" + trail_dump(s);
      return BCSIM_E_HIP;
    }
    if (s.trail_h) std::memset(s.trail_h, 0, s.NT * 8ull);
    Ctl c;
    HIPCHK(hipMemcpy(&c, s.ctl_d, sizeof c, hipMemcpyDeviceToHost));
    if (c.err) {
      g_detail = std::string(name) + " cell " + std::to_string(s.cells) + " err " + std::to_string(c.err) +
                 (c.dbg ? " at engine.hip:" + std::to_string(c.dbg) : std::string());
      return c.err;
    }
  }
  return BCSIM_OK;
}
#define launch(s, cls, kernel, ...) launch_named(s, #kernel, cls, kernel, __VA_ARGS__)

// debug (BCSIM_WGT=1): k_mesh_tile phase clocks of a launch (100 MHz s_memrealtime): span, mean
// per phase over the workgroups that had jobs, and how many were running at each 10 us
static int tile_phase_report(Sim& s, long long cell, uint32_t nt) {
  std::vector<unsigned long long> w(8ull * nt);
  HIPCHK(hipStreamSynchronize(s.stream));
  HIPCHK(hipMemcpy(w.data(), s.kp.wgtt, w.size() * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(s.kp.wgtt, 0, w.size() * 8));
  unsigned long long t0 = ~0ull, t1 = 0;
  double m[5] = {0, 0, 0, 0, 0};
  uint32_t n = 0;
  for (uint32_t b = 0; b < nt; ++b) {
    const unsigned long long* q = &w[8ull * b];
    if (!q[0] || !q[5]) continue;
    ++n;
    t0 = std::min(t0, q[0]);
    t1 = std::max(t1, q[5]);
    for (int k = 0; k < 5; ++k) m[k] += static_cast<double>(q[k + 1] - q[k]);
  }
  if (!n || t1 - t0 < 5000) return BCSIM_OK;
  {  // (k_mesh_row: tiles walked, row classes)
    unsigned long long a6 = 0, a7 = 0;
    for (uint32_t b = 0; b < nt; ++b) {
      a6 += w[8ull * b + 6];
      a7 += w[8ull * b + 7];
    }
    if (a7)
      std::fprintf(stderr, "[row] cell %lld rows %llu no-uniform %llu beyond-ring %llu off-idle-bucket %llu tiles walked %llu\n", cell,
                   a7 & 0xFFFF, (a7 >> 16) & 0xFFFF, (a7 >> 32) & 0xFFFF, a7 >> 48, a6);
  }
  std::fprintf(stderr, "[tile] cell %lld span %.1f us, %u WGs, mean us: prologue %.2f lw %.2f edges %.2f barrier %.2f out %.2f; running per 10 us:",
               cell, (t1 - t0) / 100.0, n, m[0] / n / 100, m[1] / n / 100, m[2] / n / 100, m[3] / n / 100, m[4] / n / 100);
  for (unsigned long long t = t0; t < t1; t += 1000) {
    uint32_t r = 0;
    for (uint32_t b = 0; b < nt; ++b) {
      const unsigned long long* q = &w[8ull * b];
      if (q[0] && q[5] && q[0] <= t + 500 && q[5] >= t + 500) ++r;
    }
    std::fprintf(stderr, " %u", r);
  }
  std::fprintf(stderr, "\n");
  std::vector<uint32_t> idx;
  for (uint32_t b = 0; b < nt; ++b)
    if (w[8ull * b] && w[8ull * b + 5]) idx.push_back(b);
  std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return w[8ull * a + 5] > w[8ull * b + 5]; });
  std::fprintf(stderr, "[tile]   last to finish:");
  for (size_t k = 0; k < std::min<size_t>(6, idx.size()); ++k) {
    const unsigned long long* q = &w[8ull * idx[k]];
    const uint32_t rem = idx[k] % (s.kp.n_stiles * s.kp.n_tiles);
    std::fprintf(stderr, " [st %u rt %u start +%.1f total %.1f:", rem / s.kp.n_tiles, rem % s.kp.n_tiles, (q[0] - t0) / 100.0,
                 (q[5] - q[0]) / 100.0);
    for (int j = 0; j < 5; ++j) std::fprintf(stderr, " %.1f", (q[j + 1] - q[j]) / 100.0);
    std::fprintf(stderr, "]");
  }
  std::fprintf(stderr, "\n");
  return BCSIM_OK;
}

// k_mesh_row's cell arithmetic (no 64-bit divisions per workgroup): {cell % B, (cell / B) % 32,
// the idle-link arrival buckets of a small message sent at lo / hi - 1 (0xFFFF: outside the
// ring) as lo | hi << 16, 0}
static uint4 row_hq(const Sim& s, long long cell, long long lo, long long hi) {
  const long long B = s.B;
  uint32_t cb[2];
  for (int h = 0; h < 2; ++h) {
    const long long ca = ((h ? hi - 1 : lo) + s.kp.tx_tot[0] + s.kp.prop_const) / s.L;
    cb[h] = s.kp.prop_const >= 0 && ca - cell >= 1 && ca - cell < B ? static_cast<uint32_t>(ca % B) : 0xFFFFu;
  }
  return make_uint4(static_cast<uint32_t>(cell % B), static_cast<uint32_t>((cell / B) & 31), cb[0] | (cb[1] << 16), 0u);
}

static int do_scan(Sim& s, long long cell, long long lo, long long hi, long long cs, bool final_win) {
  const size_t lds = scan_lds_bytes(s.kp);
  dim3 grid(s.grid_scan), block(s.bs_scan);
  const int fw = final_win ? 1 : 0, xa = s.x_active;
  int rc = BCSIM_OK;
  // dense gossip: groups of G lanes walk all gnodes and take the simple ones; small looped
  // grids the rest (lists 2, 3) -- no k_active and no read-back in the window
  if (s.gossip_link && s.kp.dbg_tmax <= lo) {
    const uint32_t per_wg = 256 / s.gossip_g;
    const dim3 gg(static_cast<uint32_t>((static_cast<uint64_t>(s.R) * s.nloc + per_wg - 1) / per_wg));
    // the generic kernel only has work with a timer, START/STOP or extras in the window
    const int loop = lo <= 0 || xa || s.next_timer < hi || (s.cfg.stop_ns >= 0 && s.cfg.stop_ns < hi);
    // the fused scan + link kernel and the generic kernels after it as ONE timed launch of the
    // k_link class (it moves every record: the 16 B read, the link word, the 16 B write)
    const bool timed = (kstat_mask() >> KS_LINK) & 1u;
    if (timed && (rc = ev_begin(s, KS_LINK))) return rc;
    // the frontier list unless START / STOP makes every node active
    const int fl = s.gossip_frontier && !(lo <= 0 && 0 < hi) && !(s.cfg.stop_ns >= 0 && lo <= s.cfg.stop_ns && s.cfg.stop_ns < hi);
    const uint32_t na = static_cast<uint32_t>(static_cast<uint64_t>(s.R) * s.nloc);
    if ((fl && (rc = launch(s, -1, k_gossip_active, dim3((na + 1023) / 1024), dim3(1024), 0, s.kp_dev, cell, hi))) ||
        (rc = launch(s, -1, k_gossip_cell, gg, dim3(256), 0, s.kp_dev, cell, lo, hi, cs, xa, s.gossip_g, loop, fw, fl)) ||
        (loop &&
         (rc = launch(s, -1, (k_scan<BCSIM_GOSSIP, false, true>), dim3(256), block, lds, s.kp_dev, cell, lo, hi,
                      cs, fw, xa))) ||
        // (the looped grid may not exceed the workgroups the per-workgroup staging areas
        // were allocated for: xstage / xmeta hold grid_link of them)
        // (list 3 is almost always empty here; BCSIM_GL3: its grid, 8-256 measured alike)
        ((s.ev_stop_attach = timed && s.ext_events), false) ||
        (rc = launch(s, -1, (k_link<false, false, true>), dim3(std::min<uint32_t>(s.chain_l3_grid, s.grid_link)), dim3(s.bs_link),
                     link_lds_bytes(s.kp), s.kp_dev, cell, lo, hi, fw)))
      return rc;
    if (timed) return ev_end(s);
    s.launches[KS_LINK]++;
    return BCSIM_OK;
  }
  uint32_t n_link = 1;
  uint32_t scan_n = UINT32_MAX;  // (nodes scanned in the window, when read back)
  bool scan_dsz = false;  // (summary mode: the scan grids are sized on the device)
  {  // compact lists of the window's active gnodes
    // contiguous chunks of >= 256 gnodes (<= kActChunk), at most ~1024 workgroups (N=4096:
    // 16 workgroups of one gnode per lane; 2 of 2048 took 14-22 us of dependent loads per lane)
    const uint64_t nl = static_cast<uint64_t>(s.R) * s.nloc;
    const uint64_t nb = std::max<uint64_t>((nl + kActChunk - 1) / kActChunk, std::min<uint64_t>(1024, (nl + 255) / 256));
    const uint32_t chunk = static_cast<uint32_t>(((nl + nb - 1) / nb + 255) / 256 * 256);
    // (speculation: k_next predicted this window and k_active already ran for it behind k_next)
    uint32_t act_seq = 0;
    const bool spec_hit = s.spec_seq && s.ctl_h->pred[0] && s.ctl_h->pred[1] == cell && s.ctl_h->pred[2] == lo &&
                          s.ctl_h->pred[3] == hi;
    if (spec_hit) {
      act_seq = s.spec_seq;
      ++s.spec_hits;
    } else {
      if (s.spec_seq && s.ctl_h->pred[0]) HIPCHK(hipMemsetAsync(s.kp.act_n, 0, 16, s.stream));  // (its lists)
      act_seq = ++s.mseq;
      rc = launch(s, KS_AUX, k_active, dim3(static_cast<uint32_t>((nl + chunk - 1) / chunk)), dim3(256), 0, s.kp_dev, lo, hi,
                  static_cast<uint32_t>(cell % s.B), static_cast<uint32_t>((cell + kOpRing - 1) % kOpRing), chunk, act_seq, 0);
      if (rc) return rc;
    }
    s.spec_seq = 0;
    static const bool no_sync = [] {
      const char* e = std::getenv("BCSIM_NO_ACTSYNC");
      return e && *e == '1';
    }();
    // summary mode (heavy and light PBFT windows alike): k_scan_rt's fixed grid, looped generic
    // grids and device-sized link kernels -- the window makes no round trip to the host here
    const bool ss = (lo <= 0 && 0 < hi) || (s.cfg.stop_ns >= 0 && lo <= s.cfg.stop_ns && s.cfg.stop_ns < hi);
    static const uint32_t dmask = [] {  // (A/B: bit 0 the scan, bit 1 the link stage device-sized)
      const char* e = std::getenv("BCSIM_DEVSZ");
      return e && *e ? static_cast<uint32_t>(std::atoi(e)) : 3u;
    }();
    const bool dsz = s.sum && s.dev_sized && s.scan_fast && !ss && s.kp.wgtt == nullptr && !s.kp.wgs;
    if (dsz && dmask == 3u) {
      grid = dim3((s.NT + 7) / 8 * 8);  // (list_range: a multiple of 8 workgroups)
      scan_dsz = true;
      n_link = kDevSized;
    } else if (!s.sparse && !s.pdes && !no_sync) {
      // dense layout: read the list lengths back and launch exactly one workgroup per entry
      // (an idle node costs nothing; an empty list no launch).  A k_scan workgroup holds
      // ~140 KB of LDS, so even workgroups that exit at once go through the CUs one at a time
      // per CU: 4096 of them took ~24 us, the read-back takes ~10.
      const int w = s.act_m ? mirror_wait(s, s.act_m + 2, act_seq) : 1;
      if (w < 0) return w;
      if (w == 0) {  // (k_active's last workgroup published them)
        s.act_h[0] = s.act_m[0];
        s.act_h[1] = s.act_m[1];
      } else {
        HIPCHK(hipMemcpyAsync(s.act_h, s.kp.act_n, 16, hipMemcpyDeviceToHost, s.stream));
        if (!s.act_m) ++s.host_syncs;  // (with a mirror, mirror_wait counted it)
        HIPCHK(hipStreamSynchronize(s.stream));
      }
      grid = dim3((s.act_h[0] + 7) / 8 * 8);
      n_link = s.act_h[1];
      scan_n = s.act_h[0];
      if (dsz && (dmask & 1u)) {
        grid = dim3((s.NT + 7) / 8 * 8);
        scan_dsz = true;
      }
      if (dsz && (dmask & 2u)) n_link = kDevSized;
      static const bool winlog = std::getenv("BCSIM_WINLOG") != nullptr;  // (debug: one line per window)
      if (winlog)
        std::fprintf(stderr, "[win] cell %lld [%lld, %lld) +%lld us scan %u link %u xa %d spec %d (pred %lld %lld %lld %lld)\n", cell, lo,
                     hi, (lo - cell * s.L) / 1000, s.act_h[0], s.act_h[1], xa, spec_hit ? 1 : 0, s.ctl_h->pred[0], s.ctl_h->pred[1],
                     s.ctl_h->pred[2], s.ctl_h->pred[3]);
    } else if (!s.sparse) {
      // node-partitioned: a rank holds 1/P of the nodes, so a workgroup per local node costs
      // less than the round trip (the cell already has several collectives)
      grid = dim3((s.R * s.nloc + 7) / 8 * 8);
      n_link = s.R * s.nloc;
    }
  }
#define BCSIM_SCAN(P)                                                                                   \
  (s.sparse ? launch(s, KS_SCAN, k_scan<P, true>, grid, block, lds, s.kp_dev, cell, lo, hi, cs, fw, xa) \
            : launch(s, KS_SCAN, k_scan<P, false>, grid, block, lds, s.kp_dev, cell, lo, hi, cs, fw, xa))
  // summary mode: the scan reads the summaries itself (k_scan_rt), or the rows
  // of the window's nodes are materialised for the kernels that read slots only
  const dim3 grid_rt(s.R * s.kp.n_tiles);
  const bool ss_win = (lo <= 0 && 0 < hi) || (s.cfg.stop_ns >= 0 && lo <= s.cfg.stop_ns && s.cfg.stop_ns < hi);
  const bool use_rt = s.sum && grid.x && s.scan_fast && !ss_win &&
                      (scan_dsz || (!(s.kp_dev_big && grid.x <= s.few_scan) && grid.x >= s.rt_min));
  if (s.sum && grid.x && !use_rt &&
      (rc = launch(s, KS_SCAN, k_scan_rt, grid_rt, dim3(1024), 0, s.kp_dev, cell, lo, hi, cs, xa, 0u, 1)))
    return rc;
  if (grid.x == 0)
    rc = BCSIM_OK;  // no node has work in the window
  else if (use_rt) {
    // the scan of every receiver tile; the nodes it leaves (list 2, materialised) to the generic
    // kernel as after k_scan_pbft
    const uint32_t wep = s.l2_all ? (++s.win_epoch == 0 ? ++s.win_epoch : s.win_epoch) : 0u;
    rc = launch(s, KS_SCAN, k_scan_rt, grid_rt, dim3(1024), 0, s.kp_dev, cell, lo, hi, cs, xa, wep, 0);
    if (!rc && wep) {
      HIPCHK(hipEventRecord(s.ev_fork, s.stream));
      HIPCHK(hipStreamWaitEvent(s.stream2, s.ev_fork, 0));
      std::swap(s.stream, s.stream2);
      s.l2_pending = wep;
    }
    if (!rc)
      rc = s.kp_dev_big
               ? launch(s, KS_SCAN, (k_scan<BCSIM_PBFT, false, true>), dim3(std::min<uint32_t>(grid.x, kLoopGrid)), dim3(1024),
                        s.lds_big, s.kp_dev_big, cell, lo, hi, cs, fw, xa)
               : launch(s, KS_SCAN, (k_scan<BCSIM_PBFT, false, true>), dim3(std::min<uint32_t>(grid.x, 512)), block, lds,
                        s.kp_dev, cell, lo, hi, cs, fw, xa);
    if (wep) std::swap(s.stream, s.stream2);
  }
  else if (s.kp_dev_big && !s.sparse && !s.pdes && grid.x <= s.few_scan) {
    // a few nodes (the leader's cells): the doubled staging window, a 1024-lane workgroup each.
    // With the list-2 overlap they are scanned and linked on the second stream, beside the
    // other nodes' link stage (which skips them)
    const uint32_t wep = s.l2_overlap && s.mesh_link ? (++s.win_epoch == 0 ? ++s.win_epoch : s.win_epoch) : 0u;
    if (wep) {
      rc = launch(s, -1, k_l2_take, dim3(1), dim3(256), 0, s.kp_dev, wep);
      if (!rc) {
        HIPCHK(hipEventRecord(s.ev_fork, s.stream));
        HIPCHK(hipStreamWaitEvent(s.stream2, s.ev_fork, 0));
        std::swap(s.stream, s.stream2);
        s.l2_pending = wep;
      }
    }
    if (!rc)
      rc = launch(s, KS_SCAN, (k_scan<BCSIM_PBFT, false>), grid, dim3(1024), s.lds_big, s.kp_dev_big, cell, lo, hi, cs, fw,
                  xa);
    if (wep) std::swap(s.stream, s.stream2);
  }
  else if (s.scan_fast && !(lo <= 0 && 0 < hi) && !(s.cfg.stop_ns >= 0 && lo <= s.cfg.stop_ns && s.cfg.stop_ns < hi)) {
    // PBFT heavy waves: one pass over each row in registers; the nodes it leaves (list 2) to
    // the generic kernel -- a small looped grid, with the doubled staging window if there is one
    const uint32_t wep = s.l2_all ? (++s.win_epoch == 0 ? ++s.win_epoch : s.win_epoch) : 0u;
    rc = launch(s, KS_SCAN, k_scan_pbft, grid, dim3(kFastLanes), 0, s.kp_dev, cell, lo, hi, cs, xa, wep);
    if (!rc && wep) {  // fork: list 2 is scanned (and linked, below) on the second stream
      HIPCHK(hipEventRecord(s.ev_fork, s.stream));
      HIPCHK(hipStreamWaitEvent(s.stream2, s.ev_fork, 0));
      std::swap(s.stream, s.stream2);
      s.l2_pending = wep;
    }
    if (!rc)
      rc = s.kp_dev_big
               ? launch(s, KS_SCAN, (k_scan<BCSIM_PBFT, false, true>), dim3(std::min<uint32_t>(grid.x, kLoopGrid)), dim3(1024),
                        s.lds_big, s.kp_dev_big, cell, lo, hi, cs, fw, xa)
               : launch(s, KS_SCAN, (k_scan<BCSIM_PBFT, false, true>), dim3(std::min<uint32_t>(grid.x, 512)), block, lds,
                        s.kp_dev, cell, lo, hi, cs, fw, xa);
    if (wep) std::swap(s.stream, s.stream2);
  } else if (s.sparse && s.cfg.protocol == BCSIM_PAXOS && s.paxos_fast) {
    // sparse Paxos: one lane per node takes the acceptors' request windows; the generic
    // kernel walks the rest (list 2)
    rc = launch(s, KS_SCAN, k_paxos_scan, grid, dim3(256), 0, s.kp_dev, cell, lo, hi, cs, xa);
    if (!rc)
      rc = launch(s, KS_SCAN, (k_scan<BCSIM_PAXOS, true, true>), grid, block, lds, s.kp_dev, cell, lo, hi, cs, fw, xa);
  }
  else if (s.cfg.protocol == BCSIM_PBFT)
    rc = BCSIM_SCAN(BCSIM_PBFT);
  else if (s.cfg.protocol == BCSIM_RAFT)
    rc = BCSIM_SCAN(BCSIM_RAFT);
  else if (s.cfg.protocol == BCSIM_GOSSIP)
    rc = BCSIM_SCAN(BCSIM_GOSSIP);
  else
    rc = BCSIM_SCAN(BCSIM_PAXOS);
#undef BCSIM_SCAN
  if (rc) return rc;
  if (s.kp.fdbg) {  // debug (BCSIM_FDBG=1): why nodes of this window left the fast scan kernel
    unsigned long long fc[16];
    HIPCHK(hipStreamSynchronize(s.stream));
    HIPCHK(hipMemcpy(fc, s.kp.fdbg, sizeof fc, hipMemcpyDeviceToHost));
    HIPCHK(hipMemset(s.kp.fdbg, 0, sizeof fc));
    unsigned long long any = 0;
    for (int k = 0; k < 8; ++k) any |= fc[k];
    if (any)
      std::fprintf(stderr, "[fdbg] cell %lld [%lld,%lld) scan grid %u: nowork %llu ss %llu timer %llu extras %llu deg %llu cfg %llu bad %llu instants %llu\n",
                   cell, lo, hi, grid.x, fc[0], fc[1], fc[2], fc[3], fc[4], fc[5], fc[6], fc[7]);
  }
  if (s.kp.wgs) {  // debug (BCSIM_WGT=1): mean k_scan phase times of a heavy launch
    std::vector<unsigned long long> w(8ull * s.NT);
    HIPCHK(hipStreamSynchronize(s.stream));
    HIPCHK(hipMemcpy(w.data(), s.kp.wgs, w.size() * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemset(s.kp.wgs, 0, w.size() * 8));
    double acc[8] = {0};
    unsigned long long tmin = ~0ull, tmax = 0;
    uint32_t nw = 0;
    for (uint32_t g = 0; g < s.NT; ++g) {
      const unsigned long long* q = &w[8ull * g];
      if (!q[7] || !q[0]) continue;
      ++nw;
      tmin = std::min(tmin, q[0]);
      tmax = std::max(tmax, q[7]);
      unsigned long long prev = q[0];
      for (int k = 1; k < 8; ++k) {
        if (q[k] >= prev) {
          acc[k] += static_cast<double>(q[k] - prev);
          prev = q[k];
        }
      }
      acc[0] += static_cast<double>(q[7] - q[0]);
    }
    if (nw && tmax - tmin > 5000) {
      std::fprintf(stderr, "[wgs] cell %lld k_scan span %.2f ms, %u WGs, mean us: total %.1f stage %.1f sort %.1f A %.1f B %.1f C %.1f D %.1f E+wb %.1f\n",
                   cell, (tmax - tmin) / 1e5, nw, acc[0] / nw / 100, acc[1] / nw / 100, acc[2] / nw / 100,
                   acc[3] / nw / 100, acc[4] / nw / 100, acc[5] / nw / 100, acc[6] / nw / 100, acc[7] / nw / 100);
      uint32_t gs = 0;  // the slowest workgroup's phases
      unsigned long long ws = 0;
      for (uint32_t g = 0; g < s.NT; ++g) {
        const unsigned long long* q = &w[8ull * g];
        if (q[7] && q[0] && q[7] - q[0] > ws) {
          ws = q[7] - q[0];
          gs = g;
        }
      }
      const unsigned long long* q = &w[8ull * gs];
      std::fprintf(stderr, "[wgs]   slowest g%u %.1f us:", gs, ws / 100.0);
      for (int k = 1; k < 8; ++k) std::fprintf(stderr, " %.1f", q[k] >= q[k - 1] ? (q[k] - q[k - 1]) / 100.0 : -1.0);
      std::fprintf(stderr, "\n");
    }
  }
  grid = dim3(s.sparse ? s.grid_link : n_link == kDevSized ? (s.NT + 7) / 8 * 8 : (n_link + 7) / 8 * 8);
  if (grid.x == 0 && s.l2_pending) grid = dim3(8);  // (list 2 is in list 1; the join below must run anyway)
  if (grid.x == 0)
    rc = BCSIM_OK;
  else if (s.sparse && s.paxos_fast && s.kp.qmodel == 0 && !s.pdes) {
    // sparse Paxos: one lane per acceptor first, the generic kernel over the rest (list 3)
    const bool timed = (kstat_mask() >> KS_LINK) & 1u;
    if (timed && (rc = ev_begin(s, KS_LINK))) return rc;
    if ((rc = s.px_cap4 ? launch(s, -1, k_paxos_link<4>, grid, dim3(kPxLinkThreads), 0, s.kp_dev, cell, lo, hi)
                        : launch(s, -1, k_paxos_link<kPxCap>, grid, dim3(kPxLinkThreads), 0, s.kp_dev, cell, lo, hi)) ||
        ((s.ev_stop_attach = timed && s.ext_events), false) ||
        (rc = launch(s, -1, k_link_sparse, grid, dim3(s.bs_link), 0, s.kp_dev, cell, lo, hi, fw, 3)))
      return rc;
    if (timed) {
      if ((rc = ev_end(s))) return rc;
    } else {
      s.launches[KS_LINK]++;
    }
  } else if (s.sparse)
    rc = launch(s, KS_LINK, k_link_sparse, grid, dim3(s.bs_link), 0, s.kp_dev, cell, lo, hi, fw, 1);
  else if (s.mesh_link) {
    // full mesh, fixed app delay: the lean kernel takes the nodes whose due ops are all
    // broadcasts, the generic kernel (a small looped grid) the rest (list 3); timed as ONE
    // launch of the k_link class
    const bool timed = (kstat_mask() >> KS_LINK) & 1u;
    if (timed && (rc = ev_begin(s, KS_LINK))) return rc;
    // (list 3 holds a few nodes, the leader's cells among them: wide workgroups)
    // (node-partitioned: the kernels that stage records for other ranks)
    const dim3 gl(std::min<uint32_t>(kLoopGrid, s.grid_link)), bl(std::min<uint32_t>(kLinkLoopThreads, 4 * s.bs_link));
    const size_t mlds = static_cast<size_t>(s.deg_max) * 8;  // (the PF variant's link words)
    const uint32_t z = 0, wep = s.l2_pending;
    if (wep) {  // list 2's link stage on the second stream, after its scan there
      std::swap(s.stream, s.stream2);
      // (the generic link stage flushes the nodes' descriptors first, as k_link_mesh does for the
      // nodes it hands on)
      rc = launch(s, -1, (k_link<false, false, true>), gl, bl, link_lds_bytes(s.kp), s.kp_dev2, cell, lo, hi, fw);
      std::swap(s.stream, s.stream2);
      if (rc) return rc;
      HIPCHK(hipEventRecord(s.ev_join, s.stream2));
    }
    if (s.pdes) {
      // (node-partitioned: one out-edge per lane per step, no parked link words -- 119 VGPRs and
      // no scratch, where the two-edge / prefetching variants spill at 4 waves per SIMD; the reply
      // descriptors, which need the parked words, are off at P > 1)
      if ((rc = launch(s, -1, k_link_mesh<true, 1, false>, grid, dim3(256), 0, s.kp_dev, cell, lo, hi, fw, z, z)) ||
          (rc = launch(s, -1, (k_link<false, true, true>), gl, bl, link_lds_bytes(s.kp), s.kp_dev, cell, lo, hi, fw)))
        return rc;
    } else if (s.kp_dev_l1 && !wep && n_link != kDevSized && n_link <= s.link_few && scan_n == 0) {
      // (few senders, nothing scanned: the generic stage flushes their uniform row words and
      // descriptors and links them -- what k_mesh_prep hands it anyway for the leader's block)
      s.ev_stop_attach = timed && s.ext_events;
      if ((rc = launch(s, -1, (k_link<false, false, true>), gl, bl, link_lds_bytes(s.kp), s.kp_dev_l1, cell, lo, hi, fw)))
        return rc;
      ++s.link_few_windows;
    } else if (s.mesh_tile && (n_link >= s.tile_min || s.sum)) {  // (summary mode: k_mesh_row keeps row-uniform link state)
      // the simple nodes' edges by 32 x 64 (sender x receiver) tiles; a launch
      // epoch tells this launch's jobs from stale ones
      const uint32_t ep = ++s.mesh_epoch == 0 ? ++s.mesh_epoch : s.mesh_epoch;
      const uint32_t nt = s.R * s.kp.n_stiles * s.kp.n_tiles;
      // k_mesh_row: a wave per sender, 16 per workgroup; a launch of few senders (the leader's
      // block broadcast) gives each sender a workgroup, its 16 waves over the sender's tiles
      // (device-sized: the kernel decides from the list length; its grid covers both shapes)
      const bool dsz = n_link == kDevSized;
      const uint32_t rsplit = dsz ? (kRowSplitDev | s.row_split_max) : n_link <= s.row_split_max ? 16u : 1u;
      const dim3 rgrid(dsz ? std::max<uint32_t>(s.row_split_max, (s.NT + kRowThreads / 64 - 1) / (kRowThreads / 64))
                           : rsplit > 1 ? n_link : (n_link + kRowThreads / 64 - 1) / (kRowThreads / 64)),
          rblock(kRowThreads);
      if ((rc = launch(s, -1, k_mesh_prep, grid, dim3(64), 0, s.kp_dev, cell, lo, hi, fw, ep, wep)) ||
          // (summary mode: the uniform jobs' rows; the tiles take the rest)
          (s.sum && (rc = launch(s, -1, k_mesh_row, rgrid, rblock, 0, s.kp_dev, cell, lo, hi, ep, row_hq(s, cell, lo, hi), rsplit))) ||
          (s.sum && s.kp.wgtt && (rc = tile_phase_report(s, cell, rgrid.x))) ||
          (!s.sum && (rc = launch(s, -1, k_mesh_tile, dim3(nt), dim3(kTileThreads), 0, s.kp_dev, cell, lo, hi, ep))) ||
          (!s.sum && s.kp.wgtt && (rc = tile_phase_report(s, cell, nt))) ||
          ((s.ev_stop_attach = timed && s.ext_events && !wep), false) ||
          (rc = launch(s, -1, (k_link<false, false, true>), gl, bl, link_lds_bytes(s.kp), s.kp_dev, cell, lo, hi, fw)))
        return rc;
    } else {
      // (a few nodes -- the leader's block broadcast at a tick -- get 1024-lane workgroups:
      // the launch is one workgroup's latency)
      if ((rc = s.mesh_pf ? launch(s, -1, k_link_mesh<false, 2, true>, grid, dim3(n_link <= 64 ? 1024 : 256), mlds,
                                   s.kp_dev, cell, lo, hi, fw, z, wep)
                          : launch(s, -1, k_link_mesh<false, 2, false>, grid, dim3(n_link <= 64 ? 1024 : 256), 0,
                                   s.kp_dev, cell, lo, hi, fw, z, wep)) ||
          (rc = launch(s, -1, (k_link<false, false, true>), gl, bl, link_lds_bytes(s.kp), s.kp_dev, cell, lo, hi, fw)))
        return rc;
    }
    if (wep) {  // join (inside the timed k_link class: it ends when both streams are done)
      HIPCHK(hipStreamWaitEvent(s.stream, s.ev_join, 0));
      s.l2_pending = 0;
    }
    if (timed) {
      if ((rc = ev_end(s))) return rc;
    } else {
      s.launches[KS_LINK]++;
    }
  } else {
    const size_t ll = link_lds_bytes(s.kp);
    const bool qm = s.kp.qmodel != 0, xr = s.kp.nranks > 1;
    if (s.kp.qmodel == 2)
      rc = xr ? launch(s, KS_LINK, (k_link<2, true>), grid, dim3(s.bs_link), ll, s.kp_dev, cell, lo, hi, fw)
              : launch(s, KS_LINK, (k_link<2, false>), grid, dim3(s.bs_link), ll, s.kp_dev, cell, lo, hi, fw);
    else
    rc = qm ? (xr ? launch(s, KS_LINK, k_link<true, true>, grid, dim3(s.bs_link), ll, s.kp_dev, cell, lo, hi, fw)
                  : launch(s, KS_LINK, k_link<true, false>, grid, dim3(s.bs_link), ll, s.kp_dev, cell, lo, hi, fw))
            : (xr ? launch(s, KS_LINK, k_link<false, true>, grid, dim3(s.bs_link), ll, s.kp_dev, cell, lo, hi, fw)
                  : launch(s, KS_LINK, k_link<false, false>, grid, dim3(s.bs_link), ll, s.kp_dev, cell, lo, hi, fw));
  }
  if (!rc && s.kp.fdbg) {  // debug (BCSIM_FDBG=1): nodes k_link_mesh left to the generic kernel
    unsigned long long fc[16];
    HIPCHK(hipStreamSynchronize(s.stream));
    HIPCHK(hipMemcpy(fc, s.kp.fdbg, sizeof fc, hipMemcpyDeviceToHost));
    HIPCHK(hipMemset(s.kp.fdbg, 0, sizeof fc));
    if (fc[8] | fc[9] | fc[10] | fc[11] | fc[12] | fc[13] | fc[14] | fc[15])
      std::fprintf(stderr, "[fdbg] cell %lld [%lld,%lld) link grid %u: listed %llu bcasts %llu | generic: listed %llu bcasts %llu rxe %llu slots %llu 2desc %llu other %llu\n",
                   cell, lo, hi, grid.x, fc[8], fc[9], fc[10], fc[11], fc[12], fc[13], fc[14], fc[15]);
  }
  if (rc || !s.kp.wgt) return rc;
  // debug (BCSIM_WGT=1): report the slowest k_link workgroups of this launch
  std::vector<unsigned long long> w(8ull * s.NT);
  HIPCHK(hipStreamSynchronize(s.stream));
  HIPCHK(hipMemcpy(w.data(), s.kp.wgt, w.size() * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(s.kp.wgt, 0, w.size() * 8));
  std::vector<uint32_t> idx;
  unsigned long long tmin = ~0ull, tmax = 0;
  for (uint32_t g = 0; g < s.NT; ++g)
    if (w[8 * g + 1]) {
      idx.push_back(g);
      tmin = std::min(tmin, w[8 * g]);
      tmax = std::max(tmax, w[8 * g + 1]);
    }
  std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return w[8 * a + 1] - w[8 * a] > w[8 * b + 1] - w[8 * b]; });
  if (!idx.empty() && tmax - tmin > 20000) {  // > 0.2 ms (100 MHz clock)
    double m[5] = {0, 0, 0, 0, 0};
    for (uint32_t g : idx) {
      const unsigned long long* q = &w[8 * g];
      m[0] += q[1] - q[0];
      m[1] += q[3] - q[0];
      m[2] += q[4] - q[3];
      m[3] += q[5] - q[4];
      m[4] += q[1] - q[6];
    }
    for (double& v : m) v /= 100.0 * idx.size();
    std::fprintf(stderr, "[wgt] cell %lld k_link span %.2f ms, %zu WGs, mean us: total %.1f classify %.1f scan+place %.1f edges %.1f compact %.1f; slowest:",
                 cell, (tmax - tmin) / 1e5, idx.size(), m[0], m[1], m[2], m[3], m[4]);
    for (size_t k = 0; k < std::min<size_t>(5, idx.size()); ++k) {
      const uint32_t g = idx[k];
      const unsigned long long* q = &w[8 * g];
      std::fprintf(stderr, " [g%u %.2fms n=%llu kept=%llu classify=%.0f scan+place=%.0f edges=%.0f gap=%.0f compact=%.0f us]", g,
                   (q[1] - q[0]) / 1e5, q[2] >> 32, q[2] & 0xFFFFFFFFull, (q[3] - q[0]) / 100.0, (q[4] - q[3]) / 100.0,
                   (q[5] - q[4]) / 100.0, (q[6] - q[5]) / 100.0, (q[1] - q[6]) / 100.0);
    }
    std::fprintf(stderr, "\n");
  }
  return BCSIM_OK;
}

// Prepare cell `cell`: move overflow records whose cell entered the ring into
// the inbox, and group the cell's extras (second records of one edge) by
// receiver.
static int group_cell(Sim& s, long long cell) {
  const uint32_t b = static_cast<uint32_t>(cell % s.B);
  if (s.ov_min <= cell + static_cast<long long>(s.B) - 1 && s.ctl_m) {
    // the overflow count as of the last read-back (nothing appends to the list between the
    // end-of-cell read-back and here); the launch resets the bound and the list itself and
    // publishes the control block: one spin, no copies (the path below without a mirror)
    const uint32_t nov = s.ctl_h->ov_cnt;
    s.next_seq = ++s.mseq;
    int rc = launch(s, KS_GROUP, k_rebin, dim3(std::max<uint32_t>(1u, (nov + 255) / 256)), dim3(256), 0, s.kp_dev, cell, nov,
                    s.next_seq);
    if (rc || (rc = readback(s, true))) return rc;
    // (compacted: the records that stay go back to the list's front before anything appends)
    const uint32_t ns = s.ctl_h->ov_cnt;
    if (s.kp.ov_tmp && ns &&
        (rc = launch(s, KS_GROUP, k_ov_back, dim3(std::min<uint32_t>(1024, (ns + 255) / 256)), dim3(256), 0, s.kp_dev)))
      return rc;
  } else if (s.ov_min <= cell + static_cast<long long>(s.B) - 1) {
    const uint32_t nov = s.ctl_h->ov_cnt;
    HIPCHK(hipMemcpyAsync(s.kp.scal + 1, s.act_h + 4, 8, hipMemcpyHostToDevice, s.stream));  // LLONG_MAX (pinned)
    if (nov) {
      int rc = launch(s, KS_GROUP, k_rebin, dim3((nov + 255) / 256), dim3(256), 0, s.kp_dev, cell, nov, 0u);
      if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(s.bcnt_h, s.kp.bucket_cnt, 8ull * s.B, hipMemcpyDeviceToHost, s.stream));
    HIPCHK(hipMemcpyAsync(&s.ov_min, s.kp.scal + 1, 8, hipMemcpyDeviceToHost, s.stream));
    ++s.host_syncs;
    HIPCHK(hipStreamSynchronize(s.stream));
    for (uint32_t k = 0; k < s.B; ++k) {
      s.bcnt[k] = s.bcnt_h[k];
      s.xcnt[k] = s.xcnt_h[k];
    }
    if (s.ov_min == LLONG_MAX) {
      // everything rebinned: reset the overflow list
      HIPCHK(hipMemsetAsync(s.kp.ov_cnt, 0, 4, s.stream));
    }
  }
  const uint32_t nx = s.xcnt[b];
  if (nx > s.kp.cap_x) {
    g_detail = "extras list of a cell overflowed (cap_bucket_records)";
    return BCSIM_E_OVERFLOW;
  }
  s.x_active = 0;
  if (nx) {
    HIPCHK(hipMemsetAsync(s.kp.seg_cnt, 0, s.NT * 4ull, s.stream));
    HIPCHK(hipMemsetAsync(s.kp.cursor, 0, s.NT * 4ull, s.stream));
    int rc;
    if ((rc = launch(s, KS_GROUP, k_xcount, dim3((nx + 255) / 256), dim3(256), 0, s.kp_dev, b, nx))) return rc;
    if (s.NT <= (1u << 20)) {
      if ((rc = launch(s, KS_GROUP, k_offsets, dim3(1), dim3(1024), 0, s.kp_dev))) return rc;
    } else {  // multi-block scan
      const uint32_t np = static_cast<uint32_t>((s.NT + kSegChunk - 1) / kSegChunk);
      if ((rc = launch(s, KS_GROUP, k_seg_sums, dim3(np), dim3(1024), 0, s.kp_dev, s.seg_part)) ||
          (rc = launch(s, KS_GROUP, k_seg_top, dim3(1), dim3(1024), 0, s.seg_part, np)) ||
          (rc = launch(s, KS_GROUP, k_seg_apply, dim3(np), dim3(1024), 0, s.kp_dev, s.seg_part)))
        return rc;
    }
    if ((rc = launch(s, KS_GROUP, k_xplace, dim3((nx + 255) / 256), dim3(256), 0, s.kp_dev, b, nx))) return rc;
    s.x_active = 1;
  }
  s.grouped_cell = cell;
  return BCSIM_OK;
}

// Wait for the kernel just launched to publish sequence number s.mseq to the host-mapped
// word w: 0 = published (the mirror holds its data), 1 = the stream drained without it (the
// kernel bailed on an error flag: read the device copy), < 0 = a HIP error.  The spin sees the
// kernel's last store ~1 us after it lands; a stream sync adds the completion signal's
// wake-up and the end-of-kernel cache release (~10-20 us per read-back).  With
// BCSIM_SPIN=0, a plain stream sync.
constexpr int kSpinUs = 500;  // mirror_wait: spin at most this long, then a stream sync
static int mirror_wait(Sim& s, const uint32_t* w, uint32_t seq) {
  ++s.host_syncs;
  struct HostClock {  // (host time spent waiting: bcsim_read_host_stats)
    Sim& s;
    std::chrono::steady_clock::time_point t0;
    ~HostClock() { s.host_wait_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(); }
  } hclock{s, std::chrono::steady_clock::now()};
  static const bool spin = [] {
    const char* e = std::getenv("BCSIM_SPIN");
    return !(e && *e == '0');
  }();
  if (!spin) {
    HIPCHK(hipStreamSynchronize(s.stream));
    return __atomic_load_n(w, __ATOMIC_ACQUIRE) == seq ? 0 : 1;
  }
  // (a pause per spin, and a stream sync once the wait is long -- a window with heavy kernels --
  // so that ranks sharing the host's cores do not lose them to spinning peers)
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t it = 1;; ++it) {
    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) return 0;
    __builtin_ia32_pause();
    if ((it & 255u) == 0) {
      const hipError_t q = hipStreamQuery(s.stream);
      if (q == hipSuccess) return __atomic_load_n(w, __ATOMIC_ACQUIRE) == seq ? 0 : 1;
      if (q != hipErrorNotReady) HIPCHK(q);
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSpinUs)) {
        HIPCHK(hipStreamSynchronize(s.stream));
        return __atomic_load_n(w, __ATOMIC_ACQUIRE) == seq ? 0 : 1;
      }
    }
  }
}

// after_next: right after k_next, which published the control block to the host-mapped
// mirror -- the read-back is the stream sync alone
static int readback(Sim& s, bool after_next) {
  const size_t nb = sizeof(Ctl) + 8ull * s.B + 4ull * kMaxRanks;
  int w = 1;
  if (after_next && s.ctl_m && (w = mirror_wait(s, reinterpret_cast<uint32_t*>(s.ctl_m) + nb / 4, s.next_seq)) < 0) return w;
  if (w == 0) {
    std::memcpy(s.ctl_h, s.ctl_m, nb);
  } else {
    HIPCHK(hipMemcpyAsync(s.ctl_h, s.ctl_d, nb, hipMemcpyDeviceToHost, s.stream));
    if (!(after_next && s.ctl_m)) ++s.host_syncs;
    HIPCHK(hipStreamSynchronize(s.stream));
  }
  return readback_apply(s);
}

// the host's copy of the control block (in ctl_h) into its bookkeeping
static int readback_apply(Sim& s) {
  // per-launch timing events: read in batches (reading them needs their completion signals)
  int rc = s.ev_used >= kEvBatch ? ev_collect(s) : 0;
  if (rc) return rc;
  for (uint32_t k = 0; k < s.B; ++k) {
    s.bcnt[k] = s.bcnt_h[k];
    s.xcnt[k] = s.xcnt_h[k];
  }
  s.next_local = s.ctl_h->scal[0];
  s.next_timer = s.ctl_h->scal[3];
  s.ov_min = s.ctl_h->scal[1];
  if (s.ctl_h->err) {
    g_detail = std::string(bcsim_strerror(s.ctl_h->err)) + " raised at engine.hip:" + std::to_string(s.ctl_h->dbg) +
               " (cell " + std::to_string(s.cells) + ")";
    return s.ctl_h->err;
  }
  return BCSIM_OK;
}

// ---- multi-GPU steps (all ranks call them in the same order) -------------
// Records for other ranks' receivers, staged by k_link during the cell, go
// out in one all-to-all; k_import places what came in.
// `lrc` is this rank's status of the cell so far: a failed rank sends the kPeerErr
// count to everyone instead of data, so every rank leaves together (no rank is left
// waiting in a collective the failed one never joins).
static long long local_next_cell(const Sim& s, bool with_tick);

// The per-cell exchange of a node-partitioned run: ONE control all-to-all --
// per peer the byte size of the records staged for it (kPeerErr: this rank failed), this
// rank's next-cell candidate, the earliest arrival cell it ships to anyone, and (tick cells)
// its ticking PBFT nodes -- from which every rank derives the same next cell, PBFT n_alive
// and status; then the records themselves (sizes known on both sides) and k_import.
static int exchange(Sim& s, long long cell, int lrc, bool tick) {
  const uint32_t P = s.P, W = Xport::kCtlWords;
  std::vector<int64_t> snd(static_cast<size_t>(P) * W), rcv(static_cast<size_t>(P) * W);
  std::vector<uint64_t> sb(P), rb(P);
  int rc;
  if (s.ctlw_d) {
    // device control words (RCCL): k_ctl computes this rank's words from the control block on the
    // device, the all-to-all runs on device buffers, and ONE sync brings back the words received
    // and the control block -- the end-of-window read-back and the control exchange in one round
    // trip (the old path: a read-back, then a host -> device -> all-to-all -> host exchange)
    long long ch = LLONG_MAX;  // the candidate's host-only terms (local_next_cell)
    if (s.start_pending) ch = 0;
    if (s.grouped_cell >= 0) ch = std::min(ch, s.grouped_cell);
    if (s.stop_pending && s.cfg.stop_ns >= 0 && s.cfg.stop_ns >= s.t_done) ch = std::min<long long>(ch, s.cfg.stop_ns / s.L);
    if ((rc = launch(s, KS_AUX, k_ctl, dim3(1), dim3(64), 0, s.kp_dev, s.ctlw_d, P, ch, static_cast<long long>(s.t_done),
                     tick ? 1 : 0, lrc)))
      return rc;
    rc = s.xp->ctl_exchange_dev(s.stream, s.ctlw_d);
    ++s.ctl_collectives;
    if (rc) return rc;
    const size_t nb = sizeof(Ctl) + 8ull * s.B + 4ull * kMaxRanks;
    HIPCHK(hipMemcpyAsync(s.ctlw_h, s.ctlw_d, 2ull * P * W * 8, hipMemcpyDeviceToHost, s.stream));
    HIPCHK(hipMemcpyAsync(s.ctl_h, s.ctl_d, nb, hipMemcpyDeviceToHost, s.stream));
    ++s.host_syncs;
    HIPCHK(hipStreamSynchronize(s.stream));
    if (lrc) return lrc;  // (k_ctl sent kPeerErr: every peer leaves at this exchange)
    // a failure found only now, after k_ctl told the peers this rank is fine: the
    // peers go on into the record exchange, so this rank joins it too (sizes clamped to its
    // buffer) and the failure rides the next cell's control words (run(): lerr)
    int arc = readback_apply(s);
    for (uint32_t r = 0; r < P && !arc; ++r)
      if (s.scnt_h[r] > s.kp.cap_send) {
        g_detail = "multi-GPU send list overflowed";
        arc = BCSIM_E_OVERFLOW;
      }
    s.carry_err = arc;
    const uint64_t cap_b = static_cast<uint64_t>(s.kp.cap_send) * sizeof(XRec);
    for (uint32_t r = 0; r < P; ++r) sb[r] = std::min<uint64_t>(static_cast<uint64_t>(s.ctlw_h[r * W]), cap_b);
    std::memcpy(rcv.data(), s.ctlw_h + static_cast<size_t>(P) * W, static_cast<size_t>(P) * W * 8);
  } else {
  for (uint32_t r = 0; r < P && !lrc; ++r)
    if (s.scnt_h[r] > s.kp.cap_send) {
      g_detail = "multi-GPU send list overflowed";
      lrc = BCSIM_E_OVERFLOW;
    }
  const long long cand = lrc ? LLONG_MAX : local_next_cell(s, false);
  const long long xmin = lrc ? LLONG_MAX : s.ctl_h->scal[4];
  const int64_t alive = (tick && !lrc) ? s.ctl_h->scal[2] : 0;
  for (uint32_t r = 0; r < P; ++r) {
    sb[r] = lrc ? kPeerErr : static_cast<uint64_t>(s.scnt_h[r]) * sizeof(XRec);
    snd[r * W + 0] = static_cast<int64_t>(sb[r]);
    snd[r * W + 1] = cand;
    snd[r * W + 2] = xmin;
    snd[r * W + 3] = alive;
  }
  rc = s.xp->ctl_exchange(s.stream, snd.data(), rcv.data());
  ++s.ctl_collectives;
  ++s.host_syncs;  // (host words in and out)
  if (rc) return rc;
  if (lrc) return lrc;
  }
  long long nx = LLONG_MAX;
  int64_t na = 0;
  uint64_t n = 0;
  for (uint32_t r = 0; r < P; ++r) {
    rb[r] = static_cast<uint64_t>(rcv[r * W + 0]);
    if (rb[r] == kPeerErr) {
      g_detail = "rank " + std::to_string(r) + " of the partition failed";
      return BCSIM_E_PEER;
    }
    nx = std::min<long long>(nx, rcv[r * W + 1]);
    nx = std::min<long long>(nx, rcv[r * W + 2]);
    na += rcv[r * W + 3];
    n += rb[r] / sizeof(XRec);
  }
  if (tick) {
    s.n_alive = na;
    s.next_tick += s.kp.pbft_period;
  }
  if (s.n_alive > 0 && s.next_tick != INT64_MAX) nx = std::min<long long>(nx, s.next_tick / s.L);
  s.next_cell = nx;
  s.next_known = true;
  if (n > s.cap_recv) {
    g_detail = "multi-GPU receive buffer too small";
    return BCSIM_E_OVERFLOW;
  }
  if ((rc = s.xp->sendrecv_dev(s.stream, reinterpret_cast<const char*>(s.kp.sendbuf),
                               static_cast<uint64_t>(s.kp.cap_send) * sizeof(XRec), sb.data(),
                               reinterpret_cast<char*>(s.recvbuf), rb.data())))
    return rc;
  ++s.ctl_collectives;
  HIPCHK(hipMemsetAsync(s.kp.send_cnt, 0, 4ull * kMaxRanks, s.stream));
  // (from pinned memory: a pageable source makes the copy a staged, blocking one)
  HIPCHK(hipMemcpyAsync(s.kp.scal + 4, s.act_h + 4, 8, hipMemcpyHostToDevice, s.stream));
  s.last_import = n;
  if (n) {
    rc = launch(s, KS_GROUP, k_import, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, s.kp_dev, cell,
                static_cast<const XRec*>(s.recvbuf), static_cast<uint32_t>(n));
    if (rc) return rc;
  }
  return BCSIM_OK;
}

// Share the v-log entries written since the last sync (PBFT file-scope `v`,
// pbft-node.cc:26, written by VIEW_CHANGE receipts on every node).
static int sync_vlog(Sim& s, int lrc = 0) {
  if (lrc) {  // tell the other ranks (their SUM goes negative), then leave
    int64_t bad = -(1ll << 40);
    int rc = s.xp->allreduce_i64(s.stream, &bad, 1, 1);
    return rc ? rc : lrc;
  }
  uint32_t cnt = 0;
  HIPCHK(hipMemcpyAsync(&cnt, s.kp.vlog_cnt, 4, hipMemcpyDeviceToHost, s.stream));
  ++s.host_syncs;
  HIPCHK(hipStreamSynchronize(s.stream));
  cnt = std::min(cnt, s.kp.cap_vlog);
  const uint32_t mine = cnt - s.vsync;
  std::vector<VLog> loc(mine);
  if (mine) HIPCHK(hipMemcpy(loc.data(), s.kp.vlog + s.vsync, mine * sizeof(VLog), hipMemcpyDeviceToHost));
  // everyone gets my new entries
  std::vector<char> snd(static_cast<size_t>(mine) * sizeof(VLog) * s.P);
  std::vector<uint64_t> sb(s.P, static_cast<uint64_t>(mine) * sizeof(VLog)), rb(s.P);
  for (uint32_t r = 0; r < s.P; ++r)
    if (mine) std::memcpy(snd.data() + static_cast<size_t>(r) * mine * sizeof(VLog), loc.data(), mine * sizeof(VLog));
  int64_t tot = mine;
  int rc = s.xp->allreduce_i64(s.stream, &tot, 1, 1);
  if (rc) return rc;
  if (tot < 0) {
    g_detail = "another rank of the partition failed";
    return BCSIM_E_PEER;
  }
  std::vector<char> rcv(static_cast<size_t>(tot) * sizeof(VLog) + 16);
  rc = s.xp->alltoallv_host(s.stream, snd.data(), sb.data(), rcv.data(), rcv.size(), rb.data());
  if (rc) return rc;
  std::vector<VLog> add;
  uint64_t off = 0;
  for (uint32_t r = 0; r < s.P; ++r) {
    const uint64_t k = rb[r] / sizeof(VLog);
    if (r != s.prank)
      for (uint64_t j = 0; j < k; ++j) add.push_back(reinterpret_cast<const VLog*>(rcv.data() + off)[j]);
    off += rb[r];
  }
  if (cnt + add.size() > s.kp.cap_vlog) return BCSIM_E_OVERFLOW;
  if (!add.empty()) {
    HIPCHK(hipMemcpy(s.kp.vlog + cnt, add.data(), add.size() * sizeof(VLog), hipMemcpyHostToDevice));
    const uint32_t ncnt = cnt + static_cast<uint32_t>(add.size());
    HIPCHK(hipMemcpy(s.kp.vlog_cnt, &ncnt, 4, hipMemcpyHostToDevice));
    cnt = ncnt;
  }
  s.vsync = cnt;
  return BCSIM_OK;
}

// Leader flags of every rank for the PBFT tick (bytes are 0/1 and disjoint
// across ranks, so an int64 SUM of the packed bytes is their union).
static int sync_leaders(Sim& s) {
  int rc = launch(s, KS_AUX, k_lead, dim3(s.R), dim3(1024), 0, s.kp_dev);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(s.lead_w.data(), s.kp.lead_loc, s.NT, hipMemcpyDeviceToHost, s.stream));
  ++s.host_syncs;
  HIPCHK(hipStreamSynchronize(s.stream));
  for (size_t k = 0; k < s.lead_w.size(); k += 4096) {  // (one call for N <= 32768 nodes)
    const uint32_t n = static_cast<uint32_t>(std::min<size_t>(4096, s.lead_w.size() - k));
    if ((rc = s.xp->allreduce_i64(s.stream, s.lead_w.data() + k, n, 1))) return rc;
    ++s.ctl_collectives;
  }
  HIPCHK(hipMemcpyAsync((void*)s.kp.lead_all, s.lead_w.data(), s.NT, hipMemcpyHostToDevice, s.stream));
  return BCSIM_OK;
}

// the reference's full mesh (blockchain-simulator.cc:34-51) unless a CSR was given; built
// lazily so that large sparse configs never materialise N*(N-1) edges
static int ensure_topology(Sim& s) {
  if (s.topo_ready) return BCSIM_OK;
  int rc;
  if ((rc = build_mesh(s)) || (rc = build_rev(s))) return rc;
  s.E = s.row[s.N];
  s.deg_max = 0;
  for (uint32_t i = 0; i < s.N; ++i) s.deg_max = std::max(s.deg_max, s.row[i + 1] - s.row[i]);
  s.topo_ready = true;
  return BCSIM_OK;
}

// Inbox-slot records carry a 5-bit ring-turn tag (engine.hip cell_tag: (cell / B) mod 32), so
// a delivered record needs no clear; the invariant that makes a matching tag mean "live" is
// that bucket b holds no record of turn T - 32k when turn T of b begins.  It holds because
// every cell s whose turn ends a 32-turn period ((s / B) % 32 == 31) zeroes its bucket once it
// is over -- the cells run() processes to their end AND the cells it skips for lack of work
// (no live record sits in a skipped cell's bucket, and none for a later turn of it exists
// yet: such a record is emitted at a cell > s, or rebinned by group_cell of a cell > s, both
// after this call).  Cells [a, b] are finished or skipped; at most B memsets.
static int zero_tag_buckets(Sim& s, long long a, long long b) {
  if (s.sparse || b < a) return BCSIM_OK;
  const size_t per = static_cast<size_t>(s.R) * s.kp.E_loc;
  std::vector<uint8_t> hit(s.B, 0);
  if (b - a + 1 >= 32ll * s.B) {
    std::fill(hit.begin(), hit.end(), 1);
  } else {
    for (long long x = a; x <= b; ++x)
      if ((x / s.B) % 32 == 31) hit[x % s.B] = 1;
  }
  for (uint32_t k = 0; k < s.B; ++k)
    if (hit[k]) {
      {  // (a store kernel: hipMemsetAsync of a 268 MB bucket ran at ~0.2-0.8 TB/s)
        const uint64_t n16 = per * sizeof(Rec) / 16;
        const uint32_t nb = static_cast<uint32_t>(std::min<uint64_t>(8192, (n16 + 255) / 256));
        int rc = launch(s, KS_AUX, k_zero16, dim3(nb), dim3(256), 0, reinterpret_cast<uint4*>(s.kp.inbox + static_cast<size_t>(k) * per),
                        n16);
        if (rc) return rc;
      }
      if (s.sum) {  // the bucket's summary entries and explicit-slot bytes carry the same tags
        const size_t ns = static_cast<size_t>(s.R) * s.kp.n_tiles * s.N;
        const uint32_t nb = static_cast<uint32_t>(std::min<uint64_t>(8192, (ns * 2 + 255) / 256));
        int rc = launch(s, KS_AUX, k_zero16, dim3(nb), dim3(256), 0, s.kp.msum + static_cast<size_t>(k) * ns * 2,
                        static_cast<uint64_t>(ns * 2));
        if (rc) return rc;
        HIPCHK(hipMemsetAsync(s.kp.xsum + static_cast<size_t>(k) * ns, 0, ns, s.stream));
      }
      ++s.tag_zeroes;
      // the latest turn of bucket k in [a, b]
      const long long lastk = b - ((b % s.B - k + s.B) % s.B);
      s.zeroed_turn[k] = std::max(s.zeroed_turn[k], lastk / s.B);
    }
  return BCSIM_OK;
}

// The invariant itself, checked before turn c / B of bucket c % B begins: records of turns
// Z+1 .. T-1 (Z = the turn after which the bucket was last zeroed) may still sit in it, and
// none of them may carry the tag of T, i.e. T - Z <= 32.
static int check_tag_invariant(Sim& s, long long c) {
  if (s.sparse) return BCSIM_OK;
  const long long T = c / s.B, Z = s.zeroed_turn[c % s.B];
  if (T - Z > 32) {
    g_detail = "inbox-slot tag invariant broken: bucket " + std::to_string(c % s.B) + " last zeroed after turn " +
               std::to_string(Z) + ", turn " + std::to_string(T) + " begins";
    return BCSIM_E_STATE;
  }
  return BCSIM_OK;
}

// The earliest cell with work on this rank (the state after the cells processed so far).
// with_tick: include the PBFT tick (n_alive must then be the global one).
static long long local_next_cell(const Sim& s, bool with_tick) {
  const long long L = s.L;
  long long c = LLONG_MAX;
  const long long cdone = s.t_done / L;
  if (s.start_pending) c = 0;
  if (s.grouped_cell >= 0) c = std::min(c, s.grouped_cell);  // partially processed cell
  for (uint32_t b = 0; b < s.B; ++b) {
    if (!s.bcnt[b]) continue;
    // bucket b holds the cell c == b (mod B) in [cdone, cdone + B)
    const long long cb = cdone + ((static_cast<long long>(b) - cdone % s.B) % s.B + s.B) % s.B;
    c = std::min(c, cb);
  }
  if (s.next_local != LLONG_MAX) c = std::min(c, std::max<long long>(s.next_local, s.t_done) / L);
  if (s.ov_min != LLONG_MAX) c = std::min(c, s.ov_min);
  if (with_tick && s.n_alive > 0 && s.next_tick != INT64_MAX) c = std::min(c, s.next_tick / L);
  if (s.stop_pending && s.cfg.stop_ns >= 0 && s.cfg.stop_ns >= s.t_done) c = std::min(c, s.cfg.stop_ns / L);
  return c;
}

// Device-chained windows (dense gossip): up to K windows enqueued at once --
// k_win opens the first from the host's state, each window's kernels run with cell = -1 (the window
// from the control block's win words), and its k_next closes it and decides the next (or ends the
// chain) -- then ONE host sync on the last k_next's mirror.  The windows that were never opened run
// no-op kernels; their timing events and launch counts are dropped.  The caller has checked that the
// first window needs no host work.
static int run_chain(Sim& s, long long c, long long lim) {
  // at most one window per cell up to the first cell the host knows the chain must stop before: the
  // run limit, the next timer (its window is the host's), an overflow rebin, extras to group, the
  // ring-tag zeroing -- a window that is never opened still costs its dispatches
  const long long L = s.L, B = s.B;
  long long cend = (lim - 1) / L;
  // the window of the next timer (the origin's block tick) gets the generic scan at its chain
  // position -- one window per cell from c; a second timer ends the chain (k_win / k_next)
  unsigned long long loop_mask = 0;
  if (s.next_timer != LLONG_MAX && s.next_timer >= 0) {
    const long long j = s.next_timer / L - c;
    if (j >= 0 && j < 32) loop_mask = 1ull << j;
    else cend = std::min(cend, s.next_timer / L - 1);
  }
  if (s.ov_min != LLONG_MAX) cend = std::min(cend, s.ov_min - B);
  {
    const long long t0 = (s.last_full + 1) / B;
    const long long z = (t0 % 32 == 31) ? s.last_full + 1 : ((t0 / 32) * 32 + 31) * B;
    cend = std::min(cend, z - 1);
  }
  for (long long x = c + 1; x <= cend && x < c + B; ++x)
    if (s.xcnt[x % B]) {
      cend = x - 1;
      break;
    }
  const uint32_t K = static_cast<uint32_t>(std::max<long long>(1, std::min<long long>(s.chain_k, cend - c + 1)));
  const bool timed = (kstat_mask() >> KS_LINK) & 1u;
  const uint32_t per_wg = 256 / s.gossip_g;
  const dim3 gg(static_cast<uint32_t>((static_cast<uint64_t>(s.R) * s.nloc + per_wg - 1) / per_wg));
  const uint32_t na = static_cast<uint32_t>(static_cast<uint64_t>(s.R) * s.nloc);
  const uint32_t nbn = s.NT <= 4096u ? 1u : static_cast<uint32_t>(std::min<uint64_t>(kNextBlocks, (s.NT + 2047) / 2048));
  const long long stop = s.stop_pending && s.cfg.stop_ns >= 0 ? static_cast<long long>(s.cfg.stop_ns) : -1ll;
  std::vector<size_t> ev_at(K, SIZE_MAX), ev_nx(K, SIZE_MAX);
  int rc;
  for (uint32_t k = 0; k < K; ++k) {
    // (the first window from the host's state; each later one decided by the k_next before it)
    if (k == 0 && (rc = launch(s, -1, k_win, dim3(1), dim3(64), 0, s.kp_dev, static_cast<long long>(s.t_done), s.last_full,
                               lim, stop, loop_mask)))
      return rc;
    if (timed) {
      ev_at[k] = s.ev_used;
      if ((rc = ev_begin(s, KS_LINK))) return rc;
    }
    // (the frontier: k_gossip_active for the chain's first window; later ones get it from the k_next
    // before them, or k_gossip_cell walks every gnode after a missed guess)
    if ((k == 0 && (rc = launch(s, -1, k_gossip_active, dim3((na + 1023) / 1024), dim3(1024), 0, s.kp_dev, -1ll, 0ll))) ||
        (rc = launch(s, -1, k_gossip_cell, gg, dim3(256), 0, s.kp_dev, -1ll, 0ll, 0ll, 0ll, 0, s.gossip_g, 0, 0, 1)) ||
        // (the generic scan where the host expects the origin's block tick; it exits at once when
        // the window at this position has no timer due)
        (((loop_mask >> k) & 1ull) &&
         (rc = launch(s, -1, (k_scan<BCSIM_GOSSIP, false, true>), dim3(256), dim3(s.bs_scan), scan_lds_bytes(s.kp), s.kp_dev,
                      -1ll, 0ll, 0ll, 0ll, 0, 0))) ||
        ((s.ev_stop_attach = timed && s.ext_events), false) ||
        (rc = launch(s, -1, (k_link<false, false, true>), dim3(std::min<uint32_t>(s.chain_l3_grid, s.grid_link)),
                     dim3(s.bs_link), link_lds_bytes(s.kp), s.kp_dev, -1ll, 0ll, 0ll, 0)))
      return rc;
    if (timed) {
      if ((rc = ev_end(s))) return rc;
    } else {
      s.launches[KS_LINK]++;
    }
    // (only the chain's last k_next publishes the control block to the host: the others skip the
    // host-memory writes and their system-scope fence)
    const uint32_t seq = k + 1 == K ? (s.next_seq = ++s.mseq) : 0u;
    ev_nx[k] = s.ev_used;
    if ((rc = launch(s, KS_AUX, k_next, dim3(nbn), dim3(1024), 0, s.kp_dev, kClrWin, seq, PredArgs{}, 0u))) return rc;
    if (s.ev_used == ev_nx[k]) ev_nx[k] = SIZE_MAX;  // (k_next untimed)
  }
  // the one sync: the last k_next's control block (readback without applying yet: the timing
  // events of the windows that did not run are dropped first)
  const size_t nb = sizeof(Ctl) + 8ull * s.B + 4ull * kMaxRanks;
  const int w = s.ctl_m ? mirror_wait(s, reinterpret_cast<uint32_t*>(s.ctl_m) + nb / 4, s.next_seq) : 1;
  if (w < 0) return w;
  if (w == 0) {
    std::memcpy(s.ctl_h, s.ctl_m, nb);
  } else {
    HIPCHK(hipMemcpyAsync(s.ctl_h, s.ctl_d, nb, hipMemcpyDeviceToHost, s.stream));
    if (!s.ctl_m) ++s.host_syncs;
    HIPCHK(hipStreamSynchronize(s.stream));
  }
  const long long* wv = s.ctl_h->win;
  const uint32_t done = static_cast<uint32_t>(std::min<long long>(wv[kWinCount], K));
  for (uint32_t k = done; k < K; ++k) {
    if (timed && ev_at[k] < s.ev_used) s.ev_class[ev_at[k]] = -1;
    if (ev_nx[k] < s.ev_used) s.ev_class[ev_nx[k]] = -1;
    s.launches[KS_LINK]--;
    s.launches[KS_AUX]--;
  }
  if ((rc = readback_apply(s))) return rc;
  if (done) {
    s.t_done = wv[kWinTDone];
    s.last_full = wv[kWinLastFull];
    s.grouped_cell = wv[kWinGrouped];
    s.cells += done;
    s.x_active = 0;
    s.start_pending = false;
  }
  s.chain_windows += done;
  s.chain_fr_hits += static_cast<uint64_t>(wv[kWinFrHits]);
  ++s.chains;
  // (the next chain: twice as long after a full one, as long as this one otherwise -- a window that
  // was never opened still costs its dispatches, one chain more costs a host sync)
  s.chain_k = done == K ? std::min<uint32_t>(2 * s.chain_k, 32) : std::max<uint32_t>(2, done);
  if (!done) {
    g_detail = "device window chain made no progress (k_win end reason " + std::to_string(wv[kWinDead]) + ")";
    return BCSIM_E_STATE;
  }
  return BCSIM_OK;
}

// Debug (BCSIM_CHECK_IDLE=1): the part [lo, hi) of cell `cell` that run() skips as
// idle (the tick's leading part, or a part cut by the run limit) must hold no node with work:
// k_active -- the rule every window uses -- runs for it and the run fails if either list is not
// empty.  The speculative lists of the next window are overwritten, so that window runs k_active
// itself.
static int check_idle_part(Sim& s, long long cell, long long lo, long long hi) {
  if (s.sparse) return BCSIM_OK;
  s.spec_seq = 0;
  HIPCHK(hipMemsetAsync(s.kp.act_n, 0, 16, s.stream));
  const uint64_t nl = static_cast<uint64_t>(s.R) * s.nloc;
  const uint64_t nb = std::max<uint64_t>((nl + kActChunk - 1) / kActChunk, std::min<uint64_t>(1024, (nl + 255) / 256));
  const uint32_t chunk = static_cast<uint32_t>(((nl + nb - 1) / nb + 255) / 256 * 256);
  int rc = launch(s, KS_AUX, k_active, dim3(static_cast<uint32_t>((nl + chunk - 1) / chunk)), dim3(256), 0, s.kp_dev, lo, hi,
                  static_cast<uint32_t>(cell % s.B), static_cast<uint32_t>((cell + kOpRing - 1) % kOpRing), chunk, ++s.mseq, 0);
  if (rc) return rc;
  uint32_t n[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(n, s.kp.act_n, 16, hipMemcpyDeviceToHost, s.stream));
  HIPCHK(hipStreamSynchronize(s.stream));
  if (n[0] || n[1]) {
    g_detail = "idle part [" + std::to_string(lo) + ", " + std::to_string(hi) + ") of cell " + std::to_string(cell) +
               " was skipped but k_active lists " + std::to_string(n[0]) + " / " + std::to_string(n[1]) + " nodes";
    return BCSIM_E_STATE;
  }
  HIPCHK(hipMemsetAsync(s.kp.act_n, 0, 16, s.stream));
  ++s.idle_checked;
  return BCSIM_OK;
}

static int run(Sim& s, int64_t t_until) {
  int rc;
  if (!s.started) {
    if ((rc = ensure_topology(s)) || (rc = setup_device(s))) return rc;
    s.started = true;
  }
  HIPCHK(hipSetDevice(s.dev));
  int64_t lim = t_until;
  if (s.cfg.t_end_ns > 0 && s.cfg.t_end_ns < lim) lim = s.cfg.t_end_ns;
  s.trace_valid = false;
  const long long L = s.L;
  // multi-GPU: a rank-local failure is never returned on its own between two
  // collectives; it rides the next one (next-cell MIN, the exchange counts, the v-log
  // SUM) so that every rank returns together (BCSIM_E_PEER on the others)
  int lerr = 0;
#define LOCAL(x)                                  \
  do {                                            \
    if (!lrc) {                                   \
      hipError_t e_ = (x);                        \
      if (e_ != hipSuccess) {                     \
        g_detail = std::string(#x) + ": " + hipGetErrorString(e_); \
        lrc = BCSIM_E_HIP;                        \
      }                                           \
    }                                             \
  } while (0)
  for (;;) {
    // earliest cell with work
    long long c;
    int carried = 0;  // node-partitioned: a failure after the last exchange, carried by this cell's
    if (s.xp && s.next_known) {
      // the last cell's control exchange agreed on this cell already
      s.next_known = false;
      c = s.next_cell;
      carried = lerr;
      lerr = 0;
    } else {
      c = local_next_cell(s, true);
      if (s.xp) {  // the next cell of the whole system, and every rank's status
        int64_t cv[2] = {c, lerr};
        if ((rc = s.xp->allreduce_i64(s.stream, cv, 2, 0))) return rc;
        ++s.ctl_collectives;
        ++s.host_syncs;
        if (cv[1] < 0) {
          if (lerr) return lerr;
          g_detail = "another rank of the partition failed";
          return BCSIM_E_PEER;
        }
        c = cv[0];
      } else if (lerr) {
        return lerr;
      }
    }
    if (c == LLONG_MAX || c * L >= lim) {
      if (lim != INT64_MAX) s.t_done = std::max<int64_t>(s.t_done, lim);
      if (s.xp && carried) {  // every rank leaves here: tell them, then leave with the failure
        int64_t cv[2] = {LLONG_MAX, carried};
        (void)s.xp->allreduce_i64(s.stream, cv, 2, 0);
        return carried;
      }
      if (s.xp) {  // the others may carry a failure into this exit
        int64_t cv[2] = {LLONG_MAX, 0};
        if ((rc = s.xp->allreduce_i64(s.stream, cv, 2, 0))) return rc;
        if (cv[1] < 0) {
          g_detail = "another rank of the partition failed";
          return BCSIM_E_PEER;
        }
      }
      break;
    }
    const long long cs = c * L, ce = cs + L;
    {
      static const bool cwlog = std::getenv("BCSIM_WINLOG") != nullptr;  // (debug: why this cell)
      if (cwlog) {
        uint32_t nb = 0;
        for (uint32_t b = 0; b < s.B; ++b) nb += s.bcnt[b] ? 1u : 0u;
        std::fprintf(stderr, "[cell] %lld t_done %lld next_local %lld next_timer %lld ov_min %lld busy buckets %u (this %u) tick %lld grouped %lld\n",
                     c, static_cast<long long>(s.t_done), s.next_local, s.next_timer, s.ov_min, nb, s.bcnt[c % s.B],
                     static_cast<long long>(s.next_tick), s.grouped_cell);
      }
    }
    const long long lo = std::max<long long>(cs, s.t_done);
    const long long hi = std::min<long long>(ce, lim);
    if (lo >= hi) {  // nothing left before the limit inside this cell
      if (lim != INT64_MAX) s.t_done = std::max<int64_t>(s.t_done, lim);
      // (node-partitioned: the exchange already agreed on this cell, so every rank is here; a
      // failure carried out of the last window leaves with every rank, as at the exit above)
      if (s.xp) {
        int64_t cv[2] = {LLONG_MAX, carried};
        if ((rc = s.xp->allreduce_i64(s.stream, cv, 2, 0))) return rc;
        ++s.ctl_collectives;
        if (carried) return carried;
        if (cv[1] < 0) {
          g_detail = "another rank of the partition failed";
          return BCSIM_E_PEER;
        }
      }
      break;
    }
    if (s.chain_on && s.cells > 0 && !s.start_pending && s.grouped_cell < 0 && s.xcnt[c % s.B] == 0 && s.next_timer >= lo &&
        !(s.ov_min <= c + static_cast<long long>(s.B) - 1) && !(lo <= 0 && 0 < hi) &&
        !(s.cfg.stop_ns >= 0 && lo <= s.cfg.stop_ns && s.cfg.stop_ns < hi)) {
      // no host work before this window (group_cell, START / STOP) and no ring-tag zeroing due in
      // [last_full + 1, c]: a device chain from here
      const long long t0 = (s.last_full + 1) / s.B;
      const long long z = (t0 % 32 == 31) ? s.last_full + 1 : ((t0 / 32) * 32 + 31) * static_cast<long long>(s.B);
      if (c < z) {
        if ((rc = run_chain(s, c, lim))) return rc;
        continue;
      }
    }
    int lrc = carried;  // this rank's status of the cell
    if (!lrc && s.grouped_cell != c) {
      // cells (last_full, c) had no work and were skipped: their buckets still owe the
      // once-per-32-turns zeroing of the inbox-slot tags (before group_cell can rebin into them)
      if (c > s.last_full + 1) lrc = zero_tag_buckets(s, s.last_full + 1, c - 1);
      if (!lrc) lrc = check_tag_invariant(s, c);
      if (!lrc) lrc = group_cell(s, c);
    }
    const bool tick = s.cfg.protocol == BCSIM_PBFT && s.n_alive > 0 && s.next_tick >= lo && s.next_tick < hi;
    if (tick) {
      const long long tk = s.next_tick;
      // the part of the cell before the tick, unless nothing can happen in it: no record in the
      // cell's bucket (slots, extras, rebinned overflow, reply slots due), no timer or pending op
      // before the tick (the end-of-window read-back), no START / STOP
      const bool idle = !s.xp && s.bcnt[c % s.B] == 0 && s.next_local >= tk && s.next_timer >= tk &&
                        !(lo <= 0 && 0 < tk) && !(s.cfg.stop_ns >= 0 && lo <= s.cfg.stop_ns && s.cfg.stop_ns < tk);
      if (!lrc && tk > lo && !idle) lrc = do_scan(s, c, lo, tk, cs, false);
      if (!lrc && tk > lo && idle) {
        ++s.idle_parts;
        if (s.check_idle) lrc = check_idle_part(s, c, lo, tk);
      }
      if (s.xp) {
        if ((rc = sync_vlog(s, lrc)) || (rc = sync_leaders(s))) return rc;
      } else if (lrc) {
        return lrc;
      }
      LOCAL(hipMemsetAsync(s.kp.scal + 2, 0, 8, s.stream));
      if (!lrc)
        lrc = launch(s, KS_AUX, k_pbft_tick, dim3(s.R), dim3(1024), static_cast<size_t>(s.N), s.kp_dev, tk);
      if (!lrc) lrc = do_scan(s, c, tk, hi, cs, hi == ce);
    } else if (!lrc) {
      // a part of a cell cut by the run limit (bcsim_run(t_until): the bench's step ends at the
      // next tick) in which nothing can happen -- the idle rule above, to the limit -- launches
      // nothing: it only moves t_done (no bucket is finished, so no clear or tag zeroing is due)
      const bool idle = s.cfg.protocol == BCSIM_PBFT && !s.xp && hi < ce && s.bcnt[c % s.B] == 0 && s.next_local >= hi &&
                        s.next_timer >= hi && !(lo <= 0 && 0 < hi) &&
                        !(s.cfg.stop_ns >= 0 && lo <= s.cfg.stop_ns && s.cfg.stop_ns < hi);
      if (idle) {
        if (s.check_idle && (rc = check_idle_part(s, c, lo, hi))) return rc;
        s.t_done = hi;
        ++s.cells;
        ++s.idle_parts;
        continue;
      }
      lrc = do_scan(s, c, lo, hi, cs, hi == ce);
    }
    if (!lrc && s.cfg.protocol == BCSIM_RAFT && s.cfg.rng_mode == BCSIM_RNG_GLIBC)
      lrc = launch(s, KS_AUX, k_draws, dim3(1), dim3(64), 0, s.kp_dev, 0u);
    // (one workgroup up to 4096 gnodes -- no cross-workgroup combine; above, 2048 per workgroup:
    // for gossip n=65536 the wider grid measured faster than four gnodes per lane)
    const uint32_t nbn = s.NT <= 4096u ? 1u : static_cast<uint32_t>(std::min<uint64_t>(kNextBlocks, (s.NT + 2047) / 2048));
    // (a finished cell's bucket is free again: k_next clears its counts and tile flags)
    const uint32_t clr_b = hi == ce ? static_cast<uint32_t>(c % s.B) : 0xFFFFFFFFu;
    if (!lrc && s.dbg_dev_err >= 0 && static_cast<long long>(s.cells) >= s.dbg_dev_err)
      lrc = launch(s, KS_AUX, k_dbg_err, dim3(1), dim3(64), 0, s.kp_dev);
    // speculation (dense PBFT, one rank, one k_next workgroup): k_next predicts the next window from
    // the state after this one -- the host's next-cell rule with its host-only terms passed in --
    // and k_active runs for it at once; the next do_scan uses its lists when the host's window is
    // the predicted one (else it resets them and runs k_active itself): one round trip less
    const bool spec = s.spec_on && !lrc && nbn == 1;
    PredArgs pa{};
    if (spec) {
      const long long td = hi;  // (t_done after this window)
      long long ch = LLONG_MAX;
      if (hi != ce) ch = c;  // (a part cell: grouped_cell stays)
      if (s.stop_pending && s.cfg.stop_ns >= 0 && s.cfg.stop_ns >= hi) ch = std::min<long long>(ch, s.cfg.stop_ns / L);
      int64_t tk = s.next_tick;
      const bool ticked = s.cfg.protocol == BCSIM_PBFT && s.n_alive > 0 && s.next_tick >= lo && s.next_tick < hi;
      if (ticked) tk = s.next_tick + s.kp.pbft_period;  // (the tick of this window is done)
      pa = PredArgs{td, static_cast<long long>(lim), (s.n_alive > 0 || ticked) ? static_cast<long long>(tk) : LLONG_MAX, ch,
                    s.cfg.stop_ns, 1};
    }
    s.next_seq = ++s.mseq;
    // (k_next builds the predicted window's lists itself unless BCSIM_FUSE_ACT=0: no k_active launch)
    const uint32_t fused_seq = spec && s.fuse_act ? ++s.mseq : 0u;
    if (!lrc) lrc = launch(s, KS_AUX, k_next, dim3(nbn), dim3(1024), 0, s.kp_dev, clr_b, s.next_seq, pa, fused_seq);
    if (!lrc && fused_seq) s.spec_seq = fused_seq;
    if (!lrc && spec && !fused_seq) {
      const uint64_t nl = static_cast<uint64_t>(s.R) * s.nloc;
      const uint64_t nb = std::max<uint64_t>((nl + kActChunk - 1) / kActChunk, std::min<uint64_t>(1024, (nl + 255) / 256));
      const uint32_t chunk = static_cast<uint32_t>(((nl + nb - 1) / nb + 255) / 256 * 256);
      s.spec_seq = ++s.mseq;
      lrc = launch(s, KS_AUX, k_active, dim3(static_cast<uint32_t>((nl + chunk - 1) / chunk)), dim3(256), 0, s.kp_dev, 0ll, 0ll,
                   0u, 0u, chunk, s.spec_seq, 1);
    }
    // (device control words: the read-back rides the exchange below)
    if (!lrc && !s.ctlw_d) lrc = readback(s, true);
    if (!lrc && s.dbg_fail_cell >= 0 && static_cast<long long>(s.cells) >= s.dbg_fail_cell) {
      g_detail = "injected failure (BCSIM_DBG_FAIL_CELL)";  // test hook: one rank fails alone
      lrc = BCSIM_E_OVERFLOW;
    }
    if (!s.xp && lrc) return lrc;
    // host bookkeeping of the finished window (before the exchange: the next-cell candidate a
    // rank announces there is its state after this window)
    s.start_pending = false;
    if (s.cfg.stop_ns >= 0 && s.cfg.stop_ns < hi) s.stop_pending = false;
    s.t_done = hi;
    ++s.cells;
    if (hi == ce) {
      const int zr = zero_tag_buckets(s, c, c);
      if (!lrc) lrc = zr;  // (node-partitioned: rides the exchange like any other rank-local failure)
      s.last_full = c;
      s.grouped_cell = -1;
      s.bcnt[c % s.B] = 0;
      s.xcnt[c % s.B] = 0;
      s.x_active = 0;
    }
    if (s.xp) {
      // ONE control exchange (segment sizes, next-cell candidates, status, PBFT n_alive), the
      // records for other ranks' nodes, k_import; the next cell is agreed there
      if ((rc = exchange(s, c, lrc, tick))) return rc;
      // the bucket counts after k_import (a failure here rides the next cell's exchange); with
      // nothing imported the end-of-cell read-back before the exchange is still current
      lerr = s.last_import ? readback(s) : 0;
      if (s.carry_err) {  // (the device-word exchange's late failure)
        lerr = s.carry_err;
        s.carry_err = 0;
      }
      if (!lerr && s.dbg_fail_import >= 0 && static_cast<long long>(s.cells) > s.dbg_fail_import) {
        g_detail = "injected failure after the exchange (BCSIM_DBG_FAIL_IMPORT)";  // test hook
        lerr = BCSIM_E_OVERFLOW;
      }
    } else {
      if (lrc) return lrc;
      if (tick) {
        s.n_alive = s.ctl_h->scal[2];
        s.next_tick += s.kp.pbft_period;
      }
    }
  }
#undef LOCAL
  if (s.xp && s.cfg.protocol == BCSIM_PBFT && (rc = sync_vlog(s))) return rc;
  // the end-of-window read-back spins on k_next's mirror word, not on the stream: the kernels
  // queued after it (the tag zeroing) must be done before the readers' null-stream copies
  HIPCHK(hipStreamSynchronize(s.stream));
  return BCSIM_OK;
}

static int fetch_trace(Sim& s) {
  if (s.trace_valid) return BCSIM_OK;
  s.trace.clear();
  if (!s.started) {
    s.trace_valid = true;
    return BCSIM_OK;
  }
  Ctl ctl;
  HIPCHK(hipMemcpy(&ctl, s.ctl_d, sizeof ctl, hipMemcpyDeviceToHost));
  const uint32_t n = std::min(ctl.trace_cnt, s.kp.cap_trace);
  s.trace.resize(n);
  if (n) HIPCHK(hipMemcpy(s.trace.data(), s.kp.trace, n * sizeof(bcsim_trace_rec), hipMemcpyDeviceToHost));
  // resolve the PBFT global `v` of commit lines from the v-log
  if (s.cfg.protocol == BCSIM_PBFT) {
    const uint32_t nv = std::min(ctl.vlog_cnt, s.kp.cap_vlog);
    std::vector<VLog> vl(nv);
    if (nv) HIPCHK(hipMemcpy(vl.data(), s.kp.vlog, nv * sizeof(VLog), hipMemcpyDeviceToHost));
    auto vless = [](const VLog& a, const VLog& b) {
      if (a.rep != b.rep) return a.rep < b.rep;
      if (a.t != b.t) return a.t < b.t;
      if (a.ts != b.ts) return a.ts < b.ts;
      if (a.origin != b.origin) return a.origin < b.origin;
      if (a.sub != b.sub) return a.sub < b.sub;
      return a.target < b.target;
    };
    std::sort(vl.begin(), vl.end(), vless);
    for (auto& r : s.trace) {
      if (r.kind != BCSIM_TR_PBFT_COMMIT || r.a != INT32_MIN) continue;
      VLog key{};
      key.rep = r.replica;
      key.t = r.t_ns;
      key.ts = r.key_ts;
      key.origin = r.key_origin;
      key.sub = r.key_sub;
      key.target = r.node;
      auto it = std::lower_bound(vl.begin(), vl.end(), key, vless);  // first >= key
      int32_t v = 1;
      if (it != vl.begin()) {
        auto prev = it - 1;
        if (prev->rep == r.replica) v = prev->v;
      }
      r.a = v;
    }
  }
  std::sort(s.trace.begin(), s.trace.end(), [](const bcsim_trace_rec& a, const bcsim_trace_rec& b) {
    if (a.replica != b.replica) return a.replica < b.replica;
    if (a.t_ns != b.t_ns) return a.t_ns < b.t_ns;
    if (a.key_ts != b.key_ts) return a.key_ts < b.key_ts;
    if (a.key_origin != b.key_origin) return a.key_origin < b.key_origin;
    if (a.key_sub != b.key_sub) return a.key_sub < b.key_sub;
    if (a.node != b.node) return a.node < b.node;
    return a.kind < b.kind;
  });
  s.trace_valid = true;
  return BCSIM_OK;
}

static int read_counters(Sim& s, bcsim_counters* out) {
  std::memset(out, 0, sizeof *out);
  if (!s.started) return BCSIM_OK;
  const size_t per = static_cast<size_t>(s.R) * CNT_N;
  std::vector<unsigned long long> cs(per * s.kp.cnt_stripes), c(per, 0);
  HIPCHK(hipMemcpy(cs.data(), s.kp.counters, cs.size() * 8, hipMemcpyDeviceToHost));
  for (uint32_t st = 0; st < s.kp.cnt_stripes; ++st)
    for (size_t k = 0; k < per; ++k) {
      const unsigned long long v = cs[st * per + k];
      if (k % CNT_N == CNT_TLAST)
        c[k] = st == 0 ? v : static_cast<unsigned long long>(std::max<long long>(static_cast<long long>(c[k]),
                                                                                  static_cast<long long>(v)));
      else
        c[k] += v;
    }
  Ctl ctl;
  HIPCHK(hipMemcpy(&ctl, s.ctl_d, sizeof ctl, hipMemcpyDeviceToHost));
  for (uint32_t r = 0; r < s.R; ++r) {
    const unsigned long long* x = &c[static_cast<size_t>(r) * CNT_N];
    for (int k = 0; k < BCSIM_MSG_TYPES; ++k) out->delivered[k] += x[CNT_DELIV + k];
    out->delivered_total += x[CNT_DELIV_TOTAL];
    out->echoes += x[CNT_ECHOES];
    out->sends += x[CNT_SENDS];
    out->dropped += x[CNT_DROPPED];
    out->wrong_msgs += x[CNT_WRONG];
    out->events += x[CNT_EVENTS];
    out->t_last_ns = std::max<int64_t>(out->t_last_ns, static_cast<int64_t>(x[CNT_TLAST]));
    out->frames_dropped += x[CNT_FDROP];
    out->msgs_lost += x[CNT_LOST];
  }
  out->trace_records = std::min(ctl.trace_cnt, s.kp.cap_trace);
  return BCSIM_OK;
}

static void destroy(Sim* s) {
  if (!s) return;
  if (s->started) (void)hipSetDevice(s->dev);
  for (void* q : s->allocs) (void)hipFree(q);
  for (auto& e : s->ev_pool) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (s->ctl_h) (void)hipHostFree(s->ctl_h);
  if (s->ctl_m) (void)hipHostFree(s->ctl_m);
  if (s->act_m) (void)hipHostFree(s->act_m);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  if (s->stream2) (void)hipStreamDestroy(s->stream2);
  if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
  if (s->ev_join) (void)hipEventDestroy(s->ev_join);
  delete s->xp;
  delete s;
}

}  // namespace bcsim

// ===========================================================================
// C ABI (include/bcsim.h)
using bcsim::Sim;

struct bcsim_sim {
  Sim* s;
};

extern "C" {

int bcsim_config_default(bcsim_config* c, uint32_t protocol, uint32_t n_nodes) {
  if (!c || protocol > BCSIM_GOSSIP) return BCSIM_E_INVAL;
  std::memset(c, 0, sizeof *c);
  c->abi_version = BCSIM_ABI_VERSION;
  c->protocol = protocol;
  c->n_nodes = n_nodes;
  c->n_replicas = 1;
  c->link_rate_bps = 3000000;       // blockchain-simulator.cc:23 "3Mbps"
  c->link_delay_ns = 3000000;       // :24 "3ms"
  c->mtu = 1500;
  c->delay_mode = BCSIM_DELAY_RANDOM;
  c->app_delay_ns = 0;
  c->rng_mode = BCSIM_RNG_GLIBC;
  c->time_round = BCSIM_TIME_ROUND;
  c->seed = 1;                      // rand() is never seeded: srand(1)
  c->encoding = BCSIM_ENC_EXTENDED;
  c->echo = 1;
  c->t_end_ns = 0;
  c->stop_ns = 10000000000ll;       // :55 Stop(Seconds(10.0))
  c->pbft_rounds = 40;              // pbft-node.cc:407
  c->pbft_block_bytes = 0;
  c->pbft_timeout_s = 0.05f;        // :106
  c->pbft_view_change = 1;
  c->pbft_seq_cap = 1000;           // TX tx[1000]
  c->raft_blocks = 50;              // raft-node.cc:248
  c->raft_proposal_bytes = 0;
  c->raft_heartbeat_s = 0.05f;      // :80
  c->raft_proposal_rounds = 50;     // :361
  c->raft_proposal_delay_ns = 1000000000ll;  // :216 Seconds(1)
  c->paxos_proposers = 3;           // paxos-node.cc:136
  c->queue_model = BCSIM_QUEUE_INFINITE;
  c->queue_dev_pkts = 100;          // PointToPointNetDevice TxQueue DropTail "100p"
  c->queue_disc_pkts = 1000;        // pfifo_fast "1000p" (default root queue disc)
  return BCSIM_OK;
}

int bcsim_create(const bcsim_config* cfg, bcsim_sim** out) {
  if (!cfg || !out) return BCSIM_E_INVAL;
  int rc = bcsim::validate(*cfg);
  if (rc) return rc;
  Sim* s = new (std::nothrow) Sim();
  if (!s) return BCSIM_E_NOMEM;
  s->cfg = *cfg;
  if (s->cfg.n_replicas == 0) s->cfg.n_replicas = 1;
  if (s->cfg.pbft_seq_cap == 0) s->cfg.pbft_seq_cap = 1000;
  s->N = cfg->n_nodes;
  s->R = s->cfg.n_replicas;
  if (static_cast<uint64_t>(s->N) * s->R > 0xFFFFFFF0ull) {
    delete s;
    return BCSIM_E_UNSUPPORTED;
  }
  s->NT = s->N * s->R;
  s->nloc = s->N;
  bcsim_sim* h = new (std::nothrow) bcsim_sim{s};
  if (!h) {
    delete s;
    return BCSIM_E_NOMEM;
  }
  *out = h;
  return BCSIM_OK;
}

int bcsim_set_topology_csr(bcsim_sim* h, uint32_t n, const uint32_t* row_ptr, const uint32_t* col_idx,
                           const int64_t* prop_ns) {
  if (!h || !row_ptr || !col_idx || n != h->s->N) return BCSIM_E_INVAL;
  Sim& s = *h->s;
  if (s.started) return BCSIM_E_STATE;
  const uint32_t E = row_ptr[n];
  s.row.assign(row_ptr, row_ptr + n + 1);
  s.col.assign(col_idx, col_idx + E);
  if (prop_ns)
    s.prop.assign(prop_ns, prop_ns + E);
  else
    s.prop.assign(E, s.cfg.link_delay_ns);
  for (uint32_t i = 0; i < n; ++i)
    if (s.row[i + 1] < s.row[i]) return BCSIM_E_INVAL;
  int rc = bcsim::build_rev(s);
  if (rc) return rc;
  s.E = E;
  s.deg_max = 0;
  for (uint32_t i = 0; i < n; ++i) s.deg_max = std::max(s.deg_max, s.row[i + 1] - s.row[i]);
  s.topo_ready = true;
  return BCSIM_OK;
}

int bcsim_run(bcsim_sim* h, int64_t t_until_ns) {
  if (!h) return BCSIM_E_INVAL;
  Sim& s = *h->s;
  if (s.err) return s.err;
  int rc = bcsim::run(s, t_until_ns);
  if (rc) s.err = rc;
  if (s.kp.fqlog) {  // debug (BCSIM_FQLOG=<file>): the FQCODEL link events so far
    uint32_t n = 0;
    if (hipMemcpy(&n, s.kp.fqlog_n, 4, hipMemcpyDeviceToHost) == hipSuccess) {
      n = std::min(n, s.kp.cap_fqlog);
      std::vector<uint4> v(2ull * n);
      if (n && hipMemcpy(v.data(), s.kp.fqlog, v.size() * 16, hipMemcpyDeviceToHost) != hipSuccess) n = 0;
      if (FILE* f = std::fopen(std::getenv("BCSIM_FQLOG"), "wb")) {
        std::fwrite(v.data(), 16, 2ull * n, f);
        std::fclose(f);
      }
    }
  }
  return rc;
}

int bcsim_read_trace(bcsim_sim* h, bcsim_trace_rec* buf, uint64_t cap, uint64_t* n_out) {
  if (!h || !n_out) return BCSIM_E_INVAL;
  int rc = bcsim::fetch_trace(*h->s);
  if (rc) return rc;
  const auto& t = h->s->trace;
  *n_out = t.size();
  if (buf) std::memcpy(buf, t.data(), std::min<uint64_t>(cap, t.size()) * sizeof(bcsim_trace_rec));
  return BCSIM_OK;
}

int bcsim_read_counters(bcsim_sim* h, bcsim_counters* out) {
  if (!h || !out) return BCSIM_E_INVAL;
  return bcsim::read_counters(*h->s, out);
}

int bcsim_read_status(bcsim_sim* h, bcsim_status* out) {
  if (!h || !out) return BCSIM_E_INVAL;
  Sim& s = *h->s;
  std::memset(out, 0, sizeof *out);
  out->now_ns = s.t_done;
  long long nx = LLONG_MAX;
  if (s.started) {
    for (uint32_t b = 0; b < s.B; ++b)
      if (s.bcnt[b]) nx = std::min<long long>(nx, s.t_done);  // cell granularity
    nx = std::min(nx, s.next_local);
    if (s.ov_min != LLONG_MAX) nx = std::min<long long>(nx, s.ov_min * s.L);
    if (s.n_alive > 0) nx = std::min<long long>(nx, s.next_tick);
    if (s.stop_pending && s.cfg.stop_ns >= s.t_done) nx = std::min<long long>(nx, s.cfg.stop_ns);
  } else {
    nx = 0;
  }
  out->next_ns = nx;
  out->cells = s.cells;
  out->quiescent = nx == LLONG_MAX;
  out->error = s.err;
  out->lookahead_ns = s.L;
  return BCSIM_OK;
}

int bcsim_destroy(bcsim_sim* h) {
  if (!h) return BCSIM_OK;
  bcsim::destroy(h->s);
  delete h;
  return BCSIM_OK;
}

const char* bcsim_strerror(int code) {
  switch (code) {
    case BCSIM_OK: return "ok";
    case BCSIM_E_INVAL: return "invalid argument";
    case BCSIM_E_NOMEM: return "out of memory";
    case BCSIM_E_HIP: return "HIP runtime error";
    case BCSIM_E_OVERFLOW: return "engine buffer capacity exceeded";
    case BCSIM_E_UNSUPPORTED: return "configuration not supported by the GPU engine";
    case BCSIM_E_ENCODING: return "compat encoding hit reference undefined behaviour";
    case BCSIM_E_TIE: return "tie-order precondition violated";
    case BCSIM_E_NODEVICE: return "no HIP device";
    case BCSIM_E_STATE: return "call out of order";
    case BCSIM_E_INDEX: return "PBFT tx[] index out of range";
    case BCSIM_E_PEER: return "another rank of the partition failed";
    default: return "unknown error";
  }
}

const char* bcsim_last_error_detail(void) { return bcsim::g_detail.c_str(); }

int bcsim_read_kernel_stats(bcsim_sim* h, double* us_out4, double* bytes_out4, uint64_t* launches_out4) {
  if (!h) return BCSIM_E_INVAL;
  Sim& s = *h->s;
  unsigned long long ks[8] = {0};
  if (bcsim::ev_collect(s)) return BCSIM_E_HIP;
  if (s.started) {
    unsigned long long kss[8 * bcsim::kKstStripes];
    hipError_t e = hipMemcpy(kss, s.kp.kstat, sizeof kss, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return BCSIM_E_HIP;
    for (uint32_t st = 0; st < bcsim::kKstStripes; ++st)
      for (int k = 0; k < 8; ++k) ks[k] += kss[8 * st + k];
  }
  for (int k = 0; k < 4; ++k) {
    if (us_out4) us_out4[k] = s.us[k];
    if (launches_out4) launches_out4[k] = s.launches[k];
  }
  if (bytes_out4) {
    // [link]: algorithmic bytes of the inbox scatter, SURVEY.md §8(d): 48 B per record
    // emitted (16 B record write + 16 B read by the receiver + 16 B busy_until read+write).
    // [scan]: 16 B per delivered record read.  [aux]: device-counted implementation bytes
    // of k_link (32 B per due op read, 16 B per record, 8 B per touched edge's link word
    // read+write, 32 B per kept op, 32 B per implicit echo read+clear).
    bytes_out4[bcsim::KS_LINK] = 48.0 * ks[bcsim::KST_REC];
    bytes_out4[bcsim::KS_SCAN] = 16.0 * ks[bcsim::KST_DELIV];
    bytes_out4[bcsim::KS_GROUP] = 0;
    bytes_out4[bcsim::KS_AUX] = 32.0 * ks[bcsim::KST_OPS] + 16.0 * ks[bcsim::KST_REC] + 16.0 * ks[bcsim::KST_EDGES] +
                                32.0 * ks[bcsim::KST_KEPT] + 32.0 * ks[bcsim::KST_ECHO];
  }
  return BCSIM_OK;
}

int bcsim_read_loop_stats(bcsim_sim* h, uint64_t* out4) {
  if (!h || !out4) return BCSIM_E_INVAL;
  const Sim& s = *h->s;
  out4[0] = s.cells;
  out4[1] = s.ctl_collectives;
  out4[2] = s.tag_zeroes;
  out4[3] = 0;
  return BCSIM_OK;
}

int bcsim_read_loop_stats_ex(bcsim_sim* h, uint64_t* out8) {
  if (!h || !out8) return BCSIM_E_INVAL;
  const Sim& s = *h->s;
  out8[0] = s.cells;
  out8[1] = s.ctl_collectives;
  out8[2] = s.tag_zeroes;
  out8[3] = s.spec_hits;
  out8[4] = s.idle_parts;
  out8[5] = s.host_syncs;
  out8[6] = s.idle_checked;
  out8[7] = s.chain_windows;
  return BCSIM_OK;
}

int bcsim_read_host_stats(bcsim_sim* h, double* out4) {
  if (!h || !out4) return BCSIM_E_INVAL;
  const Sim& s = *h->s;
  out4[0] = s.host_launch_us;
  out4[1] = s.host_wait_us;
  out4[2] = static_cast<double>(s.host_launches);
  out4[3] = static_cast<double>(s.chain_fr_hits);
  return BCSIM_OK;
}

int bcsim_read_engine_counters(bcsim_sim* h, uint64_t* out8) {
  if (!h || !out8) return BCSIM_E_INVAL;
  Sim& s = *h->s;
  for (int k = 0; k < 8; ++k) out8[k] = 0;
  if (!s.started) return BCSIM_OK;
  unsigned long long kss[8 * bcsim::kKstStripes];
  if (hipMemcpy(kss, s.kp.kstat, sizeof kss, hipMemcpyDeviceToHost) != hipSuccess) return BCSIM_E_HIP;
  for (uint32_t st = 0; st < bcsim::kKstStripes; ++st)
    for (int k = 0; k < 8; ++k) out8[k] += kss[8 * st + k];
  return BCSIM_OK;
}

int bcsim_set_partition(bcsim_sim* h, uint32_t rank, uint32_t nranks, const bcsim_transport* t) {
  if (!h || !t || !t->allreduce_i64 || !t->alltoallv || nranks == 0 || rank >= nranks) return BCSIM_E_INVAL;
  Sim& s = *h->s;
  if (s.started) return BCSIM_E_STATE;
  auto* x = new (std::nothrow) bcsim::CbXport();
  if (!x) return BCSIM_E_NOMEM;
  x->t = *t;
  x->rank = rank;
  x->nranks = nranks;
  delete s.xp;
  s.xp = x;
  s.P = nranks;
  s.prank = rank;
  return BCSIM_OK;
}

int bcsim_rccl_unique_id(void* out, uint64_t cap, uint64_t* n_out) {
#ifdef HIPEMU
  return BCSIM_E_UNSUPPORTED;
#else
  if (!out || !n_out || cap < sizeof(ncclUniqueId)) return BCSIM_E_INVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return BCSIM_E_HIP;
  std::memcpy(out, &id, sizeof id);
  *n_out = sizeof id;
  return BCSIM_OK;
#endif
}

int bcsim_set_partition_rccl(bcsim_sim* h, uint32_t rank, uint32_t nranks, const void* unique_id,
                             uint64_t id_bytes) {
#ifdef HIPEMU
  return BCSIM_E_UNSUPPORTED;
#else
  if (!h || !unique_id || id_bytes != sizeof(ncclUniqueId) || nranks == 0 || rank >= nranks) return BCSIM_E_INVAL;
  Sim& s = *h->s;
  if (s.started) return BCSIM_E_STATE;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return BCSIM_E_NODEVICE;
  if (hipSetDevice(static_cast<int>(s.cfg.device) % ndev) != hipSuccess) return BCSIM_E_HIP;
  auto* x = new (std::nothrow) bcsim::RcclXport();
  if (!x) return BCSIM_E_NOMEM;
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof id);
  const int rc = x->init(rank, nranks, id);
  if (rc) {
    delete x;
    return rc;
  }
  delete s.xp;
  s.xp = x;
  s.P = nranks;
  s.prank = rank;
  return BCSIM_OK;
#endif
}

int bcsim_reset_kernel_stats(bcsim_sim* h) {
  if (!h) return BCSIM_E_INVAL;
  Sim& s = *h->s;
  s.ev_used = 0;  // (timings not read yet belong to the old period)
  for (int k = 0; k < 4; ++k) {
    s.us[k] = 0;
    s.launches[k] = 0;
  }
  if (s.started && hipMemset(s.kp.kstat, 0, 64 * bcsim::kKstStripes) != hipSuccess) return BCSIM_E_HIP;
  return BCSIM_OK;
}

}  // extern "C"
