// engine.hip — MI355X (gfx950) consensus-propagation engine.
//
// Replaces the ns-3 per-packet event loop (Simulator::Run,
// blockchain-simulator.cc:57) that drives PbftNode / RaftNode / PaxosNode
// (pbft/, raft/, paxos/) with a windowed, time-stepped conservative engine:
//
//   time is cut into cells of length L = min link latency (propagation +
//   serialization of the smallest message).  Nothing sent in cell g can be
//   delivered before cell g+1, so every node's events of one cell are
//   independent of every other node's and are processed in parallel:
//
//   per cell g:
//     k_count / k_offsets / k_place   group the arrivals of cell g (bucket
//                                     g % B) by destination node
//     k_scan<P>                       one workgroup per node: LDS bitonic sort
//                                     of its arrivals by the canonical key,
//                                     then the protocol state machine in key
//                                     order; emits link ops, timers, traces
//     k_link                          one workgroup per node: per out-edge FIFO
//                                     (busy_until), serialization + propagation,
//                                     scatter of 32-byte arrival records into
//                                     the time-bucketed inboxes (chunked,
//                                     workgroup-aggregated atomics)
//     (PBFT) k_pbft_tick              the 50 ms SendBlock tick of every node,
//                                     which touches the file-scope globals
//                                     n, n_round, v (pbft-node.cc:24-30)
//     (Raft, glibc rng) k_draws       election-timeout draws in canonical
//                                     global order
//
// Semantics are specified in DESIGN.md §2 and restated serially by oracle/
// (the parity checker).  No code here calls the oracle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "engine.h"
#include "host_math.h"

namespace bcsim {

// ---------------------------------------------------------------------------
// kernel parameter block (passed by value)
struct KP {
  uint32_t N, R, NT, E;
  uint32_t protocol, delay_mode, rng_mode, encoding, echo;
  uint32_t deg_max;
  int64_t L;
  int64_t app_delay;
  int64_t tx_tot[2], tx_last[2];
  int64_t pbft_period, raft_hb, raft_prop_delay, stop_ns;
  uint32_t pbft_rounds, pbft_seq_cap, pbft_view_change, raft_blocks;
  uint32_t raft_prop_rounds, paxos_proposers;
  uint64_t seed;
  int64_t *pbft_delay, *raft_delay, *raft_elec, *paxos_delay;
  int64_t* jit_delay;  // the running protocol's getRandomDelay table
  uint32_t jit_mod;
  // topology (per replica, shared)
  const uint32_t *row, *col, *rev;
  const int64_t* prop;
  // common node state
  uint32_t* sub;
  uint64_t* draws;
  // PBFT
  int32_t *leader, *block_num;
  uint8_t* tick_alive;
  uint32_t* tick_sub;
  int32_t *tx_val, *tx_pv, *tx_cv;
  int32_t *g_n, *g_nround;  // per replica
  // Raft / Paxos
  int32_t *is_leader, *has_voted, *m_value, *vote_s, *vote_f, *acv, *blockNum, *round;
  uint32_t *next_election, *next_heartbeat;
  int32_t *t_max, *command, *t_store, *ticket, *is_commit, *proposal;
  // timers / ops
  TimerEnt* timers;
  uint32_t cap_timers;
  Op* ops;
  uint32_t* n_ops;
  uint32_t cap_ops;
  // links
  int64_t* busy;
  // buckets / grouping
  Rec* bucket;
  uint32_t* bucket_cnt;
  uint32_t n_buckets, cap_bucket;
  OvRec* ov;
  uint32_t* ov_cnt;
  uint32_t cap_ov;
  uint32_t *seg_cnt, *seg_off, *cursor;
  Rec* grp;
  uint32_t cap_arr;  // LDS sort capacity (power of two)
  // outputs
  bcsim_trace_rec* trace;
  uint32_t* trace_cnt;
  uint32_t cap_trace;
  VLog* vlog;
  uint32_t* vlog_cnt;
  uint32_t cap_vlog;
  DrawReq* dreq;
  uint32_t* dreq_cnt;
  uint32_t cap_dreq;
  const int32_t* glibc;
  uint32_t glibc_len;
  uint32_t* glibc_pos;  // per replica
  unsigned long long* counters;  // R * CNT_N
  unsigned long long* kstat;     // link kernel algorithmic counters
  int32_t* err;
  int32_t* dbg;  // BCSIM_CHECKED builds: first out-of-bounds source line
  unsigned long long* trail;  // BCSIM_CHECKED + BCSIM_TRAIL: host-mapped breadcrumbs
  uint64_t cap_E, cap_EB, cap_txn, cap_glibc;
  long long *node_tnext, *node_onext;
  long long* scal;  // [0] next_local, [1] ov_min_cell, [2] n_alive_ticks
};

// ---------------------------------------------------------------------------
// device helpers
// First error wins; its source line goes to p.dbg so the host can name the
// exact capacity or invariant that failed (bcsim_last_error_detail).
__device__ inline void set_err_(const KP& p, int32_t code, int line) {
  if (atomicCAS(p.err, 0, code) == 0) atomicCAS(p.dbg, 0, line);
}
#define set_err(pp, code) set_err_((pp), (code), __LINE__)

__device__ __attribute__((aligned(64))) char g_dummy[256];

// Checked array access.  In BCSIM_CHECKED builds an out-of-range index is
// recorded (source line in p.dbg, BCSIM_E_OVERFLOW in p.err) and redirected
// to a per-thread dummy element instead of faulting the GPU.
template <typename T>
__device__ inline T& at_(const KP& p, T* base, uint64_t idx, uint64_t cap, int line) {
#ifdef BCSIM_CHECKED
  if (idx >= cap) {
    atomicCAS(p.dbg, 0, line);
    atomicCAS(p.err, 0, BCSIM_E_OVERFLOW);
    __builtin_amdgcn_endpgm();  // stop this wave: no access through garbage
  }
#endif
  return base[idx];
}
#ifdef BCSIM_CHECKED
#define BAIL_IF_ERR() \
  do {                \
    if (*p.err) return; \
  } while (0)
#else
#define BAIL_IF_ERR() \
  do {                \
  } while (0)
#endif
#ifdef BCSIM_CHECKED
#define TRAIL_AT(pp, g)                                                                        \
  do {                                                                                         \
    if ((pp).trail)                                                                            \
      __hip_atomic_store(&(pp).trail[g], (static_cast<unsigned long long>(g) << 32) | __LINE__, \
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);                          \
  } while (0)
#else
#define TRAIL_AT(pp, g) \
  do {                  \
  } while (0)
#endif
#define TRAIL(c) TRAIL_AT(*(c).p, (c).g)
#define AT(arr, idx, cap) at_(p, (arr), static_cast<uint64_t>(idx), static_cast<uint64_t>(cap), __LINE__)

struct Key {
  int64_t t, ts;
  uint32_t origin, sub;
};
__device__ inline bool key_less(const Key& a, const Key& b) {
  if (a.t != b.t) return a.t < b.t;
  if (a.ts != b.ts) return a.ts < b.ts;
  if (a.origin != b.origin) return a.origin < b.origin;
  return a.sub < b.sub;
}

__device__ inline uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// order-independent rand(): splitmix64(seed, replica, node, draw index)
__device__ inline int32_t ctr_rand(uint64_t seed, uint32_t rep, uint32_t node, uint64_t k) {
  uint64_t h = sm64(seed);
  h = sm64(h ^ static_cast<uint64_t>(rep));
  h = sm64(h ^ static_cast<uint64_t>(node));
  h = sm64(h ^ k);
  return static_cast<int32_t>(h >> 33);
}

// getRandomDelay() of the running protocol: jit_delay/jit_mod are chosen on
// the host (pbft-node.cc:68 / raft-node.cc:65 / paxos-node.cc:399).  A
// device-side three-way branch on p.protocol here was miscompiled by the
// ROCm 7.2 compiler in divergent code (the paxos arm used an unset address
// register -> aperture violation), so there is deliberately no branch.
__device__ inline int64_t delay_from_draw(const KP& p, int32_t r) {
  return AT(p.jit_delay, static_cast<uint32_t>(r) % p.jit_mod, p.jit_mod);
}

// intToChar through the wire (raw char code); compat = signed char wrap
__device__ inline int32_t enc_raw(const KP& p, int32_t a) {
  int32_t c = a + '0';
  if (p.encoding == BCSIM_ENC_COMPAT) c = static_cast<int32_t>(static_cast<int8_t>(static_cast<uint8_t>(c)));
  return c;
}
__device__ inline int16_t to16(const KP& p, int32_t c) {
  if (c > 32767 || c < -32768) set_err(p, BCSIM_E_OVERFLOW);
  return static_cast<int16_t>(c);
}

struct Msg {
  int32_t type;
  int32_t f[3];
  int32_t big;
};
// msg[i] after getPacketContent's NUL truncation (pbft-node.cc:305-320)
__device__ inline int32_t mch(const Msg& m, int i) {
  if (i == 0) return m.type + '0';
  for (int k = 0; k < i - 1; ++k)
    if (m.f[k] == 0) return 0;
  return m.f[i - 1];
}
__device__ inline int32_t c2i(int32_t c) { return c - '0'; }

// ---------------------------------------------------------------------------
// grouping: counting sort of bucket records by destination node
__global__ void k_count(const KP* __restrict__ pk, uint32_t b, uint32_t n) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t d = AT(p.bucket, static_cast<size_t>(b) * p.cap_bucket + k, static_cast<uint64_t>(p.n_buckets) * p.cap_bucket).dest;
  if (d != kInvalid) atomicAdd(&AT(p.seg_cnt, d, p.NT), 1u);
}

// single-block exclusive scan of seg_cnt[0..NT) -> seg_off[0..NT]
__global__ __launch_bounds__(1024) void k_offsets(const KP* __restrict__ pk) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < p.NT; base += 1024) {
    const uint32_t idx = base + tid;
    const uint32_t v = idx < p.NT ? AT(p.seg_cnt, idx, p.NT) : 0u;
    // inclusive wave scan
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off, 64);
      if (lane >= static_cast<uint32_t>(off)) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      for (int k = 0; k < 16; ++k) {
        const uint32_t s = wsum[k];
        wsum[k] = acc;
        acc += s;
      }
    }
    __syncthreads();
    const uint32_t excl = carry + wsum[w] + x - v;
    if (idx < p.NT) AT(p.seg_off, idx, p.NT + 1) = excl;
    __syncthreads();
    if (tid == 1023) carry = excl + v;
    __syncthreads();
  }
  if (tid == 0) AT(p.seg_off, p.NT, p.NT + 1) = carry;
}

__global__ void k_place(const KP* __restrict__ pk, uint32_t b, uint32_t n) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const Rec r = AT(p.bucket, static_cast<size_t>(b) * p.cap_bucket + k, static_cast<uint64_t>(p.n_buckets) * p.cap_bucket);
  if (r.dest == kInvalid) return;
  const uint32_t pos = AT(p.seg_off, r.dest, p.NT + 1) + atomicAdd(&AT(p.cursor, r.dest, p.NT), 1u);
  AT(p.grp, pos, p.cap_bucket) = r;
}

// move far-future arrivals whose cell entered the ring into their bucket
__global__ void k_rebin(const KP* __restrict__ pk, long long g_cur, uint32_t n) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  OvRec& o = AT(p.ov, k, p.cap_ov);
  if (o.cell < 0) return;
  if (o.cell < g_cur + static_cast<long long>(p.n_buckets)) {
    const uint32_t b = static_cast<uint32_t>(o.cell % p.n_buckets);
    const uint32_t pos = atomicAdd(&p.bucket_cnt[b], 1u);
    if (pos >= p.cap_bucket) {
      set_err(p, BCSIM_E_OVERFLOW);
      return;
    }
    AT(p.bucket, static_cast<size_t>(b) * p.cap_bucket + pos, static_cast<uint64_t>(p.n_buckets) * p.cap_bucket) = o.r;
    o.cell = -1;
  } else {
    atomicMin(&p.scal[1], o.cell);
  }
}

// ---------------------------------------------------------------------------
// per-node serial protocol context (thread 0 of the node's workgroup)
struct Ctx {
  const KP* p;
  uint32_t g, rep, i, deg;
  Key cur;  // key of the executing event
  uint32_t sub;
  uint64_t draws;
  Op* ops;
  uint32_t nops;
  TimerEnt* tm;  // LDS copy of the node's timers
  uint32_t cap_t;
  unsigned long long deliv[BCSIM_MSG_TYPES];
  unsigned long long echoes, wrong, events;
};

__device__ inline void ctx_trace(Ctx& c, uint32_t kind, int32_t a, int32_t b, int32_t cc) {
  const KP& p = *c.p;
  TRAIL(c);
  const uint32_t pos = atomicAdd(p.trace_cnt, 1u);
  if (pos >= p.cap_trace) {
    set_err(p, BCSIM_E_OVERFLOW);
    return;
  }
  bcsim_trace_rec r;
  r.t_ns = c.cur.t;
  r.key_ts = c.cur.ts;
  r.key_origin = c.cur.origin;
  r.key_sub = c.cur.sub;
  r.replica = c.rep;
  r.node = c.i;
  r.kind = kind;
  r.a = a;
  r.b = b;
  r.c = cc;
  AT(p.trace, pos, p.cap_trace) = r;
}

__device__ inline void ctx_op(Ctx& c, const Op& o) {
  const KP& p = *c.p;
  TRAIL(c);
  if (c.nops >= c.p->cap_ops) {
    set_err(*c.p, BCSIM_E_OVERFLOW);
    return;
  }
  AT(c.ops, c.nops++, p.cap_ops) = o;
}

__device__ inline Op mk_op(const KP& p, int64_t t, uint32_t dt, uint32_t origin, uint32_t sub,
                           uint32_t edge, const Msg& m, uint8_t kind, uint8_t flags) {
  Op o;
  o.t = t;
  o.dt = dt;
  o.origin = origin;
  o.sub = sub;
  o.edge = edge;
  o.f0 = to16(p, m.f[0]);
  o.f1 = to16(p, m.f[1]);
  o.f2 = to16(p, m.f[2]);
  o.type = static_cast<uint8_t>(m.type);
  o.kind_flags = static_cast<uint8_t>(kind | ((flags | (m.big ? OPF_BIG : 0)) << 2));
  return o;
}

__device__ inline int32_t ctx_draw(Ctx& c) {
  const KP& p = *c.p;
  TRAIL(c);
  if (p.rng_mode == BCSIM_RNG_COUNTER) return ctr_rand(p.seed, c.rep, c.i, c.draws++);
  set_err(p, BCSIM_E_UNSUPPORTED);  // glibc draws inside a cell: unsupported
  return 0;
}

// Simulator::Schedule(Seconds(getRandomDelay()), SendPacket, ...) x peers
__device__ void ctx_bcast(Ctx& c, const Msg& m, bool paxos) {
  const KP& p = *c.p;
  TRAIL(c);
  const uint8_t fl = paxos ? OPF_PAXOS : 0;
  if (p.delay_mode == BCSIM_DELAY_FIXED) {
    ctx_op(c, mk_op(p, c.cur.t + p.app_delay, static_cast<uint32_t>(p.app_delay), c.i, c.sub, 0, m,
                    OP_BCAST, fl));
  } else {
    // jitter: expanded per edge by k_link; edge field carries the draw base
    Op o = mk_op(p, c.cur.t, 0, c.i, c.sub, static_cast<uint32_t>(c.draws), m, OP_BCAST_J, fl);
    ctx_op(c, o);
    c.draws += c.deg;
  }
  c.sub += c.deg;
}

// Send(data, from): reply on the reverse edge of the arrival
// out_edge = the reverse of the arrival's edge (resolved when the arrival was
// staged into LDS)
__device__ void ctx_unicast(Ctx& c, uint32_t out_edge, const Msg& m) {
  const KP& p = *c.p;
  TRAIL(c);
  const int64_t d = p.delay_mode == BCSIM_DELAY_FIXED ? p.app_delay : delay_from_draw(p, ctx_draw(c));
  TRAIL(c);
  ctx_op(c, mk_op(p, c.cur.t + d, static_cast<uint32_t>(d), c.i, c.sub++, out_edge, m,
                  OP_SEND, 0));
}

__device__ uint32_t ctx_timer(Ctx& c, uint8_t kind, int64_t delay, bool pending = false) {
  const uint32_t id = c.sub++;
  for (uint32_t k = 0; k < c.cap_t; ++k) {
    if (!c.tm[k].alive) {
      c.tm[k].t = pending ? INT64_MAX : c.cur.t + delay;
      c.tm[k].ts = c.cur.t;
      c.tm[k].sub = id;
      c.tm[k].kind = kind;
      c.tm[k].alive = 1;
      c.tm[k].pending_draw = pending ? 1 : 0;
      return id;
    }
  }
  set_err(*c.p, BCSIM_E_OVERFLOW);
  return id;
}

__device__ void ctx_cancel(Ctx& c, uint32_t id) {
  if (id == 0) return;
  for (uint32_t k = 0; k < c.cap_t; ++k)
    if (c.tm[k].alive && c.tm[k].sub == id) c.tm[k].alive = 0;
}

__device__ inline Msg mkmsg(int32_t type, int32_t f0, int32_t f1, int32_t f2, int32_t big) {
  Msg m;
  m.type = type;
  m.f[0] = f0;
  m.f[1] = f1;
  m.f[2] = f2;
  m.big = big;
  return m;
}

// ---------------------------------------------------------------------------
// PBFT handlers (pbft/pbft-node.cc).  Message types pbft-node.h:80-91.
enum { PB_PRE_PREPARE = 1, PB_PREPARE = 2, PB_COMMIT = 3, PB_PREPARE_RES = 5, PB_VIEW_CHANGE = 8 };

struct PbftState {
  int32_t leader, block_num;
};

__device__ bool pbft_index(const KP& p, int32_t idx) {
  if (idx < 0) {
    set_err(p, BCSIM_E_ENCODING);
    return false;
  }
  if (static_cast<uint32_t>(idx) >= p.pbft_seq_cap) {
    set_err(p, BCSIM_E_INDEX);
    return false;
  }
  return true;
}

__device__ void pbft_recv(Ctx& c, PbftState& s, const Msg& m, uint32_t back_edge) {
  const KP& p = *c.p;
  const size_t base = static_cast<size_t>(c.g) * p.pbft_seq_cap;
  const int32_t N = static_cast<int32_t>(p.N);
  switch (c2i(mch(m, 0))) {
    case PB_PRE_PREPARE: {  // :193-211
      const Msg r = mkmsg(PB_PREPARE, mch(m, 1), mch(m, 2), mch(m, 3), 0);
      const int32_t num = c2i(mch(m, 2));
      if (!pbft_index(p, num)) return;
      AT(p.tx_val, base + num, p.cap_txn) = c2i(mch(m, 3));
      ctx_bcast(c, r, false);
      break;
    }
    case PB_PREPARE: {  // :212-222
      const Msg r = mkmsg(PB_PREPARE_RES, mch(m, 1), mch(m, 2), enc_raw(p, 0), 0);
      ctx_unicast(c, back_edge, r);
      break;
    }
    case PB_PREPARE_RES: {  // :223-240
      const int32_t idx = c2i(mch(m, 2));
      if (!pbft_index(p, idx)) return;
      int32_t v = AT(p.tx_pv, base + idx, p.cap_txn);
      if (c2i(mch(m, 3)) == 0) ++v;
      if (v >= N / 2) {
        const Msg r = mkmsg(PB_COMMIT, mch(m, 1), mch(m, 2), 0, 0);
        ctx_bcast(c, r, false);
        v = 0;
      }
      AT(p.tx_pv, base + idx, p.cap_txn) = v;
      break;
    }
    case PB_COMMIT: {  // :241-265
      const int32_t idx = c2i(mch(m, 2));
      if (!pbft_index(p, idx)) return;
      int32_t v = AT(p.tx_cv, base + idx, p.cap_txn) + 1;
      if (v > N / 2) {
        v = 0;
        // a = global v, resolved from the v-log on the host (INT32_MIN marker)
        ctx_trace(c, BCSIM_TR_PBFT_COMMIT, INT32_MIN, s.block_num, AT(p.tx_val, base + idx, p.cap_txn));
        ++s.block_num;
      }
      AT(p.tx_cv, base + idx, p.cap_txn) = v;
      break;
    }
    case PB_VIEW_CHANGE: {  // :271-286 (falls through to "Wrong msg")
      const int32_t vt = c2i(mch(m, 1));
      const int32_t lt = c2i(mch(m, 2));
      const uint32_t pos = atomicAdd(p.vlog_cnt, 1u);
      if (pos < p.cap_vlog) {
        VLog e;
        e.t = c.cur.t;
        e.ts = c.cur.ts;
        e.origin = c.cur.origin;
        e.sub = c.cur.sub;
        e.target = c.i;
        e.rep = c.rep;
        e.v = vt;
        e.pad = 0;
        AT(p.vlog, pos, p.cap_vlog) = e;
      } else {
        set_err(p, BCSIM_E_OVERFLOW);
      }
      s.leader = lt;
      if (static_cast<int32_t>(c.i) == lt) ctx_trace(c, BCSIM_TR_PBFT_VIEW, vt, lt, 0);
      ++c.wrong;
      break;
    }
    default:
      ++c.wrong;
      break;
  }
}

// ---------------------------------------------------------------------------
// Raft handlers (raft/raft-node.cc).  Message types raft-node.h:81-89.
enum { RF_VOTE_REQ = 2, RF_VOTE_RES = 3, RF_HEARTBEAT = 4, RF_HEARTBEAT_RES = 5 };

struct RaftState {
  int32_t is_leader, has_voted, m_value, vs, vf, acv, blockNum, round;
  uint32_t next_election, next_heartbeat;
};

__device__ void raft_arm_election(Ctx& c, RaftState& s) {  // getElectionTimeout :69-72
  const KP& p = *c.p;
  if (p.rng_mode == BCSIM_RNG_COUNTER) {
    const int32_t r = ctr_rand(p.seed, c.rep, c.i, c.draws++);
    s.next_election = ctx_timer(c, TM_RAFT_ELECTION, AT(p.raft_elec, r % 150, 150));
  } else {
    s.next_election = ctx_timer(c, TM_RAFT_ELECTION, 0, true);
    const uint32_t pos = atomicAdd(p.dreq_cnt, 1u);
    if (pos >= p.cap_dreq) {
      set_err(p, BCSIM_E_OVERFLOW);
      return;
    }
    DrawReq d;
    d.t = c.cur.t;
    d.ts = c.cur.ts;
    d.origin = c.cur.origin;
    d.sub = c.cur.sub;
    d.target = c.i;
    d.rep = c.rep;
    d.timer_sub = s.next_election;
    d.pad = 0;
    AT(p.dreq, pos, p.cap_dreq) = d;
  }
}

__device__ void raft_heartbeat(Ctx& c, RaftState& s) {  // sendHeartBeat :404-429
  const KP& p = *c.p;
  s.has_voted = 1;
  if (s.acv == 1) {
    s.next_heartbeat = ctx_timer(c, TM_RAFT_HEARTBEAT, p.raft_hb);
    ctx_trace(c, BCSIM_TR_RAFT_PROPOSAL, s.round, 0, 0);  // SendTX :342
    ctx_bcast(c, mkmsg(RF_HEARTBEAT, enc_raw(p, 1), '1', '1', 1), false);
    ++s.round;
    if (s.round == static_cast<int32_t>(p.raft_prop_rounds)) s.acv = 0;
  } else {
    s.next_heartbeat = ctx_timer(c, TM_RAFT_HEARTBEAT, p.raft_hb);
    ctx_bcast(c, mkmsg(RF_HEARTBEAT, enc_raw(p, 0), 0, 0, 0), false);
  }
}

__device__ void raft_recv(Ctx& c, RaftState& s, const Msg& m, uint32_t back_edge) {
  const KP& p = *c.p;
  const int32_t N = static_cast<int32_t>(p.N);
  switch (c2i(mch(m, 0))) {
    case RF_VOTE_REQ: {  // :154-168
      int32_t st = 1;
      if (s.has_voted == 0) {
        st = 0;
        s.has_voted = 1;
      }
      ctx_unicast(c, back_edge, mkmsg(RF_VOTE_RES, enc_raw(p, st), 0, 0, 0));
      break;
    }
    case RF_HEARTBEAT: {  // :170-194
      const int32_t type = c2i(mch(m, 1));
      int32_t d1;
      if (type == 0) {
        d1 = enc_raw(p, 0);
      } else {
        d1 = enc_raw(p, 1);
        s.m_value = c2i(mch(m, 2));
      }
      ctx_cancel(c, s.next_election);
      ctx_unicast(c, back_edge, mkmsg(RF_HEARTBEAT_RES, d1, enc_raw(p, 0), 0, 0));
      break;
    }
    case RF_VOTE_RES: {  // :196-232
      if (!s.is_leader) {
        if (c2i(mch(m, 1)) == 0)
          ++s.vs;
        else
          ++s.vf;
        if (s.vs + 1 > N / 2) {
          s.vs = 0;
          s.vf = 0;
          ctx_trace(c, BCSIM_TR_RAFT_LEADER, 0, 0, 0);
          ctx_cancel(c, s.next_election);
          (void)ctx_timer(c, TM_RAFT_PROPOSAL, p.raft_prop_delay);
          raft_heartbeat(c, s);
          s.is_leader = 1;
        } else if (s.vf >= N / 2) {
          s.vs = 0;
          s.vf = 0;
          s.has_voted = 0;
        }
      }
      break;
    }
    case RF_HEARTBEAT_RES: {  // :233-266
      if (c2i(mch(m, 1)) == 1) {
        if (c2i(mch(m, 2)) == 0)
          ++s.vs;
        else
          ++s.vf;
        if (s.vs + s.vf == N - 1) {
          if (s.vs + 1 > N / 2) {
            s.vs = 0;
            s.vf = 0;
            ctx_trace(c, BCSIM_TR_RAFT_BLOCK, s.blockNum, 0, 0);
            s.blockNum += 1;
            if (s.blockNum >= static_cast<int32_t>(p.raft_blocks)) {
              ctx_trace(c, BCSIM_TR_RAFT_DONE, s.blockNum, 0, 0);
              ctx_cancel(c, s.next_heartbeat);
            }
          } else {
            s.vs = 0;
            s.vf = 0;
          }
        }
      }
      break;
    }
    default:
      ++c.wrong;
      break;
  }
}

// ---------------------------------------------------------------------------
// Paxos handlers (paxos/paxos-node.cc).  Message types paxos-node.h:72-81.
enum {
  PX_REQ_TICKET = 0, PX_REQ_PROPOSE = 1, PX_REQ_COMMIT = 2, PX_RES_TICKET = 3,
  PX_RES_PROPOSE = 4, PX_RES_COMMIT = 5, PX_CLIENT = 6
};

struct PaxosState {
  int32_t t_max, command, t_store, ticket, is_commit, proposal, vs, vf;
};

__device__ void paxos_ticket(Ctx& c, PaxosState& s) {  // requireTicket :510-522
  const KP& p = *c.p;
  ++s.ticket;
  ctx_bcast(c, mkmsg(PX_REQ_TICKET, enc_raw(p, s.ticket), 0, 0, 0), true);
  ctx_trace(c, BCSIM_TR_PAXOS_TICKET, s.ticket, 0, 0);
}

__device__ void paxos_recv(Ctx& c, PaxosState& s, const Msg& m, uint32_t back_edge) {
  const KP& p = *c.p;
  TRAIL(c);
  const int32_t N = static_cast<int32_t>(p.N);
  const int32_t ty = c2i(mch(m, 0));
  switch (ty) {
    case PX_REQ_TICKET: {  // :177-198
      const int32_t t = c2i(mch(m, 1));
      Msg r;
      if (t > s.t_max) {
        s.t_max = t;
        r = mkmsg(PX_RES_TICKET, enc_raw(p, 0), s.command, 0, 0);
      } else {
        r = mkmsg(PX_RES_TICKET, enc_raw(p, 1), 0, 0, 0);
      }
      ctx_unicast(c, back_edge, r);
      break;
    }
    case PX_REQ_PROPOSE: {  // :199-221
      const int32_t t = c2i(mch(m, 1));
      int32_t st = 1;
      if (t == s.t_max) {
        s.command = mch(m, 2);
        s.t_store = t;
        st = 0;
      }
      ctx_unicast(c, back_edge, mkmsg(PX_RES_PROPOSE, enc_raw(p, st), 0, 0, 0));
      break;
    }
    case PX_REQ_COMMIT: {  // :222-247
      const int32_t t = c2i(mch(m, 1));
      const int32_t cc = mch(m, 2);
      int32_t st = 1;
      if (t == s.t_store && cc == s.command) {
        s.is_commit = 1;
        st = 0;
      }
      ctx_unicast(c, back_edge, mkmsg(PX_RES_COMMIT, enc_raw(p, st), 0, 0, 0));
      break;
    }
    case PX_RES_TICKET:
    case PX_RES_PROPOSE:
    case PX_RES_COMMIT: {  // :248-353
      if (c2i(mch(m, 1)) == 0)
        ++s.vs;
      else
        ++s.vf;
      if (s.vs + s.vf == N - 2) {
        if (s.vs >= N / 2) {
          s.vs = 0;
          s.vf = 0;
          if (ty == PX_RES_TICKET) {
            if (mch(m, 2) != 'e') s.proposal = mch(m, 2);
            ctx_bcast(c, mkmsg(PX_REQ_PROPOSE, enc_raw(p, s.ticket), s.proposal, 0, 0), true);
          } else if (ty == PX_RES_PROPOSE) {
            ctx_bcast(c, mkmsg(PX_REQ_COMMIT, enc_raw(p, s.ticket), s.proposal, 0, 0), true);
          } else {
            ctx_trace(c, BCSIM_TR_PAXOS_COMMIT, s.ticket, 0, 0);
          }
        } else {
          s.vs = 0;
          s.vf = 0;
          paxos_ticket(c, s);
        }
      }
      break;
    }
    case PX_CLIENT:
      paxos_ticket(c, s);
      break;
    default:
      ++c.wrong;
      break;
  }
}

// ---------------------------------------------------------------------------
// k_scan: one workgroup per node.  Sort the node's arrivals of [t_lo, t_hi)
// by (t, t_sched, origin) in LDS, then run the state machine in canonical
// key order merged with the node's timers and START/STOP.
constexpr int kScanThreads = 256;
constexpr int kScanMaxArr = 4096;  // LDS window: 32 B per staged arrival
constexpr int kScanPerThread = kScanMaxArr / kScanThreads;

struct SKey {
  uint64_t hi;  // t_off << 32 | ~dt
  uint32_t lo;  // origin
  uint32_t idx;
};

__device__ inline bool skey_gt(const SKey& a, const SKey& b) {
  return a.hi > b.hi || (a.hi == b.hi && a.lo > b.lo);
}

// Count this node's arrivals with t in [a, b) (all threads; block-uniform result).
__device__ inline uint32_t scan_count(const KP& p, uint32_t* slot, uint32_t seg_b, uint32_t m, long long cs,
                                      long long a, long long b) {
  const uint32_t tid = threadIdx.x;
  __syncthreads();
  if (tid == 0) *slot = 0;
  __syncthreads();
  uint32_t mine = 0;
  for (uint32_t k = tid; k < m; k += blockDim.x) {
    const long long t = cs + AT(p.grp, seg_b + k, p.cap_bucket).t_off;
    mine += (t >= a && t < b);
  }
  if (mine) atomicAdd(slot, mine);
  __syncthreads();
  return *slot;
}

template <int PROTO>
__global__ __launch_bounds__(kScanThreads) void k_scan(const KP* __restrict__ pk, long long cell, long long t_lo,
                                                      long long t_hi, long long cs) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  // LDS: [0,64) control | cap_arr x Rec (sorted window; the SKey sort runs in
  // the same bytes first) | cap_timers x TimerEnt
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* ctl = reinterpret_cast<uint32_t*>(smem);
  SKey* keys = reinterpret_cast<SKey*>(smem + 64);
  Rec* recs = reinterpret_cast<Rec*>(smem + 64);
  TimerEnt* tm = reinterpret_cast<TimerEnt*>(smem + 64 + static_cast<size_t>(p.cap_arr) * sizeof(Rec));

  const uint32_t g = blockIdx.x;
  if (g >= p.NT) return;
  const uint32_t tid = threadIdx.x;
  const uint32_t seg_b = AT(p.seg_off, g, p.NT + 1);
  const uint32_t m = AT(p.seg_off, g + 1, p.NT + 1) - seg_b;
  const bool has_start = (t_lo <= 0 && 0 < t_hi);
  const bool has_stop = (p.stop_ns >= 0 && t_lo <= p.stop_ns && p.stop_ns < t_hi);
  if (m == 0 && AT(p.node_tnext, g, p.NT) >= t_hi && !has_start && !has_stop) return;
  if (tid < p.cap_timers)
    tm[tid] = AT(p.timers, static_cast<size_t>(g) * p.cap_timers + tid, static_cast<uint64_t>(p.NT) * p.cap_timers);

  // ---- serial state (lane 0 only) ----
  const uint32_t rep = g / p.N, i = g % p.N;
  Ctx c;
  PbftState ps{};
  RaftState rs{};
  PaxosState xs{};
  bool start_pending = has_start, stop_pending = has_stop;
  if (tid == 0) {
    c.p = pk;
    c.g = g;
    c.rep = rep;
    c.i = i;
    c.deg = AT(p.row, i + 1, p.N + 1) - AT(p.row, i, p.N + 1);
    c.sub = AT(p.sub, g, p.NT);
    c.draws = AT(p.draws, g, p.NT);
    c.ops = p.ops + static_cast<size_t>(g) * p.cap_ops;
    c.nops = AT(p.n_ops, g, p.NT);
    c.tm = tm;
    c.cap_t = p.cap_timers;
    for (int k = 0; k < BCSIM_MSG_TYPES; ++k) c.deliv[k] = 0;
    c.echoes = c.wrong = c.events = 0;
    if (PROTO == BCSIM_PBFT) {
      ps.leader = AT(p.leader, g, p.NT);
      ps.block_num = AT(p.block_num, g, p.NT);
    } else if (PROTO == BCSIM_RAFT) {
      rs.is_leader = AT(p.is_leader, g, p.NT);
      rs.has_voted = AT(p.has_voted, g, p.NT);
      rs.m_value = AT(p.m_value, g, p.NT);
      rs.vs = AT(p.vote_s, g, p.NT);
      rs.vf = AT(p.vote_f, g, p.NT);
      rs.acv = AT(p.acv, g, p.NT);
      rs.blockNum = AT(p.blockNum, g, p.NT);
      rs.round = AT(p.round, g, p.NT);
      rs.next_election = AT(p.next_election, g, p.NT);
      rs.next_heartbeat = AT(p.next_heartbeat, g, p.NT);
    } else {
      xs.t_max = AT(p.t_max, g, p.NT);
      xs.command = AT(p.command, g, p.NT);
      xs.t_store = AT(p.t_store, g, p.NT);
      xs.ticket = AT(p.ticket, g, p.NT);
      xs.is_commit = AT(p.is_commit, g, p.NT);
      xs.proposal = AT(p.proposal, g, p.NT);
      xs.vs = AT(p.vote_s, g, p.NT);
      xs.vf = AT(p.vote_f, g, p.NT);
    }
    TRAIL(c);
  }

  // ---- windows: [t_lo, t_hi) split so that each holds <= cap_arr arrivals.
  // At one instant a node receives at most one record per in-edge (links are
  // FIFO and serialise), and cap_arr > deg, so every window is non-empty.
  long long tmax_ev = LLONG_MIN;
  long long wa = t_lo;
  for (;;) {
    long long wb = t_hi;
    uint32_t n;
    if (m > p.cap_arr && scan_count(p, &ctl[1], seg_b, m, cs, wa, t_hi) > p.cap_arr) {
      long long lo = wa, hi = t_hi;  // count(lo) <= cap < count(hi)
      while (hi - lo > 1) {
        const long long mid = lo + (hi - lo) / 2;
        if (scan_count(p, &ctl[1], seg_b, m, cs, wa, mid) <= p.cap_arr)
          lo = mid;
        else
          hi = mid;
      }
      wb = lo;
      if (wb == wa) {  // > cap_arr arrivals at one instant (cap_arr <= deg)
        if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
        return;
      }
    }
    // select this window's arrivals and sort them by (t, t_sched, origin)
    __syncthreads();
    if (tid == 0) ctl[0] = 0;
    __syncthreads();
    for (uint32_t k = tid; k < m; k += blockDim.x) {
      const Rec r = AT(p.grp, seg_b + k, p.cap_bucket);
      const long long t = cs + r.t_off;
      if (t >= wa && t < wb) {
        const uint32_t slot = atomicAdd(&ctl[0], 1u);
        if (slot < p.cap_arr) {
          SKey s;
          s.hi = (static_cast<uint64_t>(r.t_off) << 32) | static_cast<uint32_t>(~r.dt);
          s.lo = r.origin;
          s.idx = k;
          keys[slot] = s;
        }
      }
    }
    __syncthreads();
    n = ctl[0];
    if (n > p.cap_arr) {  // unreachable by construction
      if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
      return;
    }
    uint32_t P2 = 2;
    while (P2 < n) P2 <<= 1;
    for (uint32_t k = n + tid; k < P2; k += blockDim.x) {
      SKey s;
      s.hi = ~0ull;
      s.lo = ~0u;
      s.idx = 0;
      keys[k] = s;
    }
    __syncthreads();
    for (uint32_t k2 = 2; k2 <= P2; k2 <<= 1) {
      for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
        for (uint32_t t = tid; t < P2; t += blockDim.x) {
          const uint32_t ixj = t ^ j;
          if (ixj > t) {
            const SKey a = keys[t], b = keys[ixj];
            const bool up = (t & k2) == 0;
            if (up ? skey_gt(a, b) : skey_gt(b, a)) {
              keys[t] = b;
              keys[ixj] = a;
            }
          }
        }
        __syncthreads();
      }
    }
    // gather the records in key order into LDS (same bytes as the keys:
    // indices go through registers first); edge -> reverse edge here
    uint32_t ix[kScanPerThread];
#pragma unroll
    for (int j = 0; j < kScanPerThread; ++j) {
      const uint32_t k = tid + j * kScanThreads;
      ix[j] = k < n ? keys[k].idx : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kScanPerThread; ++j) {
      const uint32_t k = tid + j * kScanThreads;
      if (k < n) {
        Rec r = AT(p.grp, seg_b + ix[j], p.cap_bucket);
        r.edge = AT(p.rev, r.edge, p.E);
        recs[k] = r;
      }
    }
    __syncthreads();

    if (tid == 0) {
      uint32_t ai = 0;
      for (;;) {
        // candidates
        int which = -1;  // 0 arrival, 1 timer, 2 start, 3 stop
        Key best{};
        Rec rec{};
        int tsel = -1;
        if (ai < n) {
          rec = recs[ai];
          best.t = cs + rec.t_off;
          best.ts = best.t - rec.dt;
          best.origin = rec.origin;
          best.sub = rec.sub;
          which = 0;
        }
        for (uint32_t k = 0; k < c.cap_t; ++k) {
          const TimerEnt& te = tm[k];
          if (!te.alive || te.pending_draw || te.t >= wb || te.t < t_lo) continue;
          const Key kk{te.t, te.ts, i, te.sub};
          if (which < 0 || key_less(kk, best)) {
            best = kk;
            which = 1;
            tsel = static_cast<int>(k);
          }
        }
        if (start_pending && 0 < wb) {
          const Key kk{0, -1, i, 0};
          if (which < 0 || key_less(kk, best)) {
            best = kk;
            which = 2;
          }
        }
        if (stop_pending && p.stop_ns < wb) {
          const Key kk{p.stop_ns, -1, i, 1};
          if (which < 0 || key_less(kk, best)) {
            best = kk;
            which = 3;
          }
        }
        TRAIL(c);
        if (which < 0) break;
        c.cur = best;
        if (best.t > tmax_ev) tmax_ev = best.t;
        ++c.events;
        if (which == 0) {
          ++ai;
          Msg msg;
          msg.type = rec.type;
          msg.f[0] = rec.f0;
          msg.f[1] = rec.f1;
          msg.f[2] = rec.f2;
          msg.big = rec.big;
          if (rec.type < BCSIM_MSG_TYPES) ++c.deliv[rec.type];
          TRAIL(c);
          // rec.edge is the reverse edge (receiver -> sender) from the gather
          if (p.echo) {  // socket->SendTo(packet, 0, from): reverse-link occupancy
            ctx_op(c, mk_op(p, best.t, rec.dt, rec.origin, rec.sub, rec.edge, msg, OP_ECHO, 0));
            ++c.echoes;
          }
          if (PROTO == BCSIM_PBFT) {
            if (best.t == ((best.t / p.pbft_period) * p.pbft_period) && best.ts <= best.t - p.pbft_period)
              set_err(p, BCSIM_E_TIE);  // arrival ordered before a same-time tick
            pbft_recv(c, ps, msg, rec.edge);
          } else if (PROTO == BCSIM_RAFT) {
            raft_recv(c, rs, msg, rec.edge);
          } else {
            paxos_recv(c, xs, msg, rec.edge);
          }
        } else if (which == 1) {
          TimerEnt& te = tm[tsel];
          te.alive = 0;
          if (PROTO == BCSIM_RAFT) {
            if (te.kind == TM_RAFT_ELECTION) {  // sendVote :391-401
              rs.has_voted = 1;
              ctx_bcast(c, mkmsg(RF_VOTE_REQ, enc_raw(p, static_cast<int32_t>(i)), 0, 0, 0), false);
              ctx_trace(c, BCSIM_TR_RAFT_ELECTION, 0, 0, 0);
              raft_arm_election(c, rs);
            } else if (te.kind == TM_RAFT_HEARTBEAT) {
              raft_heartbeat(c, rs);
            } else if (te.kind == TM_RAFT_PROPOSAL) {  // setProposal :432-435
              rs.acv = 1;
            }
          } else if (PROTO == BCSIM_PAXOS) {
            if (te.kind == TM_PAXOS_TICKET) paxos_ticket(c, xs);
          }
        } else if (which == 2) {  // StartApplication
          start_pending = false;
          if (PROTO == BCSIM_PBFT) {  // :97-158; globals reset host-side
            ps.leader = 0;
            ps.block_num = 0;
            AT(p.tick_sub, g, p.NT) = c.sub++;  // Schedule(Seconds(timeout), SendBlock) :155
            AT(p.tick_alive, g, p.NT) = 1;
          } else if (PROTO == BCSIM_RAFT) {  // :75-115
            rs.m_value = 0;
            rs.vs = 0;
            rs.vf = 0;
            rs.has_voted = 0;
            rs.acv = 0;
            rs.is_leader = 0;
            rs.round = 0;
            rs.blockNum = 0;
            if (p.rng_mode == BCSIM_RNG_COUNTER) {
              raft_arm_election(c, rs);
            } else {  // START draws run in node order at t=0: stream index = node id
              const int32_t r = AT(p.glibc, static_cast<size_t>(rep) * p.glibc_len + i, p.cap_glibc);
              rs.next_election = ctx_timer(c, TM_RAFT_ELECTION, AT(p.raft_elec, r % 150, 150));
            }
          } else {  // :58-139
            xs.t_max = 0;
            xs.command = 'e';
            xs.t_store = 0;
            xs.ticket = 0;
            xs.is_commit = 0;
            xs.proposal = enc_raw(p, static_cast<int32_t>(i));
            xs.vs = 0;
            xs.vf = 0;
            if (i < p.paxos_proposers) (void)ctx_timer(c, TM_PAXOS_TICKET, 0);
          }
        } else {  // StopApplication
          stop_pending = false;
          if (PROTO == BCSIM_RAFT && rs.is_leader == 1)
            ctx_trace(c, BCSIM_TR_RAFT_STOP, rs.blockNum, rs.round, 0);
        }
      }
    }
    if (wb >= t_hi) break;
    wa = wb;
  }
  if (tid != 0) return;
  // write back
  TRAIL(c);
  AT(p.sub, g, p.NT) = c.sub;
  AT(p.draws, g, p.NT) = c.draws;
  AT(p.n_ops, g, p.NT) = c.nops;
  long long tnext = LLONG_MAX;
  for (uint32_t k = 0; k < c.cap_t; ++k) {
    AT(p.timers, static_cast<size_t>(g) * p.cap_timers + k, static_cast<uint64_t>(p.NT) * p.cap_timers) = tm[k];
    if (tm[k].alive && tm[k].t < tnext) tnext = tm[k].t;
  }
  AT(p.node_tnext, g, p.NT) = tnext;
  if (c.nops > 0) AT(p.node_onext, g, p.NT) = LLONG_MIN;  // link stage recomputes
  if (PROTO == BCSIM_PBFT) {
    AT(p.leader, g, p.NT) = ps.leader;
    AT(p.block_num, g, p.NT) = ps.block_num;
  } else if (PROTO == BCSIM_RAFT) {
    AT(p.is_leader, g, p.NT) = rs.is_leader;
    AT(p.has_voted, g, p.NT) = rs.has_voted;
    AT(p.m_value, g, p.NT) = rs.m_value;
    AT(p.vote_s, g, p.NT) = rs.vs;
    AT(p.vote_f, g, p.NT) = rs.vf;
    AT(p.acv, g, p.NT) = rs.acv;
    AT(p.blockNum, g, p.NT) = rs.blockNum;
    AT(p.round, g, p.NT) = rs.round;
    AT(p.next_election, g, p.NT) = rs.next_election;
    AT(p.next_heartbeat, g, p.NT) = rs.next_heartbeat;
  } else {
    AT(p.t_max, g, p.NT) = xs.t_max;
    AT(p.command, g, p.NT) = xs.command;
    AT(p.t_store, g, p.NT) = xs.t_store;
    AT(p.ticket, g, p.NT) = xs.ticket;
    AT(p.is_commit, g, p.NT) = xs.is_commit;
    AT(p.proposal, g, p.NT) = xs.proposal;
    AT(p.vote_s, g, p.NT) = xs.vs;
    AT(p.vote_f, g, p.NT) = xs.vf;
  }
  unsigned long long* cnt = &AT(p.counters, static_cast<size_t>(rep) * CNT_N, static_cast<uint64_t>(p.R) * CNT_N);
  unsigned long long tot = 0;
  for (int k = 0; k < BCSIM_MSG_TYPES; ++k)
    if (c.deliv[k]) {
      atomicAdd(&cnt[CNT_DELIV + k], c.deliv[k]);
      tot += c.deliv[k];
    }
  if (tot) atomicAdd(&cnt[CNT_DELIV_TOTAL], tot);
  if (c.echoes) atomicAdd(&cnt[CNT_ECHOES], c.echoes);
  if (c.wrong) atomicAdd(&cnt[CNT_WRONG], c.wrong);
  if (c.events) atomicAdd(&cnt[CNT_EVENTS], c.events);
  if (tmax_ev > LLONG_MIN) atomicMax(reinterpret_cast<long long*>(&cnt[CNT_TLAST]), tmax_ev);
}

// ---------------------------------------------------------------------------
// k_link: per-node link stage.  Ops due in [.., t_hi) are applied to their
// out-edge's FIFO in canonical key order; every non-echo op produces one
// 32-byte arrival record, scattered into the bucket of its arrival cell.
constexpr int kHot = 8;       // arrival cells g+1 .. g+kHot get chunked appends
constexpr int kBcastCap = 64; // due broadcasts per node per cell

__device__ inline bool op_key_less(const Op& a, uint32_t sa, const Op& b, uint32_t sb) {
  if (a.t != b.t) return a.t < b.t;
  const int64_t tsa = a.t - a.dt, tsb = b.t - b.dt;
  if (tsa != tsb) return tsa < tsb;
  if (a.origin != b.origin) return a.origin < b.origin;
  return sa < sb;
}

struct LinkLds {
  uint32_t n_bc;
  uint32_t n_due;
  uint32_t n_keep;
  uint32_t hot_cnt[kHot];
  uint32_t hot_base[kHot];
  uint32_t hot_fill[kHot];
  uint32_t bc[kBcastCap];
};

// iterate the ops of edge `le` of node i in key order, calling f(op, sub, is_echo, dropped)
template <typename F>
__device__ inline void edge_ops(const KP& p, const Op* ops, const uint32_t* eidx, uint32_t eb,
                                uint32_t ee, const uint32_t* bc, uint32_t n_bc, uint32_t le,
                                uint32_t deg, F&& f) {
  // eidx[eb..ee) are this edge's SEND/ECHO op indices, sorted by key already
  uint32_t a = eb, b = 0;
  for (;;) {
    // next bcast that targets this edge
    while (b < n_bc) {
      const Op& o = AT(ops, bc[b], p.cap_ops);
      const bool paxos = (op_flags(o) & OPF_PAXOS) != 0;
      if (paxos && le == 0) {
        ++b;
        continue;
      }
      break;
    }
    const bool ha = a < ee, hb = b < n_bc;
    if (!ha && !hb) break;
    bool take_a;
    uint32_t sub_b = 0;
    if (hb) {
      const Op& ob = AT(ops, bc[b], p.cap_ops);
      const bool paxos = (op_flags(ob) & OPF_PAXOS) != 0;
      sub_b = ob.sub + (paxos ? le - 1 : le);
    }
    if (ha && hb) {
      const Op& oa = AT(ops, eidx[a], p.cap_ops);
      take_a = op_key_less(oa, oa.sub, AT(ops, bc[b], p.cap_ops), sub_b);
    } else {
      take_a = ha;
    }
    if (take_a) {
      const Op& oa = AT(ops, eidx[a++], p.cap_ops);
      f(oa, oa.sub, op_kind(oa) == OP_ECHO);
    } else {
      f(AT(ops, bc[b++], p.cap_ops), sub_b, false);
    }
  }
}

__global__ __launch_bounds__(256) void k_link(const KP* __restrict__ pk, long long cell, long long t_hi) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ LinkLds L;
  const uint32_t g = blockIdx.x;
  if (g >= p.NT) return;
  uint32_t n = AT(p.n_ops, g, p.NT);
  if (n == 0) return;
  const uint32_t tid = threadIdx.x;
  const uint32_t rep = g / p.N, i = g % p.N;
  const uint32_t e0 = AT(p.row, i, p.N + 1), deg = AT(p.row, i + 1, p.N + 1) - e0;
  Op* ops = p.ops + static_cast<size_t>(g) * p.cap_ops;
  uint32_t* ecnt = reinterpret_cast<uint32_t*>(smem);   // deg+1
  uint32_t* efill = ecnt + (p.deg_max + 1);              // deg
  uint32_t* eidx = efill + p.deg_max;                    // cap_ops
  int64_t* busy = p.busy + static_cast<size_t>(rep) * p.E + e0;
  const int64_t* prop = p.prop + e0;
  unsigned long long* cnt = &AT(p.counters, static_cast<size_t>(rep) * CNT_N, static_cast<uint64_t>(p.R) * CNT_N);

  // ---- 0. expand jitter broadcasts into per-edge SEND ops ----
  if (p.delay_mode != BCSIM_DELAY_FIXED) {
    for (uint32_t k = 0; k < n; ++k) {  // uniform loop over the (few) ops
      Op o = AT(ops, k, p.cap_ops);
      if (op_kind(o) != OP_BCAST_J || (op_flags(o) & OPF_DONE)) continue;
      if (n + deg > p.cap_ops) {
        if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
        return;
      }
      const bool paxos = (op_flags(o) & OPF_PAXOS) != 0;
      const uint64_t dbase = static_cast<uint64_t>(o.edge);
      for (uint32_t it = tid; it < deg; it += blockDim.x) {
        const int32_t r = ctr_rand(p.seed, rep, i, dbase + it);
        const int64_t d = delay_from_draw(p, r);
        Op s = o;
        s.t = o.t + d;
        s.dt = static_cast<uint32_t>(d);
        s.sub = o.sub + it;
        s.edge = paxos ? (it + 1 < deg ? e0 + it + 1 : kInvalid) : e0 + it;
        s.kind_flags = static_cast<uint8_t>(OP_SEND | ((op_flags(o) & OPF_BIG) << 2));
        AT(ops, n + it, p.cap_ops) = s;
      }
      __syncthreads();
      if (tid == 0) AT(ops, k, p.cap_ops).kind_flags = static_cast<uint8_t>(OP_BCAST_J | (OPF_DONE << 2));
      n += deg;
      __syncthreads();
    }
  }

  // ---- 1. classify due ops ----
  for (uint32_t k = tid; k <= deg; k += blockDim.x) ecnt[k] = 0;
  if (tid == 0) {
    L.n_bc = 0;
    L.n_due = 0;
    for (int h = 0; h < kHot; ++h) {
      L.hot_cnt[h] = 0;
      L.hot_fill[h] = 0;
    }
  }
  __syncthreads();
  unsigned long long dropped = 0, sends = 0;
  unsigned long long st_rec = 0, st_ops = 0, st_edges = 0;
  for (uint32_t k = tid; k < n; k += blockDim.x) {
    const Op& o = AT(ops, k, p.cap_ops);
    const uint8_t kind = op_kind(o);
    if (kind == OP_BCAST_J) continue;  // expanded (done) marker
    if (o.t >= t_hi) continue;
    ++st_ops;
    if (kind == OP_BCAST) {
      const uint32_t pos = atomicAdd(&L.n_bc, 1u);
      if (pos < kBcastCap) L.bc[pos] = k;
      sends += deg;
      if (op_flags(o) & OPF_PAXOS) dropped += 1;
    } else if (o.edge == kInvalid) {  // Paxos *end(): no route, dropped
      dropped += 1;
      sends += 1;
    } else {
      if (kind == OP_SEND) sends += 1;
      atomicAdd(&ecnt[o.edge - e0], 1u);
    }
  }
  __syncthreads();
  if (L.n_bc > kBcastCap) {
    if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
    return;
  }
  // exclusive scan of ecnt[0..deg] (single thread; deg is small next to the op count)
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k <= deg; ++k) {
      const uint32_t v = ecnt[k];
      ecnt[k] = acc;
      acc += v;
    }
    L.n_due = acc;
    // sort the broadcasts by key (insertion sort, few)
    for (uint32_t a = 1; a < L.n_bc; ++a) {
      const uint32_t x = L.bc[a];
      uint32_t b2 = a;
      while (b2 > 0 && op_key_less(AT(ops, x, p.cap_ops), AT(ops, x, p.cap_ops).sub, AT(ops, L.bc[b2 - 1], p.cap_ops), AT(ops, L.bc[b2 - 1], p.cap_ops).sub)) {
        L.bc[b2] = L.bc[b2 - 1];
        --b2;
      }
      L.bc[b2] = x;
    }
  }
  for (uint32_t k = tid; k < deg; k += blockDim.x) efill[k] = 0;
  __syncthreads();
  for (uint32_t k = tid; k < n; k += blockDim.x) {
    const Op& o = AT(ops, k, p.cap_ops);
    const uint8_t kind = op_kind(o);
    if (kind == OP_BCAST_J || kind == OP_BCAST || o.t >= t_hi || o.edge == kInvalid) continue;
    const uint32_t le = o.edge - e0;
    eidx[ecnt[le] + atomicAdd(&efill[le], 1u)] = k;
  }
  __syncthreads();
  const uint32_t n_bc = L.n_bc;

  // ---- 2. per edge: sort its ops by key, merge with broadcasts, FIFO ----
  // pass A counts arrivals per hot cell; pass B writes.
  for (int pass = 0; pass < 2; ++pass) {
    for (uint32_t le = tid; le < deg; le += blockDim.x) {
      const uint32_t eb = ecnt[le], ee = ecnt[le + 1];
      if (pass == 0) {  // insertion sort this edge's op indices by key
        for (uint32_t a = eb + 1; a < ee; ++a) {
          const uint32_t x = eidx[a];
          uint32_t b2 = a;
          while (b2 > eb && op_key_less(AT(ops, x, p.cap_ops), AT(ops, x, p.cap_ops).sub, AT(ops, eidx[b2 - 1], p.cap_ops), AT(ops, eidx[b2 - 1], p.cap_ops).sub)) {
            eidx[b2] = eidx[b2 - 1];
            --b2;
          }
          eidx[b2] = x;
        }
      }
      if (ee == eb && n_bc == 0) continue;
      if (pass == 1) ++st_edges;
      int64_t bu = AT(busy, le, p.cap_E - (static_cast<uint64_t>(rep) * p.E + e0));
      const int64_t pr = prop[le];
      const uint32_t dest = rep * p.N + AT(p.col, e0 + le, p.E);
      edge_ops(p, ops, eidx, eb, ee, L.bc, n_bc, le, deg,
               [&](const Op& o, uint32_t sub, bool is_echo) {
                 const int big = (op_flags(o) & OPF_BIG) ? 1 : 0;
                 const int64_t start = bu > o.t ? bu : o.t;
                 const int64_t end = start + p.tx_tot[big];
                 bu = end;
                 if (is_echo) return;
                 const int64_t ta = end + pr;
                 const long long ca = ta / p.L;
                 const long long rel = ca - cell;
                 if (pass == 0) {
                   if (rel >= 1 && rel <= kHot && rel < static_cast<long long>(p.n_buckets))
                     atomicAdd(&L.hot_cnt[rel - 1], 1u);
                   return;
                 }
                 ++st_rec;
                 Rec r;
                 r.t_off = static_cast<uint32_t>(ta - ca * p.L);
                 r.dt = static_cast<uint32_t>(ta - (end - p.tx_last[big]));
                 r.dest = dest;
                 r.origin = i;
                 r.sub = sub;
                 r.edge = e0 + le;
                 r.f0 = o.f0;
                 r.f1 = o.f1;
                 r.f2 = o.f2;
                 r.type = o.type;
                 r.big = static_cast<uint8_t>(big);
                 if (rel >= 1 && rel <= kHot && rel < static_cast<long long>(p.n_buckets)) {
                   const uint32_t h = static_cast<uint32_t>(rel - 1);
                   const uint32_t pos = L.hot_base[h] + atomicAdd(&L.hot_fill[h], 1u);
                   const uint32_t b = static_cast<uint32_t>(ca % p.n_buckets);
                   AT(p.bucket, static_cast<size_t>(b) * p.cap_bucket + pos, static_cast<uint64_t>(p.n_buckets) * p.cap_bucket) = r;
                 } else if (rel >= 1 && rel < static_cast<long long>(p.n_buckets)) {
                   const uint32_t b = static_cast<uint32_t>(ca % p.n_buckets);
                   const uint32_t pos = atomicAdd(&p.bucket_cnt[b], 1u);
                   if (pos >= p.cap_bucket) {
                     set_err(p, BCSIM_E_OVERFLOW);
                     return;
                   }
                   AT(p.bucket, static_cast<size_t>(b) * p.cap_bucket + pos, static_cast<uint64_t>(p.n_buckets) * p.cap_bucket) = r;
                 } else if (rel >= 1) {
                   const uint32_t pos = atomicAdd(p.ov_cnt, 1u);
                   if (pos >= p.cap_ov) {
                     set_err(p, BCSIM_E_OVERFLOW);
                     return;
                   }
                   OvRec ovr;
                   ovr.cell = ca;
                   ovr.pad = 0;
                   ovr.r = r;
                   AT(p.ov, pos, p.cap_ov) = ovr;
                   atomicMin(&p.scal[1], ca);
                 } else {
                   set_err(p, BCSIM_E_TIE);  // lookahead violated
                 }
               });
      if (pass == 1) AT(busy, le, p.cap_E - (static_cast<uint64_t>(rep) * p.E + e0)) = bu;
    }
    __syncthreads();
    if (pass == 0 && tid == 0) {
      for (int h = 0; h < kHot; ++h) {
        if (L.hot_cnt[h] == 0) continue;
        const long long ca = cell + 1 + h;
        const uint32_t b = static_cast<uint32_t>(ca % p.n_buckets);
        const uint32_t base = atomicAdd(&p.bucket_cnt[b], L.hot_cnt[h]);
        if (base + L.hot_cnt[h] > p.cap_bucket) set_err(p, BCSIM_E_OVERFLOW);
        L.hot_base[h] = base;
      }
    }
    __syncthreads();
    if (*p.err) return;
  }

  // ---- 3. compact the ops that are not due yet ----
  if (tid == 0) L.n_keep = 0;
  __syncthreads();
  long long omin = LLONG_MAX;
  // stable enough: order inside the list is irrelevant (ops are re-sorted)
  Op keep[4];
  uint32_t nk = 0;
  for (uint32_t k0 = 0; k0 < n; k0 += blockDim.x * 4) {
    nk = 0;
    for (uint32_t u = 0; u < 4; ++u) {
      const uint32_t k = k0 + u * blockDim.x + tid;
      if (k >= n) continue;
      const Op o = AT(ops, k, p.cap_ops);
      const uint8_t kind = op_kind(o);
      if (kind == OP_BCAST_J) {
        if (op_flags(o) & OPF_DONE) continue;
        keep[nk++] = o;  // unexpanded (fixed mode never creates these)
        continue;
      }
      if (o.t < t_hi) continue;
      keep[nk++] = o;
      if (o.t < omin) omin = o.t;
    }
    __syncthreads();
    const uint32_t base = atomicAdd(&L.n_keep, nk);
    __syncthreads();
    for (uint32_t u = 0; u < nk; ++u) AT(ops, base + u, p.cap_ops) = keep[u];
    __syncthreads();
  }
  // min over lanes of omin
  __shared__ long long omin_s;
  if (tid == 0) omin_s = LLONG_MAX;
  __syncthreads();
  if (omin != LLONG_MAX) atomicMin(&omin_s, omin);
  if (dropped) atomicAdd(&cnt[CNT_DROPPED], dropped);
  if (sends) atomicAdd(&cnt[CNT_SENDS], sends);
  if (st_rec | st_ops | st_edges) {
    atomicAdd(&p.kstat[0], st_rec);
    atomicAdd(&p.kstat[1], st_ops);
    atomicAdd(&p.kstat[2], st_edges);
  }
  __syncthreads();
  if (tid == 0) {
    AT(p.n_ops, g, p.NT) = L.n_keep;
    AT(p.node_onext, g, p.NT) = omin_s;
    atomicAdd(&p.kstat[3], static_cast<unsigned long long>(L.n_keep));
  }
}

// ---------------------------------------------------------------------------
// PBFT SendBlock tick (pbft-node.cc:371-411) for every node of a replica.
// One workgroup per replica; nodes tick in id order (canonical key order of
// equal-time timers scheduled at the same time).
__global__ __launch_bounds__(1024) void k_pbft_tick(const KP* __restrict__ pk, long long tk) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint8_t* lead = reinterpret_cast<uint8_t*>(smem);  // N flags
  __shared__ int32_t v_cur, nround0, n_alive, n_ticked;
  __shared__ long long vk_t, vk_ts;
  __shared__ uint32_t vk_o, vk_s, vk_tg;
  const uint32_t rep = blockIdx.x, tid = threadIdx.x;
  const uint32_t N = p.N;
  const long long ts_tick = tk - p.pbft_period;
  // v = latest v-log write before this tick in canonical order
  if (tid == 0) {
    v_cur = 1;
    vk_t = LLONG_MIN;
    vk_ts = LLONG_MIN;
    vk_o = 0;
    vk_s = 0;
    vk_tg = 0;
    const uint32_t nv = min(*p.vlog_cnt, p.cap_vlog);
    for (uint32_t k = 0; k < nv; ++k) {
      const VLog& e = AT(p.vlog, k, p.cap_vlog);
      if (e.rep != rep) continue;
      // before the tick key (tk, ts_tick, 0, 0, 0)?
      bool before = e.t < tk || (e.t == tk && e.ts < ts_tick);
      if (!before) continue;
      bool later = e.t > vk_t || (e.t == vk_t && (e.ts > vk_ts || (e.ts == vk_ts && (e.origin > vk_o ||
                   (e.origin == vk_o && (e.sub > vk_s || (e.sub == vk_s && e.target > vk_tg)))))));
      if (later) {
        vk_t = e.t;
        vk_ts = e.ts;
        vk_o = e.origin;
        vk_s = e.sub;
        vk_tg = e.target;
        v_cur = e.v;
      }
    }
    nround0 = AT(p.g_nround, rep, p.R);
    n_alive = 0;
    n_ticked = 0;
  }
  __syncthreads();
  for (uint32_t i = tid; i < N; i += blockDim.x) {
    const uint32_t g = rep * N + i;
    lead[i] = (AT(p.tick_alive, g, p.NT) && AT(p.leader, g, p.NT) == static_cast<int32_t>(i)) ? 1 : 0;
  }
  __syncthreads();
  // leaders, serially in node order (rare: normally exactly one)
  if (tid == 0) {
    int32_t nround = nround0;
    for (uint32_t i = 0; i < N; ++i) {
      if (!lead[i]) continue;
      const uint32_t g = rep * N + i;
      uint32_t sub = AT(p.sub, g, p.NT);
      const uint32_t deg = AT(p.row, i + 1, p.N + 1) - AT(p.row, i, p.N + 1);
      bcsim_trace_rec tr;
      tr.t_ns = tk;
      tr.key_ts = ts_tick;
      tr.key_origin = i;
      tr.key_sub = AT(p.tick_sub, g, p.NT);
      tr.replica = rep;
      tr.node = i;
      const int32_t n_seq = AT(p.g_n, rep, p.R);
      {  // :387 leader log
        const uint32_t pos = atomicAdd(p.trace_cnt, 1u);
        if (pos < p.cap_trace) {
          tr.kind = BCSIM_TR_PBFT_BLOCK;
          tr.a = n_seq;
          tr.b = v_cur;
          tr.c = 0;
          AT(p.trace, pos, p.cap_trace) = tr;
        } else {
          set_err(p, BCSIM_E_OVERFLOW);
        }
      }
      // block = generateTX header '1', v, n, n (:79-95)
      Msg blk = mkmsg(PB_PRE_PREPARE, enc_raw(p, v_cur), enc_raw(p, n_seq), enc_raw(p, n_seq), 1);
      uint32_t nops = AT(p.n_ops, g, p.NT);
      Op* ops = p.ops + static_cast<size_t>(g) * p.cap_ops;
      uint64_t draws = AT(p.draws, g, p.NT);
      auto push_bcast = [&](const Msg& m) {
        if (nops >= p.cap_ops) {
          set_err(p, BCSIM_E_OVERFLOW);
          return;
        }
        if (p.delay_mode == BCSIM_DELAY_FIXED) {
          AT(ops, nops++, p.cap_ops) = mk_op(p, tk + p.app_delay, static_cast<uint32_t>(p.app_delay), i, sub, 0, m,
                              OP_BCAST, 0);
        } else {
          AT(ops, nops++, p.cap_ops) = mk_op(p, tk, 0, i, sub, static_cast<uint32_t>(draws), m, OP_BCAST_J, 0);
          draws += deg;
        }
        sub += deg;
      };
      push_bcast(blk);
      ++nround;
      AT(p.g_n, rep, p.R) = n_seq + 1;
      if (p.pbft_view_change) {  // rand() % 100 == 5 -> viewChange() :401-403
        int32_t r;
        if (p.rng_mode == BCSIM_RNG_GLIBC) {
          const uint32_t pos = AT(p.glibc_pos, rep, p.R)++;
          if (pos >= p.glibc_len) set_err(p, BCSIM_E_OVERFLOW);
          r = AT(p.glibc, static_cast<size_t>(rep) * p.glibc_len + (pos % p.glibc_len), p.cap_glibc);
        } else {
          r = ctr_rand(p.seed, rep, i, draws++);
        }
        if (r % 100 == 5) {  // viewChange :293-303
          const int32_t nl = (AT(p.leader, g, p.NT) + 1) % static_cast<int32_t>(N);
          AT(p.leader, g, p.NT) = nl;
          v_cur += 1;
          const uint32_t pos = atomicAdd(p.vlog_cnt, 1u);
          if (pos < p.cap_vlog) {
            VLog e;
            e.t = tk;
            e.ts = ts_tick;
            e.origin = i;
            e.sub = AT(p.tick_sub, g, p.NT);
            e.target = i;
            e.rep = rep;
            e.v = v_cur;
            e.pad = 0;
            AT(p.vlog, pos, p.cap_vlog) = e;
          } else {
            set_err(p, BCSIM_E_OVERFLOW);
          }
          push_bcast(mkmsg(PB_VIEW_CHANGE, enc_raw(p, v_cur), enc_raw(p, nl), 0, 0));
        }
      }
      AT(p.sub, g, p.NT) = sub;
      AT(p.n_ops, g, p.NT) = nops;
      AT(p.draws, g, p.NT) = draws;
      AT(p.node_onext, g, p.NT) = LLONG_MIN;
    }
    AT(p.g_nround, rep, p.R) = nround;
  }
  __syncthreads();
  // every alive node: n_round seen = n_round0 + #leaders with id <= i
  // (prefix over the leader flags), reschedule, stop check.
  __shared__ int32_t chunk_base;
  if (tid == 0) chunk_base = 0;
  __syncthreads();
  for (uint32_t base = 0; base < N; base += blockDim.x) {
    const uint32_t i = base + tid;
    const uint32_t f = (i < N) ? lead[i] : 0u;
    // block inclusive prefix of f
    __shared__ int32_t sc[1024];
    sc[tid] = static_cast<int32_t>(f);
    __syncthreads();
    for (uint32_t off = 1; off < blockDim.x; off <<= 1) {
      const int32_t y = tid >= off ? sc[tid - off] : 0;
      __syncthreads();
      sc[tid] += y;
      __syncthreads();
    }
    if (i < N) {
      const uint32_t g = rep * N + i;
      if (AT(p.tick_alive, g, p.NT)) {
        const int32_t nr = nround0 + chunk_base + sc[tid];
        const uint32_t fired = AT(p.tick_sub, g, p.NT);  // sub of the executing SendBlock
        const uint32_t s = AT(p.sub, g, p.NT);
        AT(p.tick_sub, g, p.NT) = s;  // blockEvent = Schedule(Seconds(timeout), SendBlock) :406
        AT(p.sub, g, p.NT) = s + 1;
        atomicAdd(&n_ticked, 1);
        if (nr == static_cast<int32_t>(p.pbft_rounds)) {  // :407-410
          const uint32_t pos = atomicAdd(p.trace_cnt, 1u);
          if (pos < p.cap_trace) {
            bcsim_trace_rec tr;
            tr.t_ns = tk;
            tr.key_ts = ts_tick;
            tr.key_origin = i;
            tr.key_sub = fired;
            tr.replica = rep;
            tr.node = i;
            tr.kind = BCSIM_TR_PBFT_STOP;
            tr.a = nr;
            tr.b = 0;
            tr.c = 0;
            AT(p.trace, pos, p.cap_trace) = tr;
          } else {
            set_err(p, BCSIM_E_OVERFLOW);
          }
          AT(p.tick_alive, g, p.NT) = 0;
        } else {
          atomicAdd(&n_alive, 1);
        }
      }
    }
    __syncthreads();
    if (tid == blockDim.x - 1) chunk_base += sc[tid];
    __syncthreads();
  }
  if (tid == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(&p.scal[2]), static_cast<unsigned long long>(n_alive));
    if (n_ticked > 0) {
      unsigned long long* cnt = &AT(p.counters, static_cast<size_t>(rep) * CNT_N, static_cast<uint64_t>(p.R) * CNT_N);
      atomicAdd(&cnt[CNT_EVENTS], static_cast<unsigned long long>(n_ticked));
      atomicMax(reinterpret_cast<long long*>(&cnt[CNT_TLAST]), tk);
    }
  }
}

// ---------------------------------------------------------------------------
// glibc election-timeout draws (Raft), canonical global order per replica.
__global__ void k_draws(const KP* __restrict__ pk, uint32_t) {
  const KP& p = *pk;
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t n = min(*p.dreq_cnt, p.cap_dreq);
  if (n == 0) return;
  // insertion sort by (rep, t, ts, origin, sub, target): n is small
  for (uint32_t a = 1; a < n; ++a) {
    const DrawReq x = AT(p.dreq, a, p.cap_dreq);
    uint32_t b = a;
    while (b > 0) {
      const DrawReq& y = AT(p.dreq, b - 1, p.cap_dreq);
      bool less = x.rep != y.rep ? x.rep < y.rep
                : x.t != y.t ? x.t < y.t
                : x.ts != y.ts ? x.ts < y.ts
                : x.origin != y.origin ? x.origin < y.origin
                : x.sub != y.sub ? x.sub < y.sub
                : x.target < y.target;
      if (!less) break;
      AT(p.dreq, b, p.cap_dreq) = AT(p.dreq, b - 1, p.cap_dreq);
      --b;
    }
    AT(p.dreq, b, p.cap_dreq) = x;
  }
  for (uint32_t k = 0; k < n; ++k) {
    const DrawReq& d = AT(p.dreq, k, p.cap_dreq);
    const uint32_t pos = AT(p.glibc_pos, d.rep, p.R)++;
    if (pos >= p.glibc_len) {
      set_err(p, BCSIM_E_OVERFLOW);
      return;
    }
    const int32_t r = AT(p.glibc, static_cast<size_t>(d.rep) * p.glibc_len + pos, p.cap_glibc);
    const uint32_t g = d.rep * p.N + d.target;
    TimerEnt* tm = p.timers + static_cast<size_t>(g) * p.cap_timers;
    for (uint32_t s = 0; s < p.cap_timers; ++s) {
      if (tm[s].pending_draw && tm[s].sub == d.timer_sub) {
        tm[s].pending_draw = 0;
        tm[s].t = d.t + AT(p.raft_elec, r % 150, 150);
        if (tm[s].alive && tm[s].t < AT(p.node_tnext, g, p.NT)) AT(p.node_tnext, g, p.NT) = tm[s].t;
      }
    }
  }
  *p.dreq_cnt = 0;
}

// global min over node_tnext / node_onext
__global__ __launch_bounds__(1024) void k_next(const KP* __restrict__ pk) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ long long red[1024];
  long long m = LLONG_MAX;
  for (uint32_t k = threadIdx.x; k < p.NT; k += blockDim.x) {
    const long long a = AT(p.node_tnext, k, p.NT), b = AT(p.node_onext, k, p.NT);
    m = min(m, min(a, b));
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (uint32_t s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = min(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) p.scal[0] = red[0];
}

}  // namespace bcsim
