/*
 * bcsim_oracle.c — serial CPU ORACLE (discrete-event restatement) of the
 * blockchain-simulator hot path.  TEST INFRASTRUCTURE ONLY: loaded by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline, never by the product.
 *
 * PARITY STATUS (header as required by DESIGN.md §3):
 *   - glibc rand(): PINNED (restated TYPE_3 generator, checked against libc).
 *   - protocol handlers: restated line by line from the reference sources,
 *     citations below; quirks kept (echo, Paxos off-by-one broadcast, PBFT
 *     shared globals, Raft vote counters shared with heartbeat counters).
 *   - ns-3 L1 semantics (event tie order, p2p link FIFO/serialization,
 *     IPv4 fragmentation, float->Time rounding): PARITY UNPINNED.  ns-3 is not
 *     present anywhere in this image and the reference has no tests or golden
 *     logs; the model below is documented in DESIGN.md §2 and is the contract
 *     the GPU engine is held to bit-exactly.
 *
 * Undefined behaviour in the reference gets one fixed meaning:
 *   uninitialised payload bytes = 0 (NUL; getPacketContent then truncates);
 *   PbftNode::tx[] zero-initialised; generateTX's dangling pointer = the
 *   intended header bytes; Paxos *end() broadcast target = dropped send that
 *   still consumes one rand() draw and one schedule; compat-encoded negative
 *   tx[] index -> BCSIM_E_ENCODING, index >= pbft_seq_cap -> BCSIM_E_INDEX.
 *
 * Event order (canonical key): (t, t_sched, origin, sub, target) where
 *   t_sched = time the event was scheduled (START/STOP: -1; RECV: transmit
 *   start of the packet's last frame), origin = node whose code scheduled it
 *   (RECV: the sender), sub = origin's running schedule counter (RECV: the
 *   sub of the SendPacket that produced it).  Equal-time events on one node
 *   therefore run in ns-3's scheduling order whenever their schedulers ran at
 *   different times; true ties fall back to node id.
 */
#include "oracle.h"

#include <limits.h>
#include <stdio.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* glibc TYPE_3 random() restatement (glibc stdlib/random_r.c, srandom_r +
 * random_r; rand() == random()).  Reference call sites: pbft-node.cc:68,401,
 * raft-node.cc:65,71, paxos-node.cc:399.  Never seeded in the reference
 * (default seed 1).                                                        */
typedef struct {
  int32_t st[31];
  int f, r;
} glibc_rng;

static int32_t glibc_next(glibc_rng* g) {
  uint32_t val = (uint32_t)g->st[g->f] + (uint32_t)g->st[g->r];
  g->st[g->f] = (int32_t)val;
  int32_t out = (int32_t)(val >> 1);
  if (++g->f >= 31) {
    g->f = 0;
    ++g->r;
  } else if (++g->r >= 31) {
    g->r = 0;
  }
  return out;
}

static void glibc_seed(glibc_rng* g, uint32_t seed) {
  int32_t word = (int32_t)(seed == 0 ? 1u : seed);
  g->st[0] = word;
  for (int i = 1; i < 31; ++i) {
    long hi = word / 127773;
    long lo = word % 127773;
    long w = 16807 * lo - 2836 * hi;
    if (w < 0) w += 2147483647;
    word = (int32_t)w;
    g->st[i] = word;
  }
  g->f = 3;
  g->r = 0;
  for (int k = 0; k < 310; ++k) (void)glibc_next(g);
}

void oracle_glibc_rand_seq(uint32_t seed, uint32_t n, int32_t* out) {
  glibc_rng g;
  glibc_seed(&g, seed);
  for (uint32_t i = 0; i < n; ++i) out[i] = glibc_next(&g);
}

/* Counter RNG (build extension, order independent): splitmix64 chain. */
static uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
uint32_t oracle_ctr_rand(uint64_t seed, uint32_t replica, uint32_t node,
                         uint64_t k) {
  uint64_t h = sm64(seed);
  h = sm64(h ^ (uint64_t)replica);
  h = sm64(h ^ (uint64_t)node);
  h = sm64(h ^ k);
  return (uint32_t)(h >> 33);
}

/* ------------------------------------------------------------------------ */
/* ns-3 Seconds(double) -> int64 ns.  int64x64_t(double) keeps 64 fractional
 * bits (truncating below 2^-64), multiplication by the integer factor 1e9 is
 * exact, then Time(int64x64_t) takes Round() (half away from zero) or
 * GetHigh() (floor).  Unpinned: the ns-3 version is not recorded.          */
int64_t oracle_seconds_to_ns(double s, int mode) {
  if (s == 0.0) return 0;
  int neg = s < 0;
  double v = neg ? -s : s;
  int e;
  double m = frexp(v, &e); /* v = m * 2^e, m in [0.5,1) */
  uint64_t M = (uint64_t)ldexp(m, 53);
  int E = e - 53; /* v = M * 2^E */
  unsigned __int128 q; /* floor(v * 2^64) */
  int sh = E + 64;
  if (sh >= 0)
    q = (unsigned __int128)M << sh;
  else if (sh > -128)
    q = (unsigned __int128)M >> (-sh);
  else
    q = 0;
  uint64_t hi = (uint64_t)(q >> 64);
  uint64_t lo = (uint64_t)q;
  unsigned __int128 f = (unsigned __int128)lo * 1000000000ull;
  uint64_t ns = hi * 1000000000ull + (uint64_t)(f >> 64);
  uint64_t rem = (uint64_t)f;
  if (mode == BCSIM_TIME_ROUND && rem >= (1ull << 63)) ns += 1;
  return neg ? -(int64_t)ns : (int64_t)ns;
}

/* DataRate::CalculateBytesTxTime: Seconds(double(bytes) * 8 / bps). */
int64_t oracle_tx_ns(uint32_t wire_bytes, uint64_t rate_bps, int mode) {
  double s = (double)wire_bytes * 8 / (double)rate_bps;
  return oracle_seconds_to_ns(s, mode);
}

/* UDP(8) + IPv4(20) + PPP(2); IPv4 fragments of (mtu-20)&~7 payload bytes. */
void oracle_msg_tx(uint32_t payload, uint32_t mtu, uint64_t rate_bps, int mode,
                   int64_t* tx_total, int64_t* tx_last, uint32_t* n_frames,
                   uint32_t* wire_total) {
  uint32_t ipp = payload + 8;
  uint32_t room = mtu - 20;
  uint32_t frag = room & ~7u;
  int64_t tot = 0, last = 0;
  uint32_t nf = 0, wt = 0;
  if (ipp <= room) {
    uint32_t w = ipp + 22;
    last = oracle_tx_ns(w, rate_bps, mode);
    tot = last;
    nf = 1;
    wt = w;
  } else {
    uint32_t left = ipp;
    while (left > 0) {
      uint32_t p = left > frag ? frag : left;
      uint32_t w = p + 22;
      last = oracle_tx_ns(w, rate_bps, mode);
      tot += last;
      wt += w;
      ++nf;
      left -= p;
    }
  }
  if (tx_total) *tx_total = tot;
  if (tx_last) *tx_last = last;
  if (n_frames) *n_frames = nf;
  if (wire_total) *wire_total = wt;
}

/* float seconds from the reference's delay helpers, then Seconds(). */
static int64_t fsec_ns(float f, int mode) {
  return oracle_seconds_to_ns((double)f, mode);
}

/* ------------------------------------------------------------------------ */
/* Events */
enum { EV_START = 0, EV_STOP = 1, EV_TIMER = 2, EV_SEND = 3, EV_RECV = 4,
       EV_WAKE = 5 /* FQCODEL: a link's device queue has room again (t_sched -2) */ };
/* timer kinds */
enum {
  TM_PBFT_BLOCK = 0,
  TM_RAFT_ELECTION = 1,
  TM_RAFT_HEARTBEAT = 2,
  TM_RAFT_PROPOSAL = 3,
  TM_PAXOS_TICKET = 4,
  TM_GOSSIP_BLOCK = 5
};

typedef struct {
  int32_t type;  /* charToInt(msg[0]) */
  int32_t f[3];  /* raw chars data[1..3] (0 = NUL / uninitialised) */
  int32_t big;   /* 0 = small control payload, 1 = block / proposal */
} omsg;

typedef struct {
  int64_t t, ts;
  uint32_t origin, sub, target, kind;
  uint32_t aux;  /* TIMER: kind; SEND: edge (UINT32_MAX = dropped);
                    RECV: edge the packet travelled */
  omsg m;
} oev;

typedef struct {
  uint32_t sub;
  uint64_t draws;
  /* PBFT (pbft-node.h:39-56) */
  int32_t leader, block_num;
  uint32_t block_ev;
  /* Raft (raft-node.h:39-53) */
  int32_t is_leader, has_voted, m_value, vote_success, vote_failed;
  int32_t add_change_value, blockNum, round;
  uint32_t next_election, next_heartbeat;
  /* Paxos (paxos-node.h:40-52); acceptor fields per decree in o->px */
  int32_t ticket, proposal, decree;
  /* cancelled timer ids (ns-3 Simulator::Cancel) */
  uint32_t* cancelled;
  uint32_t n_cancelled, cap_cancelled;
} onode;

typedef struct {
  oev* a;
  size_t n, cap;
} oheap;

/* DROPTAIL link queue: the messages of the link's current busy
 * period, back to back in FIFO order; k = frames accepted (a prefix of the message) */
typedef struct {
  int64_t start;
  uint32_t k, big;
} qent;
typedef struct {
  qent* a;
  uint32_t head, n, cap;
  uint64_t frames; /* frames of the entries in the deque */
} oqueue;

/* FQCODEL link: ns-3 FqCoDelQueueDisc in front of the device queue.
 * A packet is one IPv4 fragment of a message; flows are the <= 3 distinct flow indices
 * of the link's traffic classes (first fragments of application sends, first fragments
 * of echoes, later fragments of either: ports 0). */
typedef struct {
  int64_t enq;    /* enqueue time (CoDel timestamp) */
  uint32_t msg;   /* index into the link's message table */
  uint32_t size;  /* IPv4 packet bytes (QueueDiscItem::GetSize) */
  uint32_t frame; /* fragment index */
} fqpkt;
typedef struct {
  fqpkt* a;
  uint32_t head, n, cap;
  uint32_t bytes;
  /* CoDelQueueDisc state (codel time units: ns >> 10) */
  uint32_t first_above, drop_next, count, last_count;
  uint16_t rec_inv_sqrt;
  int dropping;
  int status;  /* 0 inactive, 1 new, 2 old */
  int32_t deficit;
  int created; /* queue-disc class index (creation order), -1 = not created */
} fqflow;
typedef struct {
  omsg m;
  uint32_t sub, left;
  int echo, lost, used;
} fqmsg;
typedef struct {
  fqflow f[3];
  int newl[3], oldl[3], n_new, n_old, n_created;
  int64_t* dev; /* start times of the waiting device frames (ring of dcap <= fq_devcap, grown) */
  uint32_t dh, dn, dcap;
  uint32_t edge;
  int64_t dev_end;
  int stopped;
  uint32_t qpkts;
  fqmsg* msg;
  uint32_t nmsg, capmsg;
  /* flow of each packet class (app / echo first fragments, later fragments), bound when the
   * class first reaches the disc: its slot and Murmur3 flow index (fq_class_slot) */
  uint32_t cslot[3], chash[3];
  int cbound[3];
} fqlink;

struct bcsim_oracle {
  bcsim_config cfg;
  uint32_t N;
  /* topology (sender-major CSR) */
  uint32_t *row, *col, *rev, *eid_of_pos;
  int64_t* prop;
  int topo_set;
  /* per replica state */
  uint32_t R;
  uint32_t cur_rep;
  onode* nodes;          /* N, for the replica being run */
  int32_t *tx_val, *tx_pv, *tx_cv; /* N * seq_cap */
  uint8_t* gseen;        /* GOSSIP: N * seq_cap first-receipt flags */
  int32_t* px;           /* PAXOS: [N][decrees][4] t_max, command, t_store, isCommit */
  uint32_t K;            /* Paxos decrees (>= 1) */
  int64_t* busy;         /* per edge */
  oqueue* q;             /* per edge (DROPTAIL only) */
  fqlink** fq;           /* per edge (FQCODEL only), created at the edge's first packet: at
                          * n=4096 the full mesh has 16.8 M links, most of them holding a few
                          * packets, so every per-link array starts small and grows */
  uint32_t* fqlnk;       /* per edge: its link's number in the mesh loop (the /24 network) */
  uint32_t* fqport;      /* per edge: UDP port of the sender's client socket, 0 = not bound yet */
  uint32_t* fqnport;     /* per node: client sockets bound so far (ephemeral ports 49153, ...) */
  uint8_t* fqphant;      /* per node: the Paxos *end() socket is bound */
  uint32_t fq_limit, fq_quantum, fq_flows, fq_batch, fq_min_bytes, fq_devcap;
  uint32_t fq_target_c, fq_interval_c; /* CoDel units (ns >> 10) */
  uint32_t ip_full[2], ip_last[2];     /* IPv4 packet bytes of a full / the last fragment */
  /* debug (ORACLE_FQLOG=<file>): FQCODEL link events, the engine's BCSIM_FQLOG format */
  uint32_t* flog;
  size_t nflog, capflog;
  int64_t flog_t0, flog_t1;
  int flog_on;
  uint32_t nfr[2];       /* frames per message class (small, big) */
  int64_t tx_full[2];    /* time of a full (non-last) fragment frame */
  oheap heap;
  glibc_rng grng;
  int32_t g_v, g_n, g_nround; /* PBFT file-scope globals pbft-node.cc:24-30 */
  /* precomputed times */
  int64_t tx_tot[2], tx_last[2];
  int64_t pbft_period, raft_hb, pbft_delay[3], raft_delay[3], raft_elec[150],
      paxos_delay[50];
  uint32_t small_bytes, big_bytes;
  /* outputs */
  bcsim_trace_rec* tr;
  uint64_t ntr, cap_tr;
  bcsim_counters cnt;
  int64_t now;
  int32_t err;
  int started;
  /* per-replica run bookkeeping (replicas run one after another) */
  int64_t* rep_now;
  int run_all_done;
};

/* canonical key compare */
static int ev_less(const oev* x, const oev* y) {
  if (x->t != y->t) return x->t < y->t;
  if (x->ts != y->ts) return x->ts < y->ts;
  if (x->origin != y->origin) return x->origin < y->origin;
  if (x->sub != y->sub) return x->sub < y->sub;
  return x->target < y->target;
}

static int heap_push(oheap* h, const oev* e) {
  if (h->n == h->cap) {
    size_t nc = h->cap ? h->cap * 2 : 1024;
    oev* na = (oev*)realloc(h->a, nc * sizeof(oev));
    if (!na) return BCSIM_E_NOMEM;
    h->a = na;
    h->cap = nc;
  }
  size_t i = h->n++;
  while (i > 0) {
    size_t p = (i - 1) / 2;
    if (!ev_less(e, &h->a[p])) break;
    h->a[i] = h->a[p];
    i = p;
  }
  h->a[i] = *e;
  return BCSIM_OK;
}

static void heap_pop(oheap* h, oev* out) {
  *out = h->a[0];
  oev last = h->a[--h->n];
  size_t i = 0, n = h->n;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    const oev* best = &last;
    if (l < n && ev_less(&h->a[l], best)) {
      m = l;
      best = &h->a[l];
    }
    if (r < n && ev_less(&h->a[r], best)) m = r;
    if (m == i) break;
    h->a[i] = h->a[m];
    i = m;
  }
  if (n) h->a[i] = last;
}

/* ------------------------------------------------------------------------ */
/* helpers */
static int32_t enc(const bcsim_oracle* o, int32_t a) { /* intToChar */
  int32_t c = a + '0';
  if (o->cfg.encoding == BCSIM_ENC_COMPAT) c = (int32_t)(int8_t)(uint8_t)c;
  return c;
}
static int32_t dec(int32_t c) { return c - '0'; } /* charToInt */
static int32_t as_char(const bcsim_oracle* o, int32_t c) { /* char member */
  if (o->cfg.encoding == BCSIM_ENC_COMPAT) c = (int32_t)(int8_t)(uint8_t)c;
  return c;
}
/* msg[i] after getPacketContent's NUL truncation (pbft-node.cc:305-320) */
static int32_t mchar(const omsg* m, int i) {
  if (i == 0) return m->type + '0';
  for (int k = 0; k < i - 1; ++k)
    if (m->f[k] == 0) return 0;
  return m->f[i - 1];
}

static void set_err(bcsim_oracle* o, int32_t e) {
  if (!o->err) o->err = e;
}

static int32_t draw(bcsim_oracle* o, uint32_t node) {
  onode* nd = &o->nodes[node];
  if (o->cfg.rng_mode == BCSIM_RNG_GLIBC) return glibc_next(&o->grng);
  return (int32_t)oracle_ctr_rand(o->cfg.seed, o->cur_rep, node, nd->draws++);
}

static void emit(bcsim_oracle* o, const oev* e, uint32_t node, uint32_t kind,
                 int32_t a, int32_t b, int32_t c) {
  if (o->ntr == o->cap_tr) {
    uint64_t nc = o->cap_tr ? o->cap_tr * 2 : 4096;
    bcsim_trace_rec* nt =
        (bcsim_trace_rec*)realloc(o->tr, nc * sizeof(bcsim_trace_rec));
    if (!nt) {
      set_err(o, BCSIM_E_NOMEM);
      return;
    }
    o->tr = nt;
    o->cap_tr = nc;
  }
  bcsim_trace_rec* r = &o->tr[o->ntr++];
  r->t_ns = e->t;
  r->key_ts = e->ts;
  r->key_origin = e->origin;
  r->key_sub = e->sub;
  r->replica = o->cur_rep;
  r->node = node;
  r->kind = kind;
  r->a = a;
  r->b = b;
  r->c = c;
}

static uint32_t sched_timer(bcsim_oracle* o, uint32_t node, uint32_t tk,
                            int64_t delay) {
  onode* nd = &o->nodes[node];
  oev e;
  memset(&e, 0, sizeof e);
  e.t = o->now + delay;
  e.ts = o->now;
  e.origin = node;
  e.sub = nd->sub++;
  e.target = node;
  e.kind = EV_TIMER;
  e.aux = tk;
  int rc = heap_push(&o->heap, &e);
  if (rc) set_err(o, rc);
  return e.sub;
}

static void cancel_timer(bcsim_oracle* o, uint32_t node, uint32_t id) {
  onode* nd = &o->nodes[node];
  if (id == 0) return;
  if (nd->n_cancelled == nd->cap_cancelled) {
    uint32_t nc = nd->cap_cancelled ? nd->cap_cancelled * 2 : 8;
    uint32_t* na = (uint32_t*)realloc(nd->cancelled, nc * sizeof(uint32_t));
    if (!na) {
      set_err(o, BCSIM_E_NOMEM);
      return;
    }
    nd->cancelled = na;
    nd->cap_cancelled = nc;
  }
  nd->cancelled[nd->n_cancelled++] = id;
}

static int take_cancelled(onode* nd, uint32_t id) {
  for (uint32_t i = 0; i < nd->n_cancelled; ++i)
    if (nd->cancelled[i] == id) {
      nd->cancelled[i] = nd->cancelled[--nd->n_cancelled];
      return 1;
    }
  return 0;
}

/* Simulator::Schedule(Seconds(delay), SendPacket, sock, p) */
static void sched_send(bcsim_oracle* o, uint32_t node, uint32_t edge,
                       int64_t delay, const omsg* m) {
  onode* nd = &o->nodes[node];
  oev e;
  memset(&e, 0, sizeof e);
  e.t = o->now + delay;
  e.ts = o->now;
  e.origin = node;
  e.sub = nd->sub++;
  e.target = node;
  e.kind = EV_SEND;
  e.aux = edge;
  e.m = *m;
  int rc = heap_push(&o->heap, &e);
  if (rc) set_err(o, rc);
}

static int64_t app_delay(bcsim_oracle* o, uint32_t node) {
  if (o->cfg.delay_mode == BCSIM_DELAY_FIXED) return o->cfg.app_delay_ns;
  int32_t r = draw(o, node);
  switch (o->cfg.protocol) {
    case BCSIM_PBFT:
      return o->pbft_delay[r % 3];
    case BCSIM_RAFT:
      return o->raft_delay[r % 3];
    case BCSIM_GOSSIP: /* PBFT-style: getRandomDelay pbft-node.cc:66-69 */
      return o->pbft_delay[r % 3];
    default:
      return o->paxos_delay[r % 50];
  }
}

/* broadcast Send(uint8_t[]): pbft-node.cc:349-368, raft-node.cc:370-388 */
static void bcast(bcsim_oracle* o, uint32_t node, const omsg* m) {
  for (uint32_t p = o->row[node]; p < o->row[node + 1]; ++p) {
    int64_t d = app_delay(o, node);
    sched_send(o, node, p, d, m);
  }
}
/* Paxos broadcast paxos-node.cc:450-505: iterator advanced before use, so
 * peers[1..deg-1] are reached and the last iteration targets *end()
 * (dropped); every iteration draws a delay and schedules a SendPacket.     */
static void bcast_paxos(bcsim_oracle* o, uint32_t node, const omsg* m) {
  uint32_t b = o->row[node], e = o->row[node + 1];
  for (uint32_t p = b; p < e; ++p) {
    int64_t d = app_delay(o, node);
    uint32_t edge = (p + 1 < e) ? p + 1 : UINT32_MAX;
    sched_send(o, node, edge, d, m);
  }
}
/* unicast Send(data, from): pbft-node.cc:328-346 */
static void unicast(bcsim_oracle* o, uint32_t node, uint32_t in_edge,
                    const omsg* m) {
  int64_t d = app_delay(o, node);
  sched_send(o, node, o->rev[in_edge], d, m);
}

static omsg mk(int32_t type, int32_t f0, int32_t f1, int32_t f2, int32_t big) {
  omsg m;
  m.type = type;
  m.f[0] = f0;
  m.f[1] = f1;
  m.f[2] = f2;
  m.big = big;
  return m;
}

/* DROPTAIL: frames of queue entry e that started transmission by time t (frame j
 * of a message starting at s starts at s + j * tx_full; a frame starting at t is
 * no longer waiting) */
static uint32_t q_started(const bcsim_oracle* o, const qent* e, int64_t t) {
  if (t < e->start) return 0;
  if (o->nfr[e->big] == 1) return e->k;
  int64_t j = (t - e->start) / o->tx_full[e->big] + 1;
  return j < (int64_t)e->k ? (uint32_t)j : e->k;
}

/* DROPTAIL admission at o->now of a message of class big that would start at
 * `start`: frames are accepted while fewer than queue_dev_pkts + queue_disc_pkts
 * frames wait on the link (pfifo_fast in front of the device queue, flow control;
 * the frame in transmission does not count).  Returns the accepted prefix. */
static uint32_t q_admit(bcsim_oracle* o, uint32_t edge, int big, int64_t start) {
  oqueue* q = &o->q[edge];
  while (q->n && q_started(o, &q->a[q->head], o->now) == q->a[q->head].k) {
    q->frames -= q->a[q->head].k;
    q->head = (q->head + 1) % q->cap;
    --q->n;
  }
  uint64_t waiting = q->n ? q->frames - q_started(o, &q->a[q->head], o->now) : 0;
  uint64_t cap = (uint64_t)o->cfg.queue_dev_pkts + o->cfg.queue_disc_pkts;
  uint32_t F = o->nfr[big];
  uint32_t k = waiting >= cap ? 0 : (uint32_t)((cap - waiting) < F ? (cap - waiting) : F);
  if (!k) return 0;
  if (q->n == q->cap) { /* grow the ring */
    uint32_t nc = q->cap ? 2 * q->cap : 16;
    qent* na = (qent*)malloc(nc * sizeof(qent));
    if (!na) {
      set_err(o, BCSIM_E_NOMEM);
      return 0;
    }
    for (uint32_t i = 0; i < q->n; ++i) na[i] = q->a[(q->head + i) % q->cap];
    free(q->a);
    q->a = na;
    q->head = 0;
    q->cap = nc;
  }
  qent* e = &q->a[(q->head + q->n) % q->cap];
  e->start = start;
  e->k = k;
  e->big = (uint32_t)big;
  ++q->n;
  q->frames += k;
  return k;
}

/* link FIFO (+ DROPTAIL): returns the arrival time and sets *ts_last, or returns
 * -1 if a fragment was dropped (the message is lost; its accepted frames still
 * occupy the link) */
static int64_t link_xmit(bcsim_oracle* o, uint32_t edge, int big,
                         int64_t* ts_last) {
  int64_t start = o->busy[edge] > o->now ? o->busy[edge] : o->now;
  if (o->cfg.queue_model == BCSIM_QUEUE_DROPTAIL) {
    uint32_t F = o->nfr[big];
    uint32_t k = q_admit(o, edge, big, start);
    if (k < F) {
      o->cnt.frames_dropped += F - k;
      if (k) o->busy[edge] = start + (int64_t)k * o->tx_full[big];
      return -1;
    }
  }
  int64_t end = start + o->tx_tot[big];
  o->busy[edge] = end;
  *ts_last = end - o->tx_last[big];
  return end + o->prop[edge];
}

/* ------------------------------------------------------------------------ */
/* FQCODEL.  ns-3 FqCoDelQueueDisc / CoDelQueueDisc restated
 * (src/traffic-control/model/fq-codel-queue-disc.cc, codel-queue-disc.cc; the
 * ns-3 version is not recorded, so this is PARITY UNPINNED like the rest of L1):
 *   classify: Ipv4QueueDiscItem::Hash = Murmur3-32 (seed 0x8BADF00D) of
 *             src | dst | proto 17 | sport | dport | perturbation (17 bytes, big
 *             endian; ports 0 for a non-first fragment) mod Flows;
 *   enqueue:  an inactive flow becomes new with deficit = Quantum; more than
 *             MaxSize packets -> FqCoDelDrop (half the fattest flow's bytes, at
 *             most DropBatchSize packets, from its head);
 *   dequeue:  DRR over new then old flows; each flow is a CoDel queue (Target,
 *             Interval, MinBytes, Newton-step inverse sqrt control law).
 * The device queue (queue_dev_pkts) stops the disc when full and wakes it when
 * its oldest waiting frame starts transmission (flow control); a wake at t runs
 * before every other event at t. */

/* sender of edge e (sender-major CSR) */
static uint32_t edge_src(const bcsim_oracle* o, uint32_t e) {
  uint32_t lo = 0, hi = o->N; /* row[lo] <= e < row[hi] */
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) / 2;
    if (o->row[mid] <= e)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

/* MurmurHash3_x86_32 (Austin Appleby's public algorithm; ns-3 hash-murmur3.cc) */
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
uint32_t oracle_murmur3_32(const uint8_t* data, uint32_t len, uint32_t seed) {
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  uint32_t h = seed, nb = len / 4;
  for (uint32_t i = 0; i < nb; ++i) {
    uint32_t k = (uint32_t)data[4 * i] | ((uint32_t)data[4 * i + 1] << 8) |
                 ((uint32_t)data[4 * i + 2] << 16) | ((uint32_t)data[4 * i + 3] << 24);
    k *= c1;
    k = rotl32(k, 15);
    k *= c2;
    h ^= k;
    h = rotl32(h, 13);
    h = h * 5 + 0xe6546b64u;
  }
  const uint8_t* t = data + 4 * nb;
  uint32_t k = 0;
  switch (len & 3) {
    case 3: k ^= (uint32_t)t[2] << 16; /* fall through */
    case 2: k ^= (uint32_t)t[1] << 8;  /* fall through */
    case 1:
      k ^= t[0];
      k *= c1;
      k = rotl32(k, 15);
      k *= c2;
      h ^= k;
  }
  h ^= len;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

/* Ipv4QueueDiscItem::Hash(perturbation) % flows for one packet class */
uint32_t oracle_fq_flow(uint32_t src, uint32_t dst, uint32_t sport, uint32_t dport,
                        uint32_t perturbation, uint32_t flows) {
  uint8_t b[17];
  uint32_t w[2] = {src, dst};
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < 4; ++j) b[4 * k + j] = (uint8_t)(w[k] >> (24 - 8 * j));
  b[8] = 17; /* UDP */
  b[9] = (uint8_t)(sport >> 8);
  b[10] = (uint8_t)sport;
  b[11] = (uint8_t)(dport >> 8);
  b[12] = (uint8_t)dport;
  for (int j = 0; j < 4; ++j) b[13 + j] = (uint8_t)(perturbation >> (24 - 8 * j));
  return oracle_murmur3_32(b, 17, 0x8BADF00Du) % flows;
}

/* The k-th link of the mesh loop (blockchain-simulator.cc:34-51, i outer, j < i inner) gets
 * network 1.0.0.0 + k*256 (address.NewNetwork), node i .1 and node j .2; a CSR graph numbers
 * its links the same way (larger endpoint ascending, then smaller). */
static void fq_build_links(bcsim_oracle* o) {
  uint32_t k = 0;
  for (uint32_t a = 0; a < o->N; ++a)
    for (uint32_t e = o->row[a]; e < o->row[a + 1]; ++e)
      if (o->col[e] < a) {
        o->fqlnk[e] = k;
        o->fqlnk[o->rev[e]] = k;
        ++k;
      }
}

/* Client sockets are created and Connect()ed in peer order at StartApplication
 * (pbft-node.cc:131-140, raft-node.cc:100-111, paxos-node.cc:110-119), but ns-3's
 * UdpSocketImpl::Connect only records the default peer: the socket binds -- takes the node's
 * next ephemeral port, 49153, 49154, ... (Ipv4EndPointDemux::AllocateEphemeralPort) -- in
 * DoSend, at its FIRST SendPacket.  Ports therefore follow the order of first sends, i.e. the
 * event order of the node's SendPacket events.  edge = UINT32_MAX is Paxos's *end() socket
 * (paxos-node.cc:481-493): it binds too, then the datagram finds no route. */
static void fq_bind(bcsim_oracle* o, uint32_t node, uint32_t edge) {
  if (edge == UINT32_MAX) {
    if (o->fqphant[node]) return;
    o->fqphant[node] = 1;
  } else if (o->fqport[edge]) {
    return;
  }
  uint32_t port = 49153 + o->fqnport[node]++;
  if (port > 65535) { /* the 16383 ephemeral ports are used up (the reference's Bind fails) */
    set_err(o, BCSIM_E_UNSUPPORTED);
    return;
  }
  if (edge != UINT32_MAX) o->fqport[edge] = port;
}

/* the flow slot of packet class cls (0 app, 1 echo first fragment, 2 later fragment) on edge:
 * bound at the class's first packet -- it shares the slot of an already bound class with the
 * same flow index (hash collision), else takes slot cls.  App packets travel from the
 * sender's client port to 7071, echoes from 7071 to the receiver's client port for the
 * sender (the reverse edge's), later fragments carry no ports. */
static uint32_t fq_class_slot(bcsim_oracle* o, uint32_t edge, fqlink* l, int cls) {
  if (l->cbound[cls]) return l->cslot[cls];
  uint32_t s = edge_src(o, edge), d = o->col[edge];
  uint32_t net = 0x01000000u + (o->fqlnk[edge] << 8);
  uint32_t src = net + (s > d ? 1u : 2u), dst = net + (d > s ? 1u : 2u);
  uint32_t sp = 0, dp = 0;
  if (cls == 0) {
    sp = o->fqport[edge];
    dp = 7071;
  } else if (cls == 1) {
    sp = 7071;
    dp = o->fqport[o->rev[edge]];
  }
  if (cls < 2 && (sp | dp) == 7071) set_err(o, BCSIM_E_STATE); /* a send from an unbound socket */
  uint32_t h = oracle_fq_flow(src, dst, sp, dp, o->cfg.fq_perturbation, o->fq_flows);
  uint32_t slot = (uint32_t)cls;
  for (int c = 0; c < 3; ++c)
    if (l->cbound[c] && l->chash[c] == h) {
      slot = l->cslot[c];
      break;
    }
  l->cbound[cls] = 1;
  l->chash[cls] = h;
  l->cslot[cls] = slot;
  return slot;
}

static void fq_free_link(fqlink* l) {
  for (int f = 0; f < 3; ++f) free(l->f[f].a);
  free(l->dev);
  free(l->msg);
  free(l);
}

/* the edge's link state, created at its first use */
static fqlink* fq_get(bcsim_oracle* o, uint32_t edge) {
  fqlink* l = o->fq[edge];
  if (l) return l;
  l = (fqlink*)calloc(1, sizeof(fqlink));
  if (!l) {
    set_err(o, BCSIM_E_NOMEM);
    return NULL;
  }
  for (int f = 0; f < 3; ++f) {
    l->f[f].rec_inv_sqrt = (uint16_t)(~0u >> 16);
    l->f[f].created = -1;
  }
  l->edge = edge;
  o->fq[edge] = l;
  return l;
}

static void fq_reset(bcsim_oracle* o) {
  for (uint32_t e = 0; e < o->row[o->N]; ++e)
    if (o->fq[e]) {
      fq_free_link(o->fq[e]);
      o->fq[e] = NULL;
    }
  memset(o->fqport, 0, (size_t)o->row[o->N] * sizeof(uint32_t));
  memset(o->fqnport, 0, (size_t)o->N * sizeof(uint32_t));
  memset(o->fqphant, 0, o->N);
}

static void free_fq(bcsim_oracle* o) {
  if (o->fq && o->row)
    for (uint32_t e = 0; e < o->row[o->N]; ++e)
      if (o->fq[e]) fq_free_link(o->fq[e]);
  free(o->fq);
  free(o->fqlnk);
  free(o->fqport);
  free(o->fqnport);
  free(o->fqphant);
  o->fq = NULL;
  o->fqlnk = o->fqport = o->fqnport = NULL;
  o->fqphant = NULL;
}

static int codel_before(uint32_t a, uint32_t b) { return (int32_t)(a - b) < 0; }
static int codel_after(uint32_t a, uint32_t b) { return (int32_t)(a - b) > 0; }
static int codel_after_eq(uint32_t a, uint32_t b) { return (int32_t)(a - b) >= 0; }
static uint16_t codel_newton(uint16_t rec, uint32_t count) {
  uint32_t invsqrt = ((uint32_t)rec) << 16;
  uint32_t invsqrt2 = (uint32_t)(((uint64_t)invsqrt * invsqrt) >> 32);
  uint64_t val = (3ull << 32) - ((uint64_t)count * invsqrt2);
  val >>= 2;
  val = (val * invsqrt) >> (32 - 2 + 1);
  return (uint16_t)(val >> 16);
}
static uint32_t codel_control_law(uint32_t t, uint32_t interval, uint16_t rec) {
  return t + (uint32_t)(((uint64_t)interval * ((uint32_t)rec << 16)) >> 32);
}

static void fq_free_msg(fqlink* l, uint32_t m) {
  l->msg[m].used = 0;
  while (l->nmsg && !l->msg[l->nmsg - 1].used) --l->nmsg;
}

/* kinds: 1 enqueue (x = flow slot), 2 into the device queue (x = frame start), 3 drop, 4 wake
 * (x = packets in the disc) */
static void fq_log(bcsim_oracle* o, const fqlink* l, uint32_t kind, const fqpkt* pk, int64_t x) {
  if (!o->flog_on || o->now < o->flog_t0 || o->now >= o->flog_t1) return;
  if (o->nflog == o->capflog) {
    size_t nc = o->capflog ? 2 * o->capflog : 4096;
    uint32_t* na = (uint32_t*)realloc(o->flog, nc * 8 * sizeof(uint32_t));
    if (!na) return;
    o->flog = na;
    o->capflog = nc;
  }
  uint32_t* r = o->flog + 8 * o->nflog++;
  uint32_t e = l->edge;
  r[0] = (uint32_t)o->now;
  r[1] = (uint32_t)((uint64_t)o->now >> 32);
  r[2] = e;
  r[3] = (kind << 24) | (pk ? pk->frame : 0);
  r[4] = pk ? l->msg[pk->msg].sub : 0;
  r[5] = (uint32_t)x;
  r[6] = (uint32_t)((uint64_t)x >> 32);
  r[7] = pk ? (uint32_t)l->msg[pk->msg].echo : 0;
}

/* a packet leaves the disc without transmission (CoDel or overlimit drop) */
static void fq_drop(bcsim_oracle* o, fqlink* l, const fqpkt* pk) {
  fq_log(o, l, 3, pk, 0);
  o->cnt.frames_dropped++;
  fqmsg* m = &l->msg[pk->msg];
  if (!m->lost) {
    m->lost = 1;
    if (!m->echo) o->cnt.msgs_lost++;
  }
  if (--m->left == 0) fq_free_msg(l, pk->msg);
}

static int fq_pop(fqlink* l, fqflow* F, fqpkt* out) {
  if (!F->n) return 0;
  *out = F->a[F->head];
  F->head = (F->head + 1) % F->cap;
  --F->n;
  F->bytes -= out->size;
  --l->qpkts;
  return 1;
}

/* CoDelQueueDisc::OkToDrop */
static int codel_ok_to_drop(bcsim_oracle* o, fqflow* F, const fqpkt* pk, uint32_t now_c) {
  if (!pk) {
    F->first_above = 0;
    return 0;
  }
  uint32_t soj = (uint32_t)((uint64_t)(o->now - pk->enq) >> 10);
  if (codel_before(soj, o->fq_target_c) || F->bytes < o->fq_min_bytes) {
    F->first_above = 0;
    return 0;
  }
  if (F->first_above == 0) {
    F->first_above = now_c + o->fq_interval_c;
  } else if (codel_after(now_c, F->first_above)) {
    return 1;
  }
  return 0;
}

/* CoDelQueueDisc::DoDequeue; returns 0 when the flow's queue is (or became) empty */
static int codel_dequeue(bcsim_oracle* o, fqlink* l, fqflow* F, fqpkt* out) {
  fqpkt pk;
  if (!fq_pop(l, F, &pk)) {
    F->dropping = 0;
    return 0;
  }
  uint32_t now_c = (uint32_t)((uint64_t)o->now >> 10);
  int have = 1;
  int ok = codel_ok_to_drop(o, F, &pk, now_c);
  if (F->dropping) {
    if (!ok) {
      F->dropping = 0;
    } else if (codel_after_eq(now_c, F->drop_next)) {
      while (F->dropping && codel_after_eq(now_c, F->drop_next)) {
        ++F->count;
        F->rec_inv_sqrt = codel_newton(F->rec_inv_sqrt, F->count);
        fq_drop(o, l, &pk);
        have = fq_pop(l, F, &pk);
        if (!codel_ok_to_drop(o, F, have ? &pk : NULL, now_c))
          F->dropping = 0;
        else
          F->drop_next = codel_control_law(F->drop_next, o->fq_interval_c, F->rec_inv_sqrt);
      }
    }
  } else if (ok) {
    fq_drop(o, l, &pk);
    have = fq_pop(l, F, &pk);
    (void)codel_ok_to_drop(o, F, have ? &pk : NULL, now_c);
    F->dropping = 1;
    int32_t delta = (int32_t)(F->count - F->last_count);
    if (delta > 1 && codel_before(now_c - F->drop_next, 16 * o->fq_interval_c)) {
      F->count = (uint32_t)delta;
      F->rec_inv_sqrt = codel_newton(F->rec_inv_sqrt, F->count);
    } else {
      F->count = 1;
      F->rec_inv_sqrt = (uint16_t)(~0u >> 16);
    }
    F->last_count = F->count;
    F->drop_next = codel_control_law(now_c, o->fq_interval_c, F->rec_inv_sqrt);
  }
  if (have) *out = pk;
  return have;
}

static void list_pop_front(int* a, int* n) {
  for (int k = 1; k < *n; ++k) a[k - 1] = a[k];
  --*n;
}

/* FqCoDelQueueDisc::DoDequeue (DRR over new, then old flows) */
static int fq_dequeue(bcsim_oracle* o, fqlink* l, fqpkt* out) {
  for (;;) {
    int f = -1;
    while (f < 0 && l->n_new) {
      int c = l->newl[0];
      if (l->f[c].deficit <= 0) {
        l->f[c].deficit += (int32_t)o->fq_quantum;
        l->f[c].status = 2;
        l->oldl[l->n_old++] = c;
        list_pop_front(l->newl, &l->n_new);
      } else {
        f = c;
      }
    }
    while (f < 0 && l->n_old) {
      int c = l->oldl[0];
      if (l->f[c].deficit <= 0) {
        l->f[c].deficit += (int32_t)o->fq_quantum;
        list_pop_front(l->oldl, &l->n_old);
        l->oldl[l->n_old++] = c;
      } else {
        f = c;
      }
    }
    if (f < 0) return 0;
    fqflow* F = &l->f[f];
    if (codel_dequeue(o, l, F, out)) {
      F->deficit -= (int32_t)out->size;
      return 1;
    }
    if (F->status == 1 && l->n_old) { /* (a new flow is at the head of the new list) */
      F->status = 2;
      l->oldl[l->n_old++] = f;
      list_pop_front(l->newl, &l->n_new);
    } else if (F->status == 1) {
      F->status = 0;
      list_pop_front(l->newl, &l->n_new);
    } else {
      F->status = 0;
      list_pop_front(l->oldl, &l->n_old);
    }
  }
}

static void fq_schedule_wake(bcsim_oracle* o, uint32_t edge, int64_t t) {
  oev w;
  memset(&w, 0, sizeof w);
  w.t = t;
  w.ts = -2;
  w.origin = w.target = edge_src(o, edge);
  w.kind = EV_WAKE;
  w.aux = edge;
  int rc = heap_push(&o->heap, &w);
  if (rc) set_err(o, rc);
}

/* frames of the device queue that started transmission by now are no longer waiting */
static void fq_dev_settle(bcsim_oracle* o, fqlink* l) {
  while (l->dn && l->dev[l->dh] <= o->now) {
    l->dh = (l->dh + 1) % l->dcap;
    --l->dn;
  }
}

/* a packet from the disc into the device queue (PointToPointNetDevice::Send) */
static void fq_dev_push(bcsim_oracle* o, uint32_t edge, fqlink* l, const fqpkt* pk) {
  fqmsg* m = &l->msg[pk->msg];
  int big = m->m.big;
  int64_t tx = pk->frame + 1 == o->nfr[big] ? o->tx_last[big] : o->tx_full[big];
  int64_t start = l->dev_end > o->now ? l->dev_end : o->now;
  int64_t end = start + tx;
  fq_log(o, l, 2, pk, start);
  l->dev_end = end;
  fq_dev_settle(o, l);
  if (start > o->now) {
    if (l->dn == l->dcap) { /* grow the ring (capacity fq_devcap at most: the queue stops there) */
      uint32_t nc = l->dcap ? 2 * l->dcap : 4;
      if (nc > o->fq_devcap) nc = o->fq_devcap;
      int64_t* na = (int64_t*)malloc(nc * sizeof(int64_t));
      if (!na) {
        set_err(o, BCSIM_E_NOMEM);
        return;
      }
      for (uint32_t k = 0; k < l->dn; ++k) na[k] = l->dev[(l->dh + k) % l->dcap];
      free(l->dev);
      l->dev = na;
      l->dh = 0;
      l->dcap = nc;
    }
    l->dev[(l->dh + l->dn) % l->dcap] = start;
    ++l->dn;
    if (l->dn == o->fq_devcap) { /* the queue cannot take another packet: stop the disc */
      l->stopped = 1;
      fq_schedule_wake(o, edge, l->dev[l->dh]);
    }
  }
  if (--m->left) return;
  if (!m->lost && !m->echo) { /* the message's last fragment is on its way: delivery */
    oev r;
    memset(&r, 0, sizeof r);
    r.t = end + o->prop[edge];
    r.ts = end - o->tx_last[big]; /* t - prop - last-fragment frame time */
    r.origin = edge_src(o, edge);
    r.sub = m->sub;
    r.target = o->col[edge];
    r.kind = EV_RECV;
    r.aux = edge;
    r.m = m->m;
    int rc = heap_push(&o->heap, &r);
    if (rc) set_err(o, rc);
  }
  fq_free_msg(l, pk->msg);
}

/* QueueDisc::Run: dequeue into the device while it is not stopped */
static void fq_run(bcsim_oracle* o, uint32_t edge, fqlink* l) {
  fqpkt pk;
  while (!l->stopped && fq_dequeue(o, l, &pk)) fq_dev_push(o, edge, l, &pk);
}

/* the device queue wakes the disc (its oldest waiting frame starts now) */
static void fq_wake(bcsim_oracle* o, uint32_t edge) {
  fqlink* l = fq_get(o, edge);
  if (!l) return;
  fq_log(o, l, 4, NULL, l->qpkts);
  fq_dev_settle(o, l);
  l->stopped = 0;
  fq_run(o, edge, l);
}

/* FqCoDelQueueDisc::FqCoDelDrop */
static void fq_overlimit(bcsim_oracle* o, fqlink* l) {
  uint32_t maxb = 0;
  int fat = -1; /* the first class (creation order) with the most bytes; class 0 by default */
  for (int r = 0; r < l->n_created; ++r)
    for (int f = 0; f < 3; ++f)
      if (l->f[f].created == r) {
        if (fat < 0) fat = f;
        if (l->f[f].bytes > maxb) {
          maxb = l->f[f].bytes;
          fat = f;
        }
      }
  if (fat < 0) return;
  uint32_t threshold = maxb >> 1, len = 0, count = 0;
  fqpkt pk;
  do {
    if (!fq_pop(l, &l->f[fat], &pk)) break;
    fq_drop(o, l, &pk);
    len += pk.size;
  } while (++count < o->fq_batch && len < threshold);
}

static int fq_push(bcsim_oracle* o, fqflow* F, const fqpkt* pk) {
  if (F->n == F->cap) {
    uint32_t nc = F->cap ? 2 * F->cap : 4;
    fqpkt* na = (fqpkt*)malloc(nc * sizeof(fqpkt));
    if (!na) return BCSIM_E_NOMEM;
    for (uint32_t i = 0; i < F->n; ++i) na[i] = F->a[(F->head + i) % F->cap];
    free(F->a);
    F->a = na;
    F->head = 0;
    F->cap = nc;
  }
  F->a[(F->head + F->n) % F->cap] = *pk;
  ++F->n;
  F->bytes += pk->size;
  return BCSIM_OK;
}

/* a message (application send or echo) handed to the link at o->now: IPv4 fragments
 * it and hands each fragment to the traffic-control layer (enqueue, then Run) */
static void fq_send(bcsim_oracle* o, uint32_t edge, const omsg* msg, uint32_t sub, int echo) {
  fqlink* l = fq_get(o, edge);
  if (!l) return;
  uint32_t mi = 0;
  while (mi < l->nmsg && l->msg[mi].used) ++mi;
  if (mi == l->capmsg) {
    uint32_t nc = l->capmsg ? 2 * l->capmsg : 2;
    fqmsg* na = (fqmsg*)realloc(l->msg, nc * sizeof(fqmsg));
    if (!na) {
      set_err(o, BCSIM_E_NOMEM);
      return;
    }
    for (uint32_t k = l->capmsg; k < nc; ++k) na[k].used = 0;
    l->msg = na;
    l->capmsg = nc;
  }
  if (mi == l->nmsg) ++l->nmsg;
  fqmsg* m = &l->msg[mi];
  m->m = *msg;
  m->sub = sub;
  m->echo = echo;
  m->lost = 0;
  m->used = 1;
  int big = msg->big;
  uint32_t F = o->nfr[big];
  m->left = F;
  for (uint32_t j = 0; j < F; ++j) {
    int cls = j ? 2 : echo ? 1 : 0;
    int f = (int)fq_class_slot(o, edge, l, cls);
    fqflow* fl = &l->f[f];
    fqpkt pk;
    pk.enq = o->now;
    pk.msg = mi;
    pk.size = j + 1 == F ? o->ip_last[big] : o->ip_full[big];
    pk.frame = j;
    if (fl->created < 0) fl->created = l->n_created++;
    if (fl->status == 0) {
      fl->status = 1;
      fl->deficit = (int32_t)o->fq_quantum;
      l->newl[l->n_new++] = f;
    }
    int rc = fq_push(o, fl, &pk);
    if (rc) {
      set_err(o, rc);
      return;
    }
    fq_log(o, l, 1, &pk, f);
    ++l->qpkts;
    if (l->qpkts > o->fq_limit) fq_overlimit(o, l);
    fq_run(o, edge, l);
    m = &l->msg[mi]; /* (the table is not reallocated meanwhile; kept for clarity) */
  }
}

/* ------------------------------------------------------------------------ */
/* PBFT (pbft/pbft-node.cc) */
enum {
  P_PRE_PREPARE = 1, P_PREPARE = 2, P_COMMIT = 3, P_PREPARE_RES = 5,
  P_COMMIT_RES = 6, P_VIEW_CHANGE = 8
};

static void pbft_start(bcsim_oracle* o, uint32_t i) { /* :97-158 */
  onode* nd = &o->nodes[i];
  o->g_v = 1;
  o->g_n = 0;
  nd->leader = 0;
  nd->block_num = 0;
  o->g_nround = 0;
  sched_timer(o, i, TM_PBFT_BLOCK, o->pbft_period); /* :155 */
}

static int pbft_idx_ok(bcsim_oracle* o, int32_t idx) {
  if (idx < 0) {
    set_err(o, BCSIM_E_ENCODING);
    return 0;
  }
  if ((uint32_t)idx >= o->cfg.pbft_seq_cap) {
    set_err(o, BCSIM_E_INDEX);
    return 0;
  }
  return 1;
}

static void pbft_view_change(bcsim_oracle* o, uint32_t i) { /* :293-303 */
  onode* nd = &o->nodes[i];
  nd->leader = (nd->leader + 1) % (int32_t)o->N;
  o->g_v += 1;
  omsg m = mk(P_VIEW_CHANGE, enc(o, o->g_v), enc(o, nd->leader), 0, 0);
  bcast(o, i, &m);
}

static void pbft_send_block(bcsim_oracle* o, const oev* e, uint32_t i) {
  onode* nd = &o->nodes[i]; /* :371-411 */
  /* generateTX(num): header '1', v, n, n (:79-95) */
  omsg blk = mk(P_PRE_PREPARE, enc(o, o->g_v), enc(o, o->g_n), enc(o, o->g_n), 1);
  if ((int32_t)i == nd->leader) {
    emit(o, e, i, BCSIM_TR_PBFT_BLOCK, o->g_n, o->g_v, 0); /* :387 */
    bcast(o, i, &blk);                                      /* :389-396 */
    o->g_nround++;
    o->g_n++;
    if (o->cfg.pbft_view_change) {
      int32_t r = draw(o, i); /* :401 */
      if (r % 100 == 5) pbft_view_change(o, i);
    }
  }
  nd->block_ev = sched_timer(o, i, TM_PBFT_BLOCK, o->pbft_period); /* :406 */
  if (o->g_nround == (int32_t)o->cfg.pbft_rounds) {
    emit(o, e, i, BCSIM_TR_PBFT_STOP, o->g_nround, 0, 0); /* :408 */
    cancel_timer(o, i, nd->block_ev);
  }
}

static void pbft_recv(bcsim_oracle* o, const oev* e, uint32_t i) {
  onode* nd = &o->nodes[i]; /* HandleRead :166-291 */
  const omsg* m = &e->m;
  int32_t* tv = o->tx_val + (size_t)i * o->cfg.pbft_seq_cap;
  int32_t* tp = o->tx_pv + (size_t)i * o->cfg.pbft_seq_cap;
  int32_t* tc = o->tx_cv + (size_t)i * o->cfg.pbft_seq_cap;
  switch (dec(mchar(m, 0))) {
    case P_PRE_PREPARE: { /* :193-211 */
      omsg r = mk(P_PREPARE, mchar(m, 1), mchar(m, 2), mchar(m, 3), 0);
      int32_t num = dec(mchar(m, 2));
      if (!pbft_idx_ok(o, num)) return;
      tv[num] = dec(mchar(m, 3));
      bcast(o, i, &r);
      break;
    }
    case P_PREPARE: { /* :212-222 */
      omsg r = mk(P_PREPARE_RES, mchar(m, 1), mchar(m, 2), enc(o, 0), 0);
      unicast(o, i, e->aux, &r);
      break;
    }
    case P_PREPARE_RES: { /* :223-240 */
      int32_t idx = dec(mchar(m, 2));
      if (!pbft_idx_ok(o, idx)) return;
      if (dec(mchar(m, 3)) == 0) tp[idx]++;
      if (tp[idx] >= (int32_t)o->N / 2) {
        omsg r = mk(P_COMMIT, mchar(m, 1), mchar(m, 2), 0, 0);
        bcast(o, i, &r);
        tp[idx] = 0;
      }
      break;
    }
    case P_COMMIT: { /* :241-265 */
      int32_t idx = dec(mchar(m, 2));
      if (!pbft_idx_ok(o, idx)) return;
      tc[idx]++;
      if (tc[idx] > (int32_t)o->N / 2) {
        tc[idx] = 0;
        emit(o, e, i, BCSIM_TR_PBFT_COMMIT, o->g_v, nd->block_num, tv[idx]);
        nd->block_num++;
      }
      break;
    }
    case P_VIEW_CHANGE: { /* :271-286, falls through to default */
      int32_t vt = dec(mchar(m, 1));
      int32_t lt = dec(mchar(m, 2));
      o->g_v = vt;
      nd->leader = lt;
      if ((int32_t)i == nd->leader) emit(o, e, i, BCSIM_TR_PBFT_VIEW, o->g_v, lt, 0);
      o->cnt.wrong_msgs++;
      break;
    }
    default:
      o->cnt.wrong_msgs++;
      break;
  }
}

/* ------------------------------------------------------------------------ */
/* Raft (raft/raft-node.cc) */
enum { R_VOTE_REQ = 2, R_VOTE_RES = 3, R_HEARTBEAT = 4, R_HEARTBEAT_RES = 5 };

static int64_t raft_election_timeout(bcsim_oracle* o, uint32_t i) { /* :69-72 */
  int32_t r = draw(o, i);
  return o->raft_elec[r % 150];
}

static void raft_start(bcsim_oracle* o, uint32_t i) { /* :75-115 */
  onode* nd = &o->nodes[i];
  nd->m_value = 0;
  nd->vote_success = 0;
  nd->vote_failed = 0;
  nd->has_voted = 0;
  nd->add_change_value = 0;
  nd->is_leader = 0;
  nd->round = 0;
  nd->blockNum = 0;
  int64_t to = raft_election_timeout(o, i);
  nd->next_election = sched_timer(o, i, TM_RAFT_ELECTION, to); /* :114 */
}

static void raft_send_vote(bcsim_oracle* o, const oev* e, uint32_t i) {
  onode* nd = &o->nodes[i]; /* :391-401 */
  nd->has_voted = 1;
  omsg m = mk(R_VOTE_REQ, enc(o, (int32_t)i), 0, 0, 0);
  bcast(o, i, &m);
  emit(o, e, i, BCSIM_TR_RAFT_ELECTION, 0, 0, 0);
  int64_t to = raft_election_timeout(o, i);
  nd->next_election = sched_timer(o, i, TM_RAFT_ELECTION, to);
}

static void raft_heartbeat(bcsim_oracle* o, const oev* e, uint32_t i) {
  onode* nd = &o->nodes[i]; /* sendHeartBeat :404-429 */
  nd->has_voted = 1;
  if (nd->add_change_value == 1) {
    nd->next_heartbeat = sched_timer(o, i, TM_RAFT_HEARTBEAT, o->raft_hb);
    /* SendTX :340-366; generateTX: '4','1','1',... (:323-336) */
    emit(o, e, i, BCSIM_TR_RAFT_PROPOSAL, nd->round, 0, 0);
    omsg m = mk(R_HEARTBEAT, enc(o, 1), '1', '1', 1);
    bcast(o, i, &m);
    nd->round++;
    if (nd->round == (int32_t)o->cfg.raft_proposal_rounds) nd->add_change_value = 0;
  } else {
    nd->next_heartbeat = sched_timer(o, i, TM_RAFT_HEARTBEAT, o->raft_hb);
    omsg m = mk(R_HEARTBEAT, enc(o, 0), 0, 0, 0);
    bcast(o, i, &m);
  }
}

static void raft_recv(bcsim_oracle* o, const oev* e, uint32_t i) {
  onode* nd = &o->nodes[i]; /* HandleRead :127-276 */
  const omsg* m = &e->m;
  int32_t N = (int32_t)o->N;
  switch (dec(mchar(m, 0))) {
    case R_VOTE_REQ: { /* :154-168 */
      int32_t st;
      if (nd->has_voted == 0) {
        st = 0;
        nd->has_voted = 1;
      } else {
        st = 1;
      }
      omsg r = mk(R_VOTE_RES, enc(o, st), 0, 0, 0);
      unicast(o, i, e->aux, &r);
      break;
    }
    case R_HEARTBEAT: { /* :170-194 */
      int32_t type = dec(mchar(m, 1));
      int32_t d1;
      if (type == 0) {
        d1 = enc(o, 0);
        cancel_timer(o, i, nd->next_election);
      } else {
        d1 = enc(o, 1);
        nd->m_value = dec(mchar(m, 2));
        cancel_timer(o, i, nd->next_election);
      }
      omsg r = mk(R_HEARTBEAT_RES, d1, enc(o, 0), 0, 0);
      unicast(o, i, e->aux, &r);
      break;
    }
    case R_VOTE_RES: { /* :196-232 */
      if (!nd->is_leader) {
        int32_t st = dec(mchar(m, 1));
        if (st == 0)
          nd->vote_success += 1;
        else
          nd->vote_failed += 1;
        if (nd->vote_success + 1 > N / 2) {
          nd->vote_success = 0;
          nd->vote_failed = 0;
          emit(o, e, i, BCSIM_TR_RAFT_LEADER, 0, 0, 0);
          cancel_timer(o, i, nd->next_election);
          sched_timer(o, i, TM_RAFT_PROPOSAL, o->cfg.raft_proposal_delay_ns);
          raft_heartbeat(o, e, i);
          nd->is_leader = 1;
        } else if (nd->vote_failed >= N / 2) {
          nd->vote_success = 0;
          nd->vote_failed = 0;
          nd->has_voted = 0;
        }
      }
      break;
    }
    case R_HEARTBEAT_RES: { /* :233-266 */
      int32_t type = dec(mchar(m, 1));
      if (type == 1) {
        if (dec(mchar(m, 2)) == 0)
          nd->vote_success += 1;
        else
          nd->vote_failed += 1;
        if (nd->vote_success + nd->vote_failed == N - 1) {
          if (nd->vote_success + 1 > N / 2) {
            nd->vote_success = 0;
            nd->vote_failed = 0;
            emit(o, e, i, BCSIM_TR_RAFT_BLOCK, nd->blockNum, 0, 0);
            nd->blockNum += 1;
            if (nd->blockNum >= (int32_t)o->cfg.raft_blocks) {
              emit(o, e, i, BCSIM_TR_RAFT_DONE, nd->blockNum, 0, 0);
              cancel_timer(o, i, nd->next_heartbeat);
            }
          } else {
            nd->vote_success = 0;
            nd->vote_failed = 0;
          }
        }
      }
      break;
    }
    default:
      o->cnt.wrong_msgs++;
      break;
  }
}

/* ------------------------------------------------------------------------ */
/* Paxos (paxos/paxos-node.cc) */
enum {
  X_REQ_TICKET = 0, X_REQ_PROPOSE = 1, X_REQ_COMMIT = 2, X_RES_TICKET = 3,
  X_RES_PROPOSE = 4, X_RES_COMMIT = 5, X_CLIENT_PROPOSE = 6
};

/* acceptor state of node i for decree d: t_max, command, t_store, isCommit */
static int32_t* px_of(bcsim_oracle* o, uint32_t i, int32_t d) {
  if (d < 0 || (uint32_t)d >= o->K) {
    set_err(o, BCSIM_E_INDEX);
    d = 0;
  }
  return &o->px[((size_t)i * o->K + (uint32_t)d) * 4];
}

/* every Paxos message carries its decree in data[3] (f[2]): outside the
 * reference's 3-byte packet, so 0 for the single decree */
static void paxos_require_ticket(bcsim_oracle* o, const oev* e, uint32_t i) {
  onode* nd = &o->nodes[i]; /* :510-522 */
  nd->ticket += 1;
  omsg m = mk(X_REQ_TICKET, enc(o, nd->ticket), 0, nd->decree, 0);
  bcast_paxos(o, i, &m);
  emit(o, e, i, BCSIM_TR_PAXOS_TICKET, nd->ticket, nd->decree, 0);
}

static void paxos_start(bcsim_oracle* o, uint32_t i) { /* :58-139 */
  onode* nd = &o->nodes[i];
  for (uint32_t d = 0; d < o->K; ++d) {
    int32_t* a = px_of(o, i, (int32_t)d);
    a[0] = 0;   /* t_max */
    a[1] = 'e'; /* command */
    a[2] = 0;   /* t_store */
    a[3] = 0;   /* isCommit */
  }
  nd->ticket = 0;
  nd->decree = 0;
  nd->proposal = as_char(o, (int32_t)i + '0');
  nd->vote_success = 0;
  nd->vote_failed = 0;
  nd->round = 0;
  if (i < o->cfg.paxos_proposers) sched_timer(o, i, TM_PAXOS_TICKET, 0);
}

static void paxos_recv(bcsim_oracle* o, const oev* e, uint32_t i) {
  onode* nd = &o->nodes[i]; /* HandleRead :148-372 */
  const omsg* m = &e->m;
  int32_t N = (int32_t)o->N;
  switch (dec(mchar(m, 0))) {
    case X_REQ_TICKET: { /* :177-198 */
      int32_t t = dec(mchar(m, 1));
      int32_t* a = px_of(o, i, m->f[2]);
      omsg r;
      if (t > a[0]) {
        a[0] = t;
        r = mk(X_RES_TICKET, enc(o, 0), a[1], m->f[2], 0);
      } else {
        r = mk(X_RES_TICKET, enc(o, 1), 0, m->f[2], 0);
      }
      unicast(o, i, e->aux, &r);
      break;
    }
    case X_REQ_PROPOSE: { /* :199-221 */
      int32_t t = dec(mchar(m, 1));
      int32_t* a = px_of(o, i, m->f[2]);
      int32_t st;
      if (t == a[0]) {
        a[1] = mchar(m, 2);
        a[2] = t;
        st = 0;
      } else {
        st = 1;
      }
      omsg r = mk(X_RES_PROPOSE, enc(o, st), 0, m->f[2], 0);
      unicast(o, i, e->aux, &r);
      break;
    }
    case X_REQ_COMMIT: { /* :222-247 */
      int32_t t = dec(mchar(m, 1));
      int32_t c = mchar(m, 2);
      int32_t* a = px_of(o, i, m->f[2]);
      int32_t st;
      if (t == a[2] && c == a[1]) {
        a[3] = 1;
        st = 0;
      } else {
        st = 1;
      }
      omsg r = mk(X_RES_COMMIT, enc(o, st), 0, m->f[2], 0);
      unicast(o, i, e->aux, &r);
      break;
    }
    case X_RES_TICKET:
    case X_RES_PROPOSE:
    case X_RES_COMMIT: { /* :248-353 */
      int32_t ty = dec(mchar(m, 0));
      int32_t st = dec(mchar(m, 1));
      if (m->f[2] != nd->decree) break; /* a response of a finished decree: not counted */
      if (st == 0)
        nd->vote_success += 1;
      else
        nd->vote_failed += 1;
      if (nd->vote_success + nd->vote_failed == N - 2) {
        if (nd->vote_success >= N / 2) {
          nd->vote_success = 0;
          nd->vote_failed = 0;
          if (ty == X_RES_TICKET) {
            if (mchar(m, 2) != 'e') nd->proposal = mchar(m, 2);
            omsg r = mk(X_REQ_PROPOSE, enc(o, nd->ticket), nd->proposal, nd->decree, 0);
            bcast_paxos(o, i, &r);
          } else if (ty == X_RES_PROPOSE) {
            omsg r = mk(X_REQ_COMMIT, enc(o, nd->ticket), nd->proposal, nd->decree, 0);
            bcast_paxos(o, i, &r);
          } else {
            emit(o, e, i, BCSIM_TR_PAXOS_COMMIT, nd->ticket, nd->decree, 0);
            if ((uint32_t)nd->decree + 1 < o->K) { /* next decree: fresh ticket and proposal */
              nd->decree += 1;
              nd->ticket = 0;
              nd->proposal = as_char(o, (int32_t)i + '0');
              paxos_require_ticket(o, e, i);
            }
          }
        } else {
          nd->vote_success = 0;
          nd->vote_failed = 0;
          paxos_require_ticket(o, e, i);
        }
      }
      break;
    }
    case X_CLIENT_PROPOSE: /* :357-361 */
      paxos_require_ticket(o, e, i);
      break;
    default:
      o->cnt.wrong_msgs++;
      break;
  }
}

/* ------------------------------------------------------------------------ */
/* GOSSIP (BCSIM_GOSSIP, build extension for BASELINE configs[4]; see
 * include/bcsim.h).  Message GS_BLOCK: f[0] = sequence, f[1] = hop count
 * (raw integers, no intToChar), block-sized payload. */
enum { GS_BLOCK = 1 };

static int gossip_seq_ok(bcsim_oracle* o, int32_t seq) {
  if (seq < 0 || (uint32_t)seq >= o->cfg.pbft_seq_cap) {
    set_err(o, BCSIM_E_INDEX);
    return 0;
  }
  return 1;
}

static void gossip_start(bcsim_oracle* o, uint32_t i) {
  o->nodes[i].round = 0;
  if (i == 0) sched_timer(o, i, TM_GOSSIP_BLOCK, o->pbft_period); /* like :155 */
}

/* origin tick: SendBlock shape (pbft-node.cc:371-411) without globals */
static void gossip_tick(bcsim_oracle* o, const oev* e, uint32_t i) {
  onode* nd = &o->nodes[i];
  int32_t seq = nd->round++;
  if (!gossip_seq_ok(o, seq)) return;
  o->gseen[(size_t)i * o->cfg.pbft_seq_cap + seq] = 1;
  emit(o, e, i, BCSIM_TR_GOSSIP_BLOCK, seq, 0, 0);
  omsg m = mk(GS_BLOCK, seq, 0, 0, 1);
  bcast(o, i, &m);
  if (nd->round < (int32_t)o->cfg.pbft_rounds) sched_timer(o, i, TM_GOSSIP_BLOCK, o->pbft_period);
}

static void gossip_recv(bcsim_oracle* o, const oev* e, uint32_t i) {
  const omsg* m = &e->m;
  if (m->type != GS_BLOCK) {
    o->cnt.wrong_msgs++;
    return;
  }
  int32_t seq = m->f[0];
  if (!gossip_seq_ok(o, seq)) return;
  uint8_t* seen = &o->gseen[(size_t)i * o->cfg.pbft_seq_cap + seq];
  if (*seen) return;
  *seen = 1;
  emit(o, e, i, BCSIM_TR_GOSSIP_DELIVER, seq, m->f[1] + 1, (int32_t)e->origin);
  omsg r = mk(GS_BLOCK, seq, m->f[1] + 1, 0, 1);
  bcast(o, i, &r);
}

/* ------------------------------------------------------------------------ */
/* driver */
static void exec_event(bcsim_oracle* o, const oev* e) {
  uint32_t i = e->target;
  onode* nd = &o->nodes[i];
  switch (e->kind) {
    case EV_START:
      o->cnt.events++;
      if (o->cfg.protocol == BCSIM_PBFT)
        pbft_start(o, i);
      else if (o->cfg.protocol == BCSIM_RAFT)
        raft_start(o, i);
      else if (o->cfg.protocol == BCSIM_GOSSIP)
        gossip_start(o, i);
      else
        paxos_start(o, i);
      break;
    case EV_STOP: /* Application::StopApplication */
      o->cnt.events++;
      if (o->cfg.protocol == BCSIM_RAFT && nd->is_leader == 1)
        emit(o, e, i, BCSIM_TR_RAFT_STOP, nd->blockNum, nd->round, 0);
      break;
    case EV_TIMER:
      if (take_cancelled(nd, e->sub)) break;
      o->cnt.events++;
      switch (e->aux) {
        case TM_PBFT_BLOCK:
          pbft_send_block(o, e, i);
          break;
        case TM_RAFT_ELECTION:
          raft_send_vote(o, e, i);
          break;
        case TM_RAFT_HEARTBEAT:
          raft_heartbeat(o, e, i);
          break;
        case TM_RAFT_PROPOSAL: /* setProposal :432-435 */
          nd->add_change_value = 1;
          break;
        case TM_PAXOS_TICKET:
          paxos_require_ticket(o, e, i);
          break;
        case TM_GOSSIP_BLOCK:
          gossip_tick(o, e, i);
          break;
      }
      break;
    case EV_SEND: { /* SendPacket :323-325 -> socket->Send -> p2p device */
      o->cnt.sends++;
      if (o->cfg.queue_model == BCSIM_QUEUE_FQCODEL) fq_bind(o, i, e->aux);
      if (e->aux == UINT32_MAX) {
        o->cnt.dropped++;
        break;
      }
      if (o->cfg.queue_model == BCSIM_QUEUE_FQCODEL) { /* delivered when its last fragment leaves the disc */
        fq_send(o, e->aux, &e->m, e->sub, 0);
        break;
      }
      oev r;
      memset(&r, 0, sizeof r);
      int64_t tsl = 0;
      r.t = link_xmit(o, e->aux, e->m.big, &tsl);
      if (r.t < 0) { /* fragment dropped by a full link queue: never delivered */
        o->cnt.msgs_lost++;
        break;
      }
      r.ts = tsl;
      r.origin = i;
      r.sub = e->sub;
      r.target = o->col[e->aux];
      r.kind = EV_RECV;
      r.aux = e->aux;
      r.m = e->m;
      int rc = heap_push(&o->heap, &r);
      if (rc) set_err(o, rc);
      break;
    }
    case EV_RECV: {
      o->cnt.events++;
      int ty = e->m.type;
      if (ty >= 0 && ty < BCSIM_MSG_TYPES) o->cnt.delivered[ty]++;
      o->cnt.delivered_total++;
      if (o->cfg.echo) { /* socket->SendTo(packet, 0, from) :175 */
        int64_t tsl;
        if (o->cfg.queue_model == BCSIM_QUEUE_FQCODEL)
          fq_send(o, o->rev[e->aux], &e->m, 0, 1);
        else
          (void)link_xmit(o, o->rev[e->aux], e->m.big, &tsl);
        o->cnt.echoes++;
      }
      if (o->cfg.protocol == BCSIM_PBFT)
        pbft_recv(o, e, i);
      else if (o->cfg.protocol == BCSIM_RAFT)
        raft_recv(o, e, i);
      else if (o->cfg.protocol == BCSIM_GOSSIP)
        gossip_recv(o, e, i);
      else
        paxos_recv(o, e, i);
      break;
    }
    case EV_WAKE: /* link-internal: not a protocol event */
      fq_wake(o, e->aux);
      break;
  }
}

static int build_full_mesh(bcsim_oracle* o) {
  uint32_t N = o->N;
  uint64_t E = (uint64_t)N * (N - 1);
  uint32_t* row = (uint32_t*)malloc((N + 1) * sizeof(uint32_t));
  uint32_t* col = (uint32_t*)malloc((E ? E : 1) * sizeof(uint32_t));
  if (!row || !col) {
    free(row);
    free(col);
    return BCSIM_E_NOMEM;
  }
  uint64_t k = 0;
  for (uint32_t i = 0; i < N; ++i) { /* blockchain-simulator.cc:34-51 order */
    row[i] = (uint32_t)k;
    for (uint32_t j = 0; j < N; ++j)
      if (j != i) col[k++] = j;
  }
  row[N] = (uint32_t)k;
  int rc = bcsim_oracle_set_topology_csr(o, N, row, col, NULL);
  free(row);
  free(col);
  return rc;
}

typedef struct {
  uint32_t a, b, e;
} etrip;
static int etrip_cmp(const void* x, const void* y) {
  const etrip* p = (const etrip*)x;
  const etrip* q = (const etrip*)y;
  if (p->a != q->a) return p->a < q->a ? -1 : 1;
  if (p->b != q->b) return p->b < q->b ? -1 : 1;
  return 0;
}

static void free_queues(bcsim_oracle* o) {
  if (o->q && o->row)
    for (uint32_t e = 0; e < o->row[o->N]; ++e) free(o->q[e].a);
  free(o->q);
  o->q = NULL;
}

int bcsim_oracle_set_topology_csr(bcsim_oracle* o, uint32_t n,
                                  const uint32_t* row_ptr,
                                  const uint32_t* col_idx,
                                  const int64_t* prop_ns) {
  if (!o || n != o->N || !row_ptr || !col_idx) return BCSIM_E_INVAL;
  if (o->started) return BCSIM_E_STATE;
  uint32_t E = row_ptr[n];
  free_queues(o);
  free_fq(o);
  free(o->row);
  free(o->col);
  free(o->rev);
  free(o->prop);
  free(o->busy);
  o->row = (uint32_t*)malloc((n + 1) * sizeof(uint32_t));
  o->col = (uint32_t*)malloc((E ? E : 1) * sizeof(uint32_t));
  o->rev = (uint32_t*)malloc((E ? E : 1) * sizeof(uint32_t));
  o->prop = (int64_t*)malloc((E ? E : 1) * sizeof(int64_t));
  o->busy = (int64_t*)calloc(E ? E : 1, sizeof(int64_t));
  o->q = (oqueue*)calloc(E ? E : 1, sizeof(oqueue));
  if (!o->row || !o->col || !o->rev || !o->prop || !o->busy || !o->q) return BCSIM_E_NOMEM;
  memcpy(o->row, row_ptr, (n + 1) * sizeof(uint32_t));
  memcpy(o->col, col_idx, E * sizeof(uint32_t));
  for (uint32_t e = 0; e < E; ++e)
    o->prop[e] = prop_ns ? prop_ns[e] : o->cfg.link_delay_ns;
  /* reverse edge map: (s,d) -> edge of (d,s) */
  etrip* t = (etrip*)malloc((E ? E : 1) * sizeof(etrip));
  if (!t) return BCSIM_E_NOMEM;
  for (uint32_t s = 0; s < n; ++s)
    for (uint32_t e = row_ptr[s]; e < row_ptr[s + 1]; ++e) {
      if (col_idx[e] >= n) {
        free(t);
        return BCSIM_E_INVAL;
      }
      t[e].a = s;
      t[e].b = col_idx[e];
      t[e].e = e;
    }
  qsort(t, E, sizeof(etrip), etrip_cmp);
  for (uint32_t s = 0; s < n; ++s)
    for (uint32_t e = row_ptr[s]; e < row_ptr[s + 1]; ++e) {
      etrip key = {col_idx[e], s, 0};
      etrip* hit = (etrip*)bsearch(&key, t, E, sizeof(etrip), etrip_cmp);
      if (!hit) {
        free(t);
        return BCSIM_E_INVAL; /* asymmetric graph */
      }
      o->rev[e] = hit->e;
    }
  free(t);
  if (o->cfg.queue_model == BCSIM_QUEUE_FQCODEL) {
    o->fq = (fqlink**)calloc(E ? E : 1, sizeof(fqlink*));
    o->fqlnk = (uint32_t*)calloc(E ? E : 1, sizeof(uint32_t));
    o->fqport = (uint32_t*)calloc(E ? E : 1, sizeof(uint32_t));
    o->fqnport = (uint32_t*)calloc(o->N, sizeof(uint32_t));
    o->fqphant = (uint8_t*)calloc(o->N, 1);
    if (!o->fq || !o->fqlnk || !o->fqport || !o->fqnport || !o->fqphant) return BCSIM_E_NOMEM;
    fq_build_links(o);
  }
  o->topo_set = 1;
  return BCSIM_OK;
}

int bcsim_oracle_create(const bcsim_config* cfg, bcsim_oracle** out) {
  if (!cfg || !out) return BCSIM_E_INVAL;
  if (cfg->n_nodes < 2 || cfg->protocol > BCSIM_GOSSIP || cfg->link_rate_bps == 0 ||
      cfg->queue_model > BCSIM_QUEUE_FQCODEL)
    return BCSIM_E_INVAL;
  bcsim_oracle* o = (bcsim_oracle*)calloc(1, sizeof(bcsim_oracle));
  if (!o) return BCSIM_E_NOMEM;
  o->cfg = *cfg;
  if (o->cfg.n_replicas == 0) o->cfg.n_replicas = 1;
  if (o->cfg.mtu == 0) o->cfg.mtu = 1500;
  if (o->cfg.pbft_seq_cap == 0) o->cfg.pbft_seq_cap = 1000;
  o->N = cfg->n_nodes;
  o->R = o->cfg.n_replicas;
  int mode = (int)o->cfg.time_round;
  /* message sizes */
  if (o->cfg.protocol == BCSIM_PBFT) {
    o->small_bytes = 4; /* Create<Packet>(data, 4) pbft-node.cc:332,354 */
    uint32_t bb = o->cfg.pbft_block_bytes;
    if (bb == 0) { /* num = tx_speed / (1000 / (timeout*1000)) :377 */
      float tmo = o->cfg.pbft_timeout_s;
      int num = (int)(1000 / (1000 / (tmo * 1000)));
      bb = (uint32_t)(1000 * num);
    }
    o->big_bytes = bb;
  } else if (o->cfg.protocol == BCSIM_RAFT) {
    o->small_bytes = 3;
    uint32_t pb = o->cfg.raft_proposal_bytes;
    if (pb == 0) { /* raft-node.cc:409, tx_size 200, tx_speed 2000 */
      float hb = o->cfg.raft_heartbeat_s;
      int num = (int)(2000 / (1000 / (hb * 1000)));
      pb = (uint32_t)(200 * num);
    }
    o->big_bytes = pb;
  } else if (o->cfg.protocol == BCSIM_GOSSIP) { /* every message is a block */
    uint32_t bb = o->cfg.pbft_block_bytes ? o->cfg.pbft_block_bytes : 50000;
    o->small_bytes = bb;
    o->big_bytes = bb;
  } else {
    o->small_bytes = 3;
    o->big_bytes = 3;
  }
  oracle_msg_tx(o->small_bytes, o->cfg.mtu, o->cfg.link_rate_bps, mode,
                &o->tx_tot[0], &o->tx_last[0], &o->nfr[0], NULL);
  oracle_msg_tx(o->big_bytes, o->cfg.mtu, o->cfg.link_rate_bps, mode,
                &o->tx_tot[1], &o->tx_last[1], &o->nfr[1], NULL);
  for (int k = 0; k < 2; ++k) /* full fragment frame: (mtu - 20) & ~7 IP payload + 22 */
    o->tx_full[k] = o->nfr[k] > 1 ? (o->tx_tot[k] - o->tx_last[k]) / (o->nfr[k] - 1) : o->tx_tot[k];
  { /* IPv4 packet bytes per fragment (QueueDiscItem::GetSize) */
    uint32_t frag = (o->cfg.mtu - 20) & ~7u, bb[2] = {o->small_bytes, o->big_bytes};
    for (int k = 0; k < 2; ++k) {
      o->ip_full[k] = frag + 20;
      o->ip_last[k] = bb[k] + 8 - frag * (o->nfr[k] - 1) + 20;
    }
  }
  if (o->cfg.queue_model == BCSIM_QUEUE_FQCODEL) { /* ns-3 attribute defaults for 0 */
    o->fq_limit = o->cfg.fq_limit_pkts ? o->cfg.fq_limit_pkts : 10240;
    o->fq_flows = o->cfg.fq_flows ? o->cfg.fq_flows : 1024;
    o->fq_quantum = o->cfg.fq_quantum ? o->cfg.fq_quantum : o->cfg.mtu;
    o->fq_batch = o->cfg.fq_drop_batch ? o->cfg.fq_drop_batch : 64;
    o->fq_min_bytes = o->cfg.fq_min_bytes ? o->cfg.fq_min_bytes : 1500;
    o->fq_target_c = (uint32_t)((uint64_t)(o->cfg.fq_target_ns > 0 ? o->cfg.fq_target_ns : 5000000) >> 10);
    o->fq_interval_c = (uint32_t)((uint64_t)(o->cfg.fq_interval_ns > 0 ? o->cfg.fq_interval_ns : 100000000) >> 10);
    o->fq_devcap = o->cfg.queue_dev_pkts;
    o->flog_t0 = getenv("BCSIM_FQLOG_T0") ? atoll(getenv("BCSIM_FQLOG_T0")) : 0;
    o->flog_t1 = getenv("BCSIM_FQLOG_T1") ? atoll(getenv("BCSIM_FQLOG_T1")) : INT64_MAX;
    o->flog_on = getenv("ORACLE_FQLOG") != NULL;
    if (o->fq_devcap == 0) {
      bcsim_oracle_destroy(o);
      return BCSIM_E_INVAL;
    }
  }
  o->pbft_period = fsec_ns(o->cfg.pbft_timeout_s, mode);
  o->raft_hb = fsec_ns(o->cfg.raft_heartbeat_s, mode);
  for (int k = 0; k < 3; ++k) {
    o->pbft_delay[k] = fsec_ns((float)(((k)*1.0 + 3) / 1000), mode);
    o->raft_delay[k] = fsec_ns((float)((k)*1.0 / 1000), mode);
  }
  for (int k = 0; k < 150; ++k)
    o->raft_elec[k] = fsec_ns((float)(((k) + 150) * 1.0 / 1000), mode);
  for (int k = 0; k < 50; ++k) o->paxos_delay[k] = fsec_ns((float)((k)*1.0 / 1000), mode);
  o->nodes = (onode*)calloc(o->N, sizeof(onode));
  if (!o->nodes) {
    bcsim_oracle_destroy(o);
    return BCSIM_E_NOMEM;
  }
  if (o->cfg.protocol == BCSIM_PBFT) {
    size_t sz = (size_t)o->N * o->cfg.pbft_seq_cap;
    o->tx_val = (int32_t*)calloc(sz, sizeof(int32_t));
    o->tx_pv = (int32_t*)calloc(sz, sizeof(int32_t));
    o->tx_cv = (int32_t*)calloc(sz, sizeof(int32_t));
    if (!o->tx_val || !o->tx_pv || !o->tx_cv) {
      bcsim_oracle_destroy(o);
      return BCSIM_E_NOMEM;
    }
  }
  o->K = o->cfg.paxos_decrees ? o->cfg.paxos_decrees : 1;
  o->px = (int32_t*)calloc((size_t)o->N * (o->cfg.protocol == BCSIM_PAXOS ? o->K : 1) * 4, sizeof(int32_t));
  if (!o->px) {
    bcsim_oracle_destroy(o);
    return BCSIM_E_NOMEM;
  }
  if (o->cfg.protocol == BCSIM_GOSSIP) {
    o->gseen = (uint8_t*)calloc((size_t)o->N * o->cfg.pbft_seq_cap, 1);
    if (!o->gseen) {
      bcsim_oracle_destroy(o);
      return BCSIM_E_NOMEM;
    }
  }
  o->rep_now = (int64_t*)calloc(o->R, sizeof(int64_t));
  /* the full mesh is built at the first run unless a topology was set */
  *out = o;
  return BCSIM_OK;
}

static void reset_replica(bcsim_oracle* o, uint32_t rep) {
  o->cur_rep = rep;
  for (uint32_t i = 0; i < o->N; ++i) {
    free(o->nodes[i].cancelled);
    memset(&o->nodes[i], 0, sizeof(onode));
    o->nodes[i].sub = 2; /* 0 = START, 1 = STOP */
  }
  if (o->tx_val) {
    size_t sz = (size_t)o->N * o->cfg.pbft_seq_cap * sizeof(int32_t);
    memset(o->tx_val, 0, sz);
    memset(o->tx_pv, 0, sz);
    memset(o->tx_cv, 0, sz);
  }
  if (o->gseen) memset(o->gseen, 0, (size_t)o->N * o->cfg.pbft_seq_cap);
  memset(o->busy, 0, (size_t)o->row[o->N] * sizeof(int64_t));
  for (uint32_t e = 0; e < o->row[o->N]; ++e) {
    o->q[e].head = 0;
    o->q[e].n = 0;
    o->q[e].frames = 0;
  }
  if (o->fq) fq_reset(o);
  o->heap.n = 0;
  glibc_seed(&o->grng, (uint32_t)(o->cfg.seed + rep));
  o->g_v = 1;
  o->g_n = 0;
  o->g_nround = 0;
  /* ApplicationContainer Start(0) / Stop(stop_ns), scheduled at init in
   * node order (blockchain-simulator.cc:54-55) */
  for (uint32_t i = 0; i < o->N; ++i) {
    oev e;
    memset(&e, 0, sizeof e);
    e.t = 0;
    e.ts = -1;
    e.origin = i;
    e.sub = 0;
    e.target = i;
    e.kind = EV_START;
    heap_push(&o->heap, &e);
    if (o->cfg.stop_ns >= 0) {
      e.t = o->cfg.stop_ns;
      e.sub = 1;
      e.kind = EV_STOP;
      heap_push(&o->heap, &e);
    }
  }
}

/* Replicas are independent; the oracle runs them one after another.  For
 * R > 1 only t_until = INT64_MAX (run to the end) is supported. */
int bcsim_oracle_run(bcsim_oracle* o, int64_t t_until_ns) {
  if (!o) return BCSIM_E_INVAL;
  if (o->err) return o->err;
  if (o->R > 1 && t_until_ns != INT64_MAX) return BCSIM_E_UNSUPPORTED;
  int64_t lim = t_until_ns;
  if (o->cfg.t_end_ns > 0 && o->cfg.t_end_ns < lim) lim = o->cfg.t_end_ns;
  if (!o->started) {
    if (!o->topo_set) {
      int rc = (uint64_t)o->N * (o->N - 1) >= 0xFFFFFFFFull ? BCSIM_E_UNSUPPORTED : build_full_mesh(o);
      if (rc) {
        set_err(o, rc);
        return rc;
      }
    }
    o->started = 1;
    reset_replica(o, 0);
  }
  for (;;) {
    while (o->heap.n > 0 && o->heap.a[0].t < lim) {
      if (o->cfg.max_events && o->cnt.events >= o->cfg.max_events) {
        set_err(o, BCSIM_E_OVERFLOW);
        return o->err;
      }
      oev e;
      heap_pop(&o->heap, &e);
      o->now = e.t;
      const uint64_t ev0 = o->cnt.events;
      exec_event(o, &e);
      /* t_last: latest protocol event (START/STOP/timer/delivery), sends excluded */
      if (o->cnt.events != ev0 && e.t > o->cnt.t_last_ns) o->cnt.t_last_ns = e.t;
      if (o->err) return o->err;
    }
    if (o->R > 1 && o->cur_rep + 1 < o->R) {
      reset_replica(o, o->cur_rep + 1);
      continue;
    }
    break;
  }
  o->now = lim;
  if (getenv("ORACLE_FQLOG")) { /* debug: the FQCODEL link events so far */
    FILE* f = fopen(getenv("ORACLE_FQLOG"), "wb");
    if (f) {
      fwrite(o->flog, 32, o->nflog, f);
      fclose(f);
    }
  }
  return BCSIM_OK;
}

static int trace_cmp(const void* x, const void* y) {
  const bcsim_trace_rec* p = (const bcsim_trace_rec*)x;
  const bcsim_trace_rec* q = (const bcsim_trace_rec*)y;
#define C(f)                                 \
  if (p->f != q->f) return p->f < q->f ? -1 : 1;
  C(replica) C(t_ns) C(key_ts) C(key_origin) C(key_sub) C(node) C(kind)
#undef C
  return 0;
}

int bcsim_oracle_read_trace(bcsim_oracle* o, bcsim_trace_rec* buf, uint64_t cap,
                            uint64_t* n_out) {
  if (!o || !n_out) return BCSIM_E_INVAL;
  /* emission order within an event is ascending kind,
   * so a full sort is canonical */
  qsort(o->tr, o->ntr, sizeof(bcsim_trace_rec), trace_cmp);
  *n_out = o->ntr;
  if (buf) {
    uint64_t k = o->ntr < cap ? o->ntr : cap;
    memcpy(buf, o->tr, k * sizeof(bcsim_trace_rec));
  }
  return BCSIM_OK;
}

int bcsim_oracle_read_counters(bcsim_oracle* o, bcsim_counters* out) {
  if (!o || !out) return BCSIM_E_INVAL;
  *out = o->cnt;
  out->trace_records = o->ntr;
  return BCSIM_OK;
}

int bcsim_oracle_read_status(bcsim_oracle* o, bcsim_status* out) {
  if (!o || !out) return BCSIM_E_INVAL;
  memset(out, 0, sizeof *out);
  out->now_ns = o->now;
  out->next_ns = o->heap.n ? o->heap.a[0].t : INT64_MAX;
  out->quiescent = o->heap.n == 0;
  out->error = o->err;
  return BCSIM_OK;
}

/* test hook: the client port of every edge's socket after a run (0 = never sent), CSR order */
uint64_t oracle_fq_ports(const bcsim_oracle* o, uint32_t* out, uint64_t cap) {
  if (!o || !o->fqport) return 0;
  uint64_t E = o->row[o->N];
  for (uint64_t e = 0; e < E && e < cap; ++e) out[e] = o->fqport[e];
  return E;
}

int bcsim_oracle_destroy(bcsim_oracle* o) {
  if (!o) return BCSIM_OK;
  if (o->nodes)
    for (uint32_t i = 0; i < o->N; ++i) free(o->nodes[i].cancelled);
  free(o->nodes);
  free(o->tx_val);
  free(o->tx_pv);
  free(o->tx_cv);
  free(o->gseen);
  free(o->px);
  free_queues(o);
  free_fq(o);
  free(o->row);
  free(o->col);
  free(o->rev);
  free(o->prop);
  free(o->busy);
  free(o->heap.a);
  free(o->tr);
  free(o->flog);
  free(o->rep_now);
  free(o);
  return BCSIM_OK;
}
