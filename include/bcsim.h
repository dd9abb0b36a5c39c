/*
 * bcsim.h — C ABI of the MI355X consensus-propagation engine.
 *
 * Drop-in boundary for the hot path of vvvictorlee/blockchain-simulator:
 * the ns-3 per-packet event loop (Simulator::Run, blockchain-simulator.cc:57)
 * driving PbftNode / RaftNode / PaxosNode over the N-node point-to-point full
 * mesh built in blockchain-simulator.cc:12-59 and installed by
 * NetworkHelper (network-helper/network-helper.{h,cc}).
 *
 * Every entry point is plain C: fixed-width integers, plain pointers and
 * sizes, no C++ or torch types.  The reference interface each one replaces is
 * cited next to it.  Errors are negative return codes; nothing throws across
 * this boundary (the reference checks no error at all: pbft-node.cc:126,138,324).
 *
 * Semantics (shared with the CPU oracle under oracle/):
 *   - integer-nanosecond time, float seconds converted as ns-3 Seconds(double)
 *     does (exact product, then round or truncate: time_round);
 *   - per directed link: FIFO, serialization = wire bytes * 8 / rate
 *     (UDP 8 B + IPv4 20 B + PPP 2 B, IPv4 fragmentation at the MTU),
 *     propagation delay; every delivered packet is echoed on the reverse link;
 *   - events ordered by the canonical key (t, t_sched, origin, sub, target).
 */
#ifndef BCSIM_H
#define BCSIM_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCSIM_ABI_VERSION 2u

/* ---- enums ---------------------------------------------------------------- */
/* protocol: replaces the compile-time edit of network-helper.cc:11,17,28 */
enum { BCSIM_PBFT = 0, BCSIM_RAFT = 1, BCSIM_PAXOS = 2,
       /* build extension for BASELINE configs[4] (the reference has no gossip):
        * PBFT-style block flooding over an arbitrary CSR graph.  Node 0 (the
        * initial PBFT leader, pbft-node.cc:103) ticks every pbft_timeout_s
        * like SendBlock (pbft-node.cc:371-411) for pbft_rounds blocks and
        * broadcasts each block (pbft-node.cc:349-368); every node relays a
        * block to all its peers the first time it receives it. */
       BCSIM_GOSSIP = 3 };
/* app-level send delay model: getRandomDelay() pbft-node.cc:66-69,
 * raft-node.cc:63-66, paxos-node.cc:397-400 */
enum { BCSIM_DELAY_FIXED = 0, BCSIM_DELAY_RANDOM = 1 };
/* rand() source: GLIBC = the reference's global TYPE_3 stream (srand(seed),
 * default seed 1), consumed in canonical global event order; COUNTER = a
 * per-(replica, node, draw) splitmix64 stream (order independent). */
enum { BCSIM_RNG_GLIBC = 0, BCSIM_RNG_COUNTER = 1 };
/* float seconds -> int64 ns: ns-3 Time(int64x64_t) Round() vs GetHigh() */
enum { BCSIM_TIME_ROUND = 0, BCSIM_TIME_TRUNC = 1 };
/* wire field encoding: COMPAT = intToChar/charToInt through signed char
 * (pbft-node.cc:57-63), EXTENDED = same +48 offset without the 8-bit wrap */
enum { BCSIM_ENC_EXTENDED = 0, BCSIM_ENC_COMPAT = 1 };
/* Link queue model: INFINITE = unbounded FIFO; DROPTAIL = at most queue_dev_pkts +
 * queue_disc_pkts frames waiting per link, later frames dropped (fragment loss);
 * FQCODEL = ns-3 FqCoDelQueueDisc (the newer default root queue disc that
 * address.Assign installs, blockchain-simulator.cc:41-42) in front of the
 * queue_dev_pkts device queue with flow control: per-flow CoDel, DRR over the
 * flows, overlimit drops from the fattest flow; flows are the 5-tuple hash with
 * each client socket's ephemeral port bound at its first send */
enum { BCSIM_QUEUE_INFINITE = 0, BCSIM_QUEUE_DROPTAIL = 1, BCSIM_QUEUE_FQCODEL = 2 };
enum { BCSIM_ENGINE_AUTO = 0, BCSIM_ENGINE_DENSE = 1, BCSIM_ENGINE_SPARSE = 2 };

/* ---- status codes --------------------------------------------------------- */
enum {
  BCSIM_OK = 0,
  BCSIM_E_INVAL = -1,        /* bad argument / config */
  BCSIM_E_NOMEM = -2,        /* host or device allocation failed */
  BCSIM_E_HIP = -3,          /* HIP runtime error */
  BCSIM_E_OVERFLOW = -4,     /* a fixed-capacity engine buffer overflowed */
  BCSIM_E_UNSUPPORTED = -5,  /* config not supported by this engine */
  BCSIM_E_ENCODING = -6,     /* compat encoding hit reference UB (bad index) */
  BCSIM_E_TIE = -7,          /* a tie-order precondition of the engine failed */
  BCSIM_E_NODEVICE = -8,     /* no HIP device */
  BCSIM_E_STATE = -9,        /* call out of order */
  BCSIM_E_INDEX = -10,       /* PBFT tx[] index out of range (reference UB) */
  BCSIM_E_PEER = -11         /* multi-GPU: another rank of the partition failed */
};

/* ---- configuration -------------------------------------------------------- */
/* Mirrors the reference's hard-coded knobs (SURVEY.md §5 "Config / flag
 * system"): N blockchain-simulator.cc:67, DataRate/Delay :23-24, Stop :55,
 * PBFT pbft-node.cc:101-110,377,407, Raft raft-node.cc:23-24,80,216,248,361,
 * Paxos paxos-node.cc:136. */
typedef struct bcsim_config {
  uint32_t abi_version;        /* = BCSIM_ABI_VERSION */
  uint32_t protocol;           /* BCSIM_PBFT / RAFT / PAXOS */
  uint32_t n_nodes;            /* N (8 in the reference) */
  uint32_t n_replicas;         /* independent Monte Carlo replicas (>= 1) */
  uint64_t link_rate_bps;      /* 3 Mbps */
  int64_t  link_delay_ns;      /* 3 ms; per-edge override via CSR */
  uint32_t mtu;                /* 1500 (PointToPointNetDevice default) */
  uint32_t delay_mode;         /* BCSIM_DELAY_* */
  int64_t  app_delay_ns;       /* FIXED mode app delay before SendPacket */
  uint32_t rng_mode;           /* BCSIM_RNG_* */
  uint32_t time_round;         /* BCSIM_TIME_* */
  uint64_t seed;               /* glibc srand seed (1) / counter key */
  uint32_t encoding;           /* BCSIM_ENC_* */
  uint32_t echo;               /* 1 = echo every delivered packet (reference) */
  int64_t  t_end_ns;           /* hard stop; <= 0: until quiescence */
  int64_t  stop_ns;            /* Application Stop time (10 s); <0: none */
  /* PBFT */
  uint32_t pbft_rounds;        /* n_round cancel threshold (40) */
  uint32_t pbft_block_bytes;   /* block payload; 0 = tx_size*num (50,000) */
  float    pbft_timeout_s;     /* block interval float seconds (0.05f) */
  uint32_t pbft_view_change;   /* 1 = rand()%100==5 lottery (reference) */
  uint32_t pbft_seq_cap;       /* TX tx[1000] capacity */
  /* Raft */
  uint32_t raft_blocks;        /* blockNum stop threshold (50) */
  uint32_t raft_proposal_bytes;/* 0 = tx_size*num (20,000) */
  float    raft_heartbeat_s;   /* heartbeat float seconds (0.05f) */
  uint32_t raft_proposal_rounds; /* SendTX round stop (50) */
  int64_t  raft_proposal_delay_ns; /* Seconds(1) before proposals */
  /* Paxos */
  uint32_t paxos_proposers;    /* nodes 0..k-1 propose at t=0 (3) */
  /* engine capacities (GPU engine; 0 = automatic) */
  uint32_t device;             /* HIP device ordinal */
  uint32_t cap_ops_per_node;   /* pending link ops per node */
  uint32_t cap_bucket_records; /* arrival records per time bucket */
  uint32_t n_buckets;          /* time-bucket ring length */
  uint32_t cap_timers_per_node;
  uint64_t max_events;         /* oracle guard (0 = unlimited) */
  /* link queues: the PointToPointNetDevice
   * DropTail TX queue ("100p", blockchain-simulator.cc:20-24) behind the root
   * queue disc that address.Assign installs (:41-42; pfifo_fast "1000p" here,
   * the ns-3 default is version dependent).  DESIGN.md §2.2. */
  uint32_t queue_model;        /* BCSIM_QUEUE_INFINITE (default) / _DROPTAIL */
  uint32_t queue_dev_pkts;     /* device queue limit, packets (100) */
  uint32_t queue_disc_pkts;    /* queue-disc limit, packets (1000; 0 = none) */
  uint32_t cap_queue_msgs;     /* GPU engine: queued messages per link (0 = 256) */
  /* Paxos decrees (build extension for BASELINE configs[2]): each
   * proposer runs instances 0..paxos_decrees-1 one after another; 0/1 = the
   * reference's single decree (paxos-node.cc:510-522, :323-361) */
  uint32_t paxos_decrees;
  /* GPU engine layout: DENSE = a 16-byte inbox slot per edge and
   * bucket, one workgroup per node per launch; SPARSE = list-only inbox, launches
   * over the active nodes, hub-compact link state (Paxos on the full mesh); AUTO =
   * SPARSE when the dense per-edge state of all replicas exceeds ~96 GB */
  uint32_t engine_mode;        /* BCSIM_ENGINE_AUTO / _DENSE / _SPARSE */
  /* FQCODEL queue disc (ns-3 FqCoDelQueueDisc / CoDelQueueDisc attributes; 0 = the
   * ns-3 default in brackets) */
  uint32_t fq_limit_pkts;      /* MaxSize [10240p] */
  uint32_t fq_flows;           /* Flows [1024] */
  uint32_t fq_quantum;         /* Quantum bytes [the device MTU] */
  uint32_t fq_drop_batch;      /* DropBatchSize [64] */
  int64_t  fq_target_ns;       /* CoDel Target [5 ms] */
  int64_t  fq_interval_ns;     /* CoDel Interval [100 ms] */
  uint32_t fq_min_bytes;       /* CoDel MinBytes [1500] */
  uint32_t fq_perturbation;    /* Perturbation (hash salt) [0] */
  uint32_t reserved[2];
} bcsim_config;

/* ---- outputs -------------------------------------------------------------- */
/* Trace kinds: integer-ns restatement of the reference's NS_LOG_INFO lines. */
enum {
  BCSIM_TR_PBFT_COMMIT = 1,   /* pbft-node.cc:259  a=v(global) b=block_num c=value */
  BCSIM_TR_PBFT_BLOCK = 2,    /* pbft-node.cc:387  a=n (sequence) b=v */
  BCSIM_TR_PBFT_STOP = 3,     /* pbft-node.cc:408  a=n_round */
  BCSIM_TR_PBFT_VIEW = 4,     /* pbft-node.cc:278  a=v b=leader */
  BCSIM_TR_RAFT_ELECTION = 10,/* raft-node.cc:399 */
  BCSIM_TR_RAFT_LEADER = 11,  /* raft-node.cc:212 */
  BCSIM_TR_RAFT_BLOCK = 12,   /* raft-node.cc:246  a=blockNum */
  BCSIM_TR_RAFT_DONE = 13,    /* raft-node.cc:249  a=blockNum */
  BCSIM_TR_RAFT_PROPOSAL = 14,/* raft-node.cc:342  a=round */
  BCSIM_TR_RAFT_STOP = 15,    /* raft-node.cc:122-123 a=blockNum b=round */
  BCSIM_TR_PAXOS_COMMIT = 20, /* paxos-node.cc:339 a=ticket */
  BCSIM_TR_PAXOS_TICKET = 21, /* paxos-node.cc:518 a=ticket */
  BCSIM_TR_GOSSIP_BLOCK = 30, /* gossip origin tick  a=seq */
  BCSIM_TR_GOSSIP_DELIVER = 31/* first receipt       a=seq b=hops c=sender */
};

typedef struct bcsim_trace_rec {
  int64_t  t_ns;        /* simulated time of the logging event */
  int64_t  key_ts;      /* canonical key of that event: t_sched */
  uint32_t key_origin;  /*   origin node */
  uint32_t key_sub;     /*   origin's schedule counter */
  uint32_t replica;
  uint32_t node;
  uint32_t kind;        /* BCSIM_TR_* */
  int32_t  a, b, c;
} bcsim_trace_rec;      /* 48 bytes */

enum { BCSIM_MSG_TYPES = 16 };
typedef struct bcsim_counters {
  uint64_t delivered[BCSIM_MSG_TYPES]; /* HandleRead deliveries per msg type */
  uint64_t delivered_total;            /* echoes excluded */
  uint64_t echoes;                     /* echo transmissions (pbft-node.cc:175) */
  uint64_t sends;                      /* SendPacket executions */
  uint64_t dropped;                    /* Paxos *end() sends (no route) */
  uint64_t wrong_msgs;                 /* "Wrong msg" log lines */
  uint64_t events;                     /* protocol events processed */
  int64_t  t_last_ns;                  /* latest processed event time */
  uint64_t trace_records;
  uint64_t frames_dropped;             /* DROPTAIL: frames refused by a full link queue */
  uint64_t msgs_lost;                  /* DROPTAIL: messages with a dropped fragment (never delivered) */
  uint64_t reserved[5];
} bcsim_counters;

typedef struct bcsim_status {
  int64_t  now_ns;       /* all events with t < now_ns have been processed */
  int64_t  next_ns;      /* earliest pending event (INT64_MAX if none) */
  uint64_t cells;        /* time cells (windows) processed (GPU engine) */
  uint32_t quiescent;    /* 1 = no pending events */
  int32_t  error;        /* sticky error code */
  int64_t  lookahead_ns; /* window length L */
} bcsim_status;

typedef struct bcsim_sim bcsim_sim;

/* ---- entry points --------------------------------------------------------- */
/* Fill cfg with the reference defaults for `protocol` on N nodes
 * (blockchain-simulator.cc:23-24,55,67; per-protocol StartApplication). */
int bcsim_config_default(bcsim_config* cfg, uint32_t protocol, uint32_t n_nodes);

/* Replaces NetworkHelper::NetworkHelper(N) + NetworkHelper::Install
 * (network-helper.cc:16-37): allocates node state for cfg->n_nodes apps of
 * cfg->protocol (all replicas) on device cfg->device.  The topology defaults
 * to the reference full mesh (blockchain-simulator.cc:34-51: peers in
 * ascending id order). */
int bcsim_create(const bcsim_config* cfg, bcsim_sim** out);

/* Replaces the mesh loop blockchain-simulator.cc:34-51 +
 * m_nodesConnectionsIps (network-helper.h:19): sender-major CSR; row s lists
 * s's peers in the order the app iterates m_peersAddresses (ascending id in
 * the reference); prop_ns per edge (NULL: cfg->link_delay_ns).  The graph
 * must be symmetric (replies travel the reverse edge).  Call before run. */
int bcsim_set_topology_csr(bcsim_sim* s, uint32_t n_nodes,
                           const uint32_t* row_ptr, const uint32_t* col_idx,
                           const int64_t* prop_ns);

/* Topology builder (the reference hard-codes the full
 * mesh of blockchain-simulator.cc:34-51): a simple, symmetric random
 * d-regular graph on n nodes (configuration model paired by a seeded
 * splitmix64 Fisher-Yates shuffle, self-loops and multi-edges removed by
 * random double-edge swaps), rows sorted ascending like the reference's peer
 * lists.  row_ptr has n+1 entries, col_idx n*d.  Host-only, deterministic in
 * (n, d, seed).  Needs n*d even and d < n. */
int bcsim_topology_random_regular(uint32_t n, uint32_t d, uint64_t seed,
                                  uint32_t* row_ptr, uint32_t* col_idx);

/* Replaces Simulator::Run (blockchain-simulator.cc:57): process every event
 * with t < t_until_ns (INT64_MAX: until quiescence or cfg->t_end_ns). */
int bcsim_run(bcsim_sim* s, int64_t t_until_ns);

/* Trace records (canonical order: t, key, replica, node, record order). */
int bcsim_read_trace(bcsim_sim* s, bcsim_trace_rec* buf, uint64_t cap,
                     uint64_t* n_out);
int bcsim_read_counters(bcsim_sim* s, bcsim_counters* out);
int bcsim_read_status(bcsim_sim* s, bcsim_status* out);

/* Replaces Simulator::Destroy (blockchain-simulator.cc:58). */
int bcsim_destroy(bcsim_sim* s);

/* Trace writer: the reference's NS_LOG_INFO message for
 * one trace record -- original strings (pbft-node.cc:259,278,387,408;
 * raft-node.cc:122-123,212,246,249,342,362,399; paxos-node.cc:339,518),
 * GetSeconds() at default ostream precision, embedded newlines kept (NS_LOG
 * appends the final one).  cfg may be NULL.  Host-only; writes at most cap-1
 * bytes + NUL, *n_out = full length. */
int bcsim_format_trace_line(const bcsim_trace_rec* r, const bcsim_config* cfg, char* buf, uint64_t cap,
                            uint64_t* n_out);

const char* bcsim_strerror(int code);
/* Last HIP/engine diagnostic text (thread-unsafe, for logs). */
const char* bcsim_last_error_detail(void);

/* ---- multi-GPU: node-partitioned conservative PDES --------
 * nranks handles (one process and one GPU each) simulate ONE system: rank r
 * owns a contiguous node range of every replica; records for another rank's
 * nodes are exchanged once per cell (lookahead window), the next cell is
 * agreed by an all-reduce MIN, and the PBFT SendBlock tick gathers the
 * leader flags and the v-log.  No reference counterpart: the reference is
 * single-threaded ns-3 (blockchain-simulator.cc:57).  Call before the first
 * bcsim_run; every rank must then call bcsim_run with the same t_until.
 * Counters and traces are per rank (sum / merge them across ranks). */
typedef struct bcsim_transport {
  void* ctx;
  /* in-place all-reduce of n int64 values on host memory; op 0 = MIN, 1 = SUM */
  int (*allreduce_i64)(void* ctx, int64_t* v, uint32_t n, int32_t op);
  /* all-to-all-v of host bytes: send holds nranks consecutive segments of
   * send_bytes[r] bytes (segment r goes to rank r); recv gets the segments
   * from ranks 0..nranks-1 back to back, recv_bytes[r] each (<= recv_cap).
   * A failed rank passes send_bytes[r] = 2^62 for every r and send = NULL:
   * if any rank's count is 2^62, no payload moves, recv_bytes[r] is the count
   * rank r sent (2^62 for the failed one) and the call returns 0, so every
   * rank leaves the run together (BCSIM_E_PEER on the healthy ones). */
  int (*alltoallv)(void* ctx, const void* send, const uint64_t* send_bytes, void* recv, uint64_t recv_cap,
                   uint64_t* recv_bytes);
} bcsim_transport;

/* Partition over a caller-provided host transport (e.g. torch.distributed
 * gloo callbacks; used by the tests: several ranks may share one GPU). */
int bcsim_set_partition(bcsim_sim* s, uint32_t rank, uint32_t nranks, const bcsim_transport* t);
/* Partition over RCCL (xGMI): device-resident exchange.  unique_id is the
 * ncclUniqueId made by bcsim_rccl_unique_id on rank 0 and shared by the caller. */
int bcsim_rccl_unique_id(void* out, uint64_t cap, uint64_t* n_out);
int bcsim_set_partition_rccl(bcsim_sim* s, uint32_t rank, uint32_t nranks, const void* unique_id,
                             uint64_t id_bytes);

/* Device timing since the last reset: per-kernel-class accumulated
 * microseconds measured with hipEvents on the engine stream and launch
 * counts.  kinds: 0 scan, 1 link (fan-out scatter), 2 group, 3 tick/aux.
 * bytes_out4: [1] algorithmic bytes of the scatter (48 B per
 * record emitted), [0] 16 B per delivered record read, [2] 0, [3] k_link's
 * device-counted implementation bytes. */
int bcsim_reset_kernel_stats(bcsim_sim* s);
int bcsim_read_kernel_stats(bcsim_sim* s, double* us_out4, double* bytes_out4,
                            uint64_t* launches_out4);
/* Raw engine work counters since the last bcsim_reset_kernel_stats (testing and
 * profiling aid, no reference counterpart): [0] records emitted, [1] due ops, [2] touched
 * edges, [3] kept ops, [4] delivered records, [5] k_scan ops, [6] implicit echoes,
 * [7] k_scan windows split because a node had more arrivals than its LDS staging. */
int bcsim_read_engine_counters(bcsim_sim* s, uint64_t* out8);
/* Cell-loop statistics since bcsim_create (profiling aid): [0] windows processed, [1]
 * collectives of a node-partitioned run (control exchanges, record exchanges, all-reduces;
 * DESIGN.md §5), [2] inbox buckets zeroed for the ring-turn tag invariant, [3] 0. */
int bcsim_read_loop_stats(bcsim_sim* s, uint64_t* out4);
/* Extended cell-loop statistics since bcsim_create (profiling aid): [0..2] as
 * bcsim_read_loop_stats, [3] windows whose active lists came from the speculative k_active
 * behind k_next, [4] part cells skipped as idle (nothing can happen before the tick / run
 * limit), [5] host syncs of the cell loop (mirror spins, stream syncs, blocking collectives),
 * [6] idle parts verified empty (BCSIM_CHECK_IDLE=1), [7] windows run as device-chained windows
 * (k_win, dense gossip). */
int bcsim_read_loop_stats_ex(bcsim_sim* s, uint64_t* out8);
/* Host-side costs of the cell loop since bcsim_create (profiling aid): [0] microseconds spent
 * inside kernel launches, [1] microseconds spent waiting on the host-mapped mirror words,
 * [2] kernel launches, [3] device-chained windows whose frontier the closing k_next had built. */
int bcsim_read_host_stats(bcsim_sim* s, double* out4);

#ifdef __cplusplus
}
#endif
#endif /* BCSIM_H */
