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
//     (extras / overflow only) k_rebin, k_xcount/k_offsets/k_xplace
//     k_scan<P>     one workgroup per node: stage the node's inbox row (one
//                   16-byte slot per in-edge, ascending origin = canonical tie
//                   order) in LDS, sort by the canonical key only if needed,
//                   run the protocol:
//                     PBFT   data-parallel: wave-ballot quorum ranks per
//                            (phase, sequence), block scans for the schedule
//                            counter / rand() draw / commit prefixes, every
//                            lane emits its own echo / reply ops
//                     Raft, Paxos  serial state machine in key order (lane 0)
//     k_link        one workgroup per node: per out-edge FIFO (busy_until) in
//                   canonical key order, serialization + propagation, and the
//                   scatter of 16-byte records into the receivers' inbox
//                   slots of the arrival cell
//     (PBFT) k_pbft_tick   SendBlock tick of every node (globals n, n_round, v)
//     (Raft, glibc rng) k_draws   election-timeout draws in canonical order
//
// Semantics are specified in DESIGN.md §2 and restated serially by oracle/
// (the parity checker).  No code here calls the oracle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "engine.h"
#include "host_math.h"

namespace bcsim {

// ---------------------------------------------------------------------------
// kernel parameter block (device-resident, one per simulation).  Its arrays are global memory;
// device code reaches them through gbl() (below), so that accesses compile to global_*
// instructions instead of flat_* ones.
#define GP(T) T*
constexpr uint32_t kKstStripes = 64;
constexpr int kMaxBuckets = 64;
constexpr uint32_t kNextBlocks = 512;  // k_next workgroups at most (41 M gnodes: 2 per CU)  // kstat[kKstStripes][8]: per-workgroup stripes, summed on the host
struct KP {
  uint32_t N, R, NT, E;
  uint32_t protocol, delay_mode, rng_mode, encoding, echo;
  uint32_t deg_max;
  uint32_t deg_reg;  // every node's degree when all are equal and row[i] = i * deg_reg, else 0
  int64_t L;
  uint64_t L_magic;  // ceil(2^64 / L): x / L for x < 2^32 is the high half of x * L_magic
  int64_t app_delay;
  int64_t tx_tot[2], tx_last[2];
  int64_t pbft_period, raft_hb, raft_prop_delay, stop_ns;
  uint32_t pbft_rounds, pbft_seq_cap, pbft_view_change, raft_blocks;
  uint32_t raft_prop_rounds, paxos_proposers;
  uint32_t paxos_fast_win;  // Paxos proposer windows data-parallel (paxos_window_fast; BCSIM_PX_FAST=0: off)
  uint64_t seed;
  GP(int64_t) pbft_delay;
  GP(int64_t) raft_delay;
  GP(int64_t) raft_elec;
  GP(int64_t) paxos_delay;
  GP(int64_t) jit_delay;  // the running protocol's getRandomDelay table
  uint32_t jit_mod;
  // topology (per replica, shared)
  GP(const uint32_t) row;
  GP(const uint32_t) col;
  GP(const uint32_t) rev;
  GP(const int64_t) prop;     // per edge (sender-major)
  GP(const int64_t) prop_in;  // per in-slot q: prop[rev[q]]
  // common node state
  GP(uint32_t) sub;
  GP(uint64_t) draws;
  // PBFT
  GP(int32_t) leader;
  GP(int32_t) block_num;
  GP(uint8_t) tick_alive;
  GP(uint32_t) tick_sub;
  GP(int32_t) tx_val;
  GP(int32_t) tx_pv;
  GP(int32_t) tx_cv;
  GP(int32_t) g_n;  // per replica
  GP(int32_t) g_nround;
  // Raft / Paxos
  GP(int32_t) is_leader;
  GP(int32_t) has_voted;
  GP(int32_t) m_value;
  GP(int32_t) vote_s;
  GP(int32_t) vote_f;
  GP(int32_t) acv;
  GP(int32_t) blockNum;
  GP(int32_t) round;
  GP(uint32_t) next_election;
  GP(uint32_t) next_heartbeat;
  GP(int32_t) ticket;
  GP(int32_t) proposal;
  GP(int32_t) decree;
  GP(int32_t) px;   // Paxos acceptor state [NT][K][4]: t_max, command, t_store, isCommit (per decree)
  uint32_t K;    // Paxos decrees (>= 1)
  // Gossip (BCSIM_GOSSIP): first-receipt flag per (gnode, sequence); origin tick count in round[]
  GP(uint8_t) gseen;
  // timers / ops
  GP(TimerEnt) timers;
  uint32_t cap_timers;
  GP(Op) ops;
  GP(uint32_t) n_ops;
  uint32_t cap_ops;
  uint32_t cap_eidx;  // k_link LDS index capacity for listed due ops
  GP(uint32_t) eidx_g;   // [grid][cap_ops] k_link index area of a node with more (nullptr: cap_eidx == cap_ops)
  // per-edge reply slots: ring of kOpRing cells, one slot per
  // (replica, edge) for a unicast reply (PBFT PREPARE_RES) of the edge's main
  // inbox record.  A slot op is live while t >= the current window start;
  // nullptr = disabled (replies go to the op lists)
  // 16-byte reply slots keyed by the ARRIVAL cell (ring index = arrival cell % kOpRing):
  // a main-slot arrival has at most one reply, so a slot is never occupied when written
  // (no read-before-write); entry = {due t lo, due t hi, sub, f0 | f1 << 16} of the PBFT
  // PREPARE_RES (type, f2 = '0', dt = app delay, origin = node are implied).  Only with
  // fixed app delays < L (due cell <= arrival cell + 1).
  GP(uint4) eslot;          // [kOpRing][R][E]
  GP(uint8_t) sflag;        // [kOpRing][NT] bit k: replies of this arrival cell due in arrival cell + k
  uint64_t cap_eslot;
  // implicit echoes: k_link echoes a node's main inbox records itself (the
  // in-slot index is the reverse out-edge) and releases the slots; k_scan
  // writes echo ops only for extras records
  uint32_t impl;
  // window stamp per gnode: k_scan_pbft applied the implicit echoes of the window starting at
  // eapp[g] itself (the link kernels skip them); LLONG_MIN = never
  GP(long long) eapp;
  // PBFT heavy-wave descriptors (k_scan_pbft -> k_link_mesh): a PREPARE wave's
  // replies as ONE descriptor {due, first sub, payload} + the bitmap of in-slots that replied
  // (sub + rank), and the waves' echoes as pending {t, big} + bitmap, applied by the node's next
  // link stage that walks its edges (k_link_mesh: the link words are loaded there anyway)
  uint32_t desc;          // enabled: dense full mesh with k_link_mesh as the link stage
  uint32_t dwords;        // bitmap words per descriptor: ceil(deg_max / 32) <= kDescWords
  GP(uint4) rdesc;           // [kOpRing][NT] {due lo, due hi, sub, f0 | f1 << 16} of the arrival cell
  GP(uint32_t) rbits;        // [kOpRing][NT][dwords]
  GP(uint4) edesc;           // [NT][kEDesc] {t lo, t hi, big, 0}
  GP(uint32_t) ebits;        // [NT][kEDesc][dwords]
  GP(uint8_t) en;            // [NT] pending echo descriptors
  // full-mesh tiled link stage (k_mesh_prep -> k_mesh_tile): the job k_mesh_prep
  // leaves per gnode -- {epoch, flags, ne | n_bc << 8, 0}, the two reply descriptors, the pending
  // echo times -- its due broadcasts in key order (RawOp words), its descriptor bitmaps cut into
  // 64-receiver tiles (bit k = receiver tile base + k), and per (replica, 32-sender tile) the epoch
  // of the last launch that left a job in it
  GP(uint4) mjob;            // [NT][4]
  GP(uint4) mbc;             // [NT][kMeshBc][2]
  GP(uint4) mtb;             // [NT][n_tiles][2] reply bitmaps per receiver tile: {mask lo, mask hi, rank base, 0}
  GP(uint2) mte;             // [NT][n_tiles][kEDesc] pending echo bitmaps per receiver tile
  GP(uint32_t) mtile;        // [R][n_stiles]
  uint32_t n_stiles;
  // heavy-wave record summaries (one rank, full mesh, PBFT fast paths): the
  // slot records ONE sender writes to a 64-receiver tile in one bucket that differ only in the
  // schedule counter (sub = base + the sender's out-edge index, pbft-node.cc:360-367 fan-out)
  // are written by k_mesh_tile as one entry {mask lo, mask hi, t_off, base}{f0 | f1 << 16,
  // f2 | type << 16 | flags << 24, 0, 0} (live: the flags' ring-turn tag, a nonzero mask) instead
  // of up to 64 16-byte records; k_scan_rt reads a receiver tile's entries of all senders, and a
  // row leaving the fast kernels is materialised first.  Every other slot record is physical,
  // and the byte xsum = 0x80 | its tag tells the readers to load the (tile, sender)'s slots.
  uint32_t sum;
  GP(uint4) msum;            // [B][R][n_tiles][N][2]
  GP(uint8_t) xsum;          // [B][R][n_tiles][N]
  // (summary mode) row-uniform link state: rul[g] = 1 << 63 | w means that every out-edge of gnode g
  // whose receiver's bit in rex[g] is clear has the link word w (k_mesh_row keeps a heavy wave's
  // rows so: one word per sender instead of 4095); 0 = the physical words hold every edge.  The
  // generic link stage writes the words out first (rul_flush)
  GP(uint64_t) rul;          // [NT]
  GP(uint64_t) rex;          // [NT][n_tiles] bit k: receiver tile * 64 + k's edge has its own word
  // list-2 overlap: k_scan_pbft stamps the nodes it leaves to the generic kernels
  // with the window's epoch; their scan and link stage run on a second stream beside the other
  // nodes' link stage, which skips them.  loop_list: the list k_link<.., LOOP> walks (3; 2 in
  // the second stream's parameter block)
  GP(uint32_t) l2mark;       // [NT]
  uint32_t loop_list;
  int64_t prop_const;    // propagation delay of every edge, or -1 (per-edge array)
  // links
  GP(uint64_t) link;  // per edge: busy_until << 16 | (arrival cell of the last record & 0xFFFF)
  // DROPTAIL link queues: per edge a ring of the messages of its busy
  // period, entry = start << 17 | big << 16 | accepted frames; meta = head | n << 16 |
  // frames << 32
  uint32_t qmodel, qcap_frames, cap_q;  // qmodel: 0 INFINITE, 1 DROPTAIL, 2 FQCODEL
  uint32_t nfr[2];
  int64_t tx_full[2];
  GP(uint64_t) qring;
  GP(uint64_t) qmeta;
  // FQCODEL link queues, per rank-local edge: a header of kFqH words (three
  // flows' CoDel + DRR state, new / old flow lists, device-queue ring position, device busy end,
  // packets in the disc, message-table bitmap), the start times of the device queue's waiting
  // frames [fq_devcap], three packet rings [3][cap_fqp] {enq lo, enq hi, msg | frame << 16,
  // IPv4 bytes} and the message table [cap_fqm] {sub, f0 | f1 << 16, f2 | type << 16 | big << 24 |
  // echo << 25 | lost << 26, fragments left}.  Flow classification (oracle fq_bind /
  // fq_class_slot): fqlnk[e] = the link's number in the mesh loop (global edge), fqport = the
  // UDP port of the edge's client socket (0 until its first send binds it), fqpeer = the port of
  // the reverse edge's socket (the echo class's destination port), fqnport[g] = sockets the
  // node bound so far, fqphant[g] = Paxos's *end() socket bound, fqkey = a window's first-send
  // keys {t lo, t hi, dt, sub} (binding order scratch)
  GP(uint32_t) fqh;
  GP(int64_t) fqdev;
  GP(uint4) fqpk;
  GP(uint4) fqmsg;
  GP(const uint32_t) fqlnk;
  GP(uint32_t) fqport;
  GP(uint32_t) fqpeer;
  GP(uint32_t) fqnport;
  GP(uint32_t) fqphant;
  GP(uint4) fqkey;
  GP(const uint64_t) fqpoff;  // per edge: its packet rings' offset in fqpk | per-flow capacity << 48
  uint32_t fq_flows, fq_pert;
  uint32_t fq_devcap, cap_fqp, cap_fqm, fq_limit, fq_quantum, fq_batch, fq_min_bytes, fq_target_c, fq_interval_c;
  uint32_t ip_full[2], ip_last[2];
  // debug (BCSIM_FQLOG=<file>): every FQCODEL link event with t in [fqlog_t0, fqlog_t1) as two
  // uint4 {t lo, t hi, edge, kind << 24 | frame}, {msg sub, x lo, x hi, echo} (tools/fq_log.py)
  GP(uint4) fqlog;
  GP(uint32_t) fqlog_n;
  uint32_t cap_fqlog;
  long long fqlog_t0, fqlog_t1;
  // inbox
  GP(Rec) inbox;            // [B][R][E]  receiver-major (in-slot order)
  GP(uint8_t) rtile;        // [B][R][n_tiles] full mesh: a record for a receiver of this 64-node
                         // tile sits in the bucket (senders set one byte per tile, not one per node)
  uint32_t mesh, n_tiles;  // full-mesh topology (arithmetic peers / in-slots)
  GP(uint8_t) iflag;        // [B][NT] node has records in the bucket
  GP(long long) bmin;       // [B] lower bound of the arrival times of the bucket's records (LLONG_MAX: none):
                         // a window that ends before it skips the flagged rows (node_flagged_w)
  GP(uint32_t) bucket_cnt;  // [B] nonzero = the bucket holds records (slots + extras); see mark_busy
  // host-mapped mirror of the control block (ctl_words words from p.err on): k_next publishes
  // it at the end of a window, then the window's sequence number at word ctl_words, so the
  // host's end-of-window read-back is a spin on that word, no copy and no stream sync
  GP(uint32_t) ctl_mirror;
  uint32_t ctl_words;
  GP(uint32_t) act_mirror;  // host-mapped: k_active's list lengths [0..1] (its last workgroup), [2] sequence
  GP(uint32_t) act_done;    // k_active workgroups finished (reset by the last)
  GP(uint32_t) x_cnt;       // [B] extras in the bucket
  uint32_t n_buckets;
  GP(XRec) xbuf;            // [B][cap_x]
  uint32_t cap_x;
  GP(XRec) xgrp;            // extras of the current cell grouped by receiver
  GP(XRec) xstage;          // [NT][cap_stage] k_link staging of extras / overflow records
  GP(uint32_t) xmeta;       // [NT][cap_stage] (list << 24) | rank within the list
  uint32_t cap_stage;
  GP(XRec) ov;
  GP(uint32_t) ov_cnt;
  uint32_t cap_ov;
  GP(uint32_t) seg_cnt;
  GP(uint32_t) seg_off;
  GP(uint32_t) cursor;
  uint32_t cap_arr;  // LDS staging capacity of k_scan (power of two, <= 4096)
  // outputs
  GP(bcsim_trace_rec) trace;
  GP(uint32_t) trace_cnt;
  uint32_t cap_trace;
  GP(VLog) vlog;
  GP(uint32_t) vlog_cnt;
  uint32_t cap_vlog;
  GP(DrawReq) dreq;
  GP(uint32_t) dreq_cnt;
  uint32_t cap_dreq;
  GP(const int32_t) glibc;
  uint32_t glibc_len;
  GP(uint32_t) glibc_pos;  // per replica
  GP(unsigned long long) counters;  // R * CNT_N
  uint32_t cnt_stripes;  // counters[cnt_stripes][R][CNT_N]: workgroup b adds to stripe b % cnt_stripes
  GP(unsigned long long) kstat;     // link / scan algorithmic counters (KST_*)
  GP(int32_t) err;
  GP(int32_t) dbg;  // first error's source line
  GP(unsigned long long) trail;  // BCSIM_CHECKED + BCSIM_TRAIL: host-mapped breadcrumbs
  GP(unsigned long long) wgt;    // BCSIM_WGT: per-workgroup k_link timing [NT][8] (debug)
  GP(unsigned long long) wgtt;   // BCSIM_WGT: per-workgroup k_mesh_tile phase clocks [tiles][8] (debug)
  uint32_t exp;               // BCSIM_EXP: performance experiments that break results (debug, never in tests)
  GP(unsigned long long) wgs;    // BCSIM_WGT: per-workgroup k_scan phase timing [NT][8] (debug)
  // (the doubled-window KP of the few-node launches only) sort_window's merge area, cap_arr
  // entries per workgroup: the leader's main and extras runs are merged through it
  GP(uint4) sortbuf;
  GP(unsigned long long) fdbg;   // BCSIM_FDBG: why nodes leave the fast kernels [16] (debug; see FDBG)
  uint64_t cap_E, cap_txn, cap_glibc, cap_inbox, cap_xbuf;
  GP(long long) node_tnext;
  GP(long long) node_onext;
  GP(long long) pred;  // k_next's prediction of the next window {valid, cell, lo, hi} (control block)
  GP(long long) win;   // device-chained windows (k_win): kWin* words (control block)
  GP(long long) scal;  // [0] next_local, [1] ov_min_cell, [2] n_alive_ticks, [3] next timer,
                    // [4] earliest arrival cell shipped to another rank (node-partitioned)
  GP(long long) nxt_part;  // [kNextBlocks] k_next per-workgroup minima
  GP(uint32_t) nxt_done;   // k_next workgroups finished (the last one reduces and resets it)
  GP(long long) rb_acc;    // k_rebin (publishing): the staying records' minimum cell (LLONG_MAX between launches)
  GP(uint32_t) rb_done;    // k_rebin workgroups finished (the last one resets it)
  // k_rebin (publishing, dense): the records that stay beyond the ring, compacted (cap_ov) and
  // counted (rb_n[0] during the launch, rb_n[1] the total for k_ov_back) -- the overflow list
  // keeps only live records instead of growing by every block's far-future records
  GP(XRec) ov_tmp;
  GP(uint32_t) rb_n;
  // node partition (multi-GPU PDES): this rank owns nodes
  // [nlo, nlo + nloc) of every replica; records for other ranks' receivers
  // are staged in sendbuf and exchanged once per cell
  uint32_t nlo, nloc, rank, nranks;
  // per-edge state (inbox slots, reply slots, link words, queue rings) is rank-local: only the
  // edges in the rows of this rank's nodes, [e_lo, e_lo + E_loc) of every replica
  uint32_t e_lo;
  uint64_t E_loc;
  GP(const uint16_t) owner;    // [N] rank owning node i
  GP(XRec) sendbuf;            // [nranks][cap_send]
  GP(uint32_t) send_cnt;       // [nranks] (control block)
  uint32_t cap_send;
  GP(const uint8_t) lead_all;  // [R][N] PBFT leader flags gathered from all ranks
  GP(uint8_t) lead_loc;        // [R][N] this rank's leader flags (k_lead)
  // sparse mode: no per-edge inbox slots (every record goes through
  // the bucket lists), launches over compact lists of active gnodes, hub-compact link
  // state (hubs > 0: only edges with an endpoint < hubs carry traffic)
  uint32_t sparse, hubs;
  uint32_t cap_ops_light, n_heavy;  // nodes < n_heavy hold cap_ops pending ops, others cap_ops_light
  GP(uint32_t) act;    // [4][NT] gnodes of the window: k_scan list, k_link list, and (dense gossip)
                    // the nodes k_gossip_scan / k_gossip_link leave to the generic kernels
  GP(uint32_t) act_n;  // [4] their lengths
  // debug (BCSIM_DBG_EVENTS=<t_max ns>): Raft/Paxos/gossip serial handlers emit one
  // trace record of kind 90 + event class per handled event with t < dbg_tmax
  long long dbg_tmax;
};

constexpr int kMaxRanks = 16;
// receiver-tile flags (rtile) one per 128-byte line: every sender of a heavy wave sets its
// receiver tiles' flags, and same-line stores from thousands of workgroups serialise in an L2
// channel (k_mesh_row: ~100 us per launch with the 64 flags of a bucket in one line)
constexpr uint32_t kRtPad = 128;
constexpr uint32_t kDescWords = 128;  // descriptor bitmaps: in-slots of degree <= 4096
constexpr uint32_t kEDesc = 2;        // pending echo descriptors per node (LDS: k_link_mesh keeps 4 WGs/CU)
// sflag bits of a reply descriptor of the arrival cell (bits 0..3: reply slots due in cell + k)
constexpr uint32_t kSfD0 = 16u, kSfD1 = 32u, kSfD = kSfD0 | kSfD1;  // due in this cell / the next
// tiled mesh link stage: due broadcasts per job, senders x receivers per tile, 64-slot chunks
// k_mesh_tile build switches (A/B: tools/build_variant.sh): senders per tile; link words through
// LDS, written after the walk (1) or in the walk (0: 9 % faster, PBFT n=4096); workgroup order
// receiver-tile-major (1: the slow receiver tile 0 -- the leader's -- goes first) or sender-major
#ifndef BCSIM_TILE_TS
#define BCSIM_TILE_TS 32
#endif
#ifndef BCSIM_TILE_DEFER
#define BCSIM_TILE_DEFER 0
#endif
#ifndef BCSIM_TILE_RTMAJOR
#define BCSIM_TILE_RTMAJOR 0
#endif
constexpr uint32_t kMeshBc = 2, kTS = BCSIM_TILE_TS, kTR = 64;
constexpr uint32_t kTileThreads = kTS * 16;  // four senders per wave
constexpr uint32_t kLoopGrid = 256;  // workgroups of the looped generic grids (lists 2, 3) at most
constexpr uint32_t kLinkLoopThreads = 512;  // k_link<.., LOOP> lanes per workgroup (its launch bound: no scratch)
// job flags (mjob[g][0].y)
constexpr uint32_t kJSl0 = 1u, kJSl1 = 2u, kJSd0 = 4u, kJSd1 = 8u, kJRxe = 16u, kJBig0 = 32u, kJBig1 = 64u;


// ---------------------------------------------------------------------------
// device helpers
// A KP array pointer as a global-memory (address space 1) pointer: accesses through it compile
// to global_* instructions.  Through a plain pointer loaded from the parameter block the
// compiler emits flat_* accesses, and a flat access may alias LDS, so it drains all outstanding
// memory operations (s_waitcnt vmcnt(0)) before the next LDS access -- which serialised the LDS
// phases of the tile and scan kernels behind their global stores.  (The round trip cast back to
// a generic pointer is folded away: the access must go through the G<T> pointer itself.)
#ifdef __HIP_DEVICE_COMPILE__
template <typename T>
using G = __attribute__((address_space(1))) T;
#else
template <typename T>
using G = T;  // (host pass: the device functions are parsed, not compiled)
#endif
template <typename T>
__device__ __forceinline__ G<T>* gbl(T* q) {
  return (G<T>*)q;
}
// 16-byte global load / store through an address-space-1 pointer (native vector type: the HIP
// vector class has no address-space-qualified copy operations)
#ifdef HIPEMU
typedef uint4 u32x4;  // (debug host emulator, tools/hipemu)
#else
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#endif
__device__ __forceinline__ uint4 gld4(const void* q) {
  const u32x4 v = *(const G<u32x4>*)q;
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <typename T, typename V>
__device__ __forceinline__ void gadd(T* q, V v) {  // a global atomic add whose result is not used
  __hip_atomic_fetch_add(gbl(q), static_cast<T>(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T, typename V>
__device__ __forceinline__ T gadd_r(T* q, V v) {  // ... whose result is used
  return __hip_atomic_fetch_add(gbl(q), static_cast<T>(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T, typename V>
__device__ __forceinline__ void gmin(T* q, V v) {  // global atomic min (result not used)
  __hip_atomic_fetch_min(gbl(q), static_cast<T>(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gst4(void* q, const uint4& w) {
  u32x4 v;
  v.x = w.x;
  v.y = w.y;
  v.z = w.z;
  v.w = w.w;
  *(G<u32x4>*)q = v;
}
// whole-struct copies to / from global memory (AT() yields address-space-1 lvalues; the structs'
// own copy operations are for generic ones): 16-byte pieces when the size allows, else words
template <typename T>
__device__ __forceinline__ void gput(G<T>& d, const T& v) {
  static_assert(sizeof(T) % 4 == 0, "gput: word-sized structs");
  if constexpr (sizeof(T) % 16 == 0) {
    for (size_t k = 0; k < sizeof(T) / 16; ++k)
      ((G<u32x4>*)&d)[k] = reinterpret_cast<const u32x4*>(&v)[k];
  } else {
    for (size_t k = 0; k < sizeof(T) / 4; ++k) ((G<uint32_t>*)&d)[k] = reinterpret_cast<const uint32_t*>(&v)[k];
  }
}
template <typename T>
__device__ __forceinline__ T gget(const G<T>& s) {
  static_assert(sizeof(T) % 4 == 0, "gget: word-sized structs");
  T v;
  if constexpr (sizeof(T) % 16 == 0) {
    for (size_t k = 0; k < sizeof(T) / 16; ++k) reinterpret_cast<u32x4*>(&v)[k] = ((const G<u32x4>*)&s)[k];
  } else {
    for (size_t k = 0; k < sizeof(T) / 4; ++k) reinterpret_cast<uint32_t*>(&v)[k] = ((const G<uint32_t>*)&s)[k];
  }
  return v;
}

// First error wins; its source line goes to p.dbg so the host can name the
// exact capacity or invariant that failed (bcsim_last_error_detail).
__device__ inline void set_err_(const KP& p, int32_t code, int line) {
  int32_t z = 0;
  if (__hip_atomic_compare_exchange_strong(gbl(p.err), &z, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)) {
    z = 0;
    __hip_atomic_compare_exchange_strong(gbl(p.dbg), &z, line, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// The code and line are materialised by volatile asm INSIDE the (cold) error branch: as plain
// constants, loop-invariant code motion hoisted every call site's pair out of the per-arrival
// loops into registers live across the whole kernel, and in the 128-VGPR kernels those got
// spilled to scratch (k_scan<PBFT>: most of its 116 B/lane, written by every lane of every
// workgroup).
#define set_err(pp, code)                                                      \
  do {                                                                         \
    int32_t c_, l_;                                                            \
    asm volatile("v_mov_b32 %0, %1" : "=v"(c_) : "i"(static_cast<int32_t>(code))); \
    asm volatile("v_mov_b32 %0, %1" : "=v"(l_) : "i"(__LINE__));              \
    set_err_((pp), c_, l_);                                                    \
  } while (0)

// Checked array access.  In BCSIM_CHECKED builds an out-of-range index is
// recorded (source line in p.dbg, BCSIM_E_OVERFLOW in p.err) and the wave
// stops instead of faulting the GPU.
template <typename T>
__device__ inline G<T>& at_(const KP& p, T* base, uint64_t idx, uint64_t cap, int line) {
#ifdef BCSIM_CHECKED
  if (idx >= cap) {
    atomicCAS(p.dbg, 0, line);
    atomicCAS(p.err, 0, BCSIM_E_OVERFLOW);
    __builtin_amdgcn_endpgm();  // stop this wave: no access through garbage
  }
#endif
  return gbl(base)[idx];
}
// element 0 / 1 of a two-entry KP array (frame times by size class): two scalar loads and a
// select -- indexed by a lane's flag, the array read is a vector load per use, waited for
// before the next
template <typename T>
__device__ __forceinline__ T sel2(const T* a, bool one) {
  const T x = a[0], y = a[1];
  return one ? y : x;
}
#ifdef BCSIM_CHECKED
#define BAIL_IF_ERR() \
  do {                \
    if (*p.err) return; \
  } while (0)
#define TRAIL_AT(pp, g)                                                                        \
  do {                                                                                         \
    if ((pp).trail)                                                                            \
      __hip_atomic_store(&(pp).trail[g], (static_cast<unsigned long long>(g) << 32) | __LINE__, \
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);                          \
  } while (0)
#else
#define BAIL_IF_ERR() \
  do {                \
    (void)p;          \
  } while (0)
#define TRAIL_AT(pp, g) \
  do {                  \
  } while (0)
#endif
#define TRAIL(c) TRAIL_AT(*(c).p, (c).g)
#define AT(arr, idx, cap) at_(p, (arr), static_cast<uint64_t>(idx), static_cast<uint64_t>(cap), __LINE__)

// Workgroups are dispatched round-robin over the 8 XCDs; give each XCD a
// contiguous range of nodes so that concurrently running senders write
// neighbouring inbox slots (same L2) and receivers read their own rows.
__device__ inline uint32_t xcd_map(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, k = b >> 3, per = n >> 3, rem = n & 7u;
  return x * per + min(x, rem) + k;
}

// does gnode g (node i of replica rep) have arrivals in bucket b?  (own flag, or its
// receiver tile's flag in the full mesh)
__device__ inline bool node_flagged(const KP& p, uint32_t b, uint32_t g, uint32_t rep, uint32_t i) {
  // both bytes are loaded together (no dependent second round trip)
  const uint8_t f = AT(p.iflag, static_cast<size_t>(b) * p.NT + g, static_cast<uint64_t>(p.n_buckets) * p.NT);
  const uint8_t t = p.mesh ? AT(p.rtile, kRtPad * ((static_cast<size_t>(b) * p.R + rep) * p.n_tiles + (i >> 6)), kRtPad * (static_cast<uint64_t>(p.n_buckets) * p.R * p.n_tiles))
                           : 0;
  return (f | t) != 0;
}
// node_flagged for the window [.., t_hi): false when no record of the bucket arrives before
// t_hi (a cell split by a tick or a run() limit: the rows are read once, in the window that
// holds the arrivals, instead of in every window)
__device__ inline bool node_flagged_w(const KP& p, uint32_t b, uint32_t g, uint32_t rep, uint32_t i, long long t_hi) {
  const long long bm = p.bmin[b];
  const bool f = node_flagged(p, b, g, rep, i);
  return f && bm < t_hi;
}
// lower the bucket's arrival-time bound (read first: most writers find it already lower)
__device__ inline void bmin_lower(const KP& p, uint32_t b, long long t) {
  if (t < *reinterpret_cast<volatile G<long long>*>(gbl(p.bmin) + b))
    __hip_atomic_fetch_min(gbl(p.bmin) + b, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// start time of the cell that bucket k holds, seen from cell `cell` (records are emitted
// 1 .. B-1 cells ahead)
__device__ inline long long bucket_t0(const KP& p, long long cell, uint32_t k) {
  const uint32_t B = p.n_buckets;
  const long long rel = (static_cast<long long>(k) + B - cell % B) % B;
  return (cell + rel) * p.L;
}
// set-once byte flag (many writers of the same byte: read first, store only if clear)
__device__ inline void set_flag_once(uint8_t* f) {
  if (*reinterpret_cast<volatile G<uint8_t>*>(gbl(f)) == 0) *gbl(f) = 1;
}

// blockIdx -> gnode of this rank's partition (XCD-contiguous ranges)
__device__ inline uint32_t local_gnode(const KP& p, uint32_t b) {
  const uint32_t j = xcd_map(b, p.R * p.nloc);
  return (j / p.nloc) * p.N + p.nlo + j % p.nloc;
}

// rank-local per-edge index of edge / in-slot e of replica rep, and of an inbox slot
__device__ inline size_t edge_loc(const KP& p, uint32_t rep, uint32_t e) {
  return static_cast<size_t>(rep) * p.E_loc + (e - p.e_lo);
}
__device__ inline size_t inbox_idx(const KP& p, uint32_t b, uint32_t rep, uint32_t slot) {
  return (static_cast<size_t>(b) * p.R + rep) * p.E_loc + (slot - p.e_lo);
}

// Active-list launches (k_scan, k_link): a fixed grid (a multiple of 8) walks the list of
// the window's active gnodes built by k_active.  Workgroups are dispatched round-robin
// over the 8 XCDs, so XCD x = blockIdx & 7 takes the contiguous list chunk x (neighbouring
// senders share an L2, as with xcd_map) and its workgroups stride through the chunk.
struct ListRange {
  uint32_t k, end, step;
};
__device__ inline ListRange list_range(uint32_t na) {
  const uint32_t x = blockIdx.x & 7u, per = (na + 7u) >> 3;
  const uint32_t lo = min(na, x * per), hi = min(na, lo + per);
  return ListRange{lo + (blockIdx.x >> 3), hi, gridDim.x >> 3};
}
// dense layout: the grid has at least one workgroup per list entry (gridDim >= 8 * ceil(na / 8)),
// so a workgroup takes one entry or none -- no loop, whose loop-carried state would cost
// registers in these 128-VGPR kernels
__device__ inline bool list_one(uint32_t na, uint32_t& k) {
  const ListRange lr = list_range(na);
  k = lr.k;
  return lr.k < lr.end;
}

// pending-op list of gnode g: nodes < n_heavy of every replica have cap_ops entries,
// the others cap_ops_light (n_heavy = N: uniform)
__device__ inline size_t op_base(const KP& p, uint32_t g) {
  const uint32_t rep = g / p.N, i = g % p.N;
  const size_t per = static_cast<size_t>(p.n_heavy) * p.cap_ops + static_cast<size_t>(p.N - p.n_heavy) * p.cap_ops_light;
  return rep * per + (i < p.n_heavy ? static_cast<size_t>(i) * p.cap_ops
                                    : static_cast<size_t>(p.n_heavy) * p.cap_ops +
                                          static_cast<size_t>(i - p.n_heavy) * p.cap_ops_light);
}
__device__ inline uint32_t op_cap(const KP& p, uint32_t g) { return (g % p.N) < p.n_heavy ? p.cap_ops : p.cap_ops_light; }

// link-state word of out-edge le of node i (replica rep).  Hub-compact (sparse mode,
// full mesh): rows of the hub nodes in full, then (node, hub) pairs; an edge between
// two non-hubs has no state (BCSIM_E_UNSUPPORTED if it ever carries traffic).
__device__ inline size_t link_index(const KP& p, uint32_t rep, uint32_t i, uint32_t e0, uint32_t le) {
  if (!p.hubs) return edge_loc(p, rep, e0 + le);
  const size_t per = static_cast<size_t>(p.hubs) * (p.N - 1) + static_cast<size_t>(p.N - p.hubs) * p.hubs;
  if (i < p.hubs) return rep * per + static_cast<size_t>(i) * (p.N - 1) + le;
  const uint32_t j = le < i ? le : le + 1;  // full mesh peer
  if (j >= p.hubs) {
    set_err(p, BCSIM_E_UNSUPPORTED);
    return rep * per;
  }
  return rep * per + static_cast<size_t>(p.hubs) * (p.N - 1) + static_cast<size_t>(i - p.hubs) * p.hubs + j;
}

struct Key {
  int64_t t, ts;
  uint32_t origin, sub;
};
// d = c ? s : d word by word through an opaque lane mask: the scan loop's choice of the next
// event among arrival / timers / start / stop, written as struct assignments, was miscompiled
// once the global-address accesses changed the schedule (a timer's t and ts with an arrival's
// origin and sub: raft64_fixed), as RawOp selects were before (raw_sel)
__device__ inline void key_sel(Key& d, const Key& s, bool c) {
  uint32_t m = 0u - static_cast<uint32_t>(c);
  asm volatile("" : "+v"(m));
  const uint64_t m2 = (static_cast<uint64_t>(m) << 32) | m;
  d.t = static_cast<int64_t>((static_cast<uint64_t>(s.t) & m2) | (static_cast<uint64_t>(d.t) & ~m2));
  d.ts = static_cast<int64_t>((static_cast<uint64_t>(s.ts) & m2) | (static_cast<uint64_t>(d.ts) & ~m2));
  d.origin = (s.origin & m) | (d.origin & ~m);
  d.sub = (s.sub & m) | (d.sub & ~m);
}
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
// ROCm 7.2 compiler in divergent code, so there is no branch.
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
__device__ inline Msg rec_msg(const Rec& r) {
  Msg m;
  m.type = r.type;
  m.f[0] = r.f0;
  m.f[1] = r.f1;
  m.f[2] = r.f2;
  m.big = (r.flags & RF_BIG) ? 1 : 0;
  return m;
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

// Contended device atomics on one word serialise in L2: every workgroup of a
// launch adds its block-reduced counters to its own stripe instead, summed on the host.
__device__ inline unsigned long long* cnt_stripe(const KP& p, uint32_t rep) {
  const size_t stripe = blockIdx.x & (p.cnt_stripes - 1);
  return &AT(p.counters, (stripe * p.R + rep) * CNT_N, static_cast<uint64_t>(p.cnt_stripes) * p.R * CNT_N);
}
__device__ inline unsigned long long* kst_stripe(const KP& p) { return p.kstat + 8 * (blockIdx.x & (kKstStripes - 1)); }
// bucket_cnt is only tested for nonzero: workgroups set it once instead of all adding to it
__device__ inline void mark_busy(uint32_t* w) {
  if (__hip_atomic_load(gbl(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
    __hip_atomic_store(gbl(w), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// trace record at a reserved position (emit_trace reserves one; gossip reserves a window's worth)
__device__ inline void put_trace(const KP& p, uint32_t pos, const Key& k, uint32_t rep, uint32_t node, uint32_t kind,
                                 int32_t a, int32_t b, int32_t c) {
  if (pos >= p.cap_trace) {
    set_err(p, BCSIM_E_OVERFLOW);
    return;
  }
  bcsim_trace_rec r;
  r.t_ns = k.t;
  r.key_ts = k.ts;
  r.key_origin = k.origin;
  r.key_sub = k.sub;
  r.replica = rep;
  r.node = node;
  r.kind = kind;
  r.a = a;
  r.b = b;
  r.c = c;
  AT(p.trace, pos, p.cap_trace) = r;
}

__device__ inline void emit_trace(const KP& p, const Key& k, uint32_t rep, uint32_t node, uint32_t kind,
                                  int32_t a, int32_t b, int32_t c) {
  put_trace(p, gadd_r(p.trace_cnt, 1u), k, rep, node, kind, a, b, c);
}

__device__ inline void emit_vlog(const KP& p, const Key& k, uint32_t rep, uint32_t node, int32_t v) {
  const uint32_t pos = gadd_r(p.vlog_cnt, 1u);
  if (pos >= p.cap_vlog) {
    set_err(p, BCSIM_E_OVERFLOW);
    return;
  }
  VLog e;
  e.t = k.t;
  e.ts = k.ts;
  e.origin = k.origin;
  e.sub = k.sub;
  e.target = node;
  e.rep = rep;
  e.v = v;
  e.pad = 0;
  AT(p.vlog, pos, p.cap_vlog) = e;
}


// one 16-byte memory access per record (the compiler otherwise splits the
// mixed-width struct into byte / short / dwordx3 pieces)
__device__ inline Rec ld_rec(const Rec* p) {
  const uint4 v = gld4(p);
  Rec r;
  __builtin_memcpy(&r, &v, sizeof r);
  return r;
}
__device__ inline void st_rec(Rec* p, const Rec& r) {
  uint4 v;
  __builtin_memcpy(&v, &r, sizeof v);
  gst4(p, v);
}
__device__ inline void clr_rec(Rec* p) { gst4(p, make_uint4(0, 0, 0, 0)); }
// Inbox-slot records carry a ring-turn tag in flags bits 3-7: (arrival cell / B) mod 32.  A slot
// is live for cell c only with the tag of c, so a delivered record needs no clear: it goes stale
// when the bucket comes round again, and the host zeroes a bucket once every 32 turns
// (bcsim_capi.hip run()) before a tag can repeat.
__device__ inline uint32_t cell_tag(const KP& p, long long cell) {
  return static_cast<uint32_t>((cell / p.n_buckets) & 31);
}
__device__ inline bool slot_live(uint32_t flags, uint32_t tag) {
  return (flags & RF_VALID) && ((flags >> 3) & 31u) == tag;
}
// summary entry / explicit-slot byte of (bucket b, replica rep, receiver tile rt, sender s):
// receiver-tile-major, so that a receiver tile's entries of consecutive senders are contiguous
__device__ inline size_t sum_idx(const KP& p, uint32_t b, uint32_t rep, uint32_t rt, uint32_t s) {
  return ((static_cast<size_t>(b) * p.R + rep) * p.n_tiles + rt) * p.N + s;
}
// a physical slot record of edge s -> d (record word w3: its ring-turn tag) in bucket b
__device__ inline void xs_mark(const KP& p, uint32_t b, uint32_t rep, uint32_t s, uint32_t d, uint32_t w3) {
  if (p.sum) gbl(p.xsum)[sum_idx(p, b, rep, d >> 6, s)] = static_cast<uint8_t>(0x80u | (w3 >> 27));
}
// the tag of a record emitted in cell `cell` for cell + rel (1 <= rel < B), without a division:
// cq = cell / B, cr = cell % B
__device__ inline uint32_t emit_tag(long long cq, uint32_t cr, long long rel, uint32_t B) {
  return static_cast<uint32_t>((cq + ((cr + rel) >= B ? 1 : 0)) & 31);
}

// 32-byte ops as two dwordx4 accesses
__device__ inline Op ld_op(const Op* q) {
  const uint4* v = reinterpret_cast<const uint4*>(q);
  const uint4 a = gld4(v), b = gld4(v + 1);
  Op o;
  __builtin_memcpy(&o, &a, 16);
  __builtin_memcpy(reinterpret_cast<char*>(&o) + 16, &b, 16);
  return o;
}
__device__ inline void st_op(Op* q, const Op& o) {
  uint4 a, b;
  __builtin_memcpy(&a, &o, 16);
  __builtin_memcpy(&b, reinterpret_cast<const char*>(&o) + 16, 16);
  uint4* v = reinterpret_cast<uint4*>(q);
  gst4(v, a);
  gst4(v + 1, b);
}
// (the LDS copies of ops: plain pointers -- ld_op / st_op / ld_raw are for global memory only)
__device__ inline void st_op_lds(Op* q, const Op& o) {
  uint4 a, b;
  __builtin_memcpy(&a, &o, 16);
  __builtin_memcpy(&b, reinterpret_cast<const char*>(&o) + 16, 16);
  uint4* v = reinterpret_cast<uint4*>(q);
  v[0] = a;
  v[1] = b;
}

// An Op as its two raw dwordx4 words: a = {t lo, t hi, dt, origin}, b = {sub, edge,
// f0 | f1 << 16, f2 | type << 16 | kind_flags << 24} (the Op layout above).
struct RawOp {
  uint4 a, b;
};
// d = c ? s : d, word by word through an opaque lane mask: a plain select of RawOp values between
// several op sources in divergent code was miscompiled again in the FQCODEL edge loop (a record
// took its first 16 bytes from one source and the rest from another)
__device__ inline void raw_sel(RawOp& d, const RawOp& s, bool c) {
  uint32_t m = 0u - static_cast<uint32_t>(c);
  asm volatile("" : "+v"(m));
  d.a.x = (s.a.x & m) | (d.a.x & ~m);
  d.a.y = (s.a.y & m) | (d.a.y & ~m);
  d.a.z = (s.a.z & m) | (d.a.z & ~m);
  d.a.w = (s.a.w & m) | (d.a.w & ~m);
  d.b.x = (s.b.x & m) | (d.b.x & ~m);
  d.b.y = (s.b.y & m) | (d.b.y & ~m);
  d.b.z = (s.b.z & m) | (d.b.z & ~m);
  d.b.w = (s.b.w & m) | (d.b.w & ~m);
}
__device__ inline RawOp raw_zero() { return RawOp{make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)}; }
__device__ inline RawOp ld_raw(const Op* q) {
  const uint4* v = reinterpret_cast<const uint4*>(q);
  return RawOp{gld4(v), gld4(v + 1)};
}
__device__ inline RawOp ld_raw_lds(const Op* q) {
  const uint4* v = reinterpret_cast<const uint4*>(q);
  return RawOp{v[0], v[1]};
}
__device__ inline int64_t raw_t(const RawOp& o) {
  return static_cast<int64_t>((static_cast<uint64_t>(o.a.y) << 32) | o.a.x);
}
__device__ inline uint32_t raw_dt(const RawOp& o) { return o.a.z; }
__device__ inline uint32_t raw_origin(const RawOp& o) { return o.a.w; }
__device__ inline uint32_t raw_sub(const RawOp& o) { return o.b.x; }
__device__ inline uint32_t raw_kind(const RawOp& o) { return (o.b.w >> 24) & 3u; }
__device__ inline uint32_t raw_flags(const RawOp& o) { return o.b.w >> 26; }
__device__ inline RawOp raw_make(int64_t t, uint32_t dt, uint32_t origin, uint32_t sub, uint8_t kind_flags) {
  const uint64_t ut = static_cast<uint64_t>(t);
  return RawOp{make_uint4(static_cast<uint32_t>(ut), static_cast<uint32_t>(ut >> 32), dt, origin),
               make_uint4(sub, 0, 0, static_cast<uint32_t>(kind_flags) << 24)};
}
// canonical key order of two ops (t, t - dt, origin, sub): see op_key_less
__device__ inline bool raw_key_less(const RawOp& a, uint32_t sa, const RawOp& b, uint32_t sb) {
  const int64_t ta = raw_t(a), tb = raw_t(b);
  if (ta != tb) return ta < tb;
  const int64_t tsa = ta - raw_dt(a), tsb = tb - raw_dt(b);
  if (tsa != tsb) return tsa < tsb;
  if (raw_origin(a) != raw_origin(b)) return raw_origin(a) < raw_origin(b);
  return sa < sb;
}
static_assert(offsetof(Op, sub) == 16 && offsetof(Op, f0) == 24 && offsetof(Op, kind_flags) == 31, "RawOp layout");

// per-edge op slots
constexpr uint32_t kOpRing = 4;
__device__ inline uint4* eslot_at(const KP& p, uint32_t ob, uint32_t rep, uint32_t e) {
  return &AT(p.eslot, (static_cast<size_t>(ob) * p.R + rep) * p.E_loc + (e - p.e_lo), p.cap_eslot);
}
constexpr uint32_t kPbPrepareRes = 5;  // PBFT PREPARE_RES (pbft-node.h:80-91), the only slot reply
// the full op of a reply slot: SEND at the stored due time, dt = app delay, origin =
// this node, payload (v, n, intToChar(0)) of a PREPARE_RES
__device__ inline RawOp slot_op(const KP& p, const uint4 w, uint32_t i, uint32_t e) {
  const uint32_t f2 = static_cast<uint32_t>(static_cast<uint16_t>(enc_raw(p, 0)));
  return RawOp{make_uint4(w.x, w.y, static_cast<uint32_t>(p.app_delay), i),
               make_uint4(w.z, e, w.w, f2 | (kPbPrepareRes << 16) | (static_cast<uint32_t>(OP_SEND) << 24))};
}

// threadIdx.x behind an empty volatile asm: values derived from it (lane, wave, loop bounds
// and trip counts of the strided loops) are recomputed in each phase instead of being hoisted
// by loop-invariant code motion into registers live across the whole kernel -- in the
// 128-VGPR kernels those were spilled to scratch and reloaded by every lane
__device__ inline uint32_t tidx() {
  uint32_t t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// ---- block-wide primitives (blockDim.x a multiple of 64, <= 1024) ----------
constexpr int kMaxWaves = 16;

// Ordered compaction rank: exclusive position of this thread's flag among
// the block's set flags in thread order; `total` = number of set flags.
__device__ inline uint32_t block_rank(bool f, uint32_t* wcnt, uint32_t& total) {
  const uint32_t lane = tidx() & 63u, w = tidx() >> 6, nw = blockDim.x >> 6;
  const unsigned long long m = __ballot(f);
  const uint32_t below = static_cast<uint32_t>(__popcll(m & ((1ull << lane) - 1ull)));
  if (lane == 0) wcnt[w] = static_cast<uint32_t>(__popcll(m));
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (uint32_t k = 0; k < nw; ++k) {
    const uint32_t c = wcnt[k];
    if (k < w) off += c;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return off + below;
}

// Append one element to a global list (k_rebin: few records per launch).
__device__ inline uint32_t list_append(uint32_t* counter) { return atomicAdd(counter, 1u); }

// Exclusive block scan of four u32 lanes at once; totals in `tot`.
__device__ inline uint4 block_scan4(uint4 v, uint4* wsum, uint4& tot) {
  const uint32_t lane = tidx() & 63u, w = tidx() >> 6, nw = blockDim.x >> 6;
  uint4 x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t a = __shfl_up(x.x, off, 64), b = __shfl_up(x.y, off, 64);
    const uint32_t c = __shfl_up(x.z, off, 64), d = __shfl_up(x.w, off, 64);
    if (lane >= static_cast<uint32_t>(off)) {
      x.x += a;
      x.y += b;
      x.z += c;
      x.w += d;
    }
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint4 base = make_uint4(0, 0, 0, 0), t = make_uint4(0, 0, 0, 0);
  for (uint32_t k = 0; k < nw; ++k) {
    const uint4 s = wsum[k];
    if (k < w) {
      base.x += s.x;
      base.y += s.y;
      base.z += s.z;
      base.w += s.w;
    }
    t.x += s.x;
    t.y += s.y;
    t.z += s.z;
    t.w += s.w;
  }
  __syncthreads();
  tot = t;
  return make_uint4(base.x + x.x - v.x, base.y + x.y - v.y, base.z + x.z - v.z, base.w + x.w - v.w);
}

// In-place exclusive scan of a[0..n) (LDS) with contiguous per-thread runs;
// returns the total.  All threads must call it.
__device__ inline uint32_t block_scan_array(uint32_t* a, uint32_t n, uint4* wsum) {
  const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
  const uint32_t b0 = min(n, tidx() * per), b1 = min(n, b0 + per);
  uint32_t s = 0;
  for (uint32_t k = b0; k < b1; ++k) s += a[k];
  uint4 tot;
  const uint4 ex = block_scan4(make_uint4(s, 0, 0, 0), wsum, tot);
  uint32_t acc = ex.x;
  for (uint32_t k = b0; k < b1; ++k) {
    const uint32_t v = a[k];
    a[k] = acc;
    acc += v;
  }
  __syncthreads();
  return tot.x;
}

// Sum of v over the wave (all lanes get it).
__device__ inline uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Add `inc` to lds[key] once per distinct key of the wave (wave-aggregated
// LDS atomics; all lanes of the wave must call it).
__device__ inline void wave_add_by_key(bool act, uint32_t key, uint32_t inc, unsigned long long* lds) {
  unsigned long long rem = __ballot(act);
  const uint32_t lane = tidx() & 63u;
  while (rem) {
    const int ld = __ffsll(static_cast<long long>(rem)) - 1;
    const uint32_t kl = __shfl(key, ld, 64);
    const bool mine = act && key == kl;
    const unsigned long long same = __ballot(mine);
    unsigned long long sum = 0;
    // sum of inc over `same` lanes
    uint32_t v = mine ? inc : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    sum = v;
    if (lane == static_cast<uint32_t>(ld)) atomicAdd(&lds[kl], sum);
    rem &= ~same;
  }
}

// ---------------------------------------------------------------------------
// extras grouping: counting sort of the cell's extras by receiver gnode
// Group the cell's extras by receiver: counts, then placement.  The records of one receiver
// arrive in runs (the leader's cell: ~N of them for one node), so the per-receiver atomics are
// wave-aggregated -- one atomic per (wave, receiver) instead of one per record, which
// serialised ~4 k same-address atomics (~50 us) per kernel.
__global__ void k_xcount(const KP* __restrict__ pk, uint32_t b, uint32_t n) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  const uint32_t k = blockIdx.x * blockDim.x + tidx(), lane = tidx() & 63u;
  const bool v = k < n;
  const uint32_t g = v ? AT(p.xbuf, static_cast<size_t>(b) * p.cap_x + k, p.cap_xbuf).g : 0u;
  unsigned long long rem = __ballot(v);
  while (rem) {
    const int ld = __ffsll(static_cast<long long>(rem)) - 1;
    const uint32_t gl = __shfl(g, ld, 64);
    const unsigned long long same = __ballot(v && g == gl);
    if (lane == static_cast<uint32_t>(ld)) __hip_atomic_fetch_add(&AT(p.seg_cnt, gl, p.NT), static_cast<uint32_t>(__popcll(same)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    rem &= ~same;
  }
}

// single-block exclusive scan of seg_cnt[0..NT) -> seg_off[0..NT]
__global__ __launch_bounds__(1024) void k_offsets(const KP* __restrict__ pk) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  const uint32_t tid = tidx(), lane = tid & 63, w = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < p.NT; base += 1024) {
    const uint32_t idx = base + tid;
    const uint32_t v = idx < p.NT ? AT(p.seg_cnt, idx, p.NT) : 0u;
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

// multi-block exclusive scan of seg_cnt[0..NT) -> seg_off[0..NT] (large NT: sparse mode)
constexpr uint32_t kSegChunk = 8192;  // 1024 threads x 8 entries per block
__global__ __launch_bounds__(1024) void k_seg_sums(const KP* __restrict__ pk, uint32_t* part) {
  const KP& p = *pk;
  __shared__ uint32_t red[1024];
  const size_t b0 = static_cast<size_t>(blockIdx.x) * kSegChunk;
  uint32_t acc = 0;
  for (uint32_t k = tidx(); k < kSegChunk; k += blockDim.x)
    if (b0 + k < p.NT) acc += p.seg_cnt[b0 + k];
  red[tidx()] = acc;
  __syncthreads();
  for (uint32_t o = blockDim.x / 2; o > 0; o >>= 1) {
    if (tidx() < o) red[tidx()] += red[tidx() + o];
    __syncthreads();
  }
  if (tidx() == 0) part[blockIdx.x] = red[0];
}
__global__ __launch_bounds__(1024) void k_seg_top(uint32_t* part, uint32_t nparts) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  const uint32_t tid = tidx(), lane = tid & 63u, w = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nparts; base += 1024) {
    const uint32_t idx = base + tid;
    const uint32_t v = idx < nparts ? part[idx] : 0u;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off, 64);
      if (lane >= static_cast<uint32_t>(off)) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (tid == 0) {
      uint32_t a = 0;
      for (int k = 0; k < 16; ++k) {
        const uint32_t t = wsum[k];
        wsum[k] = a;
        a += t;
      }
    }
    __syncthreads();
    const uint32_t excl = carry + wsum[w] + x - v;
    if (idx < nparts) part[idx] = excl;
    __syncthreads();
    if (tid == 1023) carry = excl + v;
    __syncthreads();
  }
}
__global__ __launch_bounds__(1024) void k_seg_apply(const KP* __restrict__ pk, const uint32_t* part) {
  const KP& p = *pk;
  __shared__ uint32_t wsum[16];
  const uint32_t tid = tidx(), lane = tid & 63u, w = tid >> 6;
  const size_t b0 = static_cast<size_t>(blockIdx.x) * kSegChunk + static_cast<size_t>(tid) * 8;
  uint32_t v[8], sum = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] = b0 + k < p.NT ? p.seg_cnt[b0 + k] : 0u;
    sum += v[k];
  }
  uint32_t x = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= static_cast<uint32_t>(off)) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t wb = 0;
  for (uint32_t k = 0; k < w; ++k) wb += wsum[k];
  uint32_t acc = part[blockIdx.x] + wb + x - sum;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (b0 + k < p.NT) p.seg_off[b0 + k] = acc;
    acc += v[k];
  }
  if (b0 < p.NT && b0 + 8 >= p.NT) p.seg_off[p.NT] = acc;  // the thread holding the last entry
}

__global__ void k_xplace(const KP* __restrict__ pk, uint32_t b, uint32_t n) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  const uint32_t k = blockIdx.x * blockDim.x + tidx(), lane = tidx() & 63u;
  const bool v = k < n;
  XRec x{};
  if (v) x = AT(p.xbuf, static_cast<size_t>(b) * p.cap_x + k, p.cap_xbuf);
  // the wave's receiver groups first (register work only), then every group's leader takes its
  // range at once: the atomics' round trips overlap instead of following one another (a
  // broadcast's records are 64 different receivers per wave)
  unsigned long long rem = __ballot(v), mine = 0;
  uint32_t leader = lane;
  while (rem) {
    const int ld = __ffsll(static_cast<long long>(rem)) - 1;
    const uint32_t gl = __shfl(x.g, ld, 64);
    const unsigned long long same = __ballot(v && x.g == gl);
    if (v && x.g == gl) {
      leader = static_cast<uint32_t>(ld);
      mine = same;
    }
    rem &= ~same;
  }
  uint32_t base = 0;
  if (v && leader == lane)
    base = AT(p.seg_off, x.g, p.NT + 1) + __hip_atomic_fetch_add(&AT(p.cursor, x.g, p.NT), static_cast<uint32_t>(__popcll(mine)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  base = __shfl(base, leader, 64);
  if (v) AT(p.xgrp, base + static_cast<uint32_t>(__popcll(mine & ((1ull << lane) - 1ull))), p.cap_x) = x;
}

// one overflow record: into its bucket if its cell entered the ring, else `stay` = its cell
// (lbm / lb: the workgroup's per-bucket minimum arrival time and busy flags in LDS, flushed once
// per workgroup -- a leader's block of 4095 overflow records lowered one bucket's bmin and set its
// count word 4095 times: same-address atomics serialised in L2, ~50 us per k_rebin)
// (xb / xrk / xo: a second record of its edge -- the extras list of bucket xb at workgroup rank
// xrk, written by k_rebin once the workgroup's ranks have one base per bucket: a block's 4095
// records appended to one bucket's list one atomic each serialised in L2)
__device__ inline void rebin_one(const KP& p, long long g_cur, XRec& o, long long& stay, long long* lbm, uint32_t* lb,
                                 uint32_t* lx, int& xb, uint32_t& xrk, XRec& xo) {
  if (o.cell < 0) return;
  if (o.cell < g_cur + static_cast<long long>(p.n_buckets)) {
    const uint32_t b = static_cast<uint32_t>(o.cell % p.n_buckets);
    const uint32_t rep = o.g / p.N;
    XRec x = o;
    const bool owner = (x.r.flags & RF_OWNER) != 0;
    x.r.flags = static_cast<uint8_t>((x.r.flags & (RF_VALID | RF_BIG)) | (cell_tag(p, o.cell) << 3));
    if (owner) {
      st_rec(&AT(p.inbox, inbox_idx(p, b, rep, x.slot), p.cap_inbox), x.r);
      if (p.sum) {  // (summaries: full mesh, in-slot k of receiver d holds sender k < d ? k : k + 1)
        const uint32_t d = x.g % p.N, k = x.slot - d * (p.N - 1);
        xs_mark(p, b, rep, k < d ? k : k + 1, d, static_cast<uint32_t>(x.r.flags) << 24);
      }
    } else {
      xb = static_cast<int>(b);
      xrk = atomicAdd(&lx[b], 1u);
      xo = x;
    }
    AT(p.iflag, static_cast<size_t>(b) * p.NT + x.g, static_cast<uint64_t>(p.n_buckets) * p.NT) = 1;
    atomicMin(&lbm[b], o.cell * p.L + static_cast<long long>(x.r.t_off));
    lb[b] = 1u;
    o.cell = -1;
  } else {
    stay = o.cell;
  }
}

// move far-future arrivals whose cell entered the ring into their bucket.
// The overflow horizon of the records that stay is reduced per workgroup (one atomicMin
// each): a saturated PBFT leader keeps tens of thousands of PRE_PREPAREs in the list and a
// same-address atomic per record took 0.3-0.5 ms per launch.
__device__ inline void ctl_publish(const KP& p, long long s0, long long s3, uint32_t seq, const long long* pv = nullptr);

// seq != 0 (host-mapped control mirror): the launch leaves the overflow bound itself -- the last
// workgroup stores the staying records' minimum as scal[1] (no host reset before the launch),
// empties the list when nothing stays, and publishes the control block (bucket counts, scal[1])
// with seq, so that group_cell reads it with one spin instead of copies and a stream sync.
__global__ __launch_bounds__(256) void k_rebin(const KP* __restrict__ pk, long long g_cur, uint32_t n, uint32_t seq) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ long long wmin[4];
  __shared__ long long lbm[kMaxBuckets];
  __shared__ uint32_t lb[kMaxBuckets], lx[kMaxBuckets], lxb[kMaxBuckets];
  const uint32_t B = p.n_buckets;
  for (uint32_t q = tidx(); q < B; q += blockDim.x) {
    lbm[q] = LLONG_MAX;
    lb[q] = 0;
    lx[q] = 0;
  }
  __syncthreads();
  const uint32_t k = blockIdx.x * blockDim.x + tidx();
  long long stay = LLONG_MAX;
  int xb = -1;
  uint32_t xrk = 0;
  XRec xo{};
  if (k < n) rebin_one(p, g_cur, AT(p.ov, k, p.cap_ov), stay, lbm, lb, lx, xb, xrk, xo);
  if (seq && p.ov_tmp) {  // (compaction: the staying records to ov_tmp, one atomic per workgroup)
    __shared__ uint32_t cw[4], cbase;
    const bool st = stay != LLONG_MAX;
    const unsigned long long m = __ballot(st);
    const uint32_t lane = tidx() & 63u, wv = tidx() >> 6;
    if (lane == 0) cw[wv] = static_cast<uint32_t>(__popcll(m));
    __syncthreads();
    if (tidx() == 0) {
      uint32_t t = 0;
      for (uint32_t q = 0; q < (blockDim.x >> 6); ++q) {
        const uint32_t c = cw[q];
        cw[q] = t;
        t += c;
      }
      cbase = t ? gadd_r(&p.rb_n[0], t) : 0u;
    }
    __syncthreads();
    if (st) {
      const uint32_t pos = cbase + cw[wv] + static_cast<uint32_t>(__popcll(m & ((1ull << lane) - 1ull)));
      if (pos < p.cap_ov)
        AT(p.ov_tmp, pos, p.cap_ov) = AT(p.ov, k, p.cap_ov);
      else
        set_err(p, BCSIM_E_OVERFLOW);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const long long y = __shfl_xor(stay, off, 64);
    stay = y < stay ? y : stay;
  }
  if ((tidx() & 63u) == 0) wmin[tidx() >> 6] = stay;
  __syncthreads();
  for (uint32_t q = tidx(); q < B; q += blockDim.x) {
    if (lb[q]) {
      bmin_lower(p, q, lbm[q]);
      mark_busy(&p.bucket_cnt[q]);
    }
    if (lx[q]) lxb[q] = atomicAdd(&p.x_cnt[q], lx[q]);
  }
  __syncthreads();
  if (xb >= 0) {  // (the workgroup's extras: one list atomic per bucket above)
    const uint32_t pos = lxb[xb] + xrk;
    if (pos >= p.cap_x)
      set_err(p, BCSIM_E_OVERFLOW);
    else
      AT(p.xbuf, static_cast<size_t>(xb) * p.cap_x + pos, p.cap_xbuf) = xo;
  }
  if (!seq) {
    if (tidx() == 0) {
      long long m = wmin[0];
      for (uint32_t w = 1; w < (blockDim.x >> 6); ++w) m = wmin[w] < m ? wmin[w] : m;
      if (m != LLONG_MAX) gmin(&p.scal[1], m);
    }
    return;
  }
  __shared__ int s_last;
  if (tidx() == 0) {
    long long m = wmin[0];
    for (uint32_t w = 1; w < (blockDim.x >> 6); ++w) m = wmin[w] < m ? wmin[w] : m;
    if (m != LLONG_MAX) gmin(p.rb_acc, m);
    __threadfence();
    s_last = gadd_r(p.rb_done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  if (tidx() == 0) {
    const long long m = __hip_atomic_load(p.rb_acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    p.scal[1] = m;
    if (p.ov_tmp) {  // (the list is the staying records now: k_ov_back copies them to its front)
      const uint32_t ns = __hip_atomic_load(&p.rb_n[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *p.ov_cnt = ns;
      p.rb_n[1] = ns;
      __hip_atomic_store(&p.rb_n[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (m == LLONG_MAX) {
      *p.ov_cnt = 0;  // (everything rebinned: the list starts again)
    }
    __hip_atomic_store(p.rb_acc, LLONG_MAX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p.rb_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
  }
  __syncthreads();
  if (tidx() < 64) ctl_publish(p, p.scal[0], p.scal[3], seq);
}

// the compacted overflow list back to the front of the list (after a publishing k_rebin)
__global__ __launch_bounds__(256) void k_ov_back(const KP* __restrict__ pk) {
  const KP& p = *pk;
  const uint32_t n = p.rb_n[1];
  for (uint32_t k = blockIdx.x * blockDim.x + tidx(); k < n; k += gridDim.x * blockDim.x)
    AT(p.ov, k, p.cap_ov) = AT(p.ov_tmp, k, p.cap_ov);
}

// ---------------------------------------------------------------------------
// per-node serial protocol context (Raft / Paxos: lane 0 of the node's workgroup)
struct Ctx {
  const KP* p;
  uint32_t g, rep, i, deg;
  Key cur;  // key of the executing event
  uint32_t sub;
  uint64_t draws;
  Op* ops;
  uint32_t nops, cap_ops;
  TimerEnt* tm;  // LDS copy of the node's timers
  uint32_t cap_t;
  unsigned long long echoes, wrong, events;
};

__device__ inline void ctx_trace(Ctx& c, uint32_t kind, int32_t a, int32_t b, int32_t cc) {
  TRAIL(c);
  emit_trace(*c.p, c.cur, c.rep, c.i, kind, a, b, cc);
}

__device__ inline void ctx_op(Ctx& c, const Op& o) {
  const KP& p = *c.p;
  TRAIL(c);
  if (c.nops >= c.cap_ops) {
    set_err(p, BCSIM_E_OVERFLOW);
    return;
  }
  AT(c.ops, c.nops++, c.cap_ops) = o;
}

__device__ inline int32_t ctx_draw(Ctx& c) {
  const KP& p = *c.p;
  if (p.rng_mode == BCSIM_RNG_COUNTER) return ctr_rand(p.seed, c.rep, c.i, c.draws++);
  set_err(p, BCSIM_E_UNSUPPORTED);  // glibc draws inside a cell: unsupported
  return 0;
}

// Simulator::Schedule(Seconds(getRandomDelay()), SendPacket, ...) x peers
__device__ void ctx_bcast(Ctx& c, const Msg& m, bool paxos) {
  const KP& p = *c.p;
  const uint8_t fl = paxos ? OPF_PAXOS : 0;
  if (p.delay_mode == BCSIM_DELAY_FIXED) {
    ctx_op(c, mk_op(p, c.cur.t + p.app_delay, static_cast<uint32_t>(p.app_delay), c.i, c.sub, 0, m,
                    OP_BCAST, fl));
  } else {
    // jitter: expanded per edge by k_link; edge field carries the draw base
    ctx_op(c, mk_op(p, c.cur.t, 0, c.i, c.sub, static_cast<uint32_t>(c.draws), m, OP_BCAST_J, fl));
    c.draws += c.deg;
  }
  c.sub += c.deg;
}

// Send(data, from): reply on the reverse edge of the arrival (= its in-slot)
__device__ void ctx_unicast(Ctx& c, uint32_t out_edge, const Msg& m) {
  const KP& p = *c.p;
  const int64_t d = p.delay_mode == BCSIM_DELAY_FIXED ? p.app_delay : delay_from_draw(p, ctx_draw(c));
  ctx_op(c, mk_op(p, c.cur.t + d, static_cast<uint32_t>(d), c.i, c.sub++, out_edge, m, OP_SEND, 0));
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

// ---------------------------------------------------------------------------
// PBFT message types (pbft-node.h:80-91)
enum { PB_PRE_PREPARE = 1, PB_PREPARE = 2, PB_COMMIT = 3, PB_PREPARE_RES = 5, PB_VIEW_CHANGE = 8 };

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
    const uint32_t pos = gadd_r(p.dreq_cnt, 1u);
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
  int32_t ticket, proposal, vs, vf, decree;
};

// acceptor state of this node for decree d (carried in data[3] = f2 by every Paxos
// message: outside the reference's 3-byte packet, 0 for the single decree)
__device__ inline int32_t* px_of(Ctx& c, int32_t d) {
  const KP& p = *c.p;
  if (d < 0 || static_cast<uint32_t>(d) >= p.K) {
    set_err(p, BCSIM_E_INDEX);
    d = 0;
  }
  return &AT(p.px, (static_cast<size_t>(c.g) * p.K + static_cast<uint32_t>(d)) * 4, static_cast<uint64_t>(p.NT) * p.K * 4);
}

__device__ void paxos_ticket(Ctx& c, PaxosState& s) {  // requireTicket :510-522
  const KP& p = *c.p;
  ++s.ticket;
  ctx_bcast(c, mkmsg(PX_REQ_TICKET, enc_raw(p, s.ticket), 0, s.decree, 0), true);
  ctx_trace(c, BCSIM_TR_PAXOS_TICKET, s.ticket, s.decree, 0);
}

__device__ void paxos_recv(Ctx& c, PaxosState& s, const Msg& m, uint32_t back_edge) {
  const KP& p = *c.p;
  const int32_t N = static_cast<int32_t>(p.N);
  const int32_t ty = c2i(mch(m, 0));
  switch (ty) {
    case PX_REQ_TICKET: {  // :177-198
      const int32_t t = c2i(mch(m, 1));
      int32_t* a = px_of(c, m.f[2]);
      Msg r;
      if (t > a[0]) {
        a[0] = t;
        r = mkmsg(PX_RES_TICKET, enc_raw(p, 0), a[1], m.f[2], 0);
      } else {
        r = mkmsg(PX_RES_TICKET, enc_raw(p, 1), 0, m.f[2], 0);
      }
      ctx_unicast(c, back_edge, r);
      break;
    }
    case PX_REQ_PROPOSE: {  // :199-221
      const int32_t t = c2i(mch(m, 1));
      int32_t* a = px_of(c, m.f[2]);
      int32_t st = 1;
      if (t == a[0]) {
        a[1] = mch(m, 2);
        a[2] = t;
        st = 0;
      }
      ctx_unicast(c, back_edge, mkmsg(PX_RES_PROPOSE, enc_raw(p, st), 0, m.f[2], 0));
      break;
    }
    case PX_REQ_COMMIT: {  // :222-247
      const int32_t t = c2i(mch(m, 1));
      const int32_t cc = mch(m, 2);
      int32_t* a = px_of(c, m.f[2]);
      int32_t st = 1;
      if (t == a[2] && cc == a[1]) {
        a[3] = 1;
        st = 0;
      }
      ctx_unicast(c, back_edge, mkmsg(PX_RES_COMMIT, enc_raw(p, st), 0, m.f[2], 0));
      break;
    }
    case PX_RES_TICKET:
    case PX_RES_PROPOSE:
    case PX_RES_COMMIT: {  // :248-353
      if (m.f[2] != s.decree) break;  // a response of a finished decree: not counted
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
            ctx_bcast(c, mkmsg(PX_REQ_PROPOSE, enc_raw(p, s.ticket), s.proposal, s.decree, 0), true);
          } else if (ty == PX_RES_PROPOSE) {
            ctx_bcast(c, mkmsg(PX_REQ_COMMIT, enc_raw(p, s.ticket), s.proposal, s.decree, 0), true);
          } else {
            ctx_trace(c, BCSIM_TR_PAXOS_COMMIT, s.ticket, s.decree, 0);
            if (static_cast<uint32_t>(s.decree) + 1 < p.K) {  // next decree: fresh ticket and proposal
              s.decree += 1;
              s.ticket = 0;
              s.proposal = enc_raw(p, static_cast<int32_t>(c.i));
              paxos_ticket(c, s);
            }
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
// k_scan: one workgroup per node.
//
// The node's arrivals of [t_lo, t_hi) are staged from its inbox row (+ the
// cell's extras) into LDS in slot order = ascending origin.  Sort key per
// arrival: (t_off << 32 | ~dt, slot): t, then t_sched = t - dt ascending,
// then origin — the canonical key (t, t_sched, origin, sub); sub never
// decides between two arrivals at one receiver (one edge cannot deliver
// twice at the same instant).  The common full-mesh case (all arrivals of a
// phase at one instant) is already sorted and skips the LDS bitonic sort.
constexpr int kScanMaxArr = 4096;  // LDS staging window (28 B per arrival)
// staged arrival id (asec): in-slot << kSlotShift | (extras record ? kXBit | index in the node's
// extras segment : 0).  The records themselves are not copied to LDS: a main-slot record is
// read from the node's inbox row (L2-resident after the stage), an extras record from the
// grouped list, so a staged arrival costs 16 B of LDS (key, id, class) and two 512-lane
// workgroups fit a CU at N=4096.
constexpr int kSlotShift = 14;
constexpr uint32_t kXBit = 1u << 13;
constexpr uint32_t kXIdx = kXBit - 1u;
struct RecSrc {
  const Rec* slots;  // the node's inbox row (nullptr in the sparse layout)
  const XRec* xs;    // the node's extras of the cell
};
__device__ inline Rec rec_of(const RecSrc& rs, uint32_t sec) {
  return (sec & kXBit) ? rs.xs[sec & kXIdx].r : ld_rec(rs.slots + (sec >> kSlotShift));
}
__device__ inline bool is_main(uint32_t sec) { return (sec & kXBit) == 0; }
constexpr int kQuorumTab = 256;    // distinct (phase, sequence) pairs per window

// PBFT class word per staged arrival (acls): bits 30-31 class, 29 crossing, 0-28 index
// PBFT class word per staged arrival (acls): bits 30-31 class, 29 crossing, 21-28 message type
// (phases C and D and the delivery counts read it instead of the record), 0-20 sequence index
constexpr uint32_t kClsPres = 1u << 30, kClsCommit = 2u << 30, kCross = 1u << 29;
constexpr int kTypeShift = 21;
constexpr uint32_t kTypeMask = 0xFFu << kTypeShift;
constexpr uint32_t kIdxMask = (1u << kTypeShift) - 1u;
__device__ inline uint32_t cls_type(uint32_t w) { return (w & kTypeMask) >> kTypeShift; }

struct ScanShared {
  uint32_t wcnt[kMaxWaves];
  uint4 wsum[kMaxWaves];
  uint32_t n, n_main, unsorted, cnt;
  uint32_t hsel, hcnt;  // window split: selected bin, arrivals before it
  // PBFT window state
  uint32_t sub, nops, tn, npp, last_vc;
  uint64_t draws;
  int32_t block_num, leader;
  uint32_t tkey[kQuorumTab];   // (phase, sequence) keys, a contiguous prefix (0 = empty)
  uint32_t tcnt[kQuorumTab];
  uint16_t wsc[kMaxWaves][kQuorumTab];  // per-wave counts, then per-wave bases (< 2^16: T + cap_arr)
  uint32_t pp_r[64];
  int32_t pp_idx[64], pp_val[64];
  unsigned long long deliv[BCSIM_MSG_TYPES];
  unsigned long long wrong;
  long long tmax;
  uint32_t ocnt[kOpRing];  // reply-slot ops written, by due cell - cell
  uint32_t tr_n, tr_pos;   // gossip: first receipts of the window, next reserved trace position
  // Paxos proposer window (paxos_window_fast): decree and vote count on entry, verdict, the
  // quorum-crossing arrival and its prefix counts, explicit echoes, per-type deliveries
  int32_t px_dec, px_c0;
  uint32_t px_bad, px_r, px_cb, px_sb, px_eb, px_ncross, px_nops0, px_nx, px_adv, px_sr;
  uint32_t px_deliv[3];
  long long px_tmax;
  unsigned long long ph[8];  // BCSIM_WGT phase clock (debug)
};
#define SPH(k)                                                         \
  do {                                                                 \
    if (p.wgs && tidx() == 0) S.ph[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

__device__ inline int64_t prop_of_slot(const KP& p, uint32_t q) {
  return p.prop_const >= 0 ? p.prop_const : AT(p.prop_in, q, p.E);
}
__device__ inline uint64_t arr_key(const KP& p, const Rec& r, uint32_t q) {
  const uint32_t dt = static_cast<uint32_t>(prop_of_slot(p, q) + sel2(p.tx_last, (r.flags & RF_BIG) ? 1 : 0));
  return (static_cast<uint64_t>(r.t_off) << 32) | static_cast<uint32_t>(~dt);
}

// Stage this node's arrivals with t in [wa, wb): main row first (slot order),
// then extras.  Returns the total count (entries beyond cap are not stored).
__device__ uint32_t stage_window(const KP& p, ScanShared& S, const Rec* slots, uint32_t e0, uint32_t deg,
                                 const XRec* xs, uint32_t xn, long long cs, long long wa, long long wb,
                                 uint64_t* akey, uint32_t* asec, bool store) {
  const uint32_t tid = tidx();
  const uint32_t tag = cell_tag(p, cs / p.L);
  uint32_t n = 0;
  for (uint32_t base = 0; base < deg; base += 4 * blockDim.x) {
    Rec rr[4];
    bool vv[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {  // all loads in flight before the first rank
      const uint32_t k = base + j * blockDim.x + tid;
      rr[j] = k < deg ? ld_rec(slots + k) : Rec{};
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t k = base + j * blockDim.x + tid;
      const long long t = cs + rr[j].t_off;
      vv[j] = k < deg && slot_live(rr[j].flags, tag) && t >= wa && t < wb;
    }
    // one block scan ranks all four chunks: chunk j's records follow chunks < j (slot order)
    uint4 tot;
    const uint4 ex = block_scan4(make_uint4(vv[0], vv[1], vv[2], vv[3]), S.wsum, tot);
    const uint32_t pos4[4] = {n + ex.x, n + tot.x + ex.y, n + tot.x + tot.y + ex.z, n + tot.x + tot.y + tot.z + ex.w};
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t k = base + j * blockDim.x + tid, pos = pos4[j];
      if (store && vv[j] && pos < p.cap_arr) {
        asec[pos] = k << kSlotShift;
        akey[pos] = arr_key(p, rr[j], e0 + k);
      }
    }
    n += tot.x + tot.y + tot.z + tot.w;
  }
  const uint32_t n_main = n;
  for (uint32_t base = 0; base < xn; base += blockDim.x) {
    const uint32_t k = base + tid;
    XRec x{};
    bool v = false;
    if (k < xn) {
      x = xs[k];
      const long long t = cs + x.r.t_off;
      v = t >= wa && t < wb;
    }
    uint32_t tot;
    const uint32_t pos = n + block_rank(v, S.wcnt, tot);
    if (store && v && pos < p.cap_arr) {
      asec[pos] = ((x.slot - e0) << kSlotShift) | kXBit | k;
      akey[pos] = arr_key(p, x.r, x.slot);
    }
    n += tot;
  }
  if (tid == 0) S.n_main = n_main;
  __syncthreads();
  return n;
}

// The end wb of a window starting at wa: the largest wb <= hi with at most cap of the node's
// arrivals in [wa, wb), given more than cap in [wa, hi) (count(wa, wb) is monotone, so this
// is the same bound a binary search over stage_window counts finds).  Radix select over time:
// each pass histograms the arrivals of [lo, hi) into 2^kb-ns bins (LDS atomics into `hist`,
// the not yet used staging area), so ~3 passes over the row replace ~22 counting passes.
__device__ long long window_split(const KP& p, ScanShared& S, const Rec* slots, uint32_t deg, const XRec* xs,
                                  uint32_t xn, long long cs, long long wa, long long hi, uint32_t* hist) {
  const uint32_t tid = tidx(), lane = tid & 63u;
  const uint32_t tag = cell_tag(p, cs / p.L);
  const uint32_t lg = p.cap_arr >= 128 ? 8u : 6u;  // 2^lg bins (<= 2 * cap_arr u32 of staging)
  const uint32_t nb = 1u << lg;
  long long lo = wa;
  uint32_t c_lo = 0;  // arrivals in [wa, lo)
  while (hi - lo > 1) {
    uint32_t sh = 0;
    while ((static_cast<long long>(nb) << sh) < hi - lo) ++sh;
    for (uint32_t k = tid; k < nb; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    for (uint32_t base = 0; base < deg; base += 4 * blockDim.x) {
      Rec rr[4];
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t k = base + j * blockDim.x + tid;
        rr[j] = k < deg ? ld_rec(slots + k) : Rec{};
      }
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t k = base + j * blockDim.x + tid;
        const long long t = cs + rr[j].t_off;
        if (k < deg && slot_live(rr[j].flags, tag) && t >= lo && t < hi)
          atomicAdd(&hist[static_cast<uint32_t>((t - lo) >> sh)], 1u);
      }
    }
    for (uint32_t k = tid; k < xn; k += blockDim.x) {
      const long long t = cs + xs[k].r.t_off;
      if (t >= lo && t < hi) atomicAdd(&hist[static_cast<uint32_t>((t - lo) >> sh)], 1u);
    }
    __syncthreads();
    if (tid < 64) {  // wave 0: boundaries b = 0 .. nb-1 at lo + (b << sh), count c_lo + prefix(b)
      const uint32_t per = nb / 64;
      uint32_t h[4] = {0, 0, 0, 0}, sum = 0;
      for (uint32_t j = 0; j < per; ++j) {
        h[j] = hist[lane * per + j];
        sum += h[j];
      }
      uint32_t inc = sum;
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(inc, d, 64);
        if (lane >= d) inc += v;
      }
      uint32_t c = c_lo + inc - sum, ok = 0;
      for (uint32_t j = 0; j < per; ++j) {
        const uint32_t b = lane * per + j;
        if (c <= p.cap_arr && (static_cast<long long>(b) << sh) < hi - lo) ++ok;  // monotone in b
        c += h[j];
      }
      const uint32_t tot_ok = wave_sum(ok);  // boundaries with count <= cap: 0 .. tot_ok - 1
      const uint32_t best = tot_ok - 1;
      if (lane == best / per) {
        uint32_t cb = c_lo + inc - sum;
        for (uint32_t j = 0; j < best % per; ++j) cb += h[j];
        S.hsel = best;
        S.hcnt = cb;
      }
    }
    __syncthreads();
    const uint32_t best = S.hsel;
    c_lo = S.hcnt;
    const long long nlo = lo + (static_cast<long long>(best) << sh);
    const long long nhi = lo + (static_cast<long long>(best + 1) << sh);
    lo = nlo;
    if (nhi < hi) hi = nhi;
    __syncthreads();  // S.hsel / hist reuse
  }
  return lo;
}

__device__ inline bool sec_less(uint64_t ka, uint32_t sa, uint64_t kb, uint32_t sb) {
  return ka < kb || (ka == kb && sa < sb);
}

// The leader's window (the few-node launches' doubled staging window): its main-slot run
// [0, n_main) is in order -- one instant, in-slot order -- and its extras run is one key (the
// other message of the same edges, so its in-slots are distinct and in-slot order is sec
// order).  Then the two runs are merged by rank instead of the bitonic network: an extra's rank
// among the extras is the count of extras' in-slots below its own (a bitmap of in-slots in LDS
// and prefix counts), a main arrival's rank among the extras is 0, all or that count by key, and
// the rank in the other run of an extra is a binary search of the main run.  The pairs go out
// to the workgroup's area of p.sortbuf at their destination and come back in order -- no
// register staging (k_scan is at its 128-VGPR bound).  false: not this shape, nothing changed.
__device__ bool merge_runs(ScanShared& S, uint32_t n, uint64_t* akey, uint32_t* asec, G<uint4>* mg) {
  const uint32_t tid = tidx(), bs = blockDim.x, n_main = S.n_main;
  if (n_main == 0 || n_main >= n) return false;
  const uint64_t xk = akey[n_main];
  bool bad = false;
  for (uint32_t r = tid; r < n; r += bs) {
    if (r + 1 < n_main && sec_less(akey[r + 1], asec[r + 1], akey[r], asec[r])) bad = true;
    if (r > n_main && akey[r] != xk) bad = true;
    if (r >= n_main && (asec[r] >> kSlotShift) >= 32u * kQuorumTab) bad = true;
  }
  uint32_t* bm = S.tkey;
  for (uint32_t k = tid; k < static_cast<uint32_t>(kQuorumTab); k += bs) bm[k] = 0;
  if (tid == 0) S.hsel = 0;
  __syncthreads();
  if (__ballot(bad) && (tid & 63u) == 0) S.hsel = 1;
  if (!bad)
    for (uint32_t r = n_main + tid; r < n; r += bs) {
      const uint32_t sl = asec[r] >> kSlotShift;
      atomicOr(&bm[sl >> 5], 1u << (sl & 31u));
    }
  __syncthreads();
  if (S.hsel) return false;
  for (uint32_t k = tid; k < static_cast<uint32_t>(kQuorumTab); k += bs) S.tcnt[k] = static_cast<uint32_t>(__popc(bm[k]));
  __syncthreads();
  if (tid == 0) {  // (prefix over 256 words: one lane)
    uint32_t run = 0;
    for (uint32_t k = 0; k < static_cast<uint32_t>(kQuorumTab); ++k) {
      const uint32_t c = S.tcnt[k];
      S.tcnt[k] = run;
      run += c;
    }
    S.hsel = run != n - n_main ? 1u : 0u;  // (in-slots not distinct)
  }
  __syncthreads();
  if (S.hsel) return false;
  const uint32_t nx = n - n_main;
  for (uint32_t r = tid; r < n; r += bs) {
    const uint64_t k = akey[r];
    const uint32_t sc = asec[r], sl = sc >> kSlotShift;
    const uint32_t xr = S.tcnt[sl >> 5] + static_cast<uint32_t>(__popc(bm[sl >> 5] & ((1u << (sl & 31u)) - 1u)));
    uint32_t d;
    if (r < n_main) {
      d = r + (k < xk ? 0u : k > xk ? nx : xr);
    } else {
      uint32_t lo = 0, hi = n_main;  // main arrivals before it
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sec_less(akey[mid], asec[mid], k, sc)) lo = mid + 1;
        else hi = mid;
      }
      d = xr + lo;
    }
    mg[d] = make_uint4(static_cast<uint32_t>(k), static_cast<uint32_t>(k >> 32), sc, 0u);
  }
  __syncthreads();
  for (uint32_t r = tid; r < n; r += bs) {
    const uint4 v = mg[r];
    akey[r] = (static_cast<uint64_t>(v.y) << 32) | v.x;
    asec[r] = v.z;
  }
  __syncthreads();
  return true;
}

// Sort (akey, asec) pairs of [0, n) unless already ordered (mg: the merge area, or null).
__device__ void sort_window(ScanShared& S, uint32_t n, uint64_t* akey, uint32_t* asec, G<uint4>* mg) {
  const uint32_t tid = tidx();
  if (tid == 0) S.unsorted = 0;
  __syncthreads();
  bool bad = false;
  for (uint32_t r = tid; r + 1 < n; r += blockDim.x)
    if (sec_less(akey[r + 1], asec[r + 1], akey[r], asec[r])) bad = true;
  if (__ballot(bad) && (tid & 63) == 0) S.unsorted = 1;
  __syncthreads();
  if (!S.unsorted) return;
  if (mg && merge_runs(S, n, akey, asec, mg)) return;
  uint32_t P2 = 2;
  while (P2 < n) P2 <<= 1;
  for (uint32_t k = n + tid; k < P2; k += blockDim.x) {
    akey[k] = ~0ull;
    asec[k] = ~0u;
  }
  __syncthreads();
  // bitonic network; the stages with j < 64 compare inside aligned 64-element blocks, so each
  // wave runs them over its own blocks without workgroup barriers (78 -> 33 barriers at 4096)
  const uint32_t lane = tid & 63u, wv = tid >> 6, nwv = blockDim.x >> 6;
  const uint32_t blk = P2 < 64u ? P2 : 64u, ppb = blk / 2, nblk = P2 / blk;
  const uint32_t own = nblk > wv ? (nblk - wv + nwv - 1) / nwv : 0u;  // blocks of this wave
  auto ce = [&](uint32_t t, uint32_t j, uint32_t k2) {
    const uint32_t lo = 2 * t - (t & (j - 1)), hi = lo + j;
    const bool up = (lo & k2) == 0;
    const uint64_t ka = akey[lo], kb = akey[hi];
    const uint32_t sa = asec[lo], sb = asec[hi];
    if (up == sec_less(kb, sb, ka, sa)) {
      akey[lo] = kb;
      akey[hi] = ka;
      asec[lo] = sb;
      asec[hi] = sa;
    }
  };
  for (uint32_t k2 = 2; k2 <= P2; k2 <<= 1) {
    uint32_t j = k2 >> 1;
    for (; j >= blk; j >>= 1) {
#pragma unroll 4
      for (uint32_t t = tid; t < P2 / 2; t += blockDim.x) ce(t, j, k2);
      __syncthreads();
    }
    for (; j > 0; j >>= 1) {
#pragma unroll 4
      for (uint32_t u = lane; u < own * ppb; u += 64) {
        const uint32_t b = wv + nwv * (u / ppb);
        ce(b * ppb + u % ppb, j, k2);
      }
      // the wave's LDS writes complete before its next stage reads them
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
  }
}

// Table slot of a (phase, sequence) key: linear probing from 0 with a CAS
// insert, so used slots stay a contiguous prefix.
__device__ inline uint32_t quorum_slot(const KP& p, ScanShared& S, uint32_t key, bool insert) {
  for (uint32_t k = 0; k < static_cast<uint32_t>(kQuorumTab); ++k) {
    const uint32_t t = __hip_atomic_load(&S.tkey[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (t == key) return k;
    if (t == 0u) {
      if (!insert) break;
      const uint32_t old = atomicCAS(&S.tkey[k], 0u, key);
      if (old == 0u || old == key) return k;
    }
  }
  set_err(p, BCSIM_E_OVERFLOW);
  return kQuorumTab - 1;
}

// ---- PBFT, data parallel (pbft-node.cc:166-291) ----------------------------
// One window of sorted arrivals.  Sequential semantics restated as prefixes:
//   PRE_PREPARE   tx[n].val = val; bcast PREPARE          sub += deg
//   PREPARE       reply PREPARE_RES (unicast)             sub += 1
//   PREPARE_RES   ++prepare_vote; crossing (every N/2-th increment) -> bcast COMMIT
//   COMMIT        ++commit_vote; crossing (every (N/2+1)-th) -> commit, block_num++
//   VIEW_CHANGE   leader = msg (last one wins), "Wrong msg"
// Crossings are ranks within each (phase, sequence) group: wave 0 walks the
// window 64 arrivals at a time, grouping lanes by ballot.
__device__ __attribute__((always_inline)) inline void pbft_window(const KP& p, ScanShared& S, uint32_t g, uint32_t rep, uint32_t i, uint32_t e0,
                            uint32_t deg, uint32_t n, uint32_t n_main, long long cell, long long cs, long long t_lo,
                            const uint64_t* akey, const uint32_t* asec, const RecSrc rs, uint32_t* acls) {
  const uint32_t tid = tidx(), lane = tid & 63u;
  const size_t base = static_cast<size_t>(g) * p.pbft_seq_cap;
  const int32_t N = static_cast<int32_t>(p.N);
  const uint32_t T1 = static_cast<uint32_t>(N / 2), T2 = T1 + 1;
  const bool fixed = p.delay_mode == BCSIM_DELAY_FIXED;
  // ---- A: classify ----
  if (tid == 0) {
    S.tn = 0;
    S.npp = 0;
    S.last_vc = 0;
  }
  __syncthreads();
  for (uint32_t r = tid; r < n; r += blockDim.x) {
    const Rec rec = rec_of(rs, asec[r]);
    const Msg m = rec_msg(rec);
    uint32_t w = 0;
    switch (rec.type) {
      case PB_PRE_PREPARE: {
        const int32_t num = c2i(mch(m, 2));
        if (pbft_index(p, num)) {
          const uint32_t k = atomicAdd(&S.npp, 1u);
          if (k < 64) {
            S.pp_r[k] = r;
            S.pp_idx[k] = num;
            S.pp_val[k] = c2i(mch(m, 3));
          } else {
            set_err(p, BCSIM_E_OVERFLOW);
          }
        }
        break;
      }
      case PB_PREPARE_RES: {
        const int32_t idx = c2i(mch(m, 2));
        if (pbft_index(p, idx) && c2i(mch(m, 3)) == 0) w = kClsPres | static_cast<uint32_t>(idx);
        break;
      }
      case PB_COMMIT: {
        const int32_t idx = c2i(mch(m, 2));
        if (pbft_index(p, idx)) w = kClsCommit | static_cast<uint32_t>(idx);
        break;
      }
      case PB_VIEW_CHANGE:
        atomicMax(&S.last_vc, r + 1);
        break;
      default:
        break;
    }
    acls[r] = w | (static_cast<uint32_t>(rec.type) << kTypeShift);
  }
  __syncthreads();
  SPH(3);
  // ---- B: quorum ranks over all waves: each wave counts its contiguous
  // range per (phase, sequence) key; a cross-wave prefix (seeded with the
  // stored vote counters) gives every wave its bases; a second pass ranks
  // each arrival within its key group ----
  {
    const uint32_t nwv = blockDim.x >> 6, wv = tid >> 6;
    for (uint32_t k = tid; k < static_cast<uint32_t>(kQuorumTab); k += blockDim.x) S.tkey[k] = 0;
    for (uint32_t k = tid; k < static_cast<uint32_t>(kMaxWaves * kQuorumTab); k += blockDim.x) (&S.wsc[0][0])[k] = 0;
    __syncthreads();
    const uint32_t per_w = (n + nwv - 1) / nwv;
    const uint32_t rb = min(n, wv * per_w), re = min(n, rb + per_w);
    for (int pass = 0; pass < 2; ++pass) {
      for (uint32_t b0 = rb; b0 < re; b0 += 64) {  // wave-uniform bounds
        const uint32_t r = b0 + lane;
        const uint32_t w = r < re ? (acls[r] & ~kTypeMask) : 0u;  // (phase, sequence) key
        unsigned long long rem = __ballot(w != 0);
        while (rem) {
          const int ld = __ffsll(static_cast<long long>(rem)) - 1;
          const uint32_t wl = __shfl(w, ld, 64);
          const bool mine = (w == wl);
          const unsigned long long same = __ballot(mine);
          uint32_t cnt = 0;
          if (lane == static_cast<uint32_t>(ld)) {
            const uint32_t k = quorum_slot(p, S, wl, pass == 0);
            cnt = S.wsc[wv][k];
            S.wsc[wv][k] = static_cast<uint16_t>(cnt + static_cast<uint32_t>(__popcll(same)));
          }
          if (pass == 1) {
            cnt = __shfl(cnt, ld, 64);
            if (mine) {
              const uint32_t v = cnt + static_cast<uint32_t>(__popcll(same & ((1ull << lane) - 1ull))) + 1u;
              const bool cross = (w >> 30) == 1u ? (v % T1 == 0) : (v % T2 == 0);
              if (cross) acls[r] |= kCross;
            }
          }
          rem &= ~same;
        }
      }
      __syncthreads();
      if (pass == 0) {
        for (uint32_t k = tid; k < static_cast<uint32_t>(kQuorumTab); k += blockDim.x) {
          const uint32_t wl = S.tkey[k];
          if (!wl) continue;
          const uint32_t idx = wl & kIdxMask;
          uint32_t run = static_cast<uint32_t>((wl >> 30) == 1u ? AT(p.tx_pv, base + idx, p.cap_txn)
                                                                : AT(p.tx_cv, base + idx, p.cap_txn));
          for (uint32_t w2 = 0; w2 < nwv; ++w2) {
            const uint32_t c = S.wsc[w2][k];
            S.wsc[w2][k] = static_cast<uint16_t>(run);
            run += c;
          }
          S.tcnt[k] = run;
        }
        __syncthreads();
      }
    }
    // write back the vote counters (tx[idx].prepare_vote / commit_vote)
    for (uint32_t k = tid; k < static_cast<uint32_t>(kQuorumTab); k += blockDim.x) {
      const uint32_t wl = S.tkey[k];
      if (!wl) continue;
      const uint32_t idx = wl & kIdxMask;
      if ((wl >> 30) == 1u)
        AT(p.tx_pv, base + idx, p.cap_txn) = static_cast<int32_t>(S.tcnt[k] % T1);
      else
        AT(p.tx_cv, base + idx, p.cap_txn) = static_cast<int32_t>(S.tcnt[k] % T2);
    }
  }
  __syncthreads();
  SPH(4);
  // ---- C: per-arrival increments over contiguous runs, block scan ----
  const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
  const uint32_t r0 = min(n, tid * per), r1 = min(n, r0 + per);
  const uint32_t ech = p.echo ? 1u : 0u;
  const bool slots = p.eslot != nullptr;
  uint4 loc = make_uint4(0, 0, 0, 0);  // sub, draws, commits, ops
  uint32_t rslot = 0;                   // bit j: reply of arrival r0 + j goes to its edge slot
#pragma nounroll
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t sec = asec[r];
    const uint32_t w = acls[r];
    const uint32_t type = cls_type(w);
    const bool cross = (w & kCross) != 0;
    const bool main_rec = is_main(sec);
    const bool main_slot = slots && main_rec;
    uint32_t si = 0, di = 0, ci = 0, oi = (p.impl && main_rec) ? 0u : ech;
    if (type == PB_PRE_PREPARE) {
      si = deg;
      di = fixed ? 0u : deg;
      oi += 1;
    } else if (type == PB_PREPARE) {
      si = 1;
      di = fixed ? 0u : 1u;
      // the reply of a main-slot arrival owns its edge's slot of this arrival cell
      if (main_slot && fixed && r - r0 < 32)
        rslot |= 1u << (r - r0);
      else
        oi += 1;
    } else if (type == PB_PREPARE_RES && cross) {
      si = deg;
      di = fixed ? 0u : deg;
      oi += 1;
    } else if (type == PB_COMMIT && cross) {
      ci = 1;
    }
    loc.x += si;
    loc.y += di;
    loc.z += ci;
    loc.w += oi;
  }
  uint4 tot;
  const uint4 ex = block_scan4(loc, S.wsum, tot);
  SPH(5);
  // ---- D: outputs ----
  const uint32_t sub0 = S.sub, nops0 = S.nops;
  const uint64_t draws0 = S.draws;
  const int32_t bn0 = S.block_num;
  if (nops0 + tot.w > op_cap(p, g)) {
    if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
    return;
  }
  Op* ops = p.ops + op_base(p, g);
  uint32_t sp = sub0 + ex.x, op = nops0 + ex.w, cp = ex.z;
  uint64_t dp = draws0 + ex.y;
  unsigned long long wrong = 0;
  uint32_t n_slot0 = 0, n_slot1 = 0;  // slot replies due in this cell / the next (app delay < L)
  // the first tick time at or after the window start: an arrival at a tick time is checked
  // against it without a 64-bit division per arrival
  const int64_t tk0 = ((t_lo + p.pbft_period - 1) / p.pbft_period) * p.pbft_period;
  const bool one_tick = p.L < p.pbft_period;  // (windows lie inside one cell)
  // t and dt come from the staged key; the record is read only by arrivals that produce output
  // (the PREPARE_RES / COMMIT waves are almost all non-crossing: nothing to read), one arrival
  // ahead, so its load is in flight while the previous arrival's output is written
  auto needs_rec = [&](uint32_t r) -> bool {
    const uint32_t w = acls[r];
    const uint32_t type = cls_type(w);
    const bool cross = (w & kCross) != 0;
    return (ech && !(p.impl && is_main(asec[r]))) || type == PB_PRE_PREPARE || type == PB_PREPARE ||
           type == PB_VIEW_CHANGE || (cross && (type == PB_PREPARE_RES || type == PB_COMMIT));
  };
  Rec nrec{};
  if (r0 < r1 && needs_rec(r0)) nrec = rec_of(rs, asec[r0]);
#pragma nounroll
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t sec = asec[r];
    const uint32_t q = e0 + (sec >> kSlotShift);  // in-slot = reverse (reply) edge
    const uint32_t w = acls[r];
    const uint32_t type = cls_type(w);
    const bool cross = (w & kCross) != 0;
    const uint64_t kk = akey[r];
    const int64_t t = cs + static_cast<int64_t>(kk >> 32);
    const uint32_t dt = ~static_cast<uint32_t>(kk);
    const bool lecho = ech && !(p.impl && is_main(sec));
    const Rec rec = nrec;  // zero unless needs_rec(r)
    nrec = Rec{};
    if (r + 1 < r1 && needs_rec(r + 1)) nrec = rec_of(rs, asec[r + 1]);
    const Msg m = rec_msg(rec);
    const uint32_t le = q - e0;
    const uint32_t origin = p.mesh ? (le < i ? le : le + 1) : AT(p.col, q, p.E);
    const Key key{t, t - static_cast<int64_t>(dt), origin, rec.sub};
    // (a window is shorter than the period, so tk0 is its only tick time: no 64-bit modulo)
    if (t >= tk0 && (t == tk0 || (!one_tick && (t - tk0) % p.pbft_period == 0)) && key.ts <= t - p.pbft_period)
      set_err(p, BCSIM_E_TIE);  // arrival ordered before a same-time tick
    // pbft-node.cc:175 echo: implicit for main-slot records (k_link), listed otherwise
    if (lecho) st_op(&ops[op++], mk_op(p, t, dt, origin, rec.sub, q, m, OP_ECHO, 0));  // (two dwordx4 stores)
    switch (type) {
      case PB_PRE_PREPARE: {  // :193-211
        const Msg rr = mkmsg(PB_PREPARE, mch(m, 1), mch(m, 2), mch(m, 3), 0);
        ops[op++] = fixed ? mk_op(p, t + p.app_delay, static_cast<uint32_t>(p.app_delay), i, sp, 0, rr, OP_BCAST, 0)
                          : mk_op(p, t, 0, i, sp, static_cast<uint32_t>(dp), rr, OP_BCAST_J, 0);
        sp += deg;
        if (!fixed) dp += deg;
        break;
      }
      case PB_PREPARE: {  // :212-222
        const Msg rr = mkmsg(PB_PREPARE_RES, mch(m, 1), mch(m, 2), enc_raw(p, 0), 0);
        int64_t d = p.app_delay;
        if (!fixed) d = delay_from_draw(p, ctr_rand(p.seed, rep, i, dp++));
        const Op ro = mk_op(p, t + d, static_cast<uint32_t>(d), i, sp++, q, rr, OP_SEND, 0);
        if (rslot & (1u << (r - r0))) {
          // (the reply is due in this cell or the next: app delay < L -- no 64-bit division)
          const long long dc = ro.t < cs + p.L ? cell : cell + 1;
          const uint64_t ut = static_cast<uint64_t>(ro.t);
          gst4(eslot_at(p, static_cast<uint32_t>(cell % kOpRing), rep, q),
               make_uint4(static_cast<uint32_t>(ut), static_cast<uint32_t>(ut >> 32), ro.sub,
                          (static_cast<uint32_t>(static_cast<uint16_t>(ro.f0))) |
                              (static_cast<uint32_t>(static_cast<uint16_t>(ro.f1)) << 16)));
          if (dc == cell)
            ++n_slot0;
          else
            ++n_slot1;
        } else {
          ops[op++] = ro;
        }
        break;
      }
      case PB_PREPARE_RES:  // :223-240
        if (cross) {
          const Msg rr = mkmsg(PB_COMMIT, mch(m, 1), mch(m, 2), 0, 0);
          ops[op++] = fixed ? mk_op(p, t + p.app_delay, static_cast<uint32_t>(p.app_delay), i, sp, 0, rr, OP_BCAST, 0)
                            : mk_op(p, t, 0, i, sp, static_cast<uint32_t>(dp), rr, OP_BCAST_J, 0);
          sp += deg;
          if (!fixed) dp += deg;
        }
        break;
      case PB_COMMIT:  // :241-265
        if (cross) {
          const int32_t idx = static_cast<int32_t>(w & kIdxMask);
          // tx[idx].val as of this event: the latest PRE_PREPARE of the window before it
          int32_t val = 0;
          int32_t best = -1;
          for (uint32_t k = 0; k < min(S.npp, 64u); ++k)
            if (S.pp_idx[k] == idx && S.pp_r[k] < r && static_cast<int32_t>(S.pp_r[k]) > best) {
              best = static_cast<int32_t>(S.pp_r[k]);
              val = S.pp_val[k];
            }
          if (best < 0) val = AT(p.tx_val, base + idx, p.cap_txn);
          // a = global v, resolved from the v-log on the host (INT32_MIN marker)
          emit_trace(p, key, rep, i, BCSIM_TR_PBFT_COMMIT, INT32_MIN, bn0 + static_cast<int32_t>(cp), val);
          ++cp;
        }
        break;
      case PB_VIEW_CHANGE: {  // :271-286 (falls through to "Wrong msg")
        const int32_t vt = c2i(mch(m, 1));
        const int32_t lt = c2i(mch(m, 2));
        emit_vlog(p, key, rep, i, vt);
        if (static_cast<int32_t>(i) == lt) emit_trace(p, key, rep, i, BCSIM_TR_PBFT_VIEW, vt, lt, 0);
        if (r + 1 == S.last_vc) S.leader = lt;
        ++wrong;
        break;
      }
      default:
        ++wrong;
        break;
    }
  }
  // delivery counters by type (wave-aggregated)
  for (uint32_t j = 0; j < per; ++j) {
    const uint32_t r = r0 + j;
    const bool act = r < r1;
    const uint32_t ty = act ? cls_type(acls[r]) : 0u;
    wave_add_by_key(act && ty < BCSIM_MSG_TYPES, ty, 1u, S.deliv);
  }
  if (wrong) atomicAdd(&S.wrong, wrong);
  if (n_slot0) atomicAdd(&S.ocnt[0], n_slot0);
  if (n_slot1) atomicAdd(&S.ocnt[1], n_slot1);
  __syncthreads();
  SPH(6);
  // ---- E: tx[n].val of the window's PRE_PREPAREs (last one per index wins) ----
  for (uint32_t k = tid; k < min(S.npp, 64u); k += blockDim.x) {
    bool last = true;
    for (uint32_t k2 = 0; k2 < min(S.npp, 64u); ++k2)
      if (S.pp_idx[k2] == S.pp_idx[k] && S.pp_r[k2] > S.pp_r[k]) last = false;
    if (last) AT(p.tx_val, base + S.pp_idx[k], p.cap_txn) = S.pp_val[k];
  }
  if (tid == 0) {
    S.sub += tot.x;
    S.draws += tot.y;
    S.block_num += static_cast<int32_t>(tot.z);
    S.nops += tot.w;
    if (n) S.tmax = max(S.tmax, cs + static_cast<long long>(akey[n - 1] >> 32));
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Gossip (BCSIM_GOSSIP, build extension for BASELINE configs[4], include/bcsim.h):
// PBFT-style block flooding.  GS_BLOCK carries f0 = sequence, f1 = hop count.
// Same order of schedule calls as oracle/bcsim_oracle.c gossip_tick/gossip_recv.
enum { GS_BLOCK = 1 };

__device__ bool gossip_mark(Ctx& c, int32_t seq) {  // false: already seen (or bad index)
  const KP& p = *c.p;
  if (seq < 0 || static_cast<uint32_t>(seq) >= p.pbft_seq_cap) {
    set_err(p, BCSIM_E_INDEX);
    return false;
  }
  uint8_t& f = AT(p.gseen, static_cast<size_t>(c.g) * p.pbft_seq_cap + seq,
                  static_cast<uint64_t>(p.NT) * p.pbft_seq_cap);
  if (f) return false;
  f = 1;
  return true;
}

// origin tick: SendBlock shape (pbft-node.cc:371-411) without the globals
__device__ void gossip_tick(Ctx& c, int32_t& round) {
  const KP& p = *c.p;
  const int32_t seq = round++;
  if (!gossip_mark(c, seq)) return;
  ctx_trace(c, BCSIM_TR_GOSSIP_BLOCK, seq, 0, 0);
  ctx_bcast(c, mkmsg(GS_BLOCK, seq, 0, 0, 1), false);
  if (round < static_cast<int32_t>(p.pbft_rounds)) (void)ctx_timer(c, TM_GOSSIP_BLOCK, p.pbft_period);
}

// `first`: this arrival is the node's first receipt of the block (computed for the whole
// window by gossip_first_flags, which also marks the blocks seen)
__device__ void gossip_recv(Ctx& c, const Msg& m, uint32_t sender, bool first, uint32_t& tr_pos) {
  const KP& p = *c.p;
  if (m.type != GS_BLOCK) {
    ++c.wrong;
    return;
  }
  if (m.f[0] < 0 || static_cast<uint32_t>(m.f[0]) >= p.pbft_seq_cap) {
    set_err(p, BCSIM_E_INDEX);
    return;
  }
  if (!first) return;
  TRAIL(c);
  put_trace(p, tr_pos++, c.cur, c.rep, c.i, BCSIM_TR_GOSSIP_DELIVER, m.f[0], m.f[1] + 1, static_cast<int32_t>(sender));
  ctx_bcast(c, mkmsg(GS_BLOCK, m.f[0], m.f[1] + 1, 0, 1), false);
}

// Data-parallel part of the gossip handler: lane r decides whether staged arrival r (key
// order) is its node's first receipt of that block -- not seen in an earlier window, and no
// earlier arrival of this window carries the same sequence -- writes the flag to acls[r], and
// the first receipts are marked seen.  The lane-0 event loop then reads the flags from LDS.
__device__ void gossip_first_flags(const KP& p, ScanShared& S, uint32_t g, uint32_t n, const uint32_t* asec,
                                   const RecSrc rs, uint32_t* acls) {
  const uint32_t tid = tidx();
  if (tid == 0) S.tr_n = 0;
  __syncthreads();
  for (uint32_t r = tid; r < n; r += blockDim.x) {
    const Rec rc = rec_of(rs, asec[r]);
    const int32_t seq = rc.f0;
    bool first = rc.type == GS_BLOCK && seq >= 0 && static_cast<uint32_t>(seq) < p.pbft_seq_cap &&
                 AT(p.gseen, static_cast<size_t>(g) * p.pbft_seq_cap + seq,
                    static_cast<uint64_t>(p.NT) * p.pbft_seq_cap) == 0;
    for (uint32_t r2 = 0; first && r2 < r; ++r2) {
      const Rec o = rec_of(rs, asec[r2]);
      if (o.type == GS_BLOCK && o.f0 == seq) first = false;
    }
    acls[r] = first ? 1u : 0u;
    if (first) atomicAdd(&S.tr_n, 1u);
  }
  __syncthreads();
  // one trace reservation per window for all its first receipts (no per-record global atomic)
  if (tid == 0) S.tr_pos = S.tr_n ? gadd_r(p.trace_cnt, S.tr_n) : 0u;
  for (uint32_t r = tid; r < n; r += blockDim.x)
    if (acls[r])
      AT(p.gseen, static_cast<size_t>(g) * p.pbft_seq_cap + rec_of(rs, asec[r]).f0,
         static_cast<uint64_t>(p.NT) * p.pbft_seq_cap) = 1;
}

// A Paxos proposer's window of responses, data-parallel (paxos-node.cc:248-353, the serial form
// is paxos_recv): every arrival is a RESPONSE_TICKET / _PROPOSE / _COMMIT, no timer, START or
// STOP is due and at most one quorum decision falls in the window, on the arrival whose running
// count (vote_success + vote_failed, carried in) reaches N - 2 -- and no counted response
// follows it.  Then the counts are prefix sums over the key-ordered arrivals (block scans), the
// one decision runs on lane 0 with the counters as of that arrival (its broadcast follows the
// echoes of the arrivals before it), and the echo ops are written in parallel at their serial
// positions.  Anything else returns false with nothing changed: the lane-0 event loop takes the
// window.  All lanes call it; c / s are lane 0's.
__device__ bool paxos_window_fast(const KP& p, ScanShared& S, Ctx& c, PaxosState& s, uint32_t g, uint32_t n,
                                  const uint32_t* asec, const RecSrc& rsrc, uint32_t e0, long long cs, long long t_lo,
                                  long long wb, const TimerEnt* tm, bool start_pending, bool stop_pending) {
  const uint32_t tid = tidx();
  Op* ops = p.ops + op_base(p, g);
  const uint32_t ocap = op_cap(p, g);
  if (n == 0 || p.dbg_tmax > LLONG_MIN || start_pending || stop_pending) return false;
  const int32_t N2 = static_cast<int32_t>(p.N) - 2;
  if (tid == 0) {
    S.px_dec = s.decree;
    S.px_c0 = s.vs + s.vf;
    S.px_bad = 0;
    S.px_r = kInvalid;
    S.px_nops0 = c.nops;
    S.px_tmax = LLONG_MIN;
    S.px_deliv[0] = S.px_deliv[1] = S.px_deliv[2] = 0;
    S.px_nx = 0;
    for (uint32_t k = 0; k < c.cap_t; ++k)
      if (tm[k].alive && !tm[k].pending_draw && tm[k].t < wb && tm[k].t >= t_lo) S.px_bad = 1;
    if (S.px_bad && p.fdbg) gadd_r(&p.fdbg[1], 1ull);
  }
  __syncthreads();
  if (S.px_bad) return false;
  const int32_t dec = S.px_dec, c0 = S.px_c0;
  // pass 1: types, counted / successful responses, explicit echoes; the crossing arrival
  uint4 run = make_uint4(0, 0, 0, 0);
  long long tmax = LLONG_MIN;
  for (uint32_t base = 0; base < n; base += blockDim.x) {
    const uint32_t r = base + tid;
    uint32_t cnt = 0, suc = 0, ech = 0;
    if (r < n) {
      const uint32_t sec = asec[r];
      const Rec rec = rec_of(rsrc, sec);
      const int32_t ty = rec.type;
      if (ty != PX_RES_TICKET && ty != PX_RES_PROPOSE && ty != PX_RES_COMMIT) S.px_bad = 1;
      else atomicAdd(&S.px_deliv[ty - PX_RES_TICKET], 1u);
      cnt = rec.f2 == dec ? 1u : 0u;
      suc = cnt && rec.f0 == '0' ? 1u : 0u;
      if (rec.f2 == dec + 1) atomicMax(&S.px_nx, r + 1);  // a response of the next decree
      ech = p.echo && !(p.impl && is_main(sec)) ? 1u : 0u;
      tmax = max(tmax, cs + static_cast<long long>(rec.t_off));
    }
    uint4 tot;
    const uint4 ex = block_scan4(make_uint4(cnt, suc, ech, 0), S.wsum, tot);
    if (cnt && c0 + static_cast<int32_t>(run.x + ex.x) + 1 == N2) {
      S.px_r = r;
      S.px_cb = run.x + ex.x;
      S.px_sb = run.y + ex.y;
      S.px_eb = run.z + ex.z + ech;  // explicit echoes up to and including the crossing arrival
    }
    run.x += tot.x;
    run.y += tot.y;
    run.z += tot.z;
  }
  for (int d = 32; d > 0; d >>= 1) tmax = max(tmax, static_cast<long long>(__shfl_xor(tmax, d, 64)));
  if ((tid & 63u) == 0 && tmax > LLONG_MIN) atomicMax(&S.px_tmax, tmax);
  __syncthreads();
  // Counting restarts at 0 after the decision (paxos-node.cc:263-353): the counted responses after
  // it add to the fresh counters when the decree stays, unless they reach a second decision; when
  // the decision commits and opens the next decree, the rest of the window's responses are of a
  // finished decree (not counted) unless one is of the new decree.  Those cases, and foreign
  // types, take the serial loop.
  const bool cross = S.px_r != kInvalid;
  if (tid == 0 && !S.px_bad) {
    uint32_t why = 0;
    if (!cross && c0 + static_cast<int32_t>(run.x) > N2) why = 3;
    if (cross) {
      const Rec rx = rec_of(rsrc, asec[S.px_r]);
      const uint32_t suc_r = rx.f0 == '0' ? 1u : 0u;
      const bool adv = rx.type == PX_RES_COMMIT && s.vs + static_cast<int32_t>(S.px_sb + suc_r) >= static_cast<int32_t>(p.N) / 2 &&
                       static_cast<uint32_t>(dec) + 1 < p.K;
      if (adv ? S.px_nx > S.px_r + 1 : run.x - S.px_cb - 1 >= static_cast<uint32_t>(N2)) why = 3;
      S.px_adv = adv ? 1u : 0u;
      S.px_sr = suc_r;
    }
    if (!why && S.px_nops0 + run.z + (cross ? 1u : 0u) > ocap) why = 4;
    if (why) S.px_bad = 1;
    if (p.fdbg) gadd_r(&p.fdbg[why ? why : S.px_bad ? 2 : 0], 1ull);
  }
  __syncthreads();
  if (S.px_bad) return false;
  // the decision (lane 0): the event of the crossing arrival, its counters as of that arrival
  if (tid == 0) {
    for (int k = 0; k < 3; ++k) S.deliv[PX_RES_TICKET + k] += S.px_deliv[k];
    if (p.echo) c.echoes += n;
    c.events += n;
    if (S.px_tmax > S.tmax) S.tmax = S.px_tmax;
    if (cross) {
      const uint32_t r = S.px_r, sec = asec[r];
      const Rec rec = rec_of(rsrc, sec);
      const uint32_t q = e0 + (sec >> kSlotShift);
      const uint32_t dt = static_cast<uint32_t>(prop_of_slot(p, q) + sel2(p.tx_last, (rec.flags & RF_BIG) ? 1 : 0));
      c.cur.t = cs + rec.t_off;
      c.cur.ts = c.cur.t - dt;
      c.cur.origin = AT(p.col, q, p.E);
      c.cur.sub = rec.sub;
      s.vs += static_cast<int32_t>(S.px_sb);
      s.vf += static_cast<int32_t>(S.px_cb - S.px_sb);
      c.nops = S.px_nops0 + S.px_eb;
      paxos_recv(c, s, rec_msg(rec), q);
      if (!S.px_adv) {  // the counted responses after the decision, on the fresh counters
        const uint32_t ca = run.x - S.px_cb - 1, sa = run.y - S.px_sb - S.px_sr;
        s.vs += static_cast<int32_t>(sa);
        s.vf += static_cast<int32_t>(ca - sa);
      }
      S.px_ncross = c.nops - (S.px_nops0 + S.px_eb);
      c.nops = S.px_nops0 + run.z + S.px_ncross;
    } else {
      s.vs += static_cast<int32_t>(run.y);
      s.vf += static_cast<int32_t>(run.x - run.y);
      S.px_ncross = 0;
      c.nops = S.px_nops0 + run.z;
    }
  }
  __syncthreads();
  // pass 2: the echo ops at their serial positions
  const uint32_t rx = S.px_r, ncr = S.px_ncross, nops0 = S.px_nops0;
  uint32_t eb = 0;
  for (uint32_t base = 0; base < n; base += blockDim.x) {
    const uint32_t r = base + tid;
    uint32_t ech = 0;
    uint32_t sec = 0;
    if (r < n) {
      sec = asec[r];
      ech = p.echo && !(p.impl && is_main(sec)) ? 1u : 0u;
    }
    uint4 tot;
    const uint4 ex = block_scan4(make_uint4(ech, 0, 0, 0), S.wsum, tot);
    if (ech) {
      const Rec rec = rec_of(rsrc, sec);
      const uint32_t q = e0 + (sec >> kSlotShift);
      const uint32_t dt = static_cast<uint32_t>(prop_of_slot(p, q) + sel2(p.tx_last, (rec.flags & RF_BIG) ? 1 : 0));
      const long long t = cs + rec.t_off;
      const uint32_t pos = nops0 + eb + ex.x + (rx != kInvalid && r > rx ? ncr : 0u);
      st_op(&AT(ops, pos, ocap), mk_op(p, t, dt, AT(p.col, q, p.E), rec.sub, q, rec_msg(rec), OP_ECHO, 0));
    }
    eb += tot.x;
  }
  return true;
}

template <int PROTO, bool SP>
__device__ __attribute__((always_inline)) inline void scan_node(const KP* pk, uint32_t g, long long cell, long long t_lo, long long t_hi,
                          long long cs, int final_win, int x_active) {
  const KP& p = *pk;
  // LDS: akey[cap] u64 | asec[cap] u32 | acls[cap] u32 | timers
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ ScanShared S;
  const uint32_t cap = p.cap_arr;
  uint64_t* akey = reinterpret_cast<uint64_t*>(smem);
  uint32_t* asec = reinterpret_cast<uint32_t*>(akey + cap);
  uint32_t* acls = asec + cap;
  TimerEnt* tm = reinterpret_cast<TimerEnt*>(acls + cap);

  const uint32_t tid = tidx();
  const uint32_t b = static_cast<uint32_t>(cell % p.n_buckets);
  const bool has_start = (t_lo <= 0 && 0 < t_hi);
  const bool has_stop = (p.stop_ns >= 0 && t_lo <= p.stop_ns && p.stop_ns < t_hi);
  const size_t fidx = static_cast<size_t>(b) * p.NT + g;
  const uint32_t rep = g / p.N, i = g % p.N;
  // the node's row (full mesh: arithmetic, no load) and its flags, loads issued together
  const uint32_t e0 = p.mesh ? i * (p.N - 1) : AT(p.row, i, p.N + 1);
  const uint32_t deg = p.mesh ? p.N - 1 : AT(p.row, i + 1, p.N + 1) - e0;
  const bool flag = node_flagged_w(p, b, g, rep, i, t_hi);
  if (!flag && AT(p.node_tnext, g, p.NT) >= t_hi && !has_start && !has_stop) return;

  // sparse mode: no inbox slots, the node's arrivals are all in the cell's grouped lists
  const Rec* slots = SP ? nullptr : p.inbox + inbox_idx(p, b, rep, e0);
  const uint32_t deg_in = SP ? 0u : deg;
  uint32_t xn = 0;
  const XRec* xs = p.xgrp;
  if (x_active) {
    const uint32_t xb = AT(p.seg_off, g, p.NT + 1);
    xn = AT(p.seg_off, g + 1, p.NT + 1) - xb;
    xs = p.xgrp + xb;
    if (xn > kXIdx + 1) {  // staged ids index at most 8192 extras records per node and cell
      if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
      return;
    }
  }
  if (PROTO != BCSIM_PBFT && tid < p.cap_timers)
    tm[tid] = AT(p.timers, static_cast<size_t>(g) * p.cap_timers + tid, static_cast<uint64_t>(p.NT) * p.cap_timers);

  // ---- node state ----
  SPH(0);
  if (tid == 0) {
    S.sub = AT(p.sub, g, p.NT);
    S.draws = AT(p.draws, g, p.NT);
    S.nops = AT(p.n_ops, g, p.NT);
    S.block_num = PROTO == BCSIM_PBFT ? AT(p.block_num, g, p.NT) : 0;
    S.leader = PROTO == BCSIM_PBFT ? AT(p.leader, g, p.NT) : 0;
    for (int k = 0; k < BCSIM_MSG_TYPES; ++k) S.deliv[k] = 0;
    for (uint32_t k = 0; k < kOpRing; ++k) S.ocnt[k] = 0;
    S.wrong = 0;
    S.tmax = LLONG_MIN;
  }
  Ctx c;
  RaftState rs{};
  PaxosState xs_{};
  int32_t gs_round = 0;
  unsigned long long events = 0;
  bool start_pending = has_start, stop_pending = has_stop;
  if (PROTO != BCSIM_PBFT && tid == 0) {
    c.p = pk;
    c.g = g;
    c.rep = rep;
    c.i = i;
    c.deg = deg;
    c.ops = p.ops + op_base(p, g);
    c.cap_ops = op_cap(p, g);
    c.tm = tm;
    c.cap_t = p.cap_timers;
    c.echoes = c.wrong = c.events = 0;
    if (PROTO == BCSIM_RAFT) {
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
    } else if (PROTO == BCSIM_GOSSIP) {
      gs_round = AT(p.round, g, p.NT);
    } else {
      xs_.ticket = AT(p.ticket, g, p.NT);
      xs_.proposal = AT(p.proposal, g, p.NT);
      xs_.decree = AT(p.decree, g, p.NT);
      xs_.vs = AT(p.vote_s, g, p.NT);
      xs_.vf = AT(p.vote_f, g, p.NT);
    }
  }
  __syncthreads();
  if (PROTO == BCSIM_PBFT && has_start && tid == 0) {  // StartApplication pbft-node.cc:97-158
    S.leader = 0;
    S.block_num = 0;
    AT(p.tick_sub, g, p.NT) = S.sub++;  // Schedule(Seconds(timeout), SendBlock) :155
    AT(p.tick_alive, g, p.NT) = 1;
    S.tmax = 0;
  }
  if (PROTO == BCSIM_PBFT) {
    events += (has_start ? 1 : 0) + (has_stop ? 1 : 0);
    if (has_stop && tid == 0) S.tmax = max(S.tmax, static_cast<long long>(p.stop_ns));
  }

  // ---- windows of <= cap arrivals ----
  long long wa = t_lo;
  for (;;) {
    long long wb = t_hi;
    uint32_t n = flag ? stage_window(p, S, slots, e0, deg_in, xs, xn, cs, wa, wb, akey, asec, true) : 0u;
    if (n > cap) {  // more than cap arrivals: shrink the window (rare)
      wb = window_split(p, S, slots, deg_in, xs, xn, cs, wa, t_hi, reinterpret_cast<uint32_t*>(akey));
      if (tid == 0) atomicAdd(&kst_stripe(p)[KST_SPLIT], 1ull);
      if (wb == wa) {  // > cap arrivals at one instant
        if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
        return;
      }
      n = stage_window(p, S, slots, e0, deg_in, xs, xn, cs, wa, wb, akey, asec, true);
    }
    const uint32_t n_main = S.n_main;
    SPH(1);
    sort_window(S, n, akey, asec, p.sortbuf ? gbl(p.sortbuf) + static_cast<size_t>(blockIdx.x) * p.cap_arr : nullptr);
    SPH(2);

    const RecSrc rsrc{slots, xs};
    if (PROTO == BCSIM_GOSSIP) gossip_first_flags(p, S, g, n, asec, rsrc, acls);
    if (PROTO == BCSIM_PBFT) {
      pbft_window(p, S, g, rep, i, e0, deg, n, n_main, cell, cs, t_lo, akey, asec, rsrc, acls);
      events += (tid == 0) ? n : 0;
    } else {
    if (tid == 0) {
      c.sub = S.sub;
      c.draws = S.draws;
      c.nops = S.nops;
    }
    // (Paxos proposers: the window's responses data-parallel when it qualifies)
    const bool px_fast = PROTO == BCSIM_PAXOS && p.paxos_fast_win &&
                         paxos_window_fast(p, S, c, xs_, g, n, asec, rsrc, e0, cs, t_lo, wb, tm, start_pending, stop_pending);
    if (px_fast) {
      if (tid == 0) {
        S.sub = c.sub;
        S.draws = c.draws;
        S.nops = c.nops;
      }
    } else if (tid == 0) {
      uint32_t ai = 0;
      for (;;) {
        int which = -1;  // 0 arrival, 1 timer, 2 start, 3 stop
        Key best{};
        Rec rec{};
        uint32_t q = 0;
        int tsel = -1;
        if (ai < n) {
          const uint32_t sec = asec[ai];
          rec = rec_of(rsrc, sec);
          q = e0 + (sec >> kSlotShift);
          const uint32_t dt = static_cast<uint32_t>(prop_of_slot(p, q) + sel2(p.tx_last, (rec.flags & RF_BIG) ? 1 : 0));
          best.t = cs + rec.t_off;
          best.ts = best.t - dt;
          best.origin = AT(p.col, q, p.E);
          best.sub = rec.sub;
          which = 0;
        }
        for (uint32_t k = 0; k < c.cap_t; ++k) {
          const TimerEnt& te = tm[k];
          if (!te.alive || te.pending_draw || te.t >= wb || te.t < t_lo) continue;
          const Key kk{te.t, te.ts, i, te.sub};
          const bool cb = which < 0 || key_less(kk, best);
          key_sel(best, kk, cb);
          if (cb) {
            which = 1;
            tsel = static_cast<int>(k);
          }
        }
        if (start_pending && 0 < wb) {
          const Key kk{0, -1, i, 0};
          const bool cb = which < 0 || key_less(kk, best);
          key_sel(best, kk, cb);
          if (cb) which = 2;
        }
        if (stop_pending && p.stop_ns < wb) {
          const Key kk{p.stop_ns, -1, i, 1};
          const bool cb = which < 0 || key_less(kk, best);
          key_sel(best, kk, cb);
          if (cb) which = 3;
        }
        TRAIL(c);
        if (which < 0) break;
        c.cur = best;
        if (best.t > S.tmax) S.tmax = best.t;
        ++c.events;
        if (which == 0) {
          ++ai;
          const Msg msg = rec_msg(rec);
          // the per-type counts live in LDS, so that Ctx has no dynamically indexed member and
          // stays in registers (this once exposed the struct-select miscompile
          // that key_sel now avoids)
          if (rec.type < BCSIM_MSG_TYPES) ++S.deliv[rec.type];
          if (p.echo) {  // socket->SendTo(packet, 0, from): reverse-link occupancy
            const Op eo = mk_op(p, best.t, static_cast<uint32_t>(best.t - best.ts), best.origin, rec.sub, q, msg,
                                OP_ECHO, 0);
            if (!(p.impl && is_main(asec[ai - 1]))) ctx_op(c, eo);  // else implicit (k_link)
            ++c.echoes;
          }
          if (PROTO == BCSIM_RAFT)
            raft_recv(c, rs, msg, q);
          else if (PROTO == BCSIM_GOSSIP)
            gossip_recv(c, msg, best.origin, acls[ai - 1] != 0, S.tr_pos);
          else
            paxos_recv(c, xs_, msg, q);
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
          } else if (PROTO == BCSIM_GOSSIP) {
            if (te.kind == TM_GOSSIP_BLOCK) gossip_tick(c, gs_round);
          } else {
            if (te.kind == TM_PAXOS_TICKET) paxos_ticket(c, xs_);
          }
        } else if (which == 2) {  // StartApplication
          start_pending = false;
          if (PROTO == BCSIM_RAFT) {  // :75-115
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
          } else if (PROTO == BCSIM_GOSSIP) {
            gs_round = 0;
            if (i == 0) (void)ctx_timer(c, TM_GOSSIP_BLOCK, p.pbft_period);
          } else {  // paxos-node.cc:58-139
            for (uint32_t d = 0; d < p.K; ++d) {
              int32_t* a = px_of(c, static_cast<int32_t>(d));
              a[0] = 0;    // t_max
              a[1] = 'e';  // command
              a[2] = 0;    // t_store
              a[3] = 0;    // isCommit
            }
            xs_.ticket = 0;
            xs_.decree = 0;
            xs_.proposal = enc_raw(p, static_cast<int32_t>(i));
            xs_.vs = 0;
            xs_.vf = 0;
            if (i < p.paxos_proposers) (void)ctx_timer(c, TM_PAXOS_TICKET, 0);
          }
        } else {  // StopApplication
          stop_pending = false;
          if (PROTO == BCSIM_RAFT && rs.is_leader == 1) ctx_trace(c, BCSIM_TR_RAFT_STOP, rs.blockNum, rs.round, 0);
        }
        if (best.t < p.dbg_tmax)  // debug event log (BCSIM_DBG_EVENTS)
          emit_trace(p, best, rep, i, 90 + which, which == 0 ? rec.type * 256 + (rec.f0 & 255) : which == 1 ? tm[tsel].kind : 0,
                     PROTO == BCSIM_RAFT ? rs.vs * 65536 + rs.vf : xs_.vs * 65536 + xs_.vf,
                     PROTO == BCSIM_RAFT ? rs.has_voted + 2 * rs.is_leader : xs_.ticket);
      }
      S.sub = c.sub;
      S.draws = c.draws;
      S.nops = c.nops;
    }
    }
    __syncthreads();
    // consumed slots are free again
    for (uint32_t r = tid; r < n; r += blockDim.x) {
      const uint32_t sec = asec[r];
      if (!p.impl && is_main(sec)) clr_rec(const_cast<Rec*>(slots) + (sec >> kSlotShift));
    }
    __syncthreads();
    if (wb >= t_hi) break;
    wa = wb;
  }
  // (implicit echoes: k_link still reads this cell's slots and clears the flag)
  if (final_win && flag && tid == 0 && !p.impl) AT(p.iflag, fidx, static_cast<uint64_t>(p.n_buckets) * p.NT) = 0;
  // slot ops make their cells busy (bucket counts) and flag this node for k_link
  if (tid < kOpRing && S.ocnt[tid]) mark_busy(&p.bucket_cnt[(cell + tid) % p.n_buckets]);
  if (tid == 0) {
    uint32_t m = 0;
    for (uint32_t k = 0; k < kOpRing; ++k) m |= S.ocnt[k] ? (1u << k) : 0u;
    if (m) {
      uint8_t& f = AT(p.sflag, (cell % kOpRing) * p.NT + g, static_cast<uint64_t>(kOpRing) * p.NT);
      f = static_cast<uint8_t>(f | m);
    }
  }

  // ---- write back ----
  unsigned long long* cnt = cnt_stripe(p, rep);
  if (tid != 0) return;
  if (p.wgs) {
    SPH(7);
    for (int k = 0; k < 8; ++k) p.wgs[8ull * g + k] = S.ph[k];
  }
  const uint32_t nops_in = AT(p.n_ops, g, p.NT);
  AT(p.sub, g, p.NT) = S.sub;
  AT(p.draws, g, p.NT) = S.draws;
  AT(p.n_ops, g, p.NT) = S.nops;
  if (S.nops > nops_in) AT(p.node_onext, g, p.NT) = LLONG_MIN;  // link stage recomputes
  unsigned long long tot = 0;
  if (PROTO == BCSIM_PBFT) {
    AT(p.leader, g, p.NT) = S.leader;
    AT(p.block_num, g, p.NT) = S.block_num;
    for (int k = 0; k < BCSIM_MSG_TYPES; ++k)
      if (S.deliv[k]) {
        atomicAdd(&cnt[CNT_DELIV + k], S.deliv[k]);
        tot += S.deliv[k];
      }
    if (tot) {
      atomicAdd(&cnt[CNT_DELIV_TOTAL], tot);
      if (p.echo) atomicAdd(&cnt[CNT_ECHOES], tot);
      atomicAdd(&kst_stripe(p)[KST_DELIV], tot);
    }
    if (S.wrong) atomicAdd(&cnt[CNT_WRONG], S.wrong);
    if (events) atomicAdd(&cnt[CNT_EVENTS], events);
  } else {
    long long tnext = LLONG_MAX;
    for (uint32_t k = 0; k < c.cap_t; ++k) {
      AT(p.timers, static_cast<size_t>(g) * p.cap_timers + k, static_cast<uint64_t>(p.NT) * p.cap_timers) = tm[k];
      if (tm[k].alive && tm[k].t < tnext) tnext = tm[k].t;
    }
    AT(p.node_tnext, g, p.NT) = tnext;
    if (PROTO == BCSIM_RAFT) {
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
    } else if (PROTO == BCSIM_GOSSIP) {
      AT(p.round, g, p.NT) = gs_round;
    } else {
      AT(p.ticket, g, p.NT) = xs_.ticket;
      AT(p.proposal, g, p.NT) = xs_.proposal;
      AT(p.decree, g, p.NT) = xs_.decree;
      AT(p.vote_s, g, p.NT) = xs_.vs;
      AT(p.vote_f, g, p.NT) = xs_.vf;
    }
    for (int k = 0; k < BCSIM_MSG_TYPES; ++k)
      if (S.deliv[k]) {
        const unsigned long long dk = S.deliv[k];
        atomicAdd(&cnt[CNT_DELIV + k], dk);
        tot += dk;
      }
    if (tot) {
      atomicAdd(&cnt[CNT_DELIV_TOTAL], tot);
      atomicAdd(&kst_stripe(p)[KST_DELIV], tot);
    }
    if (c.echoes) atomicAdd(&cnt[CNT_ECHOES], c.echoes);
    if (c.wrong) atomicAdd(&cnt[CNT_WRONG], c.wrong);
    if (c.events) atomicAdd(&cnt[CNT_EVENTS], c.events);
  }
  if (S.tmax > LLONG_MIN) atomicMax(reinterpret_cast<long long*>(&cnt[CNT_TLAST]), S.tmax);
}

// a fixed grid over the window's active list (k_active); SP: sparse layout (no inbox slots)
// LOOP: a small grid walks list 2, the nodes k_gossip_scan / k_paxos_scan left over
// (Raft / Paxos / gossip: at most 256 lanes, so that lane 0's protocol state machine -- Ctx and
// the node state, live across the event loop -- has the registers it needs instead of scratch)
// Device-chained windows (dense gossip): k_win decides each window on the device
// and the window's kernels, launched with cell = -1, take it from the control block's win words
// (or do nothing when k_win found none: the chain ended, the host takes over).
enum : int { kWinValid = 0, kWinCell, kWinLo, kWinHi, kWinFw, kWinLoop, kWinTDone, kWinLastFull, kWinGrouped,
             kWinCount, kWinDead, kWinLim, kWinStop, kWinLoopMask, kWinFrCell, kWinFrHi, kWinFrHits, kWinWords = 20 };
// (the words are workgroup-uniform: read into scalar registers, so the kernels that take them keep
// their window bounds where the kernel arguments were)
__device__ inline long long win_word(const KP& p, int k) {
  const long long v = p.win[k];
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(static_cast<unsigned long long>(v) >> 32));
  return static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo);
}
__device__ inline bool win_take(const KP& p, long long& cell, long long& lo, long long& hi, int& fw) {
  if (cell >= 0) return true;
  if (!win_word(p, kWinValid)) return false;
  cell = win_word(p, kWinCell);
  lo = win_word(p, kWinLo);
  hi = win_word(p, kWinHi);
  fw = static_cast<int>(win_word(p, kWinFw));
  return true;
}

template <int PROTO, bool SP, bool LOOP = false>
__global__ __launch_bounds__(PROTO == BCSIM_PBFT ? 1024 : 256) void k_scan(const KP* pk, long long cell, long long t_lo,
                                               long long t_hi, long long cs, int final_win, int x_active) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  if (LOOP) {
    if constexpr (PROTO == BCSIM_GOSSIP && !SP) {
      if (cell < 0) {  // (a chained window: only when the window needs the generic scan)
        if (!win_take(p, cell, t_lo, t_hi, final_win) || !win_word(p, kWinLoop)) return;
        cs = cell * p.L;
        x_active = 0;
      }
    }
    for (ListRange lr = list_range(p.act_n[2]); lr.k < lr.end; lr.k += lr.step) {
      scan_node<PROTO, SP>(pk, p.act[2ull * p.NT + lr.k], cell, t_lo, t_hi, cs, final_win, x_active);
      __syncthreads();
    }
    return;
  }
  if (!SP) {
    uint32_t k;
    if (list_one(p.act_n[0], k)) scan_node<PROTO, false>(pk, p.act[k], cell, t_lo, t_hi, cs, final_win, x_active);
    return;
  }
  for (ListRange lr = list_range(p.act_n[0]); lr.k < lr.end; lr.k += lr.step) {
    scan_node<PROTO, true>(pk, p.act[lr.k], cell, t_lo, t_hi, cs, final_win, x_active);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_scan_pbft (dense layout, PBFT, fixed app delay < L with reply slots, degree <= 4096): the
// k_scan of a node whose window holds only main-slot PRE_PREPARE / PREPARE / PREPARE_RES /
// COMMIT arrivals that all carry one canonical key prefix (t, dt) -- the PBFT heavy waves,
// where a row holds one record per in-edge, all at one instant.  The same state changes and
// outputs as scan_node + pbft_window (pbft-node.cc:166-265) for such a node, in ONE pass over
// its inbox row: every lane keeps kFastRPL records in registers (slot j * 512 + lane: the row
// is read with coalesced 16-byte loads, all in flight at once).  With equal (t, dt) the
// canonical order is the slot order (sort_window breaks ties by slot), so every prefix the
// handler needs -- quorum ranks per (phase, sequence), the schedule counter, op positions,
// commit numbers -- is a count of flagged arrivals before this one: wave ballots + popcounts
// plus per-(chunk, wave) totals in LDS.  No key staging, no sort, no second or third read of
// the row, 3 KB of LDS instead of 76 KB.  A node that does not qualify (an extras record,
// another message type, arrivals at different instants, more than kFastKeys (phase, sequence)
// groups or kFastPP PRE_PREPAREs, a bad index, START / STOP, a due timer) is appended to
// list 2, untouched, for k_scan<PBFT, false, LOOP>.
#ifndef BCSIM_SCANPBFT_WPE
#define BCSIM_SCANPBFT_WPE 4  // k_scan_pbft occupancy target (waves per SIMD; 6 = three 512-lane workgroups per CU)
#endif
constexpr uint32_t kFastLanes = 512, kFastRPL = 8, kFastWaves = kFastLanes / 64, kFastKeys = 8, kFastPP = 16;
constexpr uint32_t kFastSeg = kFastRPL * kFastWaves;  // (chunk, wave) segments in arrival order
struct FastShared {
  uint4 seg[kFastSeg];                 // per segment (PREPAREs, deg-steps, commits, arrivals); then exclusive bases
  uint32_t qc[kFastSeg][kFastKeys];    // quorum group counts per segment, then bases
  uint32_t tkey[kFastKeys];            // (phase, sequence) groups of the window
  uint32_t tcnt[kFastKeys];            // stored vote count + the window's
  unsigned long long kmin, kmax;       // (t_off, ~dt) of the arrivals
  uint32_t bad, npp;
  uint32_t pp_k[kFastPP];
  int32_t pp_idx[kFastPP], pp_val[kFastPP];
  uint32_t tcount[4];  // deliveries: PRE_PREPARE, PREPARE, COMMIT, PREPARE_RES
  uint32_t ocnt[2];    // reply slots due in this cell / the next
  uint32_t fmin, fmax;  // PREPAREs' reply payload words (one reply descriptor if equal)
  uint32_t bigs;        // bit 0: a big arrival, bit 1: a small one (one echo descriptor if not both)
  uint64_t lw[kFastRPL * kFastLanes];  // link words of the node's out-edges (echo pass)
};

// record words {t_off, sub, f0 | f1 << 16, f2 | type << 16 | flags << 24} -> payload chars after
// getPacketContent's NUL truncation (mch)
__device__ inline int32_t fr_f0(const uint4& r) { return static_cast<int16_t>(r.z & 0xFFFFu); }
__device__ inline int32_t fr_m2(const uint4& r) { return fr_f0(r) ? static_cast<int16_t>(r.z >> 16) : 0; }
__device__ inline int32_t fr_m3(const uint4& r) {
  return (fr_f0(r) && static_cast<int16_t>(r.z >> 16)) ? static_cast<int16_t>(r.w & 0xFFFFu) : 0;
}
__device__ inline uint32_t fr_type(const uint4& r) { return (r.w >> 16) & 0xFFu; }
// quorum group of an arrival (kClsPres / kClsCommit | sequence) or 0; indices checked in pass 1
__device__ inline uint32_t fr_group(const uint4& r) {
  const uint32_t type = fr_type(r);
  const uint32_t idx = static_cast<uint32_t>(c2i(fr_m2(r))) & kIdxMask;
  if (type == PB_COMMIT) return kClsCommit | idx;
  if (type == PB_PREPARE_RES && c2i(fr_m3(r)) == 0) return kClsPres | idx;
  return 0u;
}

__device__ inline uint32_t fast_key_slot(FastShared& F, uint32_t key) {
  for (uint32_t k = 0; k < kFastKeys; ++k) {
    const uint32_t t = __hip_atomic_load(&F.tkey[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (t == key) return k;
    if (t == 0u) {
      const uint32_t old = atomicCAS(&F.tkey[k], 0u, key);
      if (old == 0u || old == key) return k;
    }
  }
  F.bad = 1;
  return kFastKeys;
}
__device__ inline uint32_t fast_key_find(const FastShared& F, uint32_t key) {
  uint32_t s = 0;
  for (uint32_t k = 0; k < kFastKeys; ++k)
    if (F.tkey[k] == key) s = k;
  return s;
}

// BCSIM_FDBG=1 (debug): count why a node leaves k_scan_pbft (0 no work .. 7 several instants) /
// k_link_mesh (8 listed ops, 9 too many broadcasts) for the generic kernels
#define FDBG(k)                                             \
  do {                                                      \
    if (p.fdbg) gadd_r(&p.fdbg[(k)], 1ull);              \
  } while (0)
// BCSIM_WGT=1 (debug): per-workgroup phase clock of k_scan_pbft, same slots as scan_node's SPH
#define FPH(k)                                                                              \
  do {                                                                                      \
    if (p.wgs && tid == 0) p.wgs[8ull * g + (k)] = __builtin_amdgcn_s_memrealtime();       \
  } while (0)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(BCSIM_SCANPBFT_WPE, 8))) void k_scan_pbft(const KP* __restrict__ pk, long long cell, long long t_lo,
                                                   long long t_hi, long long cs, int x_active, uint32_t wep) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ FastShared F;
  uint32_t kk;
  if (!list_one(p.act_n[0], kk)) return;
  const uint32_t g = p.act[kk];
  const uint32_t tid = tidx(), lane = tid & 63u, wv = tid >> 6;
  const uint32_t b = static_cast<uint32_t>(cell % p.n_buckets);
  const uint32_t rep = g / p.N, i = g % p.N;
  const uint32_t e0 = p.mesh ? i * (p.N - 1) : AT(p.row, i, p.N + 1);
  const uint32_t deg = p.mesh ? p.N - 1 : AT(p.row, i + 1, p.N + 1) - e0;
  // the row's loads go out first: the node's checks below are dependent global reads (its
  // bucket flag, timer, extras) that would otherwise serialise in front of them.  A node that
  // does not qualify leaves them unused (the heavy waves' nodes all qualify).
#ifndef BCSIM_SCANPBFT_SPEC
#define BCSIM_SCANPBFT_SPEC 1  // (0: the row loads after the checks, for an A/B)
#endif
  const bool spec = deg <= kFastLanes * kFastRPL && blockDim.x == kFastLanes && deg > 0;
  uint4 rv[kFastRPL];
  const Rec* slots = p.inbox + inbox_idx(p, b, rep, e0);
  // (unconditional loads at clamped slots, used only for k < deg: a per-load `k < deg` branch
  // made the compiler wait for each load before the next -- eight serial round trips)
  // (no branch at all: a zeroing else-path made the join wait for every load)
  auto row_loads = [&]() {
    const uint4* rb = reinterpret_cast<const uint4*>(deg ? slots : p.inbox);
    const uint32_t dm = deg ? deg - 1u : 0u;
#pragma unroll
    for (uint32_t j = 0; j < kFastRPL; ++j) rv[j] = gld4(rb + min(j * kFastLanes + tid, dm));
  };
  if (BCSIM_SCANPBFT_SPEC) row_loads();
  // the node's earliest pending op and its two slot-flag bytes (the echo rule below) with them,
  // unconditionally (a null flag array reads a dummy word)
  uint8_t* const sfa = p.sflag ? p.sflag : reinterpret_cast<uint8_t*>(p.act_n);
  const uint8_t sfv0 = gbl(sfa)[p.sflag ? static_cast<size_t>(cell % kOpRing) * p.NT + g : 0u];
  const uint8_t sfv1 = gbl(sfa)[p.sflag ? static_cast<size_t>((cell + kOpRing - 1) % kOpRing) * p.NT + g : 0u];
  const long long onext0 = AT(p.node_onext, g, p.NT);  // earliest pending op (LLONG_MIN: unknown)
  const bool flag = node_flagged_w(p, b, g, rep, i, t_hi);
  const bool has_ss = (t_lo <= 0 && 0 < t_hi) || (p.stop_ns >= 0 && t_lo <= p.stop_ns && p.stop_ns < t_hi);
  const bool timer = AT(p.node_tnext, g, p.NT) < t_hi;
  uint32_t xn = 0;
  if (x_active) xn = AT(p.seg_off, g + 1, p.NT + 1) - AT(p.seg_off, g, p.NT + 1);
  if (!flag && !has_ss && !timer) return;  // nothing in the window (scan_node returns too)
  if (!flag || has_ss || timer || xn || !spec || deg > p.cap_arr ||
      !p.impl || !p.eslot || p.delay_mode != BCSIM_DELAY_FIXED) {
    if (tid == 0) {
      AT(p.act, 2ull * p.NT + gadd_r(&p.act_n[2], 1u), 4ull * p.NT) = g;
      if (wep) AT(p.l2mark, g, p.NT) = wep;
      FDBG(!flag ? 0 : has_ss ? 1 : timer ? 2 : xn ? 3 : (deg > kFastLanes * kFastRPL || deg > p.cap_arr) ? 4 : 5);
    }
    return;
  }
  FPH(0);
  // The implicit echoes (pbft-node.cc:175: every delivery goes back out on the reverse edge,
  // occupying it) are applied here, on the link words of the node's out-edges, when no op of
  // the node is due in the window apart from the ones this scan creates -- those are due
  // app_delay after the arrivals, so they follow the echoes in key order (t, then t - dt).
  // The link kernels then skip the echoes of this window (eapp stamp) instead of reading the
  // row a second time; otherwise they do them, merged with the due ops, as before.
  // With descriptors (p.desc) the echoes are not applied here but recorded as one pending echo
  // descriptor {t, big} + the bitmap of the arrivals' in-slots, which the node's next link
  // stage that walks its edges applies before anything else (k_link_mesh: it loads and stores
  // those link words anyway) -- unless kEDesc descriptors are pending: then the link stage
  // does the echoes of this window from the row (no eapp stamp), after the pending ones.
  const bool echo_here = p.echo && p.qmodel == 0 && onext0 >= t_hi && !(sfv0 & (1u | kSfD0)) && !(sfv1 & (2u | kSfD1));
  const bool echo_dir = echo_here && !p.desc;
  if (!BCSIM_SCANPBFT_SPEC) row_loads();
  // the link words of its out-edges (LDS; used by the echo pass at the end)
  if (echo_dir) {
    const uint64_t* lrow = p.link + edge_loc(p, rep, e0);
    uint64_t lv[kFastRPL];
#pragma unroll
    for (uint32_t j = 0; j < kFastRPL; ++j) lv[j] = gbl(lrow)[min(j * kFastLanes + tid, deg - 1u)];  // (as the row)
#pragma unroll
    for (uint32_t j = 0; j < kFastRPL; ++j) F.lw[j * kFastLanes + tid] = lv[j];
  }
  if (tid == 0) {
    F.bad = 0;
    F.npp = 0;
    F.kmin = ~0ull;
    F.kmax = 0ull;
  }
  if (tid < kFastKeys) F.tkey[tid] = 0;
  if (tid < 4) F.tcount[tid] = 0;
  if (tid < 2) F.ocnt[tid] = 0;
  if (tid == 0) {
    F.fmin = ~0u;
    F.fmax = 0u;
    F.bigs = 0u;
  }
  for (uint32_t k = tid; k < kFastSeg * kFastKeys; k += kFastLanes) (&F.qc[0][0])[k] = 0;
  __syncthreads();
  const uint32_t tag = cell_tag(p, cell);
  const uint64_t lt = (1ull << lane) - 1ull;
  // (the frame times in scalar registers: indexed by a lane's flag they were a vector load per
  // record, each waited for before the next)
  const int64_t txl0 = p.tx_last[0], txl1 = p.tx_last[1], txt0 = p.tx_tot[0], txt1 = p.tx_tot[1];
  auto key_of = [&](const uint4& r, uint32_t k) -> unsigned long long {
    const uint32_t dt = static_cast<uint32_t>(prop_of_slot(p, e0 + k) + (((r.w >> 24) & RF_BIG) ? txl1 : txl0));
    return (static_cast<unsigned long long>(r.x) << 32) | static_cast<uint32_t>(~dt);
  };
  // ---- pass 1: window membership, message types and indices, quorum group counts, key range ----
  uint32_t vmask = 0;  // bit j: slot j * 512 + tid holds an arrival of the window
  bool bad = false;
  unsigned long long kmn = ~0ull, kmx = 0ull;
#pragma unroll
  for (uint32_t j = 0; j < kFastRPL; ++j) {
    const uint32_t k = j * kFastLanes + tid;
    const uint4 r = rv[j];
    const long long t = cs + r.x;
    const bool v = k < deg && slot_live(r.w >> 24, tag) && t >= t_lo && t < t_hi;
    uint32_t w = 0;
    if (v) {
      vmask |= 1u << j;
      const unsigned long long key = key_of(r, k);
      kmn = min(kmn, key);
      kmx = max(kmx, key);
      const uint32_t type = fr_type(r);
      const int32_t idx = c2i(fr_m2(r));
      const bool inr = idx >= 0 && static_cast<uint32_t>(idx) < p.pbft_seq_cap;
      if (type == PB_PRE_PREPARE) {
        const uint32_t q = inr ? atomicAdd(&F.npp, 1u) : kFastPP;
        if (q < kFastPP) {
          F.pp_k[q] = k;
          F.pp_idx[q] = idx;
          F.pp_val[q] = c2i(fr_m3(r));
        } else {
          bad = true;
        }
      } else if (type == PB_PREPARE_RES || type == PB_COMMIT) {
        if (!inr) bad = true;
        else w = fr_group(r);
      } else if (type != PB_PREPARE) {
        bad = true;  // VIEW_CHANGE / "Wrong msg": the generic path
      }
    }
    unsigned long long rem = __ballot(w != 0);
    while (rem) {
      const int ld = __ffsll(static_cast<long long>(rem)) - 1;
      const uint32_t wl = __shfl(w, ld, 64);
      const unsigned long long same = __ballot(w == wl);
      if (lane == static_cast<uint32_t>(ld)) {
        const uint32_t s = fast_key_slot(F, wl);
        if (s < kFastKeys) F.qc[j * kFastWaves + wv][s] = static_cast<uint32_t>(__popcll(same));
      }
      rem &= ~same;
    }
  }
  for (int d = 32; d > 0; d >>= 1) {
    kmn = min(kmn, static_cast<unsigned long long>(__shfl_xor(kmn, d, 64)));
    kmx = max(kmx, static_cast<unsigned long long>(__shfl_xor(kmx, d, 64)));
  }
  if (lane == 0) {
    atomicMin(&F.kmin, kmn);
    atomicMax(&F.kmax, kmx);
  }
  if (bad) F.bad = 1;
  __syncthreads();
  FPH(1);
  // group bases: the stored vote counters, then the segments in arrival order
  const size_t base = static_cast<size_t>(g) * p.pbft_seq_cap;
  if (tid < kFastKeys) {
    const uint32_t wl = F.tkey[tid];
    if (wl) {
      const uint32_t idx = wl & kIdxMask;
      uint32_t run = static_cast<uint32_t>((wl >> 30) == 1u ? AT(p.tx_pv, base + idx, p.cap_txn)
                                                            : AT(p.tx_cv, base + idx, p.cap_txn));
      for (uint32_t s = 0; s < kFastSeg; ++s) {
        const uint32_t c = F.qc[s][tid];
        F.qc[s][tid] = run;
        run += c;
      }
      F.tcnt[tid] = run;
    }
  }
  __syncthreads();
  // uniform: several instants in the window (the slot order may not be the key order), or
  // anything else the generic path must take -- nothing has been written
  if (F.bad || F.kmin != F.kmax) {
    if (tid == 0) {
      AT(p.act, 2ull * p.NT + gadd_r(&p.act_n[2], 1u), 4ull * p.NT) = g;
      if (wep) AT(p.l2mark, g, p.NT) = wep;
      FDBG(F.bad ? 6 : 7);
    }
    return;
  }
  FPH(2);
  const int32_t N = static_cast<int32_t>(p.N);
  const uint32_t T1 = static_cast<uint32_t>(N / 2), T2 = T1 + 1;
  // ---- pass 2: quorum crossings; per-segment counts of the flagged arrivals ----
  uint32_t xmask = 0;  // bit j: the arrival crosses its quorum
#pragma unroll
  for (uint32_t j = 0; j < kFastRPL; ++j) {
    const uint4 r = rv[j];
    const bool v = (vmask >> j) & 1u;
    const uint32_t w = v ? fr_group(r) : 0u;
    unsigned long long rem = __ballot(w != 0);
    while (rem) {
      const int ld = __ffsll(static_cast<long long>(rem)) - 1;
      const uint32_t wl = __shfl(w, ld, 64);
      const unsigned long long same = __ballot(w == wl);
      if (w == wl) {
        const uint32_t vv = F.qc[j * kFastWaves + wv][fast_key_find(F, wl)] + static_cast<uint32_t>(__popcll(same & lt)) + 1u;
        if ((wl >> 30) == 1u ? (vv % T1 == 0) : (vv % T2 == 0)) xmask |= 1u << j;
      }
      rem &= ~same;
    }
    const uint32_t type = fr_type(r);
    const bool cross = (xmask >> j) & 1u;
    const unsigned long long mp = __ballot(v && type == PB_PREPARE);
    const unsigned long long md = __ballot(v && (type == PB_PRE_PREPARE || (type == PB_PREPARE_RES && cross)));
    const unsigned long long mc = __ballot(v && type == PB_COMMIT && cross);
    const unsigned long long mv = __ballot(v);
    if (p.desc) {  // descriptor checks: one reply payload over the PREPAREs, one frame size
      if (mp) {
        const int fl = __ffsll(static_cast<long long>(mp)) - 1;
        const uint32_t f01 = static_cast<uint32_t>(static_cast<uint16_t>(to16(p, fr_f0(r)))) |
                             (static_cast<uint32_t>(static_cast<uint16_t>(to16(p, fr_m2(r)))) << 16);
        const uint32_t ref = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(f01), fl));
        const unsigned long long dif = __ballot(v && type == PB_PREPARE && f01 != ref);
        if (lane == 0) {
          atomicMin(&F.fmin, dif ? 0u : ref);
          atomicMax(&F.fmax, dif ? ~0u : ref);
        }
      }
      const unsigned long long mb = __ballot(v && ((r.w >> 24) & RF_BIG));
      if (lane == 0 && mv) atomicOr(&F.bigs, (mb ? 1u : 0u) | (mb != mv ? 2u : 0u));
    }
    if (lane == 0)
      F.seg[j * kFastWaves + wv] = make_uint4(static_cast<uint32_t>(__popcll(mp)), static_cast<uint32_t>(__popcll(md)),
                                              static_cast<uint32_t>(__popcll(mc)), static_cast<uint32_t>(__popcll(mv)));
  }
  // write back the vote counters (tx[idx].prepare_vote / commit_vote)
  if (tid < kFastKeys) {
    const uint32_t wl = F.tkey[tid];
    if (wl) {
      const uint32_t idx = wl & kIdxMask;
      if ((wl >> 30) == 1u)
        AT(p.tx_pv, base + idx, p.cap_txn) = static_cast<int32_t>(F.tcnt[tid] % T1);
      else
        AT(p.tx_cv, base + idx, p.cap_txn) = static_cast<int32_t>(F.tcnt[tid] % T2);
    }
  }
  __syncthreads();
  FPH(3);
  // exclusive segment bases (wave 0: one segment per lane); totals to every lane
  uint4 tot;
  {
    const uint4 x = lane < kFastSeg ? F.seg[lane] : make_uint4(0, 0, 0, 0);
    uint4 in = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t a = __shfl_up(in.x, off, 64), bq = __shfl_up(in.y, off, 64);
      const uint32_t c = __shfl_up(in.z, off, 64), d = __shfl_up(in.w, off, 64);
      if (lane >= static_cast<uint32_t>(off)) {
        in.x += a;
        in.y += bq;
        in.z += c;
        in.w += d;
      }
    }
    // (wave-uniform: readlane puts the totals in scalar registers)
    tot = make_uint4(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(in.x), 63)),
                     static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(in.y), 63)),
                     static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(in.z), 63)),
                     static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(in.w), 63)));
    __syncthreads();  // every wave has read its totals before wave 0 overwrites the counts
    if (wv == 0 && lane < kFastSeg) F.seg[lane] = make_uint4(in.x - x.x, in.y - x.y, in.z - x.z, in.w - x.w);
  }
  const uint32_t sub0 = AT(p.sub, g, p.NT), nops0 = AT(p.n_ops, g, p.NT);
  const int32_t bn0 = AT(p.block_num, g, p.NT);
  // descriptors (uniform): the echoes of the window (one instant, one frame size), and the
  // replies when every arrival is a PREPARE with one reply payload (one due instant, subs
  // sub0 + rank) and the arrival cell's descriptor is free (none, or one already sent)
  // (re-read here, not kept live across the passes: the pending echo count, the slot flags)
  const uint32_t ne0 = p.desc ? AT(p.en, g, p.NT) : 0u;
  const bool echo_desc = p.desc && echo_here && ne0 < kEDesc && F.bigs != 3u;
  bool rdesc_on = false;
  if (p.desc && tot.x == tot.w && tot.x != 0 && F.fmin == F.fmax) {
    rdesc_on = !(AT(p.sflag, static_cast<size_t>(cell % kOpRing) * p.NT + g, static_cast<uint64_t>(kOpRing) * p.NT) & kSfD);
    if (!rdesc_on) {
      const uint4 od = gld4(p.rdesc + static_cast<size_t>(cell % kOpRing) * p.NT + g);
      rdesc_on = static_cast<long long>((static_cast<uint64_t>(od.y) << 32) | od.x) < t_lo;
    }
  }
  if (nops0 + tot.y > op_cap(p, g)) {
    if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
    return;
  }
  __syncthreads();
  FPH(4);
  // ---- pass 3: outputs, every arrival with its counter values from the bases + popcounts ----
  Op* ops = p.ops + op_base(p, g);
  const int64_t app = p.app_delay;
  const int64_t tk0 = ((t_lo + p.pbft_period - 1) / p.pbft_period) * p.pbft_period;
  const uint32_t deg_u = deg;
  uint32_t n_slot0 = 0, n_slot1 = 0, cnt_t[4] = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t j = 0; j < kFastRPL; ++j) {
    const uint4 r = rv[j];
    const bool v = (vmask >> j) & 1u;
    const uint32_t type = fr_type(r);
    const bool cross = (xmask >> j) & 1u;
    const unsigned long long mp = __ballot(v && type == PB_PREPARE);
    const unsigned long long md = __ballot(v && (type == PB_PRE_PREPARE || (type == PB_PREPARE_RES && cross)));
    const unsigned long long mc = __ballot(v && type == PB_COMMIT && cross);
    if (!v) continue;
    const uint4 sb = F.seg[j * kFastWaves + wv];
    const uint32_t np = sb.x + static_cast<uint32_t>(__popcll(mp & lt));
    const uint32_t nd = sb.y + static_cast<uint32_t>(__popcll(md & lt));
    const uint32_t nc = sb.z + static_cast<uint32_t>(__popcll(mc & lt));
    const uint32_t sp = sub0 + np + nd * deg_u, op = nops0 + nd;
    const uint32_t k = j * kFastLanes + tid;
    const uint32_t q = e0 + k;  // in-slot = the reverse (reply) edge
    const uint32_t dt = ~static_cast<uint32_t>(F.kmax);  // (every arrival has the one key)
    const int64_t t = cs + static_cast<int64_t>(r.x);
    const uint32_t origin = p.mesh ? (k < i ? k : k + 1) : AT(p.col, q, p.E);
    const Key key{t, t - static_cast<int64_t>(dt), origin, r.y};
    if (t >= tk0 && (t == tk0 || (t - tk0) % p.pbft_period == 0) && key.ts <= t - p.pbft_period)
      set_err(p, BCSIM_E_TIE);  // arrival ordered before a same-time tick
    const int32_t m1 = fr_f0(r), m2 = fr_m2(r);
    if (type == PB_PRE_PREPARE) {  // :193-211
      ++cnt_t[0];
      st_op(&ops[op], mk_op(p, t + app, static_cast<uint32_t>(app), i, sp, 0, mkmsg(PB_PREPARE, m1, m2, fr_m3(r), 0),
                            OP_BCAST, 0));
    } else if (type == PB_PREPARE) {  // :212-222, the reply into its edge's slot of this arrival cell
      ++cnt_t[1];
      const int64_t due = t + app;
      const uint64_t ut = static_cast<uint64_t>(due);
      if (!rdesc_on)
        gst4(eslot_at(p, static_cast<uint32_t>(cell % kOpRing), rep, q),
             make_uint4(static_cast<uint32_t>(ut), static_cast<uint32_t>(ut >> 32), sp,
                        static_cast<uint32_t>(static_cast<uint16_t>(to16(p, m1))) |
                            (static_cast<uint32_t>(static_cast<uint16_t>(to16(p, m2))) << 16)));
      if (due < cs + p.L)  // (due >= t >= cs: the arrival cell, without a 64-bit division)
        ++n_slot0;
      else
        ++n_slot1;
    } else if (type == PB_PREPARE_RES) {  // :223-240
      ++cnt_t[3];
      if (cross)
        st_op(&ops[op], mk_op(p, t + app, static_cast<uint32_t>(app), i, sp, 0, mkmsg(PB_COMMIT, m1, m2, 0, 0), OP_BCAST, 0));
    } else {  // PB_COMMIT :241-265
      ++cnt_t[2];
      if (cross) {
        const int32_t idx = c2i(m2);
        int32_t val = 0, best = -1;  // tx[idx].val as of this event
        for (uint32_t u = 0; u < F.npp; ++u)
          if (F.pp_idx[u] == idx && F.pp_k[u] < k && static_cast<int32_t>(F.pp_k[u]) > best) {
            best = static_cast<int32_t>(F.pp_k[u]);
            val = F.pp_val[u];
          }
        if (best < 0) val = AT(p.tx_val, base + idx, p.cap_txn);
        emit_trace(p, key, rep, i, BCSIM_TR_PBFT_COMMIT, INT32_MIN, bn0 + static_cast<int32_t>(nc), val);
      }
    }
  }
  FPH(5);
  if (echo_dir) {  // one link word per arrival (distinct in-slots = distinct out-edges), coalesced
    uint64_t* lrow = p.link + edge_loc(p, rep, e0);
#pragma unroll
    for (uint32_t j = 0; j < kFastRPL; ++j) {
      if (!((vmask >> j) & 1u)) continue;
      const uint4 r = rv[j];
      const uint64_t lw = F.lw[j * kFastLanes + tid];
      const int64_t t = cs + static_cast<int64_t>(r.x);
      const int64_t bu0 = static_cast<int64_t>(lw >> 16);
      const int64_t bu = (bu0 > t ? bu0 : t) + (((r.w >> 24) & RF_BIG) ? txt1 : txt0);
      if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
      gbl(lrow)[j * kFastLanes + tid] = (static_cast<uint64_t>(bu) << 16) | (lw & 0xFFFFull);
    }
  }
  if (rdesc_on || echo_desc) {  // descriptor bitmaps: bit k = in-slot k holds an arrival
    uint32_t* rb = p.rbits + (static_cast<size_t>(cell % kOpRing) * p.NT + g) * p.dwords;
    uint32_t* eb = p.ebits + (static_cast<size_t>(g) * kEDesc + ne0) * p.dwords;
#pragma unroll 1
    for (uint32_t j = 0; j < kFastRPL; ++j) {
      const unsigned long long mv = __ballot((vmask >> j) & 1u);
      const uint32_t w0 = j * (kFastLanes / 32) + wv * 2 + lane;
      if (lane < 2 && w0 < p.dwords) {
        const uint32_t word = static_cast<uint32_t>(mv >> (32 * lane));
        if (rdesc_on) gbl(rb)[w0] = word;
        if (echo_desc) gbl(eb)[w0] = word;
      }
    }
  }
#pragma unroll
  for (int t4 = 0; t4 < 4; ++t4) {
    const uint32_t s = wave_sum(cnt_t[t4]);
    if (lane == 0 && s) atomicAdd(&F.tcount[t4], s);
  }
  {
    const uint32_t s0 = wave_sum(n_slot0), s1 = wave_sum(n_slot1);
    if (lane == 0) {
      if (s0) atomicAdd(&F.ocnt[0], s0);
      if (s1) atomicAdd(&F.ocnt[1], s1);
    }
  }
  __syncthreads();
  FPH(6);
  // ---- tx[n].val of the window's PRE_PREPAREs (the last one per index wins) ----
  for (uint32_t u = tid; u < F.npp; u += kFastLanes) {
    bool last = true;
    for (uint32_t u2 = 0; u2 < F.npp; ++u2)
      if (F.pp_idx[u2] == F.pp_idx[u] && F.pp_k[u2] > F.pp_k[u]) last = false;
    if (last) AT(p.tx_val, base + F.pp_idx[u], p.cap_txn) = F.pp_val[u];
  }
  // slot replies make their cells busy and flag this node for k_link
  if (tid < 2 && F.ocnt[tid]) mark_busy(&p.bucket_cnt[(cell + tid) % p.n_buckets]);
  if (tid != 0) return;
  const uint32_t sm = (F.ocnt[0] ? 1u : 0u) | (F.ocnt[1] ? 2u : 0u);
  if (sm) {
    uint8_t& f = AT(p.sflag, (cell % kOpRing) * p.NT + g, static_cast<uint64_t>(kOpRing) * p.NT);
    if (rdesc_on) {  // kSfD0 / kSfD1: the descriptor's replies are due in this cell / the next
      const uint64_t ud = static_cast<uint64_t>(cs + static_cast<long long>(F.kmax >> 32) + app);
      gst4(p.rdesc + static_cast<size_t>(cell % kOpRing) * p.NT + g,
           make_uint4(static_cast<uint32_t>(ud), static_cast<uint32_t>(ud >> 32), sub0, F.fmin));
      f = static_cast<uint8_t>((f & ~kSfD) | (sm << 4));
    } else {
      f = static_cast<uint8_t>(f | sm);
    }
  }
  AT(p.sub, g, p.NT) = sub0 + tot.x + tot.y * deg_u;
  AT(p.n_ops, g, p.NT) = nops0 + tot.y;
  // the new ops are all due at t + app_delay (one instant): the earliest pending op stays exact,
  // so a link stage with nothing due can skip the node (k_link_mesh)
  if (tot.y) {
    const long long on = AT(p.node_onext, g, p.NT);  // (re-read: not kept live across the passes)
    AT(p.node_onext, g, p.NT) = on == LLONG_MIN ? LLONG_MIN : min(on, cs + static_cast<long long>(F.kmax >> 32) + app);
  }
  AT(p.block_num, g, p.NT) = bn0 + static_cast<int32_t>(tot.z);
  FPH(7);
  if (echo_desc) {
    const uint64_t ut = static_cast<uint64_t>(cs + static_cast<long long>(F.kmax >> 32));
    gst4(p.edesc + static_cast<size_t>(g) * kEDesc + ne0,
         make_uint4(static_cast<uint32_t>(ut), static_cast<uint32_t>(ut >> 32), F.bigs == 1u ? 1u : 0u, 0u));
    AT(p.en, g, p.NT) = static_cast<uint8_t>(ne0 + 1);
  }
  if (echo_dir || echo_desc) {
    AT(p.eapp, g, p.NT) = t_lo;
    if (tot.w) gadd(&kst_stripe(p)[KST_ECHO], static_cast<unsigned long long>(tot.w));
  }
  unsigned long long* cnt = cnt_stripe(p, rep);
  const uint32_t type_of[4] = {PB_PRE_PREPARE, PB_PREPARE, PB_COMMIT, PB_PREPARE_RES};
  for (int t4 = 0; t4 < 4; ++t4)
    if (F.tcount[t4]) gadd(&cnt[CNT_DELIV + type_of[t4]], static_cast<unsigned long long>(F.tcount[t4]));
  const unsigned long long n = tot.w;
  if (n) {
    gadd(&cnt[CNT_DELIV_TOTAL], n);
    if (p.echo) gadd(&cnt[CNT_ECHOES], n);
    gadd(&kst_stripe(p)[KST_DELIV], n);
    gadd(&cnt[CNT_EVENTS], n);
    // every arrival is at one instant: t = cs + t_off of any of them
    __hip_atomic_fetch_max(gbl(reinterpret_cast<long long*>(&cnt[CNT_TLAST])), cs + static_cast<long long>(F.kmax >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------
// k_scan_rt (summary mode): the PBFT scan of a window, one workgroup per
// 64-receiver tile (lane = receiver d), its 16 waves over the senders in chunks of 64.  A chunk
// is two coalesced loads of the tile's summary entries (lane = sender) and the explicit-slot
// bytes; a 64 x 64 bit transpose turns the senders' receiver masks into each receiver's
// arrival bits, and the senders whose slots are explicit are loaded per receiver.  A receiver
// whose window holds arrivals of ONE message (type, payload) at ONE instant -- the heavy waves:
// PRE_PREPARE, the PREPAREs, the PREPARE_RES replies of one sequence, the COMMITs of one
// sequence -- is handled here with the same state changes and outputs as k_scan_pbft
// (pbft-node.cc:193-265): its quorum crossings are the ranks where the stored vote count plus
// the rank reaches a multiple of the threshold, so only a COMMIT crossing needs its sender
// (commit trace key).  Any other receiver with work is materialised (its summary records
// written as slot records, their mask bits cleared) and goes to list 2 for the generic kernel,
// as do receivers whose echoes the link stage must do from the row.  mode 1: materialise
// every receiver with work, nothing else (before a generic scan of list 0).
constexpr uint32_t kRtWaves = 16, kRtWords = 8;  // N <= 4096: four 64-sender chunks per wave
struct RtShared {
  uint32_t bits[kRtWaves][kRtWords][64];  // per wave: the receiver's arrival bits of its senders
  uint32_t cnt[kRtWaves][64];
  uint32_t ftof[kRtWaves][64], fw2[kRtWaves][64], fw3[kRtWaves][64];  // the first arrival's words
  uint32_t fl[kRtWaves][64];  // bit 0: has arrivals, bit 1: not one message / instant
  uint32_t st[64];            // receiver status (below)
  uint32_t ne[64];            // pending echo descriptors (the ebits row it writes)
  unsigned long long any, mat;
  uint32_t tcount[4];  // deliveries: PRE_PREPARE, PREPARE, COMMIT, PREPARE_RES
  uint32_t echo, l2;
  long long tlast;
};
enum : uint32_t { kRtWork = 1u, kRtFast = 2u, kRtEchoHere = 4u, kRtEchoDesc = 8u, kRtMat = 16u, kRtGen = 32u,
                  kRtRbits = 64u, kRtEbits = 128u };

// lane k holds row k (bit j: column j) of a 64 x 64 bit matrix; returns column `lane` (bit k: row k's bit lane)
__device__ inline unsigned long long transpose64(unsigned long long x, uint32_t lane) {
#pragma unroll
  for (int st = 0; st < 6; ++st) {
    const uint32_t sh = 32u >> st;
    const unsigned long long m = st == 0 ? 0x00000000FFFFFFFFull
                                 : st == 1 ? 0x0000FFFF0000FFFFull
                                 : st == 2 ? 0x00FF00FF00FF00FFull
                                 : st == 3 ? 0x0F0F0F0F0F0F0F0Full
                                 : st == 4 ? 0x3333333333333333ull
                                           : 0x5555555555555555ull;
    const unsigned long long o = static_cast<unsigned long long>(__shfl_xor(x, static_cast<int>(sh), 64));
    x = (lane & sh) ? ((x & ~m) | ((o & ~m) >> sh)) : ((x & m) | ((o & m) << sh));
  }
  return x;
}

__global__ __launch_bounds__(1024) void k_scan_rt(const KP* __restrict__ pk, long long cell, long long t_lo, long long t_hi,
                                                  long long cs, int x_active, uint32_t wep, int mode) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ RtShared S;
  const uint32_t N = p.N, nrt = p.n_tiles;
  const uint32_t rep = blockIdx.x / nrt, rt = blockIdx.x % nrt;
  const uint32_t tid = tidx(), lane = tid & 63u, wv = tid >> 6;
  const uint32_t d = rt * 64u + lane;
  const bool dv = d < N;
  const uint32_t g = rep * N + (dv ? d : 0u);
  const uint32_t B = p.n_buckets, b = static_cast<uint32_t>(cell % B), tag = cell_tag(p, cell);
  const uint32_t ob = static_cast<uint32_t>(cell % kOpRing), obp = static_cast<uint32_t>((cell + kOpRing - 1) % kOpRing);
  const size_t R4 = static_cast<uint64_t>(kOpRing) * p.NT;
  // ---- wave 0: the receivers' k_scan_pbft checks ----
  if (wv == 0) {
    uint32_t st = 0;
    if (dv) {
      const bool flag = node_flagged_w(p, b, g, rep, d, t_hi);
      const bool has_ss = (t_lo <= 0 && 0 < t_hi) || (p.stop_ns >= 0 && t_lo <= p.stop_ns && p.stop_ns < t_hi);
      const bool timer = AT(p.node_tnext, g, p.NT) < t_hi;
      const uint32_t xn = x_active ? AT(p.seg_off, g + 1, p.NT + 1) - AT(p.seg_off, g, p.NT + 1) : 0u;
      const long long onext0 = AT(p.node_onext, g, p.NT);
      const uint8_t sfv0 = AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, R4);
      const uint8_t sfv1 = AT(p.sflag, static_cast<size_t>(obp) * p.NT + g, R4);
      const uint32_t ne0 = AT(p.en, g, p.NT);
      if (flag || has_ss || timer) {
        st = kRtWork;
        if (mode || !flag || has_ss || timer || xn || N - 1 > p.cap_arr) {
          st |= kRtGen | kRtMat;
        } else {
          st |= kRtFast;
          // the echo rule of k_scan_pbft: no op of the node due in the window but the ones this
          // scan creates (those follow the echoes in key order)
          if (p.echo && p.qmodel == 0 && onext0 >= t_hi && !(sfv0 & (1u | kSfD0)) && !(sfv1 & (2u | kSfD1)))
            st |= kRtEchoHere | (ne0 < kEDesc ? kRtEchoDesc : 0u);
        }
      }
      S.ne[lane] = ne0;
    }
    S.st[lane] = st;
    const unsigned long long any = __ballot(st != 0);
    if (lane == 0) {
      S.any = any;
      S.mat = 0ull;
      S.echo = 0u;
      S.l2 = 0u;
      S.tlast = LLONG_MIN;
    }
    if (lane < 4) S.tcount[lane] = 0u;
  }
  __syncthreads();
  if (!S.any) return;  // (uniform) no receiver of the tile has work
  const uint32_t nch = (N + 63u) / 64u, cpw = (nch + kRtWaves - 1u) / kRtWaves;
  // ---- all waves: each receiver's arrival bits and message words over this wave's senders ----
  if (!mode) {
    uint32_t cnt = 0, r_tof = 0, r_w2 = 0, r_w3 = 0;
    bool have = false, bad = false;
    auto take = [&](uint32_t tof, uint32_t w2, uint32_t w3) {
      if (!have) {
        have = true;
        r_tof = tof;
        r_w2 = w2;
        r_w3 = w3;
      } else if (tof != r_tof || w2 != r_w2 || w3 != r_w3) {
        bad = true;
      }
    };
    for (uint32_t c = 0; c < cpw; ++c) {
      const uint32_t ch = wv * cpw + c;
      unsigned long long col = 0ull;
      if (ch < nch) {  // (uniform)
        const uint32_t sb = ch * 64u + lane;  // this lane loads sender sb's entry
        const bool sv = sb < N;
        const size_t si = sum_idx(p, b, rep, rt, sv ? sb : 0u);
        const uint4 ea = sv ? gld4(p.msum + si * 2) : make_uint4(0, 0, 0, 0);
        const uint4 eb = sv ? gld4(p.msum + si * 2 + 1) : make_uint4(0, 0, 0, 0);
        const uint32_t xf = sv ? gbl(p.xsum)[si] : 0u;
        const long long ts = cs + static_cast<long long>(ea.z);
        const bool vs = (ea.x | ea.y) != 0u && slot_live(eb.y >> 24, tag) && ts >= t_lo && ts < t_hi;
        const unsigned long long vm = __ballot(vs);
        if (vm) {
          // one message over the chunk's entries of the window, or its receivers take the generic path
          const int rl = __ffsll(static_cast<long long>(vm)) - 1;
          const uint32_t c_tof = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ea.z), rl));
          const uint32_t c_w2 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(eb.x), rl));
          const uint32_t c_w3 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(eb.y), rl));
          const bool mixed = __ballot(vs && (ea.z != c_tof || eb.x != c_w2 || eb.y != c_w3)) != 0ull;
          col = transpose64(vs ? ((static_cast<unsigned long long>(ea.y) << 32) | ea.x) : 0ull, lane);
          if (col) {
            if (mixed) bad = true;
            take(c_tof, c_w2, c_w3);
          }
        }
        // the senders with explicit slot records for this tile: this receiver's slot of each
        unsigned long long xm = __ballot(sv && xf == (0x80u | tag));
        while (xm) {  // (uniform) four loads at a time
          int kx[4];
          uint4 rx[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            kx[u] = xm ? __ffsll(static_cast<long long>(xm)) - 1 : -1;
            if (xm) xm &= xm - 1ull;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t s = ch * 64u + static_cast<uint32_t>(kx[u] < 0 ? 0 : kx[u]);
            const bool ld = kx[u] >= 0 && dv && s != d;
            rx[u] = ld ? gld4(p.inbox + inbox_idx(p, b, rep, d * (N - 1) + (s < d ? s : s - 1))) : make_uint4(0, 0, 0, 0);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (kx[u] < 0) continue;
            const uint4 r = rx[u];
            const long long ta = cs + static_cast<long long>(r.x);
            if (slot_live(r.w >> 24, tag) && ta >= t_lo && ta < t_hi) {
              const unsigned long long bit = 1ull << kx[u];
              if (col & bit) bad = true;  // (a summary record and a slot record of one edge: cannot happen)
              col |= bit;
              take(r.x, r.z, r.w);
            }
          }
        }
      }
      S.bits[wv][2 * c][lane] = static_cast<uint32_t>(col);
      S.bits[wv][2 * c + 1][lane] = static_cast<uint32_t>(col >> 32);
      cnt += static_cast<uint32_t>(__popcll(col));
    }
    for (uint32_t j = 2 * cpw; j < kRtWords; ++j) S.bits[wv][j][lane] = 0u;
    S.cnt[wv][lane] = cnt;
    S.ftof[wv][lane] = r_tof;
    S.fw2[wv][lane] = r_w2;
    S.fw3[wv][lane] = r_w3;
    S.fl[wv][lane] = (have ? 1u : 0u) | (bad ? 2u : 0u);
  }
  __syncthreads();
  // ---- wave 0: per receiver, one message at one instant -> k_scan_pbft's outputs ----
  if (wv == 0) {
    uint32_t st = S.st[lane];
    uint32_t n = 0, tof = 0, w2 = 0, w3 = 0;
    bool have = false, bad = false;
    if (!mode && (st & kRtFast)) {
      for (uint32_t w = 0; w < kRtWaves; ++w) {
        const uint32_t f = S.fl[w][lane];
        n += S.cnt[w][lane];
        bad = bad || (f & 2u);
        if (f & 1u) {
          const uint32_t a = S.ftof[w][lane], bw = S.fw2[w][lane], cw = S.fw3[w][lane];
          if (!have) {
            have = true;
            tof = a;
            w2 = bw;
            w3 = cw;
          } else if (a != tof || bw != w2 || cw != w3) {
            bad = true;
          }
        }
      }
    }
    const uint4 r = make_uint4(tof, 0u, w2, w3);  // (the message's record words)
    const uint32_t type = fr_type(r);
    const int32_t idx = c2i(fr_m2(r));
    const bool inr = idx >= 0 && static_cast<uint32_t>(idx) < p.pbft_seq_cap;
    const size_t base = static_cast<size_t>(g) * p.pbft_seq_cap;
    if ((st & kRtFast) && n) {
      bool ok = !bad && inr;
      if (type == PB_PRE_PREPARE)
        ok = ok && n == 1;
      else if (type == PB_PREPARE_RES)
        ok = ok && c2i(fr_m3(r)) == 0;
      else if (type != PB_PREPARE && type != PB_COMMIT)
        ok = false;  // VIEW_CHANGE / "Wrong msg": the generic path
      if (ok && type == PB_PREPARE) {  // the replies as one descriptor: the arrival cell's must be free
        ok = !(AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, R4) & kSfD);
        if (!ok) {
          const uint4 od = gld4(p.rdesc + static_cast<size_t>(ob) * p.NT + g);
          ok = static_cast<long long>((static_cast<uint64_t>(od.y) << 32) | od.x) < t_lo;
        }
      }
      if (!ok) st = (st & ~kRtFast) | kRtGen | kRtMat;
    }
    if ((st & kRtFast) && n) {
      const int64_t t = cs + static_cast<int64_t>(tof);
      const int big = ((w3 >> 24) & RF_BIG) ? 1 : 0;
      const uint32_t dt = static_cast<uint32_t>(p.prop_const + (big ? p.tx_last[1] : p.tx_last[0]));
      const int64_t tk0 = ((t_lo + p.pbft_period - 1) / p.pbft_period) * p.pbft_period;
      if (t >= tk0 && (t == tk0 || (t - tk0) % p.pbft_period == 0) && t - static_cast<int64_t>(dt) <= t - p.pbft_period)
        set_err(p, BCSIM_E_TIE);  // arrival ordered before a same-time tick
      const uint32_t deg = N - 1;
      const int32_t NN = static_cast<int32_t>(N);
      const uint32_t T1 = static_cast<uint32_t>(NN / 2), T2 = T1 + 1;
      const uint32_t sub0 = AT(p.sub, g, p.NT), nops0 = AT(p.n_ops, g, p.NT);
      const int32_t bn0 = AT(p.block_num, g, p.NT);
      const int64_t app = p.app_delay;
      const int32_t m1 = fr_f0(r), m2 = fr_m2(r);
      Op* ops = p.ops + op_base(p, g);
      uint32_t nd = 0, np = 0, nc = 0;  // broadcasts (PRE_PREPARE, crossing PREPARE_RES), PREPAREs, commits
      if (type == PB_PRE_PREPARE) {  // :193-211
        nd = 1;
      } else if (type == PB_PREPARE) {  // :212-222
        np = n;
      } else if (type == PB_PREPARE_RES) {  // :223-240
        const uint32_t c0 = static_cast<uint32_t>(AT(p.tx_pv, base + idx, p.cap_txn));
        nd = (c0 + n) / T1;
        AT(p.tx_pv, base + idx, p.cap_txn) = static_cast<int32_t>((c0 + n) % T1);
      } else {  // PB_COMMIT :241-265
        const uint32_t c0 = static_cast<uint32_t>(AT(p.tx_cv, base + idx, p.cap_txn));
        nc = (c0 + n) / T2;
        AT(p.tx_cv, base + idx, p.cap_txn) = static_cast<int32_t>((c0 + n) % T2);
        if (nc) {
          const int32_t val = AT(p.tx_val, base + idx, p.cap_txn);
          for (uint32_t j = 0; j < nc; ++j) {
            // the crossing arrival: rank (j + 1) T2 - c0 - 1 among the window's, in sender order
            uint32_t rk = (j + 1) * T2 - c0 - 1, w = 0;
            for (; w < kRtWaves - 1 && rk >= S.cnt[w][lane]; ++w) rk -= S.cnt[w][lane];
            uint32_t jw = 0, word = 0;
            for (; jw < kRtWords; ++jw) {
              word = S.bits[w][jw][lane];
              const uint32_t pc = static_cast<uint32_t>(__popc(word));
              if (rk < pc) break;
              rk -= pc;
            }
            for (uint32_t u = 0; u < rk; ++u) word &= word - 1u;
            const uint32_t s = (w * cpw * 2u + jw) * 32u + static_cast<uint32_t>(__ffs(word) - 1);
            // its sub: the summary entry's base + d's out-edge index in s's row, or the slot record
            const size_t si = sum_idx(p, b, rep, rt, s);
            const uint4 ea = gld4(p.msum + si * 2), eb = gld4(p.msum + si * 2 + 1);
            const unsigned long long em = (static_cast<unsigned long long>(ea.y) << 32) | ea.x;
            uint32_t sub_s;
            if (slot_live(eb.y >> 24, tag) && ((em >> lane) & 1ull))
              sub_s = ea.w + (d < s ? d : d - 1u);
            else
              sub_s = gld4(p.inbox + inbox_idx(p, b, rep, d * (N - 1) + (s < d ? s : s - 1u))).y;
            const Key key{t, t - static_cast<int64_t>(dt), s, sub_s};
            emit_trace(p, key, rep, d, BCSIM_TR_PBFT_COMMIT, INT32_MIN, bn0 + static_cast<int32_t>(j), val);
          }
        }
      }
      if (nops0 + nd > op_cap(p, g)) {
        set_err(p, BCSIM_E_OVERFLOW);
        nd = 0;
      }
      for (uint32_t j = 0; j < nd; ++j) {
        const Msg m = type == PB_PRE_PREPARE ? mkmsg(PB_PREPARE, m1, m2, fr_m3(r), 0) : mkmsg(PB_COMMIT, m1, m2, 0, 0);
        st_op(&ops[nops0 + j], mk_op(p, t + app, static_cast<uint32_t>(app), d, sub0 + j * deg, 0, m, OP_BCAST, 0));
      }
      if (type == PB_PRE_PREPARE) AT(p.tx_val, base + idx, p.cap_txn) = c2i(fr_m3(r));
      if (np) {  // the replies: one descriptor {due, first sub, payload} + the bitmap (all waves, below)
        const int64_t due = t + app;
        const uint64_t ud = static_cast<uint64_t>(due);
        const uint32_t f01 = static_cast<uint32_t>(static_cast<uint16_t>(to16(p, m1))) |
                             (static_cast<uint32_t>(static_cast<uint16_t>(to16(p, m2))) << 16);
        gst4(p.rdesc + static_cast<size_t>(ob) * p.NT + g, make_uint4(static_cast<uint32_t>(ud), static_cast<uint32_t>(ud >> 32), sub0, f01));
        const uint32_t sm = due < cs + p.L ? 1u : 2u;  // due in the arrival cell or the next
        uint8_t& f = AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, R4);
        f = static_cast<uint8_t>((f & ~kSfD) | (sm << 4));
        mark_busy(&p.bucket_cnt[(cell + (sm == 1u ? 0 : 1)) % B]);
        st |= kRtRbits;
      }
      AT(p.sub, g, p.NT) = sub0 + np + nd * deg;
      AT(p.n_ops, g, p.NT) = nops0 + nd;
      if (nd) {
        const long long on = AT(p.node_onext, g, p.NT);
        AT(p.node_onext, g, p.NT) = on == LLONG_MIN ? LLONG_MIN : min(on, static_cast<long long>(t + app));
      }
      if (nc) AT(p.block_num, g, p.NT) = bn0 + static_cast<int32_t>(nc);
      if (st & kRtEchoDesc) {  // the echoes as one pending descriptor {t, big} + the bitmap (below)
        const uint32_t ne0 = S.ne[lane];
        const uint64_t ut = static_cast<uint64_t>(t);
        gst4(p.edesc + static_cast<size_t>(g) * kEDesc + ne0,
             make_uint4(static_cast<uint32_t>(ut), static_cast<uint32_t>(ut >> 32), big ? 1u : 0u, 0u));
        AT(p.en, g, p.NT) = static_cast<uint8_t>(ne0 + 1);
        AT(p.eapp, g, p.NT) = t_lo;
        st |= kRtEbits;
        atomicAdd(&S.echo, n);
      } else {
        st |= kRtMat;  // the link stage does the echoes from the row
      }
      const uint32_t t4 = type == PB_PRE_PREPARE ? 0u : type == PB_PREPARE ? 1u : type == PB_COMMIT ? 2u : 3u;
      atomicAdd(&S.tcount[t4], n);
      atomicMax(&S.tlast, static_cast<long long>(t));
    } else if ((st & kRtFast) && (st & kRtEchoHere)) {
      AT(p.eapp, g, p.NT) = t_lo;  // no arrival in the window: no echo to leave to the link stage
    }
    S.st[lane] = st;
    const unsigned long long mat = __ballot((st & kRtMat) != 0u);
    // the receivers that leave for the generic kernel: list 2 (one atomic per workgroup)
    const unsigned long long gm = __ballot(!mode && (st & kRtGen));
    if (lane == 0) S.mat = mat;
    if (gm) {
      uint32_t pos0 = 0;
      if (lane == 0) pos0 = gadd_r(&p.act_n[2], static_cast<uint32_t>(__popcll(gm)));
      pos0 = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(pos0)));
      if (st & kRtGen) {
        AT(p.act, 2ull * p.NT + pos0 + static_cast<uint32_t>(__popcll(gm & ((1ull << lane) - 1ull))), 4ull * p.NT) = g;
        if (wep) AT(p.l2mark, g, p.NT) = wep;
      }
    }
  }
  __syncthreads();
  const uint32_t st = S.st[lane];
  // ---- all waves: the descriptor bitmaps in in-slot order (in-slot k of d = sender k < d ? k : k + 1) ----
  if (st & (kRtRbits | kRtEbits)) {
    const uint32_t dw = p.dwords;
    uint32_t* rb = p.rbits + (static_cast<size_t>(ob) * p.NT + g) * dw;
    uint32_t* eb = p.ebits + (static_cast<size_t>(g) * kEDesc + S.ne[lane]) * dw;
    const uint32_t nw = 2u * cpw;  // (this wave's sender words: in-slot words wv * nw .. + nw)
    for (uint32_t j = 0; j < nw; ++j) {
      const uint32_t m = wv * nw + j;
      if (m >= dw) break;
      const uint32_t sw = S.bits[wv][j][lane];
      const uint32_t nx = j + 1 < nw ? S.bits[wv][j + 1][lane] : (wv + 1 < kRtWaves ? S.bits[wv + 1][0][lane] : 0u);
      const uint32_t lo = 32u * m;
      const uint32_t keep = d <= lo ? 0u : (d >= lo + 32u ? ~0u : (1u << (d - lo)) - 1u);
      const uint32_t word = (sw & keep) | (((sw >> 1) | (nx << 31)) & ~keep);
      if (st & kRtRbits) gbl(rb)[m] = word;
      if (st & kRtEbits) gbl(eb)[m] = word;
    }
  }
  // ---- all waves: materialise the summary records of the receivers that need their rows ----
  const unsigned long long mat = S.mat;
  if (mat) {
    for (uint32_t c = 0; c < cpw; ++c) {
      const uint32_t ch = wv * cpw + c;
      if (ch >= nch) break;
      const uint32_t sb = ch * 64u + lane;
      const bool sv = sb < N;
      const size_t si = sum_idx(p, b, rep, rt, sv ? sb : 0u);
      const uint4 ea = sv ? gld4(p.msum + si * 2) : make_uint4(0, 0, 0, 0);
      const uint4 eb = sv ? gld4(p.msum + si * 2 + 1) : make_uint4(0, 0, 0, 0);
      const unsigned long long em = (static_cast<unsigned long long>(ea.y) << 32) | ea.x;
      const unsigned long long mm = (sv && slot_live(eb.y >> 24, tag)) ? (em & mat) : 0ull;
      if (mm) {  // the entry keeps the other receivers; the slots are explicit from now on
        if (static_cast<uint32_t>(mm)) atomicAnd(reinterpret_cast<uint32_t*>(p.msum + si * 2), ~static_cast<uint32_t>(mm));
        if (static_cast<uint32_t>(mm >> 32))
          atomicAnd(reinterpret_cast<uint32_t*>(p.msum + si * 2) + 1, ~static_cast<uint32_t>(mm >> 32));
        gbl(p.xsum)[si] = static_cast<uint8_t>(0x80u | tag);
      }
      unsigned long long sm = __ballot(mm != 0ull);
      while (sm) {  // (uniform) per sender with records to write: its receivers' slots
        const int k = __ffsll(static_cast<long long>(sm)) - 1;
        sm &= sm - 1ull;
        const uint32_t lo32 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(mm)), k));
        const uint32_t hi32 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(mm >> 32)), k));
        const unsigned long long mk = (static_cast<unsigned long long>(hi32) << 32) | lo32;
        if (!((mk >> lane) & 1ull) || !dv) continue;
        const uint32_t s = ch * 64u + static_cast<uint32_t>(k);
        const uint32_t tofk = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ea.z), k));
        const uint32_t basek = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ea.w), k));
        const uint32_t w2k = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(eb.x), k));
        const uint32_t w3k = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(eb.y), k));
        gst4(p.inbox + inbox_idx(p, b, rep, d * (N - 1) + (s < d ? s : s - 1u)),
             make_uint4(tofk, basek + (d < s ? d : d - 1u), w2k, w3k));
      }
    }
  }
  // ---- counters: one add per workgroup ----
  __syncthreads();
  if (tid == 0 && !mode) {
    unsigned long long* cnt = cnt_stripe(p, rep);
    const uint32_t type_of[4] = {PB_PRE_PREPARE, PB_PREPARE, PB_COMMIT, PB_PREPARE_RES};
    unsigned long long tot = 0;
    for (int t4 = 0; t4 < 4; ++t4)
      if (S.tcount[t4]) {
        gadd(&cnt[CNT_DELIV + type_of[t4]], static_cast<unsigned long long>(S.tcount[t4]));
        tot += S.tcount[t4];
      }
    if (tot) {
      gadd(&cnt[CNT_DELIV_TOTAL], tot);
      if (p.echo) gadd(&cnt[CNT_ECHOES], tot);
      gadd(&kst_stripe(p)[KST_DELIV], tot);
      gadd(&cnt[CNT_EVENTS], tot);
      __hip_atomic_fetch_max(gbl(reinterpret_cast<long long*>(&cnt[CNT_TLAST])), S.tlast, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (S.echo) gadd(&kst_stripe(p)[KST_ECHO], static_cast<unsigned long long>(S.echo));
  }
}

// ---------------------------------------------------------------------------
// k_paxos_scan (sparse layout, BCSIM_PAXOS): one LANE per active node.  A node whose window
// holds only acceptor requests (REQ_TICKET / REQ_PROPOSE / REQ_COMMIT, at most kPxCap, no
// timer, START or STOP due) is handled here in canonical key order exactly as the lane-0
// loop of scan_node does it (paxos_recv, paxos-node.cc:177-247): per arrival the echo op,
// the acceptor state of the message's decree, and the reply on the reverse edge with the
// node's next schedule counter and (jitter) counter-RNG draw.  Every other node of the
// list (proposers counting responses, START, timers, ...) is appended to list 2 for
// k_scan<PAXOS, true, LOOP>.  The lane keeps its window's keys in LDS and selects them in
// order (<= kPxCap^2 LDS reads).
constexpr int kPxCap = 8;
// The per-replica counters of one lane's acceptor window (arrivals, REQ_TICKET and REQ_PROPOSE
// among them, latest arrival): added once per wave when the wave's nodes are of one replica.
struct PxCnt {
  uint32_t rep, n, d0, d1;
  long long tmax;
};
__device__ __attribute__((always_inline)) inline void px_accept(const KP& p, uint32_t g, long long t_lo, long long t_hi,
                                                                long long cs, int x_active, bool can, bool jit,
                                                                uint64_t (*skey)[256], uint32_t (*sref)[256], uint32_t tid,
                                                                PxCnt& o) {
  {
    const uint32_t rep = g / p.N, i = g % p.N;
    bool fast = can && AT(p.node_tnext, g, p.NT) >= t_hi;
    uint32_t xb = 0, xn = 0;
    if (x_active) {
      xb = AT(p.seg_off, g, p.NT + 1);
      xn = AT(p.seg_off, g + 1, p.NT + 1) - xb;
    }
    const uint32_t e0 = AT(p.row, i, p.N + 1);
    uint32_t cnt = 0;
    for (uint32_t j = 0; fast && j < xn; ++j) {
      const XRec& x = p.xgrp[xb + j];
      const Rec r = x.r;
      const long long t = cs + r.t_off;
      if (!(t >= t_lo && t < t_hi)) continue;
      if (cnt == static_cast<uint32_t>(kPxCap) || r.type > PX_REQ_COMMIT || r.f2 < 0 ||
          static_cast<uint32_t>(r.f2) >= p.K || x.slot - e0 > 0xFFFFu) {
        fast = false;
        break;
      }
      const uint32_t dt = static_cast<uint32_t>(prop_of_slot(p, x.slot) + sel2(p.tx_last, (r.flags & RF_BIG) ? 1 : 0));
      skey[cnt][tid] = (static_cast<uint64_t>(r.t_off) << 32) | static_cast<uint32_t>(~dt);
      sref[cnt][tid] = ((x.slot - e0) << 16) | j;
      ++cnt;
    }
    uint32_t nops = 0, ocap = 0;
    if (fast) {
      nops = AT(p.n_ops, g, p.NT);
      ocap = op_cap(p, g);
      if (nops + 2 * cnt > ocap) fast = false;  // the generic path raises the overflow
    }
    if (!fast) {
      const uint32_t pos = gadd_r(&p.act_n[2], 1u);
      AT(p.act, 2ull * p.NT + pos, 4ull * p.NT) = g;
      return;
    }
    if (cnt == 0) return;  // only arrivals of a later window of this cell
    uint32_t sub = AT(p.sub, g, p.NT);
    uint64_t draws = AT(p.draws, g, p.NT);
    Op* ops = p.ops + op_base(p, g);
    long long tmax = LLONG_MIN;
    uint32_t d0 = 0, d1 = 0;
    uint32_t done = 0;
    for (uint32_t s2 = 0; s2 < cnt; ++s2) {
      uint32_t best = 0;
      bool have = false;
      for (uint32_t c2 = 0; c2 < cnt; ++c2) {  // next arrival in (t, ~dt, slot) order
        if (done & (1u << c2)) continue;
        if (!have || skey[c2][tid] < skey[best][tid] ||
            (skey[c2][tid] == skey[best][tid] && sref[c2][tid] < sref[best][tid])) {
          best = c2;
          have = true;
        }
      }
      done |= 1u << best;
      const XRec x = p.xgrp[xb + (sref[best][tid] & 0xFFFFu)];
      const uint32_t q = x.slot;
      const Rec r = x.r;
      const Msg m = rec_msg(r);
      const int64_t t = cs + r.t_off;
      const uint32_t dt = static_cast<uint32_t>(prop_of_slot(p, q) + sel2(p.tx_last, m.big));
      const uint32_t origin = AT(p.col, q, p.E);
      if (t > tmax) tmax = t;
      d0 += r.type == PX_REQ_TICKET ? 1u : 0u;
      d1 += r.type == PX_REQ_PROPOSE ? 1u : 0u;
      if (p.echo) AT(ops, nops++, ocap) = mk_op(p, t, dt, origin, r.sub, q, m, OP_ECHO, 0);
      int32_t* a = &AT(p.px, (static_cast<size_t>(g) * p.K + static_cast<uint32_t>(r.f2)) * 4,
                       static_cast<uint64_t>(p.NT) * p.K * 4);
      const int32_t tk = c2i(mch(m, 1));
      Msg rr;
      if (r.type == PX_REQ_TICKET) {  // :177-198
        if (tk > a[0]) {
          a[0] = tk;
          rr = mkmsg(PX_RES_TICKET, enc_raw(p, 0), a[1], m.f[2], 0);
        } else {
          rr = mkmsg(PX_RES_TICKET, enc_raw(p, 1), 0, m.f[2], 0);
        }
      } else if (r.type == PX_REQ_PROPOSE) {  // :199-221
        int32_t st = 1;
        if (tk == a[0]) {
          a[1] = mch(m, 2);
          a[2] = tk;
          st = 0;
        }
        rr = mkmsg(PX_RES_PROPOSE, enc_raw(p, st), 0, m.f[2], 0);
      } else {  // PX_REQ_COMMIT :222-247
        int32_t st = 1;
        if (tk == a[2] && mch(m, 2) == a[1]) {
          a[3] = 1;
          st = 0;
        }
        rr = mkmsg(PX_RES_COMMIT, enc_raw(p, st), 0, m.f[2], 0);
      }
      const int64_t d = jit ? delay_from_draw(p, ctr_rand(p.seed, rep, i, draws++)) : p.app_delay;
      AT(ops, nops++, ocap) = mk_op(p, t + d, static_cast<uint32_t>(d), i, sub++, q, rr, OP_SEND, 0);
    }
    AT(p.sub, g, p.NT) = sub;
    if (jit) AT(p.draws, g, p.NT) = draws;
    AT(p.n_ops, g, p.NT) = nops;
    AT(p.node_onext, g, p.NT) = LLONG_MIN;  // k_link recomputes
    o = PxCnt{rep, cnt, d0, d1, tmax};
  }
}
// v added to replica rep's counter idx (all 64 lanes call it): one atomic per wave when the
// wave's nonzero lanes are of one replica
__device__ inline void wave_cnt_add(const KP& p, uint32_t rep, uint32_t v, int idx) {
  const unsigned long long any = __ballot(v != 0);
  if (!any) return;
  const int first = __ffsll(static_cast<long long>(any)) - 1;
  const uint32_t r0 = __shfl(rep, first, 64);
  if (__ballot(v != 0 && rep != r0) == 0) {
    uint32_t sum = v;
    for (int d = 32; d > 0; d >>= 1) sum += __shfl_xor(sum, d, 64);
    if ((tidx() & 63u) == static_cast<uint32_t>(first)) atomicAdd(&cnt_stripe(p, r0)[idx], static_cast<unsigned long long>(sum));
  } else if (v) {
    atomicAdd(&cnt_stripe(p, rep)[idx], static_cast<unsigned long long>(v));
  }
}
__device__ inline void px_count_add(const KP& p, const PxCnt& o) {
  unsigned long long* cs_ = cnt_stripe(p, o.rep);
  const unsigned long long n = o.n, d2 = o.n - o.d0 - o.d1;
  if (o.d0) atomicAdd(&cs_[CNT_DELIV + PX_REQ_TICKET], static_cast<unsigned long long>(o.d0));
  if (o.d1) atomicAdd(&cs_[CNT_DELIV + PX_REQ_PROPOSE], static_cast<unsigned long long>(o.d1));
  if (d2) atomicAdd(&cs_[CNT_DELIV + PX_REQ_COMMIT], d2);
  atomicAdd(&cs_[CNT_DELIV_TOTAL], n);
  atomicAdd(&kst_stripe(p)[KST_DELIV], n);
  if (p.echo) atomicAdd(&cs_[CNT_ECHOES], n);
  atomicAdd(&cs_[CNT_EVENTS], n);
  atomicMax(reinterpret_cast<long long*>(&cs_[CNT_TLAST]), o.tmax);
}
__global__ __launch_bounds__(256) void k_paxos_scan(const KP* __restrict__ pk, long long cell, long long t_lo,
                                                    long long t_hi, long long cs, int x_active) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ uint64_t skey[kPxCap][256];
  __shared__ uint32_t sref[kPxCap][256];  // slot << 16 | index in the node's list segment
  const uint32_t tid = tidx();
  const uint32_t na = p.act_n[0];
  const bool has_start = (t_lo <= 0 && 0 < t_hi);
  const bool has_stop = (p.stop_ns >= 0 && t_lo <= p.stop_ns && p.stop_ns < t_hi);
  const bool jit = p.delay_mode != BCSIM_DELAY_FIXED;
  const bool can = !has_start && !has_stop && t_lo >= p.dbg_tmax && (!jit || p.rng_mode == BCSIM_RNG_COUNTER);
  // (the trip count is uniform over the workgroup, so the wave reduction below has every lane)
  for (uint32_t kb = blockIdx.x * blockDim.x; kb < na; kb += gridDim.x * blockDim.x) {
    const uint32_t k = kb + tid;
    PxCnt o{0, 0, 0, 0, LLONG_MIN};
    if (k < na) px_accept(p, p.act[k], t_lo, t_hi, cs, x_active, can, jit, skey, sref, tid, o);
    const unsigned long long any = __ballot(o.n != 0);
    if (!any) continue;
    const int first = __ffsll(static_cast<long long>(any)) - 1;
    const uint32_t r0 = __shfl(o.rep, first, 64);
    if (__ballot(o.n != 0 && o.rep != r0) == 0) {  // one replica: one lane adds the wave's sums
      uint32_t v = o.n | (o.d0 << 10) | (o.d1 << 20);  // <= 64 * kPxCap per field
      long long tm = o.tmax;
      for (int d = 32; d > 0; d >>= 1) {
        v += __shfl_xor(v, d, 64);
        tm = max(tm, static_cast<long long>(__shfl_xor(tm, d, 64)));
      }
      if ((tid & 63u) == static_cast<uint32_t>(first))
        px_count_add(p, PxCnt{r0, v & 1023u, (v >> 10) & 1023u, (v >> 20) & 1023u, tm});
    } else if (o.n) {
      px_count_add(p, o);
    }
  }
}

// ---------------------------------------------------------------------------
// k_gossip_scan (dense layout, BCSIM_GOSSIP, degree <= 64): the common window of a gossip
// node -- only main-slot arrivals, no timer, START or STOP due, no extras -- handled by a
// group of G lanes (lane j = in-slot j) instead of a workgroup with a lane-0 event loop.
// Same result as scan_node<BCSIM_GOSSIP> (gossip_first_flags + gossip_recv in key order):
//   rank   = position of the arrival in the canonical key order (t, t - dt, origin)
//   first  = GS_BLOCK, not seen before the window, no earlier arrival of the window with
//            the same sequence -> GOSSIP_DELIVER trace + one broadcast (sub += deg each)
// The kernel walks all of this rank's gnodes (no k_active): a node with work in the window
// (k_active's rule) that is not simple is appended to list 2 for k_scan<.., LOOP>.
// The dense-gossip scan of one workgroup's node groups; returns true for a lane whose node the
// generic k_scan must take (appended to list 2).
// node k of the dense-gossip walk: the k-th gnode of this rank, or (fl) the k-th entry of the
// window's frontier list (list 0, built by k_gossip_active)
__device__ inline uint32_t gossip_gnode(const KP& p, uint32_t k, bool fl) {
  return fl ? AT(p.act, k, 4ull * p.NT) : (k / p.nloc) * p.N + p.nlo + k % p.nloc;
}
__device__ __attribute__((always_inline)) inline bool gossip_scan_body(const KP* __restrict__ pk, long long cell,
                                                                       long long t_lo, long long t_hi, long long cs,
                                                                       int x_active, uint32_t G, int loop, bool fl) {
  const KP& p = *pk;
  __shared__ uint32_t s_deliv[BCSIM_MSG_TYPES];
  __shared__ uint32_t s_ev, s_wr, s_nf, s_trbase;
  __shared__ long long s_tmax;
  const uint32_t tid = tidx(), lane = tid & 63u, j = tid & (G - 1u), gb = lane & ~(G - 1u);
  const uint32_t per_wg = blockDim.x / G;
  if (tid < BCSIM_MSG_TYPES) s_deliv[tid] = 0;
  if (tid == 0) {
    s_ev = s_wr = s_nf = 0;
    s_tmax = LLONG_MIN;
  }
  __syncthreads();
  const uint32_t na = fl ? p.act_n[0] : p.R * p.nloc;
  const uint32_t kl = blockIdx.x * per_wg + tid / G;
  const uint32_t k0 = blockIdx.x * per_wg;
  const uint32_t g0 = k0 < na ? gossip_gnode(p, k0, fl) : 0u;
  const uint32_t g = kl < na ? gossip_gnode(p, kl, fl) : 0u;
  const uint32_t rep = g / p.N, i = g % p.N;
  const uint32_t rep0 = g0 / p.N;  // counters of this replica go through LDS
  const uint32_t b = static_cast<uint32_t>(cell % p.n_buckets);
  const bool has_start = (t_lo <= 0 && 0 < t_hi);
  const bool has_stop = (p.stop_ns >= 0 && t_lo <= p.stop_ns && p.stop_ns < t_hi);
  // every load that depends on g alone goes out before any of them is used (one round trip,
  // not a chain of short-circuit branches each waiting for its load): unconditional, at valid
  // addresses (g = 0 past the list's end), used only under the conditions below.  On a regular
  // graph the row offsets are arithmetic and this lane's in-slot record is among them.
  const bool kin = kl < na;
  const uint32_t e0r = p.deg_reg ? i * p.deg_reg : 0u;
  uint4 rsv = make_uint4(0, 0, 0, 0);  // (raw words: unpacking a Rec here would wait for the load)
  if (p.deg_reg) rsv = gld4(p.inbox + inbox_idx(p, b, rep, e0r + min(j, p.deg_reg - 1u)));
  const uint8_t f8 = AT(p.iflag, static_cast<size_t>(b) * p.NT + g, static_cast<uint64_t>(p.n_buckets) * p.NT);
  const uint8_t t8 = p.mesh ? AT(p.rtile, kRtPad * ((static_cast<size_t>(b) * p.R + rep) * p.n_tiles + (i >> 6)), kRtPad * (static_cast<uint64_t>(p.n_buckets) * p.R * p.n_tiles))
                            : static_cast<uint8_t>(0);
  const long long tn = AT(p.node_tnext, g, p.NT);
  const uint32_t sub0p = AT(p.sub, g, p.NT), nops0p = AT(p.n_ops, g, p.NT);
  const uint64_t draws0p = p.delay_mode != BCSIM_DELAY_FIXED ? AT(p.draws, g, p.NT) : 0ull;
  const uint32_t rw0 = p.deg_reg ? 0u : AT(p.row, i, p.N + 1), rw1 = p.deg_reg ? 0u : AT(p.row, i + 1, p.N + 1);
  const uint32_t so0 = x_active ? AT(p.seg_off, g, p.NT + 1) : 0u, so1 = x_active ? AT(p.seg_off, g + 1, p.NT + 1) : 0u;
  const bool flagged = kin && (f8 | t8) != 0 && p.bmin[b] < t_hi;  // (node_flagged_w)
  const bool tdue = kin && tn < t_hi;
  const bool have = kin && (has_start || has_stop || flagged || tdue);  // k_active's k_scan rule
  const uint32_t e0 = !have ? 0u : p.deg_reg ? e0r : rw0;
  const uint32_t deg = !have ? 0u : p.deg_reg ? p.deg_reg : rw1 - rw0;
  bool fast = have && deg <= G && !has_start && !has_stop && !tdue;
  if (fast && x_active) fast = so1 == so0;
  if (have && !fast && j == 0) {
    // (loop == 0: the host skips k_scan<.., LOOP> -- no timer, START, STOP or extras can be
    // due in the window -- so no node may be left over)
    if (!loop) set_err(p, BCSIM_E_TIE);
    const uint32_t pos = gadd_r(&p.act_n[2], 1u);
    AT(p.act, 2ull * p.NT + pos, 3ull * p.NT) = g;
  }
  // this lane's in-slot
  bool v = false;
  Rec r{};
  uint64_t k64 = 0;
  long long t = 0;
  uint32_t dt = 0;
  if (fast && j < deg && flagged) {
    if (p.deg_reg)
      __builtin_memcpy(&r, &rsv, sizeof r);
    else
      r = ld_rec(p.inbox + inbox_idx(p, b, rep, e0 + j));
    t = cs + r.t_off;
    v = slot_live(r.flags, cell_tag(p, cell)) && t >= t_lo && t < t_hi;
    dt = static_cast<uint32_t>(prop_of_slot(p, e0 + j) + sel2(p.tx_last, (r.flags & RF_BIG) ? 1 : 0));
    k64 = (static_cast<uint64_t>(r.t_off) << 32) | static_cast<uint32_t>(~dt);
  }
  // key-order rank within the node's group (ties of (t, dt) by in-slot = origin order)
  uint32_t rank = 0;
  for (uint32_t q = 0; q < G; ++q) {
    const bool vq = __shfl(v ? 1 : 0, gb + q, 64) != 0;
    const uint64_t kq = (static_cast<uint64_t>(__shfl(static_cast<uint32_t>(k64 >> 32), gb + q, 64)) << 32) |
                        __shfl(static_cast<uint32_t>(k64), gb + q, 64);
    if (vq && (kq < k64 || (kq == k64 && q < j))) ++rank;
  }
  const int32_t seq = r.f0;
  const bool blk = v && r.type == GS_BLOCK;
  const bool inrange = seq >= 0 && static_cast<uint32_t>(seq) < p.pbft_seq_cap;
  if (blk && !inrange) set_err(p, BCSIM_E_INDEX);
  bool first = blk && inrange &&
               AT(p.gseen, static_cast<size_t>(g) * p.pbft_seq_cap + seq, static_cast<uint64_t>(p.NT) * p.pbft_seq_cap) == 0;
  for (uint32_t q = 0; q < G; ++q) {  // an earlier arrival of the window with the same block
    const bool bq = __shfl(blk ? 1 : 0, gb + q, 64) != 0;
    const int32_t sq = __shfl(seq, gb + q, 64);
    const uint32_t rq = __shfl(rank, gb + q, 64);
    if (bq && sq == seq && rq < rank) first = false;
  }
  uint32_t nf = 0, nfb = 0;  // first receipts of the node, and those before this one
  for (uint32_t q = 0; q < G; ++q) {
    const bool fq = __shfl(first ? 1 : 0, gb + q, 64) != 0;
    const uint32_t rq = __shfl(rank, gb + q, 64);
    if (fq) {
      ++nf;
      if (rq < rank) ++nfb;
    }
  }
  // counters (LDS for this workgroup's first replica)
  uint32_t li = 0;
  if (v) {
    if (rep == rep0) {
      if (r.type < BCSIM_MSG_TYPES) atomicAdd(&s_deliv[r.type], 1u);
      atomicAdd(&s_ev, 1u);
      if (r.type != GS_BLOCK) atomicAdd(&s_wr, 1u);
      atomicMax(&s_tmax, t);
    } else {
      unsigned long long* cnt = cnt_stripe(p, rep);
      if (r.type < BCSIM_MSG_TYPES) {
        atomicAdd(&cnt[CNT_DELIV + r.type], 1ull);
        atomicAdd(&cnt[CNT_DELIV_TOTAL], 1ull);
        atomicAdd(&kst_stripe(p)[KST_DELIV], 1ull);
      }
      if (p.echo) atomicAdd(&cnt[CNT_ECHOES], 1ull);
      if (r.type != GS_BLOCK) atomicAdd(&cnt[CNT_WRONG], 1ull);
      atomicAdd(&cnt[CNT_EVENTS], 1ull);
      atomicMax(reinterpret_cast<long long*>(&cnt[CNT_TLAST]), t);
    }
  }
  if (first) li = atomicAdd(&s_nf, 1u);
  // node state: sub (+deg per broadcast), draws (jitter), pending ops -- read by every lane
  // of the group before the barrier, written by lane 0 after it
  const uint32_t sub0 = sub0p, nops0 = nops0p;
  const uint64_t draws0 = draws0p;
  __syncthreads();
  if (tid == 0) s_trbase = s_nf ? gadd_r(p.trace_cnt, s_nf) : 0u;
  __syncthreads();
  if (nf) {
    const uint32_t ocap = op_cap(p, g);
    if (nops0 + nf > ocap) {
      if (j == 0) set_err(p, BCSIM_E_OVERFLOW);
    } else {
      if (first) {
        const uint32_t origin = p.mesh ? (j < i ? j : j + 1) : AT(p.col, e0 + j, p.E);
        const Key key{t, t - static_cast<int64_t>(dt), origin, r.sub};
        put_trace(p, s_trbase + li, key, rep, i, BCSIM_TR_GOSSIP_DELIVER, seq, r.f1 + 1, static_cast<int32_t>(origin));
        const Msg m = mkmsg(GS_BLOCK, seq, r.f1 + 1, 0, 1);
        const uint32_t sb = sub0 + nfb * deg;
        const Op o = p.delay_mode == BCSIM_DELAY_FIXED
                         ? mk_op(p, t + p.app_delay, static_cast<uint32_t>(p.app_delay), i, sb, 0, m, OP_BCAST, 0)
                         : mk_op(p, t, 0, i, sb, static_cast<uint32_t>(draws0 + static_cast<uint64_t>(nfb) * deg), m,
                                 OP_BCAST_J, 0);
        st_op(&AT(p.ops + op_base(p, g), nops0 + nfb, ocap), o);
        AT(p.gseen, static_cast<size_t>(g) * p.pbft_seq_cap + seq, static_cast<uint64_t>(p.NT) * p.pbft_seq_cap) = 1;
      }
      if (j == 0) {
        AT(p.sub, g, p.NT) = sub0 + nf * deg;
        if (p.delay_mode != BCSIM_DELAY_FIXED) AT(p.draws, g, p.NT) = draws0 + static_cast<uint64_t>(nf) * deg;
        AT(p.n_ops, g, p.NT) = nops0 + nf;
        AT(p.node_onext, g, p.NT) = LLONG_MIN;  // k_link recomputes
      }
    }
  }
  if (tid == 0) {
    unsigned long long* cnt = cnt_stripe(p, rep0);
    unsigned long long tot = 0;
    for (int k = 0; k < BCSIM_MSG_TYPES; ++k)
      if (s_deliv[k]) {
        atomicAdd(&cnt[CNT_DELIV + k], static_cast<unsigned long long>(s_deliv[k]));
        tot += s_deliv[k];
      }
    if (tot) {
      atomicAdd(&cnt[CNT_DELIV_TOTAL], tot);
      atomicAdd(&kst_stripe(p)[KST_DELIV], tot);
    }
    if (s_ev) {
      atomicAdd(&cnt[CNT_EVENTS], static_cast<unsigned long long>(s_ev));
      if (p.echo) atomicAdd(&cnt[CNT_ECHOES], static_cast<unsigned long long>(s_ev));
    }
    if (s_wr) atomicAdd(&cnt[CNT_WRONG], static_cast<unsigned long long>(s_wr));
    if (s_tmax > LLONG_MIN) atomicMax(reinterpret_cast<long long*>(&cnt[CNT_TLAST]), s_tmax);
  }
  return have && !fast;
}

__global__ __launch_bounds__(256) void k_gossip_scan(const KP* __restrict__ pk, long long cell, long long t_lo,
                                                     long long t_hi, long long cs, int x_active, uint32_t G,
                                                     int loop) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  (void)gossip_scan_body(pk, cell, t_lo, t_hi, cs, x_active, G, loop, false);
}

// ---------------------------------------------------------------------------
// k_link: per-node link stage.  Ops due in [.., t_hi) are applied to their
// out-edge's FIFO in canonical key order; every non-echo op produces one
// 16-byte arrival record, stored in the receiver's inbox slot of the arrival
// cell (a second record of the same edge and cell goes to the extras list,
// a cell beyond the ring to the overflow list).
constexpr int kBcastCap = 64;  // due broadcasts per node per cell
constexpr int kTile = 64;        // receiver tile of the full-mesh tile flags (rtile)
static_assert(kTile == static_cast<int>(kTR), "k_mesh_tile: one receiver tile per workgroup");
constexpr int kMaxTiles = 1024;  // 64-node tiles (N <= 65536)

__device__ inline bool op_key_less(const Op& a, uint32_t sa, const Op& b, uint32_t sb) {
  if (a.t != b.t) return a.t < b.t;
  const int64_t tsa = a.t - a.dt, tsb = b.t - b.dt;
  if (tsa != tsb) return tsa < tsb;
  if (a.origin != b.origin) return a.origin < b.origin;
  return sa < sb;
}

// ---- DROPTAIL link queue (oracle/bcsim_oracle.c q_admit restated) ----------
// frames of a queue entry that started transmission by time t
__device__ inline uint32_t q_started(const KP& p, uint64_t ent, int64_t t) {
  const int64_t s = static_cast<int64_t>(ent >> 17);
  const uint32_t big = static_cast<uint32_t>(ent >> 16) & 1u, k = static_cast<uint32_t>(ent & 0xFFFFu);
  if (t < s) return 0;
  if (sel2(p.nfr, big) == 1) return k;
  const int64_t j = (t - s) / sel2(p.tx_full, big) + 1;
  return j < static_cast<int64_t>(k) ? static_cast<uint32_t>(j) : k;
}
// admit a message of class `big` enqueued at t that would start at `start`: pops the
// entries whose frames all started, counts the waiting frames, accepts a prefix of the
// message while fewer than qcap_frames frames wait; returns the accepted frame count
__device__ inline uint32_t q_admit(const KP& p, uint64_t* ring, uint64_t& meta, int64_t t, int big, int64_t start) {
  uint32_t head = static_cast<uint32_t>(meta & 0xFFFFu), n = static_cast<uint32_t>((meta >> 16) & 0xFFFFu);
  uint32_t frames = static_cast<uint32_t>(meta >> 32);
  while (n) {
    const uint64_t e = ring[head];
    const uint32_t k = static_cast<uint32_t>(e & 0xFFFFu);
    if (q_started(p, e, t) != k) break;
    frames -= k;
    head = head + 1 == p.cap_q ? 0u : head + 1;
    --n;
  }
  const uint32_t waiting = n ? frames - q_started(p, ring[head], t) : 0u;
  const uint32_t F = sel2(p.nfr, big);
  const uint32_t room = waiting >= p.qcap_frames ? 0u : p.qcap_frames - waiting;
  const uint32_t k = room < F ? room : F;
  if (k) {
    if (n == p.cap_q) {
      set_err(p, BCSIM_E_OVERFLOW);  // more queued messages on one link than cap_queue_msgs
    } else {
      uint32_t tail = head + n;
      if (tail >= p.cap_q) tail -= p.cap_q;
      ring[tail] = (static_cast<uint64_t>(start) << 17) | (static_cast<uint64_t>(big) << 16) | k;
      ++n;
      frames += k;
    }
  }
  meta = head | (static_cast<uint64_t>(n) << 16) | (static_cast<uint64_t>(frames) << 32);
  return k;
}

// ---- FQCODEL link queue (oracle/bcsim_oracle.c fq_* restated) ------------
// One lane owns one directed edge and walks its events in time order (the link's ops in key
// order, the device-queue wakes in between), so the disc state lives in global memory and is
// read and written by that lane only.  Words only (no sub-dword struct members: DESIGN §8).
// While the lane works on the edge its 64-word header (flows, DRR lists, device-queue ring
// state) is staged in the lane's slot of LDS: every step of the disc is a chain of dependent
// header accesses (the class's flow, then its ring position, then the DRR lists ...), ~40 per
// packet, which in global memory were one round trip each.
constexpr uint32_t kFqH = 64, kFqF = 12;
enum : uint32_t { FQ_HEAD = 0, FQ_N, FQ_BYTES, FQ_FA, FQ_DNEXT, FQ_CNT, FQ_LCNT, FQ_REC, FQ_DROP, FQ_ST, FQ_DEF, FQ_CR };
enum : uint32_t { FQ_NNEW = 36, FQ_NEWL = 37, FQ_NOLD = 40, FQ_OLDL = 41, FQ_NCR = 44, FQ_STOP = 45, FQ_DH = 46,
                  FQ_DN = 47, FQ_DEND = 48, FQ_QP = 50, FQ_MBM = 52 };
constexpr uint32_t kFqLanes = 256;   // k_link<2>'s launch bound: LDS header slots per workgroup
constexpr uint32_t kFqMaxMsgs = 128;  // message-table bitmap words FQ_MBM..FQ_MBM+3
constexpr uint32_t kFqEcho = 1u << 25, kFqLost = 1u << 26;

// header words past the message bitmap: the packet classes' bound flows (slot of class c in
// bits 2c..2c+1, bound bit 8 + c) and their flow indices
constexpr uint32_t FQ_MAP = 56, FQ_HSH = 57;
// a FQCODEL record shipped to another rank carries its socket's port - 49152 in cell bits 48-61
constexpr int kXPortShift = 48;
static_assert(FQ_MBM + kFqMaxMsgs / 32 <= FQ_MAP && FQ_HSH + 3 <= kFqH, "FQCODEL header layout");
using FqW = __attribute__((address_space(3))) uint32_t;  // (the staged header: LDS)
struct FqLink {
  FqW* h;
  int64_t* dev;
  uint4* pk;
  uint4* msg;
  uint32_t e, src;  // (src: the op source of the current send, debug log only)
  uint32_t ia, ib;  // the link's sender / receiver IPv4 addresses
  uint32_t cap;     // packets per flow ring
  uint32_t pa, pe;  // client port of this edge's socket / of the reverse edge's (0: not bound)
};
// kinds: 1 enqueue, 2 into the device queue (x = frame start), 3 drop, 4 wake
__device__ inline void fq_log(const KP& p, const FqLink& L, int64_t t, uint32_t kind, const uint4& pk, int64_t x) {
  if (!p.fqlog || t < p.fqlog_t0 || t >= p.fqlog_t1) return;
  const uint32_t pos = gadd_r(p.fqlog_n, 1u);
  if (pos >= p.cap_fqlog) return;
  const uint32_t m = pk.z & 0xFFFFu;
  p.fqlog[2ull * pos] = make_uint4(static_cast<uint32_t>(t), static_cast<uint32_t>(static_cast<uint64_t>(t) >> 32), L.e,
                                   (kind << 24) | (pk.z >> 16));
  p.fqlog[2ull * pos + 1] = make_uint4(kind == 4 ? 0u : L.msg[m].x, static_cast<uint32_t>(x),
                                       static_cast<uint32_t>(static_cast<uint64_t>(x) >> 32),
                                       kind == 4 ? 0u : (L.msg[m].z & kFqEcho) ? 1u : 0u);
}
struct FqCount {
  unsigned long long fdrop, lost;
};

__device__ inline int64_t fq_ld64(const FqW* w) {
  return static_cast<int64_t>((static_cast<uint64_t>(w[1]) << 32) | w[0]);
}
__device__ inline void fq_st64(FqW* w, int64_t v) {
  w[0] = static_cast<uint32_t>(v);
  w[1] = static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32);
}
// edge e = (i -> j) at rank-local index le.  Addresses: the k-th link of the mesh loop
// (blockchain-simulator.cc:34-51) is network 1.0.0.0 + k*256, its larger endpoint .1
__device__ inline FqLink fq_link(const KP& p, size_t le, uint32_t e, uint32_t i, uint32_t j, FqW* hl) {
  FqLink L;
  {  // the header into the lane's LDS slot (16 loads in flight)
    const uint4* src = reinterpret_cast<const uint4*>(p.fqh + le * kFqH);
    uint4 v[kFqH / 4];
#pragma unroll
    for (uint32_t k = 0; k < kFqH / 4; ++k) v[k] = gld4(src + k);
#pragma unroll
    for (uint32_t k = 0; k < kFqH / 4; ++k) {
      hl[4 * k] = v[k].x;
      hl[4 * k + 1] = v[k].y;
      hl[4 * k + 2] = v[k].z;
      hl[4 * k + 3] = v[k].w;
    }
  }
  L.h = hl;
  L.dev = p.fqdev + le * p.fq_devcap;
  const uint64_t po = p.fqpoff[le];
  L.pk = p.fqpk + (po & ((1ull << 48) - 1));
  L.cap = static_cast<uint32_t>(po >> 48);
  L.msg = p.fqmsg + le * p.cap_fqm;
  L.e = e;
  L.src = 0;
  const uint32_t net = 0x01000000u + (p.fqlnk[e] << 8);
  L.ia = net + (i > j ? 1u : 2u);
  L.ib = net + (j > i ? 1u : 2u);
  L.pa = p.fqport[le];
  L.pe = p.fqpeer[le];
  return L;
}
// Ipv4QueueDiscItem::Hash: Murmur3-32 (seed 0x8BADF00D) of src | dst | proto 17 | sport |
// dport | perturbation, big endian (17 bytes; oracle_fq_flow)
// the staged header back to global memory (edge done)
__device__ inline void fq_unlink(const KP& p, const FqLink& L, size_t le) {
  uint4* dst = reinterpret_cast<uint4*>(p.fqh + le * kFqH);
#pragma unroll
  for (uint32_t k = 0; k < kFqH / 4; ++k) gst4(dst + k, make_uint4(L.h[4 * k], L.h[4 * k + 1], L.h[4 * k + 2], L.h[4 * k + 3]));
}
__device__ inline uint32_t fq_hash(uint32_t src, uint32_t dst, uint32_t sp, uint32_t dp, uint32_t pert) {
  auto bs = [](uint32_t x) { return __builtin_bswap32(x); };
  auto mix = [](uint32_t h, uint32_t k) {
    k *= 0xcc9e2d51u;
    k = (k << 15) | (k >> 17);
    k *= 0x1b873593u;
    h ^= k;
    h = (h << 13) | (h >> 19);
    return h * 5u + 0xe6546b64u;
  };
  // bytes: src(4) dst(4) | 17 sp_hi sp_lo dp_hi | dp_lo pert(3 high bytes) | pert low byte
  const uint32_t w2 = 17u | ((sp >> 8) & 0xFFu) << 8 | (sp & 0xFFu) << 16 | ((dp >> 8) & 0xFFu) << 24;
  const uint32_t w3 = (dp & 0xFFu) | ((pert >> 24) & 0xFFu) << 8 | ((pert >> 16) & 0xFFu) << 16 | ((pert >> 8) & 0xFFu) << 24;
  uint32_t h = 0x8BADF00Du;
  h = mix(h, bs(src));
  h = mix(h, bs(dst));
  h = mix(h, w2);
  h = mix(h, w3);
  uint32_t k = pert & 0xFFu;  // tail byte
  k *= 0xcc9e2d51u;
  k = (k << 15) | (k >> 17);
  k *= 0x1b873593u;
  h ^= k;
  h ^= 17u;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  return h ^ (h >> 16);
}
// the flow slot of packet class cls (0 app, 1 echo first fragment, 2 later fragment), bound at
// the class's first packet: the slot of an already bound class with the same flow index, else
// slot cls (oracle fq_class_slot)
__device__ inline uint32_t fq_class_slot(const KP& p, FqLink& L, uint32_t cls) {
  const uint32_t m = L.h[FQ_MAP];
  if (m & (0x100u << cls)) return (m >> (2 * cls)) & 3u;
  const uint32_t sp = cls == 0 ? L.pa : cls == 1 ? 7071u : 0u, dp = cls == 0 ? 7071u : cls == 1 ? L.pe : 0u;
  if (cls < 2 && (sp | dp) == 7071u) set_err(p, BCSIM_E_STATE);  // a send from an unbound socket
  const uint32_t h = fq_hash(L.ia, L.ib, sp, dp, p.fq_pert) % p.fq_flows;
  uint32_t slot = cls;
  for (uint32_t c = 0; c < 3; ++c)
    if ((m & (0x100u << c)) && L.h[FQ_HSH + c] == h) {
      slot = (m >> (2 * c)) & 3u;
      break;
    }
  L.h[FQ_HSH + cls] = h;
  L.h[FQ_MAP] = m | (0x100u << cls) | (slot << (2 * cls));
  return slot;
}
__device__ inline bool fq_pop(const KP& p, FqLink& L, uint32_t f, uint4& out) {
  FqW* F = L.h + f * kFqF;
  const uint32_t n = F[FQ_N];
  if (n == 0) return false;
  const uint32_t hd = F[FQ_HEAD];
  out = L.pk[f * L.cap + hd];
  F[FQ_HEAD] = hd + 1 == L.cap ? 0u : hd + 1;
  F[FQ_N] = n - 1;
  F[FQ_BYTES] -= out.w;
  L.h[FQ_QP] -= 1;
  return true;
}
__device__ inline void fq_free_msg(FqLink& L, uint32_t m) { L.h[FQ_MBM + (m >> 5)] &= ~(1u << (m & 31u)); }
// a packet leaves the disc untransmitted (CoDel or overlimit drop): its message is lost
__device__ inline void fq_drop(const KP& p, FqLink& L, const uint4& pk, FqCount& c, int64_t now) {
  fq_log(p, L, now, 3, pk, 0);
  ++c.fdrop;
  const uint32_t m = pk.z & 0xFFFFu;
  uint32_t z = L.msg[m].z, left = L.msg[m].w;
  if (!(z & kFqLost)) {
    z |= kFqLost;
    if (!(z & kFqEcho)) ++c.lost;
  }
  L.msg[m].z = z;
  L.msg[m].w = left - 1;
  if (left == 1) fq_free_msg(L, m);
}
// CoDelQueueDisc::OkToDrop (has: a packet was dequeued)
__device__ inline bool codel_ok(const KP& p, FqW* F, bool has, const uint4& pk, int64_t now, uint32_t now_c) {
  if (!has) {
    F[FQ_FA] = 0;
    return false;
  }
  const int64_t enq = static_cast<int64_t>((static_cast<uint64_t>(pk.y) << 32) | pk.x);
  const uint32_t soj = static_cast<uint32_t>(static_cast<uint64_t>(now - enq) >> 10);
  if (static_cast<int32_t>(soj - p.fq_target_c) < 0 || F[FQ_BYTES] < p.fq_min_bytes) {
    F[FQ_FA] = 0;
    return false;
  }
  if (F[FQ_FA] == 0) {
    F[FQ_FA] = now_c + p.fq_interval_c;
    return false;
  }
  return static_cast<int32_t>(now_c - F[FQ_FA]) > 0;
}
__device__ inline uint32_t codel_newton(uint32_t rec, uint32_t count) {
  const uint32_t invsqrt = rec << 16;
  const uint32_t invsqrt2 = static_cast<uint32_t>((static_cast<uint64_t>(invsqrt) * invsqrt) >> 32);
  uint64_t val = (3ull << 32) - static_cast<uint64_t>(count) * invsqrt2;
  val >>= 2;
  val = (val * invsqrt) >> 31;
  return static_cast<uint32_t>(val >> 16) & 0xFFFFu;
}
__device__ inline uint32_t codel_law(uint32_t t, uint32_t interval, uint32_t rec) {
  return t + static_cast<uint32_t>((static_cast<uint64_t>(interval) * (rec << 16)) >> 32);
}
// CoDelQueueDisc::DoDequeue of flow f
__device__ inline bool codel_deq(const KP& p, FqLink& L, uint32_t f, int64_t now, uint4& out, FqCount& c) {
  FqW* F = L.h + f * kFqF;
  uint4 pk;
  if (!fq_pop(p, L, f, pk)) {
    F[FQ_DROP] = 0;
    return false;
  }
  const uint32_t now_c = static_cast<uint32_t>(static_cast<uint64_t>(now) >> 10);
  bool have = true;
  const bool ok = codel_ok(p, F, true, pk, now, now_c);
  if (F[FQ_DROP]) {
    if (!ok) {
      F[FQ_DROP] = 0;
    } else if (static_cast<int32_t>(now_c - F[FQ_DNEXT]) >= 0) {
      while (F[FQ_DROP] && static_cast<int32_t>(now_c - F[FQ_DNEXT]) >= 0) {
        F[FQ_CNT] += 1;
        F[FQ_REC] = codel_newton(F[FQ_REC], F[FQ_CNT]);
        fq_drop(p, L, pk, c, now);
        have = fq_pop(p, L, f, pk);
        if (!codel_ok(p, F, have, pk, now, now_c))
          F[FQ_DROP] = 0;
        else
          F[FQ_DNEXT] = codel_law(F[FQ_DNEXT], p.fq_interval_c, F[FQ_REC]);
      }
    }
  } else if (ok) {
    fq_drop(p, L, pk, c, now);
    have = fq_pop(p, L, f, pk);
    (void)codel_ok(p, F, have, pk, now, now_c);
    F[FQ_DROP] = 1;
    const int32_t delta = static_cast<int32_t>(F[FQ_CNT] - F[FQ_LCNT]);
    if (delta > 1 && static_cast<int32_t>((now_c - F[FQ_DNEXT]) - 16u * p.fq_interval_c) < 0) {
      F[FQ_CNT] = static_cast<uint32_t>(delta);
      F[FQ_REC] = codel_newton(F[FQ_REC], F[FQ_CNT]);
    } else {
      F[FQ_CNT] = 1;
      F[FQ_REC] = 0xFFFFu;
    }
    F[FQ_LCNT] = F[FQ_CNT];
    F[FQ_DNEXT] = codel_law(now_c, p.fq_interval_c, F[FQ_REC]);
  }
  if (have) out = pk;
  return have;
}
__device__ inline void fq_list_pop(FqW* h, uint32_t nidx, uint32_t lidx) {
  const uint32_t n = h[nidx];
  for (uint32_t k = 1; k < n; ++k) h[lidx + k - 1] = h[lidx + k];
  h[nidx] = n - 1;
}
__device__ inline void fq_list_push(FqW* h, uint32_t nidx, uint32_t lidx, uint32_t f) {
  const uint32_t n = h[nidx];
  h[lidx + n] = f;
  h[nidx] = n + 1;
}
// FqCoDelQueueDisc::DoDequeue: DRR over the new, then the old flows
__device__ inline bool fq_deq(const KP& p, FqLink& L, int64_t now, uint4& out, FqCount& c) {
  FqW* h = L.h;
  for (;;) {
    int f = -1;
    while (f < 0 && h[FQ_NNEW]) {
      const uint32_t q = h[FQ_NEWL];
      FqW* F = h + q * kFqF;
      if (static_cast<int32_t>(F[FQ_DEF]) <= 0) {
        F[FQ_DEF] += p.fq_quantum;
        F[FQ_ST] = 2;
        fq_list_push(h, FQ_NOLD, FQ_OLDL, q);
        fq_list_pop(h, FQ_NNEW, FQ_NEWL);
      } else {
        f = static_cast<int>(q);
      }
    }
    while (f < 0 && h[FQ_NOLD]) {
      const uint32_t q = h[FQ_OLDL];
      FqW* F = h + q * kFqF;
      if (static_cast<int32_t>(F[FQ_DEF]) <= 0) {
        F[FQ_DEF] += p.fq_quantum;
        fq_list_pop(h, FQ_NOLD, FQ_OLDL);
        fq_list_push(h, FQ_NOLD, FQ_OLDL, q);
      } else {
        f = static_cast<int>(q);
      }
    }
    if (f < 0) return false;
    FqW* F = h + f * kFqF;
    if (codel_deq(p, L, static_cast<uint32_t>(f), now, out, c)) {
      F[FQ_DEF] -= out.w;
      return true;
    }
    if (F[FQ_ST] == 1 && h[FQ_NOLD]) {
      F[FQ_ST] = 2;
      fq_list_push(h, FQ_NOLD, FQ_OLDL, static_cast<uint32_t>(f));
      fq_list_pop(h, FQ_NNEW, FQ_NEWL);
    } else if (F[FQ_ST] == 1) {
      F[FQ_ST] = 0;
      fq_list_pop(h, FQ_NNEW, FQ_NEWL);
    } else {
      F[FQ_ST] = 0;
      fq_list_pop(h, FQ_NOLD, FQ_OLDL);
    }
  }
}
// device-queue frames that started transmission by `now` no longer wait
__device__ inline void fq_settle(const KP& p, FqLink& L, int64_t now) {
  uint32_t dh = L.h[FQ_DH], dn = L.h[FQ_DN];
  while (dn && L.dev[dh] <= now) {
    dh = dh + 1 == p.fq_devcap ? 0u : dh + 1;
    --dn;
  }
  L.h[FQ_DH] = dh;
  L.h[FQ_DN] = dn;
}
// a packet from the disc into the device queue; a message whose last fragment this was is
// delivered (emit(sub, f0|f1, f2|type, big, end of its frame)) unless a fragment was dropped
template <typename Emit>
__device__ inline void fq_dev_push(const KP& p, FqLink& L, const uint4& pk, int64_t now, Emit& emit) {
  const uint32_t m = pk.z & 0xFFFFu, frame = pk.z >> 16;
  const uint4 me = L.msg[m];
  const int big = (me.z >> 24) & 1;
  const int64_t tx = frame + 1 == sel2(p.nfr, big) ? sel2(p.tx_last, big) : sel2(p.tx_full, big);
  const int64_t dend = fq_ld64(L.h + FQ_DEND);
  const int64_t start = dend > now ? dend : now;
  const int64_t end = start + tx;
  fq_log(p, L, now, 2, pk, start);
  fq_st64(L.h + FQ_DEND, end);
  fq_settle(p, L, now);
  if (start > now) {
    const uint32_t dh = L.h[FQ_DH], dn = L.h[FQ_DN];
    uint32_t at = dh + dn;
    if (at >= p.fq_devcap) at -= p.fq_devcap;
    L.dev[at] = start;
    L.h[FQ_DN] = dn + 1;
    if (dn + 1 == p.fq_devcap) L.h[FQ_STOP] = 1;  // the device queue is full: the disc stops
  }
  if (me.w > 1) {
    L.msg[m].w = me.w - 1;
    return;
  }
  L.msg[m].w = 0;
  fq_free_msg(L, m);
  if (!(me.z & (kFqLost | kFqEcho))) emit(me.x, me.y, me.z & 0x00FFFFFFu, big, end);
}
// QueueDisc::Run
template <typename Emit>
__device__ inline void fq_run(const KP& p, FqLink& L, int64_t now, Emit& emit, FqCount& c) {
  uint4 pk;
  while (!L.h[FQ_STOP] && fq_deq(p, L, now, pk, c)) fq_dev_push(p, L, pk, now, emit);
}
// the device-queue wakes up to time t (each at its oldest waiting frame's start)
template <typename Emit>
__device__ inline void fq_advance(const KP& p, FqLink& L, int64_t t, Emit& emit, FqCount& c) {
  while (L.h[FQ_STOP]) {
    const int64_t tw = L.dev[L.h[FQ_DH]];
    if (tw > t) break;
    fq_log(p, L, tw, 4, make_uint4(0, 0, 0, 0), L.h[FQ_QP]);
    fq_settle(p, L, tw);
    L.h[FQ_STOP] = 0;
    fq_run(p, L, tw, emit, c);
  }
}
// FqCoDelQueueDisc::FqCoDelDrop: half the fattest flow's bytes (first class on ties)
__device__ inline void fq_overlimit(const KP& p, FqLink& L, FqCount& c, int64_t now) {
  uint32_t maxb = 0;
  int fat = -1;
  const uint32_t ncr = L.h[FQ_NCR];
  for (uint32_t r = 0; r < ncr; ++r)
    for (uint32_t f = 0; f < 3; ++f)
      if (L.h[f * kFqF + FQ_CR] == r) {
        if (fat < 0) fat = static_cast<int>(f);
        if (L.h[f * kFqF + FQ_BYTES] > maxb) {
          maxb = L.h[f * kFqF + FQ_BYTES];
          fat = static_cast<int>(f);
        }
      }
  if (fat < 0) return;
  const uint32_t threshold = maxb >> 1;
  uint32_t len = 0, count = 0;
  uint4 pk;
  do {
    if (!fq_pop(p, L, static_cast<uint32_t>(fat), pk)) break;
    fq_drop(p, L, pk, c, now);
    len += pk.w;
  } while (++count < p.fq_batch && len < threshold);
}
// a message handed to the link at `now`: IPv4 fragments, each enqueued, then QueueDisc::Run
template <typename Emit>
__device__ inline void fq_send(const KP& p, FqLink& L, int64_t now, uint32_t sub, uint32_t bz, uint32_t bw24, int big,
                               bool echo, Emit& emit, FqCount& c) {
  const uint32_t F = sel2(p.nfr, big);
  if (F == 1 && !p.fqlog && p.fq_limit >= 1 && L.h[FQ_QP] == 0 && !L.h[FQ_STOP] && fq_ld64(L.h + FQ_DEND) <= now) {
    // the heavy waves' case: a one-fragment message on a link whose disc is empty (so both DRR
    // lists are and every flow is inactive) and whose device is idle.  The slow path below would
    // enqueue the packet into its (new) flow, dequeue it at once (sojourn 0: CoDel leaves the
    // drop state), transmit it from now, then empty the lists again; its net effect is this:
    const uint32_t fs = fq_class_slot(p, L, echo ? 1u : 0u);
    FqW* Fh = L.h + fs * kFqF;
    if (Fh[FQ_CR] == kInvalid) Fh[FQ_CR] = L.h[FQ_NCR]++;
    int32_t d = static_cast<int32_t>(p.fq_quantum) - static_cast<int32_t>(p.ip_last[big]);
    if (d <= 0) d += static_cast<int32_t>(p.fq_quantum);  // (a second DRR round on the old list)
    Fh[FQ_DEF] = static_cast<uint32_t>(d);
    Fh[FQ_FA] = 0;
    Fh[FQ_DROP] = 0;
    fq_settle(p, L, now);  // (every waiting frame started by the idle device's end)
    const int64_t end = now + sel2(p.tx_last, big);
    fq_st64(L.h + FQ_DEND, end);
    if (!echo) emit(sub, bz, bw24, big, end);
    return;
  }
  uint32_t m = kInvalid;
  for (uint32_t w = 0; w < p.cap_fqm / 32u && m == kInvalid; ++w) {
    const uint32_t free_bits = ~L.h[FQ_MBM + w];
    if (free_bits) m = w * 32u + static_cast<uint32_t>(__builtin_ctz(free_bits));
  }
  if (m == kInvalid) {
    set_err(p, BCSIM_E_OVERFLOW);  // more messages in one link's disc than cap_fqm
    return;
  }
  L.h[FQ_MBM + (m >> 5)] |= 1u << (m & 31u);
  L.msg[m] = make_uint4(sub, bz, bw24 | (static_cast<uint32_t>(big) << 24) | (echo ? kFqEcho : 0u), F);
  const uint32_t now_lo = static_cast<uint32_t>(now), now_hi = static_cast<uint32_t>(static_cast<uint64_t>(now) >> 32);
  for (uint32_t j = 0; j < F; ++j) {
    const uint32_t cls = j ? 2u : echo ? 1u : 0u;
    const uint32_t f = fq_class_slot(p, L, cls);
    FqW* Fh = L.h + f * kFqF;
    if (Fh[FQ_CR] == kInvalid) Fh[FQ_CR] = L.h[FQ_NCR]++;
    if (Fh[FQ_ST] == 0) {
      Fh[FQ_ST] = 1;
      Fh[FQ_DEF] = p.fq_quantum;
      fq_list_push(L.h, FQ_NNEW, FQ_NEWL, f);
    }
    const uint32_t n = Fh[FQ_N];
    if (n == L.cap) {
      set_err(p, BCSIM_E_OVERFLOW);  // more packets in one flow than its ring holds
      return;
    }
    uint32_t at = Fh[FQ_HEAD] + n;
    if (at >= L.cap) at -= L.cap;
    const uint32_t size = j + 1 == F ? p.ip_last[big] : p.ip_full[big];
    L.pk[f * L.cap + at] = make_uint4(now_lo, now_hi, m | (j << 16), size);
    fq_log(p, L, now, 1, L.pk[f * L.cap + at], f | (L.src << 8));
    Fh[FQ_N] = n + 1;
    Fh[FQ_BYTES] += size;
    const uint32_t qp = L.h[FQ_QP] + 1;
    L.h[FQ_QP] = qp;
    if (qp > p.fq_limit) fq_overlimit(p, L, c, now);
    fq_run(p, L, now, emit, c);
  }
}

struct LinkShared {
  uint32_t n_bc, n_keep, n_list;
  uint32_t csum[8];  // block counters (wave sums, LDS atomics)
  uint32_t bc[kBcastCap];
  Op bco[kBcastCap];         // the due broadcasts in key order (LDS copies: every lane reads them per edge)
  uint32_t lcnt[kMaxBuckets];
  uint32_t lmin[kMaxBuckets];  // earliest arrival offset of this workgroup's records per bucket (-> bmin)
  uint4 wsum[kMaxWaves];
  uint32_t wcnt[kMaxWaves];
  uint32_t nst;                      // staged extras / overflow records
  uint32_t lst[kMaxBuckets + 1 + kMaxRanks];    // per list (bucket extras..., overflow, ranks...)
  uint32_t lbase[kMaxBuckets + 1 + kMaxRanks];  // per list base reserved in the global list
  long long omin, ovmin;
  uint8_t tflag[kMaxTiles];  // full mesh: receiver tiles this sender wrote in this launch
  uint32_t tbk;              // (the bucket of those records; one per launch in practice)
  // FQCODEL socket binding: this window's unbound sockets that send, the Paxos *end()
  // socket's first send (fqph: it has one) and its key
  uint32_t fqc, fqph, fqph_dt, fqph_sub;
  long long fqph_t;
};

// Stage one extras / overflow record of k_link (list = bucket, or B for the
// overflow list): LDS ranks now, one global atomic per list at the flush.
// A full staging area falls back to a direct (contended) global append.
template <class LS>
__device__ inline void link_stage(const KP& p, LS& L, uint32_t g, uint32_t list, const XRec& x) {
  const uint32_t spos = atomicAdd(&L.nst, 1u);
  if (spos < p.cap_stage) {
    const uint32_t rank = atomicAdd(&L.lst[list], 1u);
    const size_t k = static_cast<size_t>(blockIdx.x) * p.cap_stage + spos;  // per workgroup (sequential nodes)
    p.xstage[k] = x;
    p.xmeta[k] = (list << 24) | rank;
    return;
  }
  if (list > p.n_buckets) {  // another rank's receiver
    const uint32_t r = list - p.n_buckets - 1;
    gmin(&p.scal[4], static_cast<long long>(static_cast<uint64_t>(x.cell) & ((1ull << 48) - 1)));
    const uint32_t pos = gadd_r(&p.send_cnt[r], 1u);
    if (pos >= p.cap_send) {
      set_err(p, BCSIM_E_OVERFLOW);
      return;
    }
    p.sendbuf[static_cast<size_t>(r) * p.cap_send + pos] = x;
  } else if (list == p.n_buckets) {
    const uint32_t pos = gadd_r(p.ov_cnt, 1u);
    if (pos >= p.cap_ov) {
      set_err(p, BCSIM_E_OVERFLOW);
      return;
    }
    AT(p.ov, pos, p.cap_ov) = x;
  } else {
    const uint32_t pos = gadd_r(&p.x_cnt[list], 1u);
    if (pos >= p.cap_x) {
      set_err(p, BCSIM_E_OVERFLOW);
      return;
    }
    AT(p.xbuf, static_cast<size_t>(list) * p.cap_x + pos, p.cap_xbuf) = x;
  }
}

// per-lane statistics of a link stage: dropped, sends, records, due ops, edges, echoes,
// refused frames, lost messages (summed per workgroup in link_finish)
struct LinkCounts {
  uint32_t v[8];
};

// The end of a node's link stage (link_node, k_link_mesh): ordered compaction of the ops
// not yet due, flush of the staged extras / overflow / cross-rank records (one atomic per
// list), counters, and the node's op count and next op time.
__device__ __attribute__((always_inline)) inline void link_finish(const KP& p, LinkShared& L, uint32_t g, Op* ops, uint32_t n,
                                                                  long long t_hi, uint32_t n_lists, long long ovmin,
                                                                  const LinkCounts& c8, bool clr_slots, bool clr_rx,
                                                                  uint32_t obp, size_t fidx, unsigned long long wg_t0,
                                                                  unsigned long long* ph, uint32_t n_in) {
  const uint32_t tid = tidx();
  const uint32_t B = p.n_buckets;
  unsigned long long* cnt = cnt_stripe(p, g / p.N);
  // ---- 3. compact the ops that are not due yet ----
  // ordered in-place compaction: an op moves to the count of kept ops before
  // it (<= its own index); every lane has read its op before any lane writes
  long long omin = LLONG_MAX;
  uint32_t kept = 0;
  if (p.wgt && tid == 0) ph[3] = __builtin_amdgcn_s_memrealtime();
  for (uint32_t k0 = 0; k0 < n; k0 += blockDim.x) {
    const uint32_t k = k0 + tid;
    RawOp o = raw_zero();  // (raw words: an Op struct here went through scratch)
    bool keep = false;
    if (k < n) {
      o = ld_raw(&ops[k]);
      if (raw_kind(o) == OP_BCAST_J)
        keep = !(raw_flags(o) & OPF_DONE);  // unexpanded (fixed mode never creates these)
      else if (raw_t(o) >= t_hi) {
        keep = true;
        if (raw_t(o) < omin) omin = raw_t(o);
      }
    }
    uint32_t tot;
    const uint32_t pos = kept + block_rank(keep, L.wcnt, tot);
    if (keep) {
      uint4* q = reinterpret_cast<uint4*>(&ops[pos]);
      q[0] = o.a;
      q[1] = o.b;
    }
    kept += tot;
  }
  if (tid == 0) L.n_keep = kept;
  if (omin != LLONG_MAX) atomicMin(&L.omin, omin);
  if (ovmin != LLONG_MAX) atomicMin(&L.ovmin, ovmin);
  // ---- 4. flush the staged extras / overflow records: one atomic per list ----
  for (uint32_t k = tid; k < n_lists; k += blockDim.x) {
    const uint32_t c = L.lst[k];
    if (!c) continue;
    uint32_t* ctr = k < B ? &p.x_cnt[k] : k == B ? p.ov_cnt : &p.send_cnt[k - B - 1];
    const uint32_t cap = k < B ? p.cap_x : k == B ? p.cap_ov : p.cap_send;
    const uint32_t base = atomicAdd(ctr, c);
    if (base + c > cap) set_err(p, BCSIM_E_OVERFLOW);
    L.lbase[k] = base;
  }
  __syncthreads();
  const uint32_t nst = min(L.nst, p.cap_stage);
  long long xmin = LLONG_MAX;  // earliest arrival cell shipped to another rank (scal[4]: the next-cell bound)
  for (uint32_t k = tid; k < nst; k += blockDim.x) {
    const size_t sidx = static_cast<size_t>(blockIdx.x) * p.cap_stage + k;
    const uint32_t meta = p.xmeta[sidx], list = meta >> 24;
    const uint32_t pos = L.lbase[list] + (meta & 0xFFFFFFu);
    if (list > B) {
      const XRec x = p.xstage[sidx];
      xmin = min(xmin, static_cast<long long>(static_cast<uint64_t>(x.cell) & ((1ull << 48) - 1)));
      if (pos < p.cap_send) p.sendbuf[static_cast<size_t>(list - B - 1) * p.cap_send + pos] = x;
    } else if (list == B) {
      if (pos < p.cap_ov) p.ov[pos] = p.xstage[sidx];
    } else if (pos < p.cap_x) {
      p.xbuf[static_cast<size_t>(list) * p.cap_x + pos] = p.xstage[sidx];
    }
  }
  if (n_lists > B + 1) {
    for (int d = 32; d > 0; d >>= 1) xmin = min(xmin, static_cast<long long>(__shfl_xor(xmin, d, 64)));
    if ((tid & 63u) == 0 && xmin != LLONG_MAX) gmin(&p.scal[4], xmin);
  }
  // ---- 5. counters: wave sums, LDS atomics, one global atomic per workgroup ----
  {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t ws = wave_sum(c8.v[k]);
      if ((tid & 63u) == 0 && ws) atomicAdd(&L.csum[k], ws);
    }
  }
  __syncthreads();
  if (tid == 0) {
    if (L.csum[0]) atomicAdd(&cnt[CNT_DROPPED], static_cast<unsigned long long>(L.csum[0]));
    if (L.csum[1]) atomicAdd(&cnt[CNT_SENDS], static_cast<unsigned long long>(L.csum[1]));
    if (L.csum[2]) atomicAdd(&kst_stripe(p)[KST_REC], static_cast<unsigned long long>(L.csum[2]));
    if (L.csum[3]) atomicAdd(&kst_stripe(p)[KST_OPS], static_cast<unsigned long long>(L.csum[3]));
    if (L.csum[4]) atomicAdd(&kst_stripe(p)[KST_EDGES], static_cast<unsigned long long>(L.csum[4]));
    if (L.csum[5]) atomicAdd(&kst_stripe(p)[KST_ECHO], static_cast<unsigned long long>(L.csum[5]));
    if (L.csum[6]) atomicAdd(&cnt[CNT_FDROP], static_cast<unsigned long long>(L.csum[6]));
    if (L.csum[7]) atomicAdd(&cnt[CNT_LOST], static_cast<unsigned long long>(L.csum[7]));
  }
  for (uint32_t k = tid; k < B; k += blockDim.x)
    if (L.lcnt[k]) {
      mark_busy(&p.bucket_cnt[k]);
      bmin_lower(p, k, bucket_t0(p, (t_hi - 1) / p.L, k) + L.lmin[k]);
    }
  if (p.wgt && tid == 0) {
    p.wgt[8ull * g] = wg_t0;
    p.wgt[8ull * g + 1] = __builtin_amdgcn_s_memrealtime();
    p.wgt[8ull * g + 2] = (static_cast<unsigned long long>(n_in) << 32) | L.n_keep;
    p.wgt[8ull * g + 3] = ph[0];
    p.wgt[8ull * g + 4] = ph[1];
    p.wgt[8ull * g + 5] = ph[2];
    p.wgt[8ull * g + 6] = ph[3];
  }
  if (tid == 0) {
    if (L.ovmin != LLONG_MAX) gmin(&p.scal[1], L.ovmin);
    // the previous arrival cell's replies are all consumed now
    if (clr_slots) AT(p.sflag, static_cast<size_t>(obp) * p.NT + g, static_cast<uint64_t>(kOpRing) * p.NT) = 0;
    if (clr_rx) AT(p.iflag, fidx, static_cast<uint64_t>(p.n_buckets) * p.NT) = 0;
    AT(p.n_ops, g, p.NT) = L.n_keep;
    AT(p.node_onext, g, p.NT) = L.omin;
    atomicAdd(&kst_stripe(p)[KST_KEPT], static_cast<unsigned long long>(L.n_keep));
  }
}

// QM: queue model (0 INFINITE, 1 DROPTAIL, 2 FQCODEL); XR: node-partitioned run (records for
// other ranks).  Both are template parameters so the common case (infinite queues, one rank)
// carries none of their registers through the per-edge loop.
template <int QM, bool XR>
__device__ __attribute__((always_inline)) inline void link_node(const KP* __restrict__ pk, uint32_t g, long long cell, long long t_lo, long long t_hi,
                          int final_win) {
  const KP& p = *pk;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ LinkShared L;
  uint32_t n = AT(p.n_ops, g, p.NT);
  // reply slots of this arrival cell (bit 0: due now) and of the previous one (bit 1)
  const uint32_t ob = static_cast<uint32_t>(cell % kOpRing), obp = static_cast<uint32_t>((cell + kOpRing - 1) % kOpRing);
  const bool sl0 = p.eslot && (AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, static_cast<uint64_t>(kOpRing) * p.NT) & 1u);
  const bool sl1 = p.eslot && (AT(p.sflag, static_cast<size_t>(obp) * p.NT + g, static_cast<uint64_t>(kOpRing) * p.NT) & 2u);
  const bool sl = sl0 || sl1;
  const uint32_t ib = static_cast<uint32_t>(cell % p.n_buckets);
  const size_t fidx = static_cast<size_t>(ib) * p.NT + g;
  const uint32_t rep = g / p.N, i = g % p.N;
  const bool rx = p.impl && node_flagged_w(p, ib, g, rep, i, t_hi);
  // the implicit echoes, unless k_scan_pbft applied them in this window
  const bool rxe = rx && AT(p.eapp, g, p.NT) != t_lo;
  // (FQCODEL: a device-queue wake of a link with packets in its disc is due)
  const bool fqw = QM == 2 && AT(p.node_onext, g, p.NT) < t_hi;
  if (n == 0 && !sl && !rxe && !fqw) {
    if (rx && final_win && tidx() == 0) AT(p.iflag, fidx, static_cast<uint64_t>(p.n_buckets) * p.NT) = 0;
    return;
  }
  const unsigned long long wg_t0 = p.wgt ? __builtin_amdgcn_s_memrealtime() : 0;
  unsigned long long ph[4] = {0, 0, 0, 0};
  const uint32_t n_in = n;
  const uint32_t tid = tidx();
  const uint32_t e0 = AT(p.row, i, p.N + 1), deg = AT(p.row, i + 1, p.N + 1) - e0;
  Op* ops = p.ops + op_base(p, g);
  const uint32_t ocap = op_cap(p, g);
  // LDS: ecnt[deg+1] (per-edge counts -> offsets -> ends) | eidx[cap_eidx] (listed due ops
  // grouped by edge; a node with more due ops than cap_eidx uses its global area eidx_g)
  uint32_t* ecnt = reinterpret_cast<uint32_t*>(smem);
  const size_t eb0 = edge_loc(p, rep, e0);
  const int64_t* prop = p.prop + e0;
  const uint32_t B = p.n_buckets;

  // ---- 0. expand jitter broadcasts into per-edge SEND ops ----
  // The unexpanded broadcasts are found by a parallel pass (batches of kBcastCap, in op
  // order) and expanded one after another by the whole workgroup; the position of an
  // expanded op in the list does not matter (every edge sorts its ops by key).
  if (p.delay_mode != BCSIM_DELAY_FIXED) {
    for (;;) {
      if (tid == 0) L.n_bc = 0;
      __syncthreads();
      for (uint32_t k = tid; k < n; k += blockDim.x) {
        const Op& o = ops[k];
        if (op_kind(o) == OP_BCAST_J && !(op_flags(o) & OPF_DONE)) {
          const uint32_t pos = atomicAdd(&L.n_bc, 1u);
          if (pos < kBcastCap) L.bc[pos] = k;
        }
      }
      __syncthreads();
      const uint32_t nfound = L.n_bc, nb = min(nfound, static_cast<uint32_t>(kBcastCap));
      if (nb == 0) break;
      if (n + nb * deg > ocap) {
        if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
        return;
      }
      for (uint32_t b2 = 0; b2 < nb; ++b2) {
        // (raw words: an Op copy, sub-dword members and all, went through scratch)
        const RawOp o = ld_raw(&ops[L.bc[b2]]);
        const bool paxos = (raw_flags(o) & OPF_PAXOS) != 0;
        const uint64_t dbase = static_cast<uint64_t>(o.b.y);
        const uint32_t at = n + b2 * deg;
        const uint32_t w3 = (o.b.w & 0x00FFFFFFu) | (static_cast<uint32_t>(OP_SEND | ((raw_flags(o) & OPF_BIG) << 2)) << 24);
        for (uint32_t it = tid; it < deg; it += blockDim.x) {
          const int32_t r = ctr_rand(p.seed, rep, i, dbase + it);
          const int64_t d = delay_from_draw(p, r);
          const uint64_t t = static_cast<uint64_t>(raw_t(o) + d);
          uint4* w = reinterpret_cast<uint4*>(&AT(ops, at + it, ocap));
          w[0] = make_uint4(static_cast<uint32_t>(t), static_cast<uint32_t>(t >> 32), static_cast<uint32_t>(d), o.a.w);
          w[1] = make_uint4(raw_sub(o) + it, paxos ? (it + 1 < deg ? e0 + it + 1 : kInvalid) : e0 + it, o.b.z, w3);
        }
      }
      __syncthreads();
      for (uint32_t b2 = tid; b2 < nb; b2 += blockDim.x)
        AT(ops, L.bc[b2], ocap).kind_flags = static_cast<uint8_t>(OP_BCAST_J | (OPF_DONE << 2));
      n += nb * deg;
      __syncthreads();
      if (nfound <= static_cast<uint32_t>(kBcastCap)) break;
    }
  }

  // ---- 1. classify due ops: broadcast list, listed-op count ----
  for (uint32_t k = tid; k < B; k += blockDim.x) {
    L.lcnt[k] = 0;
    L.lmin[k] = ~0u;
  }
  const uint32_t n_lists = B + 1 + (XR ? p.nranks : 0);
  for (uint32_t k = tid; k < n_lists; k += blockDim.x) L.lst[k] = 0;
  const bool tmap = p.mesh && p.n_tiles <= static_cast<uint32_t>(kMaxTiles);
  if (tmap)
    for (uint32_t k = tid; k < p.n_tiles; k += blockDim.x) L.tflag[k] = 0;
  if (tid < 8) L.csum[tid] = 0;
  if (tid == 0) {
    L.n_bc = 0;
    L.n_keep = 0;
    L.n_list = 0;
    L.nst = 0;
    L.omin = LLONG_MAX;
    L.ovmin = LLONG_MAX;
    L.tbk = kInvalid;
    L.fqc = 0;
  }
  __syncthreads();
  unsigned long long dropped = 0, sends = 0, st_ops = 0;
  uint32_t cb = kInvalid, cbn = 0;  // run-length bucket count of this thread's records
  uint32_t cmn = ~0u;               // and their earliest arrival offset in the cell
  uint32_t my_list = 0;
  for (uint32_t k = tid; k < n; k += blockDim.x) {
    const Op& o = ops[k];
    const uint8_t kind = op_kind(o);
    if (kind == OP_BCAST_J || o.t >= t_hi) continue;
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
      ++my_list;
    }
  }
  {
    const uint32_t ws = wave_sum(my_list);
    if ((tid & 63u) == 0 && ws) atomicAdd(&L.n_list, ws);
  }
  __syncthreads();
  const uint32_t n_bc = L.n_bc, n_list = L.n_list;
  if (n_bc > kBcastCap) {
    if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
    return;
  }
  if (p.wgt && tid == 0) ph[0] = __builtin_amdgcn_s_memrealtime();
  // the due broadcasts: parallel copy to LDS, then key order (insertion sort, few)
  if (tid < n_bc) L.bco[tid] = ld_op(&ops[L.bc[tid]]);
  __syncthreads();
  if (tid == 0) {
    for (uint32_t a = 1; a < n_bc; ++a) {
      const Op ox = L.bco[a];
      uint32_t b2 = a;
      while (b2 > 0 && op_key_less(ox, ox.sub, L.bco[b2 - 1], L.bco[b2 - 1].sub)) {
        st_op_lds(&L.bco[b2], L.bco[b2 - 1]);
        --b2;
      }
      st_op_lds(&L.bco[b2], ox);
    }
  }
  // listed due ops (unicast / echo) grouped by edge: counting sort over the out-edges.
  // After the fill ecnt[le] is the END of edge le's range ([ecnt[le-1], ecnt[le])).
  uint32_t* eidx = ecnt + (p.deg_max + 1);
  if (n_list) {
    if (n_list > p.cap_eidx) eidx = p.eidx_g + static_cast<size_t>(blockIdx.x) * p.cap_ops;
    for (uint32_t k = tid; k <= deg; k += blockDim.x) ecnt[k] = 0;
    __syncthreads();
    for (uint32_t k = tid; k < n; k += blockDim.x) {
      const Op& o = ops[k];
      const uint8_t kind = op_kind(o);
      if (kind == OP_BCAST_J || kind == OP_BCAST || o.t >= t_hi || o.edge == kInvalid) continue;
      atomicAdd(&ecnt[o.edge - e0], 1u);
    }
    __syncthreads();
    (void)block_scan_array(ecnt, deg + 1, L.wsum);
    for (uint32_t k = tid; k < n; k += blockDim.x) {
      const Op& o = ops[k];
      const uint8_t kind = op_kind(o);
      if (kind == OP_BCAST_J || kind == OP_BCAST || o.t >= t_hi || o.edge == kInvalid) continue;
      eidx[atomicAdd(&ecnt[o.edge - e0], 1u)] = k;
    }
  }
  __syncthreads();

  if constexpr (QM == 2) {
    // ---- 1'. FQCODEL: a client socket binds -- takes the node's next ephemeral port -- at its
    // first send (oracle fq_bind).  The unbound sockets sending in this window are ranked by
    // the event key (t, t - dt, sub) of their first send; a rare pass (nothing after a node's
    // sockets have all sent once), so the rank is a plain count over the node's edges ----
    auto key_less = [](int64_t ta, uint32_t da, uint32_t sa, int64_t tb, uint32_t db, uint32_t sb) {
      if (ta != tb) return ta < tb;
      if (da != db) return da > db;
      return sa < sb;
    };
    const uint32_t pbase = AT(p.fqnport, g, p.NT);
    uint32_t my_c = 0;
    for (uint32_t le = tid; le < deg; le += blockDim.x) {
      const size_t x = eb0 + le;
      if (p.fqport[x]) continue;
      bool have = false;
      int64_t bt = 0;
      uint32_t bd = 0, bsb = 0;
      auto consider = [&](int64_t t, uint32_t d, uint32_t sb) {
        if (!have || key_less(t, d, sb, bt, bd, bsb)) {
          have = true;
          bt = t;
          bd = d;
          bsb = sb;
        }
      };
      const uint32_t eb = n_list && le ? ecnt[le - 1] : 0u, ee = n_list ? ecnt[le] : 0u;
      for (uint32_t a = eb; a < ee; ++a) {
        const Op& o = ops[eidx[a]];
        if (op_kind(o) != OP_ECHO) consider(o.t, o.dt, o.sub);
      }
      for (uint32_t bi = 0; bi < n_bc; ++bi) {  // (key order: the first one that reaches le)
        const bool px = (op_flags(L.bco[bi]) & OPF_PAXOS) != 0;
        if (px && le == 0) continue;
        consider(L.bco[bi].t, L.bco[bi].dt, L.bco[bi].sub + (px ? le - 1 : le));
        break;
      }
      const uint32_t e = e0 + le;
      if (sl0) {
        const RawOp r = slot_op(p, *eslot_at(p, ob, rep, e), i, e);
        if (raw_t(r) >= t_lo && raw_t(r) < t_hi && raw_kind(r) != OP_ECHO) consider(raw_t(r), raw_dt(r), raw_sub(r));
      }
      if (sl1) {
        const RawOp r = slot_op(p, *eslot_at(p, obp, rep, e), i, e);
        if (raw_t(r) >= t_lo && raw_t(r) < t_hi && raw_kind(r) != OP_ECHO) consider(raw_t(r), raw_dt(r), raw_sub(r));
      }
      const uint64_t ut = static_cast<uint64_t>(bt);
      p.fqkey[x] = have ? make_uint4(static_cast<uint32_t>(ut), static_cast<uint32_t>(ut >> 32), bd, bsb)
                        : make_uint4(~0u, ~0u, ~0u, ~0u);
      my_c += have ? 1u : 0u;
    }
    {
      const uint32_t ws = wave_sum(my_c);
      if ((tid & 63u) == 0 && ws) atomicAdd(&L.fqc, ws);
    }
    if (tid == 0) {  // Paxos's *end() socket (its sends carry no edge)
      L.fqph = 0;
      if (p.protocol == BCSIM_PAXOS && !AT(p.fqphant, g, p.NT)) {
        bool have = false;
        int64_t bt = 0;
        uint32_t bd = 0, bsb = 0;
        auto consider = [&](int64_t t, uint32_t d, uint32_t sb) {
          if (!have || key_less(t, d, sb, bt, bd, bsb)) {
            have = true;
            bt = t;
            bd = d;
            bsb = sb;
          }
        };
        for (uint32_t k = 0; k < n; ++k) {
          const Op& o = ops[k];
          if (op_kind(o) == OP_SEND && o.edge == kInvalid && o.t < t_hi) consider(o.t, o.dt, o.sub);
        }
        for (uint32_t bi = 0; bi < n_bc; ++bi)
          if (op_flags(L.bco[bi]) & OPF_PAXOS) {
            consider(L.bco[bi].t, L.bco[bi].dt, L.bco[bi].sub + deg - 1);
            break;
          }
        if (have) {
          L.fqph = 1;
          L.fqph_t = bt;
          L.fqph_dt = bd;
          L.fqph_sub = bsb;
        }
      }
    }
    __syncthreads();
    const uint32_t nc = L.fqc + L.fqph;
    if (nc) {
      if (pbase + nc > 16383u && tid == 0) set_err(p, BCSIM_E_UNSUPPORTED);  // ephemeral ports used up
      for (uint32_t le = tid; le < deg; le += blockDim.x) {
        const size_t x = eb0 + le;
        const uint4 kv = p.fqkey[x];
        if ((kv.x & kv.y) == ~0u) continue;
        const int64_t t = static_cast<int64_t>((static_cast<uint64_t>(kv.y) << 32) | kv.x);
        uint32_t rank = 0;
        for (uint32_t q = 0; q < deg; ++q) {
          const uint4 o = p.fqkey[eb0 + q];
          if ((o.x & o.y) == ~0u) continue;
          rank += key_less(static_cast<int64_t>((static_cast<uint64_t>(o.y) << 32) | o.x), o.z, o.w, t, kv.z, kv.w) ? 1u : 0u;
        }
        if (L.fqph && key_less(L.fqph_t, L.fqph_dt, L.fqph_sub, t, kv.z, kv.w)) ++rank;
        const uint32_t port = 49153u + pbase + rank;
        p.fqport[x] = port;
        // the echo class of the reverse edge sends to this port: its copy at the receiver (a
        // receiver on another rank learns it from the shipped records, k_import)
        const uint32_t j = p.mesh ? (le < i ? le : le + 1) : AT(p.col, e0 + le, p.E);
        if (!XR || p.owner[j] == p.rank) {
          const uint32_t slot = p.mesh ? j * (p.N - 1) + (i < j ? i : i - 1) : AT(p.rev, e0 + le, p.E);
          p.fqpeer[edge_loc(p, rep, slot)] = port;
        }
      }
      __syncthreads();
      for (uint32_t le = tid; le < deg; le += blockDim.x) {
        const size_t x = eb0 + le;
        const uint4 kv = p.fqkey[x];
        if ((kv.x & kv.y) != ~0u) p.fqkey[x] = make_uint4(~0u, ~0u, ~0u, ~0u);
      }
      if (tid == 0) {
        AT(p.fqnport, g, p.NT) = pbase + nc;
        if (L.fqph) AT(p.fqphant, g, p.NT) = 1u;
      }
    }
  }
  if (p.wgt && tid == 0) ph[1] = __builtin_amdgcn_s_memrealtime();
  // ---- 2. per edge: sort its ops by key, merge with broadcasts, FIFO, emit ----
  unsigned long long n_rec = 0, st_edges = 0, st_echo = 0, fdrop = 0, lost = 0;
  long long ovmin = LLONG_MAX;
  const long long cs = cell * p.L;
  const Rec* in_row = p.inbox + inbox_idx(p, ib, rep, e0);  // this node's row
  if constexpr (QM == 2) {
    // ---- 2'. FQCODEL: per edge, its ops in key order through the queue disc, the device-queue
    // wakes in between and up to the window end; records are emitted when a message's last
    // fragment enters the device queue (oracle fq_*) ----
    long long fq_wmin = LLONG_MAX;
    __shared__ uint32_t fq_hl_s[kFqLanes * kFqH];  // each lane's staged link header
    FqW* const fq_hl = (FqW*)(fq_hl_s);
    if (blockDim.x > kFqLanes) set_err(p, BCSIM_E_STATE);
    for (uint32_t le = tid; le < deg; le += blockDim.x) {
      const uint32_t eb = n_list && le ? ecnt[le - 1] : 0u, ee = n_list ? ecnt[le] : 0u;
      const uint32_t e = e0 + le;
      const uint32_t s = p.mesh ? (le < i ? le : le + 1) : AT(p.col, e, p.E);
      uint64_t* lwp = p.link + link_index(p, rep, i, e0, le);
      const uint64_t lw = *lwp;
      Rec* ir = const_cast<Rec*>(in_row) + le;
      Rec r0{};
      if (rxe) r0 = ld_rec(ir);
      uint4 w0 = make_uint4(0, 0, 0, 0), w1 = make_uint4(0, 0, 0, 0);
      if (sl0) w0 = *eslot_at(p, ob, rep, e);
      if (sl1) w1 = *eslot_at(p, obp, rep, e);
      bool he = false;
      RawOp eo = raw_zero();
      if (rxe) {
        const long long ta0 = cs + r0.t_off;
        if (slot_live(r0.flags, cell_tag(p, cell)) && ta0 >= t_lo && ta0 < t_hi && p.echo) {
          const int bg = (r0.flags & RF_BIG) ? 1 : 0;
          const int64_t pin = p.prop_const >= 0 ? p.prop_const : AT(p.prop_in, e, p.E);
          eo = raw_make(ta0, static_cast<uint32_t>(pin + sel2(p.tx_last, bg)), s, r0.sub,
                        static_cast<uint8_t>(OP_ECHO | (bg ? (OPF_BIG << 2) : 0)));
          he = true;
          ++st_echo;
        }
      }
      bool hr = false, hr2 = false;
      RawOp ro = raw_zero(), ro2 = raw_zero();
      if (sl0) {
        ro = slot_op(p, w0, i, e);
        hr = raw_t(ro) >= t_lo && raw_t(ro) < t_hi;
        if (hr) ++st_ops;
      }
      if (sl1) {
        ro2 = slot_op(p, w1, i, e);
        hr2 = raw_t(ro2) >= t_lo && raw_t(ro2) < t_hi;
        if (hr2) ++st_ops;
      }
      for (uint32_t a = eb + 1; a < ee; ++a) {  // insertion sort of this edge's ops (few)
        const uint32_t x = eidx[a];
        const RawOp ox = ld_raw(&ops[x]);  // (raw words: an Op copy went through scratch)
        uint32_t b2 = a;
        while (b2 > eb) {
          const RawOp oy = ld_raw(&ops[eidx[b2 - 1]]);
          if (!raw_key_less(ox, raw_sub(ox), oy, raw_sub(oy))) break;
          eidx[b2] = eidx[b2 - 1];
          --b2;
        }
        eidx[b2] = x;
      }
      ++st_edges;
      uint32_t lc = static_cast<uint32_t>(lw & 0xFFFFu);
      const int64_t pr = p.prop_const >= 0 ? p.prop_const : prop[le];
      const uint32_t slot = p.mesh ? s * (p.N - 1) + (i < s ? i : i - 1) : AT(p.rev, e, p.E);
      const uint32_t dg = rep * p.N + s;
      FqLink FL = fq_link(p, eb0 + le, e, i, s, fq_hl + tid * kFqH);
      FqCount fc{0, 0};
      // a delivery: the record for the receiver's inbox slot / extras / overflow (as link_node)
      auto emit = [&](uint32_t sub, uint32_t bz, uint32_t bw24, int big, int64_t end) {
        const int64_t ta = end + pr;
        const long long ca = ta / p.L;
        const long long rel = ca - cell;
        if (rel < 1) {
          set_err(p, BCSIM_E_TIE);  // lookahead violated
          return;
        }
        ++n_rec;
        const uint32_t tof = static_cast<uint32_t>(ta - ca * p.L);
        const uint32_t w3 = bw24 | (static_cast<uint32_t>(RF_VALID | (big ? RF_BIG : 0)) << 24) |
            (emit_tag(cell / p.n_buckets, static_cast<uint32_t>(cell % p.n_buckets), ca - cell, p.n_buckets) << 27);
        Rec r;
        {
          const uint4 rv = make_uint4(tof, sub, bz, w3);
          __builtin_memcpy(&r, &rv, sizeof r);
        }
        const bool owner = lc != (static_cast<uint32_t>(ca) & 0xFFFFu);
        lc = static_cast<uint32_t>(ca) & 0xFFFFu;
        if (XR) {
          const uint32_t orank = p.owner[s];
          if (orank != p.rank) {  // (with the sending socket's port for the receiver's echo class)
            XRec x;
            x.r = r;
            if (owner) x.r.flags = static_cast<uint8_t>(x.r.flags | RF_OWNER);
            x.cell = ca | (static_cast<long long>(FL.pa - 49152u) << kXPortShift);
            x.slot = slot;
            x.g = dg;
            link_stage(p, L, g, B + 1 + orank, x);
            return;
          }
        }
        if (rel < static_cast<long long>(B)) {
          const uint32_t bk = static_cast<uint32_t>(ca % B);
          if (owner) {
            st_rec(&AT(p.inbox, inbox_idx(p, bk, rep, slot), p.cap_inbox), r);
            if (p.mesh)
              set_flag_once(&AT(p.rtile, kRtPad * ((static_cast<size_t>(bk) * p.R + rep) * p.n_tiles + (s >> 6)), kRtPad * (static_cast<uint64_t>(B) * p.R * p.n_tiles)));
          } else {
            XRec x;
            x.r = r;
            x.cell = ca;
            x.slot = slot;
            x.g = dg;
            link_stage(p, L, g, bk, x);
          }
          if (!(owner && p.mesh)) AT(p.iflag, static_cast<size_t>(bk) * p.NT + dg, static_cast<uint64_t>(B) * p.NT) = 1;
          atomicAdd(&L.lcnt[bk], 1u);
          atomicMin(&L.lmin[bk], tof);
        } else {
          XRec x;
          x.r = r;
          if (owner) x.r.flags = static_cast<uint8_t>(x.r.flags | RF_OWNER);
          x.cell = ca;
          x.slot = slot;
          x.g = dg;
          link_stage(p, L, g, B, x);
          if (ca < ovmin) ovmin = ca;
        }
      };
      uint32_t a = eb, bi = 0;
      for (;;) {
        while (bi < n_bc && (op_flags(L.bco[bi]) & OPF_PAXOS) && le == 0) ++bi;
        // the earliest of the five sources in key order; the op is assembled word by word
        // (raw_sel), never by selecting RawOp values
        int src = -1;
        RawOp o = raw_zero();
        uint32_t sub = 0;
        if (bi < n_bc) {
          raw_sel(o, ld_raw_lds(&L.bco[bi]), true);
          sub = raw_sub(o) + ((raw_flags(o) & OPF_PAXOS) ? le - 1 : le);
          src = 1;
        }
        if (a < ee) {
          const RawOp oa = ld_raw(&ops[eidx[a]]);
          const bool c = src < 0 || raw_key_less(oa, raw_sub(oa), o, sub);
          raw_sel(o, oa, c);
          if (c) {
            sub = raw_sub(oa);
            src = 0;
          }
        }
        {
          const bool c = hr && (src < 0 || raw_key_less(ro, raw_sub(ro), o, sub));
          raw_sel(o, ro, c);
          if (c) {
            sub = raw_sub(ro);
            src = 2;
          }
        }
        {
          const bool c = hr2 && (src < 0 || raw_key_less(ro2, raw_sub(ro2), o, sub));
          raw_sel(o, ro2, c);
          if (c) {
            sub = raw_sub(ro2);
            src = 4;
          }
        }
        {
          const bool c = he && (src < 0 || raw_key_less(eo, raw_sub(eo), o, sub));
          raw_sel(o, eo, c);
          if (c) {
            sub = raw_sub(eo);
            src = 3;
          }
        }
        if (src < 0) break;
        if (src == 0)
          ++a;
        else if (src == 1)
          ++bi;
        else if (src == 2)
          hr = false;
        else if (src == 4)
          hr2 = false;
        else
          he = false;
        if ((src == 2 || src == 4) && raw_kind(o) == OP_SEND) ++sends;
        const bool is_echo = src != 1 && raw_kind(o) == OP_ECHO;
        const int big = (raw_flags(o) & OPF_BIG) ? 1 : 0;
        const int64_t ot = raw_t(o);
        fq_advance(p, FL, ot, emit, fc);  // wakes at <= ot come first
        FL.src = static_cast<uint32_t>(src);
        fq_send(p, FL, ot, sub, o.b.z, o.b.w & 0x00FFFFFFu, big, is_echo, emit, fc);
      }
      fq_advance(p, FL, t_hi - 1, emit, fc);
      // the next wake with packets waiting in the disc is this node's next link event (a wake
      // of an empty disc only resets flow states and is applied when the link is next used)
      if (FL.h[FQ_STOP] && FL.h[FQ_QP]) {
        const long long tw = FL.dev[FL.h[FQ_DH]];
        if (tw < fq_wmin) fq_wmin = tw;
      }
      fdrop += fc.fdrop;
      lost += fc.lost;
      const int64_t bu = fq_ld64(FL.h + FQ_DEND);
      if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
      *lwp = (static_cast<uint64_t>(bu) << 16) | lc;
      fq_unlink(p, FL, eb0 + le);
    }
    if (fq_wmin != LLONG_MAX) atomicMin(&L.omin, fq_wmin);
    __syncthreads();
    if (p.wgt && tid == 0) ph[2] = __builtin_amdgcn_s_memrealtime();
    const LinkCounts lc8{static_cast<uint32_t>(dropped), static_cast<uint32_t>(sends), static_cast<uint32_t>(n_rec),
                         static_cast<uint32_t>(st_ops),  static_cast<uint32_t>(st_edges), static_cast<uint32_t>(st_echo),
                         static_cast<uint32_t>(fdrop),   static_cast<uint32_t>(lost)};
    link_finish(p, L, g, ops, n, t_hi, n_lists, ovmin, lc8, sl1 && final_win, rx && final_win, obp, fidx, wg_t0, ph, n_in);
    return;
  } else {
  for (uint32_t le = tid; le < deg; le += blockDim.x) {
    const uint32_t eb = n_list && le ? ecnt[le - 1] : 0u, ee = n_list ? ecnt[le] : 0u;
    const uint32_t e = e0 + le;
    // full mesh: peers ascending without self (validated on the host)
    const uint32_t s = p.mesh ? (le < i ? le : le + 1) : AT(p.col, e, p.E);
    // link state of an edge that is certainly used: issued before the inbox / reply-slot
    // loads below so that the three HBM reads overlap instead of forming a chain
    const bool pre = n_bc != 0 || ee > eb;
    uint64_t* lwp = nullptr;
    uint64_t lw = 0;
    if (pre) {
      lwp = p.link + link_index(p, rep, i, e0, le);
      lw = *lwp;
    }
    // The four op sources of this edge are merged as raw 32-byte words (RawOp): selecting
    // whole Op structs with int16 members between sources was miscompiled on gfx950 /
    // ROCm 7.2 (a record took f0 from a broadcast and the rest from a listed op; the Raft
    // N>=300 parity gap).  Integer word selects are what the compiler sees.
    // implicit echo: this node's main inbox record of in-slot le, delivered in
    // [t_lo, t_hi), goes back out on out-edge le (the same peer); release the slot.
    // All of the edge's loads (link word above, inbox record, reply slots) are issued before
    // the slot release: a load after that store could not be moved above it (possible
    // alias) and would cost a second memory round trip per edge.
    Rec* ir = const_cast<Rec*>(in_row) + le;
    Rec r0{};
    if (rxe) r0 = ld_rec(ir);
    uint4 w0 = make_uint4(0, 0, 0, 0), w1 = make_uint4(0, 0, 0, 0);
    if (sl0) w0 = *eslot_at(p, ob, rep, e);
    if (sl1) w1 = *eslot_at(p, obp, rep, e);
    bool he = false;
    RawOp eo = raw_zero();
    if (rxe) {
      const long long ta0 = cs + r0.t_off;
      if (slot_live(r0.flags, cell_tag(p, cell)) && ta0 >= t_lo && ta0 < t_hi) {
        if (p.echo) {
          const int bg = (r0.flags & RF_BIG) ? 1 : 0;
          const int64_t pin = p.prop_const >= 0 ? p.prop_const : AT(p.prop_in, e, p.E);
          eo = raw_make(ta0, static_cast<uint32_t>(pin + sel2(p.tx_last, bg)), s, r0.sub,
                        static_cast<uint8_t>(OP_ECHO | (bg ? (OPF_BIG << 2) : 0)));
          he = true;
          ++st_echo;
        }
      }
    }
    // this edge's reply-slot ops due in [t_lo, t_hi): of this arrival cell and the previous one
    bool hr = false, hr2 = false;
    RawOp ro = raw_zero(), ro2 = raw_zero();
    if (sl0) {
      ro = slot_op(p, w0, i, e);
      hr = raw_t(ro) >= t_lo && raw_t(ro) < t_hi;
      if (hr) ++st_ops;
    }
    if (sl1) {
      ro2 = slot_op(p, w1, i, e);
      hr2 = raw_t(ro2) >= t_lo && raw_t(ro2) < t_hi;
      if (hr2) ++st_ops;
    }
    if (ee == eb && n_bc == 0 && !he && !hr && !hr2) continue;
    for (uint32_t a = eb + 1; a < ee; ++a) {  // insertion sort of this edge's ops (few)
      const uint32_t x = eidx[a];
      const RawOp ox = ld_raw(&ops[x]);  // (raw words: an Op copy went through scratch)
      uint32_t b2 = a;
      while (b2 > eb) {
        const RawOp oy = ld_raw(&ops[eidx[b2 - 1]]);
        if (!raw_key_less(ox, raw_sub(ox), oy, raw_sub(oy))) break;
        eidx[b2] = eidx[b2 - 1];
        --b2;
      }
      eidx[b2] = x;
    }
    ++st_edges;
    if (!pre) {
      lwp = p.link + link_index(p, rep, i, e0, le);
      lw = *lwp;
    }
    // link word: FIFO busy_until (ns, < 2^48) and the 16 low bits of the arrival cell of the
    // edge's last record (slot ownership; a false "not owner" after 2^16 cells only routes a
    // record through the extras list, which delivers it identically)
    int64_t bu = static_cast<int64_t>(lw >> 16);
    uint32_t lc = static_cast<uint32_t>(lw & 0xFFFFu);
    uint64_t qm = 0;
    uint64_t* qr = nullptr;
    if (QM) {
      qm = p.qmeta[eb0 + le];
      qr = p.qring + (eb0 + le) * p.cap_q;
    }
    const int64_t pr = p.prop_const >= 0 ? p.prop_const : prop[le];
    // in-slot of this edge in the receiver's row (full mesh: arithmetic)
    const uint32_t slot = p.mesh ? s * (p.N - 1) + (i < s ? i : i - 1) : AT(p.rev, e, p.E);
    const uint32_t dg = rep * p.N + s;
    uint32_t a = eb, bi = 0;
    for (;;) {
      // next broadcast that targets this edge (Paxos broadcasts skip peers[0])
      while (bi < n_bc && (op_flags(L.bco[bi]) & OPF_PAXOS) && le == 0) ++bi;
      // four sorted sources, each applied in canonical key order: broadcasts
      // (1), this edge's listed ops (0), the reply slot (2), the implicit echo (3)
      int src = -1;
      RawOp o = raw_zero();
      uint32_t sub = 0;
      if (bi < n_bc) {
        o = ld_raw_lds(&L.bco[bi]);
        sub = raw_sub(o) + ((raw_flags(o) & OPF_PAXOS) ? le - 1 : le);
        src = 1;
      }
      if (a < ee) {
        const RawOp oa = ld_raw(&ops[eidx[a]]);
        if (src < 0 || raw_key_less(oa, raw_sub(oa), o, sub)) {
          o = oa;
          sub = raw_sub(oa);
          src = 0;
        }
      }
      if (hr && (src < 0 || raw_key_less(ro, raw_sub(ro), o, sub))) {
        o = ro;
        sub = raw_sub(ro);
        src = 2;
      }
      if (hr2 && (src < 0 || raw_key_less(ro2, raw_sub(ro2), o, sub))) {
        o = ro2;
        sub = raw_sub(ro2);
        src = 4;
      }
      if (he && (src < 0 || raw_key_less(eo, raw_sub(eo), o, sub))) {
        o = eo;
        sub = raw_sub(eo);
        src = 3;
      }
      if (src < 0) break;
      if (src == 0)
        ++a;
      else if (src == 1)
        ++bi;
      else if (src == 2)
        hr = false;
      else if (src == 4)
        hr2 = false;
      else
        he = false;
      if ((src == 2 || src == 4) && raw_kind(o) == OP_SEND) ++sends;
      const bool is_echo = src != 1 && raw_kind(o) == OP_ECHO;
      const int big = (raw_flags(o) & OPF_BIG) ? 1 : 0;
      const int64_t ot = raw_t(o);
      const int64_t start = bu > ot ? bu : ot;
      if (QM) {  // DROPTAIL: a refused fragment loses the message (its accepted prefix still occupies the link)
        const uint32_t F = sel2(p.nfr, big);
        const uint32_t k = q_admit(p, qr, qm, ot, big, start);
        if (k < F) {
          fdrop += F - k;
          if (k) bu = start + static_cast<int64_t>(k) * sel2(p.tx_full, big);
          if (!is_echo) ++lost;
          continue;
        }
      }
      const int64_t end = start + sel2(p.tx_tot, big);
      bu = end;
      if (is_echo) continue;
      const int64_t ta = end + pr;
      const long long ca = ta / p.L;
      const long long rel = ca - cell;
      if (rel < 1) {
        set_err(p, BCSIM_E_TIE);  // lookahead violated
        continue;
      }
      ++n_rec;
      // the record: t_off | sub | payload word (f0, f1) | (f2, type, flags) -- raw words only
      const uint32_t tof = static_cast<uint32_t>(ta - ca * p.L);
      const uint32_t w3 = (o.b.w & 0x00FFFFFFu) | (static_cast<uint32_t>(RF_VALID | (big ? RF_BIG : 0)) << 24) |
          (emit_tag(cell / p.n_buckets, static_cast<uint32_t>(cell % p.n_buckets), ca - cell, p.n_buckets) << 27);
      Rec r;
      {
        const uint4 rv = make_uint4(tof, sub, o.b.z, w3);
        __builtin_memcpy(&r, &rv, sizeof r);
      }
      // sparse mode has no slots: every record is a list record
      const bool owner = !p.sparse && lc != (static_cast<uint32_t>(ca) & 0xFFFFu);
      lc = static_cast<uint32_t>(ca) & 0xFFFFu;
      if (XR) {
        const uint32_t orank = p.owner[s];
        if (orank != p.rank) {  // receiver on another GPU: ship the record (k_import places it)
          XRec x;
          x.r = r;
          if (owner) x.r.flags = static_cast<uint8_t>(x.r.flags | RF_OWNER);
          x.cell = ca;
          x.slot = slot;
          x.g = dg;
          link_stage(p, L, g, B + 1 + orank, x);
          continue;
        }
      }
      if (rel < static_cast<long long>(B)) {
        const uint32_t bk = static_cast<uint32_t>(ca % B);
        bool flag_rx = true;
        if (owner) {
          // the receiver's in-slot of this bucket, written directly: a receiver-major 16-byte
          // scatter from XCD-contiguous senders merges in L2 and costs ~2x a coalesced row
          // write, a third of staging sender-major and transposing (tools/microbench/scatter.hip)
          st_rec(&AT(p.inbox, inbox_idx(p, bk, rep, slot), p.cap_inbox), r);
          xs_mark(p, bk, rep, i, s, w3);
          if (p.mesh) {
            // receiver-tile flag: one LDS byte per 64-node tile, flushed once per workgroup
            uint32_t tb = kInvalid;
            if (tmap) {  // the first bucket seen owns the LDS map; others flag directly
              tb = L.tbk;
              if (tb == kInvalid) {
                const uint32_t old = atomicCAS(&L.tbk, kInvalid, bk);
                tb = old == kInvalid ? bk : old;
              }
            }
            if (tb == bk)
              L.tflag[s >> 6] = 1;
            else
              set_flag_once(&AT(p.rtile, kRtPad * ((static_cast<size_t>(bk) * p.R + rep) * p.n_tiles + (s >> 6)), kRtPad * (static_cast<uint64_t>(B) * p.R * p.n_tiles)));
            flag_rx = false;
          }
        } else {
          XRec x;
          x.r = r;
          x.cell = ca;
          x.slot = slot;
          x.g = dg;
          link_stage(p, L, g, bk, x);
        }
        if (flag_rx) AT(p.iflag, static_cast<size_t>(bk) * p.NT + dg, static_cast<uint64_t>(B) * p.NT) = 1;
        if (bk != cb) {
          if (cbn) {
            atomicAdd(&L.lcnt[cb], cbn);
            atomicMin(&L.lmin[cb], cmn);
          }
          cb = bk;
          cbn = 0;
          cmn = ~0u;
        }
        ++cbn;
        if (tof < cmn) cmn = tof;
      } else {
        XRec x;
        x.r = r;
        if (owner) x.r.flags = static_cast<uint8_t>(x.r.flags | RF_OWNER);
        x.cell = ca;
        x.slot = slot;
        x.g = dg;
        link_stage(p, L, g, B, x);
        if (ca < ovmin) ovmin = ca;
      }
    }
    if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
    *lwp = (static_cast<uint64_t>(bu) << 16) | lc;
    if (QM) p.qmeta[eb0 + le] = qm;
  }
  if (cbn) {
    atomicAdd(&L.lcnt[cb], cbn);
    atomicMin(&L.lmin[cb], cmn);
  }
  __syncthreads();
  // flush the receiver-tile flags of this sender's full-mesh records
  if (tmap && L.tbk != kInvalid) {
    const size_t tb = (static_cast<size_t>(L.tbk) * p.R + rep) * p.n_tiles;
    for (uint32_t k = tid; k < p.n_tiles; k += blockDim.x)
      if (L.tflag[k]) set_flag_once(&AT(p.rtile, kRtPad * (tb + k), kRtPad * (static_cast<uint64_t>(B) * p.R * p.n_tiles)));
  }

  if (p.wgt && tid == 0) ph[2] = __builtin_amdgcn_s_memrealtime();
  const LinkCounts lc8{static_cast<uint32_t>(dropped), static_cast<uint32_t>(sends), static_cast<uint32_t>(n_rec),
                       static_cast<uint32_t>(st_ops),  static_cast<uint32_t>(st_edges), static_cast<uint32_t>(st_echo),
                       static_cast<uint32_t>(fdrop),   static_cast<uint32_t>(lost)};
  link_finish(p, L, g, ops, n, t_hi, n_lists, ovmin, lc8, sl1 && final_win, rx && final_win, obp, fidx, wg_t0, ph, n_in);
  }  // QM != 2
}

// LOOP: a small grid walks list 3 (the nodes k_gossip_link left over)
__device__ void node_desc_flush(const KP& p, uint32_t g, long long cell, long long t_lo);
// (FQCODEL: at most 256 lanes, so that the per-edge queue-disc walk gets the registers it needs
// instead of spilling them -- 168 B/lane of scratch under the 1024-lane bound)
// (summary mode) gnode g's row-uniform link state written out to its out-edges' words (the
// generic kernels read and write physical words only); every thread of the workgroup calls it
__device__ void rul_flush(const KP& p, uint32_t g) {
  const uint64_t ru = gbl(p.rul)[g];
  if (!(ru >> 63)) return;  // (uniform)
  const uint32_t rep = g / p.N, i = g % p.N, N1 = p.N - 1;
  const uint64_t w = ru & ~(1ull << 63);
  uint64_t* lrow = p.link + edge_loc(p, rep, i * N1);
  for (uint32_t le = tidx(); le < N1; le += blockDim.x) {
    const uint32_t s = le < i ? le : le + 1;
    if (!((gbl(p.rex)[static_cast<size_t>(g) * p.n_tiles + (s >> 6)] >> (s & 63u)) & 1ull)) gbl(lrow)[le] = w;
  }
  __syncthreads();
  if (tidx() == 0) gbl(p.rul)[g] = 0ull;
}

template <int QM, bool XR, bool LOOP = false>
__global__ __launch_bounds__(QM != 0 ? 256 : (LOOP ? kLinkLoopThreads : 1024)) void k_link(const KP* __restrict__ pk, long long cell, long long t_lo,
                                              long long t_hi, int final_win) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  if (LOOP) {
    if constexpr (!QM && !XR) {
      if (cell < 0) {  // (a chained window, or none)
        if (!win_take(p, cell, t_lo, t_hi, final_win)) return;
        if (blockIdx.x == 0 && tidx() == 0)
          p.act_n[0] = 0;  // (list 0 is free again -- the closing k_next builds the next frontier)
      }
    }
    const uint32_t ll = p.loop_list;
    for (ListRange lr = list_range(p.act_n[ll]); lr.k < lr.end; lr.k += lr.step) {
      const uint32_t g = p.act[static_cast<size_t>(ll) * p.NT + lr.k];
      // (the nodes the descriptor-aware kernels handed on: their descriptors first, as
      // pending echoes on the link words and reply slots -- this kernel knows no descriptors)
      if (!QM && !XR && p.sum) rul_flush(p, g);  // (then its descriptors, below)
      if (!QM && !XR && p.desc) {
        node_desc_flush(p, g, cell, t_lo);
        __syncthreads();
      }
      link_node<QM, XR>(pk, g, cell, t_lo, t_hi, final_win);
      __syncthreads();
    }
    return;
  }
  uint32_t k;
  if (list_one(p.act_n[1], k)) link_node<QM, XR>(pk, p.act[p.NT + k], cell, t_lo, t_hi, final_win);
}

// ---------------------------------------------------------------------------
// k_link_mesh (dense layout, full mesh, fixed app delay, infinite queues, one rank): the
// link stage of a node whose due ops are all broadcasts -- the PBFT heavy waves, where
// every out-edge carries a broadcast record, a reply-slot PREPARE_RES and/or the implicit
// echo.  Same result as link_node (the merge of the four sources in key order per edge,
// the FIFO, the record into the receiver's in-slot / extras / overflow), with the
// per-edge state held as compact words instead of 32-byte ops (link_node: 127 VGPRs and
// a scratch spill), and kU out-edges per lane per iteration whose loads (link word, inbox
// record, reply slots) are all issued before the first edge's stores, so a lane has kU
// memory round trips in flight instead of one.  A node with a listed op due (unicast /
// echo op), too many broadcasts or an unexpanded jitter broadcast goes to list 3, which
// k_link<false, false, LOOP> finishes after this kernel.
// kMeshU (template): out-edges per lane per iteration, their loads issued together
__device__ inline bool kless(int64_t ta, uint32_t dta, uint32_t oa, uint32_t sa, int64_t tb, uint32_t dtb, uint32_t ob,
                             uint32_t sb) {
  if (ta != tb) return ta < tb;
  const int64_t xa = ta - dta, xb = tb - dtb;
  if (xa != xb) return xa < xb;
  if (oa != ob) return oa < ob;
  return sa < sb;
}

// Cross-rank broadcast de-duplication (SURVEY.md §8e "Collective"): a wave of k_link_mesh
// covers 64 consecutive out-edges of one sender, i.e. 64 consecutive receivers (skipping the
// sender itself).  When the lanes holding a record for one other rank form a contiguous run and
// their records are equal up to the schedule counter, which steps by one per edge (a
// broadcast: sub + le, pbft-node.cc:360-367), the run is shipped as ONE range record -- the
// first record, sender node in `slot`, first receiver in `g`, count and a range bit in the top
// bits of `cell` -- and k_import expands it on the receiving rank.  Anything else is shipped
// record by record.  Convergent: every lane of the wave calls it.
constexpr uint64_t kXRange = 1ull << 62;
constexpr int kXCountShift = 48;
constexpr uint64_t kXCellMask = (1ull << kXCountShift) - 1;
__device__ inline void xr_ship(const KP& p, LinkShared& L, uint32_t g, uint32_t i, uint32_t le, bool hp, const XRec& x,
                               uint32_t orank) {
  const uint32_t lane = tidx() & 63u;
  unsigned long long rem = __ballot(hp);
  const uint4 rw = *reinterpret_cast<const uint4*>(&x.r);
  while (rem) {
    const int ld = __ffsll(static_cast<long long>(rem)) - 1;
    const uint32_t rk = __shfl(orank, ld, 64);
    const unsigned long long grp = __ballot(hp && orank == rk);
    const uint32_t l_tof = __shfl(rw.x, ld, 64), l_sub = __shfl(rw.y, ld, 64);
    const uint32_t l_z = __shfl(rw.z, ld, 64), l_w = __shfl(rw.w, ld, 64);
    const long long l_cell = __shfl(x.cell, ld, 64);
    const uint32_t l_le = __shfl(le, ld, 64);
    const bool mine = hp && orank == rk;
    const bool ok = mine && rw.x == l_tof && rw.z == l_z && rw.w == l_w && x.cell == l_cell && rw.y == l_sub + (le - l_le);
    const unsigned long long okm = __ballot(ok);
    const unsigned long long run = grp >> ld;  // contiguous lanes ld .. ld + n - 1
    const uint32_t n = static_cast<uint32_t>(__popcll(grp));
    if (okm == grp && n >= 2 && (run & (run + 1)) == 0) {
      if (lane == static_cast<uint32_t>(ld)) {
        XRec xr = x;
        xr.cell = static_cast<long long>(static_cast<uint64_t>(x.cell) | kXRange | (static_cast<uint64_t>(n) << kXCountShift));
        xr.slot = i;  // the sender (range records: full mesh only)
        link_stage(p, L, g, p.n_buckets + 1 + rk, xr);
      }
    } else if (mine) {
      link_stage(p, L, g, p.n_buckets + 1 + rk, x);
    }
    rem &= ~grp;
  }
}

// k_link_mesh's view of the node's descriptors (k_scan_pbft): the live reply descriptors of
// this arrival cell (0) and the previous one (1) with their bitmaps and per-word rank
// prefixes, and the pending echo descriptors with theirs
// (2.6 KB: with the 32 KB of parked link words and LinkShared a 256-lane k_link_mesh workgroup
// stays under 40 KB of LDS, four per CU; a 4.7 KB layout cost 18 % of k_link_mesh time)
struct MeshDesc {
  uint32_t rb[2][kDescWords];
  uint16_t rp[2][kDescWords];  // (ranks < 4096)
  uint32_t eb[kEDesc][kDescWords];
  long long et[kEDesc];
  uint32_t ebig[kEDesc];
};

__device__ inline long long desc_due(const uint4& d) {
  return static_cast<long long>((static_cast<uint64_t>(d.y) << 32) | d.x);
}

// LDS copies of the descriptor bitmaps (reply descriptor h if use[h]; the ne pending echo
// descriptors) and the reply bitmaps' exclusive rank prefixes per word.  Block-uniform call.
__device__ inline void mesh_desc_load(const KP& p, MeshDesc& D, uint32_t g, uint32_t ob, uint32_t obp, bool use0,
                                      bool use1, uint32_t ne) {
  const uint32_t tid = tidx(), bs = blockDim.x, dw = p.dwords;
  for (uint32_t k = tid; k < dw; k += bs) {
    if (use0) D.rb[0][k] = p.rbits[(static_cast<size_t>(ob) * p.NT + g) * dw + k];
    if (use1) D.rb[1][k] = p.rbits[(static_cast<size_t>(obp) * p.NT + g) * dw + k];
  }
  for (uint32_t k = tid; k < ne * dw; k += bs) D.eb[k / dw][k % dw] = p.ebits[static_cast<size_t>(g) * kEDesc * dw + k];
  if (tid < ne) {
    const uint4 ed = p.edesc[static_cast<size_t>(g) * kEDesc + tid];
    D.et[tid] = desc_due(ed);
    D.ebig[tid] = ed.z;
  }
  __syncthreads();
  if (tid < 64 && (use0 || use1)) {  // wave 0: two words per lane (dw <= 128)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!(h ? use1 : use0)) continue;
      const uint32_t k = 2 * tid;
      const uint32_t a = k < dw ? static_cast<uint32_t>(__popc(D.rb[h][k])) : 0u;
      const uint32_t b = k + 1 < dw ? static_cast<uint32_t>(__popc(D.rb[h][k + 1])) : 0u;
      uint32_t in = a + b;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(in, off, 64);
        if (tid >= static_cast<uint32_t>(off)) in += v;
      }
      if (k < dw) D.rp[h][k] = static_cast<uint16_t>(in - a - b);
      if (k + 1 < dw) D.rp[h][k + 1] = static_cast<uint16_t>(in - b);
    }
  }
  __syncthreads();
}

// bit le of bitmap row w (LDS)
__device__ inline bool desc_bit(const uint32_t* w, uint32_t le) { return (w[le >> 5] >> (le & 31u)) & 1u; }
// rank of in-slot le among the set bits of reply bitmap h
__device__ inline uint32_t desc_rank(const MeshDesc& D, int h, uint32_t le) {
  return D.rp[h][le >> 5] + static_cast<uint32_t>(__popc(D.rb[h][le >> 5] & ((1u << (le & 31u)) - 1u)));
}

// A node leaving the descriptor-aware kernels for the generic ones (which know no descriptors):
// its pending echo descriptors go onto the link words, its live reply descriptors into reply
// slots (the slot flags they stand for).  Block-uniform call.
__device__ inline void mesh_desc_flush(const KP& p, MeshDesc& D, uint32_t g, uint32_t ob, uint32_t obp, uint32_t sf0,
                                       uint32_t sf1, const uint4& rd0, const uint4& rd1, bool dl0, bool dl1, uint32_t ne) {
  const uint32_t tid = tidx();
  const uint32_t rep = g / p.N, i = g % p.N;
  mesh_desc_load(p, D, g, ob, obp, dl0, dl1, ne);
  const uint32_t e0m = AT(p.row, i, p.N + 1), degm = AT(p.row, i + 1, p.N + 1) - e0m;
  for (uint32_t le = tid; le < degm; le += blockDim.x) {
    if (ne) {
      uint64_t* lwp = p.link + edge_loc(p, rep, e0m + le);
      const uint64_t lw = *lwp;
      int64_t bu = static_cast<int64_t>(lw >> 16);
      bool any = false;
      for (uint32_t d = 0; d < ne; ++d)
        if (desc_bit(D.eb[d], le)) {
          bu = (bu > D.et[d] ? bu : D.et[d]) + sel2(p.tx_tot, D.ebig[d] != 0);
          any = true;
        }
      if (any) {
        if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
        *lwp = (static_cast<uint64_t>(bu) << 16) | (lw & 0xFFFFull);
      }
    }
    if (dl0 && desc_bit(D.rb[0], le))
      *eslot_at(p, ob, rep, e0m + le) = make_uint4(rd0.x, rd0.y, rd0.z + desc_rank(D, 0, le), rd0.w);
    if (dl1 && desc_bit(D.rb[1], le))
      *eslot_at(p, obp, rep, e0m + le) = make_uint4(rd1.x, rd1.y, rd1.z + desc_rank(D, 1, le), rd1.w);
  }
  if (tid == 0) {
    if (ne) AT(p.en, g, p.NT) = 0;
    const size_t R4 = static_cast<uint64_t>(kOpRing) * p.NT;
    if (sf0 & kSfD)  // kSfD0 -> bit 0, kSfD1 -> bit 1 (dead descriptors just go)
      AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, R4) =
          static_cast<uint8_t>((sf0 & ~kSfD) | (dl0 ? ((sf0 >> 4) & 3u) : 0u));
    if (sf1 & kSfD1)
      AT(p.sflag, static_cast<size_t>(obp) * p.NT + g, R4) = static_cast<uint8_t>((sf1 & ~kSfD1) | (dl1 ? 2u : 0u));
  }
}

// The descriptor flush of a node handed to the generic link kernel (k_link<.., LOOP> over list 2 --
// the list-2 overlap -- and list 3 -- the nodes k_mesh_prep left): mesh_desc_flush if it has
// pending echo or live reply descriptors, as k_link_mesh does for the nodes it hands on.
// Block-uniform call.
__device__ void node_desc_flush(const KP& p, uint32_t g, long long cell, long long t_lo) {
  __shared__ MeshDesc D;
  const uint32_t ob = static_cast<uint32_t>(cell % kOpRing), obp = static_cast<uint32_t>((cell + kOpRing - 1) % kOpRing);
  const size_t R4 = static_cast<uint64_t>(kOpRing) * p.NT;
  const uint32_t sf0 = AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, R4);
  const uint32_t sf1 = AT(p.sflag, static_cast<size_t>(obp) * p.NT + g, R4);
  uint4 rd0 = make_uint4(0, 0, 0, 0), rd1 = make_uint4(0, 0, 0, 0);
  if (sf0 & kSfD) rd0 = p.rdesc[static_cast<size_t>(ob) * p.NT + g];
  if (sf1 & kSfD1) rd1 = p.rdesc[static_cast<size_t>(obp) * p.NT + g];
  const bool dl0 = (sf0 & kSfD) && desc_due(rd0) >= t_lo;
  const bool dl1 = (sf1 & kSfD1) && desc_due(rd1) >= t_lo;
  const uint32_t ne = AT(p.en, g, p.NT);
  if (ne || dl0 || dl1) mesh_desc_flush(p, D, g, ob, obp, sf0, sf1, rd0, rd1, dl0, dl1, ne);
}

template <bool XR, int kMeshU, bool PF>
__global__ __launch_bounds__(XR ? 256 : 1024) void k_link_mesh(const KP* __restrict__ pk, long long cell, long long t_lo,
                                                   long long t_hi, int final_win, uint32_t epoch, uint32_t wep) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ LinkShared L;
  __shared__ MeshDesc D;
  uint32_t kk;
  if (!list_one(p.act_n[1], kk)) return;
  const uint32_t g = p.act[p.NT + kk];
  if (wep && AT(p.l2mark, g, p.NT) == wep) return;  // left to the generic kernels (second stream)
  const uint32_t tid = tidx();
  const uint32_t n = AT(p.n_ops, g, p.NT);
  const uint32_t ob = static_cast<uint32_t>(cell % kOpRing), obp = static_cast<uint32_t>((cell + kOpRing - 1) % kOpRing);
  const uint32_t sf0 = p.eslot ? AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, static_cast<uint64_t>(kOpRing) * p.NT) : 0u;
  const uint32_t sf1 = p.eslot ? AT(p.sflag, static_cast<size_t>(obp) * p.NT + g, static_cast<uint64_t>(kOpRing) * p.NT) : 0u;
  const bool sl0 = sf0 & 1u, sl1 = sf1 & 2u;
  // reply descriptors (k_scan_pbft): live = not sent yet; sd0 / sd1 = due in this window.
  // Descriptors need the PF variant (the pending echoes are applied to the LDS link words);
  // the host enables them only with it.
  const bool dsc = PF && p.desc;
  if (!PF && p.desc) {
    if (tid == 0) set_err(p, BCSIM_E_STATE);
    return;
  }
  uint4 rd0 = make_uint4(0, 0, 0, 0), rd1 = make_uint4(0, 0, 0, 0);
  if (dsc && (sf0 & kSfD)) rd0 = p.rdesc[static_cast<size_t>(ob) * p.NT + g];
  if (dsc && (sf1 & kSfD1)) rd1 = p.rdesc[static_cast<size_t>(obp) * p.NT + g];
  const bool dl0 = dsc && (sf0 & kSfD) && desc_due(rd0) >= t_lo;
  const bool dl1 = dsc && (sf1 & kSfD1) && desc_due(rd1) >= t_lo;
  const bool sd0 = dl0 && desc_due(rd0) < t_hi, sd1 = dl1 && desc_due(rd1) < t_hi;
  const uint32_t ne = dsc ? AT(p.en, g, p.NT) : 0u;  // pending echo descriptors
  const uint32_t B = p.n_buckets;
  const uint32_t ib = static_cast<uint32_t>(cell % B);
  const size_t fidx = static_cast<size_t>(ib) * p.NT + g;
  const uint32_t rep = g / p.N, i = g % p.N;
  const bool rx = p.impl && node_flagged_w(p, ib, g, rep, i, t_hi);
  const bool rxe = rx && AT(p.eapp, g, p.NT) != t_lo;  // (see link_node)
  // nothing due in the window: no op before t_hi (node_onext is exact unless LLONG_MIN; fixed
  // app delays only, so no unexpanded jitter broadcast hides behind it), no reply slot or
  // descriptor, no echo (pending echo descriptors wait for a stage that walks the edges)
  if ((n == 0 || AT(p.node_onext, g, p.NT) >= t_hi) && !sl0 && !sl1 && !sd0 && !sd1 && !rxe) {
    if (rx && final_win && tid == 0) AT(p.iflag, fidx, static_cast<uint64_t>(B) * p.NT) = 0;
    return;
  }
  const unsigned long long wg_t0 = p.wgt ? __builtin_amdgcn_s_memrealtime() : 0;
  Op* ops = p.ops + op_base(p, g);

  // ---- classify the due ops: broadcasts to LDS; anything else sends the node to list 3 ----
  for (uint32_t k = tid; k < B; k += blockDim.x) {
    L.lcnt[k] = 0;
    L.lmin[k] = ~0u;
  }
  const uint32_t n_lists = B + 1 + (XR ? p.nranks : 0);  // extras..., overflow, ranks...
  for (uint32_t k = tid; k < n_lists; k += blockDim.x) L.lst[k] = 0;
  const bool tmap = p.n_tiles <= static_cast<uint32_t>(kMaxTiles);
  if (tmap)
    for (uint32_t k = tid; k < p.n_tiles; k += blockDim.x) L.tflag[k] = 0;
  if (tid < 8) L.csum[tid] = 0;
  if (tid == 0) {
    L.n_bc = 0;
    L.n_list = 0;
    L.nst = 0;
    L.omin = LLONG_MAX;
    L.ovmin = LLONG_MAX;
    L.tbk = kInvalid;
  }
  __syncthreads();
  const uint32_t e0 = AT(p.row, i, p.N + 1), deg = AT(p.row, i + 1, p.N + 1) - e0;
  uint32_t sends = 0, dropped = 0, st_ops = 0, other = 0;
  for (uint32_t k = tid; k < n; k += blockDim.x) {
    const Op& o = ops[k];
    const uint8_t kind = op_kind(o);
    if (kind == OP_BCAST_J) {
      other += (op_flags(o) & OPF_DONE) ? 0u : 1u;
      continue;
    }
    if (o.t >= t_hi) continue;
    if (kind != OP_BCAST) {
      ++other;
      continue;
    }
    ++st_ops;
    const uint32_t pos = atomicAdd(&L.n_bc, 1u);
    if (pos < kBcastCap) L.bc[pos] = k;
    sends += deg;
    if (op_flags(o) & OPF_PAXOS) dropped += 1;
  }
  {
    const uint32_t ws = wave_sum(other);
    if ((tid & 63u) == 0 && ws) atomicAdd(&L.n_list, ws);
  }
  __syncthreads();
  const uint32_t n_bc = L.n_bc;
  if (L.n_list || n_bc > static_cast<uint32_t>(kBcastCap)) {  // not a simple node: the generic kernel
    // which knows no descriptors: the pending echoes go onto the link words, the live reply
    // descriptors into reply slots (the slot flags they stand for)
    if (ne || dl0 || dl1) mesh_desc_flush(p, D, g, ob, obp, sf0, sf1, rd0, rd1, dl0, dl1, ne);
    if (tid == 0) {
      const uint32_t pos = gadd_r(&p.act_n[3], 1u);
      AT(p.act, 3ull * p.NT + pos, 4ull * p.NT) = g;
      FDBG(L.n_list ? 8 : 9);
    }
    return;
  }
  // (BCSIM_WGT=1: phase clocks -- classify, descriptors + parked link words, edges, compaction)
  unsigned long long ph[4] = {wg_t0, wg_t0, wg_t0, wg_t0};
  if (p.wgt && tid == 0) ph[0] = __builtin_amdgcn_s_memrealtime();
  // the due broadcasts in key order (LDS copies: every lane reads them per edge)
  if (tid < n_bc) L.bco[tid] = ld_op(&ops[L.bc[tid]]);
  __syncthreads();
  if (tid == 0) {
    for (uint32_t a = 1; a < n_bc; ++a) {
      const Op ox = L.bco[a];
      uint32_t b2 = a;
      while (b2 > 0 && op_key_less(ox, ox.sub, L.bco[b2 - 1], L.bco[b2 - 1].sub)) {
        st_op_lds(&L.bco[b2], L.bco[b2 - 1]);
        --b2;
      }
      st_op_lds(&L.bco[b2], ox);
    }
  }
  __syncthreads();

  // ---- per out-edge: merge broadcasts / reply slots / implicit echo in key order, FIFO, emit ----
  uint32_t n_rec = 0, st_edges = 0, st_echo = 0;
  long long ovmin = LLONG_MAX;
  uint32_t cb = kInvalid, cbn = 0;
  uint32_t cmn = ~0u;
  const long long cs = cell * p.L;
  const uint32_t N1 = p.N - 1;
  const uint32_t L32 = static_cast<uint32_t>(p.L);  // (< 2^32: checked on the host)
  const long long cq_b = cell / B;
  const uint32_t cr_b = static_cast<uint32_t>(cell % B);
  Rec* in_row = p.inbox + inbox_idx(p, ib, rep, e0);
  const int64_t app = p.app_delay;
  const uint32_t f2r = static_cast<uint32_t>(static_cast<uint16_t>(enc_raw(p, 0)));
  const uint32_t w3r = f2r | (kPbPrepareRes << 16);  // a reply slot's (f2, type) word
  const uint32_t bs = blockDim.x;
  // (a node whose broadcasts are not due yet and that has no reply slot or echo to send skips
  // the edges: their link words would be loaded for nothing)
  const uint32_t deg_w = (n_bc || sl0 || sl1 || sd0 || sd1 || rxe) ? deg : 0u;
  const uint32_t ne_w = deg_w ? ne : 0u;  // pending echo descriptors applied by this walk
  if (sd0 || sd1 || ne_w) mesh_desc_load(p, D, g, ob, obp, sd0, sd1, ne_w);
  const bool xr = XR;  // (a template flag: the one-rank kernel carries no staging registers)
  // PF: the link words of all the node's out-edges in flight at once, parked in LDS (dynamic,
  // deg_max words), so that the edge loop of a pure broadcast has no dependent global load --
  // instead of one round trip per kMeshU edges per lane
  extern __shared__ __attribute__((aligned(16))) uint64_t mlw[];
  if (PF) {
    constexpr int kPF = 8;
    const uint64_t* lrow = p.link + edge_loc(p, rep, e0);
    for (uint32_t k0 = 0; k0 < deg_w; k0 += kPF * bs) {
      uint64_t v[kPF];
#pragma unroll
      for (int q = 0; q < kPF; ++q) {
        const uint32_t k = k0 + q * bs + tid;
        v[q] = k < deg_w ? lrow[k] : 0ull;
      }
#pragma unroll
      for (int q = 0; q < kPF; ++q) {
        const uint32_t k = k0 + q * bs + tid;
        if (k < deg_w) mlw[k] = v[q];
      }
    }
    if (ne_w) {  // the pending echo descriptors, oldest first, onto the parked link words
      for (uint32_t le = tid; le < deg_w; le += bs) {
        uint64_t lw = 0;
        int64_t bu = 0;
        bool any = false;
        for (uint32_t d = 0; d < ne_w; ++d)
          if (desc_bit(D.eb[d], le)) {
            if (!any) {
              lw = mlw[le];
              bu = static_cast<int64_t>(lw >> 16);
              any = true;
            }
            bu = (bu > D.et[d] ? bu : D.et[d]) + sel2(p.tx_tot, D.ebig[d] != 0);
          }
        if (any) {
          if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
          mlw[le] = (static_cast<uint64_t>(bu) << 16) | (lw & 0xFFFFull);
        }
      }
    }
    __syncthreads();
  }
  if (p.wgt && tid == 0) ph[1] = __builtin_amdgcn_s_memrealtime();
  // (a wave-uniform trip count: the cross-rank range step after the edges is convergent)
  for (uint32_t b0 = 0; b0 < deg_w; b0 += kMeshU * bs) {
    const uint32_t base = b0 + tid;
    // node-partitioned run: each edge's first record for another rank's receiver waits here,
    // so that a wave can ship a run of them as one range record (xr_ship)
    XRec xp[kMeshU];
    bool hp[kMeshU];
    uint32_t xo[kMeshU];
#pragma unroll
    for (int u = 0; u < kMeshU; ++u) {
      hp[u] = false;
      xo[u] = 0;
    }
    // all loads of the kU edges first (independent addresses), then the per-edge work
    uint64_t lw[kMeshU];
    uint4 r0[kMeshU], w0[kMeshU], w1[kMeshU];
    uint64_t* lwp[kMeshU];
#pragma unroll
    for (int u = 0; u < kMeshU; ++u) {
      const uint32_t le = base + u * bs;
      const bool v = le < deg;
      lwp[u] = p.link + edge_loc(p, rep, e0 + (v ? le : 0u));
      lw[u] = v ? (PF ? mlw[le] : *lwp[u]) : 0ull;
      r0[u] = (v && rxe) ? *reinterpret_cast<const uint4*>(in_row + le) : make_uint4(0, 0, 0, 0);
      w0[u] = (v && sl0) ? *eslot_at(p, ob, rep, e0 + le) : make_uint4(0, 0, 0, 0);
      w1[u] = (v && sl1) ? *eslot_at(p, obp, rep, e0 + le) : make_uint4(0, 0, 0, 0);
    }
    // reply descriptors: the edge's reply as a reply-slot word (in-slots of a reply
    // descriptor and of the cell's reply slots are disjoint: one main record per edge and cell)
    bool hd0[kMeshU], hd1[kMeshU];
#pragma unroll
    for (int u = 0; u < kMeshU; ++u) {
      const uint32_t le = base + u * bs;
      hd0[u] = sd0 && le < deg && desc_bit(D.rb[0], le);
      hd1[u] = sd1 && le < deg && desc_bit(D.rb[1], le);
      if (hd0[u]) w0[u] = make_uint4(rd0.x, rd0.y, rd0.z + desc_rank(D, 0, le), rd0.w);
      if (hd1[u]) w1[u] = make_uint4(rd1.x, rd1.y, rd1.z + desc_rank(D, 1, le), rd1.w);
    }
#pragma unroll
    for (int u = 0; u < kMeshU; ++u) {
      const uint32_t le = base + u * bs;
      if (le >= deg) break;
      const uint32_t e = e0 + le;
      const uint32_t s = le < i ? le : le + 1;  // full mesh: peers ascending without self
      // implicit echo of in-slot le (record {t_off, sub, f0|f1, f2|type|flags})
      bool he = false;
      int64_t et = 0;
      uint32_t edt = 0, esub = 0;
      int ebig = 0;
      if (rxe) {
        const uint32_t fl = r0[u].w >> 24;
        const long long ta0 = cs + r0[u].x;
        if (slot_live(fl, cell_tag(p, cell)) && ta0 >= t_lo && ta0 < t_hi) {
          if (p.echo) {
            ebig = (fl & RF_BIG) ? 1 : 0;
            const int64_t pin = p.prop_const >= 0 ? p.prop_const : AT(p.prop_in, e, p.E);
            et = ta0;
            edt = static_cast<uint32_t>(pin + sel2(p.tx_last, ebig));
            esub = r0[u].y;
            he = true;
            ++st_echo;
          }
        }
      }
      // reply slots {due t lo, hi, sub, f0 | f1 << 16} of this arrival cell and the previous one
      const int64_t rt1 = static_cast<int64_t>((static_cast<uint64_t>(w0[u].y) << 32) | w0[u].x);
      const int64_t rt2 = static_cast<int64_t>((static_cast<uint64_t>(w1[u].y) << 32) | w1[u].x);
      bool hr = (sl0 || hd0[u]) && rt1 >= t_lo && rt1 < t_hi;
      bool hr2 = (sl1 || hd1[u]) && rt2 >= t_lo && rt2 < t_hi;
      st_ops += (hr ? 1u : 0u) + (hr2 ? 1u : 0u);
      // pending echo descriptors on this edge: already on its parked link word (PF prefetch)
      bool pe = false;
      for (uint32_t d = 0; d < ne_w; ++d) pe = pe || desc_bit(D.eb[d], le);
      if (n_bc == 0 && !he && !hr && !hr2 && !pe) continue;
      ++st_edges;
      int64_t bu = static_cast<int64_t>(lw[u] >> 16);
      uint32_t lc = static_cast<uint32_t>(lw[u] & 0xFFFFu);
      const int64_t pr = p.prop_const >= 0 ? p.prop_const : p.prop[e];
      const uint32_t slot = s * N1 + (i < s ? i : i - 1);
      const uint32_t dg = rep * p.N + s;
      uint32_t bi = 0;
      for (;;) {
        while (bi < n_bc && (op_flags(L.bco[bi]) & OPF_PAXOS) && le == 0) ++bi;
        // the earliest source: 1 broadcast, 2 / 4 reply slots, 3 echo
        int src = 0;
        int64_t ot = 0;
        uint32_t odt = 0, oor = 0, osub = 0, ow2 = 0, ow3 = 0;
        int big = 0;
        if (bi < n_bc) {
          const uint4* bw = reinterpret_cast<const uint4*>(&L.bco[bi]);
          const uint4 a = bw[0], b = bw[1];
          ot = static_cast<int64_t>((static_cast<uint64_t>(a.y) << 32) | a.x);
          odt = a.z;
          oor = a.w;
          osub = b.x + (((b.w >> 26) & OPF_PAXOS) ? le - 1 : le);
          ow2 = b.z;
          ow3 = b.w & 0x00FFFFFFu;
          big = ((b.w >> 26) & OPF_BIG) ? 1 : 0;
          src = 1;
        }
        if (hr && (src == 0 || kless(rt1, static_cast<uint32_t>(app), i, w0[u].z, ot, odt, oor, osub))) {
          ot = rt1;
          odt = static_cast<uint32_t>(app);
          oor = i;
          osub = w0[u].z;
          ow2 = w0[u].w;
          ow3 = w3r;
          big = 0;
          src = 2;
        }
        if (hr2 && (src == 0 || kless(rt2, static_cast<uint32_t>(app), i, w1[u].z, ot, odt, oor, osub))) {
          ot = rt2;
          odt = static_cast<uint32_t>(app);
          oor = i;
          osub = w1[u].z;
          ow2 = w1[u].w;
          ow3 = w3r;
          big = 0;
          src = 4;
        }
        if (he && (src == 0 || kless(et, edt, s, esub, ot, odt, oor, osub))) {
          ot = et;
          big = ebig;
          src = 3;
        }
        if (src == 0) break;
        if (src == 1)
          ++bi;
        else if (src == 2)
          hr = false;
        else if (src == 4)
          hr2 = false;
        else
          he = false;
        if (src == 2 || src == 4) ++sends;
        const int64_t start = bu > ot ? bu : ot;
        const int64_t end = start + sel2(p.tx_tot, big);
        bu = end;
        if (src == 3) continue;  // the echo only occupies the link
        const int64_t ta = end + pr;
        // arrival cell and offset: a 32-bit division of the offset from the cell start (a
        // record lands at most a ring or so ahead; 64-bit only beyond 2^32 ns)
        long long ca;
        uint32_t tof;
        {
          const int64_t dtf = ta - cs;
          if (dtf >= 0 && dtf < (1ll << 32)) {
            // floor(x / L) exactly: x * ceil(2^64/L) / 2^64 exceeds x / L by less than x / 2^64
            // < 1/L (x, L < 2^32), which cannot reach the next integer
            const uint32_t x = static_cast<uint32_t>(dtf);
            const uint32_t q = static_cast<uint32_t>(__umul64hi(static_cast<uint64_t>(x), p.L_magic));
            ca = cell + q;
            tof = x - q * L32;
          } else {
            ca = ta / p.L;
            tof = static_cast<uint32_t>(ta - ca * p.L);
          }
        }
        const long long rel = ca - cell;
        if (rel < 1) {
          set_err(p, BCSIM_E_TIE);  // lookahead violated
          continue;
        }
        ++n_rec;
        const uint32_t w3 = ow3 | (static_cast<uint32_t>(RF_VALID | (big ? RF_BIG : 0)) << 24) |
            (emit_tag(cq_b, cr_b, rel, B) << 27);
        Rec r;
        {
          const uint4 rv = make_uint4(tof, osub, ow2, w3);
          __builtin_memcpy(&r, &rv, sizeof r);
        }
        const bool owner = lc != (static_cast<uint32_t>(ca) & 0xFFFFu);
        lc = static_cast<uint32_t>(ca) & 0xFFFFu;
        if (xr) {
          const uint32_t orank = p.owner[s];
          if (orank != p.rank) {  // receiver on another GPU: shipped, k_import places it
            XRec x;
            x.r = r;
            if (owner) x.r.flags = static_cast<uint8_t>(x.r.flags | RF_OWNER);
            x.cell = ca;
            x.slot = slot;
            x.g = dg;
            if (!hp[u]) {
              xp[u] = x;
              hp[u] = true;
              xo[u] = orank;
            } else {
              link_stage(p, L, g, B + 1 + orank, x);
            }
            continue;
          }
        }
        if (rel < static_cast<long long>(B)) {
          uint32_t bk = cr_b + static_cast<uint32_t>(rel);  // (ca % B, rel < B)
          if (bk >= B) bk -= B;
          if (owner) {
            st_rec(&AT(p.inbox, inbox_idx(p, bk, rep, slot), p.cap_inbox), r);
            xs_mark(p, bk, rep, i, s, w3);
            uint32_t tb = kInvalid;
            if (tmap) {  // the first bucket seen owns the LDS tile map; others flag directly
              tb = L.tbk;
              if (tb == kInvalid) {
                const uint32_t old = atomicCAS(&L.tbk, kInvalid, bk);
                tb = old == kInvalid ? bk : old;
              }
            }
            if (tb == bk)
              L.tflag[s >> 6] = 1;
            else
              set_flag_once(&AT(p.rtile, kRtPad * ((static_cast<size_t>(bk) * p.R + rep) * p.n_tiles + (s >> 6)), kRtPad * (static_cast<uint64_t>(B) * p.R * p.n_tiles)));
          } else {
            XRec x;
            x.r = r;
            x.cell = ca;
            x.slot = slot;
            x.g = dg;
            link_stage(p, L, g, bk, x);
            AT(p.iflag, static_cast<size_t>(bk) * p.NT + dg, static_cast<uint64_t>(B) * p.NT) = 1;
          }
          if (bk != cb) {
            if (cbn) {
              atomicAdd(&L.lcnt[cb], cbn);
              atomicMin(&L.lmin[cb], cmn);
            }
            cb = bk;
            cbn = 0;
            cmn = ~0u;
          }
          ++cbn;
          if (tof < cmn) cmn = tof;
        } else {
          XRec x;
          x.r = r;
          if (owner) x.r.flags = static_cast<uint8_t>(x.r.flags | RF_OWNER);
          x.cell = ca;
          x.slot = slot;
          x.g = dg;
          link_stage(p, L, g, B, x);
          if (ca < ovmin) ovmin = ca;
        }
      }
      if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
      *lwp[u] = (static_cast<uint64_t>(bu) << 16) | lc;
    }
    if (xr) {
#pragma unroll
      for (int u = 0; u < kMeshU; ++u) xr_ship(p, L, g, i, base + u * bs, hp[u], xp[u], xo[u]);
    }
  }
  if (cbn) {
    atomicAdd(&L.lcnt[cb], cbn);
    atomicMin(&L.lmin[cb], cmn);
  }
  __syncthreads();
  if (p.wgt && tid == 0) ph[2] = __builtin_amdgcn_s_memrealtime();
  if (tmap && L.tbk != kInvalid) {  // flush the receiver-tile flags of this sender's records
    const size_t tb = (static_cast<size_t>(L.tbk) * p.R + rep) * p.n_tiles;
    for (uint32_t k = tid; k < p.n_tiles; k += blockDim.x)
      if (L.tflag[k]) set_flag_once(&AT(p.rtile, kRtPad * (tb + k), kRtPad * (static_cast<uint64_t>(B) * p.R * p.n_tiles)));
  }
  if (tid == 0) {
    if (ne_w) AT(p.en, g, p.NT) = 0;  // every edge walked: the echo descriptors are applied
    // a reply descriptor is sent whole (one due instant): its flag goes (a stale flag would keep
    // k_scan_pbft from taking the echoes of a later window)
    const size_t R4 = static_cast<uint64_t>(kOpRing) * p.NT;
    if (sd0) AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, R4) = static_cast<uint8_t>(sf0 & ~kSfD0);
    if (sd1) AT(p.sflag, static_cast<size_t>(obp) * p.NT + g, R4) = static_cast<uint8_t>(sf1 & ~kSfD1);
  }
  const unsigned long long t0 = p.wgt ? wg_t0 : 0ull;
  const LinkCounts c8{dropped, sends, n_rec, st_ops, st_edges, st_echo, 0u, 0u};
  // every op due (the broadcasts just sent): nothing to compact, no op to read again
  link_finish(p, L, g, ops, n_bc == n ? 0u : n, t_hi, n_lists, ovmin, c8, (sl1 || sd1) && final_win, rx && final_win, obp,
              fidx, t0, ph, n);
}

// ---------------------------------------------------------------------------
// The tiled full-mesh link stage (one rank, fixed app delay, infinite queues):
//   k_mesh_prep   one wave per active node: classify its due ops (pbft-node.cc:349-368
//                 broadcasts, the reply descriptors of k_scan_pbft, :212-222), leave a job for the
//                 tiles -- the due broadcasts in key order, flags, descriptor times and the
//                 descriptor bitmaps cut into 64-receiver tiles -- and do the node's own bookkeeping
//                 (op compaction, counters, slot / descriptor flags); a node whose due ops are not
//                 all broadcasts (or more than kMeshBc) goes to list 3 (generic kernel)
//   k_mesh_tile   32 senders x 64 receivers per workgroup: the per-edge FIFO and records
//   k_link<.., LOOP> over list 3 (descriptors flushed first: node_desc_flush)
// Same results as k_link_mesh's edge walk.

// bits [a, a + 64) of a descriptor bitmap held in LDS (words >= dw read as 0)
__device__ inline uint64_t bits64(const uint32_t* w, uint32_t dw, uint32_t a) {
  const uint32_t q = a >> 5, r = a & 31u;
  const uint64_t w0 = q < dw ? w[q] : 0u, w1 = q + 1 < dw ? w[q + 1] : 0u, w2 = q + 2 < dw ? w[q + 2] : 0u;
  const uint64_t lo = w0 | (w1 << 32);
  return r ? (lo >> r) | (w2 << (64 - r)) : lo;
}
// the bitmap of sender i's out-edges cut to receiver tile s0 .. s0 + 63: bit k = out-edge to
// receiver s0 + k (the full mesh's out-edge index le = s - (s > i), no bit for s == i or s >= N)
__device__ inline uint64_t tile_mask(const uint32_t* w, uint32_t dw, uint32_t i, uint32_t s0, uint32_t N) {
  uint64_t m;
  if (i < s0) {
    m = bits64(w, dw, s0 - 1);
  } else if (i >= s0 + 64) {
    m = bits64(w, dw, s0);
  } else {
    const uint32_t j = i - s0;
    const uint64_t A = bits64(w, dw, s0);
    const uint64_t below = j ? (~0ull >> (64 - j)) : 0ull;  // bits < j
    m = (A & below) | ((A << 1) & ~below & ~(1ull << j));
  }
  const uint32_t nv = N - s0;  // receivers of the tile that exist
  return nv >= 64 ? m : (m & ((1ull << nv) - 1ull));
}

// the heavy waves' job shape (uniform over the sender's edges): one kind of source per edge -- the
// one due broadcast, or the one due reply descriptor -- no echo from the row, no reply slot, and a
// constant propagation delay (k_mesh_tile's fast lanes; in summary mode k_mesh_row takes them)
__device__ inline bool job_uniform(uint32_t fl, uint32_t jz, int64_t prc) {
  const uint32_t n_bc = (jz >> 8) & 0xFFu;
  const bool sd0 = fl & kJSd0, sd1 = fl & kJSd1;
  return !(fl & (kJRxe | kJSl0 | kJSl1)) && prc >= 0 && ((n_bc == 1 && !sd0 && !sd1) || (n_bc == 0 && sd0 != sd1));
}

__global__ __launch_bounds__(64) void k_mesh_prep(const KP* __restrict__ pk, long long cell, long long t_lo, long long t_hi,
                                                  int final_win, uint32_t epoch, uint32_t wep) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ LinkShared L;
  __shared__ MeshDesc D;
  uint32_t kk;
  if (!list_one(p.act_n[1], kk)) return;
  const uint32_t g = p.act[p.NT + kk];
  if (wep && AT(p.l2mark, g, p.NT) == wep) return;  // left to the generic kernels (second stream)
  const uint32_t tid = tidx();
  const uint32_t n = AT(p.n_ops, g, p.NT);
  const uint32_t ob = static_cast<uint32_t>(cell % kOpRing), obp = static_cast<uint32_t>((cell + kOpRing - 1) % kOpRing);
  const size_t R4 = static_cast<uint64_t>(kOpRing) * p.NT;
  const uint32_t sf0 = AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, R4);
  const uint32_t sf1 = AT(p.sflag, static_cast<size_t>(obp) * p.NT + g, R4);
  const bool sl0 = sf0 & 1u, sl1 = sf1 & 2u;
  const bool dsc = p.desc != 0;
  uint4 rd0 = make_uint4(0, 0, 0, 0), rd1 = make_uint4(0, 0, 0, 0);
  if (dsc && (sf0 & kSfD)) rd0 = p.rdesc[static_cast<size_t>(ob) * p.NT + g];
  if (dsc && (sf1 & kSfD1)) rd1 = p.rdesc[static_cast<size_t>(obp) * p.NT + g];
  const bool dl0 = dsc && (sf0 & kSfD) && desc_due(rd0) >= t_lo;
  const bool dl1 = dsc && (sf1 & kSfD1) && desc_due(rd1) >= t_lo;
  const bool sd0 = dl0 && desc_due(rd0) < t_hi, sd1 = dl1 && desc_due(rd1) < t_hi;
  const uint32_t ne = dsc ? AT(p.en, g, p.NT) : 0u;
  const uint32_t B = p.n_buckets;
  const uint32_t ib = static_cast<uint32_t>(cell % B);
  const size_t fidx = static_cast<size_t>(ib) * p.NT + g;
  const uint32_t rep = g / p.N, i = g % p.N;
  const bool rx = p.impl && node_flagged_w(p, ib, g, rep, i, t_hi);
  const bool rxe = rx && AT(p.eapp, g, p.NT) != t_lo;
  if ((n == 0 || AT(p.node_onext, g, p.NT) >= t_hi) && !sl0 && !sl1 && !sd0 && !sd1 && !rxe) {
    if (rx && final_win && tid == 0) AT(p.iflag, fidx, static_cast<uint64_t>(B) * p.NT) = 0;
    return;
  }
  for (uint32_t k = tid; k < B; k += blockDim.x) {
    L.lcnt[k] = 0;
    L.lmin[k] = ~0u;
  }
  const uint32_t n_lists = B + 1;
  for (uint32_t k = tid; k < n_lists; k += blockDim.x) L.lst[k] = 0;
  if (tid < 8) L.csum[tid] = 0;
  if (tid == 0) {
    L.n_bc = 0;
    L.n_list = 0;
    L.nst = 0;
    L.omin = LLONG_MAX;
    L.ovmin = LLONG_MAX;
  }
  __syncthreads();
  const uint32_t deg = AT(p.row, i + 1, p.N + 1) - AT(p.row, i, p.N + 1);
  Op* ops = p.ops + op_base(p, g);
  uint32_t sends = 0, st_ops = 0, other = 0;
  for (uint32_t k = tid; k < n; k += blockDim.x) {
    const RawOp o = ld_raw(&ops[k]);
    const uint32_t kind = raw_kind(o);
    if (kind == OP_BCAST_J) {
      other += (raw_flags(o) & OPF_DONE) ? 0u : 1u;
      continue;
    }
    if (raw_t(o) >= t_hi) continue;
    if (kind != OP_BCAST || (raw_flags(o) & OPF_PAXOS)) {  // (Paxos broadcasts: k_link_mesh / generic)
      ++other;
      continue;
    }
    ++st_ops;
    const uint32_t pos = atomicAdd(&L.n_bc, 1u);
    if (pos < kBcastCap) L.bc[pos] = k;
    sends += deg;
  }
  {
    const uint32_t ws = wave_sum(other);
    if (tid == 0 && ws) L.n_list = ws;
  }
  __syncthreads();
  const uint32_t n_bc = L.n_bc;
  // (summary mode: k_mesh_row takes the uniform jobs and the generic kernel every other -- no
  // tile launch)
  const uint32_t flu = (sl0 ? kJSl0 : 0u) | (sl1 ? kJSl1 : 0u) | (sd0 ? kJSd0 : 0u) | (sd1 ? kJSd1 : 0u) | (rxe ? kJRxe : 0u);
  if (L.n_list || n_bc > kMeshBc || (p.sum && !job_uniform(flu, n_bc << 8, p.prop_const))) {
    // the generic kernel takes the node (node_desc_flush first)
    if (tid == 0 && p.fdbg)
      FDBG(L.n_list ? 10 : n_bc > kMeshBc ? 11 : rxe ? 12 : (sl0 || sl1) ? 13 : (sd0 && sd1) ? 14 : 15);
    if (tid == 0) {
      const uint32_t pos = gadd_r(&p.act_n[3], 1u);
      AT(p.act, 3ull * p.NT + pos, 4ull * p.NT) = g;
    }
    return;
  }
  // the due broadcasts in key order (<= 2), as RawOp words
  const size_t jb = static_cast<size_t>(g) * kMeshBc * 2;
  if (tid < 2 * n_bc) {
    uint32_t k = tid >> 1;
    if (n_bc == 2) {
      const RawOp a = ld_raw(&ops[L.bc[0]]), b = ld_raw(&ops[L.bc[1]]);
      const bool swap = raw_key_less(b, raw_sub(b), a, raw_sub(a));
      k = swap ? 1u - k : k;
    }
    p.mbc[jb + tid] = reinterpret_cast<const uint4*>(&ops[L.bc[k]])[tid & 1u];
  }
  // descriptor bitmaps cut to receiver tiles (lane = tile)
  const uint32_t ne_j = ne;  // (every edge is walked: any pending echo descriptor is applied)
  if (sd0 || sd1 || ne_j) {
    mesh_desc_load(p, D, g, ob, obp, sd0, sd1, ne_j);
    const uint32_t dw = p.dwords, nt = p.n_tiles;
    for (uint32_t rt = tid; rt < nt; rt += blockDim.x) {
      const uint32_t s0 = rt * kTR;
      const uint32_t le0 = s0 > i ? s0 - 1 : s0;  // out-edge index of the tile's first receiver
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (!(h ? sd1 : sd0)) continue;
        const uint64_t m = tile_mask(D.rb[h], dw, i, s0, p.N);
        const uint32_t base = le0 < deg ? desc_rank(D, h, le0) : 0u;
        p.mtb[(static_cast<size_t>(g) * nt + rt) * 2 + h] =
            make_uint4(static_cast<uint32_t>(m), static_cast<uint32_t>(m >> 32), base, 0u);
      }
      for (uint32_t d = 0; d < ne_j; ++d) {
        const uint64_t m = tile_mask(D.eb[d], dw, i, s0, p.N);
        p.mte[(static_cast<size_t>(g) * nt + rt) * kEDesc + d] = make_uint2(static_cast<uint32_t>(m), static_cast<uint32_t>(m >> 32));
      }
    }
  }
  if (tid == 0) {
    uint32_t fl = (sl0 ? kJSl0 : 0u) | (sl1 ? kJSl1 : 0u) | (sd0 ? kJSd0 : 0u) | (sd1 ? kJSd1 : 0u) | (rxe ? kJRxe : 0u);
    uint4 q3 = make_uint4(0, 0, 0, 0);
    if (ne_j) {
      const uint4 ed0 = p.edesc[static_cast<size_t>(g) * kEDesc];
      q3.x = ed0.x;
      q3.y = ed0.y;
      if (ed0.z) fl |= kJBig0;
      if (ne_j > 1) {
        const uint4 ed1 = p.edesc[static_cast<size_t>(g) * kEDesc + 1];
        q3.z = ed1.x;
        q3.w = ed1.y;
        if (ed1.z) fl |= kJBig1;
      }
    }
    uint4* J = p.mjob + static_cast<size_t>(g) * 4;
    J[1] = rd0;
    J[2] = rd1;
    J[3] = q3;
    J[0] = make_uint4(epoch, fl, ne_j | (n_bc << 8), 0u);
    if (!(p.sum && job_uniform(fl, ne_j | (n_bc << 8), p.prop_const)))  // (summary mode: k_mesh_row's)
      p.mtile[static_cast<size_t>(rep) * p.n_stiles + i / kTS] = epoch;
    if (ne_j) AT(p.en, g, p.NT) = 0;
    // a due reply descriptor is sent whole: its flag goes (as in k_link_mesh)
    if (sd0) AT(p.sflag, static_cast<size_t>(ob) * p.NT + g, R4) = static_cast<uint8_t>(sf0 & ~kSfD0);
    if (sd1) AT(p.sflag, static_cast<size_t>(obp) * p.NT + g, R4) = static_cast<uint8_t>(sf1 & ~kSfD1);
  }
  unsigned long long ph[4] = {0, 0, 0, 0};
  const LinkCounts c8{0u, sends, 0u, st_ops, 0u, 0u, 0u, 0u};
  link_finish(p, L, g, ops, n_bc == n ? 0u : n, t_hi, n_lists, LLONG_MAX, c8, (sl1 || sd1) && final_win, rx && final_win,
              obp, fidx, 0ull, ph, n);
}

// k_mesh_tile: the edges of the jobs k_mesh_prep left, for a tile of 32 senders x 64 receivers
// per workgroup.  The same per-edge work as k_link_mesh's edge loop (the pending echo
// descriptors onto the link word, then the due broadcasts, reply slots / descriptors and the
// implicit echo merged in key order through the FIFO, pbft-node.cc:349-368 fan-out, :175
// echo), but the memory side is coalesced both ways: a wave walks one sender's out-edges to the
// tile's 64 receivers (link words, own inbox row and reply slots are 64 consecutive words of
// the sender's row; the link words of all of a wave's senders are loaded at once, parked in
// the record area), and the records are transposed in LDS and written receiver by receiver --
// 32 consecutive in-slots (512 B) of each receiver's row instead of 16-byte stores 64 KB apart.
// A second slot record of an edge is stored directly; extras / overflow records are staged in
// LDS and appended with one atomic per list (the leader's block broadcast: 64 per tile).
constexpr uint32_t kTX = 64;  // staged extras / overflow records per tile
struct TileShared {
  uint4 rec[kTR * kTS];     // link words (.x, .y), then slot records; receiver-major, sender swizzled (tsw)
  uint8_t rbk[kTR * kTS];   // the record's bucket (0xFF: none)
  uint4 job[kTS][4];
  uint4 bc[kTS][kMeshBc * 2];
  uint4 mtb[kTS][2];        // reply descriptor tile masks {lo, hi, rank base}
  uint2 mte[kTS][kEDesc];   // pending echo descriptor tile masks
  XRec xs[kTX];
  uint32_t xm[kTX];         // list << 24 | rank
  uint32_t xn;
  uint32_t lst[kMaxBuckets + 1];
  uint32_t lcnt[kMaxBuckets];
  uint32_t lmin[kMaxBuckets];
  uint32_t csum[8];
  unsigned long long bkm;   // buckets holding slot records of this tile
  long long ovmin;
  long long bmin[kMaxBuckets];  // the buckets' arrival-time bounds as of the start (read early)
  uint64_t lwo[BCSIM_TILE_DEFER ? kTS : 1][kTR];  // updated link words (0: unchanged), written out after the walk
  uint4 sold[kTS][2][2];    // (summaries) the senders' entries of the buckets sbk[0 / 1] as of the start
  uint32_t sbk[2];
};
// (receiver, sender) -> LDS index: the sender index XOR the receiver's low bits, so that a wave
// writing one sender's 64 receivers and a wave reading two receivers' 32 senders both spread
// over the banks
__device__ inline uint32_t tsw(uint32_t s, uint32_t i) { return s * kTS + (i ^ (s & (kTS - 1u))); }

__device__ inline void tile_append(const KP& p, TileShared& T, uint32_t list, const XRec& x) {
  const uint32_t pos = atomicAdd(&T.xn, 1u);
  if (pos < kTX) {
    const uint32_t rank = atomicAdd(&T.lst[list], 1u);
    T.xs[pos] = x;
    T.xm[pos] = (list << 24) | rank;
    return;
  }
  // (staging full: a direct, contended append)
  uint32_t* ctr = list == p.n_buckets ? p.ov_cnt : &p.x_cnt[list];
  const uint32_t cap = list == p.n_buckets ? p.cap_ov : p.cap_x;
  const uint32_t at = gadd_r(ctr, 1u);
  if (at >= cap) {
    set_err(p, BCSIM_E_OVERFLOW);
    return;
  }
  uint4* dst = reinterpret_cast<uint4*>(list == p.n_buckets ? p.ov + at : p.xbuf + static_cast<size_t>(list) * p.cap_x + at);
  const uint4* src = reinterpret_cast<const uint4*>(&x);
  gst4(dst, src[0]);
  gst4(dst + 1, src[1]);
}

__global__ __launch_bounds__(kTileThreads) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_mesh_tile(const KP* __restrict__ pk, long long cell, long long t_lo, long long t_hi,
                                                   uint32_t epoch) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ TileShared T;
  const uint32_t nrt = p.n_tiles, nst = p.n_stiles;
  const uint32_t rep = blockIdx.x / (nst * nrt), rem = blockIdx.x % (nst * nrt);
  const uint32_t st = BCSIM_TILE_RTMAJOR ? rem % nst : rem / nrt, rt = BCSIM_TILE_RTMAJOR ? rem / nst : rem % nrt;
  if (gbl(p.mtile)[static_cast<size_t>(rep) * nst + st] != epoch) return;  // no job among these senders
  const uint32_t tid = tidx(), lane = tid & 63u, wv = tid >> 6, nwv = blockDim.x >> 6;
  G<unsigned long long>* tph = p.wgtt ? gbl(p.wgtt) + 8ull * blockIdx.x : nullptr;  // (debug phase clocks)
#define TPH(k)                                                       \
  do {                                                               \
    if (tph && tid == 0) tph[(k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  TPH(0);
  const uint32_t N = p.N, N1 = N - 1, B = p.n_buckets;
  const uint32_t i0 = st * kTS, s0 = rt * kTR;
  const size_t gb = static_cast<size_t>(rep) * N + i0;  // gnode of the tile's first sender
  const uint32_t s = s0 + lane;
  // the link words of every edge of this wave's senders first (whether or not the sender has a
  // job: the loads need not wait for the job words), all in flight with the job loads below
  uint64_t lv[4];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t il = wv + k * nwv;
    const uint32_t i = i0 + il;
    const bool v = il < kTS && i < N && s < N && s != i;
    lv[k] = v ? gbl(p.link)[edge_loc(p, rep, i * N1 + (s < i ? s : s - 1))] : 0ull;
  }
  // the buckets' arrival-time bounds with them (a second round trip for wave 0 otherwise)
  const long long bm_v = tid < B ? *reinterpret_cast<volatile G<long long>*>(&gbl(p.bmin)[tid]) : LLONG_MAX;
  // jobs, broadcasts and descriptor tile masks of the 32 senders, all loads at once (a stale job
  // is told by its epoch; the other words are used only under its flags)
  if (tid < kTS * 4) {
    const uint32_t il = tid >> 2;
    T.job[il][tid & 3u] = i0 + il < N ? gld4(p.mjob + (gb + il) * 4 + (tid & 3u)) : make_uint4(0, 0, 0, 0);
  } else if (tid < kTS * 4 + kTS * kMeshBc * 2) {
    const uint32_t k = tid - kTS * 4, il = k / (kMeshBc * 2);
    if (i0 + il < N) T.bc[il][k % (kMeshBc * 2)] = gld4(p.mbc + (gb + il) * kMeshBc * 2 + k % (kMeshBc * 2));
  } else if (tid < kTS * 4 + kTS * kMeshBc * 2 + kTS * 2) {
    const uint32_t k = tid - kTS * 4 - kTS * kMeshBc * 2, il = k >> 1;
    if (i0 + il < N) T.mtb[il][k & 1u] = gld4(p.mtb + ((gb + il) * nrt + rt) * 2 + (k & 1u));
  } else if (tid < kTS * 4 + kTS * kMeshBc * 2 + kTS * 2 + kTS * kEDesc) {
    const uint32_t k = tid - kTS * 4 - kTS * kMeshBc * 2 - kTS * 2, il = k / kEDesc;
    if (i0 + il < N) {
      const uint64_t m = gbl(reinterpret_cast<uint64_t*>(p.mte))[((gb + il) * nrt + rt) * kEDesc + k % kEDesc];
      T.mte[il][k % kEDesc] = make_uint2(static_cast<uint32_t>(m), static_cast<uint32_t>(m >> 32));
    }
  } else if (p.sum && tid < kTS * 4 + kTS * kMeshBc * 2 + kTS * 2 + kTS * kEDesc + kTS * 4) {
    // (summaries) the senders' entries of the (at most two) buckets a small message sent in this
    // window lands in on an idle link -- the heavy waves' jobs -- for the walk's merge check
    const uint32_t k = tid - (kTS * 4 + kTS * kMeshBc * 2 + kTS * 2 + kTS * kEDesc), il = k >> 2, h = (k >> 1) & 1u;
    const long long ca = ((h ? t_hi - 1 : t_lo) + p.tx_tot[0] + p.prop_const) / p.L;
    const bool in = p.prop_const >= 0 && ca - cell >= 1 && ca - cell < static_cast<long long>(B);
    const uint32_t bk = static_cast<uint32_t>(ca % B);
    T.sold[il][h][k & 1u] = in && i0 + il < N ? gld4(p.msum + sum_idx(p, bk, rep, rt, i0 + il) * 2 + (k & 1u)) : make_uint4(0, 0, 0, 0);
    if (il == 0 && (k & 1u) == 0) T.sbk[h] = in && (h == 0 || ca != ((t_lo + p.tx_tot[0] + p.prop_const) / p.L)) ? bk : kInvalid;
  }
  for (uint32_t k = tid; k < kTR * kTS / 4; k += blockDim.x) reinterpret_cast<uint32_t*>(T.rbk)[k] = 0xFFFFFFFFu;
  if (BCSIM_TILE_DEFER)
    for (uint32_t k = tid; k < kTR * kTS; k += blockDim.x) (&T.lwo[0][0])[k] = 0ull;
  for (uint32_t k = tid; k < B; k += blockDim.x) {
    T.lcnt[k] = 0;
    T.lmin[k] = ~0u;
  }
  for (uint32_t k = tid; k <= B; k += blockDim.x) T.lst[k] = 0;
  if (tid < B) T.bmin[tid] = bm_v;  // (B <= kMaxBuckets <= blockDim.x)
  if (tid < 8) T.csum[tid] = 0;
  if (tid == 0) {
    T.bkm = 0ull;
    T.ovmin = LLONG_MAX;
    T.xn = 0;
  }
  TPH(1);
  // the link words parked in the edges' record slots (each lane reads back only its own)
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t il = wv + k * nwv;
    if (il < kTS) {
      T.rec[tsw(lane, il)].x = static_cast<uint32_t>(lv[k]);
      T.rec[tsw(lane, il)].y = static_cast<uint32_t>(lv[k] >> 32);
    }
  }
  __syncthreads();
  TPH(2);
  const uint32_t ib = static_cast<uint32_t>(cell % B);
  const uint32_t ob = static_cast<uint32_t>(cell % kOpRing), obp = static_cast<uint32_t>((cell + kOpRing - 1) % kOpRing);
  const long long cs = cell * p.L;
  const uint32_t L32 = static_cast<uint32_t>(p.L);
  const long long cq_b = cell / B;
  const uint32_t cr_b = static_cast<uint32_t>(cell % B);
  const uint32_t tag = cell_tag(p, cell);
  const int64_t app = p.app_delay;
  const uint32_t w3r = static_cast<uint32_t>(static_cast<uint16_t>(enc_raw(p, 0))) | (kPbPrepareRes << 16);
  const unsigned long long lbit = 1ull << lane, lbelow = lbit - 1ull;
  // (the fast path's parameters, read once)
  // (scalar registers: indexed by a lane's flag, a KP array is a vector load per use)
  const int64_t tx0 = p.tx_tot[0], tx1 = p.tx_tot[1], txl0 = p.tx_last[0], txl1 = p.tx_last[1], prc = p.prop_const;
  const uint64_t Lmag = p.L_magic;
  uint32_t n_rec = 0, st_edges = 0, st_echo = 0, st_ops = 0, sends = 0;
  unsigned long long bkm = 0ull;
  long long ovmin = LLONG_MAX;
  uint32_t cb = kInvalid, cbn = 0, cmn = ~0u;
  const bool sum_on = p.sum != 0;
#pragma unroll 1
  for (uint32_t il = wv; il < kTS; il += nwv) {
    // the sender's job words are uniform: scalar registers, scalar branches
    if (static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(T.job[il][0].x))) != epoch) continue;
    const uint32_t fl = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(T.job[il][0].y)));
    const uint32_t jz = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(T.job[il][0].z)));
    if (sum_on && job_uniform(fl, jz, prc)) continue;  // (summary mode: k_mesh_row's)
    const uint32_t i = i0 + il;
    const uint32_t ne = jz & 0xFFu, n_bc = (jz >> 8) & 0xFFu;
    const bool sl0 = fl & kJSl0, sl1 = fl & kJSl1, sd0 = fl & kJSd0, sd1 = fl & kJSd1, rxe = fl & kJRxe;
    const bool v = s < N && s != i;
    const uint32_t le = s < i ? s : s - 1;
    const uint32_t e = i * N1 + (v ? le : 0u);
    const uint32_t q = tsw(lane, il);
    const uint64_t lw0 = (static_cast<uint64_t>(T.rec[q].y) << 32) | T.rec[q].x;
    // ---- the heavy waves' shape (uniform): one kind of source per edge -- the one due broadcast,
    // or the one due reply descriptor -- and a constant propagation delay.  A lane whose record is
    // the edge's first slot record of a cell 1 .. B-1 ahead is finished here; any other lane goes
    // to the general merge below with nothing changed.
    if (!rxe && !sl0 && !sl1 && prc >= 0 && ((n_bc == 1 && !sd0 && !sd1) || (n_bc == 0 && sd0 != sd1))) {
      // the source's uniform words: due time, the first edge's sub, payload words, frame size
      uint32_t u_tlo, u_thi, u_sub, u_w2, u_w3;
      bool has;
      if (n_bc) {
        u_tlo = T.bc[il][0].x;
        u_thi = T.bc[il][0].y;
        u_sub = T.bc[il][1].x;
        u_w2 = T.bc[il][1].z;
        u_w3 = T.bc[il][1].w;
        has = v;
      } else {
        const int h = sd0 ? 0 : 1;
        const uint4 mb = T.mtb[il][h];
        const unsigned long long m = (static_cast<unsigned long long>(mb.y) << 32) | mb.x;
        has = v && (m & lbit);
        u_tlo = T.job[il][1 + h].x;
        u_thi = T.job[il][1 + h].y;
        u_sub = T.job[il][1 + h].z + mb.z + static_cast<uint32_t>(__popcll(m & lbelow)) - le;  // (+ le below)
        u_w2 = T.job[il][1 + h].w;
        u_w3 = w3r;
      }
      u_tlo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(u_tlo)));
      u_thi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(u_thi)));
      u_w2 = n_bc ? static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(u_w2))) : u_w2;
      u_w3 = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(u_w3)));
      const int big = (n_bc && ((u_w3 >> 26) & OPF_BIG)) ? 1 : 0;
      const int64_t ot = static_cast<int64_t>((static_cast<uint64_t>(u_thi) << 32) | u_tlo);
      const int64_t txu = big ? tx1 : tx0;
      const uint32_t w3u = (u_w3 & 0x00FFFFFFu) | (static_cast<uint32_t>(RF_VALID | (big ? RF_BIG : 0)) << 24);
      int64_t bu = static_cast<int64_t>(lw0 >> 16);
      bool pe = false;
      for (uint32_t d = 0; d < ne; ++d) {  // pending echo descriptors, oldest first
        const uint2 em = T.mte[il][d];
        const unsigned long long m = (static_cast<unsigned long long>(em.y) << 32) | em.x;
        const uint4 q3 = T.job[il][3];
        const int64_t et = static_cast<int64_t>(d ? ((static_cast<uint64_t>(q3.w) << 32) | q3.z)
                                                  : ((static_cast<uint64_t>(q3.y) << 32) | q3.x));
        const int64_t eb = (bu > et ? bu : et) + ((fl & (d ? kJBig1 : kJBig0)) ? tx1 : tx0);
        const bool hit = v && (m & lbit);
        bu = hit ? eb : bu;
        pe = pe || hit;
      }
      const int64_t start = bu > ot ? bu : ot;
      const int64_t end = start + txu;
      const int64_t dtf = end + prc - cs;
      const uint32_t x = static_cast<uint32_t>(dtf);
      const uint32_t qq = static_cast<uint32_t>(__umul64hi(static_cast<uint64_t>(x), Lmag));
      const uint32_t lc0 = static_cast<uint32_t>(lw0 & 0xFFFFu);
      const uint32_t ca16 = static_cast<uint32_t>(cell + qq) & 0xFFFFu;
      const uint32_t bq = cr_b + qq;
      const bool wrap = bq >= B;
      const bool ok = has && (static_cast<uint64_t>(dtf) >> 32) == 0 && qq - 1u < B - 1u && lc0 != ca16;
      const uint32_t lc = ok ? ca16 : lc0;
      const uint32_t bk = wrap ? bq - B : bq;
      const uint32_t tof = x - qq * L32;
      const uint32_t w3f = w3u | (static_cast<uint32_t>((cq_b + (wrap ? 1 : 0)) & 31) << 27);
      // (summaries) the lanes whose record has the first such lane's bucket, offset
      // and base (sub - out-edge index) become ONE entry of (bucket, receiver tile, this sender),
      // merged with the entry an earlier launch left for the same turn when its words are the
      // same (else they go out as records, below)
      bool uni = false;
      if (sum_on) {
        const unsigned long long okm = __ballot(ok);
        if (okm) {
          const int rl = __ffsll(static_cast<long long>(okm)) - 1;
          const uint32_t r_tof = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(tof), rl));
          const uint32_t r_base = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(u_sub), rl));
          const uint32_t r_bk = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(bk), rl));
          const uint32_t r_w2 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(u_w2), rl));
          const uint32_t r_w3 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(w3f), rl));
          uni = ok && tof == r_tof && u_sub == r_base && bk == r_bk;
          unsigned long long um = __ballot(uni);
          uint4 oa, ob;
          uint4* const se = p.msum + sum_idx(p, r_bk, rep, rt, i) * 2;
          if (r_bk == T.sbk[0] || r_bk == T.sbk[1]) {  // (prefetched in the prologue)
            const uint32_t h = r_bk == T.sbk[0] ? 0u : 1u;
            oa = T.sold[il][h][0];
            ob = T.sold[il][h][1];
          } else {
            oa = gld4(se);
            ob = gld4(se + 1);
          }
          const bool olive = (oa.x | oa.y) != 0u && slot_live(ob.y >> 24, r_w3 >> 27);
          if (olive && (oa.z != r_tof || oa.w != r_base || ob.x != r_w2 || ob.y != r_w3)) um = 0ull;
          if (um) {
            const unsigned long long mm = um | (olive ? ((static_cast<unsigned long long>(oa.y) << 32) | oa.x) : 0ull);
            if (lane < 2u)
              gst4(se + lane,
                   lane ? make_uint4(r_w2, r_w3, 0u, 0u)
                        : make_uint4(static_cast<uint32_t>(mm), static_cast<uint32_t>(mm >> 32), r_tof, r_base));
          }
          uni = (um >> lane) & 1ull;
        }
      }
      if (ok) {
        if (!uni) {
          T.rec[q] = make_uint4(tof, u_sub + le, u_w2, w3f);
          T.rbk[q] = static_cast<uint8_t>(bk);
        }
        bkm |= 1ull << bk;
        ++n_rec;
        if (!n_bc) {
          ++sends;
          ++st_ops;
        }
        const bool nb = bk != cb;
        if (nb && cbn) {
          atomicAdd(&T.lcnt[cb], cbn);
          atomicMin(&T.lmin[cb], cmn);
        }
        cbn = nb ? 1u : cbn + 1u;
        cmn = nb ? tof : (tof < cmn ? tof : cmn);
        cb = bk;
      }
      const bool done = ok || !has;
      if (done && (ok || pe)) {
        ++st_edges;
        const uint64_t nw = (static_cast<uint64_t>(ok ? end : bu) << 16) | lc;
        if (BCSIM_TILE_DEFER)
          T.lwo[BCSIM_TILE_DEFER ? il : 0][lane] = nw;
        else
          gbl(p.link)[edge_loc(p, rep, e)] = nw;
      }
      if (done) continue;
    }
    // ---- the general merge ----
    // (rare in the heavy waves: the implicit echo and reply slots of the edge)
    const uint4 r0 = (v && rxe) ? gld4(p.inbox + inbox_idx(p, ib, rep, e)) : make_uint4(0, 0, 0, 0);
    uint4 w0 = (v && sl0) ? gld4(eslot_at(p, ob, rep, e)) : make_uint4(0, 0, 0, 0);
    uint4 w1 = (v && sl1) ? gld4(eslot_at(p, obp, rep, e)) : make_uint4(0, 0, 0, 0);
    bool hd0 = false, hd1 = false;
    if (sd0) {
      const uint4 mb = T.mtb[il][0];
      const unsigned long long m = (static_cast<unsigned long long>(mb.y) << 32) | mb.x;
      hd0 = v && (m & lbit);
      if (hd0) w0 = make_uint4(T.job[il][1].x, T.job[il][1].y, T.job[il][1].z + mb.z + static_cast<uint32_t>(__popcll(m & lbelow)),
                               T.job[il][1].w);
    }
    if (sd1) {
      const uint4 mb = T.mtb[il][1];
      const unsigned long long m = (static_cast<unsigned long long>(mb.y) << 32) | mb.x;
      hd1 = v && (m & lbit);
      if (hd1) w1 = make_uint4(T.job[il][2].x, T.job[il][2].y, T.job[il][2].z + mb.z + static_cast<uint32_t>(__popcll(m & lbelow)),
                               T.job[il][2].w);
    }
    if (!v) continue;
    // pending echo descriptors, oldest first, onto the link word
    int64_t bu = static_cast<int64_t>(lw0 >> 16);
    uint32_t lc = static_cast<uint32_t>(lw0 & 0xFFFFu);
    bool pe = false;
    for (uint32_t d = 0; d < ne; ++d) {
      const uint2 em = T.mte[il][d];
      const unsigned long long m = (static_cast<unsigned long long>(em.y) << 32) | em.x;
      if (m & lbit) {
        const uint4 q3 = T.job[il][3];
        const int64_t et = static_cast<int64_t>(d ? ((static_cast<uint64_t>(q3.w) << 32) | q3.z)
                                                  : ((static_cast<uint64_t>(q3.y) << 32) | q3.x));
        bu = (bu > et ? bu : et) + ((fl & (d ? kJBig1 : kJBig0)) ? tx1 : tx0);
        pe = true;
      }
    }
    // implicit echo of in-slot le
    bool he = false;
    int64_t et = 0;
    uint32_t edt = 0, esub = 0;
    int ebig = 0;
    if (rxe) {
      const uint32_t rfl = r0.w >> 24;
      const long long ta0 = cs + r0.x;
      if (slot_live(rfl, tag) && ta0 >= t_lo && ta0 < t_hi && p.echo) {
        ebig = (rfl & RF_BIG) ? 1 : 0;
        const int64_t pin = p.prop_const >= 0 ? p.prop_const : gbl(p.prop_in)[e];
        et = ta0;
        edt = static_cast<uint32_t>(pin + (ebig ? txl1 : txl0));
        esub = r0.y;
        he = true;
        ++st_echo;
      }
    }
    const int64_t rt1 = static_cast<int64_t>((static_cast<uint64_t>(w0.y) << 32) | w0.x);
    const int64_t rt2 = static_cast<int64_t>((static_cast<uint64_t>(w1.y) << 32) | w1.x);
    bool hr = (sl0 || hd0) && rt1 >= t_lo && rt1 < t_hi;
    bool hr2 = (sl1 || hd1) && rt2 >= t_lo && rt2 < t_hi;
    st_ops += (hr ? 1u : 0u) + (hr2 ? 1u : 0u);
    if (n_bc == 0 && !he && !hr && !hr2 && !pe) continue;
    ++st_edges;
    const int64_t pr = p.prop_const >= 0 ? p.prop_const : gbl(p.prop)[e];
    const uint32_t slot = s * N1 + (i < s ? i : i - 1);
    const uint32_t dg = rep * N + s;
    bool in_lds = false;
    // one message through the FIFO and out as a record (slot via the LDS transpose, direct,
    // extras or overflow)
    auto emit = [&](int64_t ot, uint32_t osub, uint32_t ow2, uint32_t ow3, int big) {
      const int64_t start = bu > ot ? bu : ot;
      const int64_t end = start + (big ? tx1 : tx0);
      bu = end;
      const int64_t ta = end + pr;
      long long ca;
      uint32_t tof;
      {
        const int64_t dtf = ta - cs;
        if (dtf >= 0 && dtf < (1ll << 32)) {  // (floor by the reciprocal, see k_link_mesh)
          const uint32_t x = static_cast<uint32_t>(dtf);
          const uint32_t qq = static_cast<uint32_t>(__umul64hi(static_cast<uint64_t>(x), p.L_magic));
          ca = cell + qq;
          tof = x - qq * L32;
        } else {
          ca = ta / p.L;
          tof = static_cast<uint32_t>(ta - ca * p.L);
        }
      }
      const long long rel = ca - cell;
      if (rel < 1) {
        set_err(p, BCSIM_E_TIE);  // lookahead violated
        return;
      }
      ++n_rec;
      const uint32_t w3 = ow3 | (static_cast<uint32_t>(RF_VALID | (big ? RF_BIG : 0)) << 24) |
                          (emit_tag(cq_b, cr_b, rel, B) << 27);
      const uint4 rv = make_uint4(tof, osub, ow2, w3);
      const bool owner = lc != (static_cast<uint32_t>(ca) & 0xFFFFu);
      lc = static_cast<uint32_t>(ca) & 0xFFFFu;
      if (rel < static_cast<long long>(B)) {
        uint32_t bk = cr_b + static_cast<uint32_t>(rel);
        if (bk >= B) bk -= B;
        if (owner) {
          if (!in_lds) {  // the edge's first slot record: through the LDS transpose
            T.rec[q] = rv;
            T.rbk[q] = static_cast<uint8_t>(bk);
            bkm |= 1ull << bk;
            in_lds = true;
          } else {
            gst4(p.inbox + inbox_idx(p, bk, rep, slot), rv);
            xs_mark(p, bk, rep, i, s, w3);
            set_flag_once(&AT(p.rtile, kRtPad * ((static_cast<size_t>(bk) * p.R + rep) * p.n_tiles + (s >> 6)), kRtPad * (static_cast<uint64_t>(B) * p.R * p.n_tiles)));
          }
        } else {
          XRec x;
          __builtin_memcpy(&x.r, &rv, sizeof rv);
          x.cell = ca;
          x.slot = slot;
          x.g = dg;
          tile_append(p, T, bk, x);
          gbl(p.iflag)[static_cast<size_t>(bk) * p.NT + dg] = 1;
        }
        if (bk != cb) {
          if (cbn) {
            atomicAdd(&T.lcnt[cb], cbn);
            atomicMin(&T.lmin[cb], cmn);
          }
          cb = bk;
          cbn = 0;
          cmn = ~0u;
        }
        ++cbn;
        if (tof < cmn) cmn = tof;
      } else {
        XRec x;
        __builtin_memcpy(&x.r, &rv, sizeof rv);
        if (owner) x.r.flags = static_cast<uint8_t>(x.r.flags | RF_OWNER);
        x.cell = ca;
        x.slot = slot;
        x.g = dg;
        tile_append(p, T, B, x);
        if (ca < ovmin) ovmin = ca;
      }
    };
    if (static_cast<uint32_t>(n_bc) + (hr ? 1u : 0u) + (hr2 ? 1u : 0u) + (he ? 1u : 0u) == 1u) {
      // one source (the heavy waves: a broadcast, or a reply): no merge
      if (n_bc) {
        const uint4 a = T.bc[il][0], bw = T.bc[il][1];
        emit(static_cast<int64_t>((static_cast<uint64_t>(a.y) << 32) | a.x), bw.x + le, bw.z, bw.w & 0x00FFFFFFu,
             ((bw.w >> 26) & OPF_BIG) ? 1 : 0);
      } else if (hr || hr2) {
        ++sends;
        const uint4 w = hr ? w0 : w1;
        emit(hr ? rt1 : rt2, w.z, w.w, w3r, 0);
      } else {  // the echo only occupies the link
        bu = (bu > et ? bu : et) + (ebig ? tx1 : tx0);
      }
    } else {
      uint32_t bi = 0;
      for (;;) {
        // the earliest source: 1 broadcast, 2 / 4 reply slots, 3 echo (Paxos broadcasts never get here)
        int src = 0;
        int64_t ot = 0;
        uint32_t odt = 0, oor = 0, osub = 0, ow2 = 0, ow3 = 0;
        int big = 0;
        if (bi < n_bc) {
          const uint4 a = T.bc[il][2 * bi], bw = T.bc[il][2 * bi + 1];
          ot = static_cast<int64_t>((static_cast<uint64_t>(a.y) << 32) | a.x);
          odt = a.z;
          oor = a.w;
          osub = bw.x + le;
          ow2 = bw.z;
          ow3 = bw.w & 0x00FFFFFFu;
          big = ((bw.w >> 26) & OPF_BIG) ? 1 : 0;
          src = 1;
        }
        if (hr && (src == 0 || kless(rt1, static_cast<uint32_t>(app), i, w0.z, ot, odt, oor, osub))) {
          ot = rt1;
          odt = static_cast<uint32_t>(app);
          oor = i;
          osub = w0.z;
          ow2 = w0.w;
          ow3 = w3r;
          big = 0;
          src = 2;
        }
        if (hr2 && (src == 0 || kless(rt2, static_cast<uint32_t>(app), i, w1.z, ot, odt, oor, osub))) {
          ot = rt2;
          odt = static_cast<uint32_t>(app);
          oor = i;
          osub = w1.z;
          ow2 = w1.w;
          ow3 = w3r;
          big = 0;
          src = 4;
        }
        if (he && (src == 0 || kless(et, edt, s, esub, ot, odt, oor, osub))) {
          ot = et;
          big = ebig;
          src = 3;
        }
        if (src == 0) break;
        if (src == 1)
          ++bi;
        else if (src == 2)
          hr = false;
        else if (src == 4)
          hr2 = false;
        else
          he = false;
        if (src == 3) {  // the echo only occupies the link
          bu = (bu > ot ? bu : ot) + (big ? tx1 : tx0);
          continue;
        }
        if (src == 2 || src == 4) ++sends;
        emit(ot, osub, ow2, ow3, big);
      }
    }
    if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
    if (BCSIM_TILE_DEFER)
      T.lwo[BCSIM_TILE_DEFER ? il : 0][lane] = (static_cast<uint64_t>(bu) << 16) | lc;
    else
      gbl(p.link)[edge_loc(p, rep, e)] = (static_cast<uint64_t>(bu) << 16) | lc;
  }
  if (cbn) {
    atomicAdd(&T.lcnt[cb], cbn);
    atomicMin(&T.lmin[cb], cmn);
  }
  for (int d = 32; d > 0; d >>= 1) {
    bkm |= static_cast<unsigned long long>(__shfl_xor(bkm, d, 64));
    ovmin = min(ovmin, static_cast<long long>(__shfl_xor(ovmin, d, 64)));
  }
  {
    const uint32_t c5[5] = {sends, n_rec, st_ops, st_edges, st_echo};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const uint32_t ws = wave_sum(c5[k]);
      if (lane == 0 && ws) atomicAdd(&T.csum[k], ws);
    }
  }
  if (lane == 0) {
    if (bkm) atomicOr(&T.bkm, bkm);
    if (ovmin != LLONG_MAX) atomicMin(&T.ovmin, ovmin);
  }
  TPH(3);
  __syncthreads();
  TPH(4);
  // the link words, sender-major (one sender's 64 out-edges per wave-instruction)
  for (uint32_t x = tid; BCSIM_TILE_DEFER && x < kTR * kTS; x += blockDim.x) {
    const uint32_t il = x / kTR, sl = x % kTR;
    const uint64_t w = T.lwo[BCSIM_TILE_DEFER ? il : 0][sl];
    if (!w) continue;
    const uint32_t i = i0 + il, sr = s0 + sl;
    gbl(p.link)[edge_loc(p, rep, i * N1 + (sr < i ? sr : sr - 1))] = w;
  }
  // the transposed slot records: each receiver's in-slots of this sender tile in one run
  for (uint32_t x = tid; x < kTR * kTS; x += blockDim.x) {
    const uint32_t sl = x / kTS, il = x % kTS;
    const uint32_t q = tsw(sl, il);
    const uint32_t bk = T.rbk[q];
    if (bk == 0xFFu || (p.exp & 4u)) continue;
    const uint32_t sr = s0 + sl, i = i0 + il;
    const uint32_t slot = sr * N1 + (i < sr ? i : i - 1);
    const uint4 rq = T.rec[q];
    gst4(p.inbox + inbox_idx(p, bk, rep, slot), rq);
    xs_mark(p, bk, rep, i, sr, rq.w);
  }
  // staged extras / overflow records: one atomic per list
  if (T.xn) {
    for (uint32_t k = tid; k <= B; k += blockDim.x) {
      const uint32_t c = T.lst[k];
      if (!c) continue;
      uint32_t* ctr = k == B ? p.ov_cnt : &p.x_cnt[k];
      const uint32_t cap = k == B ? p.cap_ov : p.cap_x;
      const uint32_t base = gadd_r(ctr, c);
      if (base + c > cap) set_err(p, BCSIM_E_OVERFLOW);
      T.lst[k] = base;  // (this lane's list only: no other lane reads it before the barrier)
    }
    __syncthreads();
    const uint32_t nx = min(T.xn, kTX);
    for (uint32_t k = tid; k < nx; k += blockDim.x) {
      const uint32_t list = T.xm[k] >> 24, at = T.lst[list] + (T.xm[k] & 0xFFFFFFu);
      if (list == B) {
        if (at < p.cap_ov) {
          const uint4* src = reinterpret_cast<const uint4*>(&T.xs[k]);
          uint4* dst = reinterpret_cast<uint4*>(p.ov + at);
          gst4(dst, src[0]);
          gst4(dst + 1, src[1]);
        }
      } else if (at < p.cap_x) {
        const uint4* src = reinterpret_cast<const uint4*>(&T.xs[k]);
        uint4* dst = reinterpret_cast<uint4*>(p.xbuf + static_cast<size_t>(list) * p.cap_x + at);
        gst4(dst, src[0]);
        gst4(dst + 1, src[1]);
      }
    }
  }
  // receiver-tile flags of the buckets written, busy buckets, arrival-time bounds: stores and
  // atomics that return nothing (no round trip at the end of the workgroup); the bound is
  // lowered only below the value read at the start
  if (tid < B && ((T.bkm >> tid) & 1ull))
    gbl(p.rtile)[kRtPad * ((static_cast<size_t>(tid) * p.R + rep) * p.n_tiles + rt)] = 1;
  for (uint32_t k = tid; k < B; k += blockDim.x)
    if (T.lcnt[k]) {
      gbl(p.bucket_cnt)[k] = 1u;
      const long long t = bucket_t0(p, (t_hi - 1) / p.L, k) + T.lmin[k];
      if (t < T.bmin[k]) __hip_atomic_fetch_min(gbl(p.bmin) + k, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  if (tid == 0) {
    unsigned long long* cnt = cnt_stripe(p, rep);
    unsigned long long* ks = kst_stripe(p);
    if (T.csum[0]) gadd(&cnt[CNT_SENDS], static_cast<unsigned long long>(T.csum[0]));
    if (T.csum[1]) gadd(&ks[KST_REC], static_cast<unsigned long long>(T.csum[1]));
    if (T.csum[2]) gadd(&ks[KST_OPS], static_cast<unsigned long long>(T.csum[2]));
    if (T.csum[3]) gadd(&ks[KST_EDGES], static_cast<unsigned long long>(T.csum[3]));
    if (T.csum[4]) gadd(&ks[KST_ECHO], static_cast<unsigned long long>(T.csum[4]));
    if (T.ovmin != LLONG_MAX) __hip_atomic_fetch_min(gbl(p.scal) + 1, T.ovmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  TPH(5);
#undef TPH
}

// ---------------------------------------------------------------------------
// k_mesh_row (summary mode): the edges of a sender whose job has the heavy
// waves' uniform shape (job_uniform: the one due broadcast, pbft-node.cc:349-368, or the one
// due reply descriptor, :212-222), one 256-lane workgroup per sender walking its row one
// receiver tile (64 out-edges) per wave-iteration.  With summaries no record needs the tile
// kernel's transpose: the link words are read and written coalesced (a sender's row is
// contiguous), the tile's records that differ only in sub are ONE summary entry (merged as in
// k_mesh_tile), any other slot record is stored directly, and second records of an edge
// (extras) and records beyond the ring (overflow) are appended with one atomic per list and
// wave.  The first pass takes a row-uniform sender's whole row at once (lane = receiver tile).
// The per-edge work and its results are k_mesh_tile's.
constexpr uint32_t kRowSplitDev = 1u << 31;  // k_mesh_row's split argument: decide from the list length
constexpr uint32_t kDevSized = 0xFFFFFFFFu;    // (host) a window whose kernels are sized on the device
constexpr uint32_t kRowThreads = 1024;  // 16 senders per workgroup, one wave each (or one sender over 16 waves)
struct RowShared {
  XRec xs[kTX];  // staged extras / overflow records: one global atomic per list and workgroup
  uint32_t xm[kTX];  // list << 24 | rank
  uint32_t xn;
  uint32_t lst[kMaxBuckets + 1];
  uint32_t lcnt[kMaxBuckets];
  uint32_t lmin[kMaxBuckets];
  uint32_t csum[8];
  long long ovmin;
  long long bmin[kMaxBuckets];  // the buckets' arrival-time bounds as of the start (read early)
};
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(5, 8))) void k_mesh_row(
    const KP* __restrict__ pk, long long cell, long long t_lo, long long t_hi, uint32_t epoch, uint4 hq, uint32_t split) {
  // hq (host arithmetic, no 64-bit divisions here): {cell % B, (cell / B) % 32, the bucket a small
  // message sent at t_lo lands in on an idle link (0xFFFF: outside the ring), 0}
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ RowShared T;
  const uint32_t tid = tidx(), lane = tid & 63u, wv = tid >> 6, nwv = blockDim.x >> 6;
  G<unsigned long long>* tph = p.wgtt ? gbl(p.wgtt) + 8ull * blockIdx.x : nullptr;  // (debug phase clocks)
#define RPH(k)                                                       \
  do {                                                               \
    if (tph && tid == 0) tph[(k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  RPH(0);
  const uint32_t N = p.N, N1 = N - 1, B = p.n_buckets, nrt = p.n_tiles;
  const int64_t prc = p.prop_const;
  const long long cs = cell * p.L;
  const uint32_t cr_b = hq.x, cq_b = hq.y;
  const uint32_t cbk0 = (hq.z & 0xFFFFu) == 0xFFFFu ? kInvalid : (hq.z & 0xFFFFu);
  auto rl = [](uint32_t x, uint32_t k) { return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), static_cast<int>(k))); };
  // this wave's sender (list-1 entry blockIdx * (waves / split) + wave / split; `split` waves share
  // a sender's row when the launch has few senders -- the leader's block broadcast -- each one a
  // contiguous range of its receiver tiles) and, all at once, its job words (lanes 0-3), its
  // broadcast (4-5) and its row's uniform link word (6)
  if (split & kRowSplitDev) split = p.act_n[1] <= (split & 0xFFFFu) ? 16u : 1u;  // (device-sized launch)
  const uint32_t part = wv % split, kk = blockIdx.x * (nwv / split) + wv / split;
  const uint32_t tpp = (p.n_tiles + split - 1) / split, t0 = min(p.n_tiles, part * tpp), t1 = min(p.n_tiles, t0 + tpp);
  const bool own_t = lane >= t0 && lane < t1;  // (lane k: tile k is this wave's)
  bool act = kk < p.act_n[1];
  const uint32_t g = act ? rl(p.act[p.NT + kk], 0) : 0u;
  uint4 jw = make_uint4(0, 0, 0, 0);
  if (act) {
    if (lane < 4) jw = gld4(p.mjob + static_cast<size_t>(g) * 4 + lane);
    else if (lane < 6) jw = gld4(p.mbc + static_cast<size_t>(g) * kMeshBc * 2 + (lane - 4));
    else if (lane == 6) {
      const uint64_t r = gbl(p.rul)[g];
      jw = make_uint4(static_cast<uint32_t>(r), static_cast<uint32_t>(r >> 32), 0u, 0u);
    }
  }
  for (uint32_t k = tid; k < B; k += blockDim.x) {
    T.lcnt[k] = 0;
    T.lmin[k] = ~0u;
  }
  for (uint32_t k = tid; k <= B; k += blockDim.x) T.lst[k] = 0;
  if (tid < 8) T.csum[tid] = 0;
  if (tid == 0) {
    T.ovmin = LLONG_MAX;
    T.xn = 0;
  }
  if (tid >= 64 && tid < 64 + B) T.bmin[tid - 64] = *reinterpret_cast<volatile G<long long>*>(&gbl(p.bmin)[tid - 64]);
  const uint32_t fl = rl(jw.y, 0), jz = rl(jw.z, 0);
  act = act && rl(jw.x, 0) == epoch && job_uniform(fl, jz, prc);
  const uint32_t ne = jz & 0xFFu, n_bc = (jz >> 8) & 0xFFu;
  const uint32_t h = (fl & kJSd0) ? 0u : 1u;
  const uint32_t rep = g / N, i = g % N;
  // per receiver tile k (lane k): its exception bits, reply bitmap {lo, hi, rank base}, pending
  // echo bitmaps, and the summary entry of the bucket an idle link delivers in -- one round
  uint64_t rexo = 0;
  uint4 tmb = make_uint4(0, 0, 0, 0), tme = make_uint4(0, 0, 0, 0), soa = make_uint4(0, 0, 0, 0), sob = make_uint4(0, 0, 0, 0);
  if (act && own_t) {
    rexo = gbl(p.rex)[static_cast<size_t>(g) * nrt + lane];
    if (!n_bc) tmb = gld4(p.mtb + (static_cast<size_t>(g) * nrt + lane) * 2 + h);
    if (ne) tme = gld4(reinterpret_cast<const uint4*>(p.mte + (static_cast<size_t>(g) * nrt + lane) * kEDesc));
    if (cbk0 != kInvalid) {
      const uint4* se = p.msum + sum_idx(p, cbk0, rep, lane, i) * 2;
      soa = gld4(se);
      sob = gld4(se + 1);
    }
  }
  RPH(1);
  uint32_t n_rec = 0, st_edges = 0, st_ops = 0, nu = 0;
  long long ovmin = LLONG_MAX;
  uint32_t cb = kInvalid, cbn = 0, cmn = ~0u;
  uint64_t rexn = 0, rtm = 0;  // (lane k: tile k's new exception bits; bit k: tile k holds records of bucket bk_u)
  uint32_t tof_u = 0, bk_u = 0;
  bool ring_u = false;
  uint64_t nw_u = 0;
  if (act) {
    const uint32_t L32 = static_cast<uint32_t>(p.L);
    const int64_t tx0 = p.tx_tot[0], tx1 = p.tx_tot[1];
    const uint64_t Lmag = p.L_magic;
    const unsigned long long lbit = 1ull << lane, lbelow = lbit - 1ull;
    // the source's uniform words: due time, the first edge's sub, payload, frame size
    const uint32_t sa_x = rl(n_bc ? jw.x : (h ? jw.x : jw.x), n_bc ? 4 : 1 + h), sa_y = rl(jw.y, n_bc ? 4 : 1 + h);
    const uint32_t sa_z = rl(jw.z, 1 + h), sa_w = rl(jw.w, 1 + h);
    const uint32_t u_s0 = n_bc ? rl(jw.x, 5) : sa_z;
    const uint32_t u_w2 = n_bc ? rl(jw.z, 5) : sa_w;
    const uint32_t u_w3 = n_bc ? rl(jw.w, 5) : static_cast<uint32_t>(static_cast<uint16_t>(enc_raw(p, 0))) | (kPbPrepareRes << 16);
    const int big = (n_bc && ((u_w3 >> 26) & OPF_BIG)) ? 1 : 0;
    const int64_t ot = static_cast<int64_t>((static_cast<uint64_t>(sa_y) << 32) | sa_x);
    const int64_t txu = big ? tx1 : tx0;
    const uint32_t w3u = (u_w3 & 0x00FFFFFFu) | (static_cast<uint32_t>(RF_VALID | (big ? RF_BIG : 0)) << 24);
    const int64_t et0 = static_cast<int64_t>((static_cast<uint64_t>(rl(jw.y, 3)) << 32) | rl(jw.x, 3));
    const int64_t et1 = static_cast<int64_t>((static_cast<uint64_t>(rl(jw.w, 3)) << 32) | rl(jw.z, 3));
    const int64_t etx0 = (fl & kJBig0) ? tx1 : tx0, etx1 = (fl & kJBig1) ? tx1 : tx0;
    const uint64_t ru = (static_cast<uint64_t>(rl(jw.y, 6)) << 32) | rl(jw.x, 6);
    const bool ruv = (ru >> 63) != 0;
    const uint64_t ruw = ru & ~(1ull << 63);
    uint64_t* const lrow = p.link + edge_loc(p, rep, i * N1);
    // the heavy waves' case, computed once: the link is free by the due time, so every message
    // starts at it and arrives at one instant in one cell (uniform over the row)
    const int64_t end_u = ot + txu;
    uint32_t ca16_u = 0, w3f_u = 0;
    {
      const int64_t dtf = end_u + prc - cs;
      if (dtf >= 0 && dtf < (1ll << 32) && end_u < (1ll << 47)) {
        const uint32_t x = static_cast<uint32_t>(dtf);
        const uint32_t qq = static_cast<uint32_t>(__umul64hi(static_cast<uint64_t>(x), Lmag));
        ring_u = qq >= 1u && qq < B;
        ca16_u = static_cast<uint32_t>(cell + qq) & 0xFFFFu;
        tof_u = x - qq * L32;
        const uint32_t bq = cr_b + qq;
        bk_u = bq >= B ? bq - B : bq;
        w3f_u = w3u | (static_cast<uint32_t>((cq_b + (bq >= B ? 1 : 0)) & 31) << 27);
      }
    }
    nw_u = (static_cast<uint64_t>(end_u) << 16) | ca16_u;
    const bool pfd_u = bk_u == cbk0;
    // ---- the heavy waves' case over the whole row at once, lane = receiver tile: under a
    // row-uniform link state every edge without its own word has the row's word; after the pending
    // echoes (at most four classes of edges) the ones with a message whose link is free by the due
    // time (and that own the arrival cell) send one uniform record each -- the tile's records are
    // ONE summary entry (one base when the reply bitmap is contiguous), and their new link word is
    // the row's new word nw_u, i.e. nothing per edge.  The rest of the tile (its residue) takes the
    // per-tile walk below.
    uint64_t fset = 0, res = 0;
    if (own_t) {
      const uint32_t s0 = lane * 64u, nvr = min(64u, N - s0);
      uint64_t vm = nvr >= 64u ? ~0ull : ((1ull << nvr) - 1ull);
      if (i >= s0 && i < s0 + 64u) vm &= ~(1ull << (i - s0));
      const uint64_t hm = n_bc ? vm : (((static_cast<uint64_t>(tmb.y) << 32) | tmb.x) & vm);
      if (ruv && ring_u && pfd_u && hm) {
        const uint64_t e0m = ne ? (((static_cast<uint64_t>(tme.y) << 32) | tme.x) & vm) : 0ull;
        const uint64_t e1m = ne > 1 ? (((static_cast<uint64_t>(tme.w) << 32) | tme.z) & vm) : 0ull;
        const int64_t bA = static_cast<int64_t>(ruw >> 16);
        const int64_t bB = (bA > et0 ? bA : et0) + etx0, bC = (bA > et1 ? bA : et1) + etx1;
        const int64_t bD = (bB > et1 ? bB : et1) + etx1;
        const bool own_c = static_cast<uint32_t>(ruw & 0xFFFFu) != ca16_u;
        const uint64_t okm = ((bA <= ot) ? (~e0m & ~e1m) : 0ull) | ((bB <= ot) ? (e0m & ~e1m) : 0ull) |
                             ((bC <= ot) ? (~e0m & e1m) : 0ull) | ((bD <= ot) ? (e0m & e1m) : 0ull);
        uint64_t fs = own_c ? (hm & ~(rexo & vm) & okm) : 0ull;
        uint32_t base = u_s0;
        if (!n_bc && fs) {  // sub = first sub + rank: sub - out-edge index is one value on a contiguous bitmap
          const uint32_t lo = static_cast<uint32_t>(__builtin_ctzll(hm));
          const uint32_t slo = s0 + lo;
          if ((vm & ~hm) >> lo) fs = 0ull;
          else base = u_s0 + tmb.z - (slo < i ? slo : slo - 1u);
        }
        const bool olive = (soa.x | soa.y) != 0u && slot_live(sob.y >> 24, w3f_u >> 27);
        if (olive && (soa.z != tof_u || soa.w != base || sob.x != u_w2 || sob.y != w3f_u)) fs = 0ull;
        if (fs) {
          const uint64_t mm = fs | (olive ? ((static_cast<uint64_t>(soa.y) << 32) | soa.x) : 0ull);
          uint4* const se = p.msum + sum_idx(p, bk_u, rep, lane, i) * 2;
          gst4(se, make_uint4(static_cast<uint32_t>(mm), static_cast<uint32_t>(mm >> 32), tof_u, base));
          gst4(se + 1, make_uint4(u_w2, w3f_u, 0u, 0u));
          const uint32_t nf = static_cast<uint32_t>(__popcll(fs));
          n_rec += nf;
          st_edges += nf;
          if (!n_bc) st_ops += nf;
        }
        fset = fs;
      }
      res = vm & ~fset;
    }
    rtm = __ballot(fset != 0ull);
    nu = wave_sum(static_cast<uint32_t>(__popcll(fset)));
    unsigned long long* const tdb = tph ? reinterpret_cast<unsigned long long*>(const_cast<unsigned long long*>(
                                              reinterpret_cast<volatile unsigned long long*>(tph))) : nullptr;
    if (tdb && lane == 0)  // (debug, BCSIM_WGT: rows / without a uniform state / beyond the ring / off the idle bucket)
      atomicAdd(tdb + 7, 1ull | ((ruv ? 0ull : 1ull) << 16) | ((ring_u ? 0ull : 1ull) << 32) | ((pfd_u ? 0ull : 1ull) << 48));
#pragma unroll 1
    for (uint32_t rt = t0; rt < t1; ++rt) {
      const uint64_t rmask = (static_cast<uint64_t>(rl(static_cast<uint32_t>(res >> 32), rt)) << 32) | rl(static_cast<uint32_t>(res), rt);
      if (!rmask) continue;  // (uniform) every edge of the tile done above
      if (tdb && lane == 0) atomicAdd(tdb + 6, 1ull);  // (debug: tiles walked)
      // (a tile with an entry from above writes its other records as records)
      const bool fdone = (rl(static_cast<uint32_t>(fset), rt) | rl(static_cast<uint32_t>(fset >> 32), rt)) != 0u;
      const uint32_t s = rt * 64u + lane;
      const bool v = (rmask >> lane) & 1ull;
      const uint32_t le = s < i ? s : s - 1;
      const uint64_t xo = (static_cast<uint64_t>(rl(static_cast<uint32_t>(rexo >> 32), rt)) << 32) | rl(static_cast<uint32_t>(rexo), rt);
      const bool wex = ruv && ((xo >> lane) & 1ull);  // (had its own word under the row's uniform state)
      // the edge's link word: its own (loaded here: a row's exception edges, or every edge of a
      // row without a uniform state), else the row's uniform word
      const bool own = v && (!ruv || wex);
      uint64_t lw0 = ruw;
      if (__ballot(own)) {
        const uint64_t x = own ? gbl(lrow)[le] : 0ull;
        lw0 = own ? x : ruw;
      }
      const uint32_t lc0 = static_cast<uint32_t>(lw0 & 0xFFFFu);
      // its new link word: the row's new uniform word nw_u (no store, exception bit clear), else its
      // own -- stored when it changed, or when it was the row's old uniform word
      auto put_lw = [&](uint64_t nv) {
        const bool un = ring_u && v && nv == nw_u;
        if (v && !un && (nv != lw0 || (ruv && !wex))) gbl(lrow)[le] = nv;
        const unsigned long long xm = __ballot(v && !un);
        rexn = lane == rt ? xm : rexn;
      };
      bool has = v;
      uint32_t u_sub = u_s0;
      if (!n_bc) {  // the reply descriptor's bitmap of this tile: sub = first sub + rank
        const unsigned long long m = (static_cast<unsigned long long>(rl(tmb.y, rt)) << 32) | rl(tmb.x, rt);
        has = v && (m & lbit);
        u_sub = u_s0 + rl(tmb.z, rt) + static_cast<uint32_t>(__popcll(m & lbelow)) - le;
      }
      int64_t bu = static_cast<int64_t>(lw0 >> 16);
      bool pe = false;
      if (ne) {  // pending echo descriptors, oldest first
        const unsigned long long m0 = (static_cast<unsigned long long>(rl(tme.y, rt)) << 32) | rl(tme.x, rt);
        const bool h0 = v && (m0 & lbit);
        bu = h0 ? (bu > et0 ? bu : et0) + etx0 : bu;
        pe = h0;
        if (ne > 1) {
          const unsigned long long m1 = (static_cast<unsigned long long>(rl(tme.w, rt)) << 32) | rl(tme.z, rt);
          const bool h1 = v && (m1 & lbit);
          bu = h1 ? (bu > et1 ? bu : et1) + etx1 : bu;
          pe = pe || h1;
        }
      }
      // the uniform case: every edge with a message finds its link free by the due time (after its
      // pending echoes) and owns the arrival cell -- the tile's records are one summary entry (the
      // lanes with the first one's base), the link words one value
      if (ring_u && __ballot(has && !(bu <= ot && lc0 != ca16_u)) == 0ull) {
        const unsigned long long hm = __ballot(has);
        if (hm) {
          const uint32_t r_base = n_bc ? u_s0 : rl(u_sub, static_cast<uint32_t>(__ffsll(static_cast<long long>(hm)) - 1));
          bool uni = has && u_sub == r_base;
          unsigned long long um = __ballot(uni);
          // the entry an earlier launch may have left for this (bucket, tile, sender) turn
          const uint32_t oax = rl(soa.x, rt), oay = rl(soa.y, rt), oaz = rl(soa.z, rt), oaw = rl(soa.w, rt);
          const uint32_t obx = rl(sob.x, rt), oby = rl(sob.y, rt);
          const bool olive = (oax | oay) != 0u && slot_live(oby >> 24, w3f_u >> 27);
          if (fdone || !pfd_u || (olive && (oaz != tof_u || oaw != r_base || obx != u_w2 || oby != w3f_u))) um = 0ull;
          if (um) {
            const unsigned long long mm = um | (olive ? ((static_cast<unsigned long long>(oay) << 32) | oax) : 0ull);
            uint4* const se = p.msum + sum_idx(p, bk_u, rep, rt, i) * 2;
            if (lane < 2u)
              gst4(se + lane, lane ? make_uint4(u_w2, w3f_u, 0u, 0u)
                                   : make_uint4(static_cast<uint32_t>(mm), static_cast<uint32_t>(mm >> 32), tof_u, r_base));
          }
          uni = (um >> lane) & 1ull;
          if (has && !uni) {  // (another base, or an entry of other words: a slot record)
            gst4(p.inbox + inbox_idx(p, bk_u, rep, s * N1 + (i < s ? i : i - 1)), make_uint4(tof_u, u_sub + le, u_w2, w3f_u));
            gbl(p.xsum)[sum_idx(p, bk_u, rep, rt, i)] = static_cast<uint8_t>(0x80u | (w3f_u >> 27));
          }
          rtm |= 1ull << rt;
          nu += static_cast<uint32_t>(__popcll(hm));
        }
        if (has) {
          ++n_rec;
          if (!n_bc) ++st_ops;
        }
        if (has || pe) ++st_edges;
        put_lw(has ? nw_u : pe ? ((static_cast<uint64_t>(bu) << 16) | lc0) : lw0);
        continue;
      }
      // the message through the FIFO (k_mesh_tile's emit)
      const int64_t start = bu > ot ? bu : ot;
      const int64_t end = start + txu;
      const int64_t ta = end + prc;
      long long ca;
      uint32_t tof;
      {
        const int64_t dtf = ta - cs;
        if (dtf >= 0 && dtf < (1ll << 32)) {
          const uint32_t x = static_cast<uint32_t>(dtf);
          const uint32_t qq = static_cast<uint32_t>(__umul64hi(static_cast<uint64_t>(x), Lmag));
          ca = cell + qq;
          tof = x - qq * L32;
        } else {
          ca = ta / p.L;
          tof = static_cast<uint32_t>(ta - ca * p.L);
        }
      }
      const long long rel = ca - cell;
      if (has && rel < 1) set_err(p, BCSIM_E_TIE);  // lookahead violated
      const bool emit = has && rel >= 1;
      const bool owner = lc0 != (static_cast<uint32_t>(ca) & 0xFFFFu);
      const bool inring = rel < static_cast<long long>(B);
      const uint32_t bq = cr_b + static_cast<uint32_t>(inring ? rel : 0);
      const bool wrap = bq >= B;
      const uint32_t bk = wrap ? bq - B : bq;
      const uint32_t w3f = w3u | (static_cast<uint32_t>((cq_b + (wrap ? 1 : 0)) & 31) << 27);
      const bool ok = emit && inring && owner;  // the edge's slot record of its arrival cell
      // (summaries) the ok lanes with the first one's bucket, offset and base -- merged only with a
      // prefetched entry (the idle-link bucket), else written as records
      const unsigned long long okm = __ballot(ok);
      bool uni = false;
      if (okm) {
        const uint32_t q = static_cast<uint32_t>(__ffsll(static_cast<long long>(okm)) - 1);
        const uint32_t r_tof = rl(tof, q), r_base = rl(u_sub, q), r_w3 = rl(w3f, q), r_bk = rl(bk, q);
        uni = ok && tof == r_tof && u_sub == r_base && bk == r_bk;
        unsigned long long um = __ballot(uni);
        const uint32_t oax = rl(soa.x, rt), oay = rl(soa.y, rt), oaz = rl(soa.z, rt), oaw = rl(soa.w, rt);
        const uint32_t obx = rl(sob.x, rt), oby = rl(sob.y, rt);
        const bool olive = (oax | oay) != 0u && slot_live(oby >> 24, r_w3 >> 27);
        if (fdone || r_bk != cbk0 || (olive && (oaz != r_tof || oaw != r_base || obx != u_w2 || oby != r_w3))) um = 0ull;
        if (um) {
          const unsigned long long mm = um | (olive ? ((static_cast<unsigned long long>(oay) << 32) | oax) : 0ull);
          uint4* const se = p.msum + sum_idx(p, r_bk, rep, rt, i) * 2;
          if (lane < 2u)
            gst4(se + lane, lane ? make_uint4(u_w2, r_w3, 0u, 0u)
                                 : make_uint4(static_cast<uint32_t>(mm), static_cast<uint32_t>(mm >> 32), r_tof, r_base));
        }
        uni = (um >> lane) & 1ull;
        if (ok) gbl(p.rtile)[kRtPad * ((static_cast<size_t>(bk) * p.R + rep) * nrt + rt)] = 1;
      }
      if (emit) {
        ++n_rec;
        const uint32_t slot = s * N1 + (i < s ? i : i - 1);
        const uint4 rv = make_uint4(tof, u_sub + le, u_w2, w3f);
        if (ok && !uni) {
          gst4(p.inbox + inbox_idx(p, bk, rep, slot), rv);
          gbl(p.xsum)[sum_idx(p, bk, rep, rt, i)] = static_cast<uint8_t>(0x80u | (w3f >> 27));
        }
        if (!ok) {
          if (inring) gbl(p.iflag)[static_cast<size_t>(bk) * p.NT + rep * N + s] = 1;  // (extras)
          else if (ca < ovmin) ovmin = ca;
        }
        if (inring) {
          if (bk != cb) {
            if (cbn) {
              atomicAdd(&T.lcnt[cb], cbn);
              atomicMin(&T.lmin[cb], cmn);
            }
            cb = bk;
            cbn = 0;
            cmn = ~0u;
          }
          ++cbn;
          if (tof < cmn) cmn = tof;
        }
        if (!n_bc) ++st_ops;
      }
      const uint64_t nb = static_cast<uint64_t>(emit ? end : bu);
      if (emit || pe) {
        ++st_edges;
        if (nb >= (1ull << 47)) set_err(p, BCSIM_E_OVERFLOW);
      }
      put_lw((emit || pe) ? ((nb << 16) | (emit ? (static_cast<uint32_t>(ca) & 0xFFFFu) : lc0)) : lw0);
      // the records that are not their edge's slot record -- a second record of the edge in its
      // arrival cell (extras of bucket bk) or one beyond the ring (overflow) -- appended with one
      // atomic per list and wave (a leader's block broadcast puts its whole row beyond the ring)
      unsigned long long xmk = __ballot(emit && !ok);
      if (xmk) {
        const uint32_t list = inring ? bk : B;
        XRec x;
        {
          const uint4 rv = make_uint4(tof, u_sub + le, u_w2, w3f);
          __builtin_memcpy(&x.r, &rv, sizeof rv);
        }
        if (!inring && owner) x.r.flags = static_cast<uint8_t>(x.r.flags | RF_OWNER);
        x.cell = ca;
        x.slot = s * N1 + (i < s ? i : i - 1);
        x.g = rep * N + s;
        // the lanes grouped by list: each group's lowest lane reserves the group's span, all
        // groups in one atomic instruction (one round trip per tile)
        uint32_t ldr = 0, rk = 0, gc = 0;
        unsigned long long rem = xmk;
        while (rem) {
          const uint32_t q = static_cast<uint32_t>(__ffsll(static_cast<long long>(rem)) - 1);
          const uint32_t lq = rl(list, q);
          const unsigned long long mm = __ballot(((rem >> lane) & 1ull) && list == lq);
          if ((mm >> lane) & 1ull) {
            ldr = q;
            rk = static_cast<uint32_t>(__popcll(mm & lbelow));
          }
          if (lane == q) gc = static_cast<uint32_t>(__popcll(mm));
          rem &= ~mm;
        }
        // staged in LDS while the workgroup's area has room (one global atomic per list at the
        // end: the heavy waves' extras all go to one list), else reserved in the global lists
        const uint32_t nxa = static_cast<uint32_t>(__popcll(xmk));
        uint32_t p0 = kInvalid;
        if (lane == 0) {
          uint32_t cur = __hip_atomic_load(&T.xn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          while (cur + nxa <= kTX) {
            const uint32_t prev = atomicCAS(&T.xn, cur, cur + nxa);
            if (prev == cur) {
              p0 = cur;
              break;
            }
            cur = prev;
          }
        }
        p0 = rl(p0, 0);
        if (p0 != kInvalid) {
          uint32_t lb = 0;
          if (gc) lb = atomicAdd(&T.lst[list], gc);
          lb = static_cast<uint32_t>(__shfl(static_cast<int>(lb), static_cast<int>(ldr), 64));
          if ((xmk >> lane) & 1ull) {
            const uint32_t pos = p0 + static_cast<uint32_t>(__popcll(xmk & lbelow));
            T.xs[pos] = x;
            T.xm[pos] = (list << 24) | (lb + rk);
          }
          xmk = 0;
        }
        uint32_t b0 = 0;
        if (gc && xmk) b0 = gadd_r(list == B ? p.ov_cnt : &p.x_cnt[list], gc);
        b0 = static_cast<uint32_t>(__shfl(static_cast<int>(b0), static_cast<int>(ldr), 64));
        if ((xmk >> lane) & 1ull) {
          const uint32_t at = b0 + rk;
          if (at >= (list == B ? p.cap_ov : p.cap_x)) {
            set_err(p, BCSIM_E_OVERFLOW);
          } else {
            uint4* dst = reinterpret_cast<uint4*>(list == B ? p.ov + at : p.xbuf + static_cast<size_t>(list) * p.cap_x + at);
            const uint4* src = reinterpret_cast<const uint4*>(&x);
            gst4(dst, src[0]);
            gst4(dst + 1, src[1]);
          }
        }
      }
    }
    // the row's new state: the exception bits per tile (lane k: tile k), the tiles' flags of the
    // uniform records' bucket, the uniform word (or none: every edge has its own word now)
    if (own_t) {
      if (ring_u) gbl(p.rex)[static_cast<size_t>(g) * nrt + lane] = rexn;
      if ((rtm >> lane) & 1ull) gbl(p.rtile)[kRtPad * ((static_cast<size_t>(bk_u) * p.R + rep) * nrt + lane)] = 1;
    }
  }
  RPH(2);
  if (cbn) {
    atomicAdd(&T.lcnt[cb], cbn);
    atomicMin(&T.lmin[cb], cmn);
  }
  if (nu && lane == 0) {
    atomicAdd(&T.lcnt[bk_u], nu);
    atomicMin(&T.lmin[bk_u], tof_u);
  }
  for (int d = 32; d > 0; d >>= 1) ovmin = min(ovmin, static_cast<long long>(__shfl_xor(ovmin, d, 64)));
  {
    const uint32_t c4[4] = {n_bc ? 0u : st_ops, n_rec, st_ops, st_edges};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t ws = wave_sum(c4[k]);
      if (lane == 0 && ws) atomicAdd(&T.csum[k], ws);
    }
  }
  if (lane == 0 && ovmin != LLONG_MAX) atomicMin(&T.ovmin, ovmin);
  __syncthreads();
  RPH(3);
  // (after the barrier: every wave of the sender has read the old word)
  if (act && part == 0 && lane == 0) gbl(p.rul)[g] = ring_u ? ((1ull << 63) | nw_u) : 0ull;
  // the staged extras / overflow records: one atomic per list
  if (T.xn) {
    for (uint32_t k = tid; k <= B; k += blockDim.x) {
      const uint32_t c = T.lst[k];
      if (!c) continue;
      uint32_t* ctr = k == B ? p.ov_cnt : &p.x_cnt[k];
      const uint32_t cap = k == B ? p.cap_ov : p.cap_x;
      const uint32_t base = gadd_r(ctr, c);
      if (base + c > cap) set_err(p, BCSIM_E_OVERFLOW);
      T.lst[k] = base;
    }
    __syncthreads();
    const uint32_t nx = min(T.xn, kTX);
    for (uint32_t k = tid; k < nx; k += blockDim.x) {
      const uint32_t list = T.xm[k] >> 24, at = T.lst[list] + (T.xm[k] & 0xFFFFFFu);
      const uint4* src = reinterpret_cast<const uint4*>(&T.xs[k]);
      if (at < (list == B ? p.cap_ov : p.cap_x)) {
        uint4* dst = reinterpret_cast<uint4*>(list == B ? p.ov + at : p.xbuf + static_cast<size_t>(list) * p.cap_x + at);
        gst4(dst, src[0]);
        gst4(dst + 1, src[1]);
      }
    }
  }
  // busy buckets and their arrival-time bounds, counters
  for (uint32_t k = tid; k < B; k += blockDim.x)
    if (T.lcnt[k]) {
      gbl(p.bucket_cnt)[k] = 1u;
      const long long t = (cell + static_cast<long long>((k + B - cr_b) % B)) * p.L + T.lmin[k];  // (bucket_t0)
      if (t < T.bmin[k]) __hip_atomic_fetch_min(gbl(p.bmin) + k, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  if (tid == 0) {
    unsigned long long* cnt = cnt_stripe(p, rep);
    unsigned long long* ks = kst_stripe(p);
    if (T.csum[0]) gadd(&cnt[CNT_SENDS], static_cast<unsigned long long>(T.csum[0]));
    if (T.csum[1]) gadd(&ks[KST_REC], static_cast<unsigned long long>(T.csum[1]));
    if (T.csum[2]) gadd(&ks[KST_OPS], static_cast<unsigned long long>(T.csum[2]));
    if (T.csum[3]) gadd(&ks[KST_EDGES], static_cast<unsigned long long>(T.csum[3]));
    if (T.ovmin != LLONG_MAX) __hip_atomic_fetch_min(gbl(p.scal) + 1, T.ovmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  RPH(4);
  RPH(5);
#undef RPH
}

// ---------------------------------------------------------------------------
// k_gossip_link (dense layout, BCSIM_GOSSIP, not the full mesh, fixed app delay, infinite
// queues, one rank, degree <= G): the link stage of a node whose due ops are all broadcasts
// (<= G pending ops), by a group of G lanes, lane j = out-edge j.  Same result as
// link_node: per edge the due broadcasts (key order, sub + j) merged with the implicit
// echo of in-slot j, FIFO busy_until, one record per broadcast into the receiver's
// in-slot (first record of the edge and arrival cell), its extras list or the overflow
// list; then the ordered compaction of the ops not yet due.  Other nodes of the k_link
// The kernel walks all of this rank's gnodes: a node with an echo to send or an op due that
// is not simple is appended to list 3 for k_link<.., LOOP>.
// The dense-gossip link stage of one workgroup's node groups.  scan_left: this lane's node was
// left to the generic k_scan in the same window (fused k_gossip_cell), so its link stage waits
// for the generic k_link after it (list 3).
__device__ __attribute__((always_inline)) inline void gossip_link_body(const KP* __restrict__ pk, long long cell,
                                                                       long long t_lo, long long t_hi, int final_win,
                                                                       uint32_t G, bool scan_left, bool fl) {
  const KP& p = *pk;
  __shared__ RawOp sop[256];  // due broadcasts of each group in key order (group base + rank)
  __shared__ uint32_t s_c[6];  // sends, records, due ops, edges, echoes, kept
  __shared__ uint8_t s_busy[kMaxBuckets];
  __shared__ long long s_bmin[kMaxBuckets];
  const uint32_t tid = tidx(), lane = tid & 63u, j = tid & (G - 1u), gb = lane & ~(G - 1u);
  const uint32_t gbase = tid & ~(G - 1u);
  const uint32_t per_wg = blockDim.x / G;
  const uint32_t B = p.n_buckets;
  if (tid < 6) s_c[tid] = 0;
  for (uint32_t k = tid; k < B; k += blockDim.x) {
    s_busy[k] = 0;
    s_bmin[k] = LLONG_MAX;
  }
  __syncthreads();
  const uint32_t na = fl ? p.act_n[0] : p.R * p.nloc;
  const uint32_t k0 = blockIdx.x * per_wg, kl = k0 + tid / G;
  const uint32_t g0 = k0 < na ? gossip_gnode(p, k0, fl) : 0u;
  const uint32_t g = kl < na ? gossip_gnode(p, kl, fl) : 0u;
  const uint32_t rep = g / p.N, i = g % p.N;
  const uint32_t rep0 = g0 / p.N;
  const uint32_t ib = static_cast<uint32_t>(cell % B);
  // (as in the scan: the loads that depend on g alone at once -- on a regular graph also this
  // lane's edge words and in-slot record, and its op slot, before it is known they are needed)
  // (all of them unconditional, at valid addresses -- g = 0 past the list's end, in-slot and op
  // indices clamped -- and used only under the conditions below)
  const bool kin = kl < na;
  const uint32_t e0r = p.deg_reg ? i * p.deg_reg : 0u;
  const bool pre = p.deg_reg != 0u;
  uint32_t sp_p = 0, slot_p = 0;
  uint64_t lw_p = 0;
  uint4 r0v = make_uint4(0, 0, 0, 0);  // (raw words, as in the scan)
  if (pre) {
    const uint32_t jc = min(j, p.deg_reg - 1u), e = e0r + jc;
    sp_p = AT(p.col, e, p.E);
    slot_p = AT(p.rev, e, p.E);
    lw_p = p.link[link_index(p, rep, i, e0r, jc)];
    if (p.impl) r0v = gld4(p.inbox + inbox_idx(p, ib, rep, e));
  }
  Op* const ops_p = p.ops + op_base(p, g);
  const RawOp o_p = ld_raw(ops_p + min(j, op_cap(p, g) - 1u));
  const uint8_t f8 = AT(p.iflag, static_cast<size_t>(ib) * p.NT + g, static_cast<uint64_t>(B) * p.NT);
  const uint8_t t8 = p.mesh ? AT(p.rtile, kRtPad * ((static_cast<size_t>(ib) * p.R + rep) * p.n_tiles + (i >> 6)), kRtPad * (static_cast<uint64_t>(B) * p.R * p.n_tiles))
                            : static_cast<uint8_t>(0);
  const uint32_t n0l = AT(p.n_ops, g, p.NT);
  const long long onl = AT(p.node_onext, g, p.NT);
  const uint32_t rw0 = pre ? 0u : AT(p.row, i, p.N + 1), rw1 = pre ? 0u : AT(p.row, i + 1, p.N + 1);
  const bool rx = kin && p.impl && (f8 | t8) != 0 && p.bmin[ib] < t_hi;  // (node_flagged_w)
  const uint32_t n0 = kin ? n0l : 0u;
  // nodes link_node would change: an echo to send, or an op due (k_active's rule minus the
  // nodes for which link_node only recomputes an unchanged node_onext)
  const bool have = rx || (n0 && onl < t_hi) || scan_left;
  const uint32_t n = have ? n0 : 0u;
  const uint32_t e0 = !have ? 0u : pre ? e0r : rw0;
  const uint32_t deg = !have ? 0u : pre ? p.deg_reg : rw1 - rw0;
  Op* ops = have ? ops_p : p.ops;
  // this lane's pending op
  RawOp o = raw_zero();
  bool due = false, bc = false, keep = false;
  if (have && n <= G && j < n) {
    o = o_p;
    const uint32_t kind = raw_kind(o);
    due = kind != OP_BCAST_J && raw_t(o) < t_hi;
    bc = due && kind == OP_BCAST;
    keep = !due && (kind != OP_BCAST_J || !(raw_flags(o) & OPF_DONE));
  }
  const unsigned long long gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gb;
  const unsigned long long listed = __ballot(due && !bc) & gmask;
  const bool fast = have && n <= G && deg <= G && listed == 0 && !scan_left;
  if (have && !fast && j == 0) {
    const uint32_t pos = gadd_r(&p.act_n[3], 1u);
    AT(p.act, 3ull * p.NT + pos, 4ull * p.NT) = g;
  }
  // key-order rank of this lane's due broadcast; the group's broadcasts to LDS in that order
  uint32_t rank = 0, nb = 0;
  for (uint32_t q = 0; q < G; ++q) {
    const bool bq = __shfl(bc ? 1 : 0, gb + q, 64) != 0;
    RawOp oq;
    oq.a.x = __shfl(o.a.x, gb + q, 64);
    oq.a.y = __shfl(o.a.y, gb + q, 64);
    oq.a.z = __shfl(o.a.z, gb + q, 64);
    oq.a.w = __shfl(o.a.w, gb + q, 64);
    oq.b.x = __shfl(o.b.x, gb + q, 64);
    if (bq) {
      ++nb;
      if (bc && raw_key_less(oq, raw_sub(oq), o, raw_sub(o))) ++rank;
    }
  }
  if (fast && bc) sop[gbase + rank] = o;
  __syncthreads();
  uint32_t c_rec = 0, c_edges = 0, c_echo = 0;
  if (fast && j < deg && (nb || rx)) {
    const uint32_t e = e0 + j;
    const uint32_t sp = pre ? sp_p : AT(p.col, e, p.E);
    uint64_t* lwp = p.link + link_index(p, rep, i, e0, j);
    uint64_t lw = pre ? lw_p : *lwp;
    bool he = false;
    RawOp eo = raw_zero();
    if (rx) {
      Rec r0;
      if (pre)
        __builtin_memcpy(&r0, &r0v, sizeof r0);
      else
        r0 = ld_rec(p.inbox + inbox_idx(p, ib, rep, e));
      const long long ta0 = cell * p.L + r0.t_off;
      if (slot_live(r0.flags, cell_tag(p, cell)) && ta0 >= t_lo && ta0 < t_hi) {
        if (p.echo) {
          const int bg = (r0.flags & RF_BIG) ? 1 : 0;
          const int64_t pin = p.prop_const >= 0 ? p.prop_const : AT(p.prop_in, e, p.E);
          eo = raw_make(ta0, static_cast<uint32_t>(pin + sel2(p.tx_last, bg)), sp, r0.sub,
                        static_cast<uint8_t>(OP_ECHO | (bg ? (OPF_BIG << 2) : 0)));
          he = true;
          ++c_echo;
        }
      }
    }
    if (nb || he) {
      ++c_edges;
      int64_t bu = static_cast<int64_t>(lw >> 16);
      uint32_t lc = static_cast<uint32_t>(lw & 0xFFFFu);
      const int64_t pr = p.prop_const >= 0 ? p.prop_const : AT(p.prop, e, p.E);
      const uint32_t slot = pre ? slot_p : AT(p.rev, e, p.E);
      const uint32_t dg = rep * p.N + sp;
      uint32_t q = 0;
      for (;;) {
        RawOp x = raw_zero();
        uint32_t sub = 0;
        int src = -1;
        if (q < nb) {
          x = sop[gbase + q];
          sub = raw_sub(x) + j;
          src = 1;
        }
        if (he && (src < 0 || raw_key_less(eo, raw_sub(eo), x, sub))) {
          x = eo;
          sub = raw_sub(eo);
          src = 3;
        }
        if (src < 0) break;
        if (src == 1)
          ++q;
        else
          he = false;
        const int big = (raw_flags(x) & OPF_BIG) ? 1 : 0;
        const int64_t ot = raw_t(x);
        const int64_t start = bu > ot ? bu : ot;
        bu = start + sel2(p.tx_tot, big);
        if (src == 3) continue;  // echo: link occupancy only
        const int64_t ta = bu + pr;
        const long long ca = ta / p.L;
        if (ca - cell < 1) {
          set_err(p, BCSIM_E_TIE);
          continue;
        }
        ++c_rec;
        const uint32_t tof = static_cast<uint32_t>(ta - ca * p.L);
        const uint32_t w3 = (x.b.w & 0x00FFFFFFu) | (static_cast<uint32_t>(RF_VALID | (big ? RF_BIG : 0)) << 24) |
            (emit_tag(cell / p.n_buckets, static_cast<uint32_t>(cell % p.n_buckets), ca - cell, p.n_buckets) << 27);
        XRec xr;
        {
          const uint4 rv = make_uint4(tof, sub, x.b.z, w3);
          __builtin_memcpy(&xr.r, &rv, sizeof xr.r);
        }
        const bool owner = lc != (static_cast<uint32_t>(ca) & 0xFFFFu);
        lc = static_cast<uint32_t>(ca) & 0xFFFFu;
        xr.cell = ca;
        xr.slot = slot;
        xr.g = dg;
        if (ca - cell < static_cast<long long>(B)) {
          const uint32_t bk = static_cast<uint32_t>(ca % B);
          if (owner) {
            st_rec(&AT(p.inbox, inbox_idx(p, bk, rep, slot), p.cap_inbox), xr.r);
          } else {
            const uint32_t pos = gadd_r(&p.x_cnt[bk], 1u);
            if (pos >= p.cap_x)
              set_err(p, BCSIM_E_OVERFLOW);
            else
              AT(p.xbuf, static_cast<size_t>(bk) * p.cap_x + pos, p.cap_xbuf) = xr;
          }
          AT(p.iflag, static_cast<size_t>(bk) * p.NT + dg, static_cast<uint64_t>(B) * p.NT) = 1;
          s_busy[bk] = 1;
          atomicMin(&s_bmin[bk], static_cast<long long>(ta));
        } else {
          if (owner) xr.r.flags = static_cast<uint8_t>(xr.r.flags | RF_OWNER);
          const uint32_t pos = gadd_r(p.ov_cnt, 1u);
          if (pos >= p.cap_ov)
            set_err(p, BCSIM_E_OVERFLOW);
          else
            AT(p.ov, pos, p.cap_ov) = xr;
          gmin(&p.scal[1], static_cast<long long>(ca));
        }
      }
      if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
      *lwp = (static_cast<uint64_t>(bu) << 16) | lc;
    }
  }
  // ordered compaction of the ops not yet due; their earliest time
  const unsigned long long km = __ballot(fast && keep) & gmask;
  long long om = (fast && keep) ? raw_t(o) : LLONG_MAX;
  for (uint32_t off = 1; off < G; off <<= 1) {
    const long long y = __shfl_xor(om, off, 64);
    om = y < om ? y : om;
  }
  if (fast && keep) {
    const uint32_t pos = static_cast<uint32_t>(__popcll(km & ((1ull << lane) - 1ull) & gmask));
    uint4* w = reinterpret_cast<uint4*>(ops + pos);
    w[0] = o.a;
    w[1] = o.b;
  }
  const uint32_t kept = static_cast<uint32_t>(__popcll(km));
  if (fast && j == 0 && (n || rx)) {  // (link_node returns early for a node with neither)
    AT(p.n_ops, g, p.NT) = kept;
    AT(p.node_onext, g, p.NT) = om;
    if (rx && final_win) AT(p.iflag, static_cast<size_t>(ib) * p.NT + g, static_cast<uint64_t>(B) * p.NT) = 0;
  }
  // counters
  {
    const uint32_t v[6] = {fast && j == 0 && rep == rep0 ? nb * deg : 0u, c_rec, fast && j == 0 ? nb : 0u, c_edges,
                           c_echo, fast && j == 0 ? kept : 0u};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const uint32_t ws = wave_sum(v[k]);
      if (lane == 0 && ws) atomicAdd(&s_c[k], ws);
    }
    if (fast && rep != rep0 && j == 0 && nb) atomicAdd(&cnt_stripe(p, rep)[CNT_SENDS], static_cast<unsigned long long>(nb * deg));
  }
  __syncthreads();
  for (uint32_t k = tid; k < B; k += blockDim.x)
    if (s_busy[k]) {
      mark_busy(&p.bucket_cnt[k]);
      bmin_lower(p, k, s_bmin[k]);
    }
  if (tid == 0) {
    // (sends of another replica's node in this workgroup went straight to its stripe)
    unsigned long long* cnt = cnt_stripe(p, rep0);
    if (s_c[0]) atomicAdd(&cnt[CNT_SENDS], static_cast<unsigned long long>(s_c[0]));
    unsigned long long* ks = kst_stripe(p);
    if (s_c[1]) atomicAdd(&ks[KST_REC], static_cast<unsigned long long>(s_c[1]));
    if (s_c[2]) atomicAdd(&ks[KST_OPS], static_cast<unsigned long long>(s_c[2]));
    if (s_c[3]) atomicAdd(&ks[KST_EDGES], static_cast<unsigned long long>(s_c[3]));
    if (s_c[4]) atomicAdd(&ks[KST_ECHO], static_cast<unsigned long long>(s_c[4]));
    if (s_c[5]) atomicAdd(&ks[KST_KEPT], static_cast<unsigned long long>(s_c[5]));
  }
}

__global__ __launch_bounds__(256) void k_gossip_link(const KP* __restrict__ pk, long long cell, long long t_lo,
                                                     long long t_hi, int final_win, uint32_t G) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  gossip_link_body(pk, cell, t_lo, t_hi, final_win, G, false, false);
}

// Dense gossip, one kernel per window: each workgroup scans its node groups and then runs their
// link stage.  A node's link stage needs only the node's own state -- its ops (the ones due now,
// including those its scan just created when the app delay ends inside the window) and its own
// inbox row (implicit echoes) -- and writes only records of later cells and its own out-edges,
// so no other node's scan in this window can affect it.  One launch per window instead of two,
// and the row is read while still in this CU's cache.
// fl: the grid walks the window's frontier list (k_gossip_active) instead of every gnode; the
// workgroups past its end leave at once.
__global__ __launch_bounds__(256) void k_gossip_cell(const KP* __restrict__ pk, long long cell, long long t_lo,
                                                     long long t_hi, long long cs, int x_active, uint32_t G, int loop,
                                                     int final_win, int fl) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  if (cell < 0) {  // (a chained window, or none)
    if (!win_take(p, cell, t_lo, t_hi, final_win)) return;
    cs = cell * p.L;
    x_active = 0;
    loop = static_cast<int>(p.win[kWinLoop]);
    // the frontier list when one was built (by k_gossip_active, -2, or by the closing k_next);
    // after a missed guess (-1, no k_gossip_active in the chain's later windows) every gnode
    fl = p.win[kWinFrCell] != -1 ? 1 : 0;
  }
  if (fl && blockIdx.x * (blockDim.x / G) >= p.act_n[0]) return;
  const bool left = gossip_scan_body(pk, cell, t_lo, t_hi, cs, x_active, G, loop, fl != 0);
  __syncthreads();  // (the node's new ops, n_ops and node_onext: written by one lane of its group)
  gossip_link_body(pk, cell, t_lo, t_hi, final_win, G, left, fl != 0);
}

// k_gossip_active: the window's frontier -- the gnodes k_gossip_cell has anything to do for
// (arrivals in the cell's bucket, a timer or a pending op due before t_hi) -- into list 0,
// workgroup-aggregated: ONE list atomic per 1024 gnodes (a per-wave atomic on the one counter
// serialised in L2: 14 us per launch at 65536 gnodes); any order, each node's work is its own
__global__ __launch_bounds__(1024) void k_gossip_active(const KP* __restrict__ pk, long long cell, long long t_hi) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  if (cell < 0) {  // (a chained window, or none)
    if (!p.win[kWinValid] || p.win[kWinFrCell] >= 0) return;  // (none, or its frontier built by k_next)
    cell = p.win[kWinCell];
    t_hi = p.win[kWinHi];
    if (blockIdx.x == 0 && tidx() == 0) p.win[kWinFrCell] = -2;  // (list 0 built here)
  }
  __shared__ uint32_t wcnt[kMaxWaves], s_base;
  const uint32_t na = p.R * p.nloc, lane = tidx() & 63u, wv = tidx() >> 6;
  const uint32_t k = blockIdx.x * blockDim.x + tidx();
  bool a = false;
  uint32_t g = 0;
  if (k < na) {
    g = gossip_gnode(p, k, false);
    const uint32_t rep = g / p.N, i = g % p.N, b = static_cast<uint32_t>(cell % p.n_buckets);
    // every load issued at once (no short-circuit chain of round trips)
    const bool f = node_flagged_w(p, b, g, rep, i, t_hi);
    const long long tn = AT(p.node_tnext, g, p.NT), on = AT(p.node_onext, g, p.NT);
    const uint32_t no = AT(p.n_ops, g, p.NT);
    a = f | (tn < t_hi) | ((no != 0) & (on < t_hi));
  }
  const unsigned long long m = __ballot(a);
  if (lane == 0) wcnt[wv] = static_cast<uint32_t>(__popcll(m));
  __syncthreads();
  if (tidx() == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < (blockDim.x >> 6); ++w) {
      const uint32_t c = wcnt[w];
      wcnt[w] = t;
      t += c;
    }
    s_base = t ? gadd_r(&p.act_n[0], t) : 0u;
  }
  __syncthreads();
  if (a) AT(p.act, s_base + wcnt[wv] + static_cast<uint32_t>(__popcll(m & ((1ull << lane) - 1ull))), 4ull * p.NT) = g;
}

// ---------------------------------------------------------------------------
// k_link_sparse (sparse mode): the link stage of the window's active
// nodes, a fixed grid striding over the list.  No per-edge arrays in LDS: broadcasts
// are expanded into per-edge SEND ops, the due ops are sorted by (edge, list position)
// in LDS in edge-range batches of at most kDueCap, and one lane walks each edge's run
// in canonical key order (FIFO busy_until, DROPTAIL admission) and stages its records
// for the cell's lists.  Same semantics as link_node (the parity suite runs both).
constexpr uint32_t kDueCap = 1024;

__device__ void link_node_sparse(const KP& p, uint32_t g, long long cell, long long t_lo, long long t_hi,
                                 int final_win) {
  __shared__ LinkShared L;
  __shared__ uint32_t dkey[kDueCap], didx[kDueCap], rst[kDueCap + 1];
  __shared__ uint32_t s_cnt;
  uint32_t n = AT(p.n_ops, g, p.NT);
  if (n == 0) return;
  const uint32_t tid = tidx(), bs = blockDim.x;
  const uint32_t rep = g / p.N, i = g % p.N;
  const uint32_t e0 = AT(p.row, i, p.N + 1), deg = AT(p.row, i + 1, p.N + 1) - e0;
  Op* ops = p.ops + op_base(p, g);
  const uint32_t ocap = op_cap(p, g);
  unsigned long long* cnt = cnt_stripe(p, rep);
  const uint32_t B = p.n_buckets;
  const long long cs = cell * p.L;
  // ---- 0. broadcasts -> per-edge SEND ops (jitter: per-edge draws; fixed: when due) ----
  // The broadcasts to expand are found by a parallel pass over the ops (batches of
  // kBcastCap, in op order) and expanded one after another by the whole workgroup.
  for (;;) {
    if (tid == 0) L.n_bc = 0;
    __syncthreads();
    for (uint32_t k = tid; k < n; k += bs) {
      const Op& o = ops[k];
      const uint8_t kind = op_kind(o);
      if ((kind == OP_BCAST_J && !(op_flags(o) & OPF_DONE)) || (kind == OP_BCAST && o.t < t_hi)) {
        const uint32_t pos = atomicAdd(&L.n_bc, 1u);
        if (pos < kBcastCap) L.bc[pos] = k;
      }
    }
    __syncthreads();
    const uint32_t nfound = L.n_bc, nb = min(nfound, static_cast<uint32_t>(kBcastCap));
    if (nb == 0) break;
    if (n + nb * deg > ocap) {
      if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
      return;
    }
    for (uint32_t b2 = 0; b2 < nb; ++b2) {
      // (raw words: an Op copy, sub-dword members and all, went through scratch per edge)
      const RawOp o = ld_raw(&ops[L.bc[b2]]);
      const bool jit = raw_kind(o) == OP_BCAST_J;
      const bool paxos = (raw_flags(o) & OPF_PAXOS) != 0;
      const uint32_t at = n + b2 * deg;
      const uint32_t w3 = (o.b.w & 0x00FFFFFFu) | (static_cast<uint32_t>(OP_SEND | ((raw_flags(o) & OPF_BIG) << 2)) << 24);
      for (uint32_t it = tid; it < deg; it += bs) {
        int64_t d = 0;
        if (jit) d = delay_from_draw(p, ctr_rand(p.seed, rep, i, static_cast<uint64_t>(o.b.y) + it));
        const uint64_t t = static_cast<uint64_t>(raw_t(o) + d);
        uint4* w = reinterpret_cast<uint4*>(&AT(ops, at + it, ocap));
        w[0] = make_uint4(static_cast<uint32_t>(t), static_cast<uint32_t>(t >> 32), jit ? static_cast<uint32_t>(d) : o.a.z, o.a.w);
        // (Paxos: edge it + 1 -- peers[0] skipped -- and the last one *end())
        w[1] = make_uint4(raw_sub(o) + it, paxos ? (it + 1 < deg ? e0 + it + 1 : kInvalid) : e0 + it, o.b.z, w3);
      }
    }
    __syncthreads();
    for (uint32_t b2 = tid; b2 < nb; b2 += bs)  // consumed
      AT(ops, L.bc[b2], ocap).kind_flags = static_cast<uint8_t>(OP_BCAST_J | (OPF_DONE << 2));
    n += nb * deg;
    __syncthreads();
    if (nfound <= static_cast<uint32_t>(kBcastCap)) break;
  }
  const uint32_t n_lists = B + 1 + (p.nranks > 1 ? p.nranks : 0);
  for (uint32_t k = tid; k < B; k += bs) {
    L.lcnt[k] = 0;
    L.lmin[k] = ~0u;
  }
  for (uint32_t k = tid; k < n_lists; k += bs) L.lst[k] = 0;
  if (tid == 0) {
    L.nst = 0;
    L.omin = LLONG_MAX;
    L.ovmin = LLONG_MAX;
  }
  __syncthreads();
  unsigned long long dropped = 0, sends = 0, n_rec = 0, st_ops = 0, st_edges = 0, st_echo = 0, fdrop = 0, lost = 0;
  long long ovmin = LLONG_MAX;
  // due ops with no route (Paxos *end()): dropped at SendPacket
  for (uint32_t k = tid; k < n; k += bs) {
    const Op& o = ops[k];
    const uint8_t kind = op_kind(o);
    if ((kind == OP_SEND || kind == OP_ECHO) && o.t < t_hi && o.edge == kInvalid) {
      ++dropped;
      ++sends;
      ++st_ops;
    }
  }
  // ---- 1. due ops in edge-range batches of at most kDueCap ----
  uint32_t lo_e = 0;
  while (lo_e < deg) {  // block-uniform
    uint32_t hi_e = deg;
    for (;;) {  // the widest range [lo_e, hi_e) whose due ops fit the batch
      if (tid == 0) s_cnt = 0;
      __syncthreads();
      uint32_t c = 0;
      for (uint32_t k = tid; k < n; k += bs) {
        const Op& o = ops[k];
        const uint8_t kind = op_kind(o);
        if ((kind == OP_SEND || kind == OP_ECHO) && o.t < t_hi && o.edge != kInvalid) {
          const uint32_t le = o.edge - e0;
          c += (le >= lo_e && le < hi_e) ? 1u : 0u;
        }
      }
      if (c) atomicAdd(&s_cnt, c);
      __syncthreads();
      const uint32_t tot = s_cnt;
      __syncthreads();
      if (tot <= kDueCap) break;
      if (hi_e - lo_e <= 1) {  // more due ops on one edge than a batch holds
        if (tid == 0) set_err(p, BCSIM_E_OVERFLOW);
        return;
      }
      hi_e = lo_e + (hi_e - lo_e) / 2;
    }
    // keys: (edge in range) << 13 | list rank, in op-list order (stable)
    uint32_t nd = 0;
    for (uint32_t k0 = 0; k0 < n; k0 += bs) {
      const uint32_t k = k0 + tid;
      bool due = false;
      uint32_t le = 0;
      if (k < n) {
        const Op& o = ops[k];
        const uint8_t kind = op_kind(o);
        if ((kind == OP_SEND || kind == OP_ECHO) && o.t < t_hi && o.edge != kInvalid) {
          le = o.edge - e0;
          due = le >= lo_e && le < hi_e;
        }
      }
      uint32_t tot;
      const uint32_t pos = nd + block_rank(due, L.wcnt, tot);
      if (due) {
        dkey[pos] = ((le - lo_e) << 13) | pos;
        didx[pos] = k;
      }
      nd += tot;
    }
    // bitonic sort of the keys (ranks < 2^13 since nd <= kDueCap)
    uint32_t P2 = 1;
    while (P2 < nd) P2 <<= 1;
    for (uint32_t k = nd + tid; k < P2; k += bs) dkey[k] = ~0u;
    __syncthreads();
    for (uint32_t k2 = 2; k2 <= P2; k2 <<= 1)
      for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
        for (uint32_t t = tid; t < P2 / 2; t += bs) {
          const uint32_t lo = 2 * t - (t & (j - 1)), hi = lo + j;
          const bool up = (lo & k2) == 0;
          const uint32_t a = dkey[lo], b2 = dkey[hi];
          if (up == (b2 < a)) {
            dkey[lo] = b2;
            dkey[hi] = a;
          }
        }
        __syncthreads();
      }
    // runs of equal edge
    uint32_t nr = 0;
    for (uint32_t k0 = 0; k0 < nd; k0 += bs) {
      const uint32_t k = k0 + tid;
      const bool st = k < nd && (k == 0 || (dkey[k] >> 13) != (dkey[k - 1] >> 13));
      uint32_t tot;
      const uint32_t pos = nr + block_rank(st, L.wcnt, tot);
      if (st) rst[pos] = k;
      nr += tot;
    }
    if (tid == 0) rst[nr] = nd;
    __syncthreads();
    // ---- 2. one lane per edge run: key order, FIFO, records ----
    for (uint32_t r = tid; r < nr; r += bs) {
      const uint32_t j0 = rst[r], j1 = rst[r + 1];
      const uint32_t le = lo_e + (dkey[j0] >> 13);
      for (uint32_t a = j0 + 1; a < j1; ++a) {  // insertion sort by the canonical key (short runs)
        const uint32_t ka = dkey[a];
        const RawOp ox = ld_raw(&ops[didx[ka & 0x1FFFu]]);
        uint32_t b2 = a;
        while (b2 > j0) {
          const uint32_t kb = dkey[b2 - 1];
          const RawOp oy = ld_raw(&ops[didx[kb & 0x1FFFu]]);
          if (!raw_key_less(ox, raw_sub(ox), oy, raw_sub(oy))) break;
          dkey[b2] = kb;
          --b2;
        }
        dkey[b2] = ka;
      }
      const uint32_t e = e0 + le;
      const uint32_t sn = p.mesh ? (le < i ? le : le + 1) : AT(p.col, e, p.E);
      uint64_t* lwp = p.link + link_index(p, rep, i, e0, le);
      const uint64_t lw = *lwp;
      int64_t bu = static_cast<int64_t>(lw >> 16);
      uint32_t lc = static_cast<uint32_t>(lw & 0xFFFFu);
      uint64_t qm = 0;
      uint64_t* qr = nullptr;
      const size_t qe = edge_loc(p, rep, e);
      if (p.qmodel) {
        qm = p.qmeta[qe];
        qr = p.qring + qe * p.cap_q;
      }
      const int64_t pr = p.prop_const >= 0 ? p.prop_const : AT(p.prop, e, p.E);
      const uint32_t slot = p.mesh ? sn * (p.N - 1) + (i < sn ? i : i - 1) : AT(p.rev, e, p.E);
      const uint32_t dg = rep * p.N + sn;
      ++st_edges;
      for (uint32_t j = j0; j < j1; ++j) {
        const RawOp o = ld_raw(&ops[didx[dkey[j] & 0x1FFFu]]);
        ++st_ops;
        const uint32_t kind = raw_kind(o);
        if (kind == OP_SEND) ++sends;
        const bool is_echo = kind == OP_ECHO;
        const int big = (raw_flags(o) & OPF_BIG) ? 1 : 0;
        const int64_t ot = raw_t(o);
        const int64_t start = bu > ot ? bu : ot;
        if (p.qmodel) {
          const uint32_t F = sel2(p.nfr, big);
          const uint32_t k = q_admit(p, qr, qm, ot, big, start);
          if (k < F) {
            fdrop += F - k;
            if (k) bu = start + static_cast<int64_t>(k) * sel2(p.tx_full, big);
            if (!is_echo) ++lost;
            continue;
          }
        }
        const int64_t end = start + sel2(p.tx_tot, big);
        bu = end;
        if (is_echo) {
          ++st_echo;
          continue;
        }
        const int64_t ta = end + pr;
        const long long ca = ta / p.L;
        const long long rel = ca - cell;
        if (rel < 1) {
          set_err(p, BCSIM_E_TIE);  // lookahead violated
          continue;
        }
        ++n_rec;
        lc = static_cast<uint32_t>(ca) & 0xFFFFu;
        XRec x;
        {
          const uint32_t w3 = (o.b.w & 0x00FFFFFFu) | (static_cast<uint32_t>(RF_VALID | (big ? RF_BIG : 0)) << 24);
          const uint4 rv = make_uint4(static_cast<uint32_t>(ta - ca * p.L), raw_sub(o), o.b.z, w3);
          __builtin_memcpy(&x.r, &rv, sizeof x.r);
        }
        x.cell = ca;
        x.slot = slot;
        x.g = dg;
        uint32_t orank = p.rank;
        if (p.nranks > 1) orank = p.owner[sn];
        if (orank != p.rank) {
          link_stage(p, L, g, B + 1 + orank, x);  // receiver on another GPU (k_import places it)
        } else if (rel < static_cast<long long>(B)) {
          const uint32_t bk = static_cast<uint32_t>(ca % B);
          link_stage(p, L, g, bk, x);
          set_flag_once(&AT(p.iflag, static_cast<size_t>(bk) * p.NT + dg, static_cast<uint64_t>(B) * p.NT));
          atomicAdd(&L.lcnt[bk], 1u);
          atomicMin(&L.lmin[bk], static_cast<uint32_t>(ta - ca * p.L));
        } else {
          link_stage(p, L, g, B, x);
          if (ca < ovmin) ovmin = ca;
        }
      }
      if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
      *lwp = (static_cast<uint64_t>(bu) << 16) | lc;
      if (p.qmodel) p.qmeta[qe] = qm;
    }
    __syncthreads();
    lo_e = hi_e;
  }
  // ---- 3. keep the ops that are not due (in order) ----
  long long omin = LLONG_MAX;
  uint32_t kept = 0;
  for (uint32_t k0 = 0; k0 < n; k0 += bs) {
    const uint32_t k = k0 + tid;
    RawOp o = raw_zero();  // (raw words: an Op copy went through scratch per op)
    bool keep = false;
    if (k < n) {
      o = ld_raw(&ops[k]);
      const uint32_t kind = raw_kind(o);
      const int64_t ot = raw_t(o);
      if (kind == OP_BCAST_J)
        keep = !(raw_flags(o) & OPF_DONE);
      else if (ot >= t_hi) {
        keep = true;
        if (ot < omin) omin = ot;
      }
    }
    uint32_t tot;
    const uint32_t pos = kept + block_rank(keep, L.wcnt, tot);
    if (keep) {
      uint4* w = reinterpret_cast<uint4*>(&ops[pos]);
      w[0] = o.a;
      w[1] = o.b;
    }
    kept += tot;
  }
  if (tid == 0) L.n_keep = kept;
  if (omin != LLONG_MAX) atomicMin(&L.omin, omin);
  if (ovmin != LLONG_MAX) atomicMin(&L.ovmin, ovmin);
  // ---- 4. flush the staged records: one global atomic per list ----
  for (uint32_t k = tid; k < n_lists; k += bs) {
    const uint32_t c = L.lst[k];
    if (!c) continue;
    uint32_t* ctr = k < B ? &p.x_cnt[k] : k == B ? p.ov_cnt : &p.send_cnt[k - B - 1];
    const uint32_t cap = k < B ? p.cap_x : k == B ? p.cap_ov : p.cap_send;
    const uint32_t base = atomicAdd(ctr, c);
    if (base + c > cap) set_err(p, BCSIM_E_OVERFLOW);
    L.lbase[k] = base;
  }
  __syncthreads();
  const uint32_t nst = min(L.nst, p.cap_stage);
  long long xmin = LLONG_MAX;  // earliest arrival cell shipped to another rank (scal[4])
  for (uint32_t k = tid; k < nst; k += bs) {
    const size_t sidx = static_cast<size_t>(blockIdx.x) * p.cap_stage + k;
    const uint32_t meta = p.xmeta[sidx], list = meta >> 24;
    const uint32_t pos = L.lbase[list] + (meta & 0xFFFFFFu);
    if (list > B) {
      const XRec x = p.xstage[sidx];
      xmin = min(xmin, static_cast<long long>(static_cast<uint64_t>(x.cell) & ((1ull << 48) - 1)));
      if (pos < p.cap_send) p.sendbuf[static_cast<size_t>(list - B - 1) * p.cap_send + pos] = x;
    } else if (list == B) {
      if (pos < p.cap_ov) p.ov[pos] = p.xstage[sidx];
    } else if (pos < p.cap_x) {
      p.xbuf[static_cast<size_t>(list) * p.cap_x + pos] = p.xstage[sidx];
    }
  }
  if (xmin != LLONG_MAX) gmin(&p.scal[4], xmin);
  // ---- 5. counters ----
  uint4 t1, t2;
  (void)block_scan4(make_uint4(static_cast<uint32_t>(dropped), static_cast<uint32_t>(sends),
                               static_cast<uint32_t>(n_rec), static_cast<uint32_t>(st_ops)), L.wsum, t1);
  (void)block_scan4(make_uint4(static_cast<uint32_t>(st_edges), static_cast<uint32_t>(st_echo),
                               static_cast<uint32_t>(fdrop), static_cast<uint32_t>(lost)), L.wsum, t2);
  if (tid == 0) {
    if (t1.x) atomicAdd(&cnt[CNT_DROPPED], static_cast<unsigned long long>(t1.x));
    if (t1.y) atomicAdd(&cnt[CNT_SENDS], static_cast<unsigned long long>(t1.y));
    if (t1.z) atomicAdd(&kst_stripe(p)[KST_REC], static_cast<unsigned long long>(t1.z));
    if (t1.w) atomicAdd(&kst_stripe(p)[KST_OPS], static_cast<unsigned long long>(t1.w));
    if (t2.x) atomicAdd(&kst_stripe(p)[KST_EDGES], static_cast<unsigned long long>(t2.x));
    if (t2.y) atomicAdd(&kst_stripe(p)[KST_ECHO], static_cast<unsigned long long>(t2.y));
    if (t2.z) atomicAdd(&cnt[CNT_FDROP], static_cast<unsigned long long>(t2.z));
    if (t2.w) atomicAdd(&cnt[CNT_LOST], static_cast<unsigned long long>(t2.w));
  }
  __syncthreads();
  for (uint32_t k = tid; k < B; k += bs)
    if (L.lcnt[k]) {
      mark_busy(&p.bucket_cnt[k]);
      bmin_lower(p, k, bucket_t0(p, (t_hi - 1) / p.L, k) + L.lmin[k]);
    }
  if (tid == 0) {
    if (L.ovmin != LLONG_MAX) gmin(&p.scal[1], L.ovmin);
    AT(p.n_ops, g, p.NT) = L.n_keep;
    AT(p.node_onext, g, p.NT) = L.omin;
    atomicAdd(&kst_stripe(p)[KST_KEPT], static_cast<unsigned long long>(L.n_keep));
  }
  (void)final_win;
  (void)cs;
}

// list 1: the window's k_link list; list 3: the nodes k_paxos_link left over
__global__ __launch_bounds__(256) void k_link_sparse(const KP* __restrict__ pk, long long cell, long long t_lo,
                                                     long long t_hi, int final_win, int list) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  const uint32_t li = list == 3 ? 3u : 1u;
  for (ListRange lr = list_range(p.act_n[li]); lr.k < lr.end; lr.k += lr.step) {
    link_node_sparse(p, p.act[li * p.NT + lr.k], cell, t_lo, t_hi, final_win);
    __syncthreads();
  }
}

// k_paxos_link (sparse layout, BCSIM_PAXOS, infinite queues): one LANE per node of the
// k_link list whose pending ops (<= kPxCap) are all unicasts / echoes on real edges -- the
// acceptors.  Same result as link_node_sparse: the due ops in (edge, canonical key) order
// through each edge's FIFO, one list record per SEND (staged per workgroup, one global
// atomic per list and batch), the ops not yet due compacted in order.  Other nodes go to
// list 3 for k_link_sparse.  256 lanes per workgroup; the lane's ops live in registers (the
// selection and compaction loops are unrolled over kPxCap), so the workgroup's LDS is the
// list staging alone (~0.5 KB) and occupancy is set by VGPRs.
struct PxLinkShared {
  uint32_t lcnt[kMaxBuckets];
  uint32_t lmin[kMaxBuckets];
  uint32_t nst;
  uint32_t lst[kMaxBuckets + 1];  // per list (bucket extras..., overflow)
  uint32_t lbase[kMaxBuckets + 1];
  long long ovmin;
  uint32_t c[5];  // records, due ops, edges, echoes, kept
  uint32_t rp[256 * kPxCap];  // (list << 24 | rank) of each lane's records, in walk order (CAP <= kPxCap)
};
constexpr uint32_t kPxLinkThreads = 256;
// CAP: the most pending ops a lane holds in registers (nodes with more go to list 3); 8 by
// default, 4 with BCSIM_PX_CAP=4 (fewer registers: more waves in flight on the latency-bound walk)
template <int CAP>
__global__ __launch_bounds__(kPxLinkThreads) void k_paxos_link(const KP* __restrict__ pk, long long cell, long long t_lo,
                                                               long long t_hi) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ PxLinkShared L;
  const uint32_t tid = tidx(), bs = blockDim.x;
  const uint32_t na = p.act_n[1];
  const uint32_t B = p.n_buckets;
  const uint32_t n_lists = B + 1;
  for (uint32_t base = blockIdx.x * bs; base < na; base += gridDim.x * bs) {  // workgroup-uniform
    for (uint32_t k = tid; k < B; k += bs) {
      L.lcnt[k] = 0;
      L.lmin[k] = ~0u;
    }
    for (uint32_t k = tid; k < n_lists; k += bs) L.lst[k] = 0;
    if (tid < 5) L.c[tid] = 0;
    if (tid == 0) {
      L.nst = 0;
      L.ovmin = LLONG_MAX;
    }
    __syncthreads();
    const uint32_t kl = base + tid;
    const uint32_t g = kl < na ? p.act[p.NT + kl] : 0u;
    const uint32_t n = kl < na ? AT(p.n_ops, g, p.NT) : 0u;
    bool fast = kl < na && n <= static_cast<uint32_t>(CAP);
    Op* ops = p.ops + (kl < na ? op_base(p, g) : 0);
    // the ops, all loads in flight at once; bit c of due: op c is due
    RawOp o[CAP];
#pragma unroll
    for (int c = 0; c < CAP; ++c) o[c] = (fast && static_cast<uint32_t>(c) < n) ? ld_raw(ops + c) : raw_zero();
    uint32_t due = 0;
#pragma unroll
    for (int c = 0; c < CAP; ++c) {
      if (static_cast<uint32_t>(c) >= n) continue;
      const uint32_t kind = raw_kind(o[c]);
      if ((kind != OP_SEND && kind != OP_ECHO) || o[c].b.y == kInvalid) fast = false;
      if (raw_t(o[c]) < t_hi) due |= 1u << c;
    }
    if (kl < na && !fast) {
      const uint32_t pos = gadd_r(&p.act_n[3], 1u);
      AT(p.act, 3ull * p.NT + pos, 4ull * p.NT) = g;
    }
    uint32_t c_rec = 0, c_ops = 0, c_edges = 0, c_echo = 0, c_sends = 0;
    long long ovmin = LLONG_MAX;
    // The due ops in (edge, key) order through each edge's FIFO, twice: pass 0 counts each record
    // into its list (an LDS rank, kept in L.rp) and reads the link words only; after one global
    // atomic per list, pass 1 repeats the identical walk and writes every record straight to its
    // list position and the link words back -- no per-workgroup staging copy of the records.
    auto walk = [&](const int pass) {
      if (!(fast && due)) return;
      const uint32_t rep = g / p.N, i = g % p.N;
      const uint32_t e0 = AT(p.row, i, p.N + 1);
      uint32_t left = due, ri = 0;
      uint32_t cur_e = kInvalid;
      uint64_t* lwp = nullptr;
      int64_t bu = 0;
      uint32_t lc = 0, slot = 0, dg = 0;
      int64_t pr = 0;
      while (left) {
        // next due op in (edge, key) order: a scan over the register-resident ops
        RawOp ob = raw_zero();
        uint32_t best = kInvalid;
#pragma unroll
        for (int c = 0; c < CAP; ++c) {
          const bool cand = (left >> c) & 1u;
          const bool take = cand && (best == kInvalid || o[c].b.y < ob.b.y ||
                                     (o[c].b.y == ob.b.y && raw_key_less(o[c], raw_sub(o[c]), ob, raw_sub(ob))));
          raw_sel(ob, o[c], take);
          best = take ? static_cast<uint32_t>(c) : best;
        }
        left &= ~(1u << best);
        const uint32_t e = ob.b.y;
        if (e != cur_e) {  // a new edge: store the previous one's link word (pass 1), load this one's
          if (lwp && pass) {
            if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
            *lwp = (static_cast<uint64_t>(bu) << 16) | lc;
          }
          cur_e = e;
          const uint32_t le = e - e0;
          lwp = p.link + link_index(p, rep, i, e0, le);
          const uint64_t lw = *lwp;
          bu = static_cast<int64_t>(lw >> 16);
          lc = static_cast<uint32_t>(lw & 0xFFFFu);
          const uint32_t sn = p.mesh ? (le < i ? le : le + 1) : AT(p.col, e, p.E);
          slot = p.mesh ? sn * (p.N - 1) + (i < sn ? i : i - 1) : AT(p.rev, e, p.E);
          dg = rep * p.N + sn;
          pr = p.prop_const >= 0 ? p.prop_const : AT(p.prop, e, p.E);
          if (!pass) ++c_edges;
        }
        const uint32_t kind = raw_kind(ob);
        if (!pass) {
          ++c_ops;
          if (kind == OP_SEND) ++c_sends;
        }
        const int big = (raw_flags(ob) & OPF_BIG) ? 1 : 0;
        const int64_t ot = raw_t(ob);
        const int64_t start = bu > ot ? bu : ot;
        bu = start + sel2(p.tx_tot, big);
        if (kind == OP_ECHO) {
          if (!pass) ++c_echo;
          continue;
        }
        const int64_t ta = bu + pr;
        const long long ca = ta / p.L;
        const long long rel = ca - cell;
        if (rel < 1) {
          if (!pass) set_err(p, BCSIM_E_TIE);
          continue;
        }
        lc = static_cast<uint32_t>(ca) & 0xFFFFu;
        const uint32_t list = rel < static_cast<long long>(B) ? static_cast<uint32_t>(ca % B) : B;
        const uint32_t rs = tid * CAP + ri++;
        if (!pass) {
          ++c_rec;
          L.rp[rs] = (list << 24) | atomicAdd(&L.lst[list], 1u);
          if (list < B) {
            atomicAdd(&L.lcnt[list], 1u);
            atomicMin(&L.lmin[list], static_cast<uint32_t>(ta - ca * p.L));
          } else if (ca < ovmin) {
            ovmin = ca;
          }
          continue;
        }
        XRec x;
        {
          const uint32_t w3 = (ob.b.w & 0x00FFFFFFu) | (static_cast<uint32_t>(RF_VALID | (big ? RF_BIG : 0)) << 24);
          const uint4 rv = make_uint4(static_cast<uint32_t>(ta - ca * p.L), raw_sub(ob), ob.b.z, w3);
          __builtin_memcpy(&x.r, &rv, sizeof x.r);
        }
        x.cell = ca;
        x.slot = slot;
        x.g = dg;
        const uint32_t pos = L.lbase[list] + (L.rp[rs] & 0xFFFFFFu);
        if (list == B) {
          if (pos < p.cap_ov) p.ov[pos] = x;
        } else {
          if (pos < p.cap_x) p.xbuf[static_cast<size_t>(list) * p.cap_x + pos] = x;
          set_flag_once(&AT(p.iflag, static_cast<size_t>(list) * p.NT + dg, static_cast<uint64_t>(B) * p.NT));
        }
      }
      if (lwp && pass) {
        if (bu >= (1ll << 47)) set_err(p, BCSIM_E_OVERFLOW);
        *lwp = (static_cast<uint64_t>(bu) << 16) | lc;
      }
    };
    walk(0);
    if (fast && (due || n)) {  // ordered compaction of the ops not yet due
      uint32_t kept = 0;
      long long omin = LLONG_MAX;
#pragma unroll
      for (int c = 0; c < CAP; ++c) {
        if (static_cast<uint32_t>(c) >= n || ((due >> c) & 1u)) continue;
        if (raw_t(o[c]) < omin) omin = raw_t(o[c]);
        uint4* w = reinterpret_cast<uint4*>(ops + kept);
        w[0] = o[c].a;
        w[1] = o[c].b;
        ++kept;
      }
      AT(p.n_ops, g, p.NT) = kept;
      AT(p.node_onext, g, p.NT) = omin;
      atomicAdd(&L.c[4], kept);
    }
    wave_cnt_add(p, g / p.N, c_sends, CNT_SENDS);
    if (c_rec) atomicAdd(&L.c[0], c_rec);
    if (c_ops) atomicAdd(&L.c[1], c_ops);
    if (c_edges) atomicAdd(&L.c[2], c_edges);
    if (c_echo) atomicAdd(&L.c[3], c_echo);
    if (ovmin != LLONG_MAX) atomicMin(&L.ovmin, ovmin);
    __syncthreads();
    // flush the staged records: one global atomic per list
    for (uint32_t k = tid; k < n_lists; k += bs) {
      const uint32_t c = L.lst[k];
      if (!c) continue;
      uint32_t* ctr = k < B ? &p.x_cnt[k] : p.ov_cnt;
      const uint32_t cap = k < B ? p.cap_x : p.cap_ov;
      const uint32_t b0 = atomicAdd(ctr, c);
      if (b0 + c > cap) set_err(p, BCSIM_E_OVERFLOW);
      L.lbase[k] = b0;
    }
    __syncthreads();
    walk(1);
    for (uint32_t k = tid; k < B; k += bs)
      if (L.lcnt[k]) {
        mark_busy(&p.bucket_cnt[k]);
        bmin_lower(p, k, bucket_t0(p, (t_hi - 1) / p.L, k) + L.lmin[k]);
      }
    if (tid == 0) {
      if (L.ovmin != LLONG_MAX) gmin(&p.scal[1], L.ovmin);
      unsigned long long* ks = kst_stripe(p);
      if (L.c[0]) atomicAdd(&ks[KST_REC], static_cast<unsigned long long>(L.c[0]));
      if (L.c[1]) atomicAdd(&ks[KST_OPS], static_cast<unsigned long long>(L.c[1]));
      if (L.c[2]) atomicAdd(&ks[KST_EDGES], static_cast<unsigned long long>(L.c[2]));
      if (L.c[3]) atomicAdd(&ks[KST_ECHO], static_cast<unsigned long long>(L.c[3]));
      if (L.c[4]) atomicAdd(&ks[KST_KEPT], static_cast<unsigned long long>(L.c[4]));
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_active (sparse mode): the gnodes of this rank that have work in [t_lo, t_hi) --
// k_scan: arrivals in the bucket, a due timer, START / STOP; k_link: those plus the
// nodes with an op due -- as two compact lists (one returning atomic per wave; the
// loop bound is wave-uniform, so every ballot runs with the whole wave active)
constexpr uint32_t kActChunk = 16384;  // k_active: gnodes per workgroup at most (LDS flags)
__global__ __launch_bounds__(256) void k_active(const KP* __restrict__ pk, long long t_lo, long long t_hi, uint32_t b,
                                                uint32_t obp, uint32_t chunk, uint32_t seq, int spec) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  if (spec) {  // (speculative, behind k_next: the window it predicted, or nothing)
    if (!p.pred[0]) return;
    const long long c = p.pred[1];
    t_lo = p.pred[2];
    t_hi = p.pred[3];
    b = static_cast<uint32_t>(c % p.n_buckets);
    obp = static_cast<uint32_t>((c + kOpRing - 1) % kOpRing);
  }
  // each workgroup compacts a contiguous chunk of gnodes: flags to LDS and counts, ONE global
  // atomic per list for the chunk (a per-wave atomic on the two list counters serialised:
  // 1.5 ms per launch at 8 M gnodes), then the ordered writes
  __shared__ uint8_t fl[kActChunk];
  __shared__ uint32_t s_n[2], s_base[2], wcnt[kMaxWaves];
  const bool has_start = (t_lo <= 0 && 0 < t_hi);
  const bool has_stop = (p.stop_ns >= 0 && t_lo <= p.stop_ns && p.stop_ns < t_hi);
  const uint32_t tid = tidx();
  const uint64_t n_loc = static_cast<uint64_t>(p.R) * p.nloc;
  const uint64_t c0 = static_cast<uint64_t>(blockIdx.x) * chunk;
  // the last workgroup to take its list positions publishes the lengths to the host-mapped
  // mirror (the host's read-back is then a sync, no copy)
  auto publish = [&]() {
    if (!p.act_mirror) return;
    __threadfence();
    if (gadd_r(p.act_done, 1u) == gridDim.x - 1) {
      __threadfence();
      p.act_mirror[0] = __hip_atomic_load(&p.act_n[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      p.act_mirror[1] = __hip_atomic_load(&p.act_n[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.act_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(p.act_mirror + 2, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // (host spins on it)
    }
  };
  if (c0 >= n_loc) {  // uniform
    if (tidx() == 0) publish();
    return;
  }
  const uint32_t cn = static_cast<uint32_t>(min(static_cast<uint64_t>(chunk), n_loc - c0));
  if (tid < 2) s_n[tid] = 0;
  __syncthreads();
  uint32_t ns = 0, nl = 0;
  const long long bm = p.bmin[b];
  uint8_t* const sfa = p.eslot ? p.sflag : reinterpret_cast<uint8_t*>(p.act_n);  // (a dummy word without slots)
  // (gnode numbers are < 2^32: 32-bit index arithmetic; the words of kActU nodes per lane all
  // loaded before any is used -- one round trip per kActU nodes, not per node)
  constexpr uint32_t kActU = 4;
  for (uint32_t j0 = tid; j0 < cn; j0 += kActU * blockDim.x) {
    uint8_t f8[kActU], t8[kActU], sfb[kActU];
    long long tn[kActU], on[kActU];
#pragma unroll
    for (uint32_t u = 0; u < kActU; ++u) {
      const uint32_t j = j0 + u * blockDim.x;
      const uint32_t k = static_cast<uint32_t>(c0 + (j < cn ? j : 0u));
      const uint32_t g = (k / p.nloc) * p.N + p.nlo + k % p.nloc;
      const uint32_t rep = g / p.N, i = g % p.N;
      f8[u] = AT(p.iflag, static_cast<size_t>(b) * p.NT + g, static_cast<uint64_t>(p.n_buckets) * p.NT);
      t8[u] = p.mesh ? AT(p.rtile, kRtPad * ((static_cast<size_t>(b) * p.R + rep) * p.n_tiles + (i >> 6)), kRtPad * (static_cast<uint64_t>(p.n_buckets) * p.R * p.n_tiles))
                     : static_cast<uint8_t>(0);
      tn[u] = AT(p.node_tnext, g, p.NT);
      on[u] = AT(p.node_onext, g, p.NT);
      sfb[u] = gbl(sfa)[p.eslot ? static_cast<size_t>(obp) * p.NT + g : 0u];
    }
#pragma unroll
    for (uint32_t u = 0; u < kActU; ++u) {
      const uint32_t j = j0 + u * blockDim.x;
      if (j >= cn) continue;
      const bool sc = has_start || has_stop || ((f8[u] | t8[u]) != 0 && bm < t_hi) || tn[u] < t_hi;  // (node_flagged_w)
      // k_link also runs nodes with reply-slot ops of the previous arrival cell due
      const bool lk = sc || on[u] < t_hi || (p.eslot && (sfb[u] & (2u | kSfD1)));
      fl[j] = static_cast<uint8_t>((sc ? 1u : 0u) | (lk ? 2u : 0u));
      ns += sc ? 1u : 0u;
      nl += lk ? 1u : 0u;
    }
  }
  ns = wave_sum(ns);
  nl = wave_sum(nl);
  if ((tid & 63u) == 0) {
    if (ns) atomicAdd(&s_n[0], ns);
    if (nl) atomicAdd(&s_n[1], nl);
  }
  __syncthreads();
  if (tid == 0) {
    s_base[0] = s_n[0] ? gadd_r(&p.act_n[0], s_n[0]) : 0u;
    s_base[1] = s_n[1] ? gadd_r(&p.act_n[1], s_n[1]) : 0u;
    publish();
  }
  __syncthreads();
  uint32_t ps = s_base[0], pl = s_base[1];
  for (uint32_t j0 = 0; j0 < cn; j0 += blockDim.x) {  // uniform
    const uint32_t j = j0 + tid;
    const uint32_t f = j < cn ? fl[j] : 0u;
    const uint32_t k = static_cast<uint32_t>(c0 + j);
    const uint32_t g = j < cn ? (k / p.nloc) * p.N + p.nlo + k % p.nloc : 0u;
    uint32_t ts, tl;
    const uint32_t rs = block_rank((f & 1u) != 0, wcnt, ts);
    if (f & 1u) p.act[ps + rs] = g;
    const uint32_t rl = block_rank((f & 2u) != 0, wcnt, tl);
    if (f & 2u) p.act[p.NT + pl + rl] = g;
    ps += ts;
    pl += tl;
  }
}

// ---------------------------------------------------------------------------
// place one received record (the rules of a local emission)
__device__ inline void import_one(const KP& p, long long g_cur, XRec x, uint32_t* lb, long long* lbm, long long& ovmin) {
  const uint32_t B = p.n_buckets;
  const uint32_t rep = x.g / p.N;
  if (x.cell < g_cur + static_cast<long long>(B)) {
    const uint32_t b = static_cast<uint32_t>(x.cell % B);
    const bool owner = (x.r.flags & RF_OWNER) != 0;
    x.r.flags = static_cast<uint8_t>((x.r.flags & (RF_VALID | RF_BIG)) | (cell_tag(p, x.cell) << 3));
    if (owner) {
      st_rec(&AT(p.inbox, inbox_idx(p, b, rep, x.slot), p.cap_inbox), x.r);
    } else {
      const uint32_t pos = gadd_r(&p.x_cnt[b], 1u);
      if (pos < p.cap_x)
        AT(p.xbuf, static_cast<size_t>(b) * p.cap_x + pos, p.cap_xbuf) = x;
      else
        set_err(p, BCSIM_E_OVERFLOW);
    }
    set_flag_once(&AT(p.iflag, static_cast<size_t>(b) * p.NT + x.g, static_cast<uint64_t>(B) * p.NT));
    atomicMin(&lbm[b], x.cell * p.L + static_cast<long long>(x.r.t_off));  // (flushed per workgroup)
    atomicAdd(&lb[b], 1u);
  } else {
    const uint32_t pos = gadd_r(p.ov_cnt, 1u);
    if (pos < p.cap_ov)
      AT(p.ov, pos, p.cap_ov) = x;
    else
      set_err(p, BCSIM_E_OVERFLOW);
    ovmin = min(ovmin, static_cast<long long>(x.cell));
  }
}

// k_import (multi-GPU): place the records received from other ranks -- the same rules as a
// local k_link emission (slot owner -> inbox, second record of an edge -> extras, beyond the
// ring -> overflow); a range record (xr_ship) is expanded here into its per-edge records
// (receiver s, its in-slot and sub + k follow from the sender and the first receiver).
// g_cur = the cell just processed.
// k_fq_init: every edge's FQCODEL header -- flows empty, rec_inv_sqrt = ~0U >> REC_INV_SQRT_SHIFT,
// queue-disc classes not created yet -- and no first-send keys pending
__global__ __launch_bounds__(256) void k_fq_init(uint32_t* __restrict__ h, uint4* __restrict__ key, uint64_t ne) {
  const uint64_t nw = ne * kFqH;
  for (uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + tidx(); k < nw;
       k += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t w = static_cast<uint32_t>(k % kFqH);
    uint32_t v = 0;
    if (w < 3 * kFqF && w % kFqF == FQ_REC) v = 0xFFFFu;
    if (w < 3 * kFqF && w % kFqF == FQ_CR) v = kInvalid;
    h[k] = v;
    if (w == 0) key[k / kFqH] = make_uint4(~0u, ~0u, ~0u, ~0u);
  }
}

// k_l2_take (list-2 overlap of a few-node scan window, PBFT full mesh): the window's scan list
// (the leader's cells: a handful of nodes) becomes list 2 -- scanned and linked on the second
// stream -- and its nodes are stamped so that the other nodes' link stage skips them
__global__ __launch_bounds__(256) void k_l2_take(const KP* __restrict__ pk, uint32_t wep) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  const uint32_t n = p.act_n[0];
  for (uint32_t k = blockIdx.x * blockDim.x + tidx(); k < n; k += gridDim.x * blockDim.x) {
    const uint32_t g = AT(p.act, k, 4ull * p.NT);
    AT(p.act, 2ull * p.NT + k, 4ull * p.NT) = g;
    AT(p.l2mark, g, p.NT) = wep;
  }
  if (blockIdx.x == 0 && tidx() == 0) p.act_n[2] = n;
}

__global__ __launch_bounds__(256) void k_import(const KP* __restrict__ pk, long long g_cur, const XRec* __restrict__ rx,
                                                uint32_t n) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  __shared__ uint32_t lb[kMaxBuckets];
  __shared__ long long lbm[kMaxBuckets];
  __shared__ long long ovmin_s;
  const uint32_t B = p.n_buckets;
  for (uint32_t k = tidx(); k < B; k += blockDim.x) {
    lb[k] = 0;
    lbm[k] = LLONG_MAX;
  }
  if (tidx() == 0) ovmin_s = LLONG_MAX;
  __syncthreads();
  const uint32_t k = blockIdx.x * blockDim.x + tidx();
  long long ovmin = LLONG_MAX;
  if (k < n) {
    XRec x = rx[k];
    const uint64_t cw = static_cast<uint64_t>(x.cell);
    if (cw & kXRange) {
      const uint32_t cnt = static_cast<uint32_t>((cw >> kXCountShift) & 0x3FFFu);
      const uint32_t i = x.slot, rep = x.g / p.N, s0 = x.g % p.N, N1 = p.N - 1;
      if (!p.mesh || i >= p.N || s0 == i) {
        set_err(p, BCSIM_E_STATE);
      } else {
        const uint32_t le0 = s0 < i ? s0 : s0 - 1, sub0 = x.r.sub;
        x.cell = static_cast<long long>(cw & kXCellMask);
        for (uint32_t j = 0; j < cnt; ++j) {
          const uint32_t le = le0 + j, s = le < i ? le : le + 1;
          XRec y = x;
          y.r.sub = sub0 + j;
          y.slot = s * N1 + (i < s ? i : i - 1);
          y.g = rep * p.N + s;
          import_one(p, g_cur, y, lb, lbm, ovmin);
        }
      }
    } else {
      if (p.qmodel == 2) {  // FQCODEL: the sender's client port, for this receiver's echo class
        const uint32_t po = static_cast<uint32_t>((cw >> kXPortShift) & 0x3FFFu);
        if (po) p.fqpeer[edge_loc(p, x.g / p.N, x.slot)] = 49152u + po;
        x.cell = static_cast<long long>(cw & ((1ull << kXPortShift) - 1));
      }
      import_one(p, g_cur, x, lb, lbm, ovmin);
    }
  }
  if (ovmin != LLONG_MAX) atomicMin(&ovmin_s, ovmin);
  __syncthreads();
  for (uint32_t q = tidx(); q < B; q += blockDim.x)
    if (lb[q]) {
      bmin_lower(p, q, lbm[q]);
      mark_busy(&p.bucket_cnt[q]);
    }
  if (tidx() == 0 && ovmin_s != LLONG_MAX) gmin(&p.scal[1], ovmin_s);
}

// k_lead (multi-GPU, PBFT): this rank's "ticking leader" flags for k_pbft_tick
__global__ __launch_bounds__(1024) void k_lead(const KP* __restrict__ pk) {
  const KP& p = *pk;
  const uint32_t rep = blockIdx.x;
  for (uint32_t k = tidx(); k < p.nloc; k += blockDim.x) {
    const uint32_t i = p.nlo + k, g = rep * p.N + i;
    p.lead_loc[g] = (p.tick_alive[g] && p.leader[g] == static_cast<int32_t>(i)) ? 1 : 0;
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
  __shared__ unsigned long long lmask[64];  // leader flags of the current 4096-node chunk, one bit per node
  const uint32_t rep = blockIdx.x, tid = tidx();
  if (rep == 0 && tid < 4) p.act_n[tid] = 0;  // the second window of the cell builds fresh lists
  const uint32_t N = p.N;
  const long long ts_tick = tk - p.pbft_period;
  // v = latest v-log write before this tick in canonical order: every thread
  // keeps the latest of a strided share of the log (each VIEW_CHANGE delivery
  // writes one entry, N-1 per view change), then a block tree-reduction
  __shared__ uint32_t vbest[1024];
  {
    auto later = [](const VLog& a, const VLog& b) {  // key(a) > key(b)
      if (a.t != b.t) return a.t > b.t;
      if (a.ts != b.ts) return a.ts > b.ts;
      if (a.origin != b.origin) return a.origin > b.origin;
      if (a.sub != b.sub) return a.sub > b.sub;
      return a.target > b.target;
    };
    const uint32_t nv = min(*p.vlog_cnt, p.cap_vlog);
    uint32_t mine = UINT32_MAX;
    for (uint32_t k = tid; k < nv; k += blockDim.x) {
      const VLog& e = AT(p.vlog, k, p.cap_vlog);
      if (e.rep != rep) continue;
      if (!(e.t < tk || (e.t == tk && e.ts < ts_tick))) continue;  // before the tick key (tk, ts_tick, ...)
      if (mine == UINT32_MAX || later(e, AT(p.vlog, mine, p.cap_vlog))) mine = k;
    }
    vbest[tid] = mine;
    __syncthreads();
    for (uint32_t off = blockDim.x >> 1; off > 0; off >>= 1) {
      if (tid < off) {
        const uint32_t a = vbest[tid], b = vbest[tid + off];
        if (b != UINT32_MAX && (a == UINT32_MAX || later(AT(p.vlog, b, p.cap_vlog), AT(p.vlog, a, p.cap_vlog))))
          vbest[tid] = b;
      }
      __syncthreads();
    }
  }
  if (tid == 0) {
    v_cur = vbest[0] == UINT32_MAX ? 1 : AT(p.vlog, vbest[0], p.cap_vlog).v;
    nround0 = AT(p.g_nround, rep, p.R);
    n_alive = 0;
    n_ticked = 0;
  }
  __syncthreads();
  if (p.nranks > 1) {
    for (uint32_t i = tid; i < N; i += blockDim.x) lead[i] = p.lead_all[rep * N + i];
  } else {
    // four nodes per lane, both words of each loaded before any is used (a short-circuit
    // `alive && leader == i` was two round trips per node)
    for (uint32_t i0 = 0; i0 < N; i0 += 4u * blockDim.x) {
      uint8_t ta[4];
      int32_t ld[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t g = rep * N + min(i0 + u * blockDim.x + tid, N - 1u);
        ta[u] = AT(p.tick_alive, g, p.NT);
        ld[u] = AT(p.leader, g, p.NT);
      }
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t i = i0 + u * blockDim.x + tid;
        if (i < N) lead[i] = (ta[u] && ld[u] == static_cast<int32_t>(i)) ? 1 : 0;
      }
    }
  }
  __syncthreads();
  // leaders, serially in node order (rare: normally exactly one); a wave
  // ballot packs 64 flags per word so thread 0 visits set bits only
  int32_t nround = nround0;
  for (uint32_t cb = 0; cb < N; cb += 4096) {
    for (uint32_t j = tid; j < 4096; j += blockDim.x) {
      const unsigned long long m = __ballot(cb + j < N && lead[cb + j]);
      if ((j & 63) == 0) lmask[j >> 6] = m;
    }
    __syncthreads();
    if (tid == 0) {
      for (uint32_t w = 0; w < 64; ++w)
        for (unsigned long long mw = lmask[w]; mw; mw &= mw - 1) {
          const uint32_t i = cb + 64 * w + static_cast<uint32_t>(__builtin_ctzll(mw));
          const uint32_t g = rep * N + i;
          if (i < p.nlo || i >= p.nlo + p.nloc) {
            // another rank's leader: advance the replicated file-scope globals
            // (n_round, n, glibc stream position, v) exactly as its owner does
            ++nround;
            AT(p.g_n, rep, p.R) = AT(p.g_n, rep, p.R) + 1;
            if (p.pbft_view_change && p.rng_mode == BCSIM_RNG_GLIBC) {
              const uint32_t pos = AT(p.glibc_pos, rep, p.R)++;
              const int32_t r = AT(p.glibc, static_cast<size_t>(rep) * p.glibc_len + (pos % p.glibc_len), p.cap_glibc);
              if (r % 100 == 5) v_cur += 1;
            }
            continue;
          }
          // (every word the leader's tick reads, loaded before its first store: the trace record's
          // atomic and stores made the compiler issue each later load as its own round trip)
          uint32_t sub = AT(p.sub, g, p.NT);
          const uint32_t deg = AT(p.row, i + 1, p.N + 1) - AT(p.row, i, p.N + 1);
          const int32_t n_seq = AT(p.g_n, rep, p.R);
          const uint32_t tsub = AT(p.tick_sub, g, p.NT);
          uint32_t nops = AT(p.n_ops, g, p.NT);
          uint64_t draws = AT(p.draws, g, p.NT);
          const int32_t ldr = AT(p.leader, g, p.NT);
          const uint32_t gpos = AT(p.glibc_pos, rep, p.R);
          const int32_t gr = (p.pbft_view_change && p.rng_mode == BCSIM_RNG_GLIBC)
                                 ? AT(p.glibc, static_cast<size_t>(rep) * p.glibc_len + (gpos % p.glibc_len), p.cap_glibc)
                                 : 0;
          const Key tkey{tk, ts_tick, i, tsub};
          emit_trace(p, tkey, rep, i, BCSIM_TR_PBFT_BLOCK, n_seq, v_cur, 0);  // :387 leader log
          // block = generateTX header '1', v, n, n (:79-95)
          Msg blk = mkmsg(PB_PRE_PREPARE, enc_raw(p, v_cur), enc_raw(p, n_seq), enc_raw(p, n_seq), 1);
          Op* ops = p.ops + op_base(p, g);
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
              if (gpos >= p.glibc_len) set_err(p, BCSIM_E_OVERFLOW);
              AT(p.glibc_pos, rep, p.R) = gpos + 1;
              r = gr;
            } else {
              r = ctr_rand(p.seed, rep, i, draws++);
            }
            if (r % 100 == 5) {  // viewChange :293-303
              const int32_t nl = (ldr + 1) % static_cast<int32_t>(N);
              AT(p.leader, g, p.NT) = nl;
              v_cur += 1;
              emit_vlog(p, tkey, rep, i, v_cur);
              push_bcast(mkmsg(PB_VIEW_CHANGE, enc_raw(p, v_cur), enc_raw(p, nl), 0, 0));
            }
          }
          AT(p.sub, g, p.NT) = sub;
          AT(p.n_ops, g, p.NT) = nops;
          AT(p.draws, g, p.NT) = draws;
          AT(p.node_onext, g, p.NT) = LLONG_MIN;
        }
    }
    __syncthreads();
  }
  if (tid == 0) AT(p.g_nround, rep, p.R) = nround;
  __syncthreads();
  // every alive node: n_round seen = n_round0 + #leaders with id <= i
  // (prefix over the leader flags), reschedule, stop check.
  __shared__ int32_t chunk_base;
  __shared__ int32_t sc[1024];
  if (N <= 4096u) {
    // (one chunk: the leader bits of lmask, a prefix of their popcounts per word, and each lane's
    // nodes with all their words loaded at once -- no scan barriers between dependent loads)
    if (tid < 64) {
      const int32_t c = __popcll(lmask[tid]);
      int32_t x = c;
      for (int off = 1; off < 64; off <<= 1) {
        const int32_t y = __shfl_up(x, off, 64);
        if (tid >= static_cast<uint32_t>(off)) x += y;
      }
      sc[tid] = x - c;
    }
    __syncthreads();
    uint8_t al[4];
    uint32_t fs[4], ss[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      const uint32_t g = rep * N + min(u * blockDim.x + tid, N - 1u);
      al[u] = AT(p.tick_alive, g, p.NT);
      fs[u] = AT(p.tick_sub, g, p.NT);
      ss[u] = AT(p.sub, g, p.NT);
    }
    int32_t na = 0, nt = 0;
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      const uint32_t i = u * blockDim.x + tid;
      if (i >= N || i < p.nlo || i >= p.nlo + p.nloc || !al[u]) continue;
      const uint32_t g = rep * N + i;
      const int32_t nr = nround0 + sc[i >> 6] + __popcll(lmask[i >> 6] & (~0ull >> (63u - (i & 63u))));
      AT(p.tick_sub, g, p.NT) = ss[u];  // blockEvent = Schedule(Seconds(timeout), SendBlock) :406
      AT(p.sub, g, p.NT) = ss[u] + 1;
      ++nt;
      if (nr == static_cast<int32_t>(p.pbft_rounds)) {  // :407-410
        emit_trace(p, Key{tk, ts_tick, i, fs[u]}, rep, i, BCSIM_TR_PBFT_STOP, nr, 0, 0);
        AT(p.tick_alive, g, p.NT) = 0;
      } else {
        ++na;
      }
    }
    na = static_cast<int32_t>(wave_sum(static_cast<uint32_t>(na)));
    nt = static_cast<int32_t>(wave_sum(static_cast<uint32_t>(nt)));
    if ((tid & 63u) == 0) {
      if (na) atomicAdd(&n_alive, na);
      if (nt) atomicAdd(&n_ticked, nt);
    }
    __syncthreads();
  }
  if (tid == 0) chunk_base = 0;
  __syncthreads();
  for (uint32_t base = 0; N > 4096u && base < N; base += blockDim.x) {
    const uint32_t i = base + tid;
    const uint32_t f = (i < N) ? lead[i] : 0u;
    sc[tid] = static_cast<int32_t>(f);
    __syncthreads();
    for (uint32_t off = 1; off < blockDim.x; off <<= 1) {
      const int32_t y = tid >= off ? sc[tid - off] : 0;
      __syncthreads();
      sc[tid] += y;
      __syncthreads();
    }
    if (i < N && i >= p.nlo && i < p.nlo + p.nloc) {
      const uint32_t g = rep * N + i;
      if (AT(p.tick_alive, g, p.NT)) {
        const int32_t nr = nround0 + chunk_base + sc[tid];
        const uint32_t fired = AT(p.tick_sub, g, p.NT);  // sub of the executing SendBlock
        const uint32_t s = AT(p.sub, g, p.NT);
        AT(p.tick_sub, g, p.NT) = s;  // blockEvent = Schedule(Seconds(timeout), SendBlock) :406
        AT(p.sub, g, p.NT) = s + 1;
        atomicAdd(&n_ticked, 1);
        if (nr == static_cast<int32_t>(p.pbft_rounds)) {  // :407-410
          emit_trace(p, Key{tk, ts_tick, i, fired}, rep, i, BCSIM_TR_PBFT_STOP, nr, 0, 0);
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
      unsigned long long* cnt = cnt_stripe(p, rep);
      atomicAdd(&cnt[CNT_EVENTS], static_cast<unsigned long long>(n_ticked));
      atomicMax(reinterpret_cast<long long*>(&cnt[CNT_TLAST]), tk);
    }
  }
}

// ---------------------------------------------------------------------------
// glibc election-timeout draws (Raft), canonical global order per replica.
__global__ void k_draws(const KP* __restrict__ pk, uint32_t) {
  const KP& p = *pk;
  if (tidx() != 0 || blockIdx.x != 0) return;
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

// Zero n16 16-byte words (an inbox bucket for the ring-turn tag invariant): dwordx4 stores,
// a grid-stride loop over a few thousand workgroups
// k_ctl (node-partitioned over RCCL): this rank's control words of the window's
// exchange, from the control block after k_next -- per peer {segment bytes (1 << 62: this rank
// failed), next-cell candidate, earliest cell shipped, PBFT nodes alive at a tick} -- the same
// words the host computes on the other path (bcsim_capi.hip exchange / local_next_cell: ch holds
// its host-only terms, START / STOP and a partly processed cell)
__global__ void k_ctl(const KP* __restrict__ pk, int64_t* __restrict__ w, uint32_t P, long long ch, long long t_done,
                      int tick, int lrc) {
  const KP& p = *pk;
  if (tidx() != 0) return;
  bool fail = lrc != 0 || *reinterpret_cast<volatile G<int32_t>*>(gbl(p.err)) != 0;
  for (uint32_t r = 0; r < P; ++r)
    if (p.send_cnt[r] > p.cap_send) fail = true;
  long long c = ch;
  const uint32_t B = p.n_buckets;
  const long long cdone = t_done / p.L;
  for (uint32_t b = 0; b < B; ++b)
    if (p.bucket_cnt[b]) {
      const long long cb = cdone + ((static_cast<long long>(b) - cdone % B) % B + B) % B;
      c = cb < c ? cb : c;
    }
  const long long nl = p.scal[0], ov = p.scal[1];
  if (nl != LLONG_MAX) {
    const long long x = (nl > t_done ? nl : t_done) / p.L;
    c = x < c ? x : c;
  }
  if (ov != LLONG_MAX) c = ov < c ? ov : c;
  const long long xmin = fail ? LLONG_MAX : p.scal[4];
  const long long alive = (tick && !fail) ? p.scal[2] : 0;
  for (uint32_t r = 0; r < P; ++r) {
    w[4 * r] = fail ? static_cast<long long>(1ull << 62) : static_cast<long long>(p.send_cnt[r]) * static_cast<long long>(sizeof(XRec));
    w[4 * r + 1] = fail ? LLONG_MAX : c;
    w[4 * r + 2] = xmin;
    w[4 * r + 3] = alive;
  }
}

// test hook (BCSIM_DBG_DEV_ERR): raise a device error flag, as an overflow found by a kernel
// would, so that the next kernels bail and the host's read-back takes its fallback path
__global__ void k_dbg_err(const KP* __restrict__ pk) {
  if (tidx() == 0) set_err(*pk, BCSIM_E_OVERFLOW);
}

__global__ __launch_bounds__(256) void k_zero16(uint4* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k < n16; k += stride)
    dst[k] = make_uint4(0, 0, 0, 0);
}

// global min over node_tnext / node_onext
// next event time over all nodes: every workgroup reduces a strided share, the last one to
// finish (threadfence reduction) combines the partial minima
// k_next also ends the cell: the next window's active lists start empty, and a finished
// cell's bucket (clr_b < n_buckets) is free again (its counts and receiver-tile flags).
// one wave: the control words to the host-mapped mirror, with the window's next event times
// (scal[0] = words 6-7, scal[3] = words 12-13 of the control block)
// then the window's sequence number in the word after them, which the host spins on
// (the prediction's four words follow scal[6]: words 18-25)
__device__ inline void ctl_publish(const KP& p, long long s0, long long s3, uint32_t seq, const long long* pv) {
  if (!p.ctl_mirror || !seq) return;  // (seq 0: a chained window's k_next before the chain's last)
  const uint32_t lane = tidx() & 63u;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(p.err);
  for (uint32_t k = lane; k < p.ctl_words; k += 64) {
    uint32_t v = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == 6 || k == 7) v = static_cast<uint32_t>(static_cast<uint64_t>(s0) >> (32 * (k - 6)));
    if (k == 12 || k == 13) v = static_cast<uint32_t>(static_cast<uint64_t>(s3) >> (32 * (k - 12)));
    if (pv && k >= 18 && k < 26) v = static_cast<uint32_t>(static_cast<uint64_t>(pv[(k - 18) >> 1]) >> (32 * ((k - 18) & 1)));
    p.ctl_mirror[k] = v;
  }
  __threadfence_system();  // (the wave's stores done before the sequence word)
  if (lane == 0) __hip_atomic_store(p.ctl_mirror + p.ctl_words, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The host's next-window rule (bcsim_capi.hip run() / local_next_cell / group_cell), restated for
// k_next's prediction: its host-only terms come in PredArgs (t_done after the window, the run
// limit, the next PBFT tick, the candidate of a part cell / STOP).  A window is predicted only
// when the host would run k_active for it with nothing launched in between: no tick inside it,
// no START / STOP, no extras to group or overflow to rebin for its cell.
struct PredArgs {
  long long t_done, lim, tick, ch, stop_ns;
  int on;
};
// the earliest cell held by a busy bucket, seen from cell cdone (local_next_cell's bucket term) --
// one bucket per lane and a wave minimum (B <= 64; the whole wave calls it): a serial loop over the
// buckets was one dependent load round trip each
__device__ inline long long bucket_min_cell(const KP& p, long long cdone) {
  const uint32_t B = p.n_buckets, lane = tidx() & 63u;
  long long cb = LLONG_MAX;
  if (lane < B && p.bucket_cnt[lane])
    cb = cdone + ((static_cast<long long>(lane) - cdone % B) % B + B) % B;
  for (int d = 32; d > 0; d >>= 1) {
    const long long y = __shfl_xor(cb, d, 64);
    cb = y < cb ? y : cb;
  }
  return cb;
}
__device__ inline void predict_window(const KP& p, const PredArgs& a, long long next_local, long long* pv) {
  pv[0] = 0;
  pv[1] = pv[2] = pv[3] = 0;
  if (!a.on) return;
  const uint32_t B = p.n_buckets;
  const long long L = p.L, cdone = a.t_done / L;
  long long c = min(a.ch, bucket_min_cell(p, cdone));
  if (next_local != LLONG_MAX) {
    const long long x = (next_local > a.t_done ? next_local : a.t_done) / L;
    c = x < c ? x : c;
  }
  const long long ov = p.scal[1];
  if (ov != LLONG_MAX) c = ov < c ? ov : c;
  if (a.tick != LLONG_MAX) c = a.tick / L < c ? a.tick / L : c;
  if (c == LLONG_MAX || c * L >= a.lim) return;
  const long long cs = c * L, lo = cs > a.t_done ? cs : a.t_done, hi = cs + L < a.lim ? cs + L : a.lim;
  if (lo >= hi) return;
  if (a.tick >= lo && a.tick < hi) return;                       // (the tick splits it)
  if (lo <= 0 && 0 < hi) return;                                 // START
  if (a.stop_ns >= 0 && lo <= a.stop_ns && a.stop_ns < hi) return;  // STOP
  if (p.x_cnt[c % B]) return;                                    // extras to group
  if (ov != LLONG_MAX && ov <= c + static_cast<long long>(B) - 1) return;  // overflow to rebin
  if (c - cdone >= static_cast<long long>(B)) return;
  pv[0] = 1;
  pv[1] = c;
  pv[2] = lo;
  pv[3] = hi;
}

// k_active's rule for k_next's predicted window, in k_next's one workgroup (N <= 4096, the
// speculative path): the lists k_active(spec = 1) would build after k_next, without its launch.
// n_loc <= 4 * blockDim.x; the words of a lane's four gnodes are loaded before any is used, the
// lists are compacted in ascending gnode order (block ranks) like k_active's.
__device__ inline void next_active(const KP& p, const long long* pv, uint32_t act_seq) {
  const uint32_t tid = tidx();
  const uint64_t n_loc = static_cast<uint64_t>(p.R) * p.nloc;
  const long long c = pv[1], t_hi = pv[3];
  const uint32_t b = static_cast<uint32_t>(c % p.n_buckets), obp = static_cast<uint32_t>((c + kOpRing - 1) % kOpRing);
  const long long bm = p.bmin[b];
  uint8_t* const sfa = p.eslot ? p.sflag : reinterpret_cast<uint8_t*>(p.act_n);  // (a dummy word without slots)
  __shared__ uint32_t wcnt[kMaxWaves];
  constexpr uint32_t kU = 4;
  uint32_t fl[kU];
  uint8_t f8[kU], t8[kU], sfb[kU];
  long long tn[kU], on[kU];
#pragma unroll
  for (uint32_t u = 0; u < kU; ++u) {
    const uint32_t j = tid + u * blockDim.x;
    const uint32_t k = j < n_loc ? j : 0u;
    const uint32_t g = (k / p.nloc) * p.N + p.nlo + k % p.nloc;
    const uint32_t rep = g / p.N, i = g % p.N;
    f8[u] = AT(p.iflag, static_cast<size_t>(b) * p.NT + g, static_cast<uint64_t>(p.n_buckets) * p.NT);
    t8[u] = p.mesh ? AT(p.rtile, kRtPad * ((static_cast<size_t>(b) * p.R + rep) * p.n_tiles + (i >> 6)), kRtPad * (static_cast<uint64_t>(p.n_buckets) * p.R * p.n_tiles))
                   : static_cast<uint8_t>(0);
    tn[u] = AT(p.node_tnext, g, p.NT);
    on[u] = AT(p.node_onext, g, p.NT);
    sfb[u] = gbl(sfa)[p.eslot ? static_cast<size_t>(obp) * p.NT + g : 0u];
  }
#pragma unroll
  for (uint32_t u = 0; u < kU; ++u) {
    const uint32_t j = tid + u * blockDim.x;
    // (a predicted window holds neither START nor STOP)
    const bool sc = j < n_loc && (((f8[u] | t8[u]) != 0 && bm < t_hi) || tn[u] < t_hi);  // (node_flagged_w)
    const bool lk = j < n_loc && (sc || on[u] < t_hi || (p.eslot && (sfb[u] & (2u | kSfD1))));
    fl[u] = (sc ? 1u : 0u) | (lk ? 2u : 0u);
  }
  uint32_t ps = 0, pl = 0;
#pragma unroll
  for (uint32_t u = 0; u < kU; ++u) {  // (uniform: every lane runs every block rank)
    const uint32_t j = tid + u * blockDim.x;
    const uint32_t g = j < n_loc ? (j / p.nloc) * p.N + p.nlo + j % p.nloc : 0u;
    uint32_t ts, tl;
    const uint32_t rs = block_rank((fl[u] & 1u) != 0, wcnt, ts);
    if (fl[u] & 1u) p.act[ps + rs] = g;
    const uint32_t rl = block_rank((fl[u] & 2u) != 0, wcnt, tl);
    if (fl[u] & 2u) p.act[p.NT + pl + rl] = g;
    ps += ts;
    pl += tl;
  }
  if (tid == 0) {
    p.act_n[0] = ps;
    p.act_n[1] = pl;
    if (p.act_mirror) {
      p.act_mirror[0] = ps;
      p.act_mirror[1] = pl;
      __threadfence_system();
      __hip_atomic_store(p.act_mirror + 2, act_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // (host spins on it)
    }
  }
}

// A chained window is over (k_next's publishing lane, before the control block goes out): the
// host's end-of-window bookkeeping (run(): t_done, last_full, grouped_cell, cells) on the device.
constexpr uint32_t kClrWin = 0xFFFFFFFEu;  // k_next's clr_b for a chained window: from the win words
__device__ inline void win_advance(const KP& p) {
  if (!p.win[kWinValid]) return;
  const long long c = p.win[kWinCell];
  p.win[kWinTDone] = p.win[kWinHi];
  p.win[kWinCount] += 1;
  if (p.win[kWinFw]) {
    p.win[kWinLastFull] = c;
    p.win[kWinGrouped] = -1;
  } else {
    p.win[kWinGrouped] = c;  // (a part cell, cut by the run limit)
  }
  p.win[kWinValid] = 0;
  __threadfence();
}
// (kWinFrCell / kWinFrHi: the window whose frontier the closing k_next built into list 0 -- the
// guess cell + 1 -- or -1; k_gossip_active skips a window whose frontier is ready, and a guess
// that missed empties the list for it)

// The next window of a device chain -- run()'s rule (local_next_cell and the cell bounds) on the
// control block as k_next left it -- or the end of the chain when the window needs the host:
// START / STOP, extras to group, overflow to rebin, a bucket due for the ring-tag zeroing, a
// pending part cell, the run limit, a device error.  Called by a whole wave (the bucket term is one
// bucket per lane); lane 0 writes the win words.
__device__ inline void win_decide(const KP& p) {
  long long* const w = p.win;
  const bool dead0 = w[kWinDead] != 0;
  const long long td = w[kWinTDone];
  const long long bc = bucket_min_cell(p, td / p.L);  // (uniform: every lane)
  if ((tidx() & 63u) != 0 || dead0) return;
  const long long B = p.n_buckets, L = p.L, lf = w[kWinLastFull], lim = w[kWinLim], stop_ns = w[kWinStop];
  int dead = 0;
  long long c = LLONG_MAX, lo = 0, hi = 0, ce = 0;
  const long long ov = p.scal[1];
  if (*p.err) {
    dead = 1;
  } else if (w[kWinGrouped] >= 0) {
    dead = 2;
  } else {
    c = bc;
    const long long nl = p.scal[0];
    if (nl != LLONG_MAX) c = min(c, (nl > td ? nl : td) / L);
    if (ov != LLONG_MAX) c = min(c, ov);
    if (stop_ns >= 0 && stop_ns >= td) c = min(c, stop_ns / L);
    if (c == LLONG_MAX || c * L >= lim) {
      dead = 3;
    } else {
      const long long cs = c * L;
      ce = cs + L;
      lo = cs > td ? cs : td;
      hi = ce < lim ? ce : lim;
      // the first cell after last_full that ends a 32-turn ring period (zero_tag_buckets)
      const long long t0 = (lf + 1) / B;
      const long long z = (t0 % 32 == 31) ? lf + 1 : ((t0 / 32) * 32 + 31) * B;
      if (lo >= hi) dead = 4;
      else if (p.x_cnt[c % B]) dead = 5;
      else if (ov != LLONG_MAX && ov <= c + B - 1) dead = 6;
      else if (lo <= 0 && 0 < hi) dead = 7;
      else if (stop_ns >= 0 && lo <= stop_ns && stop_ns < hi) dead = 8;
      else if (c >= z) dead = 9;
      // (a timer due: the generic scan too, launched by the host only at the chain positions where
      // it expects one -- anywhere else the window is the host's)
      else if (p.scal[3] < hi && !((static_cast<unsigned long long>(w[kWinLoopMask]) >> min(w[kWinCount], 63ll)) & 1ull))
        dead = 10;
    }
  }
  const bool fr_hit = !dead && w[kWinFrCell] == c && w[kWinFrHi] == hi;
  if (fr_hit) w[kWinFrHits] += 1;
  if (!fr_hit && w[kWinFrCell] >= 0) {
    p.act_n[0] = 0;  // (the speculative frontier was for another window: k_gossip_active builds it)
    w[kWinFrCell] = -1;
  }
  if (dead) {
    w[kWinDead] = dead;
    w[kWinValid] = 0;
    __threadfence();
    return;
  }
  w[kWinCell] = c;
  w[kWinLo] = lo;
  w[kWinHi] = hi;
  w[kWinFw] = hi == ce ? 1 : 0;
  w[kWinLoop] = p.scal[3] < hi ? 1 : 0;
  __threadfence();
  w[kWinValid] = 1;
  __threadfence();
}

// k_win (one wave): a device chain's first window from the host's state (t_done, last_full, the
// run limit, the pending STOP time or -1); every later window is decided by the k_next that ends
// the one before it (k_next: win_advance, then win_decide).
__global__ __launch_bounds__(64) void k_win(const KP* __restrict__ pk, long long t_done, long long last_full, long long lim,
                                            long long stop_ns, unsigned long long loop_mask) {
  const KP& p = *pk;
  long long* const w = p.win;
  if (tidx() == 0) {
    w[kWinLoopMask] = static_cast<long long>(loop_mask);
    w[kWinFrCell] = -1;
    w[kWinFrHits] = 0;
    w[kWinTDone] = t_done;
    w[kWinLastFull] = last_full;
    w[kWinGrouped] = -1;
    w[kWinCount] = 0;
    w[kWinDead] = 0;
    w[kWinLim] = lim;
    w[kWinStop] = stop_ns;
    w[kWinValid] = 0;
    __threadfence();
  }
  __builtin_amdgcn_wave_barrier();
  win_decide(p);
}

// act_seq != 0 (one workgroup, speculation on): the predicted window's active lists too
// (next_active), published before the control block.  clr_b == kClrWin: a chained window's
// (its finished bucket from the win words; its bookkeeping by the publishing lane)
__global__ __launch_bounds__(1024) void k_next(const KP* __restrict__ pk, uint32_t clr_b, uint32_t seq, PredArgs pa,
                                               uint32_t act_seq) {
  const KP& p = *pk;
  BAIL_IF_ERR();
  const bool chained = clr_b == kClrWin;
  // a chained window being closed: the frontier of the guessed next window (cell + 1, up to the
  // run limit) into list 0 -- k_gossip_active's rule on the node state this window left; list 0's
  // count was reset by the window's k_link (after k_gossip_cell read it)
  // (not by the chain's last k_next -- seq != 0, it publishes to the host: the host's own window
  // that may follow builds list 0 from an empty count)
  const bool frs = chained && p.win[kWinValid] != 0 && seq == 0;  // (chains run dense gossip only)
  long long fr_c = -1, fr_hi = 0;
  if (chained) {
    const long long c0 = p.win[kWinCell];
    clr_b = p.win[kWinValid] && p.win[kWinFw] ? static_cast<uint32_t>(c0 % p.n_buckets) : 0xFFFFFFFFu;
    fr_c = c0 + 1;
    fr_hi = min((c0 + 2) * p.L, p.win[kWinLim]);
  }
  long long fm = LLONG_MAX, fmt = LLONG_MAX;  // (with the frontier pass: its next-event minima too)
  if (frs) {
    __shared__ uint32_t fwc[kMaxWaves], fbase;
    const uint32_t fb = static_cast<uint32_t>(fr_c % p.n_buckets), lane = tidx() & 63u, wv = tidx() >> 6;
    for (uint32_t k0 = blockIdx.x * blockDim.x; k0 < p.NT; k0 += gridDim.x * blockDim.x) {  // (uniform)
      const uint32_t g = k0 + tidx();
      bool a = false;
      if (g < p.NT) {  // (one rank: gnode = list index)
        const bool f = node_flagged_w(p, fb, g, g / p.N, g % p.N, fr_hi);
        const long long tn = AT(p.node_tnext, g, p.NT), on = AT(p.node_onext, g, p.NT);
        const uint32_t no = AT(p.n_ops, g, p.NT);
        a = f | (tn < fr_hi) | ((no != 0) & (on < fr_hi));
        fm = min(fm, min(tn, on));
        fmt = min(fmt, tn);
      }
      const unsigned long long mk = __ballot(a);
      if (lane == 0) fwc[wv] = static_cast<uint32_t>(__popcll(mk));
      __syncthreads();
      if (tidx() == 0) {
        uint32_t t = 0;
        for (uint32_t q = 0; q < (blockDim.x >> 6); ++q) {
          const uint32_t c = fwc[q];
          fwc[q] = t;
          t += c;
        }
        fbase = t ? gadd_r(&p.act_n[0], t) : 0u;
      }
      __syncthreads();
      if (a) AT(p.act, fbase + fwc[wv] + static_cast<uint32_t>(__popcll(mk & ((1ull << lane) - 1ull))), 4ull * p.NT) = g;
      __syncthreads();
    }
  }
  if (blockIdx.x == 0) {
    if (tidx() < 4 && !(frs && tidx() == 0)) p.act_n[tidx()] = 0;
    if (clr_b < p.n_buckets) {
      if (tidx() == 0) {
        p.bucket_cnt[clr_b] = 0;
        p.x_cnt[clr_b] = 0;
        p.bmin[clr_b] = LLONG_MAX;
      }
    }
  }
  // (the finished bucket's receiver-tile flags: one padded line each, cleared by every
  // workgroup -- 10,000 replicas x 64 tiles was ~0.4 ms for workgroup 0 alone)
  if (clr_b < p.n_buckets && p.mesh)
    for (uint32_t k = blockIdx.x * blockDim.x + tidx(); k < p.R * p.n_tiles; k += gridDim.x * blockDim.x)
      p.rtile[kRtPad * (static_cast<size_t>(clr_b) * p.R * p.n_tiles + k)] = 0;
  // scal[0] = the next event time (timers and pending ops), scal[3] = the next timer alone;
  // wave minima by shuffles, one LDS slot per wave, one barrier
  __shared__ long long red[kMaxWaves], redt[kMaxWaves];
  long long m = fm, mt = fmt;
  const uint32_t nb = gridDim.x, stride = nb * blockDim.x;
  // (the frontier pass covered every gnode of this workgroup's share: no second pass)
  uint32_t k = frs ? p.NT : blockIdx.x * blockDim.x + tidx();
  // four gnodes per lane per step, their eight loads issued before any is used (PBFT n=4096:
  // one workgroup, no cross-workgroup combine)
  for (; k + 3u * stride < p.NT; k += 4u * stride) {
    long long a[4], bb[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      a[u] = AT(p.node_tnext, k + u * stride, p.NT);
      bb[u] = AT(p.node_onext, k + u * stride, p.NT);
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      m = min(m, min(a[u], bb[u]));
      mt = min(mt, a[u]);
    }
  }
  for (; k < p.NT; k += stride) {
    const long long a = AT(p.node_tnext, k, p.NT), b = AT(p.node_onext, k, p.NT);
    m = min(m, min(a, b));
    mt = min(mt, a);
  }
  for (int d = 32; d > 0; d >>= 1) {
    m = min(m, static_cast<long long>(__shfl_xor(m, d, 64)));
    mt = min(mt, static_cast<long long>(__shfl_xor(mt, d, 64)));
  }
  const uint32_t lane = tidx() & 63u, wv = tidx() >> 6, nwv = blockDim.x >> 6;
  if (lane == 0) {
    red[wv] = m;
    redt[wv] = mt;
  }
  __syncthreads();
  if (nb == 1 && act_seq) {  // (uniform) every wave stays for the active lists
    __shared__ long long s_pv[4];
    m = lane < nwv ? red[lane] : LLONG_MAX;
    mt = lane < nwv ? redt[lane] : LLONG_MAX;
    for (int d = 32; d > 0; d >>= 1) {
      m = min(m, static_cast<long long>(__shfl_xor(m, d, 64)));
      mt = min(mt, static_cast<long long>(__shfl_xor(mt, d, 64)));
    }
    long long pv[4];
    if (wv == 0) {
      predict_window(p, pa, m, pv);
      if (lane == 0) {
        p.scal[0] = m;
        p.scal[3] = mt;
        for (int k = 0; k < 4; ++k) {
          p.pred[k] = pv[k];
          s_pv[k] = pv[k];
        }
      }
      // (the control block first: the host's end-of-window work overlaps the list building, as
      // it overlapped a k_active launch after k_next)
      ctl_publish(p, m, mt, seq, pv);
    }
    __syncthreads();
    for (int k = 0; k < 4; ++k) pv[k] = s_pv[k];
    if (pv[0]) next_active(p, pv, act_seq);  // (uniform)
    return;
  }
  if (wv != 0) return;
  m = lane < nwv ? red[lane] : LLONG_MAX;
  mt = lane < nwv ? redt[lane] : LLONG_MAX;
  for (int d = 32; d > 0; d >>= 1) {
    m = min(m, static_cast<long long>(__shfl_xor(m, d, 64)));
    mt = min(mt, static_cast<long long>(__shfl_xor(mt, d, 64)));
  }
  if (nb == 1) {
    long long pv[4];
    predict_window(p, pa, m, pv);
    if (lane == 0) {
      p.scal[0] = m;
      p.scal[3] = mt;
      for (int k = 0; k < 4; ++k) p.pred[k] = pv[k];
      if (chained) {
        win_advance(p);
        p.win[kWinFrCell] = frs ? fr_c : -1;
        p.win[kWinFrHi] = fr_hi;
      }
    }
    if (chained) win_decide(p);  // (the whole wave: the chain's next window)
    ctl_publish(p, m, mt, seq, pv);
    return;
  }
  bool last = false;
  if (lane == 0) {
    __hip_atomic_store(&p.nxt_part[blockIdx.x], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&p.nxt_part[kNextBlocks + blockIdx.x], mt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    last = gadd_r(p.nxt_done, 1u) == nb - 1;
  }
  if (!__shfl(static_cast<int>(last), 0, 64)) return;
  __threadfence();
  long long mm = LLONG_MAX, mmt = LLONG_MAX;
  for (uint32_t b = lane; b < nb; b += 64) {  // the last workgroup's first wave combines the partials
    mm = min(mm, __hip_atomic_load(&p.nxt_part[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    mmt = min(mmt, __hip_atomic_load(&p.nxt_part[kNextBlocks + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  for (int d = 32; d > 0; d >>= 1) {
    mm = min(mm, static_cast<long long>(__shfl_xor(mm, d, 64)));
    mmt = min(mmt, static_cast<long long>(__shfl_xor(mmt, d, 64)));
  }
  if (lane == 0) {
    p.scal[0] = mm;
    p.scal[3] = mmt;
    p.pred[0] = 0;  // (no prediction with several workgroups)
    __hip_atomic_store(p.nxt_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (chained) {
      win_advance(p);
      p.win[kWinFrCell] = frs ? fr_c : -1;
      p.win[kWinFrHi] = fr_hi;
    }
  }
  if (chained) win_decide(p);  // (the whole wave: the chain's next window)
  ctl_publish(p, mm, mmt, seq);
}

}  // namespace bcsim
