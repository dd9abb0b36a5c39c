// engine.h — device data layout of the MI355X consensus-propagation engine.
//
// Layout in HBM:
//   node state      SoA, one slot per (replica, node) = "gnode" g = rep*N + i
//   link state      busy_until[rep*E + e] and last_cell[rep*E + e], sender-major
//                   CSR edge order (edge e = i -> col[e], rows ascending)
//   inbox           B time buckets; bucket b holds cell c (c % B == b) as one
//                   16-byte Rec per directed edge, stored at the RECEIVER's
//                   in-slot: the arrival on edge i->s lives at index rev[e]
//                   (= the edge s->i, inside s's CSR row), so a receiver reads
//                   its arrivals as one contiguous row, already in ascending
//                   origin order (the canonical tie order).  A second record on
//                   the same edge in the same cell goes to the bucket's extras
//                   list; arrivals beyond the ring go to the overflow list.
//   pending ops     per gnode list of 32-byte Op (echo / unicast / broadcast)
//   timers          per gnode list of TimerEnt (Raft / Paxos)
#pragma once
#include <stdint.h>

#include "../../include/bcsim.h"

namespace bcsim {

constexpr uint32_t kInvalid = 0xFFFFFFFFu;

// Rec::flags
enum : uint8_t {
  RF_VALID = 1,  // slot holds an undelivered packet
  RF_BIG = 2,    // block / proposal sized payload
  RF_OWNER = 4   // (overflow list only) first record of its (edge, cell): goes to the slot
};

// 16-byte arrival record: one packet delivered to a listener socket.  The
// sender (col[slot]), the edge and dt = t - t_sched (= propagation + last
// frame serialisation) are implied by the slot it is stored at.
struct __attribute__((aligned(16))) Rec {
  uint32_t t_off;   // arrival time - start of the arrival cell
  uint32_t sub;     // sender's schedule counter of the SendPacket
  int16_t f0, f1;   // raw payload chars data[1], data[2]
  int16_t f2;       // data[3]
  uint8_t type;     // charToInt(data[0])
  uint8_t flags;    // RF_*
};
static_assert(sizeof(Rec) == 16, "Rec must be 16 bytes");

// Extras / overflow entry: a record that does not own its slot, or whose
// cell is beyond the bucket ring.
struct __attribute__((aligned(16))) XRec {
  Rec r;
  int64_t cell;   // arrival cell (overflow list); -1 once rebinned
  uint32_t slot;  // in-slot: edge index within the replica, in the receiver's row
  uint32_t g;     // receiver gnode
};
static_assert(sizeof(XRec) == 32, "XRec must be 32 bytes");

// op kinds
enum : uint8_t { OP_ECHO = 0, OP_SEND = 1, OP_BCAST = 2, OP_BCAST_J = 3 };
// op flags (Op::flags)
enum : uint8_t {
  OPF_BIG = 1,       // big payload
  OPF_PAXOS = 2,     // Paxos broadcast (skip peers[0], drop *end())
  OPF_DONE = 4       // expanded broadcast (jitter) -- consumed
};

// 32-byte pending link operation.
struct __attribute__((aligned(16))) Op {
  int64_t t;        // execution time (SendPacket / echo time)
  uint32_t dt;      // t - t_sched
  uint32_t origin;  // key origin (node itself; ECHO: the received packet's sender)
  uint32_t sub;     // key sub (BCAST: first edge's sub; edge k gets sub+k)
  uint32_t edge;    // edge index within replica (SEND/ECHO); BCAST_J: draw base lo
  int16_t f0, f1;
  int16_t f2;
  uint8_t type;
  uint8_t kind_flags;  // kind (2 bits) | flags << 2
};
static_assert(sizeof(Op) == 32, "Op must be 32 bytes");

__host__ __device__ inline uint8_t op_kind(const Op& o) { return o.kind_flags & 3; }
__host__ __device__ inline uint8_t op_flags(const Op& o) { return o.kind_flags >> 2; }

// timer kinds
enum : uint8_t {
  TM_RAFT_ELECTION = 1,
  TM_RAFT_HEARTBEAT = 2,
  TM_RAFT_PROPOSAL = 3,
  TM_PAXOS_TICKET = 4,
  TM_GOSSIP_BLOCK = 5
};

struct __attribute__((aligned(8))) TimerEnt {
  int64_t t;      // fire time (INT64_MAX while a glibc draw is pending)
  int64_t ts;     // t_sched
  uint32_t sub;   // schedule counter (= EventId)
  uint8_t kind;
  uint8_t alive;  // 0 = cancelled / fired (slot free)
  uint8_t pending_draw;
  uint8_t pad;
};
static_assert(sizeof(TimerEnt) == 24, "TimerEnt");

// glibc draw request (Raft election timeout in GLIBC mode), resolved in
// canonical global order at the end of the cell.
struct DrawReq {
  int64_t t;
  int64_t ts;
  uint32_t origin, sub, target;  // event key (target = node)
  uint32_t rep;
  uint32_t timer_sub;            // timer entry to fill
  uint32_t pad;
};

// PBFT global v write log (file-scope `v`, pbft-node.cc:26)
struct VLog {
  int64_t t, ts;
  uint32_t origin, sub, target, rep;
  int32_t v;
  int32_t pad;
};

// per-replica counters layout in the device counter array
enum {
  CNT_DELIV = 0,        // 16 entries
  CNT_DELIV_TOTAL = 16,
  CNT_ECHOES,
  CNT_SENDS,
  CNT_DROPPED,
  CNT_WRONG,
  CNT_EVENTS,
  CNT_TLAST,            // max event time (atomicMax)
  CNT_FDROP,            // DROPTAIL: frames refused by a full link queue
  CNT_LOST,             // DROPTAIL: messages with a dropped fragment
  CNT_N
};

// kernel-class timing slots
enum { KS_SCAN = 0, KS_LINK = 1, KS_GROUP = 2, KS_AUX = 3 };

// link-kernel algorithmic counters (KP::kstat)
enum { KST_REC = 0, KST_OPS = 1, KST_EDGES = 2, KST_KEPT = 3, KST_DELIV = 4, KST_SCAN_OPS = 5, KST_ECHO = 6, KST_SPLIT = 7 };

}  // namespace bcsim
