// host_math.h — host-side constant tables of the engine (product code).
//
// Independent implementation (not shared with oracle/): ns-3 float-second to
// integer-ns conversion, p2p serialization times with IPv4 fragmentation, and
// the glibc TYPE_3 rand() stream, all precomputed on the host and uploaded.
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/bcsim.h"

namespace bcsim {

// Seconds(double) -> ns as ns-3 Time(int64x64_t): 64 fractional bits,
// exact product with 1e9, then Round() (half away from zero) or floor.
int64_t seconds_to_ns(double s, uint32_t time_round);
inline int64_t fsec_to_ns(float f, uint32_t time_round) {
  return seconds_to_ns(static_cast<double>(f), time_round);
}

// DataRate::CalculateBytesTxTime for one frame.
int64_t frame_tx_ns(uint32_t wire_bytes, uint64_t rate_bps, uint32_t time_round);

struct MsgTx {
  int64_t total;   // all frames back to back
  int64_t last;    // last frame
  uint32_t frames;
  uint32_t wire;
};
// UDP 8 + IPv4 20 (+ fragmentation at mtu) + PPP 2 per frame.
MsgTx message_tx(uint32_t payload, uint32_t mtu, uint64_t rate_bps,
                 uint32_t time_round);

// First n outputs of glibc rand() after srand(seed) (TYPE_3 additive
// feedback generator, r[i] = r[i-3] + r[i-31], 310 discarded outputs).
std::vector<int32_t> glibc_stream(uint32_t seed, size_t n);

// FQCODEL: per directed edge the number of its link in the reference's mesh
// loop (blockchain-simulator.cc:34-51: larger endpoint ascending, then smaller), which names the
// link's 1.0.k.0/24 network.  CSR rows ascending, rev = reverse edges.  The flow of each packet
// class is bound on the device when the class first reaches the disc (engine fq_class_slot).
std::vector<uint32_t> fq_link_numbers(uint32_t N, const std::vector<uint32_t>& row, const std::vector<uint32_t>& col,
                                      const std::vector<uint32_t>& rev);

}  // namespace bcsim
