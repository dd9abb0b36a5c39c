/*
 * oracle.h — CPU ORACLE for the bcsim hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline.  The product
 * (blockchain-simulator_amd/) never links or calls it.
 *
 * Parity status: the ns-3 network semantics restated here (scheduler tie
 * order, p2p serialization/FIFO, fragmentation, Time rounding) are
 * PARITY UNPINNED: ns-3 is not vendored in /root/reference, is not installed,
 * and the reference has no tests or golden outputs.  Pinned:
 * the glibc TYPE_3 rand() restatement (checked against this container's libc
 * in tests/test_oracle_golden.py) and analytic known-answer tests derived from
 * the reference source (message counts, quorum positions, Raft timeouts).
 */
#ifndef BCSIM_ORACLE_H
#define BCSIM_ORACLE_H
#include "../include/bcsim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bcsim_oracle bcsim_oracle;

int bcsim_oracle_create(const bcsim_config* cfg, bcsim_oracle** out);
int bcsim_oracle_set_topology_csr(bcsim_oracle* o, uint32_t n,
                                  const uint32_t* row_ptr,
                                  const uint32_t* col_idx,
                                  const int64_t* prop_ns);
int bcsim_oracle_run(bcsim_oracle* o, int64_t t_until_ns);
int bcsim_oracle_read_trace(bcsim_oracle* o, bcsim_trace_rec* buf,
                            uint64_t cap, uint64_t* n_out);
int bcsim_oracle_read_counters(bcsim_oracle* o, bcsim_counters* out);
int bcsim_oracle_read_status(bcsim_oracle* o, bcsim_status* out);
int bcsim_oracle_destroy(bcsim_oracle* o);

/* building blocks exposed for golden tests */
void    oracle_glibc_rand_seq(uint32_t seed, uint32_t n, int32_t* out);
int64_t oracle_seconds_to_ns(double s, int mode);
int64_t oracle_tx_ns(uint32_t wire_bytes, uint64_t rate_bps, int mode);
void    oracle_msg_tx(uint32_t payload, uint32_t mtu, uint64_t rate_bps,
                      int mode, int64_t* tx_total, int64_t* tx_last,
                      uint32_t* n_frames, uint32_t* wire_total);
/* FQCODEL flow classification: MurmurHash3_x86_32 and
 * Ipv4QueueDiscItem::Hash(perturbation) % flows */
uint32_t oracle_murmur3_32(const uint8_t* data, uint32_t len, uint32_t seed);
uint32_t oracle_fq_flow(uint32_t src, uint32_t dst, uint32_t sport, uint32_t dport,
                        uint32_t perturbation, uint32_t flows);
/* the client port each edge's socket bound at its first send (0: never sent), CSR order;
 * returns the edge count */
uint64_t oracle_fq_ports(const bcsim_oracle* o, uint32_t* out, uint64_t cap);
uint32_t oracle_ctr_rand(uint64_t seed, uint32_t replica, uint32_t node,
                         uint64_t k);

#ifdef __cplusplus
}
#endif
#endif
