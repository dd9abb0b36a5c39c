// transport.h — host side of the multi-GPU exchange of the node-partitioned
// PDES.  Two transports behind one interface:
//   RcclXport  RCCL over xGMI, device buffers, on the engine stream (production)
//   CbXport    caller-provided host callbacks (bcsim_transport; the tests use
//              torch.distributed gloo, several ranks may share one GPU)
// Included by bcsim_capi.hip after g_detail.
#pragma once
#include <algorithm>
#include <cstring>
#ifndef HIPEMU
#include <rccl/rccl.h>
#endif

#include <vector>

namespace bcsim {

// byte count a failed rank sends in place of a segment size: a
// transport that sees it in any count of an exchange moves no data and returns OK
constexpr uint64_t kPeerErr = 1ull << 62;

struct Xport {
  uint32_t rank = 0, nranks = 1;
  virtual ~Xport() = default;
  // the ranks of the partition may share this rank's GPU (the host-callback transport of the
  // tests); RCCL runs one rank per device
  virtual bool shares_device() const { return true; }
  // the control exchange can run on device buffers (ctl_exchange_dev, no host sync)
  virtual bool device_ctl() const { return false; }
  // device words [0, nranks*kCtlWords) -> [nranks*kCtlWords, 2*nranks*kCtlWords), queued on st
  virtual int ctl_exchange_dev(hipStream_t, int64_t*) { return BCSIM_E_UNSUPPORTED; }
  // in-place all-reduce of n int64 host values; op 0 = MIN, 1 = SUM
  virtual int allreduce_i64(hipStream_t st, int64_t* v, uint32_t n, int op) = 0;
  // device segments send_dev + r*stride of send_bytes[r] bytes -> recv_dev,
  // back to back by source rank (recv_bytes[r] each)
  virtual int alltoallv_dev(hipStream_t st, const char* send_dev, uint64_t stride, const uint64_t* send_bytes,
                            char* recv_dev, uint64_t recv_cap, uint64_t* recv_bytes) = 0;
  // the same on host memory (send segments back to back)
  virtual int alltoallv_host(hipStream_t st, const char* send, const uint64_t* send_bytes, char* recv,
                             uint64_t recv_cap, uint64_t* recv_bytes) = 0;
  // all-to-all of kCtlWords int64 per peer (host arrays [nranks][kCtlWords]): the per-cell
  // control exchange -- segment sizes, next-cell candidates, status -- in ONE collective
  static constexpr uint32_t kCtlWords = 4;
  virtual int ctl_exchange(hipStream_t st, const int64_t* send, int64_t* recv) {
    std::vector<uint64_t> sb(nranks, kCtlWords * 8ull), rb(nranks);
    const int rc = alltoallv_host(st, reinterpret_cast<const char*>(send), sb.data(), reinterpret_cast<char*>(recv),
                                  nranks * kCtlWords * 8ull, rb.data());
    if (rc) return rc;
    for (uint32_t r = 0; r < nranks; ++r)
      if (rb[r] != kCtlWords * 8ull) return BCSIM_E_HIP;
    return BCSIM_OK;
  }
  // device segments of known sizes (both sides know them from ctl_exchange)
  virtual int sendrecv_dev(hipStream_t st, const char* send_dev, uint64_t stride, const uint64_t* send_bytes,
                           char* recv_dev, const uint64_t* recv_bytes) = 0;
};

#ifndef HIPEMU  // tools/hipemu (debug host emulator) has no RCCL
#define NCCLCHK(x)                                                          \
  do {                                                                      \
    ncclResult_t r_ = (x);                                                  \
    if (r_ != ncclSuccess) {                                                \
      g_detail = std::string(#x) + ": " + ncclGetErrorString(r_);           \
      return BCSIM_E_HIP;                                                   \
    }                                                                       \
  } while (0)

struct RcclXport : Xport {
  bool shares_device() const override { return false; }
  bool device_ctl() const override { return true; }
  int ctl_exchange_dev(hipStream_t st, int64_t* w) override {
    NCCLCHK(ncclAllToAll(w, w + nranks * kCtlWords, kCtlWords, ncclInt64, comm, st));
    return BCSIM_OK;
  }
  ncclComm_t comm = nullptr;
  int64_t* d_red = nullptr;    // all-reduce scratch
  uint64_t* d_cnt = nullptr;   // [2][nranks] byte counts
  char* d_host = nullptr;      // alltoallv_host staging (device)
  uint64_t host_cap = 0;
  int64_t* h_stage = nullptr;  // pinned host staging of the control words and all-reduce values
                               // (a pageable hipMemcpyAsync is a staged, blocking copy)

  ~RcclXport() override {
    if (comm) ncclCommDestroy(comm);
    if (h_stage) (void)hipHostFree(h_stage);
    if (d_red) (void)hipFree(d_red);
    if (d_cnt) (void)hipFree(d_cnt);
    if (d_host) (void)hipFree(d_host);
  }
  static constexpr uint32_t kRedMax = 4096;  // int64 per all-reduce call
  int init(uint32_t r, uint32_t n, const ncclUniqueId& id) {
    rank = r;
    nranks = n;
    NCCLCHK(ncclCommInitRank(&comm, static_cast<int>(n), id, static_cast<int>(r)));
    HIPCHK(hipMalloc(&d_red, kRedMax * sizeof(int64_t)));
    HIPCHK(hipMalloc(&d_cnt, 2ull * n * kCtlWords * sizeof(uint64_t)));
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&h_stage), std::max<size_t>(kRedMax, 2ull * n * kCtlWords) * 8ull, 0));
    return BCSIM_OK;
  }
  int ctl_exchange(hipStream_t st, const int64_t* send, int64_t* recv) override {
    const size_t nb = nranks * kCtlWords * 8ull;
    std::memcpy(h_stage, send, nb);
    HIPCHK(hipMemcpyAsync(d_cnt, h_stage, nb, hipMemcpyHostToDevice, st));
    NCCLCHK(ncclAllToAll(d_cnt, d_cnt + nranks * kCtlWords, kCtlWords, ncclInt64, comm, st));
    HIPCHK(hipMemcpyAsync(h_stage + nranks * kCtlWords, d_cnt + nranks * kCtlWords, nb, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::memcpy(recv, h_stage + nranks * kCtlWords, nb);
    return BCSIM_OK;
  }
  int sendrecv_dev(hipStream_t st, const char* send_dev, uint64_t stride, const uint64_t* send_bytes, char* recv_dev,
                   const uint64_t* recv_bytes) override {
    NCCLCHK(ncclGroupStart());
    uint64_t off = 0;
    for (uint32_t r = 0; r < nranks; ++r) {
      if (send_bytes[r]) NCCLCHK(ncclSend(send_dev + r * stride, send_bytes[r], ncclUint8, static_cast<int>(r), comm, st));
      if (recv_bytes[r]) NCCLCHK(ncclRecv(recv_dev + off, recv_bytes[r], ncclUint8, static_cast<int>(r), comm, st));
      off += recv_bytes[r];
    }
    NCCLCHK(ncclGroupEnd());
    // (no host sync: k_import follows on the same stream)
    return BCSIM_OK;
  }
  int allreduce_i64(hipStream_t st, int64_t* v, uint32_t n, int op) override {
    if (n > kRedMax) return BCSIM_E_INVAL;
    std::memcpy(h_stage, v, n * 8ull);
    HIPCHK(hipMemcpyAsync(d_red, h_stage, n * 8ull, hipMemcpyHostToDevice, st));
    NCCLCHK(ncclAllReduce(d_red, d_red, n, ncclInt64, op == 0 ? ncclMin : ncclSum, comm, st));
    HIPCHK(hipMemcpyAsync(h_stage, d_red, n * 8ull, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::memcpy(v, h_stage, n * 8ull);
    return BCSIM_OK;
  }
  int alltoallv_dev(hipStream_t st, const char* send_dev, uint64_t stride, const uint64_t* send_bytes,
                    char* recv_dev, uint64_t recv_cap, uint64_t* recv_bytes) override {
    HIPCHK(hipMemcpyAsync(d_cnt, send_bytes, nranks * 8ull, hipMemcpyHostToDevice, st));
    NCCLCHK(ncclAllToAll(d_cnt, d_cnt + nranks, 1, ncclUint64, comm, st));
    HIPCHK(hipMemcpyAsync(recv_bytes, d_cnt + nranks, nranks * 8ull, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    uint64_t tot = 0;
    bool peer_err = false;
    for (uint32_t r = 0; r < nranks; ++r) {
      tot += recv_bytes[r];
      peer_err = peer_err || recv_bytes[r] == kPeerErr || send_bytes[r] == kPeerErr;
    }
    if (peer_err) return BCSIM_OK;  // the caller reports it (every rank saw the count)
    if (tot > recv_cap) {
      g_detail = "multi-GPU receive buffer too small";
      return BCSIM_E_OVERFLOW;
    }
    NCCLCHK(ncclGroupStart());
    uint64_t off = 0;
    for (uint32_t r = 0; r < nranks; ++r) {
      if (send_bytes[r]) NCCLCHK(ncclSend(send_dev + r * stride, send_bytes[r], ncclUint8, static_cast<int>(r), comm, st));
      if (recv_bytes[r]) NCCLCHK(ncclRecv(recv_dev + off, recv_bytes[r], ncclUint8, static_cast<int>(r), comm, st));
      off += recv_bytes[r];
    }
    NCCLCHK(ncclGroupEnd());
    HIPCHK(hipStreamSynchronize(st));
    return BCSIM_OK;
  }
  int alltoallv_host(hipStream_t st, const char* send, const uint64_t* send_bytes, char* recv, uint64_t recv_cap,
                     uint64_t* recv_bytes) override {
    uint64_t smax = 0;
    for (uint32_t r = 0; r < nranks; ++r) smax = std::max(smax, send_bytes[r]);
    const uint64_t stride = std::max<uint64_t>(smax, 16);  // local layout only
    const uint64_t need = stride * nranks + recv_cap;
    if (need > host_cap) {
      if (d_host) HIPCHK(hipFree(d_host));
      HIPCHK(hipMalloc(&d_host, need));
      host_cap = need;
    }
    uint64_t off = 0;
    for (uint32_t r = 0; r < nranks; ++r) {
      if (send_bytes[r])
        HIPCHK(hipMemcpyAsync(d_host + r * stride, send + off, send_bytes[r], hipMemcpyHostToDevice, st));
      off += send_bytes[r];
    }
    const int rc = alltoallv_dev(st, d_host, stride, send_bytes, d_host + stride * nranks, recv_cap, recv_bytes);
    if (rc) return rc;
    uint64_t rt = 0;
    for (uint32_t r = 0; r < nranks; ++r) rt += recv_bytes[r];
    if (rt) HIPCHK(hipMemcpyAsync(recv, d_host + stride * nranks, rt, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return BCSIM_OK;
  }
};

#endif  // HIPEMU

struct CbXport : Xport {
  bcsim_transport t{};
  std::vector<char> hs, hr;
  int sendrecv_dev(hipStream_t st, const char* send_dev, uint64_t stride, const uint64_t* send_bytes, char* recv_dev,
                   const uint64_t* recv_bytes) override {
    uint64_t cap = 0;
    for (uint32_t r = 0; r < nranks; ++r) cap += recv_bytes[r];
    std::vector<uint64_t> rb(nranks);
    const int rc = alltoallv_dev(st, send_dev, stride, send_bytes, recv_dev, cap, rb.data());
    if (rc) return rc;
    for (uint32_t r = 0; r < nranks; ++r)
      if (rb[r] != recv_bytes[r]) {
        g_detail = "transport: received segment sizes differ from the announced ones";
        return BCSIM_E_HIP;
      }
    return BCSIM_OK;
  }
  int allreduce_i64(hipStream_t, int64_t* v, uint32_t n, int op) override {
    if (t.allreduce_i64(t.ctx, v, n, op) != 0) {
      g_detail = "transport allreduce_i64 callback failed";
      return BCSIM_E_HIP;
    }
    return BCSIM_OK;
  }
  int alltoallv_host(hipStream_t, const char* send, const uint64_t* send_bytes, char* recv, uint64_t recv_cap,
                     uint64_t* recv_bytes) override {
    if (t.alltoallv(t.ctx, send, send_bytes, recv, recv_cap, recv_bytes) != 0) {
      g_detail = "transport alltoallv callback failed";
      return BCSIM_E_HIP;
    }
    return BCSIM_OK;
  }
  int alltoallv_dev(hipStream_t st, const char* send_dev, uint64_t stride, const uint64_t* send_bytes,
                    char* recv_dev, uint64_t recv_cap, uint64_t* recv_bytes) override {
    uint64_t tot = 0;
    bool err = false;
    for (uint32_t r = 0; r < nranks; ++r) {
      err = err || send_bytes[r] == kPeerErr;
      tot += err ? 0 : send_bytes[r];
    }
    if (err) {  // no payload: the callback still runs the count exchange
      int rc = alltoallv_host(st, nullptr, send_bytes, nullptr, 0, recv_bytes);
      return rc;
    }
    hs.resize(std::max<uint64_t>(tot, 1));
    hr.resize(std::max<uint64_t>(recv_cap, 1));
    uint64_t off = 0;
    for (uint32_t r = 0; r < nranks; ++r) {
      if (send_bytes[r]) HIPCHK(hipMemcpyAsync(hs.data() + off, send_dev + r * stride, send_bytes[r], hipMemcpyDeviceToHost, st));
      off += send_bytes[r];
    }
    HIPCHK(hipStreamSynchronize(st));
    int rc = alltoallv_host(st, hs.data(), send_bytes, hr.data(), recv_cap, recv_bytes);
    if (rc) return rc;
    uint64_t rt = 0;
    for (uint32_t r = 0; r < nranks; ++r) {
      if (recv_bytes[r] == kPeerErr) return BCSIM_OK;  // a peer failed: the caller reports it
      rt += recv_bytes[r];
    }
    if (rt > recv_cap) {
      g_detail = "multi-GPU receive buffer too small";
      return BCSIM_E_OVERFLOW;
    }
    if (rt) HIPCHK(hipMemcpyAsync(recv_dev, hr.data(), rt, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    return BCSIM_OK;
  }
};

}  // namespace bcsim
