// hipemu runtime (DEBUG-ONLY): blocks run one after another, the threads of a
// block are real std::threads synchronised by a std::barrier.
#include "hip/hip_runtime.h"

#include <chrono>
#include <condition_variable>
#include <latch>
#include <cstdio>

thread_local hipemu_ctx hipemu_t;
static thread_local char* t_smem = nullptr;
char* hipemu_dyn_smem() { return t_smem; }

const char* hipGetErrorString(hipError_t e) { return e ? "hipemu error" : "no error"; }
hipError_t hipGetDeviceCount(int* n) { *n = 1; return hipSuccess; }
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) { *s = reinterpret_cast<hipStream_t>(0x1); return hipSuccess; }
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamQuery(hipStream_t) { return hipSuccess; }
hipError_t hipDeviceSynchronize() { return hipSuccess; }
hipError_t hipMalloc(void** p, size_t n) { *p = std::malloc(n ? n : 1); return *p ? hipSuccess : hipErrorUnknown; }
hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }
hipError_t hipHostMalloc(void** p, size_t n, unsigned) { return hipMalloc(p, n); }
hipError_t hipHostFree(void* p) { return hipFree(p); }
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) { *d = h; return hipSuccess; }
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) { std::memcpy(d, s, n); return hipSuccess; }
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind k, hipStream_t) { return hipMemcpy(d, s, n, k); }
hipError_t hipMemset(void* d, int v, size_t n) { std::memset(d, v, n); return hipSuccess; }
hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) { return hipMemset(d, v, n); }
struct hipemu_event { std::chrono::steady_clock::time_point t; };
hipError_t hipEventCreate(hipEvent_t* e) { *e = new hipemu_event(); return hipSuccess; }
hipError_t hipEventDestroy(hipEvent_t e) { delete e; return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t e, hipStream_t) { e->t = std::chrono::steady_clock::now(); return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
  *ms = std::chrono::duration<float, std::milli>(b->t - a->t).count();
  return hipSuccess;
}
hipError_t hipGetLastError() { return hipSuccess; }
hipError_t hipFuncSetAttribute(const void*, hipFuncAttribute, int) { return hipSuccess; }

// persistent worker pool (ASan caps the number of threads ever created)
namespace {
struct Pool {
  static constexpr unsigned kMax = 1024;
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv;
  unsigned long long gen = 0;
  // current block job
  const std::function<void()>* body = nullptr;
  dim3 grid, block;
  unsigned bid = 0, nt = 0;
  std::barrier<>* bar = nullptr;
  std::barrier<>* wbar = nullptr;
  std::latch* done = nullptr;
  char* smem = nullptr;
  unsigned long long* shfl = nullptr;
  Pool() {
    for (unsigned t = 0; t < kMax; ++t) th.emplace_back([this, t]() { run(t); });
  }
  void run(unsigned t) {
    unsigned long long seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(m);
      cv.wait(lk, [&]() { return gen != seen; });
      seen = gen;
      if (t >= nt) continue;
      auto* b = body;
      hipemu_t.tid = dim3(t);
      hipemu_t.bid = dim3(bid);
      hipemu_t.bdim = block;
      hipemu_t.gdim = grid;
      hipemu_t.bar = bar;
      hipemu_t.wbar = wbar;
      hipemu_t.shfl = shfl;
      t_smem = smem;
      auto* dn = done;
      auto* br = bar;
      auto* wb = &wbar[t / 64];
      lk.unlock();
      try {
        (*b)();
      } catch (const hipemu_exit&) {
        std::fprintf(stderr, "hipemu: wave ended by s_endpgm (block %u thread %u)\n", hipemu_t.bid.x, t);
      }
      br->arrive_and_drop();
      wb->arrive_and_drop();
      dn->count_down();
    }
  }
};
Pool& pool() {
  static Pool* p = new Pool();  // leaked on purpose: workers never exit
  return *p;
}
}  // namespace

void hipemu_launch(dim3 grid, dim3 block, size_t lds, const std::function<void()>& body) {
  Pool& P = pool();
  const unsigned nt = block.x * block.y * block.z;
  if (nt > Pool::kMax) throw std::runtime_error("hipemu: block too large");
  std::vector<char> smem(lds + 64, 0);
  std::vector<unsigned long long> shfl(nt);
  if (nt % 64) throw std::runtime_error("hipemu: block must be a multiple of 64 threads");
  for (unsigned b = 0; b < grid.x; ++b) {
    std::barrier<> bar(nt);
    std::allocator<std::barrier<>> wal;
    const unsigned nw = nt / 64;
    std::barrier<>* wb = wal.allocate(nw);
    for (unsigned w = 0; w < nw; ++w) new (&wb[w]) std::barrier<>(64);
    std::latch done(nt);
    {
      std::lock_guard<std::mutex> lk(P.m);
      P.body = &body;
      P.grid = grid;
      P.block = block;
      P.bid = b;
      P.nt = nt;
      P.bar = &bar;
      P.done = &done;
      P.smem = smem.data();
      P.shfl = shfl.data();
      P.wbar = wb;
      ++P.gen;
    }
    P.cv.notify_all();
    done.wait();
    for (unsigned w = 0; w < nw; ++w) wb[w].~barrier();
    wal.deallocate(wb, nw);
  }
}
