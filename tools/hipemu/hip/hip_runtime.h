// hipemu — DEBUG-ONLY host emulation of the small HIP subset used by
// blockchain-simulator_amd/csrc, so kernels can run under AddressSanitizer on
// the CPU when a GPU fault must be located without faulting a GPU.  Never used
// by the product, tests or bench (tools/hipemu/README.md).
#pragma once
#include <atomic>
#include <barrier>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <type_traits>
#include <vector>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static

struct dim3 {
  unsigned x = 1, y = 1, z = 1;
  dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct hipemu_ctx {
  dim3 tid, bid, bdim, gdim;
  std::barrier<>* bar;
  std::barrier<>* wbar;      // per-wave barriers (64 lanes each)
  unsigned long long* shfl;  // per-block shuffle exchange
};
struct uint4 {
  unsigned x, y, z, w;
};
inline uint4 make_uint4(unsigned a, unsigned b, unsigned c, unsigned d) { return uint4{a, b, c, d}; }
struct uint2 {
  unsigned x, y;
};
inline uint2 make_uint2(unsigned a, unsigned b) { return uint2{a, b}; }
extern thread_local hipemu_ctx hipemu_t;
#define threadIdx (hipemu_t.tid)
#define blockIdx (hipemu_t.bid)
#define blockDim (hipemu_t.bdim)
#define gridDim (hipemu_t.gdim)
struct hipemu_exit {};
inline void __syncthreads() { hipemu_t.bar->arrive_and_wait(); }
inline void __builtin_amdgcn_endpgm() { throw hipemu_exit{}; }
char* hipemu_dyn_smem();

// wave-level exchange: every lane of the wave must call (wave64)
inline void hipemu_wsync() { hipemu_t.wbar[hipemu_t.tid.x / 64].arrive_and_wait(); }
inline unsigned long long hipemu_xchg_get(unsigned lane) {
  return hipemu_t.shfl[(hipemu_t.tid.x / 64) * 64 + lane];
}
template <typename T>
inline T hipemu_from(unsigned long long v) {
  T r;
  std::memcpy(&r, &v, sizeof(T));
  return r;
}
template <typename T>
inline unsigned long long hipemu_to(T v) {
  unsigned long long r = 0;
  std::memcpy(&r, &v, sizeof(T));
  return r;
}
template <typename T>
inline T __shfl(T v, int src, int width = 64) {
  hipemu_t.shfl[hipemu_t.tid.x] = hipemu_to(v);
  hipemu_wsync();
  T r = hipemu_from<T>(hipemu_xchg_get(static_cast<unsigned>(src) & 63u));
  hipemu_wsync();
  return r;
}
template <typename T>
inline T __shfl_up(T v, unsigned d, int width = 64) {
  hipemu_t.shfl[hipemu_t.tid.x] = hipemu_to(v);
  hipemu_wsync();
  unsigned lane = hipemu_t.tid.x % 64;
  T r = lane >= d ? hipemu_from<T>(hipemu_xchg_get(lane - d)) : v;
  hipemu_wsync();
  return r;
}
template <typename T>
inline T __shfl_xor(T v, int m, int width = 64) {
  hipemu_t.shfl[hipemu_t.tid.x] = hipemu_to(v);
  hipemu_wsync();
  unsigned lane = hipemu_t.tid.x % 64;
  T r = hipemu_from<T>(hipemu_xchg_get((lane ^ static_cast<unsigned>(m)) & 63u));
  hipemu_wsync();
  return r;
}
inline unsigned long long __ballot(int pred) {
  hipemu_t.shfl[hipemu_t.tid.x] = pred ? 1ull : 0ull;
  hipemu_wsync();
  unsigned long long m = 0;
  for (unsigned l = 0; l < 64; ++l)
    if (hipemu_xchg_get(l)) m |= 1ull << l;
  hipemu_wsync();
  return m;
}
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
inline int __ffs(unsigned int x) { return __builtin_ffs(static_cast<int>(x)); }
inline int __ffsll(unsigned long long x) { return __builtin_ffsll(static_cast<long long>(x)); }
inline int __popc(unsigned x) { return __builtin_popcount(x); }
inline unsigned long long __umul64hi(unsigned long long a, unsigned long long b) { return static_cast<unsigned long long>((static_cast<unsigned __int128>(a) * b) >> 64); }
// lane-exchange / ordering builtins: every lane of the wave must reach them together
template <typename T>
inline T __builtin_amdgcn_readlane(T v, int lane) { return __shfl(v, lane); }
// (the engine reads only wave-uniform values this way)
inline int __builtin_amdgcn_readfirstlane(int v) { return v; }
inline void __builtin_amdgcn_wave_barrier() { hipemu_wsync(); }
#define __builtin_amdgcn_fence(...) std::atomic_thread_fence(std::memory_order_seq_cst)
inline unsigned long long __builtin_amdgcn_s_memrealtime() {  // 100 MHz
  return static_cast<unsigned long long>(std::chrono::steady_clock::now().time_since_epoch().count() / 10);
}
inline int __ffsll(long long x) { return __builtin_ffsll(x); }

template <typename T, typename U>
inline T atomicAdd(T* p, U v) { return __atomic_fetch_add(p, static_cast<T>(v), __ATOMIC_SEQ_CST); }
template <typename T, typename U>
inline T atomicOr(T* p, U v) { return __atomic_fetch_or(p, static_cast<T>(v), __ATOMIC_SEQ_CST); }
template <typename T, typename U>
inline T atomicAnd(T* p, U v) { return __atomic_fetch_and(p, static_cast<T>(v), __ATOMIC_SEQ_CST); }
template <typename T, typename U, typename V>
inline T atomicCAS(T* p, U cmp_, V v_) {
  T cmp = static_cast<T>(cmp_), v = static_cast<T>(v_);
  __atomic_compare_exchange_n(p, &cmp, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
  return cmp;
}
template <typename T, typename U>
inline T atomicMin(T* p, U v_) {
  T v = static_cast<T>(v_);
  T o = __atomic_load_n(p, __ATOMIC_SEQ_CST);
  while (v < o && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
  }
  return o;
}
template <typename T, typename U>
inline T atomicMax(T* p, U v_) {
  T v = static_cast<T>(v_);
  T o = __atomic_load_n(p, __ATOMIC_SEQ_CST);
  while (v > o && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
  }
  return o;
}
template <typename A, typename B>
inline std::common_type_t<A, B> min(A a, B b) { return a < b ? a : b; }
template <typename A, typename B>
inline std::common_type_t<A, B> max(A a, B b) { return a < b ? b : a; }

#define __ATOMIC_RELAXED_ __ATOMIC_RELAXED
#define __HIP_MEMORY_SCOPE_SYSTEM 0
template <typename T, typename U>
inline void __hip_atomic_store(T* p, U v, int, int) { __atomic_store_n(p, static_cast<T>(v), __ATOMIC_RELAXED); }
template <typename T>
inline T __hip_atomic_load(T* p, int, int) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
#define __HIP_MEMORY_SCOPE_AGENT 1
template <typename T, typename U>
inline T __hip_atomic_fetch_add(T* p, U v, int, int) { return __atomic_fetch_add(p, static_cast<T>(v), __ATOMIC_RELAXED); }
template <typename T, typename U>
inline T __hip_atomic_fetch_min(T* p, U v, int, int) {
  T o = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (static_cast<T>(v) < o && !__atomic_compare_exchange_n(p, &o, static_cast<T>(v), false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
  return o;
}
template <typename T, typename U>
inline T __hip_atomic_fetch_max(T* p, U v, int, int) {
  T o = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (static_cast<T>(v) > o && !__atomic_compare_exchange_n(p, &o, static_cast<T>(v), false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
  return o;
}
template <typename T, typename U>
inline bool __hip_atomic_compare_exchange_strong(T* p, T* expected, U desired, int, int, int) {
  return __atomic_compare_exchange_n(p, expected, static_cast<T>(desired), false, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
}
#define __HIP_MEMORY_SCOPE_WORKGROUP 2
inline void __threadfence() { std::atomic_thread_fence(std::memory_order_seq_cst); }
inline void __threadfence_system() { std::atomic_thread_fence(std::memory_order_seq_cst); }

// ---- runtime API subset ----
typedef int hipError_t;
enum { hipSuccess = 0, hipErrorNotReady = 600, hipErrorUnknown = 999 };
typedef struct hipemu_stream* hipStream_t;
typedef struct hipemu_event* hipEvent_t;
enum hipMemcpyKind { hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice, hipMemcpyDefault };
enum { hipStreamNonBlocking = 1, hipFuncAttributeMaxDynamicSharedMemorySize = 8 };
typedef int hipFuncAttribute;
const char* hipGetErrorString(hipError_t);
hipError_t hipGetDeviceCount(int*);
hipError_t hipSetDevice(int);
hipError_t hipStreamCreateWithFlags(hipStream_t*, unsigned);
hipError_t hipStreamDestroy(hipStream_t);
hipError_t hipStreamSynchronize(hipStream_t);
hipError_t hipStreamQuery(hipStream_t);
hipError_t hipDeviceSynchronize();
hipError_t hipMalloc(void**, size_t);
hipError_t hipFree(void*);
hipError_t hipHostMalloc(void**, size_t, unsigned = 0);
hipError_t hipHostGetDevicePointer(void**, void*, unsigned);
enum { hipHostMallocMapped = 2, hipHostMallocCoherent = 0x40000000 };
hipError_t hipHostFree(void*);
hipError_t hipMemcpy(void*, const void*, size_t, hipMemcpyKind);
inline hipError_t hipMemGetInfo(size_t* fr, size_t* tot) { *fr = *tot = 64ull << 30; return hipSuccess; }
hipError_t hipMemcpyAsync(void*, const void*, size_t, hipMemcpyKind, hipStream_t);
hipError_t hipMemset(void*, int, size_t);
hipError_t hipMemsetAsync(void*, int, size_t, hipStream_t);
hipError_t hipEventCreate(hipEvent_t*);
enum { hipEventDisableSystemFence = 0x20000000, hipEventDisableTiming = 0x2 };
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
hipError_t hipEventDestroy(hipEvent_t);
hipError_t hipEventRecord(hipEvent_t, hipStream_t);
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }  // (streams run in issue order)
hipError_t hipEventElapsedTime(float*, hipEvent_t, hipEvent_t);
hipError_t hipGetLastError();
hipError_t hipFuncSetAttribute(const void*, hipFuncAttribute, int);

void hipemu_launch(dim3 grid, dim3 block, size_t lds, const std::function<void()>& body);
#define hipLaunchKernelGGL(K, G, B, S, ST, ...) hipemu_launch(dim3(G), dim3(B), (S), [=]() { K(__VA_ARGS__); })
