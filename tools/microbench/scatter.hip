// DEBUG/MEASUREMENT ONLY: does a receiver-major scatter of 16-byte records
// (sender s writes slot s of every receiver row, N=4096 full mesh) cost more
// HBM time than a sender-major contiguous write + LDS-tiled transpose?
//   hipcc --offload-arch=gfx950 -O3 scatter.hip -o scatter && ./scatter
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__device__ inline uint32_t xcd_map(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, k = b >> 3, per = n >> 3, rem = n & 7u;
  return x * per + min(x, rem) + k;
}

// (a) sender-major: WG s writes its row contiguously
__global__ __launch_bounds__(1024) void k_rowwrite(uint4* out, uint32_t N, int xcd) {
  const uint32_t s = xcd ? xcd_map(blockIdx.x, N) : blockIdx.x;
  for (uint32_t r = threadIdx.x; r < N - 1; r += blockDim.x)
    out[static_cast<size_t>(s) * (N - 1) + r] = make_uint4(s, r, 1, 2);
}
// (b) receiver-major scatter: WG s writes slot idx(s) of every receiver row
__global__ __launch_bounds__(1024) void k_scatter(uint4* in, uint32_t N, int xcd) {
  const uint32_t s = xcd ? xcd_map(blockIdx.x, N) : blockIdx.x;
  for (uint32_t le = threadIdx.x; le < N - 1; le += blockDim.x) {
    const uint32_t r = le < s ? le : le + 1;
    in[static_cast<size_t>(r) * (N - 1) + (s < r ? s : s - 1)] = make_uint4(s, r, 1, 2);
  }
}
// (b') scatter with 8 consecutive senders per workgroup (each lane writes 8 x 16 B = 128 B? no:
// lanes of a wave take 8 senders x 8 receivers so that 8 consecutive slots of one row are one
// wave-instruction's contiguous 128 B)
__global__ __launch_bounds__(1024) void k_scatter8(uint4* in, uint32_t N) {
  const uint32_t s0 = blockIdx.x * 8;  // senders s0..s0+7
  for (uint32_t k = threadIdx.x; k < 8 * N; k += blockDim.x) {
    const uint32_t s = s0 + (k & 7), r = k >> 3;
    if (s >= N || r >= N || r == s) continue;
    in[static_cast<size_t>(r) * (N - 1) + (s < r ? s : s - 1)] = make_uint4(s, r, 1, 2);
  }
}
// (c) 64x64 tile transpose (read sender-major + write receiver-major), as k_transpose
__global__ __launch_bounds__(256) void k_tr(const uint4* ob, uint4* ib, uint32_t N) {
  __shared__ uint4 tile[64][64];
  const uint32_t nt = (N + 63) / 64;
  const uint32_t tj = blockIdx.x % nt, ti = blockIdx.x / nt;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  for (uint32_t r = w; r < 64; r += 4) {
    const uint32_t i = ti * 64 + r, s = tj * 64 + lane;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (i < N && s < N && s != i) v = ob[static_cast<size_t>(i) * (N - 1) + s - (s > i)];
    tile[r][lane ^ r] = v;
  }
  __syncthreads();
  for (uint32_t c = w; c < 64; c += 4) {
    const uint32_t s = tj * 64 + c, i = ti * 64 + lane;
    const uint4 v = tile[lane][c ^ lane];
    if (i < N && s < N && s != i) ib[static_cast<size_t>(s) * (N - 1) + i - (i > s)] = v;
  }
}
// (d) receiver row read (coalesced) + sum, as k_scan staging
__global__ __launch_bounds__(1024) void k_rowread(const uint4* in, uint32_t N, uint32_t* sink) {
  const uint32_t s = blockIdx.x;
  uint32_t acc = 0;
  for (uint32_t r = threadIdx.x; r < N - 1; r += blockDim.x) {
    const uint4 v = in[static_cast<size_t>(s) * (N - 1) + r];
    acc += v.x ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const uint32_t N = 4096;
  const size_t E = static_cast<size_t>(N) * (N - 1);
  uint4 *a, *b;
  uint32_t* sink;
  CK(hipMalloc(&a, E * 16));
  CK(hipMalloc(&b, E * 16));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a, 0, E * 16));
  CK(hipMemset(b, 0, E * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto fn, double bytes) {
    for (int w = 0; w < 3; ++w) fn();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0, 0));
    for (int k = 0; k < reps; ++k) fn();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / reps;
    printf("%-34s %9.1f us  %7.2f TB/s (%.0f MB algorithmic)\n", name, us, bytes / (us * 1e-6) / 1e12, bytes / 1e6);
    return 0;
  };
  const double rec = E * 16.0;
  run("row write (sender-major)", [&] { k_rowwrite<<<N, 1024>>>(a, N, 1); }, rec);
  run("row write, no xcd map", [&] { k_rowwrite<<<N, 1024>>>(a, N, 0); }, rec);
  run("scatter (receiver-major), xcd map", [&] { k_scatter<<<N, 1024>>>(b, N, 1); }, rec);
  run("scatter, no xcd map", [&] { k_scatter<<<N, 1024>>>(b, N, 0); }, rec);
  run("scatter, 8 senders per WG", [&] { k_scatter8<<<N / 8, 1024>>>(b, N); }, rec);
  run("tile transpose (read+write)", [&] { k_tr<<<(N / 64) * (N / 64), 256>>>(a, b, N); }, 2 * rec);
  run("row read (receiver rows)", [&] { k_rowread<<<N, 1024>>>(b, N, sink); }, rec);
  return 0;
}
