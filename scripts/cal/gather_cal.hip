// Calibration of the HBM counters and rates for the traversal's access
// patterns (gfx950): what FETCH_SIZE / WRITE_SIZE report, and what the chip
// sustains, for
//   stream   : coalesced 16-B-per-lane reads of a buffer (the guide's x2 case)
//   gather32 : one 32-B ray record (two float4) per lane at random ids
//   gather64 : one 64-B record (four float4) per lane at random ids
//   idgather : the level kernel's pattern -- a coalesced 4-B id, then the
//              32-B record it names (random)
//   amin64   : a 64-bit atomicMin per lane at random 32-B records
// Buffers are 4 GiB (far past the 256 MiB Infinity Cache).  Prints one line
// per kernel: useful bytes, time, useful GB/s.  Run it under rocprofv3 --pmc
// FETCH_SIZE / WRITE_SIZE to read the counters per dispatch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_stream(const float4* __restrict__ a, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;
}
__global__ void k_gather32(const float4* __restrict__ rec, const uint32_t* __restrict__ ids, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t id = ids[i];
    float4 a = rec[2 * (size_t)id], b = rec[2 * (size_t)id + 1];
    s += a.x + a.w + b.x + b.w;
  }
  if (s == 1234.5f) out[0] = s;
}
// the same gather with the loads' cache-policy bits set (gfx950 global_load
// sc0 / sc1 / nt): does a non-default policy fetch less than a 128-B line?
template <int POL>
__device__ __forceinline__ float4 ldpol(const float4* p) {
  float4 r;
  if constexpr (POL == 1)
    asm volatile("global_load_dwordx4 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  else if constexpr (POL == 2)
    asm volatile("global_load_dwordx4 %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  else if constexpr (POL == 3)
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  else if constexpr (POL == 4)
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  else if constexpr (POL == 5)
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  else
    asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
  return r;
}
template <int POL>
__global__ void k_gather32p(const float4* __restrict__ rec, const uint32_t* __restrict__ ids, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t id = ids[i];
    float4 a = ldpol<POL>(rec + 2 * (size_t)id), b = ldpol<POL>(rec + 2 * (size_t)id + 1);
    s += a.x + a.w + b.x + b.w;
  }
  if (s == 1234.5f) out[0] = s;
}
__global__ void k_gather64(const float4* __restrict__ rec, const uint32_t* __restrict__ ids, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t id = ids[i];
    const float4* r = rec + 4 * (size_t)id;
    float4 a = r[0], b = r[1], c = r[2], d = r[3];
    s += a.x + b.y + c.z + d.w;
  }
  if (s == 1234.5f) out[0] = s;
}
__global__ void k_amin64(float4* rec, const uint32_t* __restrict__ ids, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t id = ids[i];
    atomicMin(reinterpret_cast<unsigned long long*>(rec + 2 * (size_t)id + 1) + 1, (unsigned long long)i);
  }
}
__global__ void k_fill_ids(uint32_t* ids, size_t n, uint32_t nrec, uint32_t seed, int sorted_runs) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    ids[i] = x % nrec;
  }
}

int main() {
  const size_t bytes = 4ull << 30;
  const uint32_t nrec32 = (uint32_t)(bytes / 32), nrec64 = (uint32_t)(bytes / 64);
  const size_t n = 64ull << 20;  // 64 Mi accesses
  float4* buf;
  uint32_t* ids;
  float* out;
  CHK(hipMalloc(&buf, bytes));
  CHK(hipMalloc(&ids, n * 4));
  CHK(hipMalloc(&out, 16));
  CHK(hipMemset(buf, 0, bytes));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const dim3 g(8192), b(256);
  auto run = [&](const char* name, auto launch, double useful) {
    launch();  // warm
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-9s useful %.3f GB  %.3f ms  %.1f GB/s useful\n", name, useful / 1e9, ms, useful / (ms * 1e-3) / 1e9);
  };
  run("stream", [&] { hipLaunchKernelGGL(k_stream, g, b, 0, 0, buf, bytes / 16, out); }, (double)bytes);
  hipLaunchKernelGGL(k_fill_ids, g, b, 0, 0, ids, n, nrec32, 7u, 0);
  run("gather32", [&] { hipLaunchKernelGGL(k_gather32, g, b, 0, 0, buf, ids, n, out); }, (double)n * 36);
  run("amin64", [&] { hipLaunchKernelGGL(k_amin64, g, b, 0, 0, buf, ids, n); }, (double)n * 12);
  run("g32asm", [&] { hipLaunchKernelGGL(k_gather32p<0>, g, b, 0, 0, buf, ids, n, out); }, (double)n * 36);
  run("g32nt", [&] { hipLaunchKernelGGL(k_gather32p<1>, g, b, 0, 0, buf, ids, n, out); }, (double)n * 36);
  run("g32sc0", [&] { hipLaunchKernelGGL(k_gather32p<2>, g, b, 0, 0, buf, ids, n, out); }, (double)n * 36);
  run("g32sc1", [&] { hipLaunchKernelGGL(k_gather32p<3>, g, b, 0, 0, buf, ids, n, out); }, (double)n * 36);
  run("g32sc01", [&] { hipLaunchKernelGGL(k_gather32p<4>, g, b, 0, 0, buf, ids, n, out); }, (double)n * 36);
  run("g32sc01nt", [&] { hipLaunchKernelGGL(k_gather32p<5>, g, b, 0, 0, buf, ids, n, out); }, (double)n * 36);
  {
    // uncached allocation (MTYPE UC)
    float4* ubuf = nullptr;
    if (hipExtMallocWithFlags((void**)&ubuf, bytes, hipDeviceMallocUncached) == hipSuccess) {
      CHK(hipMemset(ubuf, 0, bytes));
      run("g32uc", [&] { hipLaunchKernelGGL(k_gather32, g, b, 0, 0, ubuf, ids, n, out); }, (double)n * 36);
      CHK(hipFree(ubuf));
    } else {
      printf("uncached allocation failed\n");
    }
  }
  hipLaunchKernelGGL(k_fill_ids, g, b, 0, 0, ids, n, nrec64, 9u, 0);
  run("gather64", [&] { hipLaunchKernelGGL(k_gather64, g, b, 0, 0, buf, ids, n, out); }, (double)n * 68);
  CHK(hipDeviceSynchronize());
  return 0;
}
