// Issue rate of v_fma_f32 against v_pk_fma_f32 on gfx950 (calibration tool):
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize scripts/cal/pk_rate.hip -o /tmp/pk_rate && /tmp/pk_rate
// 8 independent chains per lane, 4096 iterations; reports lane-FMA/s.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_scalar(float* out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < 4096; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_packed(float* out, float a, float b) {
  f2 x[4];
  for (int i = 0; i < 4; ++i) x[i] = f2{threadIdx.x * 1e-3f + i, threadIdx.x * 1e-3f - i};
  const f2 A = f2{a, a}, B = f2{b, b};
  for (int it = 0; it < 4096; ++it)
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = __builtin_elementwise_fma(x[i], A, B);
  float s = 0;
  for (int i = 0; i < 4; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  const int blocks = 256 * 8 * 4;  // 8 waves/SIMD worth of 256-thread blocks
  float* out;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep)
    for (int k = 0; k < 2; ++k) {
      hipEventRecord(e0);
      if (k == 0) k_scalar<<<blocks, 256>>>(out, 0.999f, 1e-3f);
      else k_packed<<<blocks, 256>>>(out, 0.999f, 1e-3f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double fmas = (double)blocks * 256 * 4096 * 8;
      printf("%s: %.3f ms, %.1f TFLOP/s (FMA = 2)\n", k ? "v_pk_fma_f32" : "v_fma_f32", ms, 2 * fmas / ms / 1e9);
    }
  hipFree(out);
  return 0;
}
