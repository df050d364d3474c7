// Post-process kernels (gfx950): the reference's display filter.
//
//   kernelMedianFilter   src/cudaRenderer.cu:773-842   -> k_median3
//
// Per channel the reference removes the maximum of the 3x3 neighbourhood
// three times (setting it to 0) and keeps the fourth maximum; out-of-frame
// neighbours are 1.0.  The selection is restated literally (max search from
// 0.0 with >=, last index wins) so NaN and tie cases match too.
#include "trace.h"

namespace pt {

__device__ __forceinline__ float ref_median_channel(float (&v)[9]) {
  float out = 0.0f;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    int im = 0;
    float m = 0.0f;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      if (v[j] >= m) {
        m = v[j];
        im = j;
      }
    }
    if (it < 3) {
#pragma unroll
      for (int j = 0; j < 9; ++j)
        if (j == im) v[j] = 0.0f;
    } else {
#pragma unroll
      for (int j = 0; j < 9; ++j)
        if (j == im) out = v[j];
    }
  }
  return out;
}

__global__ __launch_bounds__(TPB) void k_median3(const float4* __restrict__ in, float4* __restrict__ out, int w,
                                                 int h) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= w * h) return;
  const int r = i / w, col = i - r * w;
  float R[9], G[9], B[9];
  int k = 0;
#pragma unroll
  for (int dr = -1; dr <= 1; ++dr) {
#pragma unroll
    for (int dc = -1; dc <= 1; ++dc, ++k) {
      const int rr = r + dr, cc = col + dc;
      float4 v = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
      if (rr >= 0 && rr < h && cc >= 0 && cc < w) v = in[rr * w + cc];
      R[k] = v.x;
      G[k] = v.y;
      B[k] = v.z;
    }
  }
  out[i] = make_float4(ref_median_channel(R), ref_median_channel(G), ref_median_channel(B), 1.0f);
}

// The frame pt_get_image hands to the host (the reference's imageData after
// kernelAccumulate, cu:739-742): owned pixel q's sum / spp at its row-major
// position pix_of[q], alpha 1; pixels of other ranks stay as memset (0).
__global__ __launch_bounds__(TPB) void k_frame(const float4* __restrict__ accum, const uint32_t* __restrict__ pix_of,
                                               uint32_t npix, float ns, float4* __restrict__ frame) {
  const uint32_t q = blockIdx.x * TPB + threadIdx.x;
  if (q >= npix) return;
  const float4 a = accum[q];
  frame[pix_of[q]] = make_float4(a.x / ns, a.y / ns, a.z / ns, 1.0f);
}

// Zero n float4s / n words on the context's stream.  Kernels of ours rather
// than hipMemsetAsync: the runtime's fill kernel, queued while a frame's copy
// to the host runs on the copy stream (pt_get_image_async), does not start
// until that copy is nearly done (~300 us: a 16 MB accumulation buffer, or
// the 4-byte path-grab counters in front of the next frame's path kernel).
__global__ __launch_bounds__(TPB) void k_zero(float4* __restrict__ p, uint32_t n) {
  const uint32_t i = blockIdx.x * TPB + threadIdx.x;
  if (i < n) p[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}
__global__ __launch_bounds__(TPB) void k_zero_u32(uint32_t* __restrict__ p, uint32_t n) {
  const uint32_t i = blockIdx.x * TPB + threadIdx.x;
  if (i < n) p[i] = 0u;
}
// (a small device-to-device copy as a kernel of ours, for the same reason)
__global__ __launch_bounds__(TPB) void k_copy_u32(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                  uint32_t n) {
  const uint32_t i = blockIdx.x * TPB + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

}  // namespace pt
