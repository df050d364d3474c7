// k_shade_push in a translation unit of its own, compiled without SLP
// vectorisation (-fno-slp-vectorize, see the Makefile).  The SLP pass packs
// independent fp32 operations of the shading and root-pass code into
// v_pk_*_f32 pairs; in this kernel that costs registers (74 VGPRs instead of
// 64) and time (CBbunny shade 101 -> 93 ms without it), while the single-leaf
// kernel in pt_device.hip gains from it (+3 %).  Same operations per element,
// so the same bits either way.
//
// The kernel sources are included inside an anonymous namespace: every kernel
// they define gets internal linkage here, so the copies of the other kernels
// do not clash with pt_device.hip's; only k_shade_push is launched from here.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_api.h"

namespace {
#include "kernels/trace.hip"
#include "kernels/shade.hip"
}  // namespace

// S points at a pt::ShadeArgs of pt_device.hip (the same definition, from the
// same header, so the same layout).  e0/e1: optional dispatch timestamps.
// refa: PT_FLAG_REF_ARITH (the reference's literal arithmetic, shade.hip).
// xl: the extended light model (several / directional / hemisphere lights;
// one NEE sample per vertex, default arithmetic only).
hipError_t pt_launch_shade_push(int nsh, bool refa, bool xl, unsigned grid, hipStream_t stream, hipEvent_t e0,
                                hipEvent_t e1, const void* S) {
  const auto& A = *static_cast<const pt::ShadeArgs*>(S);
  auto k = xl ? pt::k_shade_push<1, false, true>
              : refa ? (nsh == 2 ? pt::k_shade_push<2, true> : pt::k_shade_push<1, true>)
                     : (nsh == 2 ? pt::k_shade_push<2, false> : pt::k_shade_push<1, false>);
  if (e0)
    hipExtLaunchKernelGGL(k, dim3(grid), dim3(pt::TPB), 0, stream, e0, e1, 0, A);
  else
    hipLaunchKernelGGL(k, dim3(grid), dim3(pt::TPB), 0, stream, A);
  return hipGetLastError();
}
