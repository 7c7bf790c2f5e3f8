// Stand-in for a collective's CU footprint (tools/cu_hog_ab.py): `nwg` workgroups of `threads` threads that each hold
// their CU slot for `us` microseconds of wall time (the 100 MHz s_memrealtime counter), then exit.  Used on one GPU to
// measure how the backward's persistent grids and the shared-CU launch mode (VIT_FLAG_SHARED_CUS) behave when other
// kernels occupy some CUs at the time an all-reduce would.  Bounded: every wave exits after `us` (host clamps it).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void cu_hog_kernel(uint64_t ticks, float* sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  float acc = 0.f;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    acc += 1.f;
  }
  if (acc < 0.f) sink[threadIdx.x] = acc;  // never taken; keeps the loop observable
}

extern "C" int cu_hog_launch(int nwg, int threads, double us, void* sink, void* stream) {
  if (nwg < 1 || nwg > 1024 || threads < 64 || threads > 1024 || us <= 0.0 || us > 20000.0) return 1;
  const uint64_t ticks = (uint64_t)(us * 100.0);  // 100 MHz
  hipLaunchKernelGGL(cu_hog_kernel, dim3(nwg), dim3(threads), 0, (hipStream_t)stream, ticks, (float*)sink);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
