// Shared device helpers for the gfx950 (MI355X / CDNA4) ViT kernels.
// Wave64 everywhere; bf16 handled as raw u16 with hardware RNE conversion (v_cvt_pk_bf16_f32).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <algorithm>

#include "../../include/vit_hip.h"

typedef uint16_t bf16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define VIT_DEV __device__ __forceinline__

// An opaque copy of a per-lane index: values derived from it are recomputed where used instead of being hoisted out
// of a persistent loop.  The persistent kernels run at the 256-VGPR limit, where a hoisted per-lane offset is spilled,
// and a spill reload is a VMEM access whose s_waitcnt vmcnt(0) also drains the LDS-DMA loads in flight.
VIT_DEV int remat(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// (image, head) of attention item u = b * H + h, for 0 <= u < 2^24 (hosts check B * H): a float reciprocal and one
// correction step (|u / H - u * fl(1/H)| < 1 there) instead of a 64-bit integer division, which expands to ~60 scalar
// instructions — the persistent attention kernels split 2-3 item indices per item in every wave.
VIT_DEV void item_bh(int64_t item, int64_t H, int64_t& b, int64_t& h) {
  const int u = (int)item, hh = (int)H;
  int q = (int)((float)u * (1.0f / (float)hh));
  int r = u - q * hh;
  if (r < 0) {
    --q;
    r += hh;
  } else if (r >= hh) {
    ++q;
    r -= hh;
  }
  b = q;
  h = r;
}

VIT_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
VIT_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, __float2bfloat16(f)); }

// Generic load/store of one element of storage type T (float or bf16_t) as float.
template <class T> VIT_DEV float ld1(const T* p);
template <> VIT_DEV float ld1<float>(const float* p) { return *p; }
template <> VIT_DEV float ld1<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <class T> VIT_DEV void st1(T* p, float v);
template <> VIT_DEV void st1<float>(float* p, float v) { *p = v; }
template <> VIT_DEV void st1<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// 4 consecutive elements (8 B for bf16, 16 B for f32); caller guarantees alignment.
template <class T> VIT_DEV void ld4(const T* p, float v[4]);
template <> VIT_DEV void ld4<float>(const float* p, float v[4]) {
  f32x4 x = *reinterpret_cast<const f32x4*>(p);
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
template <> VIT_DEV void ld4<bf16_t>(const bf16_t* p, float v[4]) {
  uint2 x = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
  v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
}
template <class T> VIT_DEV void st4(T* p, const float v[4]);
template <> VIT_DEV void st4<float>(float* p, const float v[4]) {
  f32x4 x = {v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p) = x;
}
template <> VIT_DEV void st4<bf16_t>(bf16_t* p, const float v[4]) {
  uint2 x;
  x.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  x.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = x;
}

// Counter-based dropout hash: murmur3 fmix32 of (idx * 0x9E3779B1 + seed).  Must match oracle.hash_u32.
VIT_DEV uint32_t vit_hash_u32(uint32_t seed, uint32_t idx) {
  uint32_t x = idx * 0x9E3779B1u + seed;
  x ^= x >> 16; x *= 0x85EBCA6Bu;
  x ^= x >> 13; x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}
// VIT_MASK4 bit masks (vit_hip.h): byte ((i/4) * ceil(n/4) + j/4) * 4 + i%4, bit j%4.  A row's 4-column group is one
// byte and a 4-row x 4-column block one dword (byte = row), so a lane owning 4 columns of a row reads or writes a
// byte, and over 4 consecutive rows a whole dword.
VIT_DEV int64_t mask4_byte(int64_t i, int64_t j, int64_t n) { return (((i >> 2) * ((n + 3) >> 2)) + (j >> 2)) * 4 + (i & 3); }

VIT_DEV uint32_t vit_drop_threshold(float p) {
  double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
}

// Wave64 reductions.
VIT_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
VIT_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

VIT_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
VIT_DEV float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// ---------------------------------------------------------------------------------------------------------------
// Host-side error plumbing (thread-local message, nonzero return code).
// ---------------------------------------------------------------------------------------------------------------
namespace vit {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// part[chunk][cols] = column sums of x rows [chunk*rows_per_chunk, ...) (vit_misc.hip; stage 1 of vit_colsum)
void colsum_parts_launch(const void* x, int64_t ldx, int dtype, int64_t rows, int64_t cols, int64_t rows_per_chunk,
                         float* part, hipStream_t s);
}  // namespace vit

// Launch options of vit_set_option (vit_hip.h), read by the host-side launchers.
namespace vit {
enum Opt : int {
  OPT_GEMM_IMPL = 0, OPT_GEMM_TAIL, OPT_GEMM_TAIL_MIN_KT, OPT_SPLITK_MIN_KT, OPT_GEMM_GROUP_M, OPT_GEMM_EPI_GENERAL,
  OPT_GEMM_PERSIST, OPT_ATTN_FWD_SPLIT, OPT_ATTN_BWD_SPLIT, OPT_ATTN_BWD_GRID, OPT_LN16, OPT_LN_AL, OPT_ATTN_FWD_RING,
  OPT_GEMM_TAIL_V2, OPT_SPLITK_ROUNDS, OPT_ATTN_FWD_GRID, OPT_COUNT
};
int64_t opt(Opt o);
}  // namespace vit

// Compute units of the current device (256 on MI355X), queried once per device.
static inline int64_t vit_cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

#define VIT_REQUIRE(cond, ...)                 \
  do {                                         \
    if (!(cond)) {                             \
      vit::set_error(__VA_ARGS__);             \
      return VIT_ERR_INVALID;                  \
    }                                          \
  } while (0)

#define VIT_STREAM(s) (reinterpret_cast<hipStream_t>(s))
