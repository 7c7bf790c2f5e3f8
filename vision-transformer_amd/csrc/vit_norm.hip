// LayerNorm forward/backward (nn.LayerNorm, eps 1e-5; transformer.py:71-72,77-78 and vit.py:72).
// One wave64 per row, the row cached in registers (NV float4 per lane, cols <= 256*NV), fp32 statistics with an
// exact two-pass variance.  Backward fuses: residual-gradient add, the producer branch's dropout backward, and
// per-workgroup dgamma/dbeta partials (reduced afterwards by vit_colsum in a fixed order).
#include "vit_common.h"

namespace {

constexpr int LN_BWD_PARTS_MAX = 2048;
#ifndef LN_BWD_RPB
#define LN_BWD_RPB 32       // rows per backward block (its dgamma / dbeta partial covers them); 16 and 64 measured slower
#endif

template <class T, int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     T* __restrict__ y, int64_t ldy, float* __restrict__ mean,
                                                     float* __restrict__ rstd, int64_t rows, int64_t cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * ldx;
  float v[NV][4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t c = ((int64_t)k * 64 + lane) * 4;
    if (c < cols) {
      ld4<T>(xr + c, v[k]);
      s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
    } else {
      v[k][0] = v[k][1] = v[k][2] = v[k][3] = 0.f;
    }
  }
  const float mu = wave_sum(s) / (float)cols;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t c = ((int64_t)k * 64 + lane) * 4;
    if (c < cols) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = v[k][r] - mu;
        q += d * d;
      }
    }
  }
  const float var = wave_sum(q) / (float)cols;
  const float rs = rsqrtf(var + eps);
  T* yr = y + row * ldy;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t c = ((int64_t)k * 64 + lane) * 4;
    if (c < cols) {
      float g[4], b[4], o[4];
      ld4<float>(gamma + c, g);
      ld4<float>(beta + c, b);
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (v[k][r] - mu) * rs * g[r] + b[r];
      st4<T>(yr + c, o);
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// 4 consecutive values of T held as loaded (bf16: 2 dwords), unpacked to fp32 when used
template <class T> struct Raw4;
template <> struct Raw4<bf16_t> {
  using type = uint2;
  static VIT_DEV uint2 zero() { return make_uint2(0u, 0u); }
  static VIT_DEV uint2 load(const bf16_t* p) { return *reinterpret_cast<const uint2*>(p); }
  static VIT_DEV void unpack(uint2 u, float (&v)[4]) {
    v[0] = __uint_as_float(u.x << 16);
    v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16);
    v[3] = __uint_as_float(u.y & 0xffff0000u);
  }
};
template <> struct Raw4<float> {
  using type = f32x4;
  static VIT_DEV f32x4 zero() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
  static VIT_DEV f32x4 load(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
  static VIT_DEV void unpack(f32x4 u, float (&v)[4]) {
    v[0] = u[0];
    v[1] = u[1];
    v[2] = u[2];
    v[3] = u[3];
  }
};

// the value of v as stored in T (bf16 rounds to nearest even)
template <class T> VIT_DEV float as_stored(float v) { return sizeof(T) == 2 ? bf2f(f2bf(v)) : v; }

// AL (accumulators in LDS): the per-column dgamma / dbeta / output sums of each wave live in its own LDS region instead
// of 3 x 4 x NV registers per lane; each lane only ever touches its own columns, so the row loop needs no barrier.
// LDS per 256-thread block is 13 KiB x NV (red[4][3][256 NV] + gamma), so the occupancy it allows is NV-dependent:
// D = 768 (NV 3, 39 KiB): 4 blocks = 4 waves per SIMD, the register form's 3 without spills (one more row of loads in
// flight per SIMD; the measured gain); D = 1024 (NV 4, 52 KiB): 3 blocks = 3 waves per SIMD; NV 6-12
// (78-156 KiB: the head's LN(4D) rows): 1-2 blocks.  The wide fp32 rows use it because their register form spilled
// ~350 VGPRs (209 -> 26.5 us); the bf16 NV 4-12 shapes are not on the C2 step (ViT-L's D = 1024 is: 3 waves / SIMD).
template <class T, int NV, bool AL>
__global__ __launch_bounds__(256, AL && NV <= 4 ? 4 : 1) void ln_bwd_kernel(const T* __restrict__ dy, int64_t lddy, const T* __restrict__ x,
                                                     int64_t ldx, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const T* __restrict__ dres, T* __restrict__ dx_out,
                                                     T* __restrict__ drop_out, uint32_t drop_thr, float drop_scale,
                                                     uint32_t drop_seed, const uint8_t* __restrict__ drop_mask,
                                                     float* __restrict__ partial, int osum,
                                                     int64_t parts, int64_t rows, int64_t cols) {
  __shared__ __attribute__((aligned(16))) float red[AL ? 4 : 1][3][256 * NV];
  __shared__ __attribute__((aligned(16))) float gms[AL ? 256 * NV : 4];     // AL: gamma, read per row from LDS
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (AL) {
    for (int c = threadIdx.x * 4; c < 256 * NV; c += 1024) {
      float g4[4] = {0.f, 0.f, 0.f, 0.f};
      if (c < cols) ld4<float>(gamma + c, g4);
      *reinterpret_cast<f32x4*>(&gms[c]) = f32x4{g4[0], g4[1], g4[2], g4[3]};
    }
    __syncthreads();
  }
  // whole groups of 4 rows per block and per wave step: a wave's 4 consecutive rows share one dword of a mask4
  const int64_t rows_per_part = (((rows + parts - 1) / parts) + 3) & ~(int64_t)3;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_part, r1 = min(rows, r0 + rows_per_part);
  float dg[NV][4], db[NV][4], os[NV][4], gm[NV][4];
  uint32_t mw[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) mw[k] = 0u;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t c = ((int64_t)k * 64 + lane) * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) dg[k][r] = db[k][r] = os[k][r] = 0.f;
    if (AL)
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) *reinterpret_cast<f32x4*>(&red[AL ? w : 0][s2][(k * 64 + lane) * 4]) = f32x4{};
    if (AL) gm[k][0] = gm[k][1] = gm[k][2] = gm[k][3] = 0.f;      // unused: gms
    else if (c < cols) ld4<float>(gamma + c, gm[k]);
    else gm[k][0] = gm[k][1] = gm[k][2] = gm[k][3] = 0.f;
  }
  // Wave w walks rows r0 + 4w + 16q + (0..3), q = 0, 1, ...: the next row's x / dy / residual (raw, packed) and mask
  // dword are loaded while the current row is reduced and stored — one memory latency per wave, not one per row.
  auto row_of = [&](int64_t n) { return r0 + 4 * (w + 4 * (n >> 2)) + (n & 3); };
  using R4 = typename Raw4<T>::type;
  R4 xc[NV], dc[NV], rc[NV], xn[NV], dn[NV], rn[NV];
  uint32_t mn[NV];
  float mu_n = 0.f, rs_n = 0.f;
  auto load_row = [&](int64_t row, R4 (&xa)[NV], R4 (&da)[NV], R4 (&ra)[NV], uint32_t (&ma)[NV], float& mu_,
                      float& rs_) {
    mu_ = mean[row];
    rs_ = rstd[row];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = ((int64_t)k * 64 + lane) * 4;
      xa[k] = da[k] = ra[k] = Raw4<T>::zero();
      if (c < cols) {
        xa[k] = Raw4<T>::load(x + row * ldx + c);
        da[k] = Raw4<T>::load(dy + row * lddy + c);
        if (dres) ra[k] = Raw4<T>::load(dres + row * cols + c);
        if (drop_mask && (row & 3) == 0)
          ma[k] = *reinterpret_cast<const uint32_t*>(drop_mask + mask4_byte(row, c, cols));
      }
    }
  };
  if (row_of(0) < r1) load_row(row_of(0), xn, dn, rn, mn, mu_n, rs_n);
  for (int64_t n = 0; row_of(n) < r1; ++n) {
    const int64_t row = row_of(n);
    const float mu = mu_n, rs = rs_n;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      xc[k] = xn[k];
      dc[k] = dn[k];
      rc[k] = rn[k];
      if ((row & 3) == 0) mw[k] = mn[k];
    }
    if (row_of(n + 1) < r1) load_row(row_of(n + 1), xn, dn, rn, mn, mu_n, rs_n);
    float xv[NV][4], dv[NV][4], rv[NV][4];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      Raw4<T>::unpack(xc[k], xv[k]);
      Raw4<T>::unpack(dc[k], dv[k]);
      Raw4<T>::unpack(rc[k], rv[k]);
    }
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if (AL) {
        const f32x4 g4 = *reinterpret_cast<const f32x4*>(&gms[(k * 64 + lane) * 4]);
        gm[k][0] = g4[0];
        gm[k][1] = g4[1];
        gm[k][2] = g4[2];
        gm[k][3] = g4[3];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {          // columns past `cols` have dv = gm = 0: they add exact zeros
        const float xh = (xv[k][r] - mu) * rs;
        const float g = dv[k][r] * gm[k][r];
        sa += g;
        sb += g * xh;
        if (!AL) {
          dg[k][r] += dv[k][r] * xh;
          db[k][r] += dv[k][r];
        }
        xv[k][r] = xh;
        dv[k][r] = g;
      }
      if (AL) {
        // the raw values are still in dc (dy) / xv (xhat): dg += dy * xhat, db += dy
        float dyv[4];
        Raw4<T>::unpack(dc[k], dyv);
        f32x4* pg = reinterpret_cast<f32x4*>(&red[AL ? w : 0][0][(k * 64 + lane) * 4]);
        f32x4* pb = reinterpret_cast<f32x4*>(&red[AL ? w : 0][1][(k * 64 + lane) * 4]);
        f32x4 ag = *pg, ab = *pb;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ag[r] += dyv[r] * xv[k][r];
          ab[r] += dyv[r];
        }
        *pg = ag;
        *pb = ab;
      }
    }
    const float a = wave_sum(sa) / (float)cols;
    const float b = wave_sum(sb) / (float)cols;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = ((int64_t)k * 64 + lane) * 4;
      if (c < cols) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = rs * (dv[k][r] - a - xv[k][r] * b) + rv[k][r];
        st4<T>(dx_out + row * cols + c, o);
        if (drop_out) {
          // the dropout mask on the value as stored, WITHOUT the 1/(1-p) scale: exact in any dtype (the scale is
          // applied by the consumers — GEMM alpha, and the column sums below), so the masked gradient adds no
          // rounding of its own
          float dd[4];
          if (drop_mask) {                    // the forward's keep bits (mask4 of the producing GEMM's dropout)
#pragma unroll
            for (int r = 0; r < 4; ++r) dd[r] = (mw[k] >> (8 * (row & 3) + r)) & 1u ? as_stored<T>(o[r]) : 0.f;
          } else {
            const uint32_t base = (uint32_t)(row * cols + c);
#pragma unroll
            for (int r = 0; r < 4; ++r) dd[r] = vit_hash_u32(drop_seed, base + r) >= drop_thr ? as_stored<T>(o[r]) : 0.f;
          }
          st4<T>(drop_out + row * cols + c, dd);
          if (osum) {
            if (AL) {
              f32x4* po = reinterpret_cast<f32x4*>(&red[AL ? w : 0][2][(k * 64 + lane) * 4]);
              f32x4 ao = *po;
#pragma unroll
              for (int r = 0; r < 4; ++r) ao[r] += dd[r];
              *po = ao;
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) os[k][r] += dd[r];
            }
          }
        } else if (osum) {
          if (AL) {
            f32x4* po = reinterpret_cast<f32x4*>(&red[AL ? w : 0][2][(k * 64 + lane) * 4]);
            f32x4 ao = *po;
#pragma unroll
            for (int r = 0; r < 4; ++r) ao[r] += as_stored<T>(o[r]);
            *po = ao;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) os[k][r] += as_stored<T>(o[r]);
          }
        }
      }
    }
  }
  const int nset = osum ? 3 : 2;
  const float oscale = drop_out ? drop_scale : 1.f;   // set 2 = column sums of drop_out * 1/(1-p)
  if (AL) {                                           // the 4 wave regions, added in a fixed order
    __syncthreads();
    for (int64_t c = threadIdx.x; c < cols; c += 256)
      for (int s2 = 0; s2 < nset; ++s2) {
        const float v = ((red[0][s2][c] + red[AL ? 1 : 0][s2][c]) + red[AL ? 2 : 0][s2][c]) + red[AL ? 3 : 0][s2][c];
        partial[(s2 * parts + blockIdx.x) * cols + c] = s2 == 2 ? v * oscale : v;
      }
    return;
  }
  // per-block partial sums: waves add into LDS in a fixed order (0, 1, 2, 3) -> bitwise reproducible
  for (int turn = 0; turn < 4; ++turn) {
    if (w == turn) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cc = (k * 64 + lane) * 4 + r;
          if (turn == 0) {
            red[0][0][cc] = dg[k][r];
            red[0][1][cc] = db[k][r];
            red[0][2][cc] = os[k][r];
          } else {
            red[0][0][cc] += dg[k][r];
            red[0][1][cc] += db[k][r];
            red[0][2][cc] += os[k][r];
          }
        }
      }
    }
    __syncthreads();
  }
  for (int64_t c = threadIdx.x; c < cols; c += 256)
    for (int s = 0; s < nset; ++s) partial[(s * parts + blockIdx.x) * cols + c] = s == 2 ? red[0][s][c] * oscale : red[0][s][c];
}

// ---------------------------------------------------------------------------------------------------------------
// bf16, 16 B per lane: a wave takes two rows at once (lanes 0-31 row 2p, lanes 32-63 row 2p + 1), each lane 8
// consecutive columns of every 256-column piece, so every load and store instruction moves 1 KiB (the 8-B-per-lane
// form moved 512 B and held both LayerNorm kernels near 3.5-3.9 TB/s).  Row statistics are half-wave reductions.
// Waves loop over row pairs with the next pair's operands in flight.  Used when cols and every row stride are
// multiples of 8 (16-B aligned rows); the kernels above cover the rest and fp32.  Measured (tools/ln_bench.py,
// 50432 x 768): 39-41 -> 38 us.  The same layout for the backward (and a 64-lane form with 16-B pairs of quads) was
// slower than ln_bwd_kernel (97-120 vs 82-102 us): its per-lane accumulators cost occupancy.
// ---------------------------------------------------------------------------------------------------------------
VIT_DEV float half_sum(float v) {          // sum over the 32 lanes of this half-wave
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

VIT_DEV void unpack8(uint4 u, float (&a)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a[2 * q] = __uint_as_float(w[q] << 16);
    a[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}

VIT_DEV uint4 pack8(const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = (uint32_t)f2bf(v[2 * q]) | ((uint32_t)f2bf(v[2 * q + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

VIT_DEV void ld8f(const float* p, float (&v)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}

template <int NV>
__global__ __launch_bounds__(256) void ln_fwd16_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       bf16_t* __restrict__ y, int64_t ldy, float* __restrict__ mean,
                                                       float* __restrict__ rstd, int64_t rows, int64_t cols, float eps) {
  const int lane = threadIdx.x & 63, l = lane & 31, hr = lane >> 5;
  const int64_t npairs = (rows + 1) >> 1, stride = (int64_t)gridDim.x * 4;
  int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= npairs) return;
  uint4 nx[NV];
  auto load = [&](int64_t pp) {
    const int64_t row = 2 * pp + hr;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t c = (int64_t)k * 256 + 8 * l;
      nx[k] = make_uint4(0u, 0u, 0u, 0u);
      if (row < rows && c < cols) nx[k] = *reinterpret_cast<const uint4*>(x + row * ldx + c);
    }
  };
  load(p);
  for (; p < npairs; p += stride) {
    float v[NV][8];
#pragma unroll
    for (int k = 0; k < NV; ++k) unpack8(nx[k], v[k]);
    if (p + stride < npairs) load(p + stride);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int r = 0; r < 8; ++r) s += v[k][r];
    const float mu = half_sum(s) / (float)cols;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if ((int64_t)k * 256 + 8 * l < cols) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float d = v[k][r] - mu;
          q += d * d;
        }
      }
    }
    const float rs = rsqrtf(half_sum(q) / (float)cols + eps);
    const int64_t row = 2 * p + hr;
    if (row < rows) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int64_t c = (int64_t)k * 256 + 8 * l;
        if (c < cols) {
          float g[8], b[8], o[8];
          ld8f(gamma + c, g);
          ld8f(beta + c, b);
#pragma unroll
          for (int r = 0; r < 8; ++r) o[r] = (v[k][r] - mu) * rs * g[r] + b[r];
          *reinterpret_cast<uint4*>(y + row * ldy + c) = pack8(o);
        }
      }
      if (l == 0) {
        mean[row] = mu;
        rstd[row] = rs;
      }
    }
  }
}

// the 16-B forward applies: bf16, cols and every row stride multiples of 8, 16-B aligned base pointers
static bool ln16_ok(int64_t cols, std::initializer_list<int64_t> lds, std::initializer_list<const void*> ptrs) {
  if (!vit::opt(vit::OPT_LN16) || cols % 8) return false;
  for (int64_t ld : lds)
    if (ld % 8) return false;
  for (const void* p : ptrs)
    if (reinterpret_cast<uintptr_t>(p) % 16) return false;
  return true;
}

template <int NV, class T>
int ln_fwd_launch(const T* x, int64_t ldx, const float* g, const float* b, T* y, int64_t ldy, float* mean,
                  float* rstd, int64_t rows, int64_t cols, float eps, hipStream_t s) {
  if constexpr (sizeof(T) == 2) {
    if (ln16_ok(cols, {ldx, ldy}, {x, y})) {
      // pairs of rows, 4 per block; enough blocks for 8 waves per SIMD, each wave looping over its pairs
      const int64_t blocks = ((rows + 1) / 2 + 3) / 4;
      const unsigned grid = (unsigned)std::min<int64_t>(blocks, vit_cu_count() * 8);
      ln_fwd16_kernel<NV><<<grid, 256, 0, s>>>(x, ldx, g, b, y, ldy, mean, rstd, rows, cols, eps);
      return 0;
    }
  }
  const unsigned grid = (unsigned)((rows + 3) / 4);
  ln_fwd_kernel<T, NV><<<grid, 256, 0, s>>>(x, ldx, g, b, y, ldy, mean, rstd, rows, cols, eps);
  return 0;
}

}  // namespace

extern "C" int64_t vit_layernorm_bwd_parts(int64_t rows, int64_t cols) {
  (void)cols;
  int64_t p = (rows + LN_BWD_RPB - 1) / LN_BWD_RPB;  // up to 2048 blocks
  // few rows (the classifier head's LN: B rows x 4D): spread them, >= 4 rows per block, up to 256 blocks
  if (p < 256) p = std::max<int64_t>(p, std::min<int64_t>(256, (rows + 3) / 4));
  if (p > LN_BWD_PARTS_MAX) p = LN_BWD_PARTS_MAX;
  if (p < 1) p = 1;
  return p;
}

#define NV_SWITCH(cols, CALL)                                           \
  switch ((int)(((cols) + 255) / 256)) {                                 \
    case 1: CALL(1); break;                                              \
    case 2: CALL(2); break;                                              \
    case 3: CALL(3); break;                                              \
    case 4: CALL(4); break;                                              \
    case 5: case 6: CALL(6); break;                                      \
    case 7: case 8: CALL(8); break;                                      \
    case 9: case 10: case 11: case 12: CALL(12); break;                  \
    case 13: case 14: case 15: case 16: CALL(16); break;                 \
    default: vit::set_error("layernorm: cols=%lld too large", (long long)(cols)); return VIT_ERR_INVALID; \
  }

extern "C" int vit_layernorm_fwd(const void* x, int64_t ldx, const float* gamma, const float* beta, void* y,
                                 int64_t ldy, float* mean, float* rstd, int64_t rows, int64_t cols, float eps,
                                 int32_t dtype, void* stream) {
  VIT_REQUIRE(x && gamma && beta && y && mean && rstd && rows > 0 && cols > 0, "vit_layernorm_fwd: bad arguments");
  VIT_REQUIRE(cols % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0, "vit_layernorm_fwd: cols/ld must be multiples of 4");
  hipStream_t s = VIT_STREAM(stream);
  if (dtype == VIT_BF16) {
#define CALLB(NV) ln_fwd_launch<NV, bf16_t>((const bf16_t*)x, ldx, gamma, beta, (bf16_t*)y, ldy, mean, rstd, rows, cols, eps, s)
    NV_SWITCH(cols, CALLB)
#undef CALLB
  } else {
#define CALLF(NV) ln_fwd_launch<NV, float>((const float*)x, ldx, gamma, beta, (float*)y, ldy, mean, rstd, rows, cols, eps, s)
    NV_SWITCH(cols, CALLF)
#undef CALLF
  }
  return vit::check_launch("vit_layernorm_fwd");
}

extern "C" int vit_layernorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* gamma,
                                 const float* mean, const float* rstd, const void* dres, void* dx_out,
                                 void* drop_out, float drop_p, uint32_t drop_seed, const void* drop_mask,
                                 float* partial, int32_t osum,
                                 int64_t rows, int64_t cols, int32_t dtype, void* stream) {
  VIT_REQUIRE(dy && x && gamma && mean && rstd && dx_out && partial && rows > 0 && cols > 0,
              "vit_layernorm_bwd: bad arguments");
  VIT_REQUIRE(cols % 4 == 0 && lddy % 4 == 0 && ldx % 4 == 0, "vit_layernorm_bwd: cols/ld must be multiples of 4");
  VIT_REQUIRE(cols <= 4096, "vit_layernorm_bwd: cols=%lld > 4096", (long long)cols);
  VIT_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "vit_layernorm_bwd: drop_p out of range");
  const int64_t parts = vit_layernorm_bwd_parts(rows, cols);
  double t = (double)drop_p * 4294967296.0;
  const uint32_t thr = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  const float scale = 1.0f / (1.0f - drop_p);
  hipStream_t s = VIT_STREAM(stream);
  // bf16 rows up to 3072 columns: per-wave accumulators in LDS (13 KiB x NV per block); option ln_al 0: registers
  const bool al = vit::opt(vit::OPT_LN_AL) != 0;
  if (dtype == VIT_BF16) {
#define CALLB(NV)                                                                                                 \
  if (al && NV <= 12)                                                                                             \
    ln_bwd_kernel<bf16_t, NV, (NV <= 12)><<<(unsigned)parts, 256, 0, s>>>(                                         \
        (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, gamma, mean, rstd, (const bf16_t*)dres, (bf16_t*)dx_out,  \
        (bf16_t*)drop_out, thr, scale, drop_seed, (const uint8_t*)drop_mask, partial, osum != 0, parts, rows, cols); \
  else                                                                                                            \
    ln_bwd_kernel<bf16_t, NV, false><<<(unsigned)parts, 256, 0, s>>>(                                             \
        (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, gamma, mean, rstd, (const bf16_t*)dres, (bf16_t*)dx_out,  \
        (bf16_t*)drop_out, thr, scale, drop_seed, (const uint8_t*)drop_mask, partial, osum != 0, parts, rows, cols)
    NV_SWITCH(cols, CALLB)
#undef CALLB
  } else {
  // fp32 (the parity path and the classifier head's LN(4D)): LDS accumulators for the wide rows (NV 6-12), whose
  // register form spilled ~350 VGPRs (the head's LN backward, B x 3072: 133 -> 26.5 us)
#define CALLF(NV)                                                                                            \
  if (NV >= 6 && NV <= 12 && al)                                                  \
    ln_bwd_kernel<float, NV, (NV >= 6 && NV <= 12)><<<(unsigned)parts, 256, 0, s>>>(                         \
        (const float*)dy, lddy, (const float*)x, ldx, gamma, mean, rstd, (const float*)dres, (float*)dx_out, \
        (float*)drop_out, thr, scale, drop_seed, (const uint8_t*)drop_mask, partial, osum != 0, parts, rows, cols); \
  else                                                                                                       \
    ln_bwd_kernel<float, NV, false><<<(unsigned)parts, 256, 0, s>>>(                                         \
        (const float*)dy, lddy, (const float*)x, ldx, gamma, mean, rstd, (const float*)dres, (float*)dx_out, \
        (float*)drop_out, thr, scale, drop_seed, (const uint8_t*)drop_mask, partial, osum != 0, parts, rows, cols)
    NV_SWITCH(cols, CALLF)
#undef CALLF
  }
  return vit::check_launch("vit_layernorm_bwd");
}
