// Multi-head self-attention forward/backward for the ViT encoder (transformer.py:9-31, :44-45).
// Reference semantics: logits are MULTIPLIED by sqrt(hd) (`scale` argument), no mask, softmax over keys.
//
// qkv[B*T][3D]: Q at column h*hd, K at D + h*hd, V at 2D + h*hd.  o[B*T][D].  lse[B][H][T] (natural log).
//
// bf16, hd == 64 — flash-style MFMA kernels (v_mfma_f32_32x32x16_bf16, wave64):
//   forward: workgroup = 4 waves x 32 queries; K/V tiles of 64 keys double-buffered in LDS; S^T = K.Q^T so each lane
//   owns one query's column (softmax statistics are per-lane scalars), P^T is reused in registers as the B operand
//   of O^T = V^T.P^T (no LDS round trip for P); V^T fragments come from ds_read_b64_tr_b16 transposed reads.
//   backward: dQ kernel (queries on lanes, K/V streamed) and dK/dV kernel (keys on lanes, Q/dO streamed); P is
//   recomputed from the saved LSE; no atomics, deterministic.
//   LDS images are [row][64 bf16] with a 16-B chunk XOR swizzle that is conflict-free for both the ds_read_b128 row
//   reads and the transposed reads.
// Other dtypes / head sizes — generic VALU kernels (exact fp32 arithmetic order per row), also used when the
// `.attention_probs` tensor is requested.
#include <stdlib.h>

#include "vit_common.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;

// ===============================================================================================================
// Generic VALU kernels
// ===============================================================================================================
constexpr int GA_TMAX = 2048;
constexpr int GA_HDMAX = 128;

template <class T>
__global__ __launch_bounds__(256) void attn_fwd_generic(const T* __restrict__ qkv, T* __restrict__ o,
                                                        float* __restrict__ lse, float* __restrict__ probs, int64_t B,
                                                        int64_t Tn, int64_t H, int64_t hd, float scale,
                                                        float* __restrict__ o32 = nullptr) {
  __shared__ float sc[4][GA_TMAX];
  __shared__ float qs[4][GA_HDMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t bh = blockIdx.y, b = bh / H, h = bh % H;
  const int64_t qv = (int64_t)blockIdx.x * 4 + w;
  const bool valid = qv < Tn;          // no early exit: every wave reaches the barriers
  const int64_t q = valid ? qv : Tn - 1;
  const int64_t D = H * hd, ld = 3 * D;
  const T* base = qkv + b * Tn * ld;
  for (int d = lane; d < hd; d += 64) qs[w][d] = ld1<T>(base + q * ld + h * hd + d);
  __syncthreads();
  float mx = -INFINITY;
  for (int64_t j = lane; j < Tn; j += 64) {
    const T* kr = base + j * ld + D + h * hd;
    float s = 0.f;
    for (int d = 0; d < hd; ++d) s += qs[w][d] * ld1<T>(kr + d);
    s *= scale;
    sc[w][j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float l = 0.f;
  for (int64_t j = lane; j < Tn; j += 64) {
    const float p = expf(sc[w][j] - mx);
    sc[w][j] = p;
    l += p;
  }
  l = wave_sum(l);
  const float inv = 1.0f / l;
  for (int64_t j = lane; j < Tn; j += 64) {
    const float p = sc[w][j] * inv;
    sc[w][j] = p;
    if (probs && valid) probs[(bh * Tn + q) * Tn + j] = p;
  }
  __syncthreads();
  for (int d = lane; d < hd; d += 64) {
    float acc = 0.f;
    for (int64_t j = 0; j < Tn; ++j) acc += sc[w][j] * ld1<T>(base + j * ld + 2 * D + h * hd + d);
    if (valid) st1<T>(o + (b * Tn + q) * D + h * hd + d, acc);
    if (valid && o32) o32[(b * Tn + q) * D + h * hd + d] = acc;
  }
  if (lane == 0 && valid) lse[bh * Tn + q] = mx + logf(l);
}

// Backward A: one wave per query row: P, dP, dS rows (dS and P to workspace) and the dQ row.
template <class T>
__global__ __launch_bounds__(256) void attn_bwd_generic_rows(const T* __restrict__ qkv, const T* __restrict__ o,
                                                             const T* __restrict__ d_o, const float* __restrict__ lse,
                                                             T* __restrict__ dqkv, float* __restrict__ Pws,
                                                             float* __restrict__ dSws, int64_t B, int64_t Tn,
                                                             int64_t H, int64_t hd, float scale,
                                                             const float* __restrict__ o32 = nullptr) {
  __shared__ float ds_s[4][GA_TMAX];
  __shared__ float qs[4][GA_HDMAX];
  __shared__ float dos[4][GA_HDMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t bh = blockIdx.y, b = bh / H, h = bh % H;
  const int64_t qv = (int64_t)blockIdx.x * 4 + w;
  const bool valid = qv < Tn;
  const int64_t q = valid ? qv : Tn - 1;
  const int64_t D = H * hd, ld = 3 * D;
  const T* base = qkv + b * Tn * ld;
  float dl = 0.f;
  for (int d = lane; d < hd; d += 64) {
    qs[w][d] = ld1<T>(base + q * ld + h * hd + d);
    const float g = ld1<T>(d_o + (b * Tn + q) * D + h * hd + d);
    dos[w][d] = g;
    dl += g * (o32 ? o32[(b * Tn + q) * D + h * hd + d] : ld1<T>(o + (b * Tn + q) * D + h * hd + d));
  }
  dl = wave_sum(dl);
  __syncthreads();
  const float L = lse[bh * Tn + q];
  for (int64_t j = lane; j < Tn; j += 64) {
    const T* kr = base + j * ld + D + h * hd;
    const T* vr = base + j * ld + 2 * D + h * hd;
    float s = 0.f, dp = 0.f;
    for (int d = 0; d < hd; ++d) {
      s += qs[w][d] * ld1<T>(kr + d);
      dp += dos[w][d] * ld1<T>(vr + d);
    }
    const float p = expf(s * scale - L);
    const float ds = p * (dp - dl);
    ds_s[w][j] = ds;
    if (valid) {
      Pws[(bh * Tn + q) * Tn + j] = p;
      dSws[(bh * Tn + q) * Tn + j] = ds;
    }
  }
  __syncthreads();
  for (int d = lane; d < hd; d += 64) {
    float acc = 0.f;
    for (int64_t j = 0; j < Tn; ++j) acc += ds_s[w][j] * ld1<T>(base + j * ld + D + h * hd + d);
    if (valid) st1<T>(dqkv + (b * Tn + q) * ld + h * hd + d, acc * scale);
  }
}

// Backward B: one wave per key row: dK row = scale * sum_q dS[q][j] Q[q], dV row = sum_q P[q][j] dO[q].
template <class T>
__global__ __launch_bounds__(256) void attn_bwd_generic_cols(const T* __restrict__ qkv, const T* __restrict__ d_o,
                                                             T* __restrict__ dqkv, const float* __restrict__ Pws,
                                                             const float* __restrict__ dSws, int64_t B, int64_t Tn,
                                                             int64_t H, int64_t hd, float scale) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t bh = blockIdx.y, b = bh / H, h = bh % H;
  const int64_t j = (int64_t)blockIdx.x * 4 + w;
  if (j >= Tn) return;
  const int64_t D = H * hd, ld = 3 * D;
  const T* base = qkv + b * Tn * ld;
  for (int d = lane; d < hd; d += 64) {
    float dk = 0.f, dv = 0.f;
    for (int64_t q = 0; q < Tn; ++q) {
      const float ds = dSws[(bh * Tn + q) * Tn + j];
      const float p = Pws[(bh * Tn + q) * Tn + j];
      dk += ds * ld1<T>(base + q * ld + h * hd + d);
      dv += p * ld1<T>(d_o + (b * Tn + q) * D + h * hd + d);
    }
    st1<T>(dqkv + (b * Tn + j) * ld + D + h * hd + d, dk * scale);
    st1<T>(dqkv + (b * Tn + j) * ld + 2 * D + h * hd + d, dv);
  }
}

// ===============================================================================================================
// bf16, hd = 64 MFMA kernels
// ===============================================================================================================
constexpr int HD = 64;
constexpr int KT = 64;                 // keys (or queries) per streamed LDS tile
constexpr int TILE = KT * HD;          // 4096 bf16 = 8 KiB

VIT_DEV int aswz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }

typedef short s16x4_lds __attribute__((ext_vector_type(4)));
VIT_DEV s16x4 tr_read(const bf16_t* p) {
  typedef __attribute__((address_space(3))) s16x4_lds* lds_ptr_t;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ptr_t)p);
}

// Stage a 64-row x 64-col bf16 tile (rows r0.., columns col0..col0+63 of a row-major matrix with leading dim ld,
// rows >= nrows zero-filled) through registers.
VIT_DEV void tile_load(const bf16_t* __restrict__ src, int64_t ld, int64_t r0, int64_t nrows, int64_t col0, int tid,
                       uint4 (&reg)[2]) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int q = tid + 256 * it;
    const int64_t r = r0 + (q >> 3);
    const int c = q & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < nrows) v = *reinterpret_cast<const uint4*>(src + r * ld + col0 + c * 8);
    reg[it] = v;
  }
}
VIT_DEV void tile_store(bf16_t* lds, int tid, const uint4 (&reg)[2]) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int q = tid + 256 * it;
    const int r = q >> 3, c = q & 7;
    *reinterpret_cast<uint4*>(lds + r * HD + ((c ^ aswz(r)) << 3)) = reg[it];
  }
}

// The same 64-row tile by LDS-DMA (global_load_lds_dwordx4: no staging registers, no ds_write): 8 pieces of 8 rows,
// wave w of the 4 issues pieces 2w and 2w + 1, lane-linear destination with the chunk swizzle applied to the source
// address (the layout tile_store writes; aswz(r) = aswz(r mod 64)).  Rows >= nrows are clamped to nrows - 1: finite
// data, and every caller masks those rows (keys: S = -inf or dS = 0; queries: lse = +inf).  Issued as inline asm so
// the compiler's waitcnt pass does not drain it at the LDS reads of the other buffer; the caller retires it with
// tile_wait() before the barrier that publishes the buffer.
VIT_DEV void tile_dma(const bf16_t* __restrict__ src, int64_t ld, int64_t r0, int64_t nrows, int64_t col0, bf16_t* img,
                      int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pc = 2 * wave + i;
    const int rl = pc * 8 + (lane >> 3);
    const int c = (lane & 7) ^ aswz(rl);
    const bf16_t* g = src + min(r0 + rl, nrows - 1) * ld + col0 + c * 8;
    const uint32_t lds = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(img + pc * 512));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds) : "memory", "m0");
#pragma clang diagnostic pop
  }
}
VIT_DEV void tile_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 32x32x16 operand fragment from a [row][64] tile, rows rb..rb+31, k-step s (d = 16s..16s+15):
// lane holds X[rb + (lane&31)][16s + 8(lane>>5) + 0..7]
VIT_DEV bf16x8_t row_frag(const bf16_t* t, int rb, int s, int lane) {
  const int r = rb + (lane & 31);
  const int c = 2 * s + (lane >> 5);
  s16x8 v = *reinterpret_cast<const s16x8*>(t + r * HD + ((c ^ aswz(r)) << 3));
  return __builtin_bit_cast(bf16x8_t, v);
}

// Transposed fragment: A operand of Y[d][x] += sum_row X^T... i.e. lane (row d = db*32 + (lane&31), half h) element j
// = t[rb + 8(j>>2) + 4h + (j&3)][db*32 + (lane&31)] — matches the k order of an accumulator used as B operand.
VIT_DEV bf16x8_t tr_frag(const bf16_t* t, int rb, int db, int lane) {
  const int G = lane >> 4, hh = G >> 1, lg = lane & 15, q = lg >> 2, p = lg & 3;
  const int r1 = rb + 4 * hh + q, r2 = r1 + 8;
  const int col = db * 32 + 16 * (G & 1) + 4 * p;
  const int c = col >> 3;
  s16x4 lo = tr_read(t + r1 * HD + ((c ^ aswz(r1)) << 3) + (p & 1) * 4);
  s16x4 hi = tr_read(t + r2 * HD + ((c ^ aswz(r2)) << 3) + (p & 1) * 4);
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// Fragment straight from global: lane holds X[row0 + (lane&31)][col0 + 16s + 8(lane>>5) + 0..7] (zero past nrows)
VIT_DEV bf16x8_t glb_frag(const bf16_t* __restrict__ src, int64_t ld, int64_t row0, int64_t nrows, int64_t col0,
                          int s, int lane) {
  const int64_t r = row0 + (lane & 31);
  s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r < nrows) v = *reinterpret_cast<const s16x8*>(src + r * ld + col0 + 16 * s + 8 * (lane >> 5));
  return __builtin_bit_cast(bf16x8_t, v);
}

// 8 consecutive accumulator registers (8s2 .. 8s2+7) -> bf16 B fragment (v_cvt_pk_bf16_f32 pairs: RNE, as f2bf)
typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
typedef float f32x2_v __attribute__((ext_vector_type(2)));
VIT_DEV bf16x8_t pack8(const float* x) {
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    w[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_v{x[2 * q], x[2 * q + 1]}, bf16x2_v));
  return __builtin_bit_cast(bf16x8_t, make_uint4(w[0], w[1], w[2], w[3]));
}

VIT_DEV f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// row index (within a 32-row MFMA tile) of accumulator register r for lane half h
VIT_DEV int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// A 32-row x 64-column block held as two 32x32 accumulators (rows on the lanes of each half-wave: lane (row, hf) holds
// columns 8k + 4hf .. 8k + 4hf + 3 of group k = 4 db + g in registers 4g..4g+3 of acc[db]) stored as bf16 16-B row
// pieces: one permlane32 swap per dword pairs groups (k, k + 1), as in the forward's O store.  `row` points at column
// 8 hf of this lane's row; the swaps run on every lane, only the stores are predicated by `ok`.
VIT_DEV void store_block_rows16(const f32x16 (&acc)[2], float mul, bf16_t* row, bool ok) {
  uint32_t pk[8][2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int k = 4 * db + g;
      pk[k][0] = (uint32_t)f2bf(acc[db][4 * g] * mul) | ((uint32_t)f2bf(acc[db][4 * g + 1] * mul) << 16);
      pk[k][1] = (uint32_t)f2bf(acc[db][4 * g + 2] * mul) | ((uint32_t)f2bf(acc[db][4 * g + 3] * mul) << 16);
    }
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
#pragma unroll
    for (int w2 = 0; w2 < 2; ++w2) {
      const auto sw = __builtin_amdgcn_permlane32_swap(pk[k][w2], pk[k + 1][w2], false, false);
      pk[k][w2] = sw[0];
      pk[k + 1][w2] = sw[1];
    }
    if (ok) *reinterpret_cast<uint4*>(row + 8 * k) = make_uint4(pk[k][0], pk[k][1], pk[k + 1][0], pk[k + 1][1]);
  }
}


// XCD-aware (block, head) of a tiled kernel (1-D grid of nblk x B*H workgroups).  Workgroups are dealt round-robin
// over the 8 XCDs (linear id % 8), each with its own L2; the nblk 128-row blocks of one (image, head) all stream the
// head's whole K / V (or Q / dO), so in launch order they sat on nblk different XCDs and each fetched the head slice
// from beyond L2 (C5 PMC: 3.5-3.7x the algorithmic bytes).  Bijective remap: XCD x runs a contiguous range of logical
// tiles, tile j = (head j / nblk, block j % nblk), so a head's blocks share one L2 and run at about the same time.
#ifndef ATT_XCD                  // A/B builds only: 0 = launch order
#define ATT_XCD 1
#endif
VIT_DEV void xcd_block(int64_t nblk, int64_t& blk, int64_t& bh) {
  const int64_t orig = blockIdx.x, nwg = gridDim.x;
  const int64_t xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t j = ATT_XCD ? (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8 : orig;
  bh = j / nblk;
  blk = j - bh * nblk;
}

__global__ __launch_bounds__(256, 3) void attn_fwd_mfma(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o,
                                                     float* __restrict__ o32, float* __restrict__ lse, int64_t Tn,
                                                     int64_t H, float scale) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * TILE];  // [buf][K,V]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hf = lane >> 5;
  int64_t blk, bh;
  xcd_block((Tn + 127) / 128, blk, bh);
  const int64_t b = bh / H, h = bh % H;
  const int64_t D = H * HD, ld = 3 * D;
  const bf16_t* base = qkv + b * Tn * ld;
  const int64_t q0 = blk * 128 + wave * 32;
  const float c2 = scale * LOG2E;

  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = glb_frag(base, ld, q0, Tn, h * HD, s, lane);

  f32x16 oacc[2] = {f32x16{}, f32x16{}};
  float m_run = -INFINITY, l_run = 0.f;
  const int ntiles = (int)((Tn + KT - 1) / KT);
  tile_dma(base, ld, 0, Tn, D + h * HD, smem, wave, lane);
  tile_dma(base, ld, 0, Tn, 2 * D + h * HD, smem + TILE, wave, lane);
  tile_wait();
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < ntiles;
    if (more) {
      bf16_t* nb = smem + (cur ^ 1) * 2 * TILE;       // read in iteration t - 1, released by its closing barrier
      tile_dma(base, ld, (int64_t)(t + 1) * KT, Tn, D + h * HD, nb, wave, lane);
      tile_dma(base, ld, (int64_t)(t + 1) * KT, Tn, 2 * D + h * HD, nb + TILE, wave, lane);
    }
    const bf16_t* Ks = smem + cur * 2 * TILE;
    const bf16_t* Vs = Ks + TILE;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int kb = sub * 32;
      // an all-padding key block (T = 577: keys 608..639) adds nothing; a wave whose queries are all >= T stores nothing
      if ((int64_t)t * KT + kb >= Tn || q0 >= Tn) continue;
      f32x16 sacc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) sacc = mfma32(row_frag(Ks, kb, s, lane), qf[s], sacc);
      const int64_t key0 = (int64_t)t * KT + kb;
      float x[16];
      float mloc = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t key = key0 + acc_row(r, hf);
        x[r] = key < Tn ? sacc[r] * c2 : -INFINITY;
        mloc = fmaxf(mloc, x[r]);
      }
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float m_new = fmaxf(m_run, mloc);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      float psum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        x[r] = __builtin_amdgcn_exp2f(x[r] - m_new);
        psum += x[r];
      }
      l_run = l_run * alpha + psum;
      m_run = m_new;
      oacc[0] *= alpha;
      oacc[1] *= alpha;
      const bf16x8_t pb0 = pack8(x), pb1 = pack8(x + 8);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        oacc[db] = mfma32(tr_frag(Vs, kb, db, lane), pb0, oacc[db]);
        oacc[db] = mfma32(tr_frag(Vs, kb + 16, db, lane), pb1, oacc[db]);
      }
    }
    tile_wait();
    __syncthreads();
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.0f / l_tot;
  const int64_t q = q0 + (lane & 31);
  const bool qok = q < Tn;
  if (qok && o32) {
#pragma unroll
    for (int db = 0; db < 2; ++db) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v[4] = {oacc[db][4 * g] * inv, oacc[db][4 * g + 1] * inv, oacc[db][4 * g + 2] * inv,
                      oacc[db][4 * g + 3] * inv};
        st4<float>(o32 + (b * Tn + q) * D + h * HD + db * 32 + 8 * g + 4 * hf, v);
      }
    }
  }
  store_block_rows16(oacc, inv, o + (b * Tn + (qok ? q : Tn - 1)) * D + h * HD + 8 * hf, qok);
  if (qok && hf == 0) lse[bh * Tn + q] = (m_run + log2f(l_tot)) / LOG2E;
}

// dQ of 128 queries per workgroup (4 waves x 32) over 64-key tiles.  It runs before attn_bwd_dkdv_mfma and forms
// delta[q] = sum_d dO . O for its own queries from the dO fragments it holds anyway and the forward's O (the fp32 copy
// when there is one): each lane dots its 32 columns of the row, the two lane halves are added (fixed order); the
// result is stored for the dK / dV kernel.  No separate delta pass re-reading dO (was attn_delta, 29 us per layer at
// C5).  With the forward's fp32 O (o32) delta is exact to fp32: under the reference's x sqrt(hd) scaling most softmax
// rows are saturated, where dS = P (dP - delta) is a tiny difference and delta from the bf16-rounded O swamps it
// (measured: the Q / K weight gradients of a saturated head 10x off the bf16-rounding oracle).
#ifndef ATT_DQ_MINB              // A/B builds only: workgroups per CU the dQ kernel's register budget is sized for
#define ATT_DQ_MINB 2
#endif
template <class TO>
__global__ __launch_bounds__(256, ATT_DQ_MINB) void attn_bwd_dq_mfma(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ d_o,
                                                        const TO* __restrict__ o, const float* __restrict__ lse,
                                                        float* __restrict__ delta, bf16_t* __restrict__ dqkv,
                                                        int64_t Tn, int64_t H, float scale) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hf = lane >> 5;
  int64_t blk, bh;
  xcd_block((Tn + 127) / 128, blk, bh);
  const int64_t b = bh / H, h = bh % H;
  const int64_t D = H * HD, ld = 3 * D;
  const bf16_t* base = qkv + b * Tn * ld;
  const int64_t q0 = blk * 128 + wave * 32;
  const int64_t q = q0 + (lane & 31);
  const float c2 = scale * LOG2E;
  bf16x8_t qf[4], gf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = glb_frag(base, ld, q0, Tn, h * HD, s, lane);
    gf[s] = glb_frag(d_o + b * Tn * D, D, q0, Tn, h * HD, s, lane);
  }
  const float nls = q < Tn ? -lse[bh * Tn + q] / scale : 0.f;   // initial S accumulator (row constant)
  // O row pieces for delta: loaded with the first K / V tile (their wait is the tile's), summed after it
  float va[4][8];
  {
    const TO* orow = o + (b * Tn + min(q, Tn - 1)) * D + h * HD + 8 * hf;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      ld4<TO>(orow + 16 * s, va[s]);
      ld4<TO>(orow + 16 * s + 4, va[s] + 4);
    }
  }
  f32x16 dq[2] = {f32x16{}, f32x16{}};
  const int ntiles = (int)((Tn + KT - 1) / KT);
  tile_dma(base, ld, 0, Tn, D + h * HD, smem, wave, lane);
  tile_dma(base, ld, 0, Tn, 2 * D + h * HD, smem + TILE, wave, lane);
  float dl = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) dl += va[s][j] * (float)gf[s][j];
  dl += __shfl_xor(dl, 32, 64);
  if (hf == 0 && q < Tn) delta[bh * Tn + q] = dl;
  const float ndl = q < Tn ? -dl : 0.f;                          // initial dP accumulator
  tile_wait();
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < ntiles;
    if (more) {
      bf16_t* nb = smem + (cur ^ 1) * 2 * TILE;       // read in iteration t - 1, released by its closing barrier
      tile_dma(base, ld, (int64_t)(t + 1) * KT, Tn, D + h * HD, nb, wave, lane);
      tile_dma(base, ld, (int64_t)(t + 1) * KT, Tn, 2 * D + h * HD, nb + TILE, wave, lane);
    }
    const bf16_t* Ks = smem + cur * 2 * TILE;
    const bf16_t* Vs = Ks + TILE;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int kb = sub * 32;
      f32x16 sacc, pacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sacc[r] = nls;
        pacc[r] = ndl;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sacc = mfma32(row_frag(Ks, kb, s, lane), qf[s], sacc);  // S' = S - lse / scale
        pacc = mfma32(row_frag(Vs, kb, s, lane), gf[s], pacc);  // dP' = dP - delta
      }
      const int64_t key0 = (int64_t)t * KT + kb;
      float ds[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) ds[r] = __builtin_amdgcn_exp2f(sacc[r] * c2) * pacc[r];
      if (key0 + 32 > Tn) {                           // wave-uniform: keys >= T (zero K rows) must not contribute
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (key0 + acc_row(r, hf) >= Tn) ds[r] = 0.f;
      }
      const bf16x8_t d0 = pack8(ds), d1 = pack8(ds + 8);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        dq[db] = mfma32(tr_frag(Ks, kb, db, lane), d0, dq[db]);
        dq[db] = mfma32(tr_frag(Ks, kb + 16, db, lane), d1, dq[db]);
      }
    }
    tile_wait();
    __syncthreads();
  }
  store_block_rows16(dq, scale, dqkv + (b * Tn + (q < Tn ? q : Tn - 1)) * ld + h * HD + 8 * hf, q < Tn);
}

#ifndef ATT_DKDV_MINB            // A/B builds only: workgroups per CU the dK / dV kernel is sized for
#define ATT_DKDV_MINB 3
#endif
__global__ __launch_bounds__(256, ATT_DKDV_MINB) void attn_bwd_dkdv_mfma(const bf16_t* __restrict__ qkv,
                                                          const bf16_t* __restrict__ d_o,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
                                                          int64_t Tn, int64_t H, float scale) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * TILE];  // [buf][Q, dO]
  // [buf][-lse / scale, -delta] per query: the initial S / dP accumulators (rows >= T: -inf -> P = 0)
  __shared__ __attribute__((aligned(16))) float stat[2][2][KT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hf = lane >> 5;
  int64_t blk, bh;
  xcd_block((Tn + 127) / 128, blk, bh);
  const int64_t b = bh / H, h = bh % H;
  const int64_t D = H * HD, ld = 3 * D;
  const bf16_t* base = qkv + b * Tn * ld;
  const bf16_t* gbase = d_o + b * Tn * D;
  const int64_t k0 = blk * 128 + wave * 32;
  const float c2 = scale * LOG2E;
  bf16x8_t kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = glb_frag(base, ld, k0, Tn, D + h * HD, s, lane);
    vf[s] = glb_frag(base, ld, k0, Tn, 2 * D + h * HD, s, lane);
  }
  f32x16 dk[2] = {f32x16{}, f32x16{}}, dv[2] = {f32x16{}, f32x16{}};
  const int ntiles = (int)((Tn + KT - 1) / KT);
  float st_l = 0.f, st_d = 0.f;
  auto load_stats = [&](int t) {
    if (tid < KT) {
      const int64_t qq = (int64_t)t * KT + tid;
      st_l = qq < Tn ? -lse[bh * Tn + qq] / scale : -INFINITY;
      st_d = qq < Tn ? -delta[bh * Tn + qq] : 0.f;
    }
  };
  tile_dma(base, ld, 0, Tn, h * HD, smem, wave, lane);
  tile_dma(gbase, D, 0, Tn, h * HD, smem + TILE, wave, lane);
  load_stats(0);
  if (tid < KT) {
    stat[0][0][tid] = st_l;
    stat[0][1][tid] = st_d;
  }
  tile_wait();
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < ntiles;
    if (more) {
      bf16_t* nb = smem + (cur ^ 1) * 2 * TILE;       // read in iteration t - 1, released by its closing barrier
      tile_dma(base, ld, (int64_t)(t + 1) * KT, Tn, h * HD, nb, wave, lane);
      tile_dma(gbase, D, (int64_t)(t + 1) * KT, Tn, h * HD, nb + TILE, wave, lane);
      load_stats(t + 1);
    }
    const bf16_t* Qs = smem + cur * 2 * TILE;
    const bf16_t* Gs = Qs + TILE;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int qb = sub * 32;
      if ((int64_t)t * KT + qb >= Tn || k0 >= Tn) continue;   // all-padding query block (P = 0) or key wave
      // row constants as the initial accumulators: S' = S - lse / scale, dP' = dP - delta (registers 4g..4g+3 <->
      // queries qb + 8g + 4hf + 0..3: b128 broadcast reads)
      f32x16 sacc, pacc;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lv = *reinterpret_cast<const f32x4*>(&stat[cur][0][qb + 8 * g + 4 * hf]);
        const f32x4 dv4 = *reinterpret_cast<const f32x4*>(&stat[cur][1][qb + 8 * g + 4 * hf]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sacc[4 * g + i] = lv[i];
          pacc[4 * g + i] = dv4[i];
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sacc = mfma32(row_frag(Qs, qb, s, lane), kf[s], sacc);   // S'[q][key]
        pacc = mfma32(row_frag(Gs, qb, s, lane), vf[s], pacc);   // dP'[q][key]
      }
      float p[16], ds[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        p[r] = __builtin_amdgcn_exp2f(sacc[r] * c2);           // queries >= T: -inf -> 0
        ds[r] = p[r] * pacc[r];
      }
      const bf16x8_t p0 = pack8(p), p1 = pack8(p + 8), d0 = pack8(ds), d1 = pack8(ds + 8);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        dv[db] = mfma32(tr_frag(Gs, qb, db, lane), p0, dv[db]);
        dv[db] = mfma32(tr_frag(Gs, qb + 16, db, lane), p1, dv[db]);
        dk[db] = mfma32(tr_frag(Qs, qb, db, lane), d0, dk[db]);
        dk[db] = mfma32(tr_frag(Qs, qb + 16, db, lane), d1, dk[db]);
      }
    }
    if (more) {
      if (tid < KT) {
        stat[cur ^ 1][0][tid] = st_l;
        stat[cur ^ 1][1][tid] = st_d;
      }
    }
    tile_wait();
    __syncthreads();
  }
  const int64_t key = k0 + (lane & 31);
  bf16_t* dkr = dqkv + (b * Tn + (key < Tn ? key : Tn - 1)) * ld + D + h * HD + 8 * hf;
  store_block_rows16(dk, scale, dkr, key < Tn);
  store_block_rows16(dv, 1.f, dkr + D, key < Tn);
}

// ---------------------------------------------------------------------------------------------------------------
// Fused backward for T <= 256 (ViT: T = 197): one 8-wave workgroup per (image, head), everything from LDS.
//   LDS: K, Q, dO (and V when it fits) as [Tp][64] images (Tp = T rounded up to 32), lse2 per query, the delta
//   partials, a double-buffered dS^T image [Tp keys][32 queries] and a double-buffered dQ staging block.
//   Wave w owns key block w (32 keys: its K / V fragments live in registers, dK / dV accumulate in registers) and
//   walks the query blocks qb:  S, dP (keys on lanes) -> P -> dV += dO^T P, delta = rowsum(P * dP) over the key
//   waves, dS = P (dP - delta) -> dK += Q^T dS, dS^T -> LDS; then dQ[qb] (32 x 64) is split over the 8 waves as
//   16x16 tiles (16x16x32 MFMA over all Tp keys): no recomputation of P, no atomics — deterministic.
// ---------------------------------------------------------------------------------------------------------------
constexpr int FB_TMAX = 256;
#ifndef ATT_DWAV
#define ATT_DWAV 1
#endif
#ifndef ATT_KVLDS
#define ATT_KVLDS 1
#endif
#ifndef ATT_ORDER                // A/B builds only: loop-body order (0 back, front, dq; 1 front, back, dq; 2 dq first;
                                 // 3 waves 4-7 dq first)
#define ATT_ORDER 0
#endif
#ifndef ATT_PRIO                 // A/B builds only: s_setprio 1 around the S / dP MFMA chain
#define ATT_PRIO 0
#endif


VIT_DEV __amdgpu_buffer_rsrc_t make_rsrc_b(const void* base, int64_t bytes) {
  const uint32_t nrec = bytes >= 0x7fffffffLL ? 0x7fffffffu : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}

// A operand (16x16x32) of X^T from a [row][64] image: lane holds X[r0 + 8(lane>>4) + j][c0 + (lane&15)] for
// j = 0..7, via two transposed reads (rows +0..3, +4..7).  `rowlen` = elements per image row; `swz` = chunk swizzle.
template <int ROWLEN, bool ASWZ>
VIT_DEV bf16x8_t col_frag16(const bf16_t* img, int r0, int c0, int lane) {
  const int g = lane >> 4, lg = lane & 15, q = lg >> 2, p = lg & 3;
  const int col = c0 + 4 * p;
  const int c = col >> 3;
  const int ra = r0 + 8 * g + q, rb = ra + 4;
  const int ca = ASWZ ? (c ^ aswz(ra)) : c, cb = ASWZ ? (c ^ aswz(rb)) : c;
  s16x4 lo = tr_read(img + ra * ROWLEN + (ca << 3) + (col & 7));
  s16x4 hi = tr_read(img + rb * ROWLEN + (cb << 3) + (col & 7));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// LDS-DMA of one [Tp][64] head slice (rows of a row-major matrix with leading dim ld, columns col0..col0+63)
// into a swizzled [Tp][64] image: 1 KiB pieces of 8 rows, lane-linear destination, the chunk swizzle applied to
// the source address; rows >= Tn are zero-filled by an out-of-range offset.
VIT_DEV void dma_head_slice(__amdgpu_buffer_rsrc_t rs, int64_t row0, int64_t ld, int64_t col0, int Tn, int Tp,
                            bf16_t* img, int wave, int lane, int nwaves = 8) {
  for (int pc = wave; pc < Tp / 8; pc += nwaves) {
    const int r = pc * 8 + (lane >> 3);
    const int c = (lane & 7) ^ aswz(r);
    const uint32_t off = r < Tn ? (uint32_t)(2 * ((row0 + r) * ld + col0 + c * 8)) : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + pc * 512), 16, off,
                                             0, 0, 0);
  }
}

// Row-contiguous store of a [rows][64] bf16 LDS image (row stride RS elements, no swizzle) to global rows (row stride
// ld): 8 lanes per 128-B row.  Rows of a stride that is not a multiple of 8 elements (the padded dQ staging, 68) are
// only 8-B aligned, so the 16-B piece is read as two 8-B LDS reads there.
template <int RS>
VIT_DEV void store_rows64(const bf16_t* img, int rows, int valid_rows, bf16_t* dst, int64_t ld, int tid,
                          int nthreads) {
  static_assert(RS % 4 == 0, "store_rows64: rows must be 8-B aligned");
  for (int q = tid; q < rows * 8; q += nthreads) {
    const int r = q >> 3, c = q & 7;
    if (r < valid_rows) {
      uint4 v;
      if (RS % 8 == 0) {
        v = *reinterpret_cast<const uint4*>(img + r * RS + c * 8);
      } else {
        const uint2 lo = *reinterpret_cast<const uint2*>(img + r * RS + c * 8);
        const uint2 hi = *reinterpret_cast<const uint2*>(img + r * RS + c * 8 + 4);
        v = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
      *reinterpret_cast<uint4*>(dst + (int64_t)r * ld + c * 8) = v;
    }
  }
}

// Workgroup barrier ordering LDS only: unlike __syncthreads() (a release fence: vmcnt(0)) it leaves global loads,
// LDS-DMA and stores in flight.  LDS-DMA targets are published by an explicit vmcnt(0) + barrier where consumed.
VIT_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One 8-row piece `pc` of a swizzled [Tp][64] head-slice image by LDS-DMA (one 16-B lane each; rows >= Tn zero).
// global_load_lds form (per-lane address): rows >= Tn are clamped to row Tn - 1 instead of zero-filled; the persistent
// backward masks them (P = 0 for queries >= T through lse = +inf, for keys >= T through kbias), finite data suffices.
// One 16-B lane of an LDS-DMA piece, addressed as a scalar base (the item's head slice: uniform) plus a 32-bit per-lane
// byte offset (the saddr form): no 64-bit per-lane address arithmetic (a row * ld product was ~3 quarter-rate VALU
// ops per piece and lane).  Issued as inline asm on purpose: the compiler's waitcnt pass cannot tell the DMA target
// from the blocks still being read and would put vmcnt(0) before every later LDS read, draining the prefetch;
// completion is awaited explicitly by the callers.
VIT_DEV void dma16_saddr(const bf16_t* sbase, uint32_t voff, bf16_t* lds_dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(lds_dst));
  // M0 is reserved (clang warns) but no compiler-generated code in these kernels reads it (checked in the ISA)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds)
               : "memory", "m0");
#pragma clang diagnostic pop
}

// Byte offset of row r, 16-B chunk c of a head slice with leading dimension ld (r <= 255 and ld < 2^20 here: the
// product fits the 24-bit multiplier and the offset 32 bits)
VIT_DEV uint32_t slice_off(int r, int64_t ld, int c) {
  return (__umul24((uint32_t)r, (uint32_t)ld) + (uint32_t)(c * 8)) * 2u;
}

VIT_DEV void dma_piece(const bf16_t* base, int64_t row0, int64_t ld, int64_t col0, int Tn, bf16_t* img, int pc,
                       int lane) {
  lane = remat(lane);
  const int r = pc * 8 + (lane >> 3);
  const int c = (lane & 7) ^ aswz(r);
  dma16_saddr(base + row0 * ld + col0, slice_off(min(r, Tn - 1), ld, c), img + pc * 512);
}
VIT_DEV void dma_slice_g(const bf16_t* base, int64_t row0, int64_t ld, int64_t col0, int Tn, int Tp, bf16_t* img,
                         int wave, int lane) {
  for (int pc = wave; pc < Tp / 8; pc += 8) dma_piece(base, row0, ld, col0, Tn, img, pc, lane);
}

// Row sums of a 32x32 accumulator tile over its 32 columns (the keys, on the lanes of each half-wave): t[r] holds
// element (row acc_row(r, hf), column lane & 31).  One v_permlane16_swap per register pair folds the two 16-lane rows
// of a half-wave (even rows keep registers 0-7, odd rows 8-15), then four DPP steps (xor 8, 7, 2, 1 inside a row)
// finish the sums.  Every lane of 16-lane row R ends with the sums of registers 8 (R & 1) + j, j = 0..7.  The pairing
// is fixed, so the result does not depend on timing (deterministic).
VIT_DEV void rowsum32(const float (&t)[16], float (&u)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(t[j]), __float_as_uint(t[j + 8]), false, false);
    u[j] = __uint_as_float(s[0]) + __uint_as_float(s[1]);
  }
  // v_add_f32 with a DPP source, 8 independent registers per step (hipcc does not fold v_mov_dpp into the add here);
  // a DPP read needs 2 wait states after the VALU write of its register: the s_nop covers the first step, later
  // steps read registers written 8 instructions earlier
#define VIT_DPP_ADD8(CTRL)                                                                                        \
  asm volatile("s_nop 1\n\t"                                                                                    \
               "v_add_f32_dpp %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                             \
               "v_add_f32_dpp %1, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                             \
               "v_add_f32_dpp %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                             \
               "v_add_f32_dpp %3, %3, %3 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                             \
               "v_add_f32_dpp %4, %4, %4 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                             \
               "v_add_f32_dpp %5, %5, %5 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                             \
               "v_add_f32_dpp %6, %6, %6 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                             \
               "v_add_f32_dpp %7, %7, %7 " CTRL " row_mask:0xf bank_mask:0xf"                                   \
               : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]))
  VIT_DPP_ADD8("row_ror:8");
  VIT_DPP_ADD8("row_half_mirror");
  VIT_DPP_ADD8("quad_perm:[2,3,0,1]");
  VIT_DPP_ADD8("quad_perm:[1,0,3,2]");
#undef VIT_DPP_ADD8
}

// Persistent: workgroup g handles items (image, head) g, g + gridDim.x, ...  The next item's operands are staged while
// this one computes: its dO / Q 32-row blocks are LDS-DMA'd into this item's blocks as they die (dO block qb after
// front(qb), Q block qb after back(qb)), its V after the first barrier, its K right after the last dQ block, its lse
// into a register.  gridDim.x == items gives one item per workgroup (no prefetch).  dK / dV leave registers directly.
//
// delta[q] = sum_k P[q][k] dP[q][k] (= rowsum(dO * O) in exact arithmetic) is formed here from the fp32 P and dP the
// backward computes anyway, so neither O nor an fp32 copy of it is read: under the reference's x sqrt(hd) logit scale
// most softmax rows saturate and dS = P (dP - delta) is a small difference, which a delta from the bf16-rounded O
// would swamp; this one is consistent with the kernel's own P to fp32 rounding.  A query block qb runs in two halves
// one barrier apart, software-pipelined with the neighbouring blocks (iteration it = one barrier interval):
//   front(it):   S, dP (keys on lanes) -> P; dV += dO^T P; each key wave's partial rowsum(P * dP) -> LDS
//   back(it-1):  delta = the key waves' partials in wave order; dS = P (dP - delta); dK += Q^T dS; dS^T -> LDS
//   dq(it-2):    dQ block = dS K over all keys, split over the 8 waves as 16x16 tiles -> LDS staging
//   store(it-3): the staged dQ block -> global, full rows
// P and dP of the block in flight stay in registers across the barrier.  No atomics, no cross-wave reduction of
// results beyond the fixed-order delta sum: deterministic.
// Diagnostic build only (-DATT_STAMPS=1, tools/attn_stamps.py): s_memtime stamps (lane 0 of every wave, workgroups
// 0-15) of the fused backward's steady iterations (first item) and of whole items (first two), read back by
// vit_diag_attn_stamps / vit_diag_attn_istamps.  Compiled out otherwise.
#ifndef ATT_STAMPS
#define ATT_STAMPS 0
#endif
#if ATT_STAMPS
__device__ unsigned long long g_att_stamps[16 * 8 * 8 * 6];
__device__ unsigned long long g_att_istamps[16 * 8 * 2 * 10];
#define ATT_STAMP(IT, K)                                                                                   \
  do {                                                                                                     \
    if (item == (int64_t)blockIdx.x && blockIdx.x < 16 && lane == 0 && (IT) < 8)                           \
      g_att_stamps[((blockIdx.x * 8 + wave) * 8 + (IT)) * 6 + (K)] = __builtin_amdgcn_s_memtime();          \
  } while (0)
#define ATT_ISTAMP(K)                                                                                      \
  do {                                                                                                     \
    const int64_t ii_ = (item - (int64_t)blockIdx.x) / gridDim.x;                                          \
    if (blockIdx.x < 16 && lane == 0 && ii_ < 2)                                                           \
      g_att_istamps[((blockIdx.x * 8 + wave) * 2 + ii_) * 10 + (K)] = __builtin_amdgcn_s_memtime();         \
  } while (0)
#else
#define ATT_STAMP(IT, K) do { } while (0)
#define ATT_ISTAMP(K) do { } while (0)
#endif

template <int NQB>
__global__ __launch_bounds__(512, 1) void attn_bwd_fused(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ d_o,
                                                         const float* __restrict__ lse, bf16_t* __restrict__ dqkv,
                                                         int64_t Tn64, int64_t H, int64_t items, float scale) {
  constexpr int Tp = NQB * 32;                        // T rounded up to 32 (compile time: the dQ sum unrolls)
  constexpr int nqb = NQB;
  constexpr int IMG = Tp * HD;                        // elements per [Tp][64] image
  // dS^T image [Tp keys][32 queries]: the 8-B unit u (4 queries) of key row r sits at unit u ^ ((r >> 1) & 7), which
  // makes both its ds_write_b64 (16 consecutive keys per lane group) and the dQ B-operand ds_read_b64_tr_b16 (8 rows x
  // 4 units per 32-lane group) bank-conflict free (the plain layout cost 28 extra LDS cycles per store instruction:
  // 8 keys on one bank pair).  dQ staging rows are padded to 68 elements (136 B: 17 8-B units, odd) so its 16-row
  // ds_write_b64 groups spread over all banks (a 128-B row put all 16 on one bank pair, 60 extra cycles per store).
  constexpr int DST = Tp * 32;                        // elements per dS^T image
  constexpr int QRS = HD + 4;                         // dQ staging row stride (elements)
  constexpr int QST = 32 * QRS;                       // dQ block staging [32][68]
  constexpr int NF = Tp + 2 * 8 * 32 + 8 * 32;        // floats: lse2 [Tp], delta partials [2][8][32], per-wave delta [8][32]
  // V image too when it fits in the 160 KiB (Tp <= 224): staged during the previous item instead of read from global
  // at the top of each item (an exposed load round trip per item)
  constexpr bool VLDS = (4 * IMG + 2 * DST + 2 * QST) * 2 + NF * 4 <= 160 * 1024;
  __shared__ __attribute__((aligned(16))) bf16_t smem[(VLDS ? 4 : 3) * IMG + 2 * DST + 2 * QST + 2 * NF];
  bf16_t* Ks = smem;
  bf16_t* Qs = Ks + IMG;
  bf16_t* Gs = Qs + IMG;
  bf16_t* dSt = Gs + IMG;                              // [2][Tp][32]
  bf16_t* dQs = dSt + 2 * DST;                         // [2][32][64]
  bf16_t* Vs = dQs + 2 * QST;                          // [Tp][64] when VLDS
  float* lse2s = reinterpret_cast<float*>(Vs + (VLDS ? IMG : 0));
  float* dpart = lse2s + Tp;                           // [2][8][32]
  float* dwav = dpart + 2 * 8 * 32;                    // [8][32]

  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Tn = (int)Tn64;
  const int64_t D = H * HD, ld = 3 * D;
  const float c2 = scale * LOG2E;

  // Wave w owns key block w; a wave without one (w >= nqb: wave 7 at T = 197) skips front / back (a dummy block
  // with every key masked, to keep the loop body free of wave-dependent branches, measured 7 us slower at C2).
  const bool kact = wave < nqb;
  const int kb = kact ? wave * 32 : 0;
  const int key = kb + (lane & 31);
  const float kbias = kact && key < Tn ? 0.f : -INFINITY;
  const int dd = wave >> 1, qh = wave & 1;            // this wave's dQ tile: d 16dd.., queries 16qh..
  // Per-lane LDS offsets (elements) inside a 32-row block: the row swizzle aswz(r) only uses bits 1..3 of r, so a
  // block starting at a multiple of 16 rows adds rb * 64 and nothing else.
  int rf_off[4];                                       // row_frag: row (lane&31), chunk 2s + hf
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int r = lane & 31;
    rf_off[s] = r * HD + (((2 * s + hf) ^ aswz(r)) << 3);
  }
  int tf_off[2][2];                                    // tr_frag rows r1 / r1 + 8, d block db
  {
    const int G = lane >> 4, hh = G >> 1, lg = lane & 15, q = lg >> 2, pp = lg & 3;
    const int r1 = 4 * hh + q, r2 = r1 + 8;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const int col = db * 32 + 16 * (G & 1) + 4 * pp;
      const int c = col >> 3;
      tf_off[db][0] = r1 * HD + ((c ^ aswz(r1)) << 3) + (pp & 1) * 4;
      tf_off[db][1] = r2 * HD + ((c ^ aswz(r2)) << 3) + (pp & 1) * 4;
    }
  }
  int cf_k[2], cf_s[2];                                // col_frag16 on K (dQ A operand) and on dS^T (B operand)
  {
    const int g = lane >> 4, lg = lane & 15, q = lg >> 2, pp = lg & 3;
    const int ra = 8 * g + q, rb2 = ra + 4;
    const int colk = dd * 16 + 4 * pp, cols = qh * 16 + 4 * pp;
    cf_k[0] = ra * HD + (((colk >> 3) ^ aswz(ra)) << 3) + (colk & 7);
    cf_k[1] = rb2 * HD + (((colk >> 3) ^ aswz(rb2)) << 3) + (colk & 7);
    cf_s[0] = ra * 32 + (((cols >> 2) ^ ((ra >> 1) & 7)) << 2);        // (kc a multiple of 32: same swizzle)
    cf_s[1] = rb2 * 32 + (((cols >> 2) ^ ((rb2 >> 1) & 7)) << 2);
  }
  auto trd = [&](const bf16_t* base, int o1, int o2) {
    s16x4 lo = tr_read(base + o1);
    s16x4 hi = tr_read(base + o2);
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  };
  auto rrd = [&](const bf16_t* base, int o) {
    return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const s16x8*>(base + o));
  };

  // lse of item `it_` -> a register (tid < Tn <= 256)
  float lreg = 0.f;
  auto load_lse = [&](int64_t it_) {
    const int t_ = remat(tid);
    if (t_ < Tn) lreg = lse[it_ * Tn + t_];
  };

  int64_t item = blockIdx.x;
  if (item < items) {                                 // first item: exposed staging
    int64_t b, h;
    item_bh(item, H, b, h);
    dma_slice_g(qkv, b * Tn, ld, D + h * HD, Tn, Tp, Ks, wave, lane);
    dma_slice_g(qkv, b * Tn, ld, h * HD, Tn, Tp, Qs, wave, lane);
    dma_slice_g(d_o, b * Tn, D, h * HD, Tn, Tp, Gs, wave, lane);
    if (VLDS) dma_slice_g(qkv, b * Tn, ld, 2 * D + h * HD, Tn, Tp, Vs, wave, lane);
    load_lse(item);
  }
#pragma unroll 1
  for (; item < items; item += gridDim.x) {
    int64_t b, h, nb_ = 0, nh_ = 0;
    item_bh(item, H, b, h);
    const int64_t nxt = item + gridDim.x;
    const bool more = nxt < items;
    if (more) item_bh(nxt, H, nb_, nh_);
    ATT_ISTAMP(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this item's K / Q / dO / V DMA, lse
    {
      const int t_ = remat(tid);
      if (t_ < Tp) lse2s[t_] = t_ < Tn ? lreg * LOG2E : INFINITY;
    }
    __syncthreads();                                  // every wave's DMA landed
    ATT_ISTAMP(1);
    bf16x8_t kf[4], vf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (!ATT_KVLDS) kf[s] = row_frag(Ks, kb, s, lane);
      if (!ATT_KVLDS || !VLDS)
        vf[s] = VLDS ? row_frag(Vs, kb, s, lane) : glb_frag(qkv + b * Tn * ld, ld, kb, Tn, 2 * D + h * HD, s, lane);
    }
    f32x16 dk[2] = {f32x16{}, f32x16{}}, dv[2] = {f32x16{}, f32x16{}};
    float pc[16], dpc[16];                            // P and dP of the block between front and back

    // front(qb): this wave's key block against query block qb -> P, dV; partial delta -> dpart[qb & 1][wave]
    auto front = [&](int qb) {
      if (!kact) return;                              // the wave without a key block (measured: cheaper than a masked dummy block)
      const int q0 = qb * 32;
      const bf16_t* Qb = Qs + q0 * HD;
      const bf16_t* Gb = Gs + q0 * HD;
      f32x16 sacc = {}, pacc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#if ATT_KVLDS
        const bf16x8_t kfs = rrd(Ks + kb * HD, rf_off[s]), vfs = VLDS ? rrd(Vs + kb * HD, rf_off[s]) : vf[s];
#else
        const bf16x8_t kfs = kf[s], vfs = vf[s];
#endif
        if (ATT_PRIO && s == 0) __builtin_amdgcn_s_setprio(1);
        sacc = mfma32(rrd(Qb, rf_off[s]), kfs, sacc);             // S[q][key]: lane = key
        pacc = mfma32(rrd(Gb, rf_off[s]), vfs, pacc);             // dP[q][key]
      }
      if (ATT_PRIO) __builtin_amdgcn_s_setprio(0);
      // registers 4g..4g+3 <-> queries q0 + 8g + 4hf + 0..3: broadcast b128 reads of lse2
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lv = *reinterpret_cast<const f32x4*>(lse2s + q0 + 8 * g + 4 * hf);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          // queries >= T have lse2 = +inf, keys >= T kbias = -inf -> P = 0 exactly
          pc[r] = __builtin_amdgcn_exp2f(sacc[r] * c2 - lv[i] + kbias);
          dpc[r] = pacc[r];
        }
      }
      const bf16x8_t p0 = pack8(pc), p1 = pack8(pc + 8);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        dv[db] = mfma32(trd(Gb, tf_off[db][0], tf_off[db][1]), p0, dv[db]);
        dv[db] = mfma32(trd(Gb + 16 * HD, tf_off[db][0], tf_off[db][1]), p1, dv[db]);
      }
      float t[16], u[8];
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = pc[r] * dpc[r];
      rowsum32(t, u);
      // lane 16R (R = 16-lane row; hf = R >> 1) writes registers 8 (R & 1) + j: queries 16 (R & 1) + 4 hf + 0..3 and
      // 16 (R & 1) + 8 + 4 hf + 0..3
      const int ln_ = remat(lane);
      if ((ln_ & 15) == 0) {
        float* dp = dpart + (qb & 1) * 256 + wave * 32 + 16 * ((ln_ >> 4) & 1) + 4 * (ln_ >> 5);
        *reinterpret_cast<f32x4*>(dp) = f32x4{u[0], u[1], u[2], u[3]};
        *reinterpret_cast<f32x4*>(dp + 8) = f32x4{u[4], u[5], u[6], u[7]};
      }
    };

    // back(qb): delta of query block qb (its partials are behind the last barrier) -> dS -> dK; dS^T -> dSt[qb & 1]
    auto back = [&](int qb) {
      if (!kact) return;
      const int q0 = qb * 32;
      const bf16_t* Qb = Qs + q0 * HD;
      float ds[16];
#if ATT_DWAV
      const float* dp = dpart + (qb & 1) * 256 + (lane & 31);
      float dsum = dp[0];
#pragma unroll
      for (int w = 1; w < nqb; ++w) dsum += dp[w * 32];  // key-block order: the same sum in every wave
      float* dw = dwav + wave * 32;
      dw[lane & 31] = dsum;                           // lanes l and l + 32 store the same value
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 dv4 = *reinterpret_cast<const f32x4*>(dw + 8 * g + 4 * hf);   // this wave's own write above
#pragma unroll
        for (int i = 0; i < 4; ++i) ds[4 * g + i] = pc[4 * g + i] * (dpc[4 * g + i] - dv4[i]);
      }
#else
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float* dp = dpart + (qb & 1) * 256 + 8 * g + 4 * hf;
        f32x4 dv4 = *reinterpret_cast<const f32x4*>(dp);
#pragma unroll
        for (int w = 1; w < nqb; ++w) dv4 += *reinterpret_cast<const f32x4*>(dp + w * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) ds[4 * g + i] = pc[4 * g + i] * (dpc[4 * g + i] - dv4[i]);
      }
#endif
      const bf16x8_t d0 = pack8(ds), d1 = pack8(ds + 8);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        dk[db] = mfma32(trd(Qb, tf_off[db][0], tf_off[db][1]), d0, dk[db]);
        dk[db] = mfma32(trd(Qb + 16 * HD, tf_off[db][0], tf_off[db][1]), d1, dk[db]);
      }
      bf16_t* dS = dSt + (qb & 1) * DST + key * 32;
      const int ksw = (key >> 1) & 7;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {                // queries 8 g4 + 4 hf + 0..3: unit 2 g4 + hf
        float v4[4] = {ds[4 * g4], ds[4 * g4 + 1], ds[4 * g4 + 2], ds[4 * g4 + 3]};
        st4<bf16_t>(dS + (((2 * g4 + hf) ^ ksw) << 2), v4);
      }
    };

    // dQ(qb) = dS K over all keys: this wave's 16x16 tile of the 32 x 64 block -> staging dQs[qb & 1]
    auto dq = [&](int qb) {
      const bf16_t* dS = dSt + (qb & 1) * DST;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < Tp; kc += 32) {
        const bf16x8_t a = trd(Ks + kc * HD, cf_k[0], cf_k[1]);
        const bf16x8_t bq = trd(dS + kc * 32, cf_s[0], cf_s[1]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq, acc, 0, 0, 0);
      }
      // D[m = d][n = q]: lane -> q = 16qh + (lane&15), d = 16dd + 4(lane>>4) + i  -> staging [32][64]
      float v4[4] = {acc[0] * scale, acc[1] * scale, acc[2] * scale, acc[3] * scale};
      st4<bf16_t>(dQs + (qb & 1) * QST + (qh * 16 + (lane & 15)) * QRS + dd * 16 + 4 * (lane >> 4), v4);
    };
    bf16_t* dq_row0 = dqkv + b * Tn * ld + h * HD;
    auto dq_store = [&](int qb) {                     // the staged dQ block -> global, full rows
      const int qs = qb * 32;
      store_rows64<QRS>(dQs + (qb & 1) * QST, 32, min(32, Tn - qs), dq_row0 + (int64_t)qs * ld, ld, tid, 512);
    };
    // The next item's staging (the last item of a workgroup re-stages itself: the blocks are dead either way, and the
    // prefetch stays unconditional).  Waves 0-3 take the Q block's 4 pieces, waves 4-7 the dO block's.
    const int64_t sb_ = more ? nb_ : b, sh_ = more ? nh_ : h;
    const bool gq = wave < 4;
    const bf16_t* pf_base = gq ? qkv : d_o;
    const int64_t pf_ld = gq ? ld : D;
    bf16_t* pf_img = gq ? Qs : Gs;
    auto prefetch = [&](int qblk) {                   // Q block qblk (waves 0-3) or dO block qblk + 1 (waves 4-7)
      dma_piece(pf_base, sb_ * Tn, pf_ld, sh_ * HD, Tn, pf_img, (qblk + (gq ? 0 : 1)) * 4 + (wave & 3), lane);
    };
    // iteration it (one barrier interval): store dQ(it-3), back(it-1), front(it), dQ(it-2); the prefetch of dO block
    // it-1 (dead since front(it-1)) and Q block it-2 (dead since back(it-2)).  Prologue and tail peeled: the steady
    // iterations 2 .. nqb-1 are branch-free.
    if constexpr (NQB >= 3) {
      front(0);
      lds_barrier();
      ATT_ISTAMP(2);
      back(0);
      front(1);
      if (wave >= 4) prefetch(-1);                    // dO block 0
      load_lse(more ? nxt : item);                    // after front(0) consumed the V fragments: no wait on it
      if (VLDS && !ATT_KVLDS) dma_slice_g(qkv, sb_ * Tn, ld, 2 * D + sh_ * HD, Tn, Tp, Vs, wave, lane);  // V: top only
      lds_barrier();
      ATT_ISTAMP(3);
      back(1);
      front(2);
      dq(0);
      prefetch(0);                                    // Q block 0, dO block 1
      lds_barrier();
      ATT_ISTAMP(4);
#pragma unroll 1
      for (int it = 3; it < nqb; ++it) {
        ATT_STAMP(it, 0);
#if ATT_STAMPS
        dq_store(it - 3);
        ATT_STAMP(it, 1);
        back(it - 1);
        ATT_STAMP(it, 2);
        front(it);
        ATT_STAMP(it, 3);
        dq(it - 2);
        ATT_STAMP(it, 4);
        prefetch(it - 2);
        ATT_STAMP(it, 5);
        lds_barrier();
        continue;
#endif
#if ATT_ORDER == 1
        dq_store(it - 3);
        front(it);
        back(it - 1);
        dq(it - 2);
#elif ATT_ORDER == 2
        dq_store(it - 3);
        dq(it - 2);
        back(it - 1);
        front(it);
#elif ATT_ORDER == 3
        // SIMD partners (waves w, w + 4) in different phases: waves 4-7 run the LDS / MFMA-heavy dQ tile first while
        // waves 0-3 run the VALU-heavy delta / dS of back(); back stays before front (front overwrites P / dP)
        dq_store(it - 3);
        if (wave < 4) {
          back(it - 1);
          front(it);
          dq(it - 2);
        } else {
          dq(it - 2);
          back(it - 1);
          front(it);
        }
#else
        dq_store(it - 3);
        back(it - 1);
        front(it);
        dq(it - 2);
#endif
        prefetch(it - 2);
        lds_barrier();                                // LDS only: the prefetch and the dQ stores stay in flight
      }
      ATT_ISTAMP(5);
      dq_store(nqb - 3);
      back(nqb - 1);
      dq(nqb - 2);
      prefetch(nqb - 2);                              // Q block nqb-2, dO block nqb-1
      if (VLDS && ATT_KVLDS) dma_slice_g(qkv, sb_ * Tn, ld, 2 * D + sh_ * HD, Tn, Tp, Vs, wave, lane);  // V: fronts done
      lds_barrier();
      dq_store(nqb - 2);
      dq(nqb - 1);
      ATT_ISTAMP(6);
      if (wave < 4) prefetch(nqb - 1);                // Q block nqb-1
      lds_barrier();
      ATT_ISTAMP(7);
      dq_store(nqb - 1);
    } else {                                          // T <= 64: the same schedule with its conditions
#pragma unroll 1
      for (int it = 0; it <= nqb + 1; ++it) {
        if (it >= 3) dq_store(it - 3);
        if (it >= 1 && it <= nqb) back(it - 1);
        if (it < nqb) front(it);
        if (it >= 2) dq(it - 2);
        if ((wave >= 4 && it >= 1 && it <= nqb) || (wave < 4 && it >= 2)) prefetch(it - 2);
        if (it == 1) load_lse(more ? nxt : item);
        if (VLDS && it == (ATT_KVLDS ? nqb : 1)) dma_slice_g(qkv, sb_ * Tn, ld, 2 * D + sh_ * HD, Tn, Tp, Vs, wave, lane);
        lds_barrier();
      }
      dq_store(nqb - 1);
    }
    ATT_ISTAMP(8);
    // K and dS^T are dead (the last dQ block ran before the final barrier): stage the next item's K
    dma_slice_g(qkv, sb_ * Tn, ld, D + sh_ * HD, Tn, Tp, Ks, wave, lane);
    if constexpr (NQB <= 7) {
      if (kact) {                                     // dK / dV leave registers as 16-B row pieces
        const int ln = remat(lane), key_ = kb + (ln & 31);
        const int kr = key_ < Tn ? key_ : Tn - 1;      // (rows >= T: swaps only, no store)
        bf16_t* dkr = dqkv + (b * Tn + kr) * ld + D + h * HD + 8 * (ln >> 5);
        store_block_rows16(dk, scale, dkr, key_ < Tn);
        store_block_rows16(dv, 1.f, dkr + D, key_ < Tn);
      }
    } else if (kact && key < Tn) {                    // NQB 8: 8-B pieces (the 16-B form spills there)
      bf16_t* dkr = dqkv + (b * Tn + key) * ld + D + h * HD;
      bf16_t* dvr = dkr + D;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float a[4] = {dk[db][4 * g] * scale, dk[db][4 * g + 1] * scale, dk[db][4 * g + 2] * scale,
                        dk[db][4 * g + 3] * scale};
          float c[4] = {dv[db][4 * g], dv[db][4 * g + 1], dv[db][4 * g + 2], dv[db][4 * g + 3]};
          st4<bf16_t>(dkr + db * 32 + 8 * g + 4 * hf, a);
          st4<bf16_t>(dvr + db * 32 + 8 * g + 4 * hf, c);
        }
      }
    }
    ATT_ISTAMP(9);
  }
  // the last item re-staged its own K / Q / dO / V (dead blocks): retire that DMA before the LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------------------------
// Fused forward for T <= 256 (ViT: T = 197): one workgroup per (image, head) with NKB = Tp/32 waves (Tp = T rounded up
// to 32).  K and V of the head are LDS-DMA'd once into swizzled [Tp][64] images (rows >= T zero-filled); wave w owns
// queries 32w..32w+31 (Q fragments straight from global) and walks the NKB key blocks with the online softmax of
// attn_fwd_mfma (S^T = K Q^T: one query per lane column; P^T reused in registers as the B operand of O^T = V^T P^T).
// Against attn_fwd_mfma (128-query workgroups over 64-key tiles) no all-padding query or key block is computed
// (T = 197: 7 x 7 blocks of 32 instead of 8 x 8) and K/V leave HBM once per (image, head); at <= 64 KiB of LDS two
// workgroups share a CU, so one's DMA prologue overlaps the other's loop.  O leaves registers as 16-B row pieces: a
// permlane32 half swap pairs the two 8-B column groups a row is split over (cdna_hip_programming.md T21).
// ---------------------------------------------------------------------------------------------------------------
// One wave's 32 queries (q0 = 32 * wave) of one (image, head) against the NKB key blocks of the K / V images: the
// online softmax of attn_fwd_mfma, then O (bf16, 16-B row pieces), optionally O unrounded (o32) and the LSE.
template <int NKB>
VIT_DEV void fwd_queries(const bf16_t* Ks, const bf16_t* Vs, const bf16x8_t (&qf)[4], int wave, int lane, int Tn,
                         float c2, bf16_t* __restrict__ o, float* __restrict__ o32, float* __restrict__ lse, int64_t b,
                         int64_t h, int64_t bh, int64_t D) {
  constexpr int Tp = NKB * 32;
  const int hf = lane >> 5;
  const int q0 = wave * 32;
  f32x16 oacc[2] = {f32x16{}, f32x16{}};
  float m_run = -INFINITY, l_run = 0.f;
#pragma unroll
  for (int kb = 0; kb < Tp; kb += 32) {
    f32x16 sacc = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) sacc = mfma32(row_frag(Ks, kb, s, lane), qf[s], sacc);
    float x[16];
    float mloc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      x[r] = kb + acc_row(r, hf) < Tn ? sacc[r] * c2 : -INFINITY;
      mloc = fmaxf(mloc, x[r]);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      x[r] = __builtin_amdgcn_exp2f(x[r] - m_new);
      psum += x[r];
    }
    l_run = l_run * alpha + psum;
    m_run = m_new;
    oacc[0] *= alpha;
    oacc[1] *= alpha;
    const bf16x8_t pb0 = pack8(x), pb1 = pack8(x + 8);
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      oacc[db] = mfma32(tr_frag(Vs, kb, db, lane), pb0, oacc[db]);
      oacc[db] = mfma32(tr_frag(Vs, kb + 16, db, lane), pb1, oacc[db]);
    }
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.0f / l_tot;
  const int q = q0 + (lane & 31);
  if (o32 && q < Tn) {                               // fp32 O for the tiled backward's delta
    float* orow32 = o32 + (b * Tn + q) * D + h * HD + 4 * hf;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float v[4] = {oacc[db][4 * g] * inv, oacc[db][4 * g + 1] * inv, oacc[db][4 * g + 2] * inv,
                            oacc[db][4 * g + 3] * inv};
        st4<float>(orow32 + db * 32 + 8 * g, v);
      }
  }
  // lane (q, hf) holds O[q][8k + 4hf .. 8k + 4hf + 3] in group k = 4db + g; one permlane32 swap per dword pairs groups
  // (k, k+1) into 16 contiguous bytes per lane: columns 8k..8k+7 on lanes < 32, 8k+8..8k+15 on lanes >= 32
  uint32_t pk[8][2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int k = 4 * db + g;
      pk[k][0] = (uint32_t)f2bf(oacc[db][4 * g] * inv) | ((uint32_t)f2bf(oacc[db][4 * g + 1] * inv) << 16);
      pk[k][1] = (uint32_t)f2bf(oacc[db][4 * g + 2] * inv) | ((uint32_t)f2bf(oacc[db][4 * g + 3] * inv) << 16);
    }
  bf16_t* orow = o + (b * Tn + q) * D + h * HD + 8 * hf;
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
#pragma unroll
    for (int w2 = 0; w2 < 2; ++w2) {
      const auto sw = __builtin_amdgcn_permlane32_swap(pk[k][w2], pk[k + 1][w2], false, false);
      pk[k][w2] = sw[0];
      pk[k + 1][w2] = sw[1];
    }
    if (q < Tn) *reinterpret_cast<uint4*>(orow + 8 * k) = make_uint4(pk[k][0], pk[k][1], pk[k + 1][0], pk[k + 1][1]);
  }
  if (q < Tn && hf == 0) lse[bh * Tn + q] = (m_run + log2f(l_tot)) / LOG2E;
}

template <int NKB>
__global__ __launch_bounds__(NKB * 64) void attn_fwd_fused(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o,
                                                           float* __restrict__ o32, float* __restrict__ lse,
                                                           int64_t Tn64, int64_t H, float scale) {
  constexpr int Tp = NKB * 32;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * Tp * HD];
  bf16_t* Ks = smem;
  bf16_t* Vs = smem + Tp * HD;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Tn = (int)Tn64;
  const int64_t bh = blockIdx.x, b = bh / H, h = bh % H;
  const int64_t D = H * HD, ld = 3 * D;
  {
    const int64_t nb = gridDim.x / H;                  // host guarantees the tensor is < 2 GiB
    const __amdgpu_buffer_rsrc_t rq = make_rsrc_b(qkv, nb * Tn * ld * 2);
    dma_head_slice(rq, b * Tn, ld, D + h * HD, Tn, Tp, Ks, wave, lane, NKB);
    dma_head_slice(rq, b * Tn, ld, 2 * D + h * HD, Tn, Tp, Vs, wave, lane, NKB);
  }
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = glb_frag(qkv + b * Tn * ld, ld, wave * 32, Tn, h * HD, s, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  fwd_queries<NKB>(Ks, Vs, qf, wave, lane, Tn, scale * LOG2E, o, o32, lse, b, h, bh, D);
}


// ---------------------------------------------------------------------------------------------------------------
// Ring forward for T <= 256 (round 5; ViT: T = 197): persistent, one workgroup of NT = ceil(T/16) waves per CU, wave w
// owning queries 16w .. 16w + 15 of every (image, head) item the workgroup takes (items g, g + grid, ...).
//   * K and V of an item are LDS-DMA'd into a [Tp][64] image pair (Tp = 16 NT: 208 rows at T = 197, 53 KB) of a ring of
//     NS slots (3 while they fit in the 160 KiB: the item two ahead streams in while this one computes; 2 above
//     T = 208).  Each wave issues 4 of the item's 4 NT pieces, so HBM sees a continuous stream instead of the burst at
//     the start of every one-item workgroup.
//   * Q of the next item is LDS-DMA'd into the K image of the current slot once every wave is past its S products
//     (2 pieces per wave), and read as MFMA fragments after the next item's first barrier.  Every global load is
//     LDS-DMA, so the counted `s_waitcnt vmcnt` at the top of an item retires exactly this item's K / V / Q pieces and
//     leaves the ring's next K / V in flight (a register load would get a compiler wait that drains it).
//   * Exact two-pass softmax on 16x16x32 MFMAs: S^T = K Q^T for all keys (NT accumulators of 4: one query per lane
//     column, keys 4g + i of each 16-key tile on lane group g), the row max and sum over a lane's 4 NT values plus two
//     permlane swaps, P = exp2(S c2 - max c2) in place, then O^T = V^T P^T with P^T as the B operand straight from the
//     accumulators: the 32 keys of a k-step are keys 4g + 0..3 of tiles (2j, 2j + 1) for lane group g, and the V^T
//     A operand reads exactly those rows (two ds_read_b64_tr_b16).  No online rescaling, no running max.
//   * LDS images: 128-B rows, 16-B chunk c of row r at position c ^ (r & 6): conflict-free for the ds_read_b128 K / Q
//     reads (16 rows x one chunk per 16-lane group) and the transposed V reads (8 rows x 2 chunks per 32-lane half).
// Numerics as oracle _FlashBF16Attention: unnormalised P rounded to bf16 for P V, normalised by the unrounded sum.
// ---------------------------------------------------------------------------------------------------------------
VIT_DEV void ring_piece(const bf16_t* base, int64_t row0, int64_t ld, int64_t col0, int Tn, bf16_t* img, int pc,
                        int lane) {
  lane = remat(lane);
  const int r = pc * 8 + (lane >> 3);
  const int c = (lane & 7) ^ (r & 6);
  // rows >= T: finite copies of row T - 1, masked
  dma16_saddr(base + row0 * ld + col0, slice_off(min(r, Tn - 1), ld, c), img + pc * 512);
}

template <int NT>
__global__ __launch_bounds__(NT * 64, 1) void attn_fwd_ring(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o,
                                                           float* __restrict__ o32, float* __restrict__ lse,
                                                           int64_t Tn64, int64_t H, int64_t items, float scale) {
  constexpr int Tp = NT * 16;
  constexpr int IMG = Tp * HD;                        // elements of one [Tp][64] image
  constexpr int SLOT = 2 * IMG;                       // K then V
// RING_QBUF 1 (default since round 6, r41): two K/V slots + a Q double buffer, one barrier per item — the next item's
// Q and K / V are issued at the top of the item.  0: three K/V slots (K / V two items ahead) with the next item's Q
// DMA'd into the current K image after the S products: that Q load sat on the critical path (a timing-only build
// without the Q pieces ran 17% faster, r40) and the Q buffer form runs 88-92 vs 96-98 us isolated (r41).  Used while
// the five images fit (T <= 208); above that the three-slot form's two-slot case runs.
#ifndef RING_QBUF              // A/B builds: 0 = the three-slot form at every T
#define RING_QBUF 1
#endif
  constexpr bool QB = RING_QBUF && 6 * IMG * 2 <= 160 * 1024;
  constexpr int NS = !QB && 3 * SLOT * 2 <= 160 * 1024 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NS * SLOT + (QB ? 2 * IMG : 0)];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, ql = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Tn = (int)Tn64;
  const int64_t D = H * HD, ld = 3 * D;
  const float c2 = scale * LOG2E;
  const int q = wave * 16 + ql;                       // this lane's query

  auto kv_item = [&](int64_t it, int slot) {          // this wave's 4 pieces: K and V pieces 2w, 2w + 1
    int64_t b, h;
    item_bh(it, H, b, h);
    bf16_t* Ks = smem + slot * SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ring_piece(qkv, b * Tn, ld, D + h * HD, Tn, Ks, 2 * wave + i, lane);
      ring_piece(qkv, b * Tn, ld, 2 * D + h * HD, Tn, Ks + IMG, 2 * wave + i, lane);
    }
  };
  auto q_item = [&](int64_t it, int slot) {           // Q pieces 2w, 2w + 1 into the K image of `slot` (QB: Q buffer)
    int64_t b, h;
    item_bh(it, H, b, h);
    bf16_t* dst = QB ? smem + NS * SLOT + slot * IMG : smem + slot * SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i) ring_piece(qkv, b * Tn, ld, h * HD, Tn, dst, 2 * wave + i, lane);
  };

  int64_t it = blockIdx.x;
  const int64_t G = gridDim.x;
  if (it >= items) return;
  // Every wave issues the same ops in the same order every item — DMA pieces past the last item are issued too, as
  // harmless re-reads of the last item into slots nothing reads again — because `s_waitcnt vmcnt(N)` retires all but
  // the N youngest ops: N must never exceed the ops actually issued after the ones it waits for.
  const auto clampi = [&](int64_t x) { return x < items ? x : items - 1; };
  // prologue: K/V of the first item (slot 0), its Q (the K image of slot NS - 1), K/V of the second (NS = 3: slot 1)
  kv_item(it, 0);
  q_item(it, QB ? 0 : NS - 1);
  if (NS == 3) kv_item(clampi(it + G), 1);
#pragma unroll 1
  for (int k = 0; it < items; it += G, ++k) {
    // this item's K / V / Q pieces: the ring's next K / V (4, issued after the 2 Q pieces) and the previous item's 5
    // stores (4 O + lse: every wave has a valid query row, so none is skipped; 4 more with o32 only make it wait
    // longer) may stay in flight
    if (k == 0) {
      if (NS == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (NS == 3) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // every wave's pieces landed
    const int slot = k % NS, pslot = (k + NS - 1) % NS;
    const bf16_t* Ks = smem + slot * SLOT;
    const bf16_t* Vs = Ks + IMG;
    if (QB) {                                         // the next item's Q and K / V: the buffers item k - 1 used
      q_item(clampi(it + G), (k + 1) & 1);
      kv_item(clampi(it + G), pslot);
    }
    const int ln = remat(lane), qs = ln & 15, gs = ln >> 4;
    // row 16t + qs of an image has swizzle (qs & 6) for every t: a lane's two chunk offsets are loop constants and the
    // 16-row tiles are immediate offsets
    const int o0 = qs * HD + ((gs ^ (qs & 6)) << 3), o1 = qs * HD + (((4 + gs) ^ (qs & 6)) << 3);
    const bf16_t* Qs = (QB ? smem + NS * SLOT + (k & 1) * IMG : smem + pslot * SLOT) + wave * 16 * HD;
    const bf16x8_t qf0 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const s16x8*>(Qs + o0));
    const bf16x8_t qf1 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const s16x8*>(Qs + o1));

    // S^T[key][q] = sum_d K[key][d] Q[q][d]: A = K rows (16-B reads), B = Q fragments
    f32x4 s[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16x8_t k0 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const s16x8*>(Ks + t * 16 * HD + o0));
      const bf16x8_t k1 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const s16x8*>(Ks + t * 16 * HD + o1));
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf0, a, 0, 0, 0);
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf1, a, 0, 0, 0);
    }
    // every wave is past its K and Q reads: the next item's Q into this slot's K image, then the ring's next K / V
    // into the slot the previous item used (its Q image was read above)
    if (!QB) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      q_item(clampi(it + G), slot);
      kv_item(clampi(it + (NS - 1) * G), pslot);
    }

    // keys >= T only in the last tile
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((NT - 1) * 16 + 4 * g + i >= Tn) s[NT - 1][i] = -INFINITY;
    float mx[4] = {s[0][0], s[0][1], s[0][2], s[0][3]};
#pragma unroll
    for (int t = 1; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) mx[i] = fmaxf(mx[i], s[t][i]);
    float m = fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3]));
    {
      const auto a32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
      m = fmaxf(__uint_as_float(a32[0]), __uint_as_float(a32[1]));
      const auto a16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
      m = fmaxf(__uint_as_float(a16[0]), __uint_as_float(a16[1]));
    }
    const float mc = m * c2;
    float ls[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[t][i], c2, -mc));   // masked keys: exp2(-inf) = 0
        s[t][i] = p;
        ls[i] += p;
      }
    float l = (ls[0] + ls[1]) + (ls[2] + ls[3]);
    {
      const auto a32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(l), __float_as_uint(l), false, false);
      l = __uint_as_float(a32[0]) + __uint_as_float(a32[1]);
      const auto a16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(l), __float_as_uint(l), false, false);
      l = __uint_as_float(a16[0]) + __uint_as_float(a16[1]);
    }
    // O^T[d][q] += V^T[d][keys] P^T[keys][q], 32 keys per step: tiles (2j, 2j + 1); an odd NT's last step pairs tile
    // NT - 1 with zeros (its second V read re-reads tile NT - 1's rows: in bounds, multiplied by 0).  Transposed read:
    // lane 4q + p of a 16-lane group reads row 16t + 4g + q (swizzle (4g + q) & 6 for every t), columns 16 dt + 4p ..:
    // chunk 2 dt + (p >> 1) sits at 2 (dt ^ (sw >> 1)) + (p >> 1) -> one lane offset per dt
    f32x4 oacc[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                     f32x4{0.f, 0.f, 0.f, 0.f}};
    const int tq = (ln >> 2) & 3, tp = ln & 3, vr = 4 * gs + tq, sw = vr & 6;
    int vo[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) vo[dt] = vr * HD + ((2 * (dt ^ (sw >> 1)) + (tp >> 1)) << 3) + 4 * (tp & 1);
#pragma unroll
    for (int j = 0; j < (NT + 1) / 2; ++j) {
      const int t0 = 2 * j, t1 = 2 * j + 1 < NT ? 2 * j + 1 : 2 * j;
      float pv[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pv[i] = s[t0][i];
        pv[4 + i] = 2 * j + 1 < NT ? s[t1][i] : 0.f;
      }
      const bf16x8_t pb = pack8(pv);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const s16x4 lo = tr_read(Vs + t0 * 16 * HD + vo[dt]);
        const s16x4 hi = tr_read(Vs + t1 * 16 * HD + vo[dt]);
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        oacc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, v), pb, oacc[dt], 0, 0, 0);
      }
    }
    // lane (q, g) holds O[q][16 dt + 4 g + i]
    int64_t b, h;
    item_bh(it, H, b, h);
    const float inv = 1.0f / l;
    const bool qok = q < Tn;
    bf16_t* orow = o + (b * Tn + q) * D + h * HD + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const float v[4] = {oacc[dt][0] * inv, oacc[dt][1] * inv, oacc[dt][2] * inv, oacc[dt][3] * inv};
      if (qok) st4<bf16_t>(orow + 16 * dt, v);
    }
    if (qok && g == 0) lse[(b * H + h) * Tn + q] = (mc + log2f(l)) / LOG2E;
    if (o32 != nullptr && qok) {                      // the tiled backward's exact delta (attn_bwd_split forced)
      float* orow32 = o32 + (b * Tn + q) * D + h * HD + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float v[4] = {oacc[dt][0] * inv, oacc[dt][1] * inv, oacc[dt][2] * inv, oacc[dt][3] * inv};
        st4<float>(orow32 + 16 * dt, v);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ---------------------------------------------------------------------------------------------------------------
// Query 0 only (vit_attn_fwd_row0 / vit_attn_bwd_row0): one 256-thread workgroup per (image, head); keys on the
// threads for the scores, the output dimension on the lanes (4 waves over the keys, partials added in wave order)
// for the value-weighted sums.  Fixed summation orders: deterministic.
// ---------------------------------------------------------------------------------------------------------------
constexpr int R0_TMAX = 4096, R0_HDMAX = 128;

template <class T>
VIT_DEV void r0_load_row(const T* p, int hd, float* dst) {          // hd elements -> dst (LDS)
  for (int d = threadIdx.x; d < hd; d += blockDim.x) dst[d] = ld1<T>(p + d);
}

// block sum of one float per thread, fixed order (per-wave tree, then waves in order)
VIT_DEV float r0_block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}
VIT_DEV float r0_block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float m = -INFINITY;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, red[i]);
  return m;
}

// dot of a row (hd elements of T) with an LDS vector
template <class T>
VIT_DEV float r0_dot(const T* row, const float* v, int hd) {
  float acc = 0.f;
  for (int d = 0; d < hd; d += 4) {
    float x[4];
    ld4<T>(row + d, x);
    acc = fmaf(x[0], v[d], acc);
    acc = fmaf(x[1], v[d + 1], acc);
    acc = fmaf(x[2], v[d + 2], acc);
    acc = fmaf(x[3], v[d + 3], acc);
  }
  return acc;
}

template <class T>
__global__ __launch_bounds__(256) void attn_fwd_row0_kernel(const T* __restrict__ qkv, T* __restrict__ o,
                                                            float* __restrict__ lse, int64_t Tn, int64_t H, int hd,
                                                            float scale) {
  __shared__ float q0[R0_HDMAX], pv[R0_TMAX], red[8], part[4][R0_HDMAX];
  const int64_t bh = blockIdx.x, b = bh / H, h = bh % H;
  const int64_t D = H * hd, ld = 3 * D;
  const T* base = qkv + b * Tn * ld;
  r0_load_row<T>(base + h * hd, hd, q0);
  __syncthreads();
  const float c2 = scale * LOG2E;
  float mloc = -INFINITY;
  for (int64_t k = threadIdx.x; k < Tn; k += blockDim.x) {
    const float s = r0_dot<T>(base + k * ld + D + h * hd, q0, hd) * c2;
    pv[k] = s;
    mloc = fmaxf(mloc, s);
  }
  const float m = r0_block_max(mloc, red);
  float lloc = 0.f;
  for (int64_t k = threadIdx.x; k < Tn; k += blockDim.x) {
    const float p = exp2f(pv[k] - m);
    pv[k] = p;
    lloc += p;
  }
  const float l = r0_block_sum(lloc, red);              // (its barriers also publish pv)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int d0 = 0; d0 < hd; d0 += 64) {
    const int d = d0 + lane;
    float acc = 0.f;
    if (d < hd)
      for (int64_t k = w; k < Tn; k += 4) acc = fmaf(pv[k], ld1<T>(base + k * ld + 2 * D + h * hd + d), acc);
    if (d < hd) part[w][d] = acc;
  }
  __syncthreads();
  const float inv = 1.0f / l;
  for (int d = threadIdx.x; d < hd; d += blockDim.x)
    st1<T>(o + b * Tn * D + h * hd + d, (((part[0][d] + part[1][d]) + part[2][d]) + part[3][d]) * inv);
  if (threadIdx.x == 0) lse[bh * Tn] = (m + log2f(l)) / LOG2E;
}

template <class T>
__global__ __launch_bounds__(256) void attn_bwd_row0_kernel(const T* __restrict__ qkv, const T* __restrict__ d_o0,
                                                            int64_t ldo, T* __restrict__ dqkv, int64_t Tn, int64_t H,
                                                            int hd, float scale) {
  // ds[0 .. T): scores, then P, then dS; ds[R0_TMAX/2 + k]: dP_k while T <= R0_TMAX / 2 (recomputed past that)
  __shared__ float q0[R0_HDMAX], g0[R0_HDMAX], ds[R0_TMAX], red[8], part[4][R0_HDMAX];
  const int64_t bh = blockIdx.x, b = bh / H, h = bh % H;
  const int64_t D = H * hd, ld = 3 * D;
  const T* base = qkv + b * Tn * ld;
  T* dbase = dqkv + b * Tn * ld;
  const bool keep_dp = Tn <= R0_TMAX / 2;
  r0_load_row<T>(base + h * hd, hd, q0);
  r0_load_row<T>(d_o0 + b * ldo + h * hd, hd, g0);
  __syncthreads();
  // P recomputed exactly as the forward forms it (max, exp2, 1/sum): no log-sum-exp round trip, so a one-key row
  // has P = 1 and dS = 0 exactly
  const float c2 = scale * LOG2E;
  float mloc = -INFINITY;
  for (int64_t k = threadIdx.x; k < Tn; k += blockDim.x) {
    const float sk = r0_dot<T>(base + k * ld + D + h * hd, q0, hd) * c2;
    ds[k] = sk;
    mloc = fmaxf(mloc, sk);
    if (keep_dp) ds[R0_TMAX / 2 + k] = r0_dot<T>(base + k * ld + 2 * D + h * hd, g0, hd);
  }
  const float m = r0_block_max(mloc, red);
  float lloc = 0.f;
  for (int64_t k = threadIdx.x; k < Tn; k += blockDim.x) {
    const float p = exp2f(ds[k] - m);
    ds[k] = p;
    lloc += p;
  }
  const float inv = 1.0f / r0_block_sum(lloc, red);
  // P_k = p_k / l; dV_k = P_k dO0; delta = sum_k P_k dP_k
  float dloc = 0.f;
  for (int64_t k = threadIdx.x; k < Tn; k += blockDim.x) {
    const float p = ds[k] * inv;
    const float dp = keep_dp ? ds[R0_TMAX / 2 + k] : r0_dot<T>(base + k * ld + 2 * D + h * hd, g0, hd);
    ds[k] = p;
    dloc = fmaf(p, dp, dloc);
    T* dv = dbase + k * ld + 2 * D + h * hd;
    for (int d = 0; d < hd; d += 4) {
      const float v[4] = {p * g0[d], p * g0[d + 1], p * g0[d + 2], p * g0[d + 3]};
      st4<T>(dv + d, v);
    }
  }
  const float delta = r0_block_sum(dloc, red);
  // dS_k = P_k (dP_k - delta); dK_k = scale dS_k q0
  for (int64_t k = threadIdx.x; k < Tn; k += blockDim.x) {
    const float dp = keep_dp ? ds[R0_TMAX / 2 + k] : r0_dot<T>(base + k * ld + 2 * D + h * hd, g0, hd);
    const float sk = ds[k] * (dp - delta);
    ds[k] = sk;
    T* dk = dbase + k * ld + D + h * hd;
    for (int d = 0; d < hd; d += 4) {
      const float v[4] = {scale * sk * q0[d], scale * sk * q0[d + 1], scale * sk * q0[d + 2], scale * sk * q0[d + 3]};
      st4<T>(dk + d, v);
    }
  }
  __syncthreads();
  // dQ0 = scale sum_k dS_k K_k: lanes over d, waves over keys, partials in wave order
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int d0 = 0; d0 < hd; d0 += 64) {
    const int d = d0 + lane;
    float acc = 0.f;
    if (d < hd)
      for (int64_t k = w; k < Tn; k += 4) acc = fmaf(ds[k], ld1<T>(base + k * ld + D + h * hd + d), acc);
    if (d < hd) part[w][d] = acc;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < hd; d += blockDim.x)
    st1<T>(dbase + h * hd + d, scale * (((part[0][d] + part[1][d]) + part[2][d]) + part[3][d]));
}

// The same two functions with the head dimension on the lanes: LPK lanes per key, one 16-B chunk each, so a wave
// reads KPW = 64 / LPK whole 16-B-aligned key rows per instruction (the kernels above give each thread a key: 64 rows
// 4.6 KB apart per load, address-bound).  Dot products: each lane's chunk in order, then a fixed xor tree over the
// LPK lanes; value-weighted sums: per lane over its keys, a fixed xor tree over the wave's key slots, waves in order.
template <class T> struct R0Chunk;
template <> struct R0Chunk<bf16_t> {
  static constexpr int CH = 8;
  static VIT_DEV void ld(const bf16_t* p, float* x) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[2 * i] = __uint_as_float(w[i] << 16);
      x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static VIT_DEV void st(bf16_t* p, const float* x) {
    uint4 u;
    u.x = (uint32_t)f2bf(x[0]) | ((uint32_t)f2bf(x[1]) << 16);
    u.y = (uint32_t)f2bf(x[2]) | ((uint32_t)f2bf(x[3]) << 16);
    u.z = (uint32_t)f2bf(x[4]) | ((uint32_t)f2bf(x[5]) << 16);
    u.w = (uint32_t)f2bf(x[6]) | ((uint32_t)f2bf(x[7]) << 16);
    *reinterpret_cast<uint4*>(p) = u;
  }
};
template <> struct R0Chunk<float> {
  static constexpr int CH = 4;
  static VIT_DEV void ld(const float* p, float* x) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p);
    x[0] = v[0]; x[1] = v[1]; x[2] = v[2]; x[3] = v[3];
  }
  static VIT_DEV void st(float* p, const float* x) {
    *reinterpret_cast<f32x4*>(p) = f32x4{x[0], x[1], x[2], x[3]};
  }
};

template <int LPK>
VIT_DEV float r0_lane_sum(float v) {          // over the LPK lanes of one key (all of them get the sum)
#pragma unroll
  for (int off = LPK / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// acc[CH] summed over the wave's key slots (lanes with the same chunk), then over the 4 waves in order -> out[hd]
template <int LPK, int CH>
VIT_DEV void r0_slot_reduce(float* acc, float (*part)[R0_HDMAX], float* out_lds) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int off = LPK; off < 64; off <<= 1)
#pragma unroll
    for (int j = 0; j < CH; ++j) acc[j] += __shfl_xor(acc[j], off, 64);
  if (lane < LPK)
#pragma unroll
    for (int j = 0; j < CH; ++j) part[w][lane * CH + j] = acc[j];
  __syncthreads();
  for (int d = threadIdx.x; d < LPK * CH; d += blockDim.x)
    out_lds[d] = ((part[0][d] + part[1][d]) + part[2][d]) + part[3][d];
}

template <class T, int LPK>
__global__ __launch_bounds__(256) void attn_fwd_row0_vec(const T* __restrict__ qkv, T* __restrict__ o,
                                                         float* __restrict__ lse, int64_t Tn, int64_t H, float scale) {
  constexpr int CH = R0Chunk<T>::CH, HDc = LPK * CH, KPW = 64 / LPK, KPB = 4 * KPW;
  __shared__ float sc[R0_TMAX], red[8], part[4][R0_HDMAX], res[R0_HDMAX];
  const int64_t bh = blockIdx.x, b = bh / H, h = bh % H;
  const int64_t D = H * HDc, ld = 3 * D;
  const T* base = qkv + b * Tn * ld + h * HDc;
  const int lane = threadIdx.x & 63, c = lane % LPK, slot = (threadIdx.x >> 6) * KPW + lane / LPK;
  float q[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) q[j] = ld1<T>(base + c * CH + j);
  const float c2 = scale * LOG2E;
  float mloc = -INFINITY;
  for (int64_t k0 = 0; k0 < Tn; k0 += KPB) {
    const int64_t k = k0 + slot;
    float x[CH];
    float d = 0.f;
    if (k < Tn) {
      R0Chunk<T>::ld(base + k * ld + D + c * CH, x);
#pragma unroll
      for (int j = 0; j < CH; ++j) d = fmaf(x[j], q[j], d);
    }
    d = r0_lane_sum<LPK>(d) * c2;
    if (k < Tn) {
      if (c == 0) sc[k] = d;
      mloc = fmaxf(mloc, d);
    }
  }
  const float m = r0_block_max(mloc, red);               // (its barriers also publish sc)
  float lloc = 0.f;
  for (int64_t k = threadIdx.x; k < Tn; k += blockDim.x) {
    const float p = exp2f(sc[k] - m);
    sc[k] = p;
    lloc += p;
  }
  const float l = r0_block_sum(lloc, red);
  float acc[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) acc[j] = 0.f;
  for (int64_t k0 = 0; k0 < Tn; k0 += KPB) {
    const int64_t k = k0 + slot;
    if (k < Tn) {
      float x[CH];
      R0Chunk<T>::ld(base + k * ld + 2 * D + c * CH, x);
      const float p = sc[k];
#pragma unroll
      for (int j = 0; j < CH; ++j) acc[j] = fmaf(p, x[j], acc[j]);
    }
  }
  r0_slot_reduce<LPK, CH>(acc, part, res);
  __syncthreads();
  const float inv = 1.0f / l;
  for (int d = threadIdx.x; d < HDc; d += blockDim.x) st1<T>(o + b * Tn * D + h * HDc + d, res[d] * inv);
  if (threadIdx.x == 0) lse[bh * Tn] = (m + log2f(l)) / LOG2E;
}

template <class T, int LPK>
__global__ __launch_bounds__(256) void attn_bwd_row0_vec(const T* __restrict__ qkv, const T* __restrict__ d_o0,
                                                         int64_t ldo, T* __restrict__ dqkv, int64_t Tn, int64_t H,
                                                         float scale) {
  constexpr int CH = R0Chunk<T>::CH, HDc = LPK * CH, KPW = 64 / LPK, KPB = 4 * KPW;
  __shared__ float sc[R0_TMAX], dpv[R0_TMAX], red[8], part[4][R0_HDMAX], res[R0_HDMAX];
  const int64_t bh = blockIdx.x, b = bh / H, h = bh % H;
  const int64_t D = H * HDc, ld = 3 * D;
  const T* base = qkv + b * Tn * ld + h * HDc;
  T* dbase = dqkv + b * Tn * ld + h * HDc;
  const int lane = threadIdx.x & 63, c = lane % LPK, slot = (threadIdx.x >> 6) * KPW + lane / LPK;
  float q[CH], g[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    q[j] = ld1<T>(base + c * CH + j);
    g[j] = ld1<T>(d_o0 + b * ldo + h * HDc + c * CH + j);
  }
  // scores and dP_k = dO0 . V_k; P recomputed as the forward forms it (row max, exp2, 1/sum)
  const float c2 = scale * LOG2E;
  float mloc = -INFINITY;
  for (int64_t k0 = 0; k0 < Tn; k0 += KPB) {
    const int64_t k = k0 + slot;
    float sd = 0.f, pd = 0.f;
    if (k < Tn) {
      float x[CH], y[CH];
      R0Chunk<T>::ld(base + k * ld + D + c * CH, x);
      R0Chunk<T>::ld(base + k * ld + 2 * D + c * CH, y);
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        sd = fmaf(x[j], q[j], sd);
        pd = fmaf(y[j], g[j], pd);
      }
    }
    sd = r0_lane_sum<LPK>(sd) * c2;
    pd = r0_lane_sum<LPK>(pd);
    if (k < Tn) {
      if (c == 0) {
        sc[k] = sd;
        dpv[k] = pd;
      }
      mloc = fmaxf(mloc, sd);
    }
  }
  const float m = r0_block_max(mloc, red);
  float lloc = 0.f;
  for (int64_t k = threadIdx.x; k < Tn; k += blockDim.x) {
    const float p = exp2f(sc[k] - m);
    sc[k] = p;
    lloc += p;
  }
  const float inv = 1.0f / r0_block_sum(lloc, red);
  float dloc = 0.f;                                       // delta = sum_k P_k dP_k
  for (int64_t k = threadIdx.x; k < Tn; k += blockDim.x) {
    const float p = sc[k] * inv;
    sc[k] = p;
    dloc = fmaf(p, dpv[k], dloc);
  }
  const float delta = r0_block_sum(dloc, red);
  // per key: dV_k = P_k dO0, dS_k = P_k (dP_k - delta), dK_k = scale dS_k q0; dQ0 = scale sum_k dS_k K_k
  float acc[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) acc[j] = 0.f;
  for (int64_t k0 = 0; k0 < Tn; k0 += KPB) {
    const int64_t k = k0 + slot;
    if (k < Tn) {
      const float p = sc[k];
      const float ds = p * (dpv[k] - delta), f = scale * ds;
      float x[CH], v[CH];
#pragma unroll
      for (int j = 0; j < CH; ++j) v[j] = p * g[j];
      R0Chunk<T>::st(dbase + k * ld + 2 * D + c * CH, v);
#pragma unroll
      for (int j = 0; j < CH; ++j) v[j] = f * q[j];
      R0Chunk<T>::st(dbase + k * ld + D + c * CH, v);
      R0Chunk<T>::ld(base + k * ld + D + c * CH, x);
#pragma unroll
      for (int j = 0; j < CH; ++j) acc[j] = fmaf(ds, x[j], acc[j]);
    }
  }
  r0_slot_reduce<LPK, CH>(acc, part, res);
  __syncthreads();
  for (int d = threadIdx.x; d < HDc; d += blockDim.x) st1<T>(dbase + d, scale * res[d]);
}

// lanes per key for the lane-chunk kernels: hd / (16 B / element), a power of two <= 64; 0: the generic kernels
int r0_lpk(int32_t dtype, int64_t hd, const void* p0, const void* p1) {
  const int ch = dtype == VIT_BF16 ? 8 : 4;
  if (hd % ch != 0 || ((uintptr_t)p0 | (uintptr_t)p1) % 16 != 0) return 0;
  const int64_t lpk = hd / ch;
  return (lpk & (lpk - 1)) == 0 && lpk <= 64 ? (int)lpk : 0;
}

bool use_mfma(int32_t dtype, int64_t hd) { return dtype == VIT_BF16 && hd == HD; }

}  // namespace

extern "C" int vit_attn_fwd(const void* qkv, void* o, float* o32, float* lse, float* probs, int64_t B, int64_t T,
                            int64_t H, int64_t hd, float scale, int32_t dtype, int64_t max_wgs, void* stream) {
  VIT_REQUIRE(qkv && o && lse && B > 0 && T > 0 && H > 0 && hd > 0, "vit_attn_fwd: bad arguments");
  hipStream_t s = VIT_STREAM(stream);
  if (use_mfma(dtype, hd) && probs == nullptr) {
    VIT_REQUIRE(((uintptr_t)qkv) % 16 == 0 && ((uintptr_t)o) % 16 == 0, "vit_attn_fwd: pointers must be 16-B aligned");
    // (the ring splits item indices with item_bh(): B * H < 2^24; the fused backward's 2 GiB bound implies it there)
    if (T <= FB_TMAX && !vit::opt(vit::OPT_ATTN_FWD_SPLIT) && vit::opt(vit::OPT_ATTN_FWD_RING) && B * H < (1LL << 24) &&
        3 * H * hd < (1LL << 20)) {                     // (slice_off: 32-bit lane offsets)
      const int64_t items = B * H;
      unsigned grid = (unsigned)std::min<int64_t>(items, vit_cu_count());
      // per call (ABI 14: max_wgs > 0, e.g. one chain of the two-stream forward on 3/4 of the CUs), else the option
      const int64_t gopt = max_wgs > 0 ? max_wgs : vit::opt(vit::OPT_ATTN_FWD_GRID);
      if (gopt > 0) grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(items, gopt));
#define RING(NT) \
  attn_fwd_ring<NT><<<grid, NT * 64, 0, s>>>((const bf16_t*)qkv, (bf16_t*)o, o32, lse, T, H, items, scale)
      switch ((int)((T + 15) / 16)) {
        case 1: RING(1); break;   case 2: RING(2); break;   case 3: RING(3); break;   case 4: RING(4); break;
        case 5: RING(5); break;   case 6: RING(6); break;   case 7: RING(7); break;   case 8: RING(8); break;
        case 9: RING(9); break;   case 10: RING(10); break; case 11: RING(11); break; case 12: RING(12); break;
        case 13: RING(13); break; case 14: RING(14); break; case 15: RING(15); break; default: RING(16); break;
      }
#undef RING
    } else if (T <= FB_TMAX && B * T * 3 * H * hd * 2 < 0x7fffffffLL && !vit::opt(vit::OPT_ATTN_FWD_SPLIT)) {
#define FWD(NK) \
  attn_fwd_fused<NK><<<(unsigned)(B * H), NK * 64, 0, s>>>((const bf16_t*)qkv, (bf16_t*)o, o32, lse, T, H, scale)
      switch ((int)((T + 31) / 32)) {
        case 1: FWD(1); break;
        case 2: FWD(2); break;
        case 3: FWD(3); break;
        case 4: FWD(4); break;
        case 5: FWD(5); break;
        case 6: FWD(6); break;
        case 7: FWD(7); break;
        default: FWD(8); break;
      }
#undef FWD
    } else {
      const unsigned grid = (unsigned)(((T + 127) / 128) * B * H);   // 1-D: xcd_block() maps it
      attn_fwd_mfma<<<grid, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)o, o32, lse, T, H, scale);
    }
  } else {
    VIT_REQUIRE(T <= GA_TMAX && hd <= GA_HDMAX, "vit_attn_fwd(generic): T<=%d, hd<=%d", GA_TMAX, GA_HDMAX);
    VIT_REQUIRE(o32 == nullptr || dtype == VIT_BF16, "vit_attn_fwd: o32 is for bf16 outputs only");
    dim3 grid((unsigned)((T + 3) / 4), (unsigned)(B * H));
    if (dtype == VIT_BF16 && o32)
      attn_fwd_generic<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)o, lse, probs, B, T, H, hd, scale, o32);
    else if (dtype == VIT_BF16)
      attn_fwd_generic<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)o, lse, probs, B, T, H, hd, scale);
    else
      attn_fwd_generic<float><<<grid, 256, 0, s>>>((const float*)qkv, (float*)o, lse, probs, B, T, H, hd, scale);
  }
  return vit::check_launch("vit_attn_fwd");
}

namespace {
bool bwd_fused(int64_t B, int64_t T, int64_t H, int64_t hd, int32_t dtype) {
  return use_mfma(dtype, hd) && T <= FB_TMAX && B * T * 3 * H * hd * 2 < 0x7fffffffLL && 3 * H * hd < (1LL << 20) &&
         !vit::opt(vit::OPT_ATTN_BWD_SPLIT);
}
}  // namespace

extern "C" int vit_attn_bwd_uses_o32(int64_t B, int64_t T, int64_t H, int64_t hd, int32_t dtype) {
  return dtype == VIT_BF16 && !bwd_fused(B, T, H, hd, dtype) ? 1 : 0;
}

extern "C" int64_t vit_attn_bwd_workspace_bytes(int64_t B, int64_t T, int64_t H, int64_t hd, int32_t dtype) {
  if (use_mfma(dtype, hd)) return B * H * T * (int64_t)sizeof(float);
  return 2 * B * H * T * T * (int64_t)sizeof(float);
}

extern "C" int vit_attn_bwd(const void* qkv, const void* o, const float* o32, const void* d_o, const float* lse,
                            void* dqkv, int64_t B, int64_t T, int64_t H, int64_t hd, float scale, int32_t dtype,
                            void* workspace, int32_t flags, void* stream) {
  VIT_REQUIRE(qkv && o && d_o && lse && dqkv && workspace && B > 0 && T > 0 && H > 0 && hd > 0,
              "vit_attn_bwd: bad arguments");
  hipStream_t s = VIT_STREAM(stream);
  if (bwd_fused(B, T, H, hd, dtype)) {
    // persistent: one workgroup per CU (the LDS footprint allows no second), items strided over the grid; delta is
    // formed in the kernel from P and dP (o and o32 are not read)
    const int64_t items = B * H;
    // VIT_FLAG_SHARED_CUS: one workgroup per item (no cross-item prefetch, any free CU)
    int64_t grid = (flags & VIT_FLAG_SHARED_CUS) ? items : std::min<int64_t>(items, vit_cu_count());
    if (const int64_t gopt = vit::opt(vit::OPT_ATTN_BWD_GRID)) grid = std::max<int64_t>(1, std::min<int64_t>(items, gopt));
#define BWD(NQ)                                                                                                  \
  attn_bwd_fused<NQ><<<(unsigned)grid, 512, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)d_o, lse, (bf16_t*)dqkv, T, H, \
                                                    items, scale)
    switch ((int)((T + 31) / 32)) {
      case 1: BWD(1); break;
      case 2: BWD(2); break;
      case 3: BWD(3); break;
      case 4: BWD(4); break;
      case 5: BWD(5); break;
      case 6: BWD(6); break;
      case 7: BWD(7); break;
      default: BWD(8); break;
    }
#undef BWD
  } else if (use_mfma(dtype, hd)) {
    float* delta = (float*)workspace;                  // written by the dQ kernel, read by the dK / dV kernel
    const unsigned grid = (unsigned)(((T + 127) / 128) * B * H);   // 1-D: xcd_block() maps it
    if (o32)
      attn_bwd_dq_mfma<float><<<grid, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)d_o, o32, lse, delta,
                                                   (bf16_t*)dqkv, T, H, scale);
    else
      attn_bwd_dq_mfma<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)d_o, (const bf16_t*)o, lse,
                                                    delta, (bf16_t*)dqkv, T, H, scale);
    attn_bwd_dkdv_mfma<<<grid, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)d_o, lse, delta, (bf16_t*)dqkv, T, H,
                                            scale);
  } else {
    VIT_REQUIRE(T <= GA_TMAX && hd <= GA_HDMAX, "vit_attn_bwd(generic): T<=%d, hd<=%d", GA_TMAX, GA_HDMAX);
    float* Pws = (float*)workspace;
    float* dSws = Pws + B * H * T * T;
    dim3 grid((unsigned)((T + 3) / 4), (unsigned)(B * H));
    if (dtype == VIT_BF16) {
      attn_bwd_generic_rows<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)o, (const bf16_t*)d_o, lse,
                                                         (bf16_t*)dqkv, Pws, dSws, B, T, H, hd, scale, o32);
      attn_bwd_generic_cols<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)d_o, (bf16_t*)dqkv, Pws,
                                                         dSws, B, T, H, hd, scale);
    } else {
      attn_bwd_generic_rows<float><<<grid, 256, 0, s>>>((const float*)qkv, (const float*)o, (const float*)d_o, lse,
                                                        (float*)dqkv, Pws, dSws, B, T, H, hd, scale);
      attn_bwd_generic_cols<float><<<grid, 256, 0, s>>>((const float*)qkv, (const float*)d_o, (float*)dqkv, Pws, dSws,
                                                        B, T, H, hd, scale);
    }
  }
  return vit::check_launch("vit_attn_bwd");
}

#if ATT_STAMPS
extern "C" int vit_diag_attn_stamps(unsigned long long* host, int64_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_att_stamps), std::min<int64_t>(n, 16 * 8 * 8 * 6) * 8) == hipSuccess
             ? 0 : 1;
}
extern "C" int vit_diag_attn_istamps(unsigned long long* host, int64_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_att_istamps), std::min<int64_t>(n, 16 * 8 * 2 * 10) * 8) == hipSuccess
             ? 0 : 1;
}
#endif

extern "C" int vit_attn_fwd_row0(const void* qkv, void* o, float* lse, int64_t B, int64_t T, int64_t H, int64_t hd,
                                 float scale, int32_t dtype, void* stream) {
  VIT_REQUIRE(qkv && o && lse && B > 0 && T > 0 && H > 0 && hd > 0, "vit_attn_fwd_row0: bad arguments");
  VIT_REQUIRE(T <= R0_TMAX && hd <= R0_HDMAX && hd % 4 == 0, "vit_attn_fwd_row0: T <= %d, hd <= %d, hd %% 4 == 0",
              R0_TMAX, R0_HDMAX);
  VIT_REQUIRE(((uintptr_t)qkv) % (dtype == VIT_BF16 ? 8 : 16) == 0, "vit_attn_fwd_row0: qkv must be aligned");
  hipStream_t s = VIT_STREAM(stream);
  const unsigned grid = (unsigned)(B * H);
  switch (r0_lpk(dtype, hd, qkv, qkv) * (dtype == VIT_BF16 ? 1 : -1)) {
#define R0F(L, TT) attn_fwd_row0_vec<TT, L><<<grid, 256, 0, s>>>((const TT*)qkv, (TT*)o, lse, T, H, scale); \
  return vit::check_launch("vit_attn_fwd_row0")
    case 1: R0F(1, bf16_t);   case 2: R0F(2, bf16_t);   case 4: R0F(4, bf16_t);  case 8: R0F(8, bf16_t);
    case 16: R0F(16, bf16_t); case -1: R0F(1, float);   case -2: R0F(2, float);  case -4: R0F(4, float);
    case -8: R0F(8, float);   case -16: R0F(16, float); case -32: R0F(32, float);
#undef R0F
    default: break;
  }
  if (dtype == VIT_BF16)
    attn_fwd_row0_kernel<bf16_t><<<(unsigned)(B * H), 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)o, lse, T, H, (int)hd,
                                                                    scale);
  else
    attn_fwd_row0_kernel<float><<<(unsigned)(B * H), 256, 0, s>>>((const float*)qkv, (float*)o, lse, T, H, (int)hd,
                                                                   scale);
  return vit::check_launch("vit_attn_fwd_row0");
}

extern "C" int vit_attn_bwd_row0(const void* qkv, const void* d_o0, int64_t ldo, void* dqkv,
                                 int64_t B, int64_t T, int64_t H, int64_t hd, float scale, int32_t dtype,
                                 void* stream) {
  VIT_REQUIRE(qkv && d_o0 && dqkv && B > 0 && T > 0 && H > 0 && hd > 0 && ldo >= H * hd,
              "vit_attn_bwd_row0: bad arguments");
  VIT_REQUIRE(T <= R0_TMAX && hd <= R0_HDMAX && hd % 4 == 0, "vit_attn_bwd_row0: T <= %d, hd <= %d, hd %% 4 == 0",
              R0_TMAX, R0_HDMAX);
  VIT_REQUIRE(((uintptr_t)qkv) % (dtype == VIT_BF16 ? 8 : 16) == 0 && ((uintptr_t)dqkv) % (dtype == VIT_BF16 ? 8 : 16) == 0,
              "vit_attn_bwd_row0: qkv / dqkv must be aligned");
  hipStream_t s = VIT_STREAM(stream);
  const unsigned grid = (unsigned)(B * H);
  switch (r0_lpk(dtype, hd, qkv, dqkv) * (dtype == VIT_BF16 ? 1 : -1)) {
#define R0B(L, TT) attn_bwd_row0_vec<TT, L><<<grid, 256, 0, s>>>((const TT*)qkv, (const TT*)d_o0, ldo, (TT*)dqkv, T, \
                                                              H, scale); \
  return vit::check_launch("vit_attn_bwd_row0")
    case 1: R0B(1, bf16_t);   case 2: R0B(2, bf16_t);   case 4: R0B(4, bf16_t);  case 8: R0B(8, bf16_t);
    case 16: R0B(16, bf16_t); case -1: R0B(1, float);   case -2: R0B(2, float);  case -4: R0B(4, float);
    case -8: R0B(8, float);   case -16: R0B(16, float); case -32: R0B(32, float);
#undef R0B
    default: break;
  }
  if (dtype == VIT_BF16)
    attn_bwd_row0_kernel<bf16_t><<<(unsigned)(B * H), 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)d_o0, ldo,
                                                                    (bf16_t*)dqkv, T, H, (int)hd, scale);
  else
    attn_bwd_row0_kernel<float><<<(unsigned)(B * H), 256, 0, s>>>((const float*)qkv, (const float*)d_o0, ldo,
                                                                   (float*)dqkv, T, H, (int)hd, scale);
  return vit::check_launch("vit_attn_bwd_row0");
}
