// GEMM + fused epilogue for the ViT training step on gfx950.
//
//   C[i][j] = epi( alpha * sum_r A(i,r) * B(j,r) )      (see include/vit_hip.h for operand layouts and epi)
//
// bf16 path: 128x128x64 workgroup tile, 4 waves (2x2) of 64x64, v_mfma_f32_16x16x32_bf16 with fp32 accumulate.
//   Operands whose reduction dim is contiguous ("kcontig": activations in the forward, dY in dgrad) are staged as
//   [rows][64 k] with a 16-B-chunk XOR swizzle and read with ds_read_b128; operands whose reduction dim is the row
//   index ("rowstrided": W in dgrad, dY/X in wgrad) are staged as [64 k][128 rows] and read with the gfx950
//   transpose read ds_read_b64_tr_b16, so no operand is ever transposed in HBM.
//   The MFMA is issued swapped (B fragment as the A operand) so each lane ends up owning 4 consecutive output
//   COLUMNS of one row: the epilogue reads bias/residual/mask and stores 8-16 B per lane.
// f32 path: 64x64x16 tile, v_mfma_f32_32x32x2_f32 (bit-for-bit an fp32 fma chain) — exact-fp32 parity path.
// Split-K (wgrad: reduction over B*T rows): fp32 slabs per K-slice, then a deterministic reduce that applies the
// same epilogue.
#include "vit_common.h"

namespace {

struct EpiParams {
  void* c;
  int64_t ldc, m, n;
  float alpha, beta;
  const float* bias;
  int act;
  const void* aux;
  int64_t ldaux;
  int aux_dtype;
  const void* res;
  int64_t ldres, res_rowmod;
  int res_dtype;
  uint32_t drop_thr, seed;
  float drop_scale;
  int use_drop;
  int64_t grp, grp_stride;
  int vec;  // all row strides/pointers allow 4-wide vector access
  int vec8; // ... and 8-wide (16 B of bf16): the v4 wide row epilogue (required for the fast bf16 kinds)
  float* csum;     // v4 fast epilogues: per-tile column sums of C as stored -> csum[tile row][n] (colsum_part)
  int64_t row0;    // global row of local row 0 (split-K tail launch): dropout indices use the global row
  uint8_t* mask_out;  // mask4 of C: dropout keep bits, else (C as stored > 0) — see vit_hip.h
  int64_t drop_rs;    // dropout index row = (i + row0) * drop_rs (rows of a row-strided view keep their global index)
};


struct GemmArgs {
  const void* a;
  const void* b;
  int64_t lda, ldb, M, N, K;
  int64_t tiles_n;
  int64_t tiles_m, group_m;  // v4: tile order inside an XCD's contiguous range = groups of group_m tile rows,
                             // column-major inside a group (group_m = 1: row-major)
  int64_t kt_per_split;  // k-tiles per split
  float* ws;             // split-K slabs [split][M][N]
  int64_t nitems;        // v4: tiles x K-slices (work items; a persistent grid loops over them)
};

VIT_DEV float ld_any(const void* p, int dt, int64_t idx) {
  return dt == VIT_BF16 ? bf2f(((const bf16_t*)p)[idx]) : ((const float*)p)[idx];
}

template <class TO>
VIT_DEV void epilogue4(const EpiParams& e, int64_t i, int64_t j, float v[4]) {
  if (i >= e.m || j >= e.n) return;
  const int64_t orow = e.grp ? (i / e.grp) * e.grp_stride + (i % e.grp) : i;
  TO* cp = (TO*)e.c + orow * e.ldc + j;
  const int64_t rrow = e.res_rowmod ? (i % e.res_rowmod) : i;
  const bool full = e.vec && (j + 3 < e.n);
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] *= e.alpha;
  if (full) {
    if (e.beta != 0.f) {
      float o[4];
      ld4<TO>(cp, o);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += e.beta * o[r];
    }
    if (e.bias) {
      float b[4];
      ld4<float>(e.bias + j, b);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += b[r];
    }
    if (e.act == VIT_ACT_RELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
    } else if (e.act == VIT_ACT_GELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
    }
    if (e.aux) {
      if (e.aux_dtype == VIT_MASK4) {
        const uint32_t bits = ((const uint8_t*)e.aux)[mask4_byte(i, j, e.n)];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bits >> r) & 1u ? v[r] : 0.f;
      } else {
        float a[4];
        if (e.aux_dtype == VIT_BF16) ld4<bf16_t>((const bf16_t*)e.aux + i * e.ldaux + j, a);
        else ld4<float>((const float*)e.aux + i * e.ldaux + j, a);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = a[r] > 0.f ? v[r] : 0.f;
      }
    }
    uint32_t keep = 0xfu;
    if (e.use_drop) {
      const uint32_t base = (uint32_t)((i + e.row0) * e.drop_rs * e.n + j);
      keep = 0u;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool k = vit_hash_u32(e.seed, base + r) >= e.drop_thr;
        keep |= (uint32_t)k << r;
        v[r] = k ? v[r] * e.drop_scale : 0.f;
      }
    }
    if (e.res) {
      float a[4];
      if (e.res_dtype == VIT_BF16) ld4<bf16_t>((const bf16_t*)e.res + rrow * e.ldres + j, a);
      else ld4<float>((const float*)e.res + rrow * e.ldres + j, a);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += a[r];
    }
    st4<TO>(cp, v);
    if (e.mask_out) {
      uint32_t bits = 0u;
#pragma unroll
      for (int r = 0; r < 4; ++r) bits |= (uint32_t)(sizeof(TO) == 2 ? bf2f(f2bf(v[r])) > 0.f : v[r] > 0.f) << r;
      e.mask_out[mask4_byte(i, j, e.n)] = (uint8_t)(e.use_drop ? keep : bits);
    }
  } else {
    uint32_t mbits = 0u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t jj = j + r;
      if (jj >= e.n) break;
      float x = v[r];
      if (e.beta != 0.f) x += e.beta * ld1<TO>(cp + r);
      if (e.bias) x += e.bias[jj];
      if (e.act == VIT_ACT_RELU) x = fmaxf(x, 0.f);
      else if (e.act == VIT_ACT_GELU) x = gelu_erf(x);
      if (e.aux) {
        const bool on = e.aux_dtype == VIT_MASK4 ? (((const uint8_t*)e.aux)[mask4_byte(i, jj, e.n)] >> (jj & 3)) & 1u
                                                  : ld_any(e.aux, e.aux_dtype, i * e.ldaux + jj) > 0.f;
        x = on ? x : 0.f;
      }
      bool k = true;
      if (e.use_drop) {
        k = vit_hash_u32(e.seed, (uint32_t)((i + e.row0) * e.drop_rs * e.n + jj)) >= e.drop_thr;
        x = k ? x * e.drop_scale : 0.f;
      }
      if (e.res) x += ld_any(e.res, e.res_dtype, rrow * e.ldres + jj);
      st1<TO>(cp + r, x);
      const float stored = ld1<TO>(cp + r);
      mbits |= (uint32_t)(e.use_drop ? k : stored > 0.f) << ((jj & 3));
    }
    if (e.mask_out) {                                   // j % 4 == 0 here: the row's 4-column group is one byte
      e.mask_out[mask4_byte(i, j, e.n)] = (uint8_t)mbits;
    }
  }
}

VIT_DEV void slab_store4(float* ws, int64_t M, int64_t N, int64_t i, int64_t j, const float v[4]) {
  if (i >= M) return;
  float* p = ws + i * N + j;
  if ((N & 3) == 0 && j + 3 < N) {
    st4<float>(p, v);
  } else {
    for (int r = 0; r < 4 && j + r < N; ++r) p[r] = v[r];
  }
}

// ------------------------------------------------------------------------------------------------------------
// bf16 MFMA kernel
// ------------------------------------------------------------------------------------------------------------
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_ELEMS = BM * BK;  // 8192 bf16 = 16 KiB per operand per buffer

// swizzle of 16-B chunk index for the [64 k][128 rows] (256-B row) image read by ds_read_b64_tr_b16:
// conflict-free per 32-lane half for the 16x16x32 operand (rows 8g+q, g in {0,1}).
VIT_DEV int swz_rs(int kr) { return ((kr & 3) << 1) | (((kr >> 3) & 1) << 3); }

typedef short s16x4_lds __attribute__((ext_vector_type(4)));

VIT_DEV s16x4 tr_read(const bf16_t* lds_elem) {
  typedef __attribute__((address_space(3))) s16x4_lds* lds_ptr_t;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ptr_t)(lds_elem));
}

template <bool KC>
VIT_DEV void load_tile_regs(const bf16_t* __restrict__ src, int64_t ld, int64_t rows, int64_t K, int64_t r0,
                            int64_t k0, int tid, uint4 (&reg)[4]) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int q = tid + 256 * it;
    int64_t gr, gk;
    if (KC) {
      gr = r0 + (q >> 3);
      gk = k0 + (q & 7) * 8;
    } else {
      gk = k0 + (q >> 4);
      gr = r0 + (q & 15) * 8;
    }
    uint4 v = make_uint4(0, 0, 0, 0);
    if (gr < rows && gk < K) {
      const bf16_t* p = KC ? src + gr * ld + gk : src + gk * ld + gr;
      v = *reinterpret_cast<const uint4*>(p);
    }
    reg[it] = v;
  }
}

template <bool KC>
VIT_DEV void store_tile_lds(bf16_t* lds, int tid, const uint4 (&reg)[4]) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int q = tid + 256 * it;
    int off;
    if (KC) {
      const int r = q >> 3, c = q & 7;
      off = r * BK + ((c ^ (r & 7)) << 3);
    } else {
      const int kr = q >> 4, c = q & 15;
      off = kr * BM + ((c ^ swz_rs(kr)) << 3);
    }
    *reinterpret_cast<uint4*>(lds + off) = reg[it];
  }
}

// fragment of 16 rows (row block starting at rb0 inside the tile) for k-step kk (32 wide): lane holds
// X[rb0 + (lane&15)][32kk + 8(lane>>4) + 0..7]
template <bool KC>
VIT_DEV bf16x8_t read_frag(const bf16_t* lds, int rb0, int kk, int lane) {
  if (KC) {
    const int r = rb0 + (lane & 15);
    const int c = kk * 4 + (lane >> 4);
    s16x8 v = *reinterpret_cast<const s16x8*>(lds + r * BK + ((c ^ (r & 7)) << 3));
    return __builtin_bit_cast(bf16x8_t, v);
  } else {
    const int lg = lane & 15, q = lg >> 2, p = lg & 3, g = lane >> 4;
    const int kr = kk * 32 + 8 * g + q;
    const int col = rb0 + 4 * p;
    const int c = col >> 3;
    const int sw = swz_rs(kr);
    const int off1 = kr * BM + ((c ^ sw) << 3) + (p & 1) * 4;
    const int off2 = (kr + 4) * BM + ((c ^ sw) << 3) + (p & 1) * 4;
    s16x4 lo = tr_read(lds + off1);
    s16x4 hi = tr_read(lds + off2);
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

template <bool AKC, bool BKC, class TO>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmArgs g, EpiParams e) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * TILE_ELEMS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t bid = blockIdx.x;
  const int64_t tm = bid / g.tiles_n, tn = bid % g.tiles_n;
  const int64_t i0 = tm * BM, j0 = tn * BN;
  const int64_t nkt = (g.K + BK - 1) / BK;
  const int64_t kt0 = (int64_t)blockIdx.y * g.kt_per_split;
  const int64_t kt1 = min(nkt, kt0 + g.kt_per_split);
  const bf16_t* A = (const bf16_t*)g.a;
  const bf16_t* B = (const bf16_t*)g.b;

  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rb[4];
  if (kt0 < kt1) {
    load_tile_regs<AKC>(A, g.lda, g.M, g.K, i0, kt0 * BK, tid, ra);
    load_tile_regs<BKC>(B, g.ldb, g.N, g.K, j0, kt0 * BK, tid, rb);
    store_tile_lds<AKC>(smem, tid, ra);
    store_tile_lds<BKC>(smem + TILE_ELEMS, tid, rb);
  }
  __syncthreads();
  for (int64_t kt = kt0; kt < kt1; ++kt) {
    const int cur = (int)((kt - kt0) & 1);
    const bool more = kt + 1 < kt1;
    if (more) {
      load_tile_regs<AKC>(A, g.lda, g.M, g.K, i0, (kt + 1) * BK, tid, ra);
      load_tile_regs<BKC>(B, g.ldb, g.N, g.K, j0, (kt + 1) * BK, tid, rb);
    }
    const bf16_t* As = smem + cur * 2 * TILE_ELEMS;
    const bf16_t* Bs = As + TILE_ELEMS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) af[x] = read_frag<AKC>(As, wm * 64 + x * 16, kk, lane);
#pragma unroll
      for (int y = 0; y < 4; ++y) bfr[y] = read_frag<BKC>(Bs, wn * 64 + y * 16, kk, lane);
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[y], af[x], acc[x][y], 0, 0, 0);
    }
    if (more) {
      bf16_t* nb = smem + (cur ^ 1) * 2 * TILE_ELEMS;
      store_tile_lds<AKC>(nb, tid, ra);
      store_tile_lds<BKC>(nb + TILE_ELEMS, tid, rb);
    }
    __syncthreads();
  }

  // acc[x][y] = D[n][m]: m = x*16 + (lane&15), n = y*16 + 4*(lane>>4) + r
#pragma unroll
  for (int x = 0; x < 4; ++x) {
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int64_t i = i0 + wm * 64 + x * 16 + (lane & 15);
      const int64_t j = j0 + wn * 64 + y * 16 + 4 * (lane >> 4);
      float v[4] = {acc[x][y][0], acc[x][y][1], acc[x][y][2], acc[x][y][3]};
      if (g.ws) slab_store4(g.ws + (int64_t)blockIdx.y * g.M * g.N, g.M, g.N, i, j, v);
      else epilogue4<TO>(e, i, j, v);
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// bf16 MFMA kernel v2: LDS-DMA staging (buffer_load ... lds), XCD-aware tile order, 2-phase pipeline.
//   Same 128x128x64 tile, wave layout, LDS images and fragment reads as v1.  Each wave issues 4 LDS-DMA
//   instructions per operand per k-tile (1 KiB each, lane-linear destination); the XOR swizzle of the LDS image is
//   applied to the per-lane SOURCE address (the destination of an LDS-DMA is base + 16*lane).  Lanes whose source
//   lies outside the matrix get an out-of-range buffer offset, so the hardware range check writes zeros: every
//   M/N/K tail is handled without branches.  Loop: issue tile t+1 -> fragments + MFMAs on tile t -> vmcnt(0) +
//   barrier (one barrier per k-tile).
// ------------------------------------------------------------------------------------------------------------
constexpr uint32_t OOB = 0x80000000u;

VIT_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
  const uint32_t nrec = bytes >= 0x7fffffffLL ? 0x7fffffffu : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nrec, 0x00020000);
}

// Per-lane byte offsets of the 4 LDS-DMA pieces one wave issues per operand per k-tile, at k-tile 0 of the
// workgroup's K range.  Invalid rows get an out-of-range offset (stays out of range after adding the k offset,
// because every operand is < 2 GiB), so the buffer range check zero-fills them.
template <bool KC>
VIT_DEV void dma_offsets(int64_t ld, int64_t rows, int64_t r0, int64_t k0, int wave, int lane, uint32_t (&off)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ii = wave * 4 + i;
    int64_t gr, gk;
    if (KC) {
      const int r = ii * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (r & 7);
      gr = r0 + r;
      gk = k0 + c * 8;
    } else {
      const int kr = ii * 4 + (lane >> 4);
      const int c = (lane & 15) ^ swz_rs(kr);
      gk = k0 + kr;
      gr = r0 + c * 8;
    }
    const int64_t eoff = KC ? gr * ld + gk : gk * ld + gr;
    off[i] = gr < rows ? (uint32_t)(eoff * 2) : OOB;
  }
}

VIT_DEV void dma_issue(__amdgpu_buffer_rsrc_t rs, const uint32_t (&off)[4], uint32_t soff, bf16_t* lds_tile,
                       int wave) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(lds_tile + (wave * 4 + i) * 512), 16, off[i], soff, 0, 0);
}

template <bool AKC, bool BKC>
VIT_DEV void read_frags(const bf16_t* As, const bf16_t* Bs, int wm, int wn, int kk, int lane, bf16x8_t (&af)[4],
                        bf16x8_t (&bfr)[4]) {
#pragma unroll
  for (int x = 0; x < 4; ++x) af[x] = read_frag<AKC>(As, wm * 64 + x * 16, kk, lane);
#pragma unroll
  for (int y = 0; y < 4; ++y) bfr[y] = read_frag<BKC>(Bs, wn * 64 + y * 16, kk, lane);
}

// 16 MFMAs on (af, bfr) with the NEXT fragments' LDS reads (into naf, nbf) issued in the MFMA gaps: the reads in
// flight are always younger than the operands the MFMAs wait for, so hipcc's waits are exact and no LDS-read latency
// is exposed.
template <bool AKC, bool BKC>
VIT_DEV void mfma_4x4_prefetch(f32x4 (&acc)[4][4], const bf16x8_t (&af)[4], const bf16x8_t (&bfr)[4],
                               const bf16_t* As, const bf16_t* Bs, int wm, int wn, int kk, int lane,
                               bf16x8_t (&naf)[4], bf16x8_t (&nbf)[4]) {
  constexpr int RA = AKC ? 1 : 2, RB = BKC ? 1 : 2;       // LDS instructions per fragment
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int x = 0; x < 4; ++x) {
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[y], af[x], acc[x][y], 0, 0, 0);
      const int idx = x * 4 + y;
      if (idx < 4) nbf[idx] = read_frag<BKC>(Bs, wn * 64 + idx * 16, kk, lane);
      else if (idx < 8) naf[idx - 4] = read_frag<AKC>(As, wm * 64 + (idx - 4) * 16, kk, lane);
    }
  }
  __builtin_amdgcn_s_setprio(0);
  // pin the interleave: (1 MFMA, one fragment's reads) x 8, then the remaining 8 MFMAs
#define VIT_PIN(R)                                   \
  __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); \
  __builtin_amdgcn_sched_group_barrier(0x100, R, 0);
  VIT_PIN(RB) VIT_PIN(RB) VIT_PIN(RB) VIT_PIN(RB)
  VIT_PIN(RA) VIT_PIN(RA) VIT_PIN(RA) VIT_PIN(RA)
#undef VIT_PIN
  __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
}

// Loop schedule per k-tile kt (tile kt in LDS slot c, fragments of its first 32-deep half already in registers):
//   read second-half fragments of slot c | MFMAs on the first half | lgkmcnt(0) + vmcnt(0) + barrier (tile kt+1 in
//   slot c^1; every wave done reading slot c) | LDS-DMA of tile kt+2 into slot c | read first-half fragments of
//   slot c^1 | MFMAs on the second half.   LDS-read latency hides under MFMAs; each DMA has one full k-tile of lead.
template <bool AKC, bool BKC, class TO>
__global__ __launch_bounds__(256, 2) void gemm_bf16_v2(GemmArgs g, EpiParams e, int64_t a_bytes, int64_t b_bytes) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * TILE_ELEMS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware bijective remap: workgroups that share an XCD (same blockIdx % 8) get a contiguous range of tiles,
  // so neighbouring tiles (same A row panel) hit that XCD's L2.
  const int64_t nwg = gridDim.x, orig = blockIdx.x;
  const int64_t xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int64_t tm = bid / g.tiles_n, tn = bid % g.tiles_n;
  const int64_t i0 = tm * BM, j0 = tn * BN;
  const int64_t nkt = g.K / BK;                       // host guarantees K % 64 == 0 for this kernel
  const int64_t kt0 = (int64_t)blockIdx.y * g.kt_per_split;
  const int nk = (int)(min(nkt, kt0 + g.kt_per_split) - kt0);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(g.a, a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(g.b, b_bytes);
  // k-tile strides in bytes (scalar): along the row for k-contiguous operands, along rows for row-strided ones
  const uint32_t sa = AKC ? BK * 2 : (uint32_t)(BK * g.lda * 2);
  const uint32_t sb = BKC ? BK * 2 : (uint32_t)(BK * g.ldb * 2);
  uint32_t oa[4], ob[4];
  dma_offsets<AKC>(g.lda, g.M, i0, kt0 * BK, wave, lane, oa);
  dma_offsets<BKC>(g.ldb, g.N, j0, kt0 * BK, wave, lane, ob);

  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8_t a0[4], b0[4], a1[4], b1[4];
  if (nk > 0) {
    dma_issue(ra, oa, 0, smem, wave);
    dma_issue(rb, ob, 0, smem + TILE_ELEMS, wave);
  }
  if (nk > 1) {
    dma_issue(ra, oa, sa, smem + 2 * TILE_ELEMS, wave);
    dma_issue(rb, ob, sb, smem + 3 * TILE_ELEMS, wave);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 landed, tile 1 (8 pieces) still in flight
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  read_frags<AKC, BKC>(smem, smem + TILE_ELEMS, wm, wn, 0, lane, a0, b0);
  uint32_t soa = 2 * sa, sob = 2 * sb;
  for (int kt = 0; kt < nk; ++kt) {
    const int c = kt & 1;
    const bf16_t* As = smem + c * 2 * TILE_ELEMS;
    const bf16_t* An = smem + (c ^ 1) * 2 * TILE_ELEMS;
    mfma_4x4_prefetch<AKC, BKC>(acc, a0, b0, As, As + TILE_ELEMS, wm, wn, 1, lane, a1, b1);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) {
      dma_issue(ra, oa, soa, smem + c * 2 * TILE_ELEMS, wave);
      dma_issue(rb, ob, sob, smem + c * 2 * TILE_ELEMS + TILE_ELEMS, wave);
    }
    soa += sa;
    sob += sb;
    // next tile's first-half fragments (a stale slot on the last k-tile: harmless, keeps the reads unconditional)
    mfma_4x4_prefetch<AKC, BKC>(acc, a1, b1, An, An + TILE_ELEMS, wm, wn, 0, lane, a0, b0);
  }
#pragma unroll
  for (int x = 0; x < 4; ++x) {
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int64_t i = i0 + wm * 64 + x * 16 + (lane & 15);
      const int64_t j = j0 + wn * 64 + y * 16 + 4 * (lane >> 4);
      float v[4] = {acc[x][y][0], acc[x][y][1], acc[x][y][2], acc[x][y][3]};
      if (g.ws) slab_store4(g.ws + (int64_t)blockIdx.y * g.M * g.N, g.M, g.N, i, j, v);
      else epilogue4<TO>(e, i, j, v);
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// bf16 MFMA kernel v4: 256x256x64 tile, 8 waves in two ping-pong groups, one LDS-DMA half-tile per phase.
//
//   LDS (one 128 KiB array): 2 k-tile buffers x 4 half-tiles {A rows 0-127, A rows 128-255, B rows 0-127,
//   B rows 128-255}; every half-tile is exactly the 128-row operand image of v1/v2 (k-contiguous [128][64] or
//   row-strided [64][128], same swizzles), so read_frag<> is shared.
//   Wave w: group wr = w>>2, column slot wc = w&3.  Its 128x64 output is 4 quadrants (mh, nh) of 64x32: rows
//   mh*128 + wr*64 + [0,64), columns nh*128 + wc*32 + [0,32) — quadrant (mh, nh) reads only half-tiles A_mh, B_nh.
//   Waves w and w+4 share a SIMD; group 1 runs one s_barrier behind group 0, so on every SIMD one wave issues
//   LDS reads / DMA while the other runs its MFMA cluster.
//
//   Global phase f = 4t + r (k-tile t, quadrant step r), each phase = [reads | stage | vmcnt] s_barrier
//   [16 MFMA] s_barrier:
//     r=0: read A_0 frags + B_0 frags, MFMA quadrant (0,0)     r=1: read B_1, MFMA (0,1)
//     r=2: read A_1, MFMA (1,1)                                  r=3: no reads, MFMA (1,0)
//   Stage sequence s = 4u + {0,1,2,3} = k-tile u's {A_0, B_0, B_1, A_1} (2 DMA instructions per lane each);
//   stage s is issued in phase s-6 and retired by `s_waitcnt vmcnt(8)` in phase s-2 (4 stages stay in flight
//   across every barrier, never drained to 0 in the steady state); it is first read in phase s-1 or later — one
//   barrier after the retiring wait, as the staggered groups require — and it overwrites a half-tile whose last
//   read was >= 2 phases earlier.
// ------------------------------------------------------------------------------------------------------------
constexpr int HALF = 128 * BK;            // elements per half-tile image (16 KiB)

// Epilogue specialisations of v4 (chosen on the host; every one computes exactly what epilogue4 computes for the
// arguments it is chosen for).  Rows are written full-width from the LDS image, with per-column state (bias) loaded
// once per tile instead of once per row.
enum EpiKind : int {
  EPI_PLAIN = 0,      // alpha * acc
  EPI_BIAS_ACT = 1,   // act(alpha * acc + bias)
  EPI_AUX = 2,        // alpha * acc masked by aux > 0 (ReLU backward)
  EPI_BDR = 3,        // dropout(alpha * acc [+ bias]) [+ res]
  EPI_SLAB = 4,       // split-K fp32 slab
  EPI_GENERAL = 5,    // epilogue4 (beta, row groups, row-modulo residual, unaligned, any combination)
  EPI_AUXM = 6,       // alpha * acc masked by a mask4 bit (ReLU backward from the forward's stored mask)
  EPI_PATCH = 7       // alpha * acc + bias + res_f32[i % res_rowmod] stored at row (i / G) * Gs + i % G: the
                      // patch embedding (conv bias, + pos, patch rows -> token rows; vit.py:21-29,42)
};

// Kinds whose row epilogue reads a second [m][n]-shaped bf16 operand (ReLU mask / residual).  Those reads are
// issued for all 32 rows a wave owns BEFORE the accumulators go through LDS (raw bf16x4 per lane and row), so the
// epilogue pays one memory latency per tile instead of one per group of rows — each dependent load also waited for
// every store issued before it (one vmcnt counter).
template <int KIND>
VIT_DEV bool v4_has_pre(const EpiParams& e) {
  return KIND == EPI_AUX || KIND == EPI_AUXM || (KIND == EPI_BDR && e.res != nullptr);
}

template <int KIND>
VIT_DEV uint2 v4_pre_load(const EpiParams& e, int64_t i, int64_t j) {
  uint2 r = make_uint2(0u, 0u);
  if (KIND == EPI_AUXM) {                          // i % 4 == 0: the dword of rows i..i+3 (row groups are allocated whole)
    if (i < e.m && j < e.n) r.x = *reinterpret_cast<const uint32_t*>((const uint8_t*)e.aux + mask4_byte(i, j, e.n));
    return r;
  }
  if (i < e.m && j < e.n) {
    const bf16_t* p = KIND == EPI_AUX ? (const bf16_t*)e.aux + i * e.ldaux + j : (const bf16_t*)e.res + i * e.ldres + j;
    r = *reinterpret_cast<const uint2*>(p);
  }
  return r;
}

VIT_DEV void unpack_bf16x4(uint2 u, float (&a)[4]) {
  a[0] = __uint_as_float(u.x << 16);
  a[1] = __uint_as_float(u.x & 0xffff0000u);
  a[2] = __uint_as_float(u.y << 16);
  a[3] = __uint_as_float(u.y & 0xffff0000u);
}

// Returns the row's mask4 nibble (dropout keep bits for EPI_BDR with dropout, else stored value > 0) for the fast
// kinds that produce one (the caller stores 4 rows' nibbles as one dword); 0 otherwise.
// ACT (EPI_BIAS_ACT only): 0 none, 1 ReLU, 2 GELU(erf) — a template argument, so the row code carries no runtime
// activation branches (the erf body was inlined four times behind them in every unrolled row).
template <class TO, int KIND, int ACT>
VIT_DEV uint32_t v4_epi_row(const EpiParams& e, const GemmArgs& g, int64_t i, int64_t j, const float (&b4)[4],
                            float v[4], uint2 pre = make_uint2(0u, 0u)) {
  if (KIND == EPI_GENERAL) {
    epilogue4<TO>(e, i, j, v);
    return 0u;
  }
  if (KIND == EPI_SLAB) {
    slab_store4(g.ws, g.M, g.N, i, j, v);          // g.ws: this workgroup's K-slice slab (set by the kernel)
    return 0u;
  }
  if (i >= e.m || j >= e.n) return 0u;              // fast kinds: n % 4 == 0 and 16-B aligned rows (e.vec)
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] *= e.alpha;
  if (KIND == EPI_BIAS_ACT || KIND == EPI_BDR) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += b4[r];
  }
  if (KIND == EPI_BIAS_ACT && ACT == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
  } else if (KIND == EPI_BIAS_ACT && ACT == 2) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
  }
  if (KIND == EPI_AUX) {                            // aux is bf16 (host-checked), prefetched
    float a[4];
    unpack_bf16x4(pre, a);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = a[r] > 0.f ? v[r] : 0.f;
  }
  if (KIND == EPI_AUXM) {                           // pre.x = this row's mask4 nibble
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (pre.x >> r) & 1u ? v[r] : 0.f;
  }
  uint32_t keep = 0u;
  if (KIND == EPI_BDR) {
    if (e.use_drop) {
      const uint32_t base = (uint32_t)((i + e.row0) * e.drop_rs * e.n + j);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool k = vit_hash_u32(e.seed, base + r) >= e.drop_thr;
        keep |= (uint32_t)k << r;
        v[r] = k ? v[r] * e.drop_scale : 0.f;
      }
    }
    if (e.res) {                                     // res is bf16 (host-checked), prefetched
      float a[4];
      unpack_bf16x4(pre, a);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += a[r];
    }
  }
  st4<TO>((TO*)e.c + i * e.ldc + j, v);
  if (KIND == EPI_BDR && e.use_drop) return keep;
  uint32_t pos = 0u;
#pragma unroll
  for (int r = 0; r < 4; ++r) pos |= (uint32_t)(sizeof(TO) == 2 ? bf2f(f2bf(v[r])) > 0.f : v[r] > 0.f) << r;
  return pos;
}

// The pieces of one half-tile, 2 per wave, by global_load_lds_dwordx4 (per-lane 64-bit source address; the buffer
// form, buffer_load ... lds, measured 2-4% slower on the k-contiguous-A shapes, neutral on the weight gradients); rows
// past the operand are clamped to its last row (their products land in output rows / columns that are never stored).
template <bool KC>
VIT_DEV void dma_offsets4g(int64_t ld, int64_t rows, int64_t r0, int64_t k0, int wave, int lane, uint32_t (&off)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ii = wave * 2 + i;
    int64_t gr, gk;
    if (KC) {
      const int r = ii * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (r & 7);
      gr = min(r0 + r, rows - 1);
      gk = k0 + c * 8;
    } else {
      const int kr = ii * 4 + (lane >> 4);
      const int c = (lane & 15) ^ swz_rs(kr);
      gk = k0 + kr;
      gr = min(r0 + c * 8, rows - 8);
    }
    off[i] = (uint32_t)((KC ? gr * ld + gk : gk * ld + gr) * 2);
  }
}

// The two pieces are issued as inline asm, not __builtin_amdgcn_global_load_lds: the compiler's waitcnt pass cannot
// tell an LDS-DMA target from the ds_read_b64_tr_b16 reads of the other ring slots and put `s_waitcnt vmcnt(0)` in
// front of the transposed-operand reads of every phase (2 per k-tile on the dgrad layout, 3 on the weight-gradient
// layout), draining the stages the ring keeps in flight.  Completion is ordered explicitly everywhere the slots are
// read (wait_stage_retired + barrier in the k-loop, vmcnt(0) before the epilogue image and the next item).
VIT_DEV void dma_half_g(const char* base, const uint32_t (&off)[2], uint32_t soff, bf16_t* half, int wave) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(half + wave * 2 * 512));
  const uint32_t lds1 = lds + 0x400;                  // second piece's LDS base (s_mov only: SCC stays untouched)
  const char* p0 = base + off[0] + soff;
  const char* p1 = base + off[1] + soff;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile(
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off" ::"v"(p0), "v"(p1), "s"(lds), "s"(lds1)
      : "memory", "m0");
#pragma clang diagnostic pop
}

// LDS ring of the v4 k-loop: V4_SLOTS half-tile images (16 KiB each); stage s (k-tile s/4, half A0/B0/B1/A1) lands in
// slot s % V4_SLOTS and is issued V4_LEAD phases before the phase that first needs it retired.  A slot is
// re-staged (stage s + SLOTS, issued in phase s + SLOTS - LEAD) >= 2 phases after stage s's last read (phase <= s),
// so LEAD <= SLOTS - 2.  Measured (tools/r2g.sh, ViT-B/16 shapes): 10 slots / lead 8 (160 KiB, 6 stages in flight
// across every barrier) and 10 / 7 are no faster than 8 / 6 (4 stages in flight), so the default stays 8 / 6.
#ifndef V4_SLOTS
#define V4_SLOTS 8
#endif
#ifndef V4_LEAD
#define V4_LEAD (V4_SLOTS - 2)
#endif
static_assert(V4_LEAD <= V4_SLOTS - 2 && V4_LEAD >= 4 && V4_LEAD <= 8, "v4 ring: 4 <= LEAD <= SLOTS - 2, LEAD <= 8");
#ifndef V4_DMA_MFMA      // A/B builds: 1 = a phase's LDS-DMA stage issued between its two MFMA half-clusters
#define V4_DMA_MFMA 0
#endif

// vmcnt for phase f: the `left` DMA stages younger than s = f+2 that exist may stay in flight (2 instructions each)
VIT_DEV void wait_stage_retired(int left) {
  if (left >= 6) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (left == 5) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if (left == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (left == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (left == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (left == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool AKC, bool BKC>
VIT_DEV void read_a4(const bf16_t* half, int wr, int lane, bf16x8_t (&af)[4][2]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int x = 0; x < 4; ++x) af[x][kk] = read_frag<AKC>(half, wr * 64 + x * 16, kk, lane);
}

template <bool BKC>
VIT_DEV void read_b4(const bf16_t* half, int wc, int lane, bf16x8_t (&bf)[2][2]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int y = 0; y < 2; ++y) bf[y][kk] = read_frag<BKC>(half, wc * 32 + y * 16, kk, lane);
}

// Half of a quadrant's MFMAs (k-step kk of the 64-deep k-tile); V4_DMA_MFMA issues the phase's LDS-DMA between the
// two halves (the MFMA segment), not in the load segment.
VIT_DEV void mfma_quadrant_half(f32x4 (&acc)[4][2], const bf16x8_t (&af)[4][2], const bf16x8_t (&bf)[2][2], int kk) {
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
      acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[y][kk], af[x][kk], acc[x][y], 0, 0, 0);
}

// (no s_setprio around the cluster: raising the MFMA wave's priority measured 0.5-1.5% slower per GEMM, r53)
VIT_DEV void mfma_quadrant(f32x4 (&acc)[4][2], const bf16x8_t (&af)[4][2], const bf16x8_t (&bf)[2][2]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[y][kk], af[x][kk], acc[x][y], 0, 0, 0);
}

// Row-contiguous epilogue through LDS, one 128-row half of the tile per pass: the fragment layout (16 rows x 32 B
// per store instruction) becomes 1 row x 256 columns per wave instruction, so output stores and residual / mask
// loads are full-line.  Image: [128][256] fp32, 16-B chunk index XOR (row & 15) -> conflict-free b128 writes
// (8 rows per lane group) and reads (16 chunks of one row per group).  A pass's 16 row reads are issued together
// before any row is processed: one row at a time (read, lgkmcnt(0), math, store) was a serial LDS-latency chain of
// ~8 us per tile at two waves per SIMD.
template <class TO, int KIND, int ACT>
VIT_DEV void v4_epilogue(const EpiParams& e, const GemmArgs& g, const f32x4 (&acc)[2][2][4][2], bf16_t* smem4,
                         int tid, int64_t i0, int64_t j0, int64_t tm) {
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  float* ep = reinterpret_cast<float*>(smem4);
  const int64_t jcol = j0 + 4 * lane;
  float b4[4] = {0.f, 0.f, 0.f, 0.f};
  if ((KIND == EPI_BIAS_ACT || KIND == EPI_BDR) && e.bias && jcol < e.n) ld4<float>(e.bias + jcol, b4);
  // second-operand rows of both passes, in flight before the LDS round trip (see v4_has_pre)
  uint2 pre[2][16];
  const bool has_pre = v4_has_pre<KIND>(e);
  // fused column sums of C as stored (the bias gradient of the Linear whose input gradient C is)
  const bool cs_on = (KIND == EPI_PLAIN || KIND == EPI_BIAS_ACT || KIND == EPI_AUX || KIND == EPI_AUXM ||
                      KIND == EPI_BDR) && e.csum != nullptr;
  // mask4 of C: 4 rows' nibbles of this lane's column group -> one dword store per 4 rows (EPI_GENERAL writes it in
  // epilogue4, the split-K reduce after EPI_SLAB)
  const bool mk_on = KIND != EPI_GENERAL && KIND != EPI_SLAB && e.mask_out != nullptr;
  uint32_t mword = 0u;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  if (has_pre) {
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        if (KIND != EPI_AUXM) pre[mh][rr] = v4_pre_load<KIND>(e, i0 + mh * 128 + wave * 16 + rr, jcol);
        else if ((rr & 3) == 0) pre[mh][rr] = v4_pre_load<KIND>(e, i0 + mh * 128 + wave * 16 + rr, jcol);
        else pre[mh][rr] = make_uint2(pre[mh][rr & ~3].x >> (8 * (rr & 3)), 0u);
      }
  }
  __syncthreads();                                        // every wave's k-loop LDS reads are done, no DMA pending
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          const int row = wr * 64 + x * 16 + (lane & 15);
          const int chunk = (nh * 128 + wc * 32 + y * 16) / 4 + (lane >> 4);
          *reinterpret_cast<f32x4*>(ep + row * 256 + ((chunk ^ (row & 15)) << 2)) = acc[mh][nh][x][y];
        }
    __syncthreads();
    f32x4 rv[16];
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const int row = wave * 16 + rr;
      rv[rr] = *reinterpret_cast<const f32x4*>(ep + row * 256 + ((lane ^ (row & 15)) << 2));
    }
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const int row = wave * 16 + rr;
      float v[4] = {rv[rr][0], rv[rr][1], rv[rr][2], rv[rr][3]};
      const int64_t i = i0 + mh * 128 + row, j = j0 + 4 * lane;
      const uint32_t nib = v4_epi_row<TO, KIND, ACT>(e, g, i, j, b4, v, has_pre ? pre[mh][rr] : make_uint2(0u, 0u));
      if (mk_on) {
        mword |= (nib & 0xfu) << (8 * (rr & 3));
        if ((rr & 3) == 3) {                            // rows i-3..i: one dword (row groups are allocated whole)
          if (i - 3 < e.m && j < e.n)
            *reinterpret_cast<uint32_t*>(e.mask_out + mask4_byte(i - 3, j, e.n)) = mword;
          mword = 0u;
        }
      }
      if (cs_on && i < e.m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[r] += sizeof(TO) == 2 ? bf2f(f2bf(v[r])) : v[r];
      }
    }
    if (mh == 0) __syncthreads();
  }
  if (cs_on) {
    // per-lane sums of the wave's 32 rows -> LDS -> the 8 wave sums added in wave order: one row of csum per tile
    __syncthreads();
    *reinterpret_cast<f32x4*>(ep + wave * 256 + 4 * lane) = f32x4{cs[0], cs[1], cs[2], cs[3]};
    __syncthreads();
    if (tid < 256 && j0 + tid < e.n) {
      float sum = 0.f;
#pragma unroll
      for (int w8 = 0; w8 < 8; ++w8) sum += ep[w8 * 256 + tid];
      e.csum[tm * e.n + j0 + tid] = sum;
    }
  }
}

// LDS-only workgroup barrier for the epilogue: retires this wave's LDS operations, not its global loads, so the
// second-operand prefetch stays in flight across it (__syncthreads()' fence waits vmcnt(0)).  The "memory" clobber
// keeps the compiler from moving LDS accesses across it.
#define V4_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Wide row epilogue (bf16 output, fast kinds, rows 8-element aligned — e.vec8): one wave instruction stores two
// whole 256-column rows, 16 B per lane (lanes 0-31 row r, lanes 32-63 row r + 1).  Per-CU store throughput is set by
// the number of store instructions (tools/gemm_stamps.py: 8-B-per-lane rows took ~16k cycles per 256^2 tile, half
// the K = 768 k-loop), so 16-B stores halve it (cdna_hip_programming.md T21).
template <int KIND>
VIT_DEV uint4 v4_pre_load8(const EpiParams& e, int64_t i, int64_t j) {
  uint4 r = make_uint4(0u, 0u, 0u, 0u);
  if (i >= e.m || j >= e.n) return r;
  if (KIND == EPI_AUXM) {        // the dwords of column groups j/4 and j/4 + 1 of row group i/4 (8-B aligned: vec8)
    const uint2 x = *reinterpret_cast<const uint2*>((const uint8_t*)e.aux + mask4_byte(i & ~(int64_t)3, j, e.n));
    r.x = x.x;
    r.y = x.y;
    return r;
  }
  const bf16_t* p = KIND == EPI_AUX ? (const bf16_t*)e.aux + i * e.ldaux + j : (const bf16_t*)e.res + i * e.ldres + j;
  return *reinterpret_cast<const uint4*>(p);
}

VIT_DEV void unpack_bf16x8(uint4 u, float (&a)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a[2 * q] = __uint_as_float(w[q] << 16);
    a[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair (one v_cvt_pk_bf16_f32, RNE — the same rounding as f2bf)
VIT_DEV uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2_t));
}

// One row piece of 8 columns (v: fp32 accumulators in, the values as stored out when MK or CS need them).  Returns
// the 8 mask bits (bit r = column j + r) when MK: dropout keep bits for EPI_BDR with dropout, else stored value > 0.
// sh = 8 * (i % 4), the row's byte in a mask4 dword (EPI_AUXM).  The caller checks the row / column bounds.
template <int KIND, int ACT, bool MK, bool CS>
VIT_DEV uint32_t v4_epi_row8(const EpiParams& e, int64_t i, int64_t j, bf16_t* cp, const float (&b8)[8],
                             float (&v)[8], uint4 pre, int sh) {
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] *= e.alpha;
  if (KIND == EPI_BIAS_ACT || KIND == EPI_BDR || KIND == EPI_PATCH) {
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += b8[r];
  }
  if (KIND == EPI_PATCH) {                  // + the fp32 residual row i % rowmod (pos, 605 KB: L2-resident)
    const float* rp = (const float*)e.res + (int64_t)((int)i % (int)e.res_rowmod) * e.ldres + j;
    const f32x4 r0 = *reinterpret_cast<const f32x4*>(rp), r1 = *reinterpret_cast<const f32x4*>(rp + 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] += r0[r];
      v[r + 4] += r1[r];
    }
  }
  if (KIND == EPI_BIAS_ACT && ACT == 1) {
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], 0.f);
  } else if (KIND == EPI_BIAS_ACT && ACT == 2) {
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = gelu_erf(v[r]);
  }
  if (KIND == EPI_AUX) {
    float a[8];
    unpack_bf16x8(pre, a);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = a[r] > 0.f ? v[r] : 0.f;
  }
  if (KIND == EPI_AUXM) {
    const uint32_t bits = ((pre.x >> sh) & 0xfu) | (((pre.y >> sh) & 0xfu) << 4);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = (bits >> r) & 1u ? v[r] : 0.f;
  }
  uint32_t keep = 0u;
  if (KIND == EPI_BDR) {
    if (e.use_drop) {
      const uint32_t base = (uint32_t)((i + e.row0) * e.drop_rs * e.n + j);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const bool k = vit_hash_u32(e.seed, base + r) >= e.drop_thr;
        keep |= (uint32_t)k << r;
        v[r] = k ? v[r] * e.drop_scale : 0.f;
      }
    }
    if (e.res) {
      float a[8];
      unpack_bf16x8(pre, a);
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] += a[r];
    }
  }
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = pack_bf16x2(v[2 * q], v[2 * q + 1]);
  *reinterpret_cast<uint4*>(cp) = make_uint4(w[0], w[1], w[2], w[3]);
  if (MK || CS) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {                                 // as stored
      v[2 * q] = __uint_as_float(w[q] << 16);
      v[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  }
  if (!MK) return 0u;
  if (KIND == EPI_BDR && e.use_drop) return keep;
  uint32_t pos = 0u;
#pragma unroll
  for (int r = 0; r < 8; ++r) pos |= (uint32_t)(v[r] > 0.f) << r;
  return pos;
}

// Accumulator image of the wide epilogue: [128][256] fp32, physical 16-B chunk = c ^ ((c >> 4) & 1) ^ (row & 15).
// Fragment writes (8 consecutive rows per ds_write_b128 lane group, one chunk) and row-piece reads (lane l of a row
// reads chunks 2l and 2l+1, one ds_read_b128 each) are both conflict-free, and each lane's two chunks arrive in
// column order.
VIT_DEV int v4w_chunk(int row, int c) { return c ^ ((c >> 4) & 1) ^ (row & 15); }

template <int KIND, int ACT, bool MK, bool CS>
VIT_DEV void v4_epilogue_w(const EpiParams& e, const f32x4 (&acc)[2][2][4][2], float* ep, int tid, int64_t i0,
                           int64_t j0, int64_t tm) {
  // ep: a [64][256] fp32 image (64 KiB, ring slots 4-7: the persistent kernel's next-tile stages fill slots 0-3
  // meanwhile).  Pass k = tile rows [64k, 64k + 64): written by the 4 waves with wr == k & 1 (accumulator half
  // mh = k >> 1), then read by all 8 waves, 8 rows = 4 row pairs each.
  const int lane = tid & 63, l = lane & 31, hr = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int64_t j = j0 + 8 * l;
  const bool jok = j < e.n;                              // n % 8 == 0: a lane's 8 columns are all in or all out
  float b8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if ((KIND == EPI_BIAS_ACT || KIND == EPI_BDR) && e.bias && jok) {
    ld4<float>(e.bias + j, b8);
    ld4<float>(e.bias + j + 4, b8 + 4);
  }
  const bool has_pre = v4_has_pre<KIND>(e);
  // second-operand row pieces (pass k, pair p: row 64k + wave*8 + 2p + hr), one pass ahead of their use
  uint4 pre[2][4];
#define V4W_PRE(K)                                                                                  \
  do {                                                                                              \
    if (has_pre) {                                                                                  \
      _Pragma("unroll") for (int p_ = 0; p_ < 4; ++p_) {                                            \
        if (KIND != EPI_AUXM || (p_ & 1) == 0)                                                      \
          pre[(K) & 1][p_] = v4_pre_load8<KIND>(e, i0 + 64 * (K) + wave * 8 + 2 * p_ + hr, j);       \
        else                                                                                        \
          pre[(K) & 1][p_] = pre[(K) & 1][p_ - 1];    /* rows 2p-2+hr, 2p+hr: one mask4 row group */ \
      }                                                                                             \
    }                                                                                               \
  } while (0)
  V4W_PRE(0);
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  uint32_t mlo = 0u, mhi = 0u;                          // mask4 dwords of column groups 2l, 2l+1 being assembled
  V4_LDS_BARRIER();                                     // every wave's k-loop reads of slots 4-7 are done
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < 3) V4W_PRE(k + 1);
    if (wr == (k & 1)) {
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y) {
            const int row = x * 16 + (lane & 15);
            const int chunk = (nh * 128 + wc * 32 + y * 16) / 4 + (lane >> 4);
            *reinterpret_cast<f32x4*>(ep + row * 256 + (v4w_chunk(row, chunk) << 2)) = acc[k >> 1][nh][x][y];
          }
    }
    V4_LDS_BARRIER();
    f32x4 rv[4][2];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = wave * 8 + 2 * p + hr;
      rv[p][0] = *reinterpret_cast<const f32x4*>(ep + row * 256 + (v4w_chunk(row, 2 * l) << 2));
      rv[p][1] = *reinterpret_cast<const f32x4*>(ep + row * 256 + (v4w_chunk(row, 2 * l + 1) << 2));
    }
    // uniform row base of this wave's 8 rows; per lane a 32-bit element offset
    const int64_t rbase = i0 + 64 * k + wave * 8;
    const int rows_left = (int)min((int64_t)8, max((int64_t)0, e.m - rbase));
    bf16_t* cbase = (bf16_t*)e.c + rbase * e.ldc + j0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float v[8] = {rv[p][0][0], rv[p][0][1], rv[p][0][2], rv[p][0][3],
                    rv[p][1][0], rv[p][1][1], rv[p][1][2], rv[p][1][3]};
      const int rr = 2 * p + hr;
      const int64_t i = rbase + rr;
      const int sh = 8 * (rr & 3);
      uint32_t bits = 0u;
      if (jok && rr < rows_left) {
        bf16_t* cp = cbase + (uint32_t)(rr * (int)e.ldc + 8 * l);
        bits = v4_epi_row8<KIND, ACT, MK, CS>(e, i, j, cp, b8, v, has_pre ? pre[k & 1][p] : make_uint4(0u, 0u, 0u, 0u),
                                             sh);
        if (CS) {
#pragma unroll
          for (int r = 0; r < 8; ++r) cs[r] += v[r];
        }
      }
      if (MK) {
        mlo |= (bits & 0xfu) << sh;
        mhi |= ((bits >> 4) & 0xfu) << sh;
        if (p & 1) {
          // rows 4q..4q+3 done: lane l (hr 0) holds bytes 0, 2 and lane l+32 bytes 1, 3 of both dwords; lane l
          // stores column group 2l, lane l+32 column group 2l+1
          const uint32_t recv = (uint32_t)__shfl_xor((int)(hr ? mlo : mhi), 32, 64);
          if (2 * (p - 1) < rows_left && jok)
            *reinterpret_cast<uint32_t*>(e.mask_out + mask4_byte(rbase + 2 * (p - 1), j + 4 * hr, e.n)) =
                (hr ? mhi : mlo) | recv;
          mlo = mhi = 0u;
        }
      }
    }
    if (k < 3) V4_LDS_BARRIER();                        // the next pass overwrites the image
  }
#undef V4W_PRE
  if (CS) {
    // even + odd rows of the wave, then the 8 wave sums in wave order through LDS: one row of csum per tile
#pragma unroll
    for (int r = 0; r < 8; ++r) cs[r] += __shfl_xor(cs[r], 32, 64);
    V4_LDS_BARRIER();
    if (hr == 0) {
      *reinterpret_cast<f32x4*>(ep + wave * 256 + 8 * l) = f32x4{cs[0], cs[1], cs[2], cs[3]};
      *reinterpret_cast<f32x4*>(ep + wave * 256 + 8 * l + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
    }
    V4_LDS_BARRIER();
    if (tid < 256 && j0 + tid < e.n) {
      float sum = 0.f;
#pragma unroll
      for (int w8 = 0; w8 < 8; ++w8) sum += ep[w8 * 256 + tid];
      e.csum[tm * e.n + j0 + tid] = sum;
    }
  }
}

// Direct wide epilogue (the persistent kernel's; no LDS image): in the 16x16 MFMA fragment a lane holds 4 consecutive
// columns of one row in each of acc[..][y = 0] (columns 4q..4q+3 of the wave's 32-column slot, q = lane / 16) and
// acc[..][y = 1] (16 + 4q..).  One v_permlane16_swap per register pair exchanges y = 1 of 16-lane row q = 0 (2) with
// y = 0 of row q = 1 (3), after which every lane holds 8 consecutive columns, cq = 16 (q & 1) + 8 (q >> 1), of its row
// and stores them as one 16-B piece; a store instruction covers 16 rows x 64 B.  No LDS round trip, no barriers, and
// the whole LDS ring is free for the next tile's stages while this runs.
VIT_DEV void swap16(f32x4& y0, f32x4& y1) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(y0[r]), __float_as_uint(y1[r]), false, false);
    y0[r] = __uint_as_float(s[0]);
    y1[r] = __uint_as_float(s[1]);
  }
}

template <int KIND, int ACT, bool MK, bool CS>
VIT_DEV void v4_epilogue_d(const EpiParams& e, f32x4 (&acc)[2][2][4][2], float* cs_lds, int tid, int64_t i0,
                           int64_t j0, int64_t tm) {
  const int lane = tid & 63, q = lane >> 4, r16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int cq = (q & 1) * 16 + (q >> 1) * 8;
  float b8[2][8];
#pragma unroll
  for (int nh = 0; nh < 2; ++nh)
#pragma unroll
    for (int r = 0; r < 8; ++r) b8[nh][r] = 0.f;
  if ((KIND == EPI_BIAS_ACT || KIND == EPI_BDR || KIND == EPI_PATCH) && e.bias) {
#pragma unroll
    for (int nh = 0; nh < 2; ++nh) {
      const int64_t j = j0 + nh * 128 + wc * 32 + cq;
      if (j < e.n) {
        ld4<float>(e.bias + j, b8[nh]);
        ld4<float>(e.bias + j + 4, b8[nh] + 4);
      }
    }
  }
  const bool has_pre = v4_has_pre<KIND>(e);
  float cs[2][8];
#pragma unroll
  for (int nh = 0; nh < 2; ++nh)
#pragma unroll
    for (int r = 0; r < 8; ++r) cs[nh][r] = 0.f;
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
    const int64_t rbase = i0 + mh * 128 + wr * 64 + r16;       // + 16 x
    uint4 pre[2][4];
    if (has_pre) {
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int x = 0; x < 4; ++x) pre[nh][x] = v4_pre_load8<KIND>(e, rbase + 16 * x, j0 + nh * 128 + wc * 32 + cq);
    }
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        f32x4 y0 = acc[mh][nh][x][0], y1 = acc[mh][nh][x][1];
        swap16(y0, y1);
        float v[8] = {y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2], y1[3]};
        const int64_t i = rbase + 16 * x, j = j0 + nh * 128 + wc * 32 + cq;
        uint32_t bits = 0u;
        if (i < e.m && j < e.n) {
          // EPI_PATCH: output row (i / G) * Gs + i % G (32-bit: the host bounds m)
          const int64_t orow = KIND == EPI_PATCH ? (int64_t)((int)i / (int)e.grp) * e.grp_stride + (int)i % (int)e.grp : i;
          bits = v4_epi_row8<KIND, ACT, MK, CS>(e, i, j, (bf16_t*)e.c + orow * e.ldc + j, b8[nh], v,
                                                has_pre ? pre[nh][x] : make_uint4(0u, 0u, 0u, 0u), 8 * (int)(i & 3));
          if (CS) {
#pragma unroll
            for (int r = 0; r < 8; ++r) cs[nh][r] += v[r];
          }
        }
        if (MK) {
          // the 4 rows of a mask4 row group are the 4 lanes of a DPP quad: OR the bytes together, then the quad's
          // first lane stores the dwords of column groups j/4 and j/4 + 1 (8 B)
          int w = (int)(bits << (8 * (r16 & 3)));
          w |= __builtin_amdgcn_mov_dpp(w, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
          w |= __builtin_amdgcn_mov_dpp(w, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
          if ((r16 & 3) == 0 && i < e.m && j < e.n) {
            const uint32_t uw = (uint32_t)w;
            *reinterpret_cast<uint2*>(e.mask_out + mask4_byte(i, j, e.n)) =
                make_uint2(uw & 0x0f0f0f0fu, (uw >> 4) & 0x0f0f0f0fu);
          }
        }
      }
  }
  if (CS) {
    // the 16 rows of a 16-lane row -> lane r16 = 0 (fixed butterfly order), then the two row halves (wr) through LDS
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        float t = cs[nh][r];
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) t += __shfl_xor(t, o, 16);
        cs[nh][r] = t;
      }
    if (r16 == 0) {
#pragma unroll
      for (int nh = 0; nh < 2; ++nh) {
        float* d = cs_lds + wr * 256 + nh * 128 + wc * 32 + cq;
        *reinterpret_cast<f32x4*>(d) = f32x4{cs[nh][0], cs[nh][1], cs[nh][2], cs[nh][3]};
        *reinterpret_cast<f32x4*>(d + 4) = f32x4{cs[nh][4], cs[nh][5], cs[nh][6], cs[nh][7]};
      }
    }
    V4_LDS_BARRIER();
    if (tid < 256 && j0 + tid < e.n) e.csum[tm * e.n + j0 + tid] = cs_lds[tid] + cs_lds[256 + tid];
  }
}

template <int KIND, int ACT>
VIT_DEV void v4_epilogue_dd(const EpiParams& e, f32x4 (&acc)[2][2][4][2], float* cs_lds, int tid, int64_t i0,
                            int64_t j0, int64_t tm) {
  const bool mk = e.mask_out != nullptr, cs = e.csum != nullptr;
  if (mk && cs) v4_epilogue_d<KIND, ACT, true, true>(e, acc, cs_lds, tid, i0, j0, tm);
  else if (mk) v4_epilogue_d<KIND, ACT, true, false>(e, acc, cs_lds, tid, i0, j0, tm);
  else if (cs) v4_epilogue_d<KIND, ACT, false, true>(e, acc, cs_lds, tid, i0, j0, tm);
  else v4_epilogue_d<KIND, ACT, false, false>(e, acc, cs_lds, tid, i0, j0, tm);
}

// mask / column-sum switches of the wide epilogue as template arguments (no dead per-row work when off)
template <int KIND, int ACT>
VIT_DEV void v4_epilogue_wd(const EpiParams& e, const f32x4 (&acc)[2][2][4][2], float* ep, int tid, int64_t i0,
                            int64_t j0, int64_t tm) {
  const bool mk = e.mask_out != nullptr, cs = e.csum != nullptr;
  if (mk && cs) v4_epilogue_w<KIND, ACT, true, true>(e, acc, ep, tid, i0, j0, tm);
  else if (mk) v4_epilogue_w<KIND, ACT, true, false>(e, acc, ep, tid, i0, j0, tm);
  else if (cs) v4_epilogue_w<KIND, ACT, false, true>(e, acc, ep, tid, i0, j0, tm);
  else v4_epilogue_w<KIND, ACT, false, false>(e, acc, ep, tid, i0, j0, tm);
}

// Work item -> (tile row, tile column, K-slice).  Items are split-major (all tiles of K-slice 0, then slice 1, ...);
// with group_m > 1 the tiles go in groups of group_m tile rows, column-major inside a group (L2 locality: the ~32
// tiles an XCD runs at once span group_m A panels x 32/group_m B panels).
// 32-bit unsigned division (the host keeps nitems < 2^31): a 64-bit division by a runtime value expands to ~60 scalar
// instructions, and every wave splits every tile index
VIT_DEV void v4_item(const GemmArgs& g, int64_t item, int64_t& tm, int64_t& tn, int64_t& sidx) {
  const uint32_t it = (uint32_t)item, tmn = (uint32_t)g.tiles_m, tnn = (uint32_t)g.tiles_n;
  const uint32_t ntile = tmn * tnn;
  const uint32_t si = it / ntile, bid = it - si * ntile;
  sidx = si;
  if (g.group_m > 1) {
    const uint32_t gm = (uint32_t)g.group_m, span = gm * tnn, grp = bid / span, first = grp * gm;
    const uint32_t gs = min(tmn - first, gm), in = bid - grp * span;
    const uint32_t inn = in / gs;
    tm = first + (in - inn * gs);
    tn = inn;
  } else {
    const uint32_t r = bid / tnn;
    tm = r;
    tn = bid - r * tnn;
  }
}

template <bool AKC, bool BKC>
VIT_DEV void v4_offsets(const GemmArgs& g, int64_t i0, int64_t j0, int64_t k0, int wave, int lane, uint32_t (&oa0)[2],
                        uint32_t (&oa1)[2], uint32_t (&ob0)[2], uint32_t (&ob1)[2]) {
  dma_offsets4g<AKC>(g.lda, g.M, i0, k0, wave, lane, oa0);
  dma_offsets4g<AKC>(g.lda, g.M, i0 + 128, k0, wave, lane, oa1);
  dma_offsets4g<BKC>(g.ldb, g.N, j0, k0, wave, lane, ob0);
  dma_offsets4g<BKC>(g.ldb, g.N, j0 + 128, k0, wave, lane, ob1);
}

// Persistent form (the wide-epilogue kinds: bf16 output, fast epilogue; the host launches one workgroup per CU): a
// workgroup loops over its items, and as soon as a tile's k-loop is done it issues the NEXT tile's first 4 stages
// (LDS ring slots 0-3, whose last reads are behind the k-loop's final barrier) before running the epilogue on a
// 64 KiB image in slots 4-7 — the next tile's pipeline fill overlaps the epilogue instead of following it
// (tools/gemm_stamps.py: the fill was ~5.5k cycles of a ~50k-cycle K = 768 tile).  Other kinds (split-K slabs, fp32
// or general epilogues) run one item per workgroup with the 128 KiB image, as before.
template <bool AKC, bool BKC, class TO, int KIND>
__global__ __launch_bounds__(512, 1) void gemm_bf16_v4(GemmArgs g, EpiParams e, int64_t a_bytes, int64_t b_bytes) {
  // the ring, then 2 KiB for the direct epilogue's column-sum combine
  __shared__ __attribute__((aligned(16))) bf16_t smem4[V4_SLOTS * HALF + 1024];
  constexpr bool WIDE = sizeof(TO) == 2 && KIND != EPI_GENERAL && KIND != EPI_SLAB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  // Workgroups are dealt round-robin over the 8 XCDs (linear id % 8).  Each XCD owns a contiguous range of items
  // (bijective split of g.nitems into 8 parts), and its workgroups take items lo + local, lo + local + step, ...: the
  // ~32 workgroups an XCD runs at once are consecutive items (tiles of ONE K-slice that share A row panels and B
  // column panels), so the XCD's L2 serves the re-reads.  With one workgroup per item this is the previous bijective
  // block remap.  (With the K-slices on gridDim.y the hardware's linear order x + y * gridDim.x scattered a panel's
  // tiles over XCDs: the weight-gradient GEMMs fetched ~3.5x their operand bytes from beyond L2.)
  const int64_t nwg = gridDim.x, orig = blockIdx.x;
  const int64_t xcd = orig % 8, q8 = g.nitems / 8, r8 = g.nitems % 8;
  const int64_t lo = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int64_t hi = lo + q8 + (xcd < r8 ? 1 : 0);
  const int64_t step = (nwg - xcd + 7) / 8;              // workgroups on this XCD
  int64_t item = lo + orig / 8;
  if (item >= hi) return;
  int64_t tm, tn, sidx;
  v4_item(g, item, tm, tn, sidx);
  int64_t i0 = tm * 256, j0 = tn * 256;
  const int64_t nkt = g.K / BK;
  int nk = (int)max((int64_t)0, min(nkt, (sidx + 1) * g.kt_per_split) - sidx * g.kt_per_split);
  const uint32_t sa = AKC ? BK * 2 : (uint32_t)(BK * g.lda * 2);
  const uint32_t sb = BKC ? BK * 2 : (uint32_t)(BK * g.ldb * 2);
  uint32_t oa0[2], oa1[2], ob0[2], ob1[2];
  v4_offsets<AKC, BKC>(g, i0, j0, sidx * g.kt_per_split * BK, wave, remat(lane), oa0, oa1, ob0, ob1);
  const char* pa_ = (const char*)g.a;
  const char* pb_ = (const char*)g.b;
#define V4_DMA(R, P, OFF, SOFF, DST) dma_half_g(P, OFF, SOFF, DST, wave)

  // stage s -> (k-tile s>>2, half order A0, B0, B1, A1) in LDS slot s % V4_SLOTS
#define V4_SLOT(S) (smem4 + ((S) % V4_SLOTS) * HALF)
#define V4_STAGE(S)                                                                              \
  do {                                                                                           \
    const int s_ = (S), u_ = s_ >> 2;                                                            \
    bf16_t* slot_ = V4_SLOT(s_);                                                                 \
    switch (s_ & 3) {                                                                            \
      case 0: V4_DMA(ra, pa_, oa0, (uint32_t)u_ * sa, slot_); break;                             \
      case 1: V4_DMA(rb, pb_, ob0, (uint32_t)u_ * sb, slot_); break;                             \
      case 2: V4_DMA(rb, pb_, ob1, (uint32_t)u_ * sb, slot_); break;                             \
      default: V4_DMA(ra, pa_, oa1, (uint32_t)u_ * sa, slot_); break;                            \
    }                                                                                            \
  } while (0)

  int nstage = 4 * nk;
  // first item's prologue: stages 0..LEAD-1; retire stages 0 and 1 (k-tile 0's A_0, B_0) before the loop barrier
  for (int s = 0; s < V4_LEAD && s < nstage; ++s) V4_STAGE(s);
  if (nstage > 0) wait_stage_retired(min(V4_LEAD - 1, nstage - 1) - 1);

  f32x4 acc[2][2][4][2];
  bf16x8_t af[4][2], b0f[2][2], b1f[2][2];
  while (true) {
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();            // group 1 runs one barrier behind group 0
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y) acc[a][b][x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

    // One phase f = 4t + r.  STEADY: the k-tiles before the last two, where every phase issues its DMA stage and the
    // retiring wait is the constant vmcnt(2 * (LEAD - 2)) — no per-phase branches (the tail's counts are computed).
#if V4_DMA_MFMA
    // the stage goes out in the MFMA segment (below), after this wait: one stage fewer is in flight here
#define V4_PHASE_DMA(F, STEADY)                                                                  \
  do {                                                                                           \
    if (STEADY) wait_stage_retired(V4_LEAD - 3);                                                 \
    else wait_stage_retired(min(V4_LEAD - 3, nstage - 1 - ((F) + 2)));                           \
  } while (0)
#define V4_MFMA_DMA(ACC, BF, F, STEADY)                                                          \
  do {                                                                                           \
    __builtin_amdgcn_s_setprio(1);                                                               \
    mfma_quadrant_half(ACC, af, BF, 0);                                                          \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    if (STEADY || (F) + V4_LEAD < nstage) V4_STAGE((F) + V4_LEAD);                               \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    mfma_quadrant_half(ACC, af, BF, 1);                                                          \
    __builtin_amdgcn_s_setprio(0);                                                               \
  } while (0)
#define V4_PHASE_MFMA(R, F, STEADY)                                                              \
  do {                                                                                           \
    if ((R) == 0) V4_MFMA_DMA(acc[0][0], b0f, F, STEADY);                                        \
    else if ((R) == 1) V4_MFMA_DMA(acc[0][1], b1f, F, STEADY);                                   \
    else if ((R) == 2) V4_MFMA_DMA(acc[1][1], b1f, F, STEADY);                                   \
    else V4_MFMA_DMA(acc[1][0], b0f, F, STEADY);                                                 \
  } while (0)
#else
#define V4_PHASE_DMA(F, STEADY)                                                                  \
  do {                                                                                           \
    if (STEADY) {                                                                                \
      V4_STAGE((F) + V4_LEAD);                                                                   \
      wait_stage_retired(V4_LEAD - 2);                                                           \
    } else {                                                                                     \
      if ((F) + V4_LEAD < nstage) V4_STAGE((F) + V4_LEAD);                                       \
      wait_stage_retired(min(V4_LEAD - 2, nstage - 1 - ((F) + 2)));                              \
    }                                                                                            \
  } while (0)
#define V4_PHASE_MFMA(R, F, STEADY)                                                              \
  do {                                                                                           \
    if ((R) == 0) mfma_quadrant(acc[0][0], af, b0f);                                             \
    else if ((R) == 1) mfma_quadrant(acc[0][1], af, b1f);                                        \
    else if ((R) == 2) mfma_quadrant(acc[1][1], af, b1f);                                        \
    else mfma_quadrant(acc[1][0], af, b0f);                                                      \
  } while (0)
#endif
#define V4_PHASE(T, R, STEADY)                                                                   \
  do {                                                                                           \
    const int f_ = 4 * (T) + (R);                                                                \
    if ((R) == 0) {                                                                              \
      read_a4<AKC, BKC>(V4_SLOT(4 * (T)), wr, lane, af);                                         \
      read_b4<BKC>(V4_SLOT(4 * (T) + 1), wc, lane, b0f);                                         \
    } else if ((R) == 1) {                                                                       \
      read_b4<BKC>(V4_SLOT(4 * (T) + 2), wc, lane, b1f);                                         \
    } else if ((R) == 2) {                                                                       \
      read_a4<AKC, BKC>(V4_SLOT(4 * (T) + 3), wr, lane, af);                                     \
    }                                                                                            \
    V4_PHASE_DMA(f_, STEADY);                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    __builtin_amdgcn_s_barrier();                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    V4_PHASE_MFMA(R, f_, STEADY);                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    __builtin_amdgcn_s_barrier();                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                           \
  } while (0)
    const int nsteady = nk > 2 ? nk - 2 : 0;          // LEAD in [4, 8]: phases of k-tiles < nk - 2 are steady
    int t = 0;
    for (; t < nsteady; ++t) {
      V4_PHASE(t, 0, true);
      V4_PHASE(t, 1, true);
      V4_PHASE(t, 2, true);
      V4_PHASE(t, 3, true);
    }
    for (; t < nk; ++t) {
      V4_PHASE(t, 0, false);
      V4_PHASE(t, 1, false);
      V4_PHASE(t, 2, false);
      V4_PHASE(t, 3, false);
    }
#undef V4_PHASE
#undef V4_PHASE_MFMA
#undef V4_PHASE_DMA
#ifdef V4_MFMA_DMA
#undef V4_MFMA_DMA
#endif
    if (wr == 0) __builtin_amdgcn_s_barrier();            // balance group 1's extra barrier

    // next item: its first stages go out now (slots 0-3), ahead of this tile's epilogue
    const int64_t next = item + step;
    const bool have_next = WIDE && !(KIND == EPI_BIAS_ACT && e.act == VIT_ACT_GELU) && next < hi;
    int64_t ni0 = 0, nj0 = 0, ntm = 0, ntn = 0, nsidx = 0;
    int nnk = 0, npre = 0;
    if (have_next) {
      v4_item(g, next, ntm, ntn, nsidx);
      ni0 = ntm * 256;
      nj0 = ntn * 256;
      nnk = (int)max((int64_t)0, min(nkt, (nsidx + 1) * g.kt_per_split) - nsidx * g.kt_per_split);
      v4_offsets<AKC, BKC>(g, ni0, nj0, nsidx * g.kt_per_split * BK, wave, remat(lane), oa0, oa1, ob0, ob1);
      npre = min(V4_LEAD, 4 * nnk);
      for (int s = 0; s < npre; ++s) V4_STAGE(s);
    }

    // The epilogue's per-lane address arithmetic is loop-invariant; hoisted out of the persistent loop it stayed live
    // across the k-loop and spilled.  An opaque copy of tid makes the compiler recompute it per tile (a few dozen VALU).
    const int tid_e = remat(tid);
    if constexpr (WIDE) {
      float* csl = reinterpret_cast<float*>(smem4 + V4_SLOTS * HALF);
      if (KIND == EPI_BIAS_ACT && e.act == VIT_ACT_RELU) v4_epilogue_dd<KIND, 1>(e, acc, csl, tid_e, i0, j0, tm);
      else if (KIND == EPI_BIAS_ACT && e.act == VIT_ACT_GELU) {  // (the head only; erf x 8 per piece spills)
        __syncthreads();
        v4_epilogue<TO, KIND, 2>(e, g, acc, smem4, tid_e, i0, j0, tm);
      } else v4_epilogue_dd<KIND, 0>(e, acc, csl, tid_e, i0, j0, tm);
    } else {
      GemmArgs gi = g;
      if (gi.ws) gi.ws += sidx * g.M * g.N;                 // this K-slice's fp32 slab (EPI_SLAB)
      v4_epilogue<TO, KIND, 0>(e, gi, acc, smem4, tid_e, i0, j0, tm);
    }
    if (!have_next) break;
    // advance: the rest of the next item's prologue (its stages 4..LEAD-1 land in slots the image used)
    item = next;
    i0 = ni0;
    j0 = nj0;
    tm = ntm;
    nk = nnk;
    nstage = 4 * nk;
    // the offsets again (recomputed rather than kept live across the epilogue: register budget)
    v4_offsets<AKC, BKC>(g, i0, j0, nsidx * g.kt_per_split * BK, wave, remat(lane), oa0, oa1, ob0, ob1);
    // stages 0..LEAD-1 went out before the epilogue; its loads and stores are younger, so retiring stages 0 and 1
    // waits for them too (vmcnt counts in order): wait for everything
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#undef V4_STAGE
#undef V4_SLOT
#undef V4_DMA
}

// ------------------------------------------------------------------------------------------------------------
// f32 MFMA kernel (exact fp32; generic strides; any M/N/K)
// ------------------------------------------------------------------------------------------------------------
constexpr int FBM = 64, FBK = 32, FPAD = 4, FLD = FBM * FBK / 256;   // FLD: elements per thread per operand tile

// One k-tile of an operand into registers (the next tile is fetched while the current one's MFMAs run)
template <bool KC>
VIT_DEV void f32_fetch(const float* __restrict__ src, int64_t ld, int64_t rows, int64_t K, int64_t r0, int64_t k0,
                       int tid, float (&v)[FLD]) {
#pragma unroll
  for (int it = 0; it < FLD; ++it) {
    const int q = tid + 256 * it;
    int ii, rr;
    if (KC) { ii = q / FBK; rr = q % FBK; }
    else { rr = q / FBM; ii = q % FBM; }
    const int64_t gi = r0 + ii, gk = k0 + rr;
    v[it] = (gi < rows && gk < K) ? (KC ? src[gi * ld + gk] : src[gk * ld + gi]) : 0.f;
  }
}
template <bool KC>
VIT_DEV void f32_put(int tid, const float (&v)[FLD], float (*S)[FBM + FPAD]) {
#pragma unroll
  for (int it = 0; it < FLD; ++it) {
    const int q = tid + 256 * it;
    if (KC) S[q % FBK][q / FBK] = v[it];
    else S[q / FBM][q % FBM] = v[it];
  }
}

template <bool AKC, bool BKC, class TO>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g, EpiParams e) {
  __shared__ float Xs[FBK][FBM + FPAD];
  __shared__ float Ws[FBK][FBM + FPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t bid = blockIdx.x;
  const int64_t tm = bid / g.tiles_n, tn = bid % g.tiles_n;
  const int64_t i0 = tm * FBM, j0 = tn * FBM;
  const int64_t nkt = (g.K + FBK - 1) / FBK;
  const int64_t kt0 = (int64_t)blockIdx.y * g.kt_per_split;
  const int64_t kt1 = min(nkt, kt0 + g.kt_per_split);
  const float* A = (const float*)g.a;
  const float* B = (const float*)g.b;
  f32x16 acc = {};
  float ra[FLD], rb[FLD];
  if (kt0 < kt1) {
    f32_fetch<AKC>(A, g.lda, g.M, g.K, i0, kt0 * FBK, tid, ra);
    f32_fetch<BKC>(B, g.ldb, g.N, g.K, j0, kt0 * FBK, tid, rb);
  }
  for (int64_t kt = kt0; kt < kt1; ++kt) {
    f32_put<AKC>(tid, ra, Xs);
    f32_put<BKC>(tid, rb, Ws);
    __syncthreads();
    if (kt + 1 < kt1) {
      f32_fetch<AKC>(A, g.lda, g.M, g.K, i0, (kt + 1) * FBK, tid, ra);
      f32_fetch<BKC>(B, g.ldb, g.N, g.K, j0, (kt + 1) * FBK, tid, rb);
    }
#pragma unroll
    for (int kk = 0; kk < FBK / 2; ++kk) {
      const float a_op = Ws[2 * kk + (lane >> 5)][wn * 32 + (lane & 31)];
      const float b_op = Xs[2 * kk + (lane >> 5)][wm * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a_op, b_op, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // D[n][m]: m = lane&31, n = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
#pragma unroll
  for (int grp = 0; grp < 4; ++grp) {
    const int64_t i = i0 + wm * 32 + (lane & 31);
    const int64_t j = j0 + wn * 32 + 8 * grp + 4 * (lane >> 5);
    float v[4] = {acc[4 * grp], acc[4 * grp + 1], acc[4 * grp + 2], acc[4 * grp + 3]};
    if (g.ws) slab_store4(g.ws + (int64_t)blockIdx.y * g.M * g.N, g.M, g.N, i, j, v);
    else epilogue4<TO>(e, i, j, v);
  }
}

template <class TO>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int64_t M, int64_t N,
                                                            int splits, EpiParams e) {
  const int64_t nq = (N + 3) / 4;
  const int64_t total = M * nq;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / nq, j = (t % nq) * 4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    int z = 0;
    if ((N & 3) == 0) {
      // four slabs' loads in flight before their adds (same slice order: the same sums bit for bit); the slabs are
      // read once: non-temporal
      for (; z + 4 <= splits; z += 4) {
        f32x4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          x[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ws + (int64_t)(z + u) * M * N + i * N + j));
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += x[u][r];
      }
    }
    for (; z < splits; ++z) {
      const float* p = ws + (int64_t)z * M * N + i * N + j;
      if ((N & 3) == 0) {
        float x[4];
        ld4<float>(p, x);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += x[r];
      } else {
        for (int r = 0; r < 4 && j + r < N; ++r) v[r] += p[r];
      }
    }
    epilogue4<TO>(e, i, j, v);
  }
}

bool aligned(const void* p, int a) { return p == nullptr || (((uintptr_t)p) % a) == 0; }

// bf16 kernels: 1 = register-staged 128x128, 2 = LDS-DMA 128x128, 4 = LDS-DMA 256x256 ping-pong with LDS-staged
// epilogue (3 = 4: the former 256-row experiment was removed).
// Option "gemm_impl" forces a kernel (A/B runs and the per-variant tests); 0 = automatic: v4 when both output dims
// span a 256 tile, else v2.
int gemm_impl_env() {
  const int64_t v = vit::opt(vit::OPT_GEMM_IMPL);
  return (v == 1 || v == 2 || v == 4) ? (int)v : 0;
}

int gemm_impl(int64_t m, int64_t n) {
  const int forced = gemm_impl_env();
  if (forced) return forced;
  return (m >= 256 && n >= 256) ? 4 : 2;
}

// Split-K tail of a v4 GEMM (see vit_gemm): the K split for the tile rows past the last whole round of the 256 CUs,
// or 1 when that last round would be more than half full (or the kernel / epilogue does not allow it).
// *m_main = the rows of the whole rounds.
int tail_split(const vit_gemm_desc* d, int64_t* m_main) {
  *m_main = d->m;
  if (d->split_k > 1 || d->in_dtype != VIT_BF16 || d->k % BK != 0 || d->m <= 0 || d->n <= 0) return 1;
  if (gemm_impl(d->m, d->n) != 4 || d->out_group_rows != 0 || d->res_rowmod != 0) return 1;
  if (!vit::opt(vit::OPT_GEMM_TAIL)) return 1;
  const int64_t tn = (d->n + 255) / 256, tm = (d->m + 255) / 256, nkt = d->k / BK;
  const int64_t rounds = tm * tn / 256;
  // measured (ViT-B/16 B=256, N = 768): a net win at K >= 2304, a loss at K = 768, where a tile's k-loop is short
  // against the slab round trip.  Re-measured with the persistent kernel (tools/bench_ab.sh, whole step): the tail
  // saves 0.45 ms/step; extending it to K = 768 (gemm_tail_min_kt 8: proj, fc1, dgrad fc2 / proj) costs 1.0 ms.
  // Round 5, with the weight gradients on a second stream filling the idle CUs of a partial round: the QKV input
  // gradient's tail (K = 2304, 36 k-tiles) costs 0.35 ms/step, the K = 3072 ones (48) still pay: minimum 40.
  const int64_t min_kt = vit::opt(vit::OPT_GEMM_TAIL_MIN_KT);
  if (rounds < 1 || nkt < min_kt) return 1;
  const int64_t mr = rounds * 256 / tn;                    // tile rows that fill whole rounds
  const int64_t tail = (tm - mr) * tn;                     // tiles of the last, partial round
  if (tail <= 0 || 2 * tail > 256) return 1;
  const int64_t sk = std::min<int64_t>(std::min<int64_t>(256 / tail, nkt / 4), 8);
  if (sk < 2) return 1;
  *m_main = mr * 256;
  return (int)sk;
}

// Option gemm_tail_v2 (off by default): the rows of a last partial round of 256x256 tiles that the split-K tail does
// not take (K below gemm_tail_min_kt k-tiles: proj and its input gradient, fc1, the fc2 input gradient at ViT-B/16
// C2) run as 128x128 tiles (v2, two workgroups per CU): the 81 tiles of the third round of an N = 768 GEMM become 324
// quarter-tiles that all run at once, instead of 81 whole tiles on a third of the CUs.  Measured (round 5, one box,
// bench.py --opt gemm_tail_v2=0/1): 31.6 vs 33.0 ms/step — the v2 tiles with the general epilogue (and the separate
// column-sum pass) cost more than the idle CUs of the whole-tile round.  Returns 1 and *m_main = the rows of the
// whole rounds.
int tail_rows_v2(const vit_gemm_desc* d, int64_t* m_main) {
  *m_main = d->m;
  if (!vit::opt(vit::OPT_GEMM_TAIL_V2)) return 0;
  if (d->split_k > 1 || d->in_dtype != VIT_BF16 || d->k % BK != 0 || d->m <= 0 || d->n <= 0) return 0;
  if (gemm_impl(d->m, d->n) != 4 || d->out_group_rows != 0 || d->res_rowmod != 0) return 0;
  const int64_t tn = (d->n + 255) / 256, tm = (d->m + 255) / 256;
  const int64_t rounds = tm * tn / 256;
  if (rounds < 1) return 0;
  const int64_t mr = rounds * 256 / tn;                    // tile rows that fill whole rounds
  const int64_t tail = (tm - mr) * tn;
  if (tail <= 0 || 2 * tail > 256) return 0;
  *m_main = mr * 256;
  return 1;
}

}  // namespace


extern "C" int64_t vit_gemm_workspace_bytes(const vit_gemm_desc* d) {
  if (!d) return 0;
  if (d->split_k > 1) return (int64_t)d->split_k * d->m * d->n * (int64_t)sizeof(float);
  int64_t m_main = 0;
  const int sk = tail_split(d, &m_main);
  return sk > 1 ? (int64_t)sk * (d->m - m_main) * d->n * (int64_t)sizeof(float) : 0;
}

extern "C" int vit_gemm_split_k_hint(int64_t m, int64_t n, int64_t k, int in_dtype) {
  if (m <= 0 || n <= 0 || k <= 0) return 1;
  if (in_dtype == VIT_BF16 && k % BK == 0 && gemm_impl(m, n) == 4) {
    const int64_t tiles = ((m + 255) / 256) * ((n + 255) / 256);
    // slices of >= 4 k-tiles; reductions of fewer than 16 k-tiles (the pruned last block's weight gradients: K = B)
    // may go down to 1 k-tile per slice (option splitk_min_kt overrides the minimum)
    const int64_t min_env = vit::opt(vit::OPT_SPLITK_MIN_KT);
    const int64_t nkt = k / BK, min_kt = min_env > 0 ? min_env : (nkt >= 16 ? 4 : 1);
    const int64_t rounds = std::max<int64_t>(1, vit::opt(vit::OPT_SPLITK_ROUNDS));
    const int64_t s = std::min<int64_t>(std::min<int64_t>(256 * rounds / tiles, nkt / min_kt), 64);
    return (int)std::max<int64_t>(1, s);
  }
  // 128x128 tiles, two per CU, two rounds (also the fp32 parity path's split: its summation order is part of the
  // tolerances the fp32 tests were calibrated on)
  const int64_t tiles = ((m + 127) / 128) * ((n + 127) / 128);
  const int64_t nkt = (k + 63) / 64;
  const int64_t s = std::min<int64_t>(std::min<int64_t>((1024 + tiles - 1) / tiles, std::max<int64_t>(1, nkt / 8)), 32);
  return (int)std::max<int64_t>(1, s);
}

// One GEMM launch (+ the split-K reduce, + the column-sum pass when it is not fused); row0 = global row of local
// row 0 (dropout indices).
static int gemm_run(const vit_gemm_desc* d, int64_t row0, void* stream, int force_impl = 0) {
  VIT_REQUIRE(d != nullptr, "vit_gemm: null descriptor");
  VIT_REQUIRE(d->a && d->b && d->c, "vit_gemm: null operand pointer");
  VIT_REQUIRE(!d->colsum_part || d->out_group_rows == 0, "vit_gemm: colsum_part needs ungrouped output rows");
  VIT_REQUIRE(d->m > 0 && d->n > 0 && d->k > 0, "vit_gemm: bad shape m=%lld n=%lld k=%lld", (long long)d->m,
              (long long)d->n, (long long)d->k);
  VIT_REQUIRE(d->in_dtype == VIT_F32 || d->in_dtype == VIT_BF16, "vit_gemm: bad in_dtype %d", d->in_dtype);
  VIT_REQUIRE(d->out_dtype == VIT_F32 || d->out_dtype == VIT_BF16, "vit_gemm: bad out_dtype %d", d->out_dtype);
  VIT_REQUIRE(d->beta == 0.f || d->out_dtype == VIT_F32, "vit_gemm: beta requires f32 output");
  VIT_REQUIRE(!d->aux || d->aux_dtype == VIT_F32 || d->aux_dtype == VIT_BF16 || d->aux_dtype == VIT_MASK4,
              "vit_gemm: bad aux_dtype %d", d->aux_dtype);
  VIT_REQUIRE(!d->mask_out || d->out_group_rows == 0, "vit_gemm: mask_out needs ungrouped output rows");
  VIT_REQUIRE(!d->mask_out || aligned(d->mask_out, 4), "vit_gemm: mask_out must be 4-B aligned");
  VIT_REQUIRE(!d->aux || d->aux_dtype != VIT_MASK4 || aligned(d->aux, 4), "vit_gemm: mask4 aux must be 4-B aligned");
  VIT_REQUIRE(d->dropout_p >= 0.f && d->dropout_p < 1.f, "vit_gemm: dropout_p out of range");
  const int split = d->split_k > 1 ? d->split_k : 1;

  EpiParams e{};
  e.c = d->c; e.ldc = d->ldc; e.m = d->m; e.n = d->n;
  e.alpha = d->alpha; e.beta = d->beta; e.bias = d->bias; e.act = d->act;
  e.aux = d->aux; e.ldaux = d->ldaux; e.aux_dtype = d->aux_dtype;
  e.res = d->res; e.ldres = d->ldres; e.res_rowmod = d->res_rowmod; e.res_dtype = d->res_dtype;
  e.use_drop = d->dropout_p > 0.f;
  e.drop_thr = 0;
  if (e.use_drop) {
    double t = (double)d->dropout_p * 4294967296.0;
    e.drop_thr = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  }
  e.seed = d->dropout_seed;
  e.drop_scale = e.use_drop ? 1.0f / (1.0f - d->dropout_p) : 1.0f;
  e.grp = d->out_group_rows;
  e.grp_stride = d->out_group_stride;
  e.csum = nullptr;
  e.row0 = row0;
  e.mask_out = (uint8_t*)d->mask_out;
  e.drop_rs = d->dropout_row_stride > 1 ? d->dropout_row_stride : 1;
  bool cs_fused = false;
  e.vec = (d->n % 4 == 0) && (d->ldc % 4 == 0) && aligned(d->c, 16) && aligned(d->bias, 16) &&
          (!d->aux || d->aux_dtype == VIT_MASK4 || (d->ldaux % 4 == 0 && aligned(d->aux, 16))) &&
          (!d->res || (d->ldres % 4 == 0 && aligned(d->res, 16)));
  e.vec8 = e.vec && d->n % 8 == 0 && d->ldc % 8 == 0 &&
           (!d->aux || d->aux_dtype == VIT_MASK4 || (d->ldaux % 8 == 0 && aligned(d->aux, 16))) &&
           (!d->res || (d->ldres % 8 == 0 && aligned(d->res, 16))) && (!d->mask_out || aligned(d->mask_out, 8)) &&
           (!d->aux || d->aux_dtype != VIT_MASK4 || aligned(d->aux, 8));

  GemmArgs g{};
  g.a = d->a; g.b = d->b; g.lda = d->lda; g.ldb = d->ldb; g.M = d->m; g.N = d->n; g.K = d->k;
  g.ws = nullptr;
  if (split > 1) {
    VIT_REQUIRE(d->workspace && d->workspace_bytes >= vit_gemm_workspace_bytes(d),
                "vit_gemm: split_k=%d needs %lld workspace bytes", split, (long long)vit_gemm_workspace_bytes(d));
    g.ws = (float*)d->workspace;
  }
  hipStream_t s = VIT_STREAM(stream);
  const bool out_bf = d->out_dtype == VIT_BF16;

  if (d->in_dtype == VIT_BF16) {
    const bool akc = d->a_kcontig != 0, bkc = d->b_kcontig != 0;
    VIT_REQUIRE(aligned(d->a, 16) && aligned(d->b, 16), "vit_gemm(bf16): operands must be 16-B aligned");
    VIT_REQUIRE(d->lda % 8 == 0 && d->ldb % 8 == 0, "vit_gemm(bf16): lda/ldb must be multiples of 8");
    VIT_REQUIRE(akc ? d->k % 8 == 0 : d->m % 8 == 0, "vit_gemm(bf16): A contiguous dim must be a multiple of 8");
    VIT_REQUIRE(bkc ? d->k % 8 == 0 : d->n % 8 == 0, "vit_gemm(bf16): B contiguous dim must be a multiple of 8");
    VIT_REQUIRE(akc || !bkc, "vit_gemm(bf16): layout (A rowstrided, B kcontig) is not provided");
    g.tiles_n = (d->n + BN - 1) / BN;
    const int64_t tiles = ((d->m + BM - 1) / BM) * g.tiles_n;
    const int64_t nkt = (d->k + BK - 1) / BK;
    g.kt_per_split = (nkt + split - 1) / split;
    dim3 grid((unsigned)tiles, (unsigned)split), block(256);
    // operand extents in bytes (for the buffer-descriptor range check of the v2 kernel)
    const int64_t a_bytes = (akc ? (d->m - 1) * d->lda + d->k : (d->k - 1) * d->lda + d->m) * 2;
    const int64_t b_bytes = (bkc ? (d->n - 1) * d->ldb + d->k : (d->k - 1) * d->ldb + d->n) * 2;
    // v2/v4 (LDS-DMA) need whole 64-deep k-tiles (split boundaries are k-tile aligned) and operands < 2 GiB
    const int impl = force_impl ? force_impl : gemm_impl(d->m, d->n);
    const bool dma_ok = d->k % BK == 0 && a_bytes < 0x7fffffffLL && b_bytes < 0x7fffffffLL;
    const bool v2 = impl == 2 && dma_ok;
    const bool v4 = (impl == 4 || impl == 3) && dma_ok;
    GemmArgs g4 = g;
    g4.tiles_n = (d->n + 255) / 256;
    g4.tiles_m = (d->m + 255) / 256;
    {
      // Tile order inside an XCD's contiguous range: with many tile columns, row-major order puts ONE A panel and ~32
      // B panels on an XCD at once (little L2 reuse); groups of 8 tile rows, column-major inside a group, give ~8 x 4.
      // Measured (tools/gemm_ab.py): 8192^3 1146 -> 1566 TF/s; neutral on the ViT shapes (<= 12 tile columns).
      const int64_t gopt = vit::opt(vit::OPT_GEMM_GROUP_M);
      g4.group_m = gopt > 0 ? gopt : (g4.tiles_n >= 16 ? 8 : 1);
      if (g4.group_m < 1) g4.group_m = 1;
    }
    g4.kt_per_split = (nkt + split - 1) / split;
    g4.nitems = ((d->m + 255) / 256) * g4.tiles_n * split;     // tiles x K-slices, split-major
    VIT_REQUIRE(g4.nitems < (1LL << 31), "vit_gemm: %lld tiles exceed the 2^31 work items of one launch",
                (long long)g4.nitems);
    dim3 grid4((unsigned)g4.nitems, 1u);
    // v4 epilogue kind
    const bool fast = e.vec && e.grp == 0 && e.res_rowmod == 0 && e.beta == 0.f;
    int kind = EPI_GENERAL;
    if (split > 1) kind = EPI_SLAB;
    else if (fast && !e.bias && e.act == VIT_ACT_NONE && !e.aux && !e.use_drop && !e.res) kind = EPI_PLAIN;
    else if (fast && e.bias && !e.aux && !e.use_drop && !e.res) kind = EPI_BIAS_ACT;
    else if (fast && e.aux && e.aux_dtype == VIT_BF16 && !e.bias && e.act == VIT_ACT_NONE && !e.use_drop && !e.res)
      kind = EPI_AUX;
    else if (fast && e.aux && e.aux_dtype == VIT_MASK4 && !e.bias && e.act == VIT_ACT_NONE && !e.use_drop && !e.res)
      kind = EPI_AUXM;
    else if (fast && !e.aux && e.act == VIT_ACT_NONE && (e.use_drop || e.res) && (!e.res || e.res_dtype == VIT_BF16))
      kind = EPI_BDR;
    else if (e.vec && e.beta == 0.f && e.grp > 0 && e.res_rowmod > 0 && e.bias && e.res && e.res_dtype == VIT_F32 &&
             e.act == VIT_ACT_NONE && !e.aux && !e.use_drop && d->m < 0x7fffffffLL && d->ldres % 8 == 0 &&
             aligned(d->res, 16))
      kind = EPI_PATCH;
    if (vit::opt(vit::OPT_GEMM_EPI_GENERAL) && kind != EPI_SLAB) kind = EPI_GENERAL;   // A/B: the general epilogue
    // the v4 epilogue instantiation that runs (fast kinds exist for bf16 output and these operand layouts only)
    int launched = EPI_GENERAL;
    if (kind == EPI_SLAB) launched = EPI_SLAB;
    else if (out_bf && kind == EPI_PLAIN) launched = EPI_PLAIN;
    else if (out_bf && akc && bkc && (kind == EPI_BIAS_ACT || kind == EPI_BDR)) launched = kind;
    else if (out_bf && akc && !bkc && kind == EPI_AUX) launched = EPI_AUX;
    else if (out_bf && akc && !bkc && kind == EPI_AUXM) launched = EPI_AUXM;
    else if (out_bf && akc && bkc && kind == EPI_PATCH) launched = EPI_PATCH;
    if (launched != EPI_SLAB && launched != EPI_GENERAL && !e.vec8) launched = EPI_GENERAL;  // wide epilogue needs 8-wide rows
    cs_fused = v4 && d->colsum_part && launched != EPI_SLAB && launched != EPI_GENERAL;
    // persistent grid (one workgroup per CU looping over items) for the wide-epilogue kinds; option gemm_persist 0:
    // one workgroup per item (A/B switch)
    {
      const bool persist = launched != EPI_SLAB && launched != EPI_GENERAL && e.act != VIT_ACT_GELU &&
                           !(d->flags & VIT_FLAG_SHARED_CUS) && vit::opt(vit::OPT_GEMM_PERSIST);
      if (persist && g4.nitems > vit_cu_count()) grid4.x = (unsigned)vit_cu_count();
    }
    e.csum = cs_fused ? d->colsum_part : nullptr;
#define V4(AK, BKK, TO, KIND) gemm_bf16_v4<AK, BKK, TO, KIND><<<grid4, 512, 0, s>>>(g4, e, a_bytes, b_bytes)
#define LAUNCH_BF(AK, BKK)                                                                                     \
  do {                                                                                                         \
    if (v4) {                                                                                                  \
      if (launched == EPI_SLAB) V4(AK, BKK, float, EPI_SLAB);                                                  \
      else if (!out_bf) V4(AK, BKK, float, EPI_GENERAL);                                                       \
      else if (launched == EPI_PLAIN) V4(AK, BKK, bf16_t, EPI_PLAIN);                                          \
      else if (AK && BKK && launched == EPI_BIAS_ACT) V4(AK, BKK, bf16_t, EPI_BIAS_ACT);                       \
      else if (AK && BKK && launched == EPI_BDR) V4(AK, BKK, bf16_t, EPI_BDR);                                 \
      else if (AK && !BKK && launched == EPI_AUX) V4(AK, BKK, bf16_t, EPI_AUX);                                \
      else if (AK && !BKK && launched == EPI_AUXM) V4(AK, BKK, bf16_t, EPI_AUXM);                              \
      else if (AK && BKK && launched == EPI_PATCH) V4(AK, BKK, bf16_t, EPI_PATCH);                             \
      else V4(AK, BKK, bf16_t, EPI_GENERAL);                                                                   \
    } else if (v2) {                                                                                           \
      if (out_bf && split == 1) gemm_bf16_v2<AK, BKK, bf16_t><<<grid, block, 0, s>>>(g, e, a_bytes, b_bytes);     \
      else gemm_bf16_v2<AK, BKK, float><<<grid, block, 0, s>>>(g, e, a_bytes, b_bytes);                         \
    } else {                                                                                                   \
      if (out_bf && split == 1) gemm_bf16_kernel<AK, BKK, bf16_t><<<grid, block, 0, s>>>(g, e);                \
      else gemm_bf16_kernel<AK, BKK, float><<<grid, block, 0, s>>>(g, e);                                      \
    }                                                                                                          \
  } while (0)
    if (akc && bkc) LAUNCH_BF(true, true);
    else if (akc && !bkc) LAUNCH_BF(true, false);
    else LAUNCH_BF(false, false);
#undef LAUNCH_BF
#undef V4
  } else {
    g.tiles_n = (d->n + FBM - 1) / FBM;
    const int64_t tiles = ((d->m + FBM - 1) / FBM) * g.tiles_n;
    const int64_t nkt = (d->k + FBK - 1) / FBK;
    g.kt_per_split = (nkt + split - 1) / split;
    dim3 grid((unsigned)tiles, (unsigned)split), block(256);
    const bool akc = d->a_kcontig != 0, bkc = d->b_kcontig != 0;
#define LAUNCH_F(AK, BKK)                                                                               \
  do {                                                                                                  \
    if (out_bf && split == 1) gemm_f32_kernel<AK, BKK, bf16_t><<<grid, block, 0, s>>>(g, e);            \
    else gemm_f32_kernel<AK, BKK, float><<<grid, block, 0, s>>>(g, e);                                  \
  } while (0)
    if (akc && bkc) LAUNCH_F(true, true);
    else if (akc) LAUNCH_F(true, false);
    else if (bkc) LAUNCH_F(false, true);
    else LAUNCH_F(false, false);
#undef LAUNCH_F
  }
  if (split > 1) {
    const int64_t total = d->m * ((d->n + 3) / 4);
    const int64_t blocks = std::min<int64_t>((total + 255) / 256, 4096);
    if (out_bf) splitk_reduce_kernel<bf16_t><<<(unsigned)blocks, 256, 0, s>>>(g.ws, d->m, d->n, split, e);
    else splitk_reduce_kernel<float><<<(unsigned)blocks, 256, 0, s>>>(g.ws, d->m, d->n, split, e);
  }
  if (d->colsum_part && !cs_fused)
    vit::colsum_parts_launch(d->c, d->ldc, d->out_dtype, d->m, d->n, 256, d->colsum_part, s);
  return vit::check_launch("vit_gemm");
}

// When the 256x256 tiles leave the last round of the 256 CUs at most half full (tail_split), the whole rounds run as
// one launch and the remaining tile rows run split-K over the otherwise idle CUs: fp32 slabs in the caller's
// workspace, then the deterministic reduce applies the same epilogue (dropout indices keep the global row; column
// sums land in the same colsum_part rows).  Without a large enough workspace the GEMM runs unsplit.
extern "C" int vit_gemm(const vit_gemm_desc* d, void* stream) {
  VIT_REQUIRE(d != nullptr, "vit_gemm: null descriptor");
  int64_t m_main = 0;
  int sk = tail_split(d, &m_main);
  const bool split_tail = sk > 1 && d->workspace && d->workspace_bytes >= vit_gemm_workspace_bytes(d);
  const bool v2_tail = !split_tail && tail_rows_v2(d, &m_main);
  if (split_tail || v2_tail) {
    vit_gemm_desc dm = *d;
    dm.m = m_main;
    const int rc = gemm_run(&dm, d->dropout_row0, stream);
    if (rc) return rc;
    auto esz = [](int32_t t) { return t == VIT_BF16 ? (int64_t)2 : (int64_t)4; };
    const int64_t r = m_main;
    vit_gemm_desc dt = *d;
    dt.a = (const char*)d->a + (d->a_kcontig ? r * d->lda : r) * 2;
    dt.c = (char*)d->c + r * d->ldc * esz(d->out_dtype);
    const int64_t mask_off = (r / 4) * ((d->n + 3) / 4) * 4;   // r % 256 == 0: whole mask4 row groups
    if (d->aux) dt.aux = (const char*)d->aux + (d->aux_dtype == VIT_MASK4 ? mask_off : r * d->ldaux * esz(d->aux_dtype));
    if (d->mask_out) dt.mask_out = (char*)d->mask_out + mask_off;
    if (d->res) dt.res = (const char*)d->res + r * d->ldres * esz(d->res_dtype);
    if (d->colsum_part) dt.colsum_part = d->colsum_part + (r / 256) * d->n;
    dt.m = d->m - r;
    if (v2_tail) return gemm_run(&dt, d->dropout_row0 + r, stream, 2);
    dt.split_k = sk;
    return gemm_run(&dt, d->dropout_row0 + r, stream);
  }
  return gemm_run(d, d->dropout_row0, stream);
}
