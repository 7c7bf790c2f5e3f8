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
};

struct GemmArgs {
  const void* a;
  const void* b;
  int64_t lda, ldb, M, N, K;
  int64_t tiles_n;
  int64_t kt_per_split;  // k-tiles per split
  float* ws;             // split-K slabs [split][M][N]
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
      float a[4];
      if (e.aux_dtype == VIT_BF16) ld4<bf16_t>((const bf16_t*)e.aux + i * e.ldaux + j, a);
      else ld4<float>((const float*)e.aux + i * e.ldaux + j, a);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = a[r] > 0.f ? v[r] : 0.f;
    }
    if (e.use_drop) {
      const uint32_t base = (uint32_t)(i * e.n + j);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] = vit_hash_u32(e.seed, base + r) >= e.drop_thr ? v[r] * e.drop_scale : 0.f;
    }
    if (e.res) {
      float a[4];
      if (e.res_dtype == VIT_BF16) ld4<bf16_t>((const bf16_t*)e.res + rrow * e.ldres + j, a);
      else ld4<float>((const float*)e.res + rrow * e.ldres + j, a);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += a[r];
    }
    st4<TO>(cp, v);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t jj = j + r;
      if (jj >= e.n) break;
      float x = v[r];
      if (e.beta != 0.f) x += e.beta * ld1<TO>(cp + r);
      if (e.bias) x += e.bias[jj];
      if (e.act == VIT_ACT_RELU) x = fmaxf(x, 0.f);
      else if (e.act == VIT_ACT_GELU) x = gelu_erf(x);
      if (e.aux) x = ld_any(e.aux, e.aux_dtype, i * e.ldaux + jj) > 0.f ? x : 0.f;
      if (e.use_drop) x = vit_hash_u32(e.seed, (uint32_t)(i * e.n + jj)) >= e.drop_thr ? x * e.drop_scale : 0.f;
      if (e.res) x += ld_any(e.res, e.res_dtype, rrow * e.ldres + jj);
      st1<TO>(cp + r, x);
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
// f32 MFMA kernel (exact fp32; generic strides; any M/N/K)
// ------------------------------------------------------------------------------------------------------------
constexpr int FBM = 64, FBK = 16, FPAD = 4;

template <bool KC>
VIT_DEV void f32_load_stage(const float* __restrict__ src, int64_t ld, int64_t rows, int64_t K, int64_t r0,
                            int64_t k0, int tid, float (*S)[FBM + FPAD]) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int q = tid + 256 * it;
    int ii, rr;
    if (KC) { ii = q >> 4; rr = q & 15; }
    else { rr = q >> 6; ii = q & 63; }
    const int64_t gi = r0 + ii, gk = k0 + rr;
    float v = 0.f;
    if (gi < rows && gk < K) v = KC ? src[gi * ld + gk] : src[gk * ld + gi];
    S[rr][ii] = v;
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
  for (int64_t kt = kt0; kt < kt1; ++kt) {
    f32_load_stage<AKC>(A, g.lda, g.M, g.K, i0, kt * FBK, tid, Xs);
    f32_load_stage<BKC>(B, g.ldb, g.N, g.K, j0, kt * FBK, tid, Ws);
    __syncthreads();
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
    for (int z = 0; z < splits; ++z) {
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

}  // namespace

extern "C" int64_t vit_gemm_workspace_bytes(const vit_gemm_desc* d) {
  if (!d || d->split_k <= 1) return 0;
  return (int64_t)d->split_k * d->m * d->n * (int64_t)sizeof(float);
}

extern "C" int vit_gemm(const vit_gemm_desc* d, void* stream) {
  VIT_REQUIRE(d != nullptr, "vit_gemm: null descriptor");
  VIT_REQUIRE(d->a && d->b && d->c, "vit_gemm: null operand pointer");
  VIT_REQUIRE(d->m > 0 && d->n > 0 && d->k > 0, "vit_gemm: bad shape m=%lld n=%lld k=%lld", (long long)d->m,
              (long long)d->n, (long long)d->k);
  VIT_REQUIRE(d->in_dtype == VIT_F32 || d->in_dtype == VIT_BF16, "vit_gemm: bad in_dtype %d", d->in_dtype);
  VIT_REQUIRE(d->out_dtype == VIT_F32 || d->out_dtype == VIT_BF16, "vit_gemm: bad out_dtype %d", d->out_dtype);
  VIT_REQUIRE(d->beta == 0.f || d->out_dtype == VIT_F32, "vit_gemm: beta requires f32 output");
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
  e.vec = (d->n % 4 == 0) && (d->ldc % 4 == 0) && aligned(d->c, 16) && aligned(d->bias, 16) &&
          (!d->aux || (d->ldaux % 4 == 0 && aligned(d->aux, 16))) &&
          (!d->res || (d->ldres % 4 == 0 && aligned(d->res, 16)));

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
#define LAUNCH_BF(AK, BKK)                                                                              \
  do {                                                                                                  \
    if (out_bf && split == 1) gemm_bf16_kernel<AK, BKK, bf16_t><<<grid, block, 0, s>>>(g, e);           \
    else gemm_bf16_kernel<AK, BKK, float><<<grid, block, 0, s>>>(g, e);                                 \
  } while (0)
    if (akc && bkc) LAUNCH_BF(true, true);
    else if (akc && !bkc) LAUNCH_BF(true, false);
    else LAUNCH_BF(false, false);
#undef LAUNCH_BF
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
  return vit::check_launch("vit_gemm");
}
