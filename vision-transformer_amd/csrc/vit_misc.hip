// Memory-bound kernels of the ViT step: patch im2col, CLS rows, column sums, strided copies, dropout backward,
// GELU, softmax cross-entropy, and the multi-tensor AdamW / shadow-weight pack.  All vectorised where the shape
// allows (8-16 B per lane), grid-stride, fixed reduction order (bitwise reproducible).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <atomic>

#include "vit_common.h"

namespace vit {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return VIT_ERR_LAUNCH;
  }
  return VIT_OK;
}
}  // namespace vit

extern "C" int vit_abi_version(void) { return VIT_ABI_VERSION; }
extern "C" const char* vit_last_error(void) { return vit::g_err; }

// ---------------------------------------------------------------------------------------------------------------
// Launch options (vit_hip.h vit_set_option): names, shipped defaults, current values.
// ---------------------------------------------------------------------------------------------------------------
namespace {
struct OptDef {
  const char* name;
  int64_t def;
};
constexpr OptDef kOpts[vit::OPT_COUNT] = {
    {"gemm_impl", 0},        {"gemm_tail", 0},          {"gemm_tail_min_kt", 40}, {"splitk_min_kt", 0},
    {"gemm_group_m", 0},     {"gemm_epi_general", 0},   {"gemm_persist", 1},      {"attn_fwd_split", 0},
    {"attn_bwd_split", 0},   {"attn_bwd_grid", 0},      {"ln16", 1},              {"ln_al", 1},
    {"attn_fwd_ring", 1},    {"gemm_tail_v2", 0},    {"splitk_rounds", 1},    {"attn_fwd_grid", 0},
};
std::atomic<int64_t> g_opt[vit::OPT_COUNT] = {0, 0, 40, 0, 0, 0, 1, 0, 0, 0, 1, 1, 1, 0, 1, 0};

int opt_index(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < vit::OPT_COUNT; ++i)
    if (strcmp(name, kOpts[i].name) == 0) return i;
  return -1;
}
}  // namespace

int64_t vit::opt(vit::Opt o) { return g_opt[o].load(std::memory_order_relaxed); }

extern "C" int vit_set_option(const char* name, int64_t value) {
  const int i = opt_index(name);
  VIT_REQUIRE(i >= 0, "vit_set_option: unknown option '%s'", name ? name : "(null)");
  g_opt[i].store(value, std::memory_order_relaxed);
  return VIT_OK;
}

extern "C" int64_t vit_get_option(const char* name) {
  const int i = opt_index(name);
  return i >= 0 ? g_opt[i].load(std::memory_order_relaxed) : INT64_MIN;
}

namespace {

inline unsigned grid_for(int64_t work, int64_t per_block, int64_t cap = 8192) {
  int64_t b = (work + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (unsigned)b;
}

// ---------------------------------------------------------------------------------------------------------------
// im2col: one thread per (row m = b*N + n, 4 consecutive columns); column (c, kh, kw) with kw fastest.
// ---------------------------------------------------------------------------------------------------------------
template <class TI, class TO>
__global__ __launch_bounds__(256) void im2col_kernel(const TI* __restrict__ x, TO* __restrict__ cols, int64_t B,
                                                     int64_t C, int64_t H, int64_t W, int64_t P) {
  const int64_t nw = W / P, nh = H / P, N = nh * nw, KC = C * P * P;
  const int64_t q4 = KC / 4, total = B * N * q4;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = t / q4, col = (t % q4) * 4;
    const int64_t b = m / N, n = m % N, ph = n / nw, pw = n % nw;
    const int64_t c = col / (P * P), rem = col % (P * P), kh = rem / P, kw = rem % P;
    const TI* src = x + ((b * C + c) * H + ph * P + kh) * W + pw * P + kw;
    float v[4];
    v[0] = ld1<TI>(src); v[1] = ld1<TI>(src + 1); v[2] = ld1<TI>(src + 2); v[3] = ld1<TI>(src + 3);
    st4<TO>(cols + m * KC + col, v);
  }
}

// col2im for k = s = P: one thread per image element (b, c, h, w), coalesced on the image write.
template <class TI, class TO>
__global__ __launch_bounds__(256) void col2im_kernel(const TI* __restrict__ cols, TO* __restrict__ x, int64_t B,
                                                     int64_t C, int64_t H, int64_t W, int64_t P) {
  const int64_t nw = W / P, N = (H / P) * nw, KC = C * P * P, total = B * C * H * W;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w = t % W, h = (t / W) % H, c = (t / (W * H)) % C, b = t / (W * H * C);
    const int64_t n = (h / P) * nw + w / P, col = (c * P + h % P) * P + w % P;
    st1<TO>(x + t, ld1<TI>(cols + (b * N + n) * KC + col));
  }
}

template <class T>
__global__ __launch_bounds__(256) void embed_cls_kernel(const float* __restrict__ cls, const float* __restrict__ pos,
                                                        T* __restrict__ x0, int64_t B, int64_t T_, int64_t D) {
  const int64_t N = T_ - 1;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < B * D; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / D, d = t % D;
    st1<T>(x0 + (b * T_ + N) * D + d, cls[b * D + d] + pos[N * D + d]);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Column sums, two deterministic stages.  Stage 1: block (64 x 4 threads) owns 256 columns (4 per lane) and a chunk
// of rows; writes partial[chunk][cols].  Stage 2: one thread per column sums the chunks in order.
// ---------------------------------------------------------------------------------------------------------------
constexpr int CS_CHUNKS_MAX = 256;

template <class T>
__global__ __launch_bounds__(256) void colsum_stage1(const T* __restrict__ x, int64_t ldx, int64_t rows,
                                                     int64_t cols, int64_t rows_per_chunk, float* __restrict__ part,
                                                     int vec, float alpha = 1.f) {
  __shared__ float red[4][256];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * 256 + tx * 4;
  const int64_t chunk = blockIdx.y;
  const int64_t r0 = chunk * rows_per_chunk, r1 = min(rows, r0 + rows_per_chunk);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t r = r0 + ty; r < r1; r += 4) {
    const T* p = x + r * ldx + c0;
    if (vec && c0 + 3 < cols) {
      float v[4];
      ld4<T>(p, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += v[k];
    } else {
      for (int k = 0; k < 4; ++k)
        if (c0 + k < cols) acc[k] += ld1<T>(p + k);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) red[ty][tx * 4 + k] = acc[k];
  __syncthreads();
  if (ty == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cc = tx * 4 + k;
      const float s = red[0][cc] + red[1][cc] + red[2][cc] + red[3][cc];
      if (c0 + k < cols) part[chunk * cols + c0 + k] = s * alpha;
    }
  }
}

// Stage 2: 64 columns per block; 16 waves stride over the chunk partials (wave w sums chunks w, w+16, ...), then the
// 16 wave sums are added in wave order through LDS -> deterministic for a given (rows, cols).
// blockIdx.y selects one of up to 3 independent sets: part + set*nchunks*cols -> outs.p[set] (vit_colsum_finish).
constexpr int CS2_WAVES = 16;
struct OutSet {
  float* p[3];
};
// One 64-column block of one set: the chunk partials summed by 16 waves (8 independent chains per lane), then the wave
// sums in wave order through LDS.
VIT_DEV void colsum_block(const float* __restrict__ part, int64_t nchunks, int64_t cols, float* __restrict__ out,
                          float beta, int64_t cblock, float (*red)[64]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = cblock * 64 + lane;
  // 8 independent chains per lane (chunk k goes to chain (k / CS2_WAVES) % 8): 8 loads in flight per lane, order fixed
  constexpr int CH = 8;
  float sc[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) sc[i] = 0.f;
  if (c < cols) {
    int64_t k = w;
    for (; k + (CH - 1) * CS2_WAVES < nchunks; k += CH * CS2_WAVES) {
#pragma unroll
      for (int i = 0; i < CH; ++i) sc[i] += part[(k + i * CS2_WAVES) * cols + c];
    }
#pragma unroll
    for (int i = 0; i < CH; ++i)
      if (k + i * CS2_WAVES < nchunks) sc[i] += part[(k + i * CS2_WAVES) * cols + c];
  }
  red[w][lane] = ((sc[0] + sc[1]) + (sc[2] + sc[3])) + ((sc[4] + sc[5]) + (sc[6] + sc[7]));
  __syncthreads();
  if (w == 0 && c < cols) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < CS2_WAVES; ++i) s += red[i][lane];
    out[c] = beta != 0.f ? beta * out[c] + s : s;
  }
}

__global__ __launch_bounds__(64 * CS2_WAVES) void colsum_stage2(const float* __restrict__ part, int64_t nchunks,
                                                                int64_t cols, OutSet outs, float beta) {
  __shared__ float red[CS2_WAVES][64];
  float* out = blockIdx.y == 0 ? outs.p[0] : (blockIdx.y == 1 ? outs.p[1] : outs.p[2]);
  colsum_block(part + (int64_t)blockIdx.y * nchunks * cols, nchunks, cols, out, beta, blockIdx.x, red);
}

// vit_colsum_finish_batch: several finishes in one launch; block b belongs to the job whose [first, first + nsets *
// colblocks) range holds it.  Each (job, set, column block) is the same computation as colsum_stage2's.
constexpr int CS_BATCH_MAX = 8;
struct CsBatch {
  vit_colsum_job job[CS_BATCH_MAX];
  int64_t first[CS_BATCH_MAX + 1];
  int n;
};
__global__ __launch_bounds__(64 * CS2_WAVES) void colsum_stage2_batch(CsBatch tab) {
  __shared__ float red[CS2_WAVES][64];
  const int64_t b = blockIdx.x;
  int j = 0;
  while (j + 1 < tab.n && b >= tab.first[j + 1]) ++j;
  const vit_colsum_job& jb = tab.job[j];
  const int64_t cbs = (jb.cols + 63) / 64, local = b - tab.first[j], set = local / cbs;
  float* out = set == 0 ? jb.out[0] : (set == 1 ? jb.out[1] : jb.out[2]);
  colsum_block(jb.part + set * jb.nparts * jb.cols, jb.nparts, jb.cols, out, jb.beta, local % cbs, red);
}

int64_t colsum_chunks(int64_t rows, int64_t cols) {
  // aim for ~2048 blocks total, each with >= 32 rows
  const int64_t cblocks = (cols + 255) / 256;
  int64_t ch = 2048 / (cblocks > 0 ? cblocks : 1);
  if (ch < 1) ch = 1;
  if (ch > CS_CHUNKS_MAX) ch = CS_CHUNKS_MAX;
  const int64_t maxch = (rows + 31) / 32;
  if (ch > maxch) ch = maxch;
  if (ch < 1) ch = 1;
  return ch;
}

// ---------------------------------------------------------------------------------------------------------------
template <class TS, class TD>
__global__ __launch_bounds__(256) void copy2d_kernel(const TS* __restrict__ src, int64_t lds, TD* __restrict__ dst,
                                                     int64_t ldd, int64_t rows, int64_t cols, int64_t grp,
                                                     int64_t grp_stride, float beta) {
  const int64_t total = rows * cols;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / cols, j = t % cols;
    const int64_t si = grp ? (i / grp) * grp_stride + (i % grp) : i;
    float v = ld1<TS>(src + si * lds + j);
    TD* d = dst + i * ldd + j;
    if (beta != 0.f) v += beta * ld1<TD>(d);
    st1<TD>(d, v);
  }
}

// Same-dtype copy without beta as 16-B chunks (bit-exact; rows and leading dimensions 16-B aligned)
__global__ __launch_bounds__(256) void copy2d_raw16_kernel(const uint8_t* __restrict__ src, int64_t lds,
                                                           uint8_t* __restrict__ dst, int64_t ldd, int64_t rows,
                                                           int64_t cpr, int64_t grp, int64_t grp_stride) {
  const int64_t total = rows * cpr;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / cpr, j = (t - i * cpr) * 16;
    const int64_t si = grp ? (i / grp) * grp_stride + (i % grp) : i;
    *reinterpret_cast<uint4*>(dst + i * ldd + j) = *reinterpret_cast<const uint4*>(src + si * lds + j);
  }
}

template <class T>
__global__ __launch_bounds__(256) void dropout_bwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                          uint32_t thr, float scale, uint32_t seed) {  // y = keep*x*scale
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    const float v = ld1<T>(x + t);
    st1<T>(y + t, vit_hash_u32(seed, (uint32_t)t) >= thr ? v * scale : 0.f);
  }
}

// y[i][j] = x[i][j] * mask4 bit (i, j) * scale, x any dtype -> y any dtype (4 columns per thread; cols % 4 == 0)
template <class TI, class TO>
__global__ __launch_bounds__(256) void mask4_apply_kernel(const TI* __restrict__ x, int64_t ldx, TO* __restrict__ y,
                                                          int64_t ldy, const uint8_t* __restrict__ mask, int64_t rows,
                                                          int64_t cols, float scale) {
  const int64_t nq = cols / 4, total = rows * nq;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / nq, j = (t % nq) * 4;
    float v[4];
    ld4<TI>(x + i * ldx + j, v);
    const uint32_t b = mask[mask4_byte(i, j, cols)];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (b >> r) & 1u ? v[r] * scale : 0.f;
    st4<TO>(y + i * ldy + j, v);
  }
}

template <class T>
__global__ __launch_bounds__(256) void relu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                       T* __restrict__ dx, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    st1<T>(dx + t, ld1<T>(y + t) > 0.f ? ld1<T>(dy + t) : 0.f);
}

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    y[t] = gelu_erf(x[t]);
}
__global__ __launch_bounds__(256) void gelu_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                       float* __restrict__ dx, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    dx[t] = dy[t] * gelu_erf_grad(x[t]);
}

// one workgroup per row: max, sum-exp, loss term, gradient row
__global__ __launch_bounds__(256) void xent_rows_kernel(const float* __restrict__ logits,
                                                        const int64_t* __restrict__ labels, int64_t classes,
                                                        float inv_rows, float* __restrict__ dlogits,
                                                        float* __restrict__ row_loss) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  const float* x = logits + r * classes;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float mx = -INFINITY;
  for (int64_t c = tid; c < classes; c += 256) mx = fmaxf(mx, x[c]);
  mx = wave_max(mx);
  if (lane == 0) red[w] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int64_t c = tid; c < classes; c += 256) s += __expf(x[c] - mx);
  s = wave_sum(s);
  if (lane == 0) red[w] = s;
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  const float lse = mx + __logf(s);
  const int64_t y = labels[r];
  for (int64_t c = tid; c < classes; c += 256) {
    const float p = __expf(x[c] - lse);
    dlogits[r * classes + c] = (p - (c == y ? 1.f : 0.f)) * inv_rows;
  }
  if (tid == 0) row_loss[r] = lse - x[y];
}

__global__ __launch_bounds__(256) void xent_reduce_kernel(const float* __restrict__ row_loss, int64_t rows,
                                                          float inv_rows, float* __restrict__ loss) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t r = threadIdx.x; r < rows; r += 256) s += row_loss[r];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *loss = (red[0] + red[1] + red[2] + red[3]) * inv_rows;
}

// ---------------------------------------------------------------------------------------------------------------
// Multi-tensor AdamW: one workgroup per table chunk (the host sets its size: 8 Ki elements, _ops.CHUNK), one element
// per lane per step (16-B accesses measured no faster: the update runs at ~5.8 TB/s over 30 B per element).
// ---------------------------------------------------------------------------------------------------------------
template <class TS>
__global__ __launch_bounds__(256) void adamw_kernel(const vit_tensor_chunk* __restrict__ tab, float lr, float b1,
                                                    float b2, float eps, float wd, float step_size,
                                                    float inv_sqrt_bc2, float gscale) {
  const vit_tensor_chunk ch = tab[blockIdx.x];
  const float decay = 1.0f - lr * wd;
  for (int64_t t = threadIdx.x; t < ch.n; t += 256) {
    float g = ch.g[t] * gscale;
    float m = ch.m[t], v = ch.v[t], p = ch.p[t];
    p *= decay;
    m = b1 * m + (1.0f - b1) * g;
    v = b2 * v + (1.0f - b2) * g * g;
    const float denom = sqrtf(v) * inv_sqrt_bc2 + eps;
    p -= step_size * (m / denom);
    ch.m[t] = m;
    ch.v[t] = v;
    ch.p[t] = p;
    if (ch.shadow) st1<TS>((TS*)ch.shadow + t, p);
  }
}

template <class TS>
__global__ __launch_bounds__(256) void pack_kernel(const vit_tensor_chunk* __restrict__ tab) {
  const vit_tensor_chunk ch = tab[blockIdx.x];
  if (!ch.shadow) return;
  for (int64_t t = threadIdx.x; t < ch.n; t += 256) st1<TS>((TS*)ch.shadow + t, ch.p[t]);
}

}  // namespace

// ===============================================================================================================
extern "C" int vit_im2col(const void* x, int32_t x_dtype, void* cols, int32_t dtype, int64_t B, int64_t C, int64_t H,
                          int64_t W, int64_t P, void* stream) {
  VIT_REQUIRE(x && cols, "vit_im2col: null pointer");
  VIT_REQUIRE(B > 0 && C > 0 && P > 0 && H % P == 0 && W % P == 0, "vit_im2col: image %lldx%lld not divisible by P=%lld",
              (long long)H, (long long)W, (long long)P);
  VIT_REQUIRE(P % 4 == 0, "vit_im2col: patch size must be a multiple of 4");
  const int64_t work = B * (H / P) * (W / P) * C * P * P / 4;
  const unsigned grid = grid_for(work, 256, 16384);
  hipStream_t s = VIT_STREAM(stream);
  if (x_dtype == VIT_F32 && dtype == VIT_BF16)
    im2col_kernel<float, bf16_t><<<grid, 256, 0, s>>>((const float*)x, (bf16_t*)cols, B, C, H, W, P);
  else if (x_dtype == VIT_F32 && dtype == VIT_F32)
    im2col_kernel<float, float><<<grid, 256, 0, s>>>((const float*)x, (float*)cols, B, C, H, W, P);
  else if (x_dtype == VIT_BF16 && dtype == VIT_BF16)
    im2col_kernel<bf16_t, bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)x, (bf16_t*)cols, B, C, H, W, P);
  else {
    vit::set_error("vit_im2col: unsupported dtype pair %d->%d", x_dtype, dtype);
    return VIT_ERR_INVALID;
  }
  return vit::check_launch("vit_im2col");
}

extern "C" int vit_col2im(const void* cols, int32_t dtype, void* x, int32_t x_dtype, int64_t B, int64_t C,
                          int64_t H, int64_t W, int64_t P, void* stream) {
  VIT_REQUIRE(x && cols, "vit_col2im: null pointer");
  VIT_REQUIRE(B > 0 && C > 0 && P > 0 && H % P == 0 && W % P == 0, "vit_col2im: image %lldx%lld not divisible by P=%lld",
              (long long)H, (long long)W, (long long)P);
  const unsigned grid = grid_for(B * C * H * W, 256, 16384);
  hipStream_t s = VIT_STREAM(stream);
  if (dtype == VIT_BF16 && x_dtype == VIT_F32)
    col2im_kernel<bf16_t, float><<<grid, 256, 0, s>>>((const bf16_t*)cols, (float*)x, B, C, H, W, P);
  else if (dtype == VIT_F32 && x_dtype == VIT_F32)
    col2im_kernel<float, float><<<grid, 256, 0, s>>>((const float*)cols, (float*)x, B, C, H, W, P);
  else if (dtype == VIT_BF16 && x_dtype == VIT_BF16)
    col2im_kernel<bf16_t, bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)cols, (bf16_t*)x, B, C, H, W, P);
  else {
    vit::set_error("vit_col2im: unsupported dtype pair %d->%d", dtype, x_dtype);
    return VIT_ERR_INVALID;
  }
  return vit::check_launch("vit_col2im");
}

extern "C" int vit_embed_cls(const float* cls, const float* pos, void* x0, int32_t dtype, int64_t B, int64_t T,
                             int64_t D, void* stream) {
  VIT_REQUIRE(cls && pos && x0 && B > 0 && T > 0 && D > 0, "vit_embed_cls: bad arguments");
  const unsigned grid = grid_for(B * D, 256);
  hipStream_t s = VIT_STREAM(stream);
  if (dtype == VIT_BF16) embed_cls_kernel<bf16_t><<<grid, 256, 0, s>>>(cls, pos, (bf16_t*)x0, B, T, D);
  else embed_cls_kernel<float><<<grid, 256, 0, s>>>(cls, pos, (float*)x0, B, T, D);
  return vit::check_launch("vit_embed_cls");
}

namespace vit {
void colsum_parts_launch(const void* x, int64_t ldx, int dtype, int64_t rows, int64_t cols, int64_t rows_per_chunk,
                         float* part, hipStream_t s) {
  const int64_t ch = (rows + rows_per_chunk - 1) / rows_per_chunk;
  const int vec = (cols % 4 == 0) && (ldx % 4 == 0) && (((uintptr_t)x) % 16 == 0);
  dim3 g1((unsigned)((cols + 255) / 256), (unsigned)ch);
  if (dtype == VIT_BF16)
    colsum_stage1<bf16_t><<<g1, 256, 0, s>>>((const bf16_t*)x, ldx, rows, cols, rows_per_chunk, part, vec);
  else
    colsum_stage1<float><<<g1, 256, 0, s>>>((const float*)x, ldx, rows, cols, rows_per_chunk, part, vec);
}
}  // namespace vit

extern "C" int64_t vit_colsum_workspace_bytes(int64_t rows, int64_t cols) {
  return colsum_chunks(rows, cols) * cols * (int64_t)sizeof(float);
}

extern "C" int vit_colsum(const void* x, int64_t ldx, int32_t dtype, int64_t rows, int64_t cols, float* out,
                          float alpha, float beta, void* workspace, void* stream) {
  VIT_REQUIRE(x && out && workspace && rows > 0 && cols > 0, "vit_colsum: bad arguments");
  const int64_t ch = colsum_chunks(rows, cols);
  const int64_t rpc = (rows + ch - 1) / ch;
  const int vec = (cols % 4 == 0) && (ldx % 4 == 0) && (((uintptr_t)x) % 16 == 0);
  dim3 g1((unsigned)((cols + 255) / 256), (unsigned)ch);
  hipStream_t s = VIT_STREAM(stream);
  if (dtype == VIT_BF16)
    colsum_stage1<bf16_t><<<g1, 256, 0, s>>>((const bf16_t*)x, ldx, rows, cols, rpc, (float*)workspace, vec, alpha);
  else
    colsum_stage1<float><<<g1, 256, 0, s>>>((const float*)x, ldx, rows, cols, rpc, (float*)workspace, vec, alpha);
  OutSet outs{{out, nullptr, nullptr}};
  colsum_stage2<<<(unsigned)((cols + 63) / 64), 64 * CS2_WAVES, 0, s>>>((const float*)workspace, ch, cols, outs, beta);
  return vit::check_launch("vit_colsum");
}

extern "C" int vit_colsum_finish(const float* part, int64_t nparts, int64_t cols, int32_t nsets, float* out0,
                                 float* out1, float* out2, float beta, void* stream) {
  VIT_REQUIRE(part && nparts > 0 && cols > 0 && nsets >= 1 && nsets <= 3, "vit_colsum_finish: bad arguments");
  OutSet outs{{out0, out1, out2}};
  for (int i = 0; i < nsets; ++i) VIT_REQUIRE(outs.p[i] != nullptr, "vit_colsum_finish: output %d is NULL", i);
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)nsets);
  colsum_stage2<<<grid, 64 * CS2_WAVES, 0, VIT_STREAM(stream)>>>(part, nparts, cols, outs, beta);
  return vit::check_launch("vit_colsum_finish");
}

extern "C" int vit_colsum_finish_batch(const vit_colsum_job* jobs, int32_t njobs, void* stream) {
  VIT_REQUIRE(jobs && njobs >= 1 && njobs <= CS_BATCH_MAX, "vit_colsum_finish_batch: 1..%d jobs", CS_BATCH_MAX);
  CsBatch tab{};
  tab.n = njobs;
  tab.first[0] = 0;
  for (int j = 0; j < njobs; ++j) {
    const vit_colsum_job& jb = jobs[j];
    VIT_REQUIRE(jb.part && jb.nparts > 0 && jb.cols > 0 && jb.nsets >= 1 && jb.nsets <= 3,
                "vit_colsum_finish_batch: bad job %d", j);
    for (int i = 0; i < jb.nsets; ++i)
      VIT_REQUIRE(jb.out[i] != nullptr, "vit_colsum_finish_batch: job %d output %d is NULL", j, i);
    tab.job[j] = jb;
    tab.first[j + 1] = tab.first[j] + jb.nsets * ((jb.cols + 63) / 64);
  }
  colsum_stage2_batch<<<(unsigned)tab.first[njobs], 64 * CS2_WAVES, 0, VIT_STREAM(stream)>>>(tab);
  return vit::check_launch("vit_colsum_finish_batch");
}

extern "C" int vit_copy2d(const void* src, int64_t lds, int32_t src_dtype, void* dst, int64_t ldd, int32_t dst_dtype,
                          int64_t rows, int64_t cols, int64_t src_group_rows, int64_t src_group_stride, float beta,
                          void* stream) {
  VIT_REQUIRE(src && dst && rows > 0 && cols > 0, "vit_copy2d: bad arguments");
  hipStream_t s = VIT_STREAM(stream);
  const int64_t es = src_dtype == VIT_F32 ? 4 : 2;
  if (src_dtype == dst_dtype && beta == 0.f && (cols * es) % 16 == 0 && (lds * es) % 16 == 0 && (ldd * es) % 16 == 0 &&
      ((uintptr_t)src | (uintptr_t)dst) % 16 == 0) {
    const int64_t cpr = cols * es / 16;
    copy2d_raw16_kernel<<<grid_for(rows * cpr, 256, 16384), 256, 0, s>>>(
        (const uint8_t*)src, lds * es, (uint8_t*)dst, ldd * es, rows, cpr, src_group_rows, src_group_stride);
    return vit::check_launch("vit_copy2d");
  }
  const unsigned grid = grid_for(rows * cols, 256, 16384);
#define CP(TS, TD)                                                                                            \
  copy2d_kernel<TS, TD><<<grid, 256, 0, s>>>((const TS*)src, lds, (TD*)dst, ldd, rows, cols, src_group_rows, \
                                             src_group_stride, beta)
  if (src_dtype == VIT_F32 && dst_dtype == VIT_F32) CP(float, float);
  else if (src_dtype == VIT_F32) CP(float, bf16_t);
  else if (dst_dtype == VIT_F32) CP(bf16_t, float);
  else CP(bf16_t, bf16_t);
#undef CP
  return vit::check_launch("vit_copy2d");
}

extern "C" int vit_dropout_bwd(const void* x, void* y, int32_t dtype, int64_t n, float p, uint32_t seed, float scale,
                               void* stream) {
  VIT_REQUIRE(x && y && n > 0 && p >= 0.f && p < 1.f, "vit_dropout_bwd: bad arguments");
  double t = (double)p * 4294967296.0;
  const uint32_t thr = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  const unsigned grid = grid_for(n, 256, 16384);
  hipStream_t s = VIT_STREAM(stream);
  if (dtype == VIT_BF16) dropout_bwd_kernel<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)x, (bf16_t*)y, n, thr, scale, seed);
  else dropout_bwd_kernel<float><<<grid, 256, 0, s>>>((const float*)x, (float*)y, n, thr, scale, seed);
  return vit::check_launch("vit_dropout_bwd");
}

extern "C" int vit_mask4_apply(const void* x, int64_t ldx, int32_t x_dtype, void* y, int64_t ldy, int32_t y_dtype,
                               const void* mask, int64_t rows, int64_t cols, float scale, void* stream) {
  VIT_REQUIRE(x && y && mask && rows > 0 && cols > 0, "vit_mask4_apply: bad arguments");
  VIT_REQUIRE(cols % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0, "vit_mask4_apply: cols/ld must be multiples of 4");
  const unsigned grid = grid_for(rows * (cols / 4), 256, 16384);
  hipStream_t s = VIT_STREAM(stream);
  const uint8_t* m = (const uint8_t*)mask;
#define MA(TI, TO) mask4_apply_kernel<TI, TO><<<grid, 256, 0, s>>>((const TI*)x, ldx, (TO*)y, ldy, m, rows, cols, scale)
  if (x_dtype == VIT_BF16 && y_dtype == VIT_BF16) MA(bf16_t, bf16_t);
  else if (x_dtype == VIT_BF16) MA(bf16_t, float);
  else if (y_dtype == VIT_BF16) MA(float, bf16_t);
  else MA(float, float);
#undef MA
  return vit::check_launch("vit_mask4_apply");
}

extern "C" int vit_relu_bwd(const void* dy, const void* y, void* dx, int32_t dtype, int64_t n, void* stream) {
  VIT_REQUIRE(dy && y && dx && n > 0, "vit_relu_bwd: bad arguments");
  const unsigned grid = grid_for(n, 256, 16384);
  hipStream_t s = VIT_STREAM(stream);
  if (dtype == VIT_BF16) relu_bwd_kernel<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)dy, (const bf16_t*)y, (bf16_t*)dx, n);
  else relu_bwd_kernel<float><<<grid, 256, 0, s>>>((const float*)dy, (const float*)y, (float*)dx, n);
  return vit::check_launch("vit_relu_bwd");
}

extern "C" int vit_gelu_fwd(const float* x, float* y, int64_t n, void* stream) {
  VIT_REQUIRE(x && y && n > 0, "vit_gelu_fwd: bad arguments");
  gelu_fwd_kernel<<<grid_for(n, 256), 256, 0, VIT_STREAM(stream)>>>(x, y, n);
  return vit::check_launch("vit_gelu_fwd");
}

extern "C" int vit_gelu_bwd(const float* x, const float* dy, float* dx, int64_t n, void* stream) {
  VIT_REQUIRE(x && dy && dx && n > 0, "vit_gelu_bwd: bad arguments");
  gelu_bwd_kernel<<<grid_for(n, 256), 256, 0, VIT_STREAM(stream)>>>(x, dy, dx, n);
  return vit::check_launch("vit_gelu_bwd");
}

extern "C" int vit_softmax_xent(const float* logits, const int64_t* labels, int64_t rows, int64_t classes, float* loss,
                                float* dlogits, float* workspace, void* stream) {
  VIT_REQUIRE(logits && labels && loss && dlogits && workspace && rows > 0 && classes > 0,
              "vit_softmax_xent: bad arguments");
  hipStream_t s = VIT_STREAM(stream);
  const float inv = 1.0f / (float)rows;
  xent_rows_kernel<<<(unsigned)rows, 256, 0, s>>>(logits, labels, classes, inv, dlogits, workspace);
  xent_reduce_kernel<<<1, 256, 0, s>>>(workspace, rows, inv, loss);
  return vit::check_launch("vit_softmax_xent");
}

extern "C" int vit_adamw(const vit_tensor_chunk* table_dev, int64_t nchunks, float lr, float beta1, float beta2,
                         float eps, float weight_decay, float bias_corr1, float bias_corr2, float grad_scale,
                         int32_t shadow_dtype, void* stream) {
  VIT_REQUIRE(table_dev && nchunks > 0 && bias_corr1 > 0.f && bias_corr2 > 0.f, "vit_adamw: bad arguments");
  const float step_size = lr / bias_corr1;
  const float inv_sqrt_bc2 = 1.0f / sqrtf(bias_corr2);
  hipStream_t s = VIT_STREAM(stream);
  if (shadow_dtype == VIT_BF16)
    adamw_kernel<bf16_t><<<(unsigned)nchunks, 256, 0, s>>>(table_dev, lr, beta1, beta2, eps, weight_decay, step_size,
                                                           inv_sqrt_bc2, grad_scale);
  else
    adamw_kernel<float><<<(unsigned)nchunks, 256, 0, s>>>(table_dev, lr, beta1, beta2, eps, weight_decay, step_size,
                                                          inv_sqrt_bc2, grad_scale);
  return vit::check_launch("vit_adamw");
}

extern "C" int vit_pack(const vit_tensor_chunk* table_dev, int64_t nchunks, int32_t shadow_dtype, void* stream) {
  VIT_REQUIRE(table_dev && nchunks > 0, "vit_pack: bad arguments");
  hipStream_t s = VIT_STREAM(stream);
  if (shadow_dtype == VIT_BF16) pack_kernel<bf16_t><<<(unsigned)nchunks, 256, 0, s>>>(table_dev);
  else pack_kernel<float><<<(unsigned)nchunks, 256, 0, s>>>(table_dev);
  return vit::check_launch("vit_pack");
}
