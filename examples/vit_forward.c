/*
 * vit_forward.c — batch-1 ViT forward in plain C over the C-ABI of libvit_hip.so (include/vit_hip.h).
 *
 * The counterpart of the reference's C prototype (csrc/vit.c: vit_alloc / vit_init / vit_forward, :443-484 and main
 * :886-939), which runs a forward-only, batch-1 ViT on the host.  Here the host side is equally plain C, but every
 * op is a gfx950 kernel behind the C-ABI, and the arithmetic is the Python reference's (src/VisionTransformer/{config,transformer,vit}.py:
 * CLS appended last, logits x sqrt(hd), ReLU MLP, token-0 GELU(erf) -> LayerNorm(4D) head), so the result can be
 * checked against the oracle: this program is the C-ABI host-side smoke test of SURVEY.md §8(f) row 4.
 *
 *   vit_forward WEIGHTS.bin LOGITS.bin [f32|bf16]
 *
 * WEIGHTS.bin: int32 header {magic 0x57544956 ("VITW"), version 1, C, img, P, D, H, L, nc}, then float32 tensors in
 * the reference state_dict order (vit.py:47-75 / transformer.py:9-90, batch 1):
 *   emdeddings.cls_tkn_embd [1][1][D], emdeddings.pos_embd [1][T][D], emdeddings.sequence.0.weight [D][C][P][P],
 *   emdeddings.sequence.0.bias [D];
 *   per block l: heads.h.{key,query,value}.weight [hd][D] for h = 0..H-1, proj.weight [D][D], proj.bias [D],
 *     ffwd.mlp.0.weight [4D][D], .bias [4D], ffwd.mlp.2.weight [D][4D], .bias [D], ln1.weight/bias [D],
 *     ln2.weight/bias [D];
 *   mlp.0.weight [4D][D], mlp.0.bias [4D], mlp.2.weight/bias [4D], mlp.3.weight [nc][4D], mlp.3.bias [nc];
 * then the image [C][img][img] float32.  LOGITS.bin receives nc float32 logits (eval mode: dropout off).
 * f32 runs every GEMM on the exact fp32 MFMA kernel; bf16 casts weights and activations to bf16 (fp32 accumulate,
 * fp32 LayerNorm statistics and head), as the training engine does.
 */
#define _POSIX_C_SOURCE 199309L
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "vit_hip.h"

#define VIT_CHECK(call)                                                                  \
  do {                                                                                   \
    int rc_ = (call);                                                                    \
    if (rc_ != 0) {                                                                      \
      fprintf(stderr, "%s:%d: %s failed (%d): %s\n", __FILE__, __LINE__, #call, rc_,     \
              vit_last_error());                                                         \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)
#define HIP_CHECK(call)                                                                  \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d: %s: %s\n", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

typedef struct {
  int C, img, P, D, H, L, nc, N, T, hd, CPP;
} Dims;

typedef struct {          /* device tensors of one block: weights in the compute dtype, vectors f32 */
  void *qkv_w, *proj_w, *fc1_w, *fc2_w;
  float *proj_b, *fc1_b, *fc2_b, *ln1_w, *ln1_b, *ln2_w, *ln2_b;
} Block;

static hipStream_t g_stream;
static void* g_ws;
static const int64_t WS_BYTES = 64ll << 20;

static void* dev_alloc(size_t bytes) {
  void* p = NULL;
  HIP_CHECK(hipMalloc(&p, bytes ? bytes : 4));
  return p;
}

static float* upload(const float* h, size_t n) {
  float* d = (float*)dev_alloc(n * sizeof(float));
  HIP_CHECK(hipMemcpy(d, h, n * sizeof(float), hipMemcpyHostToDevice));
  return d;
}

/* a [rows][cols] f32 host matrix -> device, in dtype (bf16: cast on the device by vit_copy2d) */
static void* upload_as(const float* h, int64_t rows, int64_t cols, int dtype) {
  float* f = upload(h, (size_t)(rows * cols));
  if (dtype == VIT_F32) return f;
  void* b = dev_alloc((size_t)(rows * cols) * 2);
  VIT_CHECK(vit_copy2d(f, cols, VIT_F32, b, cols, VIT_BF16, rows, cols, 0, 0, 0.f, g_stream));
  HIP_CHECK(hipStreamSynchronize(g_stream));
  HIP_CHECK(hipFree(f));
  return b;
}

/* C[m][n] = epi(A[m][k] . B[n][k]^T) — nn.Linear (transformer.py:12-18,38,56,58; vit.py:70,73) */
static void linear(const void* a, const void* b, void* c, int64_t m, int64_t n, int64_t k, int in_dt, int out_dt,
                   const float* bias, int act, const void* res, int res_dt, int64_t ldres, int64_t res_rowmod,
                   int64_t og_rows, int64_t og_stride, int64_t ldc) {
  vit_gemm_desc d;
  memset(&d, 0, sizeof(d));
  d.a = a;
  d.b = b;
  d.c = c;
  d.lda = k;
  d.ldb = k;
  d.ldc = ldc;
  d.m = m;
  d.n = n;
  d.k = k;
  d.a_kcontig = d.b_kcontig = 1;
  d.in_dtype = in_dt;
  d.out_dtype = out_dt;
  d.alpha = 1.f;
  d.bias = bias;
  d.act = act;
  d.res = res;
  d.res_dtype = res_dt;
  d.ldres = ldres;
  d.res_rowmod = res_rowmod;
  d.split_k = 1;
  d.out_group_rows = og_rows;
  d.out_group_stride = og_stride;
  d.workspace = g_ws;
  d.workspace_bytes = WS_BYTES;
  if (vit_gemm_workspace_bytes(&d) > WS_BYTES) d.workspace = NULL, d.workspace_bytes = 0;
  VIT_CHECK(vit_gemm(&d, g_stream));
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s WEIGHTS.bin LOGITS.bin [f32|bf16]\n", argv[0]);
    return 2;
  }
  const int dt = (argc > 3 && strcmp(argv[3], "bf16") == 0) ? VIT_BF16 : VIT_F32;
  const size_t es = dt == VIT_BF16 ? 2 : 4;
  if (vit_abi_version() != VIT_ABI_VERSION) {
    fprintf(stderr, "libvit_hip ABI %d, header %d\n", vit_abi_version(), VIT_ABI_VERSION);
    return 1;
  }

  /* ---- weights + image (host) */
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", argv[1]);
    return 1;
  }
  int32_t hdr[9];
  if (fread(hdr, sizeof(int32_t), 9, f) != 9 || hdr[0] != 0x57544956 || hdr[1] != 1) {
    fprintf(stderr, "%s: not a VITW v1 file\n", argv[1]);
    return 1;
  }
  Dims z = {hdr[2], hdr[3], hdr[4], hdr[5], hdr[6], hdr[7], hdr[8], 0, 0, 0, 0};
  z.N = (z.img / z.P) * (z.img / z.P);
  z.T = z.N + 1;
  z.hd = z.D / z.H;
  z.CPP = z.C * z.P * z.P;
  const int64_t D = z.D, T = z.T, N = z.N, F = 4 * D;
  const size_t per_block = (size_t)(3 * D * D + D * D + D + F * D + F + D * F + D + 4 * D);
  const size_t total = (size_t)(D + T * D + D * z.CPP + D) + z.L * per_block + (size_t)(F * D + F + 2 * F + z.nc * F +
                                                                                        z.nc) +
                       (size_t)z.C * z.img * z.img;
  float* host = (float*)malloc(total * sizeof(float));
  if (!host || fread(host, sizeof(float), total, f) != total) {
    fprintf(stderr, "%s: short file (need %zu floats)\n", argv[1], total);
    return 1;
  }
  fclose(f);
  const float* w = host;
#define TAKE(n) (w += (n), w - (n))

  HIP_CHECK(hipStreamCreate(&g_stream));
  g_ws = dev_alloc((size_t)WS_BYTES);
  float* cls = upload(TAKE(D), (size_t)D);
  float* pos = upload(TAKE(T * D), (size_t)(T * D));
  void* conv_w = upload_as(TAKE(D * z.CPP), D, z.CPP, dt);
  float* conv_b = upload(TAKE(D), (size_t)D);
  Block* blk = (Block*)calloc((size_t)z.L, sizeof(Block));
  float* qkv_host = (float*)malloc((size_t)(3 * D * D) * sizeof(float));
  for (int l = 0; l < z.L; ++l) {
    /* fused projection [3D][D]: query rows of every head, then keys, then values (transformer.py:12-18, :44-45) */
    for (int h = 0; h < z.H; ++h) {
      const float* kq[3];
      kq[1] = TAKE(z.hd * D); /* key */
      kq[0] = TAKE(z.hd * D); /* query */
      kq[2] = TAKE(z.hd * D); /* value */
      for (int s = 0; s < 3; ++s)
        memcpy(qkv_host + (s * D + (int64_t)h * z.hd) * D, kq[s], (size_t)(z.hd * D) * sizeof(float));
    }
    blk[l].qkv_w = upload_as(qkv_host, 3 * D, D, dt);
    blk[l].proj_w = upload_as(TAKE(D * D), D, D, dt);
    blk[l].proj_b = upload(TAKE(D), (size_t)D);
    blk[l].fc1_w = upload_as(TAKE(F * D), F, D, dt);
    blk[l].fc1_b = upload(TAKE(F), (size_t)F);
    blk[l].fc2_w = upload_as(TAKE(D * F), D, F, dt);
    blk[l].fc2_b = upload(TAKE(D), (size_t)D);
    blk[l].ln1_w = upload(TAKE(D), (size_t)D);
    blk[l].ln1_b = upload(TAKE(D), (size_t)D);
    blk[l].ln2_w = upload(TAKE(D), (size_t)D);
    blk[l].ln2_b = upload(TAKE(D), (size_t)D);
  }
  float* h0_w = upload(TAKE(F * D), (size_t)(F * D));
  float* h0_b = upload(TAKE(F), (size_t)F);
  float* hln_w = upload(TAKE(F), (size_t)F);
  float* hln_b = upload(TAKE(F), (size_t)F);
  float* h3_w = upload(TAKE(z.nc * F), (size_t)(z.nc * F));
  float* h3_b = upload(TAKE(z.nc), (size_t)z.nc);
  float* img = upload(TAKE(z.C * z.img * z.img), (size_t)z.C * z.img * z.img);
#undef TAKE

  /* ---- activations (batch 1: M = T token rows) */
  void* cols = dev_alloc((size_t)(N * z.CPP) * es);
  void* xa = dev_alloc((size_t)(T * D) * es);
  void* xb = dev_alloc((size_t)(T * D) * es);
  void* xm = dev_alloc((size_t)(T * D) * es);
  void* a1 = dev_alloc((size_t)(T * D) * es);
  void* qkv = dev_alloc((size_t)(T * 3 * D) * es);
  void* o = dev_alloc((size_t)(T * D) * es);
  void* hbuf = dev_alloc((size_t)(T * F) * es);
  float* mean = (float*)dev_alloc((size_t)T * sizeof(float));
  float* rstd = (float*)dev_alloc((size_t)T * sizeof(float));
  float* lse = (float*)dev_alloc((size_t)(z.H * T) * sizeof(float));
  float* zt = (float*)dev_alloc((size_t)D * sizeof(float));
  float* u = (float*)dev_alloc((size_t)F * sizeof(float));
  float* gz = (float*)dev_alloc((size_t)F * sizeof(float));
  float* zn = (float*)dev_alloc((size_t)F * sizeof(float));
  float* logits = (float*)dev_alloc((size_t)z.nc * sizeof(float));
  HIP_CHECK(hipDeviceSynchronize());

  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  /* patch embedding (vit.py:21-42): conv as im2col + GEMM, + bias + pos, rows -> tokens 0..N-1; CLS appended last */
  VIT_CHECK(vit_im2col(img, VIT_F32, cols, dt, 1, z.C, z.img, z.img, z.P, g_stream));
  linear(cols, conv_w, xa, N, D, z.CPP, dt, dt, conv_b, VIT_ACT_NONE, pos, VIT_F32, D, N, N, T, D);
  VIT_CHECK(vit_embed_cls(cls, pos, xa, dt, 1, T, D, g_stream));
  const float scale = sqrtf((float)z.hd); /* multiplied, transformer.py:24 */
  void* x = xa;
  void* y = xb;
  for (int l = 0; l < z.L; ++l) { /* Block (transformer.py:66-79), pre-LN, eval mode */
    VIT_CHECK(vit_layernorm_fwd(x, D, blk[l].ln1_w, blk[l].ln1_b, a1, D, mean, rstd, T, D, 1e-5f, dt, g_stream));
    linear(a1, blk[l].qkv_w, qkv, T, 3 * D, D, dt, dt, NULL, VIT_ACT_NONE, NULL, 0, 0, 0, 0, 0, 3 * D);
    VIT_CHECK(vit_attn_fwd(qkv, o, NULL, lse, NULL, 1, T, z.H, z.hd, scale, dt, 0, g_stream));
    linear(o, blk[l].proj_w, xm, T, D, D, dt, dt, blk[l].proj_b, VIT_ACT_NONE, x, dt, D, 0, 0, 0, D);
    VIT_CHECK(vit_layernorm_fwd(xm, D, blk[l].ln2_w, blk[l].ln2_b, a1, D, mean, rstd, T, D, 1e-5f, dt, g_stream));
    linear(a1, blk[l].fc1_w, hbuf, T, F, D, dt, dt, blk[l].fc1_b, VIT_ACT_RELU, NULL, 0, 0, 0, 0, 0, F);
    linear(hbuf, blk[l].fc2_w, y, T, D, F, dt, dt, blk[l].fc2_b, VIT_ACT_NONE, xm, dt, D, 0, 0, 0, D);
    void* t = x;
    x = y;
    y = t;
  }
  /* classifier on token 0 (vit.py:70-80): Linear -> GELU(erf) -> LayerNorm(4D) -> Linear, fp32 */
  VIT_CHECK(vit_copy2d(x, D, dt, zt, D, VIT_F32, 1, D, 0, 0, 0.f, g_stream));
  linear(zt, h0_w, u, 1, F, D, VIT_F32, VIT_F32, h0_b, VIT_ACT_NONE, NULL, 0, 0, 0, 0, 0, F);
  VIT_CHECK(vit_gelu_fwd(u, gz, F, g_stream));
  VIT_CHECK(vit_layernorm_fwd(gz, F, hln_w, hln_b, zn, F, mean, rstd, 1, F, 1e-5f, VIT_F32, g_stream));
  linear(zn, h3_w, logits, 1, z.nc, F, VIT_F32, VIT_F32, h3_b, VIT_ACT_NONE, NULL, 0, 0, 0, 0, 0, z.nc);
  HIP_CHECK(hipStreamSynchronize(g_stream));
  clock_gettime(CLOCK_MONOTONIC, &t1);

  float* out = (float*)malloc((size_t)z.nc * sizeof(float));
  HIP_CHECK(hipMemcpy(out, logits, (size_t)z.nc * sizeof(float), hipMemcpyDeviceToHost));
  FILE* g = fopen(argv[2], "wb");
  if (!g || fwrite(out, sizeof(float), (size_t)z.nc, g) != (size_t)z.nc) {
    fprintf(stderr, "cannot write %s\n", argv[2]);
    return 1;
  }
  fclose(g);
  printf("vit_forward (%s): C=%d img=%d P=%d D=%d H=%d L=%d nc=%d, %.3f ms\nlogits:", dt == VIT_BF16 ? "bf16" : "f32",
         z.C, z.img, z.P, z.D, z.H, z.L, z.nc,
         (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) / 1e6);
  for (int i = 0; i < z.nc && i < 10; ++i) printf(" %.6f", out[i]);
  printf("%s\n", z.nc > 10 ? " ..." : "");
  return 0;
}
