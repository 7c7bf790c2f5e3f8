// GPU image pipeline of the training loader (reference src/train.py:151-155, BrainTumorDataset.py:35-39):
// convert('RGB') -> Resize((S, S)) (PIL bilinear) -> ToTensor, for a batch of raw uint8 HWC images of any sizes
// (ragged batches allowed) packed into one byte buffer.  Bit-exact with Pillow's 8-bit resampler:
//   * per-axis coefficients are Pillow's (triangle filter, support scaled by the reduction factor, normalised in
//     double, 22-bit fixed point) and are computed on the device in double with FP contraction OFF, so every
//     intermediate rounds exactly as the host C code does;
//   * the horizontal pass rounds to 8 bits (clip8) before the vertical pass, exactly like Pillow's two-pass resize
//     (which runs the horizontal pass first); a pass whose size does not change is an identity in this arithmetic.
// Kernel 1 writes per-image coefficient tables to the caller's workspace; kernel 2 computes one output pixel (all 3
// channels) per thread, coalesced along output rows of each channel plane.
#include <math.h>

#include "vit_common.h"

namespace {

constexpr int PREC = 22;

struct ImgMeta {        // device view of the caller's int64 meta[B][4]
  int64_t off, h, w, c;
};

// Pillow precompute_coeffs + normalize_coeffs_8bpc for output index i of one axis.
__device__ __noinline__ void axis_coeffs(int i, int in_size, int out_size, int ksize, int* bound, int* k) {
#pragma clang fp contract(off)
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const double ss = 1.0 / filterscale;
  const double center = 0.0 + ((double)i + 0.5) * scale;
  int lo = (int)(center - support + 0.5);
  if (lo < 0) lo = 0;
  int hi = (int)(center + support + 0.5);
  if (hi > in_size) hi = in_size;
  const int n = hi - lo;
  double ww = 0.0;
  for (int j = 0; j < n; ++j) {
    double t = ((double)(j + lo) - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    ww += t < 1.0 ? 1.0 - t : 0.0;
  }
  for (int j = 0; j < ksize; ++j) {
    int kv = 0;
    if (j < n) {
      double t = ((double)(j + lo) - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      double w = t < 1.0 ? 1.0 - t : 0.0;
      if (ww != 0.0) w = w / ww;
      kv = w < 0.0 ? (int)(-0.5 + w * (double)(1 << PREC)) : (int)(0.5 + w * (double)(1 << PREC));
    }
    k[j] = kv;
  }
  bound[0] = lo;
  bound[1] = n < ksize ? n : ksize;      // never read past this row's taps (the host passes ksize >= every n)
}

// Table layout per image (ints): bounds_w[ow][2], bounds_h[oh][2], k_w[ow][ks], k_h[oh][ks].
__global__ __launch_bounds__(256) void resize_coeffs_kernel(const int64_t* __restrict__ meta, int oh, int ow, int ks,
                                                            int* __restrict__ tab) {
  const int b = blockIdx.y;
  const ImgMeta m = reinterpret_cast<const ImgMeta*>(meta)[b];
  const int64_t per = (int64_t)(ow + oh) * (2 + ks);
  int* t = tab + b * per;
  int* bw = t;
  int* bh = bw + 2 * ow;
  int* kw = bh + 2 * oh;
  int* kh = kw + (int64_t)ow * ks;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ow + oh; i += gridDim.x * blockDim.x) {
    if (i < ow) axis_coeffs(i, (int)m.w, ow, ks, bw + 2 * i, kw + (int64_t)i * ks);
    else axis_coeffs(i - ow, (int)m.h, oh, ks, bh + 2 * (i - ow), kh + (int64_t)(i - ow) * ks);
  }
}

VIT_DEV int clip8(int v) {
  v >>= PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

template <class TO>
__global__ __launch_bounds__(256) void resize_apply_kernel(const uint8_t* __restrict__ src,
                                                           const int64_t* __restrict__ meta, int oh, int ow, int ks,
                                                           const int* __restrict__ tab, TO* __restrict__ out) {
  const int b = blockIdx.z;
  const int y = blockIdx.y;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= ow) return;
  const ImgMeta m = reinterpret_cast<const ImgMeta*>(meta)[b];
  const int64_t per = (int64_t)(ow + oh) * (2 + ks);
  const int* t = tab + b * per;
  const int* bw = t;
  const int* bh = bw + 2 * ow;
  const int* kw = bh + 2 * oh + (int64_t)x * ks;
  const int* kh = bh + 2 * oh + (int64_t)ow * ks + (int64_t)y * ks;
  const int xlo = bw[2 * x], xn = bw[2 * x + 1];
  const int ylo = bh[2 * y], yn = bh[2 * y + 1];
  const int C = (int)m.c, W = (int)m.w;
  // convert('RGB'): L / LA replicate channel 0, RGB / RGBA take channels 0..2
  const int c1 = C >= 3 ? 1 : 0, c2 = C >= 3 ? 2 : 0;
  const uint8_t* img = src + m.off;
  int acc0 = 1 << (PREC - 1), acc1 = acc0, acc2 = acc0;
  for (int j = 0; j < yn; ++j) {
    const uint8_t* row = img + (int64_t)(ylo + j) * W * C;
    int h0 = 1 << (PREC - 1), h1 = h0, h2 = h0;
    for (int i = 0; i < xn; ++i) {
      const uint8_t* px = row + (int64_t)(xlo + i) * C;
      const int kk = kw[i];
      h0 += (int)px[0] * kk;
      h1 += (int)px[c1] * kk;
      h2 += (int)px[c2] * kk;
    }
    const int kv = kh[j];
    acc0 += clip8(h0) * kv;
    acc1 += clip8(h1) * kv;
    acc2 += clip8(h2) * kv;
  }
  const int64_t plane = (int64_t)oh * ow;
  TO* o = out + (int64_t)b * 3 * plane + (int64_t)y * ow + x;
  st1<TO>(o, (float)clip8(acc0) / 255.0f);           // ToTensor: uint8 / 255, IEEE division
  st1<TO>(o + plane, (float)clip8(acc1) / 255.0f);
  st1<TO>(o + 2 * plane, (float)clip8(acc2) / 255.0f);
}

}  // namespace

extern "C" int vit_resize_ksize(int64_t in_size, int64_t out_size) {
  if (in_size <= 0 || out_size <= 0) return -1;
  const double scale = (double)in_size / (double)out_size;
  const double support = scale < 1.0 ? 1.0 : scale;
  return (int)ceil(support) * 2 + 1;
}

extern "C" int64_t vit_resize_workspace_bytes(int64_t B, int64_t out_h, int64_t out_w, int64_t ksize) {
  return B * (out_h + out_w) * (2 + ksize) * (int64_t)sizeof(int);
}

extern "C" int vit_resize_to_tensor(const void* src, const int64_t* meta, int64_t B, int64_t out_h, int64_t out_w,
                                    int64_t ksize, void* out, int32_t out_dtype, void* workspace,
                                    int64_t workspace_bytes, void* stream) {
  VIT_REQUIRE(src && meta && out && workspace && B > 0 && out_h > 0 && out_w > 0 && ksize >= 3,
              "vit_resize_to_tensor: bad arguments");
  VIT_REQUIRE(out_h <= 65535 && B <= 65535 && ksize <= 4096, "vit_resize_to_tensor: size out of range");
  VIT_REQUIRE(workspace_bytes >= vit_resize_workspace_bytes(B, out_h, out_w, ksize),
              "vit_resize_to_tensor: workspace too small");
  VIT_REQUIRE(out_dtype == VIT_F32 || out_dtype == VIT_BF16, "vit_resize_to_tensor: bad out dtype");
  hipStream_t s = VIT_STREAM(stream);
  int* tab = (int*)workspace;
  const int oh = (int)out_h, ow = (int)out_w, ks = (int)ksize;
  dim3 g1((unsigned)((ow + oh + 255) / 256), (unsigned)B);
  resize_coeffs_kernel<<<g1, 256, 0, s>>>(meta, oh, ow, ks, tab);
  dim3 g2((unsigned)((ow + 255) / 256), (unsigned)oh, (unsigned)B);
  if (out_dtype == VIT_F32)
    resize_apply_kernel<float><<<g2, 256, 0, s>>>((const uint8_t*)src, meta, oh, ow, ks, tab, (float*)out);
  else
    resize_apply_kernel<bf16_t><<<g2, 256, 0, s>>>((const uint8_t*)src, meta, oh, ow, ks, tab, (bf16_t*)out);
  return vit::check_launch("vit_resize_to_tensor");
}
