// Image input transforms on the device (the input pipeline).
//
// Replaces, per batch, the reference's torchvision transforms on PIL images
// (src/main.py:139-153):
//   train: RandomResizedCrop(224) -> RandomHorizontalFlip -> ToTensor -> Normalize
//   val:   Resize(224) -> CenterCrop(224) -> ToTensor -> Normalize
// The host decodes JPEGs to uint8 RGB (PIL, as the reference) and samples the crop boxes /
// flips (capk/data.py restates torchvision's samplers); the packed uint8 images go to HBM
// once and one kernel produces the normalised [B, 3, S, S] batch.
//
// Resampling restates Pillow's ImagingResample for 8-bit images exactly (libImaging/
// Resample.c: bilinear triangle filter with support scaled by the downscale factor --
// antialiasing -- coefficients normalised in double and converted to 22-bit fixed point,
// horizontal pass first with uint8 rounding + clipping of the intermediate, then the
// vertical pass), so the output is bit-identical to PIL + torchvision (tests/
// test_gpu_data.py).  Each output pixel recomputes the horizontal taps it needs (a few
// dozen multiply-adds): the kernel is bound by the uint8 reads, ~0.6 MB per image.
#include "common.h"

#pragma clang fp contract(off)  // coefficient math in the order and rounding of Resample.c

namespace capk {

namespace {

constexpr int RS_PREC = 22;  // PRECISION_BITS = 32 - 8 - 2
constexpr int RS_KMAX = 64;  // taps per output sample (support * 2 + 1), downscale <= 31x

struct ImgDesc {
  int64_t offset;   // byte offset of the image in the packed buffer (HWC, RGB)
  int H, W;         // decoded image size
  int cy, cx;       // crop origin (rows, cols)
  int ch, cw;       // crop size; the crop is resized to rh x rw ...
  int rh, rw;
  int oy, ox;       // ... and the output window starts at (oy, ox) of the resized image
  int flip;         // horizontal flip of the output window
};

__device__ __forceinline__ double tri(double x) {
  if (x < 0.0) x = -x;
  if (x < 1.0) return 1.0 - x;
  return 0.0;
}

// Pillow precompute_coeffs for one output sample xx of an (in_size -> out_size) resize,
// then normalize_coeffs_8bpc.  Returns xmin; *n = number of taps.
__device__ int coeffs(int in_size, int out_size, int xx, int* kk, int* n) {
  const double scale = (double)in_size / (double)out_size;
  double filterscale = scale;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 1.0 * filterscale;
  const double center = (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  if (xmax > RS_KMAX) xmax = RS_KMAX;  // guarded on the host (downscale <= 31x)
  double k[RS_KMAX];
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) {
    const double w = tri((x + xmin - center + 0.5) * ss);
    k[x] = w;
    ww += w;
  }
  for (int x = 0; x < xmax; ++x) {
    if (ww != 0.0) k[x] /= ww;
    kk[x] = k[x] < 0 ? (int)(-0.5 + k[x] * (1 << RS_PREC)) : (int)(0.5 + k[x] * (1 << RS_PREC));
  }
  *n = xmax;
  return xmin;
}

__device__ __forceinline__ int clip8(int v) {
  v >>= RS_PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// One thread per (image, output row, output column): all three channels.
template <typename OutT>
__global__ __launch_bounds__(256) void resize_normalize_kernel(const uint8_t* __restrict__ src,
                                                               const ImgDesc* __restrict__ desc, int B, int Sz,
                                                               float m0, float m1, float m2, float s0, float s1,
                                                               float s2, OutT* __restrict__ out) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (gid >= (int64_t)B * Sz * Sz) return;
  const int b = (int)(gid / ((int64_t)Sz * Sz));
  const int p = (int)(gid % ((int64_t)Sz * Sz));
  const int y = p / Sz, xo = p % Sz;
  const ImgDesc d = desc[b];
  const int x = d.flip ? Sz - 1 - xo : xo;
  const int yy = d.oy + y, xx = d.ox + x;  // sample of the resized crop
  const uint8_t* img = src + d.offset;
  const bool need_h = d.rw != d.cw, need_v = d.rh != d.ch;
  int kx[RS_KMAX], ky[RS_KMAX];
  int nx = 1, ny = 1, x0 = xx, y0 = yy;
  if (need_h) x0 = coeffs(d.cw, d.rw, xx, kx, &nx);
  if (need_v) y0 = coeffs(d.ch, d.rh, yy, ky, &ny);
  int acc[3];
  if (need_v) {
    const int half = 1 << (RS_PREC - 1);
    acc[0] = acc[1] = acc[2] = half;
  }
  for (int j = 0; j < ny; ++j) {
    const uint8_t* row = img + ((int64_t)(d.cy + y0 + j) * d.W + d.cx) * 3;
    int h[3];
    if (need_h) {
      int s0i = 1 << (RS_PREC - 1), s1i = s0i, s2i = s0i;
      for (int i = 0; i < nx; ++i) {
        const uint8_t* px = row + (x0 + i) * 3;
        s0i += px[0] * kx[i];
        s1i += px[1] * kx[i];
        s2i += px[2] * kx[i];
      }
      h[0] = clip8(s0i);
      h[1] = clip8(s1i);
      h[2] = clip8(s2i);
    } else {
      const uint8_t* px = row + x0 * 3;
      h[0] = px[0];
      h[1] = px[1];
      h[2] = px[2];
    }
    if (need_v) {
      acc[0] += h[0] * ky[j];
      acc[1] += h[1] * ky[j];
      acc[2] += h[2] * ky[j];
    } else {
      acc[0] = h[0];
      acc[1] = h[1];
      acc[2] = h[2];
    }
  }
  int v[3];
  for (int c = 0; c < 3; ++c) v[c] = need_v ? clip8(acc[c]) : acc[c];
  // ToTensor (x / 255) then Normalize ((x - mean) / std), fp32 as torchvision
  const float mean[3] = {m0, m1, m2}, stdv[3] = {s0, s1, s2};
  const int64_t plane = (int64_t)Sz * Sz;
  OutT* o = out + (int64_t)b * 3 * plane + (int64_t)y * Sz + xo;
  for (int c = 0; c < 3; ++c) o[c * plane] = from_f32<OutT>(((float)v[c] / 255.0f - mean[c]) / stdv[c]);
}

}  // namespace
}  // namespace capk

using namespace capk;

extern "C" size_t capk_image_desc_bytes(void) { return sizeof(ImgDesc); }

extern "C" int capk_resize_normalize(int out_dtype, int B, int size, const void* images, const void* desc,
                                     const float* mean, const float* stdv, void* out, void* stream) {
  CAPK_CHECK_ARG(B > 0 && size > 0 && images && desc && mean && stdv && out, "capk_resize_normalize: bad arguments");
  CAPK_CHECK_ARG(out_dtype == CAPK_F32 || out_dtype == CAPK_BF16, "capk_resize_normalize: out dtype");
  const int64_t n = (int64_t)B * size * size;
  const int grid = (int)((n + 255) / 256);
  if (out_dtype == CAPK_F32)
    hipLaunchKernelGGL(resize_normalize_kernel<float>, dim3(grid), dim3(256), 0, S(stream), (const uint8_t*)images,
                       (const ImgDesc*)desc, B, size, mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2],
                       (float*)out);
  else
    hipLaunchKernelGGL(resize_normalize_kernel<bf16>, dim3(grid), dim3(256), 0, S(stream), (const uint8_t*)images,
                       (const ImgDesc*)desc, B, size, mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2],
                       (bf16*)out);
  CAPK_LAUNCH_CHECK("resize_normalize_kernel");
  return CAPK_OK;
}
