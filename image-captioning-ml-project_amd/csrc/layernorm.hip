// LayerNorm forward/backward: one wavefront per row, 16-B vector loads, fp32
// statistics by wavefront shuffles (HBM-bound: 2 passes over the row bytes fwd,
// 3 bwd).  Replaces F.layer_norm in ViTLayer (modeling_vit.py:270,278,348),
// nn.TransformerDecoderLayer norm1..3 (transformer.py:1148-1153), CLIP/GPT-2 LNs.
#include "common.h"

namespace capk {

template <typename T, int MAXC>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int rows, int cols, const T* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     float eps, T* __restrict__ y, int64_t ldy,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = cols >> 3;
  const T* xr = x + (int64_t)row * ldx;
  float v[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      Vec8<T>::load(xr + ch * 8, v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    }
  }
  const float mean = wave_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { const float d = v[c][i] - mean; q += d * d; }
    }
  }
  const float var = wave_sum(q) / cols;
  const float rstd = rsqrtf(var + eps);
  T* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float wv[8], bv[8], o[8];
      Vec8<float>::load(w + ch * 8, wv);
      Vec8<float>::load(b + ch * 8, bv);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mean) * rstd * wv[i] + bv[i];
      Vec8<T>::store(yr + ch * 8, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g*xhat)), g = dy*w ; partial dw/db per block.
template <typename T, int MAXC>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int cols, const T* __restrict__ dy, int64_t lddy,
                                                     const T* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ w, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, T* __restrict__ dx,
                                                     int64_t lddx, const T* __restrict__ dres, int64_t ldres,
                                                     float* __restrict__ part, Drop drop, T* __restrict__ dxd,
                                                     int64_t lddxd) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4 waves][2][cols]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = cols >> 3;
  float dw[MAXC][8], db[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) dw[c][i] = db[c][i] = 0.f;
  float wv[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) Vec8<float>::load(w + ch * 8, wv[c]);
  }
  for (int row = blockIdx.x * 4 + wave; row < rows; row += gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXC][8], g[MAXC][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float xv[8], d[8];
        Vec8<T>::load(x + (int64_t)row * ldx + ch * 8, xv);
        Vec8<T>::load(dy + (int64_t)row * lddy + ch * 8, d);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[c][i] = (xv[i] - mu) * rs;
          g[c][i] = d[i] * wv[c][i];
          s1 += g[c][i];
          s2 += g[c][i] * xh[c][i];
          dw[c][i] += d[i] * xh[c][i];
          db[c][i] += d[i];
        }
      }
    }
    const float m1 = wave_sum(s1) / cols, m2 = wave_sum(s2) / cols;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = rs * (g[c][i] - m1 - xh[c][i] * m2);
        if (dxd) {  // masked copy dx * keep/(1-p): gradient of the dropped branch feeding this LN
          float od[8];
          const uint64_t base = (uint64_t)row * cols + ch * 8;
#pragma unroll
          for (int i = 0; i < 8; ++i) od[i] = o[i] * drop.mul(base + i);
          Vec8<T>::store(dxd + (int64_t)row * lddxd + ch * 8, od);
        }
        if (dres) {
          float r[8];
          Vec8<T>::load(dres + (int64_t)row * ldres + ch * 8, r);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += r[i];
        }
        Vec8<T>::store(dx + (int64_t)row * lddx + ch * 8, o);
      }
    }
  }
  // block reduction of dw/db over the 4 waves
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      Vec8<float>::store(red + (wave * 2 + 0) * cols + ch * 8, dw[c]);
      Vec8<float>::store(red + (wave * 2 + 1) * cols + ch * 8, db[c]);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * cols; i += 256) {
    const int which = i / cols, col = i % cols;
    float s = 0.f;
#pragma unroll
    for (int wv2 = 0; wv2 < 4; ++wv2) s += red[(wv2 * 2 + which) * cols + col];
    part[(int64_t)blockIdx.x * 2 * cols + i] = s;
  }
}

// sum the per-block partials [nblocks][2*cols] (sum_parts / finish_parts16, common.h)
__global__ __launch_bounds__(1024) void ln_bwd_finish_kernel(int nblocks, int cols, const float* __restrict__ part,
                                                             float* __restrict__ dw, float* __restrict__ db,
                                                             int accumulate) {
  const float s = finish_parts16(part, 2 * cols, nblocks, 2 * cols);
  const int i = blockIdx.x * 16 + threadIdx.x;
  if (threadIdx.x < 16 && i < 2 * cols) {
    float* dst = i < cols ? dw + i : db + (i - cols);
    *dst = accumulate ? *dst + s : s;
  }
}

static int ln_bwd_blocks(int rows) { return std::max(1, std::min(1024, (rows + 15) / 16)); }

}  // namespace capk

using namespace capk;

extern "C" int capk_layernorm_fwd(int dtype, int rows, int cols, const void* x, int64_t ldx, const float* w,
                                  const float* b, float eps, void* y, int64_t ldy, float* mean, float* rstd,
                                  void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols > 0 && cols % 8 == 0 && cols <= 2048, "capk_layernorm_fwd: cols=%d (need %%8, <=2048)", cols);
  CAPK_CHECK_ARG(ldx % 8 == 0 && ldy % 8 == 0, "capk_layernorm_fwd: strides must be multiples of 8");
  const dim3 grid(cdiv(rows, 4)), block(256);
  hipStream_t st = S(stream);
#define L(T, MC) hipLaunchKernelGGL((ln_fwd_kernel<T, MC>), grid, block, 0, st, rows, cols, (const T*)x, ldx, w, b, eps, (T*)y, ldy, mean, rstd)
  if (dtype == CAPK_BF16) { if (cols <= 1024) L(bf16, 2); else L(bf16, 4); }
  else if (dtype == CAPK_F32) { if (cols <= 1024) L(float, 2); else L(float, 4); }
  else { set_error("capk_layernorm_fwd: dtype"); return CAPK_EINVAL; }
#undef L
  CAPK_LAUNCH_CHECK("ln_fwd_kernel");
  return CAPK_OK;
}

extern "C" size_t capk_layernorm_bwd_workspace(int rows, int cols) {
  return (size_t)ln_bwd_blocks(rows) * 2 * cols * sizeof(float);
}

extern "C" int capk_layernorm_bwd(int dtype, int rows, int cols, const void* dy, int64_t lddy, const void* x,
                                  int64_t ldx, const float* w, const float* mean, const float* rstd, void* dx,
                                  int64_t lddx, const void* dres, int64_t ldres, float* dw, float* db,
                                  int accumulate, float drop_p, uint32_t drop_seed, void* dx_drop,
                                  int64_t lddx_drop, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols > 0 && cols % 8 == 0 && cols <= 2048, "capk_layernorm_bwd: cols=%d", cols);
  const int nb = ln_bwd_blocks(rows);
  CAPK_CHECK_ARG(ws && ws_bytes >= (size_t)nb * 2 * cols * sizeof(float), "capk_layernorm_bwd: workspace too small");
  hipStream_t st = S(stream);
  const size_t shm = (size_t)8 * cols * sizeof(float);
#define L(T, MC)                                                                                              \
  hipLaunchKernelGGL((ln_bwd_kernel<T, MC>), dim3(nb), dim3(256), shm, st, rows, cols, (const T*)dy, lddy,  \
                     (const T*)x, ldx, w, mean, rstd, (T*)dx, lddx, (const T*)dres, ldres, (float*)ws,       \
                     make_drop(drop_p, drop_seed), (T*)dx_drop, lddx_drop)
  if (dtype == CAPK_BF16) { if (cols <= 1024) L(bf16, 2); else L(bf16, 4); }
  else if (dtype == CAPK_F32) { if (cols <= 1024) L(float, 2); else L(float, 4); }
  else { set_error("capk_layernorm_bwd: dtype"); return CAPK_EINVAL; }
#undef L
  CAPK_LAUNCH_CHECK("ln_bwd_kernel");
  hipLaunchKernelGGL(ln_bwd_finish_kernel, dim3(cdiv(2 * cols, 16)), dim3(1024), 0, st, nb, cols, (const float*)ws, dw,
                     db, accumulate);
  CAPK_LAUNCH_CHECK("ln_bwd_finish_kernel");
  return CAPK_OK;
}
