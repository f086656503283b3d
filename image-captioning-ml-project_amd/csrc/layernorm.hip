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
  // gamma / beta requested with the row (loaded after the statistics they were a second
  // memory round trip per row)
  float wv[MAXC][8], bv[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      Vec8<float>::load(w + ch * 8, wv[c]);
      Vec8<float>::load(b + ch * 8, bv[c]);
    }
  }
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
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mean) * rstd * wv[c][i] + bv[c][i];
      Vec8<T>::store(yr + ch * 8, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// LayerNorm of x = bf16(sum_s slab[s] + bias + res), the decode steps' GEMM -> LayerNorm pairs
// (capk_gemm_pair_slabs with no seam writes the slabs): the slab sum, bias and residual in
// splitk_reduce / epilogue8 order and the statistics in ln_fwd_kernel's order, so y (and x,
// kept in x_out for the pre-LN residual stream) are bit-identical to capk_gemm followed by
// capk_layernorm_fwd -- one launch instead of a reduce and a LayerNorm.
template <int MAXC>
__global__ __launch_bounds__(256) void ln_fwd_slabs_kernel(int rows, int cols, const float* __restrict__ ws,
                                                           int splits, const float* __restrict__ bias,
                                                           const bf16* __restrict__ res, int64_t ldr,
                                                           bf16* __restrict__ x_out, int64_t ldxo,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           float eps, bf16* __restrict__ y, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = cols >> 3;
  const int64_t ss = (int64_t)rows * cols;
  float v[MAXC][8];
  float s = 0.f;
  // the slabs of both of the lane's chunks in groups of 4 splits, every load of a group issued
  // before its first use (a per-split loop waited out one memory round trip per slab and chunk:
  // 16 for the FC2 slabs of a decode step); summed in split order as before
  float a[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) a[c][i] = 0.f;
  // the bias and residual chunks are requested with the first slab group (loaded after the
  // slab loop they were two more memory round trips per row); added after the slabs, in the
  // same order as before
  float bb[MAXC][8], rr[MAXC][8], wv[MAXC][8], bv[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      if (bias) Vec8<float>::load(bias + ch * 8, bb[c]);
      if (res) Vec8<bf16>::load(res + (int64_t)row * ldr + ch * 8, rr[c]);
      Vec8<float>::load(w + ch * 8, wv[c]);  // (gamma / beta likewise)
      Vec8<float>::load(b + ch * 8, bv[c]);
    }
  }
  for (int k0 = 0; k0 < splits; k0 += 4) {
    float t[MAXC][4][8];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ch < nch && k0 + j < splits) Vec8<float>::load(ws + (k0 + j) * ss + (int64_t)row * cols + ch * 8, t[c][j]);
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ch < nch && k0 + j < splits) {
#pragma unroll
          for (int i = 0; i < 8; ++i) a[c][i] += t[c][j][i];
        }
    }
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      if (bias) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[c][i] += bb[c][i];
      }
      if (res) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[c][i] += rr[c][i];
      }
      bf16x8 hx;
#pragma unroll
      for (int i = 0; i < 8; ++i) hx[i] = (bf16)a[c][i];
      if (x_out) *(bf16x8*)(x_out + (int64_t)row * ldxo + ch * 8) = hx;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[c][i] = (float)hx[i];
        s += v[c][i];
      }
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
  bf16* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mean) * rstd * wv[c][i] + bv[c][i];
      Vec8<bf16>::store(yr + ch * 8, o);
    }
  }
}

// Raw 8-element row segment kept in registers between its load and its use (the row loop
// is software-pipelined: the next row's operands are in flight while this row reduces).
template <typename T> struct Seg8;
template <> struct Seg8<bf16> {
  bf16x8 v;
  __device__ __forceinline__ void load(const bf16* p) { v = *(const bf16x8*)p; }
  __device__ __forceinline__ float operator[](int i) const { return (float)v[i]; }
};
template <> struct Seg8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) { a = *(const f32x4*)p; b = *(const f32x4*)(p + 4); }
  __device__ __forceinline__ float operator[](int i) const { return i < 4 ? a[i] : b[i - 4]; }
};

// dx = rstd * (g - mean(g) - xhat * mean(g*xhat)), g = dy*w (+ dres); partial dw/db (and,
// with SUM, the column sums of dx: the bias gradient of the Linear whose output gradient
// dx is) per block.  One wave per row, rows grid-strided; row r+stride's x / dy / dres are
// loaded before row r's reductions, so one memory round trip overlaps one row of work.
template <typename T, int MAXC, bool SUM>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int cols, const T* __restrict__ dy, int64_t lddy,
                                                     const T* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ w, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, T* __restrict__ dx,
                                                     int64_t lddx, const T* __restrict__ dres, int64_t ldres,
                                                     float* __restrict__ part, Drop drop, T* __restrict__ dxd,
                                                     int64_t lddxd) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4 waves][NP][cols]
  constexpr int NP = SUM ? 3 : 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = cols >> 3;
  float dw[MAXC][8], db[MAXC][8], ds[SUM ? MAXC : 1][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) dw[c][i] = db[c][i] = 0.f;
#pragma unroll
  for (int c = 0; c < (SUM ? MAXC : 1); ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) ds[c][i] = 0.f;
  float wv[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) Vec8<float>::load(w + ch * 8, wv[c]);
  }
  const int stride = gridDim.x * 4;
  Seg8<T> xs[MAXC], dys[MAXC], rss[MAXC];
  auto fetch = [&](int row) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        xs[c].load(x + (int64_t)row * ldx + ch * 8);
        dys[c].load(dy + (int64_t)row * lddy + ch * 8);
        if (dres) rss[c].load(dres + (int64_t)row * ldres + ch * 8);
      }
    }
  };
  int row = blockIdx.x * 4 + wave;
  if (row < rows) fetch(row);
  for (; row < rows; row += stride) {
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXC][8], g[MAXC][8], r[MAXC][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = dys[c][i];
          xh[c][i] = (xs[c][i] - mu) * rs;
          g[c][i] = d * wv[c][i];
          r[c][i] = dres ? rss[c][i] : 0.f;
          s1 += g[c][i];
          s2 += g[c][i] * xh[c][i];
          dw[c][i] += d * xh[c][i];
          db[c][i] += d;
        }
      }
    }
    const int next = row + stride;
    if (next < rows) fetch(next);  // registers of this row's operands are free again
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
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += r[c][i];
        if constexpr (SUM) {
#pragma unroll
          for (int i = 0; i < 8; ++i) ds[c][i] += o[i];
        }
        Vec8<T>::store(dx + (int64_t)row * lddx + ch * 8, o);
      }
    }
  }
  // block reduction of dw/db (/ds) over the 4 waves
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      Vec8<float>::store(red + (wave * NP + 0) * cols + ch * 8, dw[c]);
      Vec8<float>::store(red + (wave * NP + 1) * cols + ch * 8, db[c]);
      if constexpr (SUM) Vec8<float>::store(red + (wave * NP + 2) * cols + ch * 8, ds[c]);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NP * cols; i += 256) {
    const int which = i / cols, col = i % cols;
    float s = 0.f;
#pragma unroll
    for (int wv2 = 0; wv2 < 4; ++wv2) s += red[(wv2 * NP + which) * cols + col];
    part[(int64_t)blockIdx.x * NP * cols + i] = s;
  }
}

// bf16 rows of exactly 768 (ViT-B, the config-3 decoder, GPT-2, CLIP): 4-element (8-B)
// segments, three per lane, so every lane is busy (the 8-element kernel above leaves half
// the lanes idle on its second segment), with TWO rows of operands in flight per wave (rows
// r + stride, r + 2 stride requested while row r reduces): 72 KiB in flight per CU.  Measured 81 us on the ViT LN backward before (3.8 TB/s,
// 36 KiB in flight per CU); the dependency on HBM latency is what the deeper queue removes.
template <bool SUM>
__global__ __launch_bounds__(256) void ln_bwd768_kernel(int rows, const bf16* __restrict__ dy, int64_t lddy,
                                                        const bf16* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ w, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, bf16* __restrict__ dx,
                                                        int64_t lddx, const bf16* __restrict__ dres, int64_t ldres,
                                                        float* __restrict__ part, Drop drop, bf16* __restrict__ dxd,
                                                        int64_t lddxd) {
  constexpr int COLS = 768, NC = 3, NP = SUM ? 3 : 2;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4 waves][NP][COLS]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dw[NC][4], db[NC][4], ds[SUM ? NC : 1][4], wv[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const f32x4 t = *(const f32x4*)(w + (lane + 64 * c) * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wv[c][i] = t[i];
      dw[c][i] = db[c][i] = 0.f;
      if constexpr (SUM) ds[c][i] = 0.f;
    }
  }
  // the row's statistics travel with its operands: loaded at the head of step() they were the
  // youngest loads, and the in-order vmcnt wait for them drained the next row's prefetch too
  struct Row { bf16x4 x[NC], d[NC], r[NC]; float mu, rs; };
  auto fetch = [&](int row, Row& R) {
    R.mu = mean[row];
    R.rs = rstd[row];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = (lane + 64 * c) * 4;
      R.x[c] = *(const bf16x4*)(x + (int64_t)row * ldx + col);
      R.d[c] = *(const bf16x4*)(dy + (int64_t)row * lddy + col);
      if (dres) R.r[c] = *(const bf16x4*)(dres + (int64_t)row * ldres + col);
    }
  };
  // one row: statistics from R, then R is refilled with row `nxt` (its loads overlap this
  // row's reductions and stores), then dx
  auto step = [&](Row& R, int row, int nxt) {
    const float mu = R.mu, rs = R.rs;
    float xh[NC][4], g[NC][4], r[NC][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = (float)R.d[c][i];
        xh[c][i] = ((float)R.x[c][i] - mu) * rs;
        g[c][i] = d * wv[c][i];
        r[c][i] = dres ? (float)R.r[c][i] : 0.f;
        s1 += g[c][i];
        s2 += g[c][i] * xh[c][i];
        dw[c][i] += d * xh[c][i];
        db[c][i] += d;
      }
    if (nxt < rows) fetch(nxt, R);
    const float m1 = wave_sum(s1) * (1.f / COLS), m2 = wave_sum(s2) * (1.f / COLS);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = (lane + 64 * c) * 4;
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = rs * (g[c][i] - m1 - xh[c][i] * m2);
      if (dxd) {
        bf16x4 od;
        const uint64_t base = (uint64_t)row * COLS + col;
#pragma unroll
        for (int i = 0; i < 4; ++i) od[i] = (bf16)(o[i] * drop.mul(base + i));
        *(bf16x4*)(dxd + (int64_t)row * lddxd + col) = od;
      }
      bf16x4 ob;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o[i] += r[c][i];
        if constexpr (SUM) ds[c][i] += o[i];
        ob[i] = (bf16)o[i];
      }
      *(bf16x4*)(dx + (int64_t)row * lddx + col) = ob;
    }
  };
  // two row buffers in flight, alternating (no register copies between them: a copy would
  // wait for the younger buffer's loads)
  const int stride = gridDim.x * 4;
  Row A, B;
  int row = blockIdx.x * 4 + wave;
  if (row < rows) fetch(row, A);
  if (row + stride < rows) fetch(row + stride, B);
  for (; row < rows; row += 2 * stride) {
    step(A, row, row + 2 * stride);
    if (row + stride < rows) step(B, row + stride, row + 3 * stride);
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = (lane + 64 * c) * 4;
    *(f32x4*)(red + (wave * NP + 0) * COLS + col) = (f32x4){dw[c][0], dw[c][1], dw[c][2], dw[c][3]};
    *(f32x4*)(red + (wave * NP + 1) * COLS + col) = (f32x4){db[c][0], db[c][1], db[c][2], db[c][3]};
    if constexpr (SUM) *(f32x4*)(red + (wave * NP + 2) * COLS + col) = (f32x4){ds[c][0], ds[c][1], ds[c][2], ds[c][3]};
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NP * COLS; i += 256) {
    const int which = i / COLS, col = i % COLS;
    float s = 0.f;
#pragma unroll
    for (int wv2 = 0; wv2 < 4; ++wv2) s += red[(wv2 * NP + which) * COLS + col];
    part[(int64_t)blockIdx.x * NP * COLS + i] = s;
  }
}

// sum the per-block partials [nblocks][2*cols] (sum_parts / finish_parts16, common.h)
__global__ __launch_bounds__(1024) void ln_bwd_finish_kernel(int nblocks, int cols, int np,
                                                             const float* __restrict__ part, float* __restrict__ dw,
                                                             float* __restrict__ db, float* __restrict__ dsum,
                                                             int accumulate) {
  const float s = finish_parts16(part, np * cols, nblocks, np * cols);
  const int i = blockIdx.x * 16 + threadIdx.x;
  if (threadIdx.x < 16 && i < np * cols) {
    float* dst = i < cols ? dw + i : i < 2 * cols ? db + (i - cols) : dsum + (i - 2 * cols);
    *dst = accumulate ? *dst + s : s;
  }
}

// (the pipelined kernel holds ~200 VGPRs: 2 waves per SIMD, so 512 blocks are all resident)
static int ln_bwd_blocks(int rows) { return std::max(1, std::min(512, (rows + 15) / 16)); }
// ln_bwd768_kernel: 189 VGPRs (two waves per SIMD; held to 168 for three it spills) -> 512
// resident blocks, each wave with two rows in flight
static int ln_bwd768_blocks(int rows) { return std::max(1, std::min(512, (rows + 15) / 16)); }
static bool use768(int dtype, int cols) { return dtype == CAPK_BF16 && cols == 768; }

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

extern "C" int capk_layernorm_fwd_slabs(int rows, int cols, const float* ws, int splits, const float* bias,
                                        const void* res, int64_t ldr, void* x_out, int64_t ldxo, const float* w,
                                        const float* b, float eps, void* y, int64_t ldy, void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols > 0 && cols % 8 == 0 && cols <= 2048 && ws && splits > 0 && w && b && y,
                 "capk_layernorm_fwd_slabs: bad arguments (cols=%d)", cols);
  CAPK_CHECK_ARG(ldy % 8 == 0 && (!res || ldr % 8 == 0) && (!x_out || ldxo % 8 == 0),
                 "capk_layernorm_fwd_slabs: strides must be multiples of 8");
  const dim3 grid(cdiv(rows, 4)), block(256);
#define L(MC)                                                                                                   \
  hipLaunchKernelGGL((ln_fwd_slabs_kernel<MC>), grid, block, 0, S(stream), rows, cols, ws, splits, bias,      \
                     (const bf16*)res, ldr, (bf16*)x_out, ldxo, w, b, eps, (bf16*)y, ldy)
  if (cols <= 1024) L(2); else L(4);
#undef L
  CAPK_LAUNCH_CHECK("ln_fwd_slabs_kernel");
  return CAPK_OK;
}

extern "C" size_t capk_layernorm_bwd_workspace(int rows, int cols) {
  return (size_t)std::max(ln_bwd_blocks(rows), cols == 768 ? ln_bwd768_blocks(rows) : 0) * 3 * cols * sizeof(float);
}

extern "C" int capk_layernorm_bwd(int dtype, int rows, int cols, const void* dy, int64_t lddy, const void* x,
                                  int64_t ldx, const float* w, const float* mean, const float* rstd, void* dx,
                                  int64_t lddx, const void* dres, int64_t ldres, float* dw, float* db,
                                  float* dsum, int accumulate, float drop_p, uint32_t drop_seed, void* dx_drop,
                                  int64_t lddx_drop, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols > 0 && cols % 8 == 0 && cols <= 2048, "capk_layernorm_bwd: cols=%d", cols);
  const bool v768 = use768(dtype, cols) && ldx % 4 == 0 && lddy % 4 == 0 && lddx % 4 == 0 &&
                    (!dres || ldres % 4 == 0) && (!dx_drop || lddx_drop % 4 == 0);
  const int nb = v768 ? ln_bwd768_blocks(rows) : ln_bwd_blocks(rows);
  const int np = dsum ? 3 : 2;
  CAPK_CHECK_ARG(ws && ws_bytes >= (size_t)nb * np * cols * sizeof(float), "capk_layernorm_bwd: workspace too small");
  hipStream_t st = S(stream);
  const size_t shm = (size_t)4 * np * cols * sizeof(float);
#define L(T, MC, SM)                                                                                              \
  hipLaunchKernelGGL((ln_bwd_kernel<T, MC, SM>), dim3(nb), dim3(256), shm, st, rows, cols, (const T*)dy, lddy,  \
                     (const T*)x, ldx, w, mean, rstd, (T*)dx, lddx, (const T*)dres, ldres, (float*)ws,           \
                     make_drop(drop_p, drop_seed), (T*)dx_drop, lddx_drop)
#define LS(T, MC) \
  if (dsum) L(T, MC, true); else L(T, MC, false);
#define L768(SM)                                                                                                \
  hipLaunchKernelGGL((ln_bwd768_kernel<SM>), dim3(nb), dim3(256), shm, st, rows, (const bf16*)dy, lddy,          \
                     (const bf16*)x, ldx, w, mean, rstd, (bf16*)dx, lddx, (const bf16*)dres, ldres, (float*)ws,    \
                     make_drop(drop_p, drop_seed), (bf16*)dx_drop, lddx_drop)
  if (v768) { if (dsum) L768(true); else L768(false); }
  else if (dtype == CAPK_BF16) { if (cols <= 1024) { LS(bf16, 2) } else { LS(bf16, 4) } }
  else if (dtype == CAPK_F32) { if (cols <= 1024) { LS(float, 2) } else { LS(float, 4) } }
  else { set_error("capk_layernorm_bwd: dtype"); return CAPK_EINVAL; }
#undef LS
#undef L
#undef L768
  CAPK_LAUNCH_CHECK("ln_bwd_kernel");
  // deferred (capk_finish_defer): the weight / bias / fused-sum columns as three queued finishes
  // over the same partial rows (the same per-column sums as ln_bwd_finish_kernel)
  if (finish_enqueue((const float*)ws, (int64_t)np * cols, nb, cols, dw, accumulate, st)) {
    finish_enqueue((const float*)ws + cols, (int64_t)np * cols, nb, cols, db, accumulate, st);
    if (dsum) finish_enqueue((const float*)ws + 2 * cols, (int64_t)np * cols, nb, cols, dsum, accumulate, st);
    return CAPK_OK;
  }
  hipLaunchKernelGGL(ln_bwd_finish_kernel, dim3(cdiv(np * cols, 16)), dim3(1024), 0, st, nb, cols, np,
                     (const float*)ws, dw, db, dsum, accumulate);
  CAPK_LAUNCH_CHECK("ln_bwd_finish_kernel");
  return CAPK_OK;
}
