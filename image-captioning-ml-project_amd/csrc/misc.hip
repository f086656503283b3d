// HBM-bound kernels of the hot path: ViT patchify + token assembly, token and
// position embeddings, shifted cross entropy (fwd+bwd fused), bias-gradient
// column sums, casts/copies and the AdamW update.  All use 16-B vector
// accesses per lane (cdna guide G13).
#include <utility>
#include <vector>

#include "common.h"

namespace capk {

// ------------------------------------------------------------ patchify -----
template <typename T>
__global__ __launch_bounds__(256) void patchify_kernel(int B, int C, int H, int W, int P,
                                                       const float* __restrict__ img, T* __restrict__ out) {
  const int nw = W / P, np = (H / P) * nw, kcols = C * P * P;
  const int64_t total = (int64_t)B * np * (kcols / 8);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int chunk = (int)(i % (kcols / 8));
    const int64_t row = i / (kcols / 8);
    const int b = (int)(row / np), p = (int)(row % np);
    const int col = chunk * 8;
    const int c = col / (P * P), kh = (col / P) % P, kw = col % P;
    const int y = (p / nw) * P + kh, x = (p % nw) * P + kw;
    float v[8];
    Vec8<float>::load(img + (((int64_t)b * C + c) * H + y) * W + x, v);
    Vec8<T>::store(out + row * kcols + col, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void vit_assemble_kernel(int B, int Np, int D, const T* __restrict__ patch,
                                                           const float* __restrict__ cls, const float* __restrict__ pos,
                                                           T* __restrict__ x) {
  const int dch = D / 8;
  const int64_t total = (int64_t)B * (Np + 1) * dch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % dch);
    const int64_t row = i / dch;
    const int b = (int)(row / (Np + 1)), n = (int)(row % (Np + 1));
    float v[8], pv[8];
    if (n == 0) Vec8<float>::load(cls + c * 8, v);
    else Vec8<T>::load(patch + ((int64_t)b * Np + n - 1) * D + c * 8, v);
    Vec8<float>::load(pos + (int64_t)n * D + c * 8, pv);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += pv[k];
    Vec8<T>::store(x + row * D + c * 8, v);
  }
}

// ------------------------------------------------------------ embeddings ---
template <typename T>
__global__ __launch_bounds__(256) void embedding_fwd_kernel(int B, int T_, int D, const int64_t* __restrict__ ids,
                                                            const float* __restrict__ table,
                                                            const float* __restrict__ pos, int pos_offset,
                                                            T* __restrict__ out, Drop drop) {
  const int dch = D / 8;
  const int64_t total = (int64_t)B * T_ * dch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % dch);
    const int64_t row = i / dch;
    const int t = (int)(row % T_);
    float v[8];
    Vec8<float>::load(table + ids[row] * D + c * 8, v);
    if (pos) {
      float pv[8];
      Vec8<float>::load(pos + (int64_t)(pos_offset + t) * D + c * 8, pv);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += pv[k];
    }
    if (drop.on()) {
      const uint64_t base = (uint64_t)row * D + c * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= drop.mul(base + k);
    }
    Vec8<T>::store(out + row * D + c * 8, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void embedding_bwd_kernel(int B, int T_, int D, const int64_t* __restrict__ ids,
                                                            const T* __restrict__ dout, int padding_idx,
                                                            float* __restrict__ dtable, float* __restrict__ dpos,
                                                            int pos_offset, Drop drop) {
  const int64_t total = (int64_t)B * T_ * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const int64_t row = i / D;
    const float g = drop.on() ? to_f32(dout[i]) * drop.mul((uint64_t)i) : to_f32(dout[i]);
    const int64_t id = ids[row];
    if (dtable && id != padding_idx) atomicAdd(dtable + id * D + d, g);
    if (dpos) atomicAdd(dpos + (int64_t)(pos_offset + (int)(row % T_)) * D + d, g);
  }
}

// ------------------------------------------------------- shifted CE --------
__global__ void ce_count_kernel(int B, int T_, const int64_t* __restrict__ targets, int ignore_index,
                                float* __restrict__ cnt) {
  float c = 0.f;
  for (int i = threadIdx.x; i < B * (T_ - 1); i += blockDim.x) {
    const int b = i / (T_ - 1), t = i % (T_ - 1);
    c += targets[(int64_t)b * T_ + t + 1] != ignore_index ? 1.f : 0.f;
  }
  __shared__ float red[16];
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    cnt[0] = s;
  }
}

constexpr int CE_THREADS = 1024;
constexpr int CE_MAXCH = 8;  // up to 8*8*1024 = 65536 columns per row

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < nw; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  return r;
}

template <typename T>
__global__ __launch_bounds__(CE_THREADS) void ce_rows_kernel(int B, int T_, int V, int64_t ld,
                                                             const T* __restrict__ logits,
                                                             const int64_t* __restrict__ targets, int ignore_index,
                                                             const float* __restrict__ grad_scale, const float* __restrict__ cnt,
                                                             float* __restrict__ row_loss, T* __restrict__ dlogits,
                                                             const float* __restrict__ row_weight) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int b = row / T_, t = row % T_;
  const int64_t tgt = (t < T_ - 1) ? targets[(int64_t)b * T_ + t + 1] : (int64_t)ignore_index;
  const bool counted = tgt != ignore_index;
  const T* lr = logits + (int64_t)row * ld;
  const int nch = (int)(ld / 8);
  if (!counted) {
    if (threadIdx.x == 0 && row_loss) row_loss[row] = 0.f;
    if (dlogits) {
      const float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int c = threadIdx.x; c < nch; c += CE_THREADS) Vec8<T>::store(dlogits + (int64_t)row * ld + c * 8, z);
    }
    return;
  }
  const float tgt_logit = to_f32(lr[tgt]);  // read before any in-place gradient write
  float v[CE_MAXCH][8];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < CE_MAXCH; ++k) {
    const int c = threadIdx.x + k * CE_THREADS;
    if (c < nch) {
      Vec8<T>::load(lr + c * 8, v[k]);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (c * 8 + i >= V) v[k][i] = -INFINITY;
        mx = fmaxf(mx, v[k][i]);
      }
    }
  }
  mx = block_reduce(mx, red, true);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < CE_MAXCH; ++k) {
    const int c = threadIdx.x + k * CE_THREADS;
    if (c < nch) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[k][i] = __expf(v[k][i] - mx);
        s += v[k][i];
      }
    }
  }
  s = block_reduce(s, red, false);
  const float lse = mx + __logf(s);
  const float rw = row_weight ? row_weight[b] : 1.f;
  if (threadIdx.x == 0 && row_loss) row_loss[row] = rw * (lse - tgt_logit);
  if (dlogits) {
    const float scale = rw * (grad_scale ? grad_scale[0] : 1.f) / cnt[0];
    const float inv = 1.f / s;
#pragma unroll
    for (int k = 0; k < CE_MAXCH; ++k) {
      const int c = threadIdx.x + k * CE_THREADS;
      if (c < nch) {
        float g[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int col = c * 8 + i;
          g[i] = col < V ? (v[k][i] * inv - (col == tgt ? 1.f : 0.f)) * scale : 0.f;
        }
        Vec8<T>::store(dlogits + (int64_t)row * ld + c * 8, g);
      }
    }
  }
}

__global__ void ce_finish_kernel(int rows, const float* __restrict__ row_loss, const float* __restrict__ cnt,
                                 float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < rows; i += blockDim.x) s += row_loss[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    out[0] = t / cnt[0];
    out[1] = cnt[0];
  }
}

// ------------------------------------- shifted CE from the LM head's partials --------
// capk_linear_lse leaves per row P = 4 cdiv(Vp, 256) pairs (max, sum 2^(t - max)) of
// t = log2(e) * logit over disjoint column ranges.  Forward: CEM_ROWS rows per workgroup and
// 32 partial streams per row (lane = (stream, row): each wave-load reads 8 rows x 8 B of 8
// partials), stream s merging partials s, s + 32, ..., combined in stream order through LDS into
// lse (natural log) and the row loss lse - logit[target]; M / 8 workgroups (640 at config 3) fill
// the chip where the round-5 form (64 rows per workgroup, 197 dependent loads per lane) ran 80.
// Backward: one streaming pass, dlogits = (2^(t - lse log2 e) - [col == target]) * grad_scale /
// count with the column sums of the stored gradient (the LM-head bias gradient) as per-row-group
// partials.
constexpr int CEM_ROWS = 8, CEM_STREAMS = 32;
__device__ __forceinline__ void lse2_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;  // an empty state (a wave whose columns were all padding)
  const float mn = fmaxf(m, m2);
  s = s * __builtin_amdgcn_exp2f(m - mn) + s2 * __builtin_amdgcn_exp2f(m2 - mn);
  m = mn;
}
__global__ __launch_bounds__(256) void ce_lse_merge_kernel(int B, int T_, int M, int P, const float2* __restrict__ part,
                                                           const bf16* __restrict__ logits, int64_t ld,
                                                           const int64_t* __restrict__ targets, int ignore_index,
                                                           float* __restrict__ lse_out, float* __restrict__ row_loss) {
  __shared__ float red[2][CEM_STREAMS][CEM_ROWS];
  const int r = threadIdx.x & (CEM_ROWS - 1), st = threadIdx.x / CEM_ROWS;
  const int row = blockIdx.x * CEM_ROWS + r;
  float m = -INFINITY, sum = 0.f;
  if (row < M) {
#pragma unroll 4
    for (int p = st; p < P; p += CEM_STREAMS) {
      const float2 q = part[(int64_t)p * M + row];
      lse2_merge(m, sum, q.x, q.y);
    }
  }
  red[0][st][r] = m;
  red[1][st][r] = sum;
  __syncthreads();
  if (threadIdx.x < CEM_ROWS && row < M) {
    float mm = -INFINITY, ss = 0.f;
#pragma unroll 8
    for (int i = 0; i < CEM_STREAMS; ++i) lse2_merge(mm, ss, red[0][i][r], red[1][i][r]);
    const float lse = (mm + __log2f(ss)) * 0.6931471805599453f;
    lse_out[row] = lse;
    const int b = row / T_, t = row % T_;
    const int64_t tgt = (t < T_ - 1) ? targets[(int64_t)b * T_ + t + 1] : (int64_t)ignore_index;
    row_loss[row] = tgt != ignore_index ? lse - (float)logits[(int64_t)row * ld + tgt] : 0.f;
  }
}

constexpr int CEB_ROWS = 128;  // rows per block of the backward pass (one column-sum partial row each)
template <typename T>
__global__ __launch_bounds__(256) void ce_lse_bwd_kernel(int B, int T_, int V, int64_t ld, const T* __restrict__ logits,
                                                         const int64_t* __restrict__ targets, int ignore_index,
                                                         const float* __restrict__ lse, const float* __restrict__ cnt,
                                                         const float* __restrict__ grad_scale, T* __restrict__ dlogits,
                                                         float* __restrict__ dbias_part) {
  __shared__ float lse_s[CEB_ROWS];
  __shared__ int tgt_s[CEB_ROWS];
  const int M = B * T_;
  const int r0 = blockIdx.y * CEB_ROWS, nr = min(CEB_ROWS, M - r0);
  for (int i = threadIdx.x; i < nr; i += blockDim.x) {
    const int row = r0 + i, b = row / T_, t = row % T_;
    const int64_t tgt = (t < T_ - 1) ? targets[(int64_t)b * T_ + t + 1] : (int64_t)ignore_index;
    tgt_s[i] = tgt != ignore_index ? (int)tgt : -1;  // -1: not counted (the whole row's gradient is 0)
    lse_s[i] = lse[row] * 1.4426950408889634f;
  }
  __syncthreads();
  const float scale = (grad_scale ? grad_scale[0] : 1.f) / cnt[0];
  const int c8 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (c8 >= ld) return;
  float cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < nr; ++i) {
    const int row = r0 + i, tg = tgt_s[i];
    float g[8];
    if (tg < 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = 0.f;
    } else {
      float l[8];
      Vec8<T>::load(logits + (int64_t)row * ld + c8, l);
      const float ls = lse_s[i];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int col = c8 + k;
        const float pr = __builtin_amdgcn_exp2f(fmaf(l[k], 1.4426950408889634f, -ls));
        g[k] = col < V ? (pr - (col == tg ? 1.f : 0.f)) * scale : 0.f;
      }
    }
    Vec8<T>::store(dlogits + (int64_t)row * ld + c8, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) cs[k] += to_f32(from_f32<T>(g[k]));  // the stored (rounded) values
  }
  if (dbias_part) {
    float* dst = dbias_part + (int64_t)blockIdx.y * ld + c8;
    *(f32x4*)dst = (f32x4){cs[0], cs[1], cs[2], cs[3]};
    *(f32x4*)(dst + 4) = (f32x4){cs[4], cs[5], cs[6], cs[7]};
  }
}

// Zero the gap rows of a batch of strided row blocks: rows b * rpb + j for S <= j < rpb (and
// row < rows), row_bytes from each row start -- the rows of a [B * rpb - 1, C] gradient that a
// strided view skips (the decoder's cross-attention K / V gradient over the ViT sequence: the
// CLS rows), instead of clearing the whole buffer.
__global__ __launch_bounds__(256) void zero_gap_rows_kernel(char* __restrict__ base, int64_t ld_bytes, int chunks,
                                                            int B, int rpb, int S, int rows) {
  const int64_t total = (int64_t)B * (rpb - S) * chunks;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % chunks);
    const int64_t g = i / chunks;
    const int b = (int)(g / (rpb - S)), j = S + (int)(g % (rpb - S));
    const int64_t row = (int64_t)b * rpb + j;
    if (row < rows) *(f32x4*)(base + row * ld_bytes + (int64_t)c * 16) = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
}

// ------------------------------------------------------------ colsum --------
constexpr int CS_ROWS_PER_SPLIT = 256;
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(int M, int N, const T* __restrict__ dy, int64_t ldy,
                                                     float* __restrict__ part) {
  __shared__ float red[4][64 * 8 + 4];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int m0 = blockIdx.y * CS_ROWS_PER_SPLIT, m1 = min(M, m0 + CS_ROWS_PER_SPLIT);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c * 8 < N) {
    int m = m0 + ph;
    for (; m + 12 < m1; m += 16) {  // four independent row loads in flight
      float v0[8], v1[8], v2[8], v3[8];
      Vec8<T>::load(dy + (int64_t)m * ldy + c * 8, v0);
      Vec8<T>::load(dy + (int64_t)(m + 4) * ldy + c * 8, v1);
      Vec8<T>::load(dy + (int64_t)(m + 8) * ldy + c * 8, v2);
      Vec8<T>::load(dy + (int64_t)(m + 12) * ldy + c * 8, v3);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += (v0[i] + v1[i]) + (v2[i] + v3[i]);
    }
    for (; m < m1; m += 4) {
      float v[8];
      Vec8<T>::load(dy + (int64_t)m * ldy + c * 8, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[ph][lane * 8 + i] = acc[i];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int col = blockIdx.x * 512 + i;
    if (col < N) part[(int64_t)blockIdx.y * N + col] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

// Backward activation pass with the bias gradient fused: C (= dY.W of the next Linear)
// <- C * act'(aux) (or * aux with CAPK_ACT_DERIV) in place, and the column sums of the
// result (the producing Linear's bias gradient) as colsum_kernel's per-split partials --
// one HBM pass instead of the activation pass + a colsum pass over the same matrix.
template <typename T>
__global__ __launch_bounds__(256) void act_bwd_colsum_kernel(int M, int N, T* __restrict__ C, int64_t ldc,
                                                             const T* __restrict__ aux, int64_t ldx, int act,
                                                             float* __restrict__ part) {
  __shared__ float red[4][64 * 8 + 4];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int m0 = blockIdx.y * CS_ROWS_PER_SPLIT, m1 = min(M, m0 + CS_ROWS_PER_SPLIT);
  const int a = act & 15;
  const bool deriv = act & CAPK_ACT_DERIV;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c * 8 < N) {
    int m = m0 + ph;
    for (; m + 4 < m1; m += 8) {  // two rows (four loads) in flight
      float v0[8], g0[8], v1[8], g1[8];
      Vec8<T>::load(C + (int64_t)m * ldc + c * 8, v0);
      Vec8<T>::load(aux + (int64_t)m * ldx + c * 8, g0);
      Vec8<T>::load(C + (int64_t)(m + 4) * ldc + c * 8, v1);
      Vec8<T>::load(aux + (int64_t)(m + 4) * ldx + c * 8, g1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v0[i] *= deriv ? g0[i] : act_grad_fast<T>(a, g0[i]);
        v1[i] *= deriv ? g1[i] : act_grad_fast<T>(a, g1[i]);
        acc[i] += v0[i] + v1[i];
      }
      Vec8<T>::store(C + (int64_t)m * ldc + c * 8, v0);
      Vec8<T>::store(C + (int64_t)(m + 4) * ldc + c * 8, v1);
    }
    for (; m < m1; m += 4) {
      float v[8], g[8];
      Vec8<T>::load(C + (int64_t)m * ldc + c * 8, v);
      Vec8<T>::load(aux + (int64_t)m * ldx + c * 8, g);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[i] *= deriv ? g[i] : act_grad_fast<T>(a, g[i]);
        acc[i] += v[i];
      }
      Vec8<T>::store(C + (int64_t)m * ldc + c * 8, v);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[ph][lane * 8 + i] = acc[i];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int col = blockIdx.x * 512 + i;
    if (col < N) part[(int64_t)blockIdx.y * N + col] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

__global__ __launch_bounds__(1024) void colsum_finish_kernel(int splits, int N, const float* __restrict__ part,
                                                             float* __restrict__ out, int accumulate) {
  const float s = finish_parts16(part, N, splits, N);
  const int n = blockIdx.x * 16 + threadIdx.x;
  if (threadIdx.x < 16 && n < N) out[n] = accumulate ? out[n] + s : s;
}

// ------------------------------------------------------------ copies -------
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void cast_kernel(int64_t n, const TI* __restrict__ x, TO* __restrict__ y) {
  const int64_t n8 = n / 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    Vec8<TI>::load(x + i * 8, v);
    Vec8<TO>::store(y + i * 8, v);
  }
  for (int64_t i = n8 * 8 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = from_f32<TO>(to_f32(x[i]));
}

template <typename T>
__global__ __launch_bounds__(256) void copy_rows_kernel(int rows, int cols, const T* __restrict__ x, int64_t ldx,
                                                        T* __restrict__ y, int64_t ldy) {
  const int ch = cols / 8;
  const int64_t total = (int64_t)rows * ch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / ch;
    const int c = (int)(i % ch);
    float v[8];
    Vec8<T>::load(x + r * ldx + c * 8, v);
    Vec8<T>::store(y + r * ldy + c * 8, v);
  }
}


// y = x * keep(seed, r*cols + c) / (1-p): the GEMM-epilogue dropout mask of an [rows, cols]
// output re-applied to its gradient (pre-LN residual branches: GPT-2 resid dropout).
template <typename T>
__global__ __launch_bounds__(256) void dropout_apply_kernel(int rows, int cols, const T* __restrict__ x, int64_t ldx,
                                                            T* __restrict__ y, int64_t ldy, Drop d) {
  const int ch = cols / 8;
  const int64_t total = (int64_t)rows * ch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / ch;
    const int c = (int)(i % ch) * 8;
    float v[8];
    Vec8<T>::load(x + r * ldx + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= d.mul((uint64_t)r * cols + c + j);
    Vec8<T>::store(y + r * ldy + c, v);
  }
}

// y[g][r][c] (+)= sum_s x[g][r][s*seg + c]   (fp32 out): e.g. the GPT-2 prefix gradient
// dP = dK[:, :10] + dV[:, :10] summed over layers (K = V = prefix).
template <typename T>
__global__ __launch_bounds__(256) void add_rows_kernel(int G, int rows, int cols, const T* __restrict__ x, int64_t gsx,
                                                       int64_t ldx, int nseg, int64_t seg, float* __restrict__ y,
                                                       int64_t gsy, int64_t ldy, int accumulate) {
  const int64_t total = (int64_t)G * rows * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % cols);
    const int64_t gr = i / cols;
    const int r = (int)(gr % rows), g = (int)(gr / rows);
    const T* xp = x + g * gsx + (int64_t)r * ldx + c;
    float acc = 0.f;
    for (int sgi = 0; sgi < nseg; ++sgi) acc += to_f32(xp[sgi * seg]);
    float* yp = y + g * gsy + (int64_t)r * ldy + c;
    *yp = accumulate ? *yp + acc : acc;
  }
}

// ------------------------------------------------------------ AdamW --------
// One pass, ADAM_U float4 groups per thread (all loads issued before the arithmetic), each
// byte touched once: nontemporal loads / stores keep the 30 B/param stream out of the way
// of L2 / MALL.  Same per-element arithmetic as adamw_kernel (the grid-stride reference
// form kept for the tail).
constexpr int ADAM_U = 4;
__global__ __launch_bounds__(256) void adamw_u_kernel(int64_t n4, f32x4* __restrict__ p, const f32x4* __restrict__ g,
                                                      f32x4* __restrict__ m, f32x4* __restrict__ v,
                                                      bf16x4* __restrict__ pb, float lr, float wd, float b1, float b2,
                                                      float eps, float bc1, float bc2) {
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const float decay = 1.f - lr * wd;
  const int64_t base = (int64_t)blockIdx.x * 256 * ADAM_U + threadIdx.x;
  f32x4 pv[ADAM_U], gv[ADAM_U], mv[ADAM_U], vv[ADAM_U];
#pragma unroll
  for (int u = 0; u < ADAM_U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n4) {
      gv[u] = __builtin_nontemporal_load(g + i);
      pv[u] = __builtin_nontemporal_load(p + i);
      mv[u] = __builtin_nontemporal_load(m + i);
      vv[u] = __builtin_nontemporal_load(v + i);
    }
  }
#pragma unroll
  for (int u = 0; u < ADAM_U; ++u) {
    const int64_t i = base + u * 256;
    if (i >= n4) break;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pv[u][k] *= decay;
      mv[u][k] = mv[u][k] + (gv[u][k] - mv[u][k]) * (1.f - b1);
      vv[u][k] = vv[u][k] * b2 + (1.f - b2) * gv[u][k] * gv[u][k];
      const float denom = sqrtf(vv[u][k]) / bc2s + eps;
      pv[u][k] = pv[u][k] - step_size * (mv[u][k] / denom);
    }
    __builtin_nontemporal_store(pv[u], p + i);
    __builtin_nontemporal_store(mv[u], m + i);
    __builtin_nontemporal_store(vv[u], v + i);
    if (pb) {
      bf16x4 o;
      o[0] = (bf16)pv[u][0]; o[1] = (bf16)pv[u][1]; o[2] = (bf16)pv[u][2]; o[3] = (bf16)pv[u][3];
      __builtin_nontemporal_store(o, pb + i);
    }
  }
}

__global__ __launch_bounds__(256) void adamw_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16* __restrict__ pb, float lr, float wd, float b1, float b2,
                                                    float eps, float bc1, float bc2) {
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const float decay = 1.f - lr * wd;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 pv = ((f32x4*)p)[i], gv = ((const f32x4*)g)[i], mv = ((f32x4*)m)[i], vv = ((f32x4*)v)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pv[k] *= decay;
      mv[k] = mv[k] + (gv[k] - mv[k]) * (1.f - b1);
      vv[k] = vv[k] * b2 + (1.f - b2) * gv[k] * gv[k];
      const float denom = sqrtf(vv[k]) / bc2s + eps;
      pv[k] = pv[k] - step_size * (mv[k] / denom);
    }
    ((f32x4*)p)[i] = pv;
    ((f32x4*)m)[i] = mv;
    ((f32x4*)v)[i] = vv;
    if (pb) {
      bf16x4 o;
      o[0] = (bf16)pv[0]; o[1] = (bf16)pv[1]; o[2] = (bf16)pv[2]; o[3] = (bf16)pv[3];
      ((bf16x4*)pb)[i] = o;
    }
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float pv = p[i] * decay, gv = g[i];
    float mv = m[i] + (gv - m[i]) * (1.f - b1);
    float vv = v[i] * b2 + (1.f - b2) * gv * gv;
    pv = pv - step_size * (mv / (sqrtf(vv) / bc2s + eps));
    p[i] = pv; m[i] = mv; v[i] = vv;
    if (pb) pb[i] = (bf16)pv;
  }
}

// ------------------------------------------------------- activation bwd ----
template <typename T>
__global__ __launch_bounds__(256) void act_bwd_kernel(int64_t n, int act, const T* __restrict__ dy,
                                                      const T* __restrict__ aux, T* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = from_f32<T>(to_f32(dy[i]) * act_grad(act, to_f32(aux[i])));
}

static int grid_for(int64_t work, int per_block = 256) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(8192, (work + per_block - 1) / per_block));
}

// ---- deferred partial-sum finishes: one launch for the finishes a layer's backward issues
// (its LayerNorm weight / bias / fused-bias sums and bias column sums: 4-9 launches of ~5 us,
// each a handful of workgroups, the rest of the chip idle).  Every queued finish keeps its
// own column blocks and the same summation order (finish_parts16), so the results are
// bit-identical to the single launches.
struct FinishDesc {
  const float* part;
  int64_t ld;
  int nparts, ncols;
  float* out;
  int accumulate;
};
constexpr int FB_MAX = 16;
struct FinishBatch {
  FinishDesc d[FB_MAX];
  int start[FB_MAX + 1];  // first column block of each finish; start[n] = the grid
  int n;
};
__global__ __launch_bounds__(1024) void finish_batch_kernel(FinishBatch fb) {
  int k = 0;
  while (k + 1 < fb.n && (int)blockIdx.x >= fb.start[k + 1]) ++k;  // (block-uniform)
  const FinishDesc d = fb.d[k];
  const int cb = (int)blockIdx.x - fb.start[k];
  const float s = finish_parts16(d.part, d.ld, d.nparts, d.ncols, cb);
  const int n = cb * 16 + threadIdx.x;
  if (threadIdx.x < 16 && n < d.ncols) d.out[n] = d.accumulate ? d.out[n] + s : s;
}
static thread_local bool t_defer = false;
static thread_local std::vector<std::pair<hipStream_t, std::vector<FinishDesc>>> t_queues;
static int flush_finishes(hipStream_t st) {
  for (auto& qe : t_queues) {
    if (qe.first != st || qe.second.empty()) continue;
    std::vector<FinishDesc>& q = qe.second;
    FinishBatch fb{};
    fb.n = (int)q.size();
    int blocks = 0;
    for (int i = 0; i < fb.n; ++i) {
      fb.d[i] = q[i];
      fb.start[i] = blocks;
      blocks += cdiv(q[i].ncols, 16);
    }
    fb.start[fb.n] = blocks;
    q.clear();
    hipLaunchKernelGGL(finish_batch_kernel, dim3(blocks), dim3(1024), 0, st, fb);
    CAPK_LAUNCH_CHECK("finish_batch_kernel");
  }
  return CAPK_OK;
}
bool finish_enqueue(const float* part, int64_t ld, int nparts, int ncols, float* out, int accumulate, hipStream_t st) {
  if (!t_defer) return false;
  std::vector<FinishDesc>* q = nullptr;
  for (auto& qe : t_queues)
    if (qe.first == st) q = &qe.second;
  if (!q) {
    t_queues.emplace_back(st, std::vector<FinishDesc>());
    q = &t_queues.back().second;
  }
  // a queued finish writing an overlapping output must land first (accumulation order), and
  // a full batch goes out
  bool clash = (int)q->size() >= FB_MAX;
  for (const FinishDesc& d : *q) clash |= out < d.out + d.ncols && d.out < out + ncols;
  if (clash) flush_finishes(st);
  q->push_back(FinishDesc{part, ld, nparts, ncols, out, accumulate});
  return true;
}

int launch_colsum_finish(int parts, int N, const float* part, float* out, int accumulate, hipStream_t st) {
  if (finish_enqueue(part, N, parts, N, out, accumulate, st)) return CAPK_OK;
  hipLaunchKernelGGL(colsum_finish_kernel, dim3(cdiv(N, 16)), dim3(1024), 0, st, parts, N, part, out, accumulate);
  CAPK_LAUNCH_CHECK("colsum_finish_kernel");
  return CAPK_OK;
}

}  // namespace capk

using namespace capk;

#define DT_DISPATCH(dtype, NAME, ...)                                        \
  if ((dtype) == CAPK_BF16) { NAME(bf16, __VA_ARGS__); }                     \
  else if ((dtype) == CAPK_F32) { NAME(float, __VA_ARGS__); }                \
  else { set_error("%s: bad dtype %d", __func__, (int)(dtype)); return CAPK_EINVAL; }

extern "C" int capk_patchify(int out_dtype, int B, int C, int H, int W, int P, const float* images, void* out,
                             void* stream) {
  CAPK_CHECK_ARG(B > 0 && C > 0 && P > 0 && H % P == 0 && W % P == 0 && P % 8 == 0, "capk_patchify: bad shape");
  const int64_t work = (int64_t)B * (H / P) * (W / P) * C * P * P / 8;
#define L(T, _) hipLaunchKernelGGL(patchify_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), B, C, H, W, P, images, (T*)out)
  DT_DISPATCH(out_dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("patchify_kernel");
  return CAPK_OK;
}

extern "C" int capk_vit_assemble(int dtype, int B, int Np, int D, const void* patch_out, const float* cls,
                                 const float* pos, void* x, void* stream) {
  CAPK_CHECK_ARG(B > 0 && Np > 0 && D % 8 == 0, "capk_vit_assemble: bad shape");
  const int64_t work = (int64_t)B * (Np + 1) * D / 8;
#define L(T, _) hipLaunchKernelGGL(vit_assemble_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), B, Np, D, (const T*)patch_out, cls, pos, (T*)x)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("vit_assemble_kernel");
  return CAPK_OK;
}

extern "C" size_t capk_colsum_workspace(int M, int N) {
  return (size_t)cdiv(M, CS_ROWS_PER_SPLIT) * N * sizeof(float);
}

extern "C" int capk_colsum(int dtype, int M, int N, const void* dy, int64_t ldy, float* db, int accumulate, void* ws,
                           size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(M > 0 && N > 0 && N % 8 == 0 && ldy % 8 == 0, "capk_colsum: N and ldy must be multiples of 8");
  const int splits = cdiv(M, CS_ROWS_PER_SPLIT);
  CAPK_CHECK_ARG(ws && ws_bytes >= (size_t)splits * N * sizeof(float), "capk_colsum: workspace too small");
  dim3 grid(cdiv(N, 512), splits);
#define L(T, _) hipLaunchKernelGGL(colsum_kernel<T>, grid, dim3(256), 0, S(stream), M, N, (const T*)dy, ldy, (float*)ws)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("colsum_kernel");
  return launch_colsum_finish(splits, N, (const float*)ws, db, accumulate, S(stream));
}

extern "C" int capk_act_bwd_colsum(int dtype, int M, int N, void* C, int64_t ldc, const void* aux, int64_t ldx,
                                   int act, float* db, int accumulate, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(M > 0 && N > 0 && N % 8 == 0 && ldc % 8 == 0 && ldx % 8 == 0 && C && aux && db,
                 "capk_act_bwd_colsum: N, ldc, ldx must be multiples of 8");
  CAPK_CHECK_ARG((act & 15) != 0, "capk_act_bwd_colsum: no activation");
  const int splits = cdiv(M, CS_ROWS_PER_SPLIT);
  CAPK_CHECK_ARG(ws && ws_bytes >= (size_t)splits * N * sizeof(float), "capk_act_bwd_colsum: workspace too small");
  dim3 grid(cdiv(N, 512), splits);
#define L(T, _)                                                                                                  \
  hipLaunchKernelGGL(act_bwd_colsum_kernel<T>, grid, dim3(256), 0, S(stream), M, N, (T*)C, ldc, (const T*)aux, ldx, \
                     act, (float*)ws)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("act_bwd_colsum_kernel");
  return launch_colsum_finish(splits, N, (const float*)ws, db, accumulate, S(stream));
}

extern "C" size_t capk_vit_assemble_bwd_workspace(int B, int Np, int D) {
  return capk_colsum_workspace(B, (Np + 1) * D);
}

extern "C" int capk_vit_assemble_bwd(int dtype, int B, int Np, int D, const void* dx, void* dpatch, float* dcls,
                                     float* dpos, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(B > 0 && Np > 0 && D % 8 == 0, "capk_vit_assemble_bwd: bad shape");
  const int64_t esz = dtype == CAPK_BF16 ? 2 : 4;
  {
    // one 2D copy: B "rows" of Np*D elements with source pitch (Np+1)*D
    hipError_t e = hipMemcpy2DAsync(dpatch, (size_t)Np * D * esz, (const char*)dx + D * esz, (size_t)(Np + 1) * D * esz,
                                    (size_t)Np * D * esz, B, hipMemcpyDeviceToDevice, S(stream));
    if (e != hipSuccess) return hip_status(e, "capk_vit_assemble_bwd memcpy2d");
  }
  int rc = capk_colsum(dtype, B, (Np + 1) * D, dx, (int64_t)(Np + 1) * D, dpos, 0, ws, ws_bytes, stream);
  if (rc) return rc;
  hipError_t e = hipMemcpyAsync(dcls, dpos, D * sizeof(float), hipMemcpyDeviceToDevice, S(stream));
  if (e != hipSuccess) return hip_status(e, "capk_vit_assemble_bwd dcls");
  return CAPK_OK;
}

extern "C" int capk_embedding_fwd(int dtype, int B, int T, int D, const int64_t* ids, const float* table,
                                  const float* pos, int pos_offset, float drop_p, uint32_t drop_seed, void* out,
                                  void* stream) {
  CAPK_CHECK_ARG(B > 0 && T > 0 && D % 8 == 0, "capk_embedding_fwd: bad shape");
  const int64_t work = (int64_t)B * T * D / 8;
#define L(T_, _) hipLaunchKernelGGL(embedding_fwd_kernel<T_>, dim3(grid_for(work)), dim3(256), 0, S(stream), B, T, D, ids, table, pos, pos_offset, (T_*)out, make_drop(drop_p, drop_seed))
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("embedding_fwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_embedding_bwd(int dtype, int B, int T, int D, const int64_t* ids, const void* dout,
                                  int padding_idx, float* dtable, float* dpos, int pos_offset, float drop_p,
                                  uint32_t drop_seed, void* stream) {
  CAPK_CHECK_ARG(B > 0 && T > 0 && D > 0, "capk_embedding_bwd: bad shape");
  const int64_t work = (int64_t)B * T * D;
#define L(T_, _) hipLaunchKernelGGL(embedding_bwd_kernel<T_>, dim3(grid_for(work)), dim3(256), 0, S(stream), B, T, D, ids, (const T_*)dout, padding_idx, dtable, dpos, pos_offset, make_drop(drop_p, drop_seed))
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("embedding_bwd_kernel");
  return CAPK_OK;
}

extern "C" size_t capk_shifted_ce_workspace(int B, int T) { return (size_t)(B * T + 4) * sizeof(float); }

static int shifted_ce_impl(const float* row_weight, int dtype, int B, int T, int V, int64_t ld, const void* logits,
                               const int64_t* targets, int ignore_index, const float* grad_scale, float* loss_out,
                               void* dlogits, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(B > 0 && T > 1 && V > 0 && ld >= V && ld % 8 == 0, "capk_shifted_ce: bad shape (ld %% 8)");
  CAPK_CHECK_ARG(ld <= (int64_t)CE_MAXCH * 8 * CE_THREADS, "capk_shifted_ce: row too long");
  CAPK_CHECK_ARG(ws && ws_bytes >= capk_shifted_ce_workspace(B, T), "capk_shifted_ce: workspace too small");
  float* cnt = (float*)ws;
  float* row_loss = loss_out ? cnt + 4 : nullptr;
  hipStream_t st = S(stream);
  hipLaunchKernelGGL(ce_count_kernel, dim3(1), dim3(1024), 0, st, B, T, targets, ignore_index, cnt);
  CAPK_LAUNCH_CHECK("ce_count_kernel");
#define L(T_, _) hipLaunchKernelGGL(ce_rows_kernel<T_>, dim3(B * T), dim3(CE_THREADS), 0, st, B, T, V, ld, (const T_*)logits, targets, ignore_index, grad_scale, cnt, row_loss, (T_*)dlogits, row_weight)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("ce_rows_kernel");
  if (loss_out) {
    hipLaunchKernelGGL(ce_finish_kernel, dim3(1), dim3(1024), 0, st, B * T, row_loss, cnt, loss_out);
    CAPK_LAUNCH_CHECK("ce_finish_kernel");
  }
  return CAPK_OK;
}

extern "C" int capk_zero_gap_rows(void* base, int64_t ld_bytes, int64_t row_bytes, int B, int rpb, int nk, int rows,
                                  void* stream) {
  CAPK_CHECK_ARG(base && B > 0 && nk > 0 && rpb >= nk && rows > 0 && row_bytes > 0 && row_bytes % 16 == 0 &&
                     ld_bytes % 16 == 0 && (uintptr_t)base % 16 == 0 && row_bytes <= ld_bytes,
                 "capk_zero_gap_rows: bad arguments");
  if (rpb == nk) return CAPK_OK;
  const int chunks = (int)(row_bytes / 16);
  const int64_t total = (int64_t)B * (rpb - nk) * chunks;
  hipLaunchKernelGGL(zero_gap_rows_kernel, dim3(grid_for(total)), dim3(256), 0, S(stream), (char*)base, ld_bytes, chunks,
                     B, rpb, nk, rows);
  CAPK_LAUNCH_CHECK("zero_gap_rows_kernel");
  return CAPK_OK;
}

extern "C" size_t capk_ce_lse_workspace(int B, int T, int64_t ld) {
  const int M = B * T;
  return (size_t)(4 + M) * sizeof(float) + (size_t)cdiv(M, CEB_ROWS) * ld * sizeof(float);
}

extern "C" int capk_ce_lse_fwd(int B, int T, int V, int64_t ld, const void* logits, const int64_t* targets,
                               int ignore_index, const float* part, int nparts, float* lse_out, float* loss_out,
                               void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(B > 0 && T > 1 && V > 0 && ld >= V && logits && targets && part && nparts > 0 && lse_out && loss_out,
                 "capk_ce_lse_fwd: bad arguments");
  const int M = B * T;  // (the forward uses only the count and the row losses: 4 + M floats)
  CAPK_CHECK_ARG(ws && ws_bytes >= (size_t)(4 + M) * sizeof(float), "capk_ce_lse_fwd: workspace too small");
  float* cnt = (float*)ws;
  float* row_loss = cnt + 4;
  hipStream_t st = S(stream);
  hipLaunchKernelGGL(ce_count_kernel, dim3(1), dim3(1024), 0, st, B, T, targets, ignore_index, cnt);
  CAPK_LAUNCH_CHECK("ce_count_kernel");
  hipLaunchKernelGGL(ce_lse_merge_kernel, dim3(cdiv(M, CEM_ROWS)), dim3(CEM_ROWS * CEM_STREAMS), 0, st, B, T, M, nparts, (const float2*)part,
                     (const bf16*)logits, ld, targets, ignore_index, lse_out, row_loss);
  CAPK_LAUNCH_CHECK("ce_lse_merge_kernel");
  hipLaunchKernelGGL(ce_finish_kernel, dim3(1), dim3(1024), 0, st, M, row_loss, cnt, loss_out);
  CAPK_LAUNCH_CHECK("ce_finish_kernel");
  return CAPK_OK;
}

extern "C" int capk_ce_lse_bwd(int dtype, int B, int T, int V, int64_t ld, const void* logits, const int64_t* targets,
                               int ignore_index, const float* lse, const float* cnt, const float* grad_scale,
                               void* dlogits, float* dbias, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(B > 0 && T > 1 && V > 0 && ld >= V && ld % 8 == 0 && logits && targets && lse && cnt && dlogits,
                 "capk_ce_lse_bwd: bad arguments");
  CAPK_CHECK_ARG(((uintptr_t)logits % 16 == 0) && ((uintptr_t)dlogits % 16 == 0), "capk_ce_lse_bwd: alignment");
  CAPK_CHECK_ARG(!dbias || (ws && ws_bytes >= capk_ce_lse_workspace(B, T, ld)), "capk_ce_lse_bwd: workspace too small");
  const int M = B * T, groups = cdiv(M, CEB_ROWS);
  float* dpart = dbias ? (float*)ws + 4 + M : nullptr;
  hipStream_t st = S(stream);
  const dim3 grid(cdiv((int)(ld / 8), 256), groups);
#define L(T_, _) hipLaunchKernelGGL(ce_lse_bwd_kernel<T_>, grid, dim3(256), 0, st, B, T, V, ld, (const T_*)logits, targets, ignore_index, lse, cnt, grad_scale, (T_*)dlogits, dpart)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("ce_lse_bwd_kernel");
  if (dbias) return launch_colsum_finish(groups, (int)ld, dpart, dbias, 0, st);
  return CAPK_OK;
}

extern "C" int capk_shifted_ce(int dtype, int B, int T, int V, int64_t ld, const void* logits,
                               const int64_t* targets, int ignore_index, const float* grad_scale, float* loss_out,
                               void* dlogits, void* ws, size_t ws_bytes, void* stream) {
  return shifted_ce_impl(nullptr, dtype, B, T, V, ld, logits, targets, ignore_index, grad_scale, loss_out, dlogits, ws,
                         ws_bytes, stream);
}

extern "C" int capk_shifted_ce_weighted(int dtype, int B, int T, int V, int64_t ld, const void* logits,
                                        const int64_t* targets, int ignore_index, const float* row_weight,
                                        const float* grad_scale, float* loss_out, void* dlogits, void* ws,
                                        size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(row_weight != nullptr, "capk_shifted_ce_weighted: row_weight");
  return shifted_ce_impl(row_weight, dtype, B, T, V, ld, logits, targets, ignore_index, grad_scale, loss_out, dlogits,
                         ws, ws_bytes, stream);
}

extern "C" int capk_cast(int in_dtype, int out_dtype, int64_t n, const void* x, void* y, void* stream) {
  CAPK_CHECK_ARG(n >= 0, "capk_cast: n");
  if (n == 0) return CAPK_OK;
  const dim3 g(grid_for(n / 8 + 1)), b(256);
  hipStream_t st = S(stream);
  if (in_dtype == CAPK_F32 && out_dtype == CAPK_BF16) hipLaunchKernelGGL((cast_kernel<float, bf16>), g, b, 0, st, n, (const float*)x, (bf16*)y);
  else if (in_dtype == CAPK_BF16 && out_dtype == CAPK_F32) hipLaunchKernelGGL((cast_kernel<bf16, float>), g, b, 0, st, n, (const bf16*)x, (float*)y);
  else if (in_dtype == CAPK_F32 && out_dtype == CAPK_F32) hipLaunchKernelGGL((cast_kernel<float, float>), g, b, 0, st, n, (const float*)x, (float*)y);
  else if (in_dtype == CAPK_BF16 && out_dtype == CAPK_BF16) hipLaunchKernelGGL((cast_kernel<bf16, bf16>), g, b, 0, st, n, (const bf16*)x, (bf16*)y);
  else { set_error("capk_cast: dtype"); return CAPK_EINVAL; }
  CAPK_LAUNCH_CHECK("cast_kernel");
  return CAPK_OK;
}

extern "C" int capk_copy_rows(int dtype, int rows, int cols, const void* x, int64_t ldx, void* y, int64_t ldy,
                              void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0, "capk_copy_rows: need multiples of 8");
  const int64_t work = (int64_t)rows * cols / 8;
#define L(T, _) hipLaunchKernelGGL(copy_rows_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), rows, cols, (const T*)x, ldx, (T*)y, ldy)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("copy_rows_kernel");
  return CAPK_OK;
}


extern "C" int capk_dropout_apply(int dtype, int rows, int cols, const void* x, int64_t ldx, float p, uint32_t seed,
                                  void* y, int64_t ldy, void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0, "capk_dropout_apply: need multiples of 8");
  const int64_t work = (int64_t)rows * cols / 8;
#define L(T, _) hipLaunchKernelGGL(dropout_apply_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), rows, cols, (const T*)x, ldx, (T*)y, ldy, make_drop(p, seed))
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("dropout_apply_kernel");
  return CAPK_OK;
}

extern "C" int capk_add_rows(int dtype, int groups, int rows, int cols, const void* x, int64_t gsx, int64_t ldx,
                             int nseg, int64_t seg_stride, float* y, int64_t gsy, int64_t ldy, int accumulate,
                             void* stream) {
  CAPK_CHECK_ARG(groups > 0 && rows > 0 && cols > 0 && nseg > 0, "capk_add_rows: sizes");
  const int64_t work = (int64_t)groups * rows * cols;
#define L(T, _) hipLaunchKernelGGL(add_rows_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), groups, rows, cols, (const T*)x, gsx, ldx, nseg, seg_stride, y, gsy, ldy, accumulate)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("add_rows_kernel");
  return CAPK_OK;
}

extern "C" int capk_adamw(int64_t n, float* param, const float* grad, float* m, float* v, void* param_bf16, float lr,
                          float weight_decay, float beta1, float beta2, float eps, float bc1, float bc2,
                          void* stream) {
  CAPK_CHECK_ARG(n >= 0 && param && grad && m && v, "capk_adamw: null");
  CAPK_CHECK_ARG((uintptr_t)param % 16 == 0 && (uintptr_t)grad % 16 == 0 && (uintptr_t)m % 16 == 0 &&
                     (uintptr_t)v % 16 == 0 && (uintptr_t)param_bf16 % 8 == 0,
                 "capk_adamw: buffers must be 16-B aligned");
  if (n == 0) return CAPK_OK;
  static const bool one_pass = [] { const char* e = getenv("CAPK_ADAMW_GRIDSTRIDE"); return !(e && e[0] == '1'); }();
  const int64_t n4 = n / 4;
  if (one_pass && n4 > 0) {
    const int64_t blocks = (n4 + 256 * ADAM_U - 1) / (256 * ADAM_U);
    CAPK_CHECK_ARG(blocks < (1ll << 31), "capk_adamw: n too large");
    hipLaunchKernelGGL(adamw_u_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream), n4, (f32x4*)param,
                       (const f32x4*)grad, (f32x4*)m, (f32x4*)v, (bf16x4*)param_bf16, lr, weight_decay, beta1, beta2,
                       eps, bc1, bc2);
    CAPK_LAUNCH_CHECK("adamw_u_kernel");
    if (n4 * 4 == n) return CAPK_OK;
    // the < 4 trailing elements: the reference kernel on the tail
    const int64_t off = n4 * 4;
    hipLaunchKernelGGL(adamw_kernel, dim3(1), dim3(64), 0, S(stream), n - off, param + off, grad + off, m + off, v + off,
                       param_bf16 ? (bf16*)param_bf16 + off : nullptr, lr, weight_decay, beta1, beta2, eps, bc1, bc2);
    CAPK_LAUNCH_CHECK("adamw_kernel");
    return CAPK_OK;
  }
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, S(stream), n, param, grad, m, v,
                     (bf16*)param_bf16, lr, weight_decay, beta1, beta2, eps, bc1, bc2);
  CAPK_LAUNCH_CHECK("adamw_kernel");
  return CAPK_OK;
}

extern "C" int capk_act_bwd(int dtype, int64_t n, int act, const void* dy, const void* aux, void* out, void* stream) {
  CAPK_CHECK_ARG(n >= 0 && dy && aux && out, "capk_act_bwd: null");
  if (n == 0) return CAPK_OK;
#define L(T, _) hipLaunchKernelGGL(act_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, S(stream), n, act, (const T*)dy, (const T*)aux, (T*)out)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("act_bwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_zero(void* ptr, size_t bytes, void* stream) {
  if (bytes == 0) return CAPK_OK;
  CAPK_CHECK_ARG(ptr, "capk_zero: null");
  hipError_t e = hipMemsetAsync(ptr, 0, bytes, S(stream));
  if (e != hipSuccess) return hip_status(e, "capk_zero");
  return CAPK_OK;
}

// Debug/test view of the dropout mask: out[i] = keep(seed, offset + i) ? 1 : 0.
__global__ void drop_mask_kernel(int64_t n, uint64_t offset, Drop d, uint8_t* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = d.mul(offset + (uint64_t)i) != 0.f;
}
extern "C" int capk_dropout_mask(int64_t n, uint64_t offset, float p, uint32_t seed, uint8_t* out, void* stream) {
  CAPK_CHECK_ARG(n >= 0 && out, "capk_dropout_mask: bad args");
  if (n == 0) return CAPK_OK;
  hipLaunchKernelGGL(drop_mask_kernel, dim3(grid_for(n)), dim3(256), 0, S(stream), n, offset, make_drop(p, seed), out);
  CAPK_LAUNCH_CHECK("drop_mask_kernel");
  return CAPK_OK;
}

extern "C" int capk_finish_defer(int on) {
  capk::t_defer = on != 0;
  return CAPK_OK;
}

extern "C" int capk_finish_flush(void* stream) { return capk::flush_finishes(S(stream)); }

namespace capk {
// ------------------------------------------------------- batched transpose --
// dst[c][r] = src[r][c] (bf16 bits) for up to TR_MAX matrices per launch: one workgroup per
// 64 x 64 tile, 16-B row loads into an LDS tile, 16-B stores of its columns.  The weight
// copies are a few MB each (HBM-bound, ~0.4 GB per training step in all).
constexpr int TR_MAX = 64;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct TrDesc {
  const uint16_t* src;
  uint16_t* dst;
  int64_t lds, ldd;
  int rows, cols, tiles_c, tile0;
};
struct TrBatch {
  TrDesc d[TR_MAX];
  int n;
};
__global__ __launch_bounds__(256) void transpose_batch_kernel(TrBatch b) {
  __shared__ __attribute__((aligned(16))) uint16_t t[64][64 + 8];
  // the matrix of this tile: binary search over the tile offsets (a linear scan is a chain of
  // up to 64 dependent argument loads per workgroup)
  int lo = 0, hi = b.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int)blockIdx.x >= b.d[mid].tile0) lo = mid;
    else hi = mid - 1;
  }
  const TrDesc d = b.d[lo];
  const int tile = (int)blockIdx.x - d.tile0;
  const int r0 = (tile / d.tiles_c) * 64, c0 = (tile % d.tiles_c) * 64;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = threadIdx.x + h * 256, r = idx >> 3, ch = idx & 7;
    if (r0 + r < d.rows && c0 + ch * 8 < d.cols) {
      const u32x4 v = *(const u32x4*)(d.src + (int64_t)(r0 + r) * d.lds + c0 + ch * 8);
      *(u32x4*)&t[r][ch * 8] = v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = threadIdx.x + h * 256, c = idx >> 3, rch = idx & 7;
    if (c0 + c < d.cols && r0 + rch * 8 < d.rows) {
      uint16_t o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = t[rch * 8 + i][c];
      u32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = ((uint32_t)o[2 * i] | ((uint32_t)o[2 * i + 1] << 16));
      *(u32x4*)(d.dst + (int64_t)(c0 + c) * d.ldd + r0 + rch * 8) = v;
    }
  }
}
}  // namespace capk

extern "C" int capk_transpose_bf16_batch(int n, const capk_transpose_desc* descs, void* stream) {
  CAPK_CHECK_ARG(n >= 0 && (n == 0 || descs), "capk_transpose_bf16_batch: null descriptors");
  for (int i0 = 0; i0 < n; i0 += capk::TR_MAX) {
    capk::TrBatch b{};
    int tiles = 0;
    b.n = std::min(capk::TR_MAX, n - i0);
    for (int k = 0; k < b.n; ++k) {
      const capk_transpose_desc& s = descs[i0 + k];
      CAPK_CHECK_ARG(s.src && s.dst && s.rows > 0 && s.cols > 0 && s.rows % 8 == 0 && s.cols % 8 == 0 &&
                         s.ld_src % 8 == 0 && s.ld_dst % 8 == 0 && s.ld_src >= s.cols && s.ld_dst >= s.rows &&
                         (uintptr_t)s.src % 16 == 0 && (uintptr_t)s.dst % 16 == 0,
                     "capk_transpose_bf16_batch: descriptor %d (rows=%d cols=%d): sizes / strides must be "
                     "multiples of 8, pointers 16-B aligned", i0 + k, s.rows, s.cols);
      const int tc = cdiv(s.cols, 64);
      b.d[k] = capk::TrDesc{(const uint16_t*)s.src, (uint16_t*)s.dst, s.ld_src, s.ld_dst, s.rows, s.cols, tc, tiles};
      tiles += cdiv(s.rows, 64) * tc;
    }
    hipLaunchKernelGGL(capk::transpose_batch_kernel, dim3(tiles), dim3(256), 0, S(stream), b);
    CAPK_LAUNCH_CHECK("transpose_batch_kernel");
  }
  return CAPK_OK;
}

extern "C" int capk_finish_flush_all(void) {
  for (auto& qe : capk::t_queues) {
    const int rc = capk::flush_finishes(qe.first);
    if (rc != CAPK_OK) return rc;
  }
  return CAPK_OK;
}
