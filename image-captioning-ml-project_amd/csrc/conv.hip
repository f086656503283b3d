// Convolutional encoder kernels (HF ResNetModel / torchvision
// resnet101 trunk).  Activations are channels-last ([B, H, W, C] rows of C, the
// token-major layout of every other capk buffer), so a 1x1 convolution is a plain
// GEMM on the activation rows and a KxK convolution is a GEMM on an im2col panel
// whose K order is (kh, kw, c) — the order of the channels-last weight storage
// [Cout, KH, KW, Cin] (zero-padded to Kp, a multiple of 64, for the MFMA tiles).
//
//   im2col / col2im   — HBM-bound gathers, 16-B vectors along C; col2im is a
//                       deterministic gather-sum (no atomics): each input pixel sums
//                       the <= KH*KW panel entries it fed.
//   BatchNorm (train) — two-pass column statistics (mean, then centred sum of
//                       squares: no E[x^2]-E[x]^2 cancellation) with per-split fp32
//                       partials reduced in a fixed order; apply fuses the affine,
//                       the residual add and the ReLU; backward reduces (dz, dz*xhat)
//                       and applies dx in a second pass.  nn.BatchNorm2d semantics
//                       (torch/nn/modules/batchnorm.py): biased variance for the
//                       normalisation, unbiased for running_var, momentum update.
//   max-pool / adaptive average pool — NHWC, first-max tie rule of aten max_pool2d.
#include "common.h"

namespace capk {

// ------------------------------------------------------------------ im2col --
// col[m, k] for m = (b, oh, ow), k = (kh*KW + kw)*C + c (k >= KH*KW*C -> 0).
// Input element (b, h, w, c) at x[b*sb + h*sh + w*sw + c*sc] (NCHW images or NHWC rows).
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void im2col_vec_kernel(int B, int H, int W, int C, int64_t sb, int64_t sh,
                                                         int64_t sw, int KH, int KW, int st, int pad, int OH, int OW,
                                                         int Kp, const TI* __restrict__ x, TO* __restrict__ col) {
  const int k8n = Kp / 8;
  const int64_t total = (int64_t)B * OH * OW * k8n;
  const int Kr = KH * KW * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / k8n;
    const int k = (int)(i % k8n) * 8;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (k < Kr) {
      const int tap = k / C, c = k % C;
      const int kh = tap / KW, kw = tap % KW;
      const int ow = (int)(m % OW);
      const int64_t t = m / OW;
      const int oh = (int)(t % OH), b = (int)(t / OH);
      const int ih = oh * st - pad + kh, iw = ow * st - pad + kw;
      if (ih >= 0 && ih < H && iw >= 0 && iw < W) Vec8<TI>::load(x + b * sb + ih * sh + iw * sw + c, v);
    }
    Vec8<TO>::store(col + m * Kp + k, v);
  }
}

// Strided / odd-C inputs (the stem: NCHW fp32 images, C = 3): eight consecutive k of one row
// per thread -- one 16-B store, the row / tap decomposition done once and then stepped (the
// per-element form spent its time in 64-bit divisions: ~1 ms for config 2's stem).
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void im2col_gather8_kernel(int B, int H, int W, int C, int64_t sb, int64_t sh,
                                                             int64_t sw, int64_t sc, int KH, int KW, int st, int pad,
                                                             int OH, int OW, int Kp, const TI* __restrict__ x,
                                                             TO* __restrict__ col) {
  const int k8n = Kp / 8;
  const int64_t total = (int64_t)B * OH * OW * k8n;
  const int Kr = KH * KW * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / k8n;
    const int k0 = (int)(i - m * k8n) * 8;
    const int ow = (int)(m % OW);
    const int64_t t = m / OW;
    const int oh = (int)(t % OH), b = (int)(t / OH);
    const int ih0 = oh * st - pad, iw0 = ow * st - pad;
    const int tap = k0 / C;
    int c = k0 - tap * C, kh = tap / KW, kw = tap - (tap / KW) * KW;
    const TI* xb = x + b * sb;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ih = ih0 + kh, iw = iw0 + kw;
      v[j] = (k0 + j < Kr && ih >= 0 && ih < H && iw >= 0 && iw < W) ? to_f32(xb[ih * sh + iw * sw + c * sc]) : 0.f;
      if (++c == C) {
        c = 0;
        if (++kw == KW) kw = 0, ++kh;
      }
    }
    Vec8<TO>::store(col + m * Kp + k0, v);
  }
}

// dx[b,h,w,c] = beta*dx + sum over the taps that read (h, w) of dcol[m(oh,ow), (kh,kw,c)]
template <typename T>
__global__ __launch_bounds__(256) void col2im_kernel(int B, int H, int W, int C, int KH, int KW, int st, int pad,
                                                     int OH, int OW, int Kp, const T* __restrict__ dcol,
                                                     T* __restrict__ dx, float beta) {
  const int c8n = C / 8;
  const int64_t total = (int64_t)B * H * W * c8n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % c8n) * 8;
    int64_t t = i / c8n;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H), b = (int)(t / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int kh = 0; kh < KH; ++kh) {
      const int th = h + pad - kh;
      if (th < 0 || th % st) continue;
      const int oh = th / st;
      if (oh >= OH) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int tw = w + pad - kw;
        if (tw < 0 || tw % st) continue;
        const int ow = tw / st;
        if (ow >= OW) continue;
        float v[8];
        Vec8<T>::load(dcol + ((int64_t)(b * OH + oh) * OW + ow) * Kp + (kh * KW + kw) * C + c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
    }
    T* p = dx + (((int64_t)b * H + h) * W + w) * C + c;
    if (beta != 0.f) {
      float o[8];
      Vec8<T>::load(p, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += beta * o[j];
    }
    Vec8<T>::store(p, acc);
  }
}

// -------------------------------------------------------------- BatchNorm ---
// Column reductions over M rows of a [M, C] (ld) buffer.  A block covers CPB =
// min(C, 2048) columns (8 per thread) and a contiguous row range of one split.
//   MODE 0: s0 = sum x
//   MODE 1: s0 = sum (x - mean)^2
//   MODE 2: dz = dy * [y > 0] (if ymask), s0 = sum dz, s1 = sum dz * (x - mean) * rstd
//   MODE 3: s0 = sum x, s1 = sum (x - mean_b)^2 about the block's own mean mean_b = s0 / n_b,
//           from sums of x - K and (x - K)^2 with the shift K = the block's first row (a sample
//           of the column, so no cancellation to speak of), merged by bn_finish_stats_kernel --
//           the forward statistics in one sweep over x
constexpr int BN_MAX_CPB = 2048;

template <typename T, int MODE>
__global__ __launch_bounds__(256) void bn_reduce_kernel(int M, int C, int rows_per_split, const T* __restrict__ x,
                                                        int64_t ldx, const T* __restrict__ dy, int64_t lddy,
                                                        const T* __restrict__ ym, int64_t ldym,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, float* __restrict__ part,
                                                        const float* __restrict__ mg, const float* __restrict__ mb) {
  constexpr int NACC = MODE >= 2 ? 2 : 1;
  __shared__ float red[NACC][256 * 8];
  const int cpb = C < BN_MAX_CPB ? C : BN_MAX_CPB;
  const int tpr = cpb / 8, rg = 256 / tpr;
  const int tid = threadIdx.x;
  const int lc = tid % tpr, r0 = tid / tpr;
  const int c = blockIdx.x * cpb + lc * 8;
  const int m0 = blockIdx.y * rows_per_split, m1 = min(M, m0 + rows_per_split);
  float a0[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8], rs[8];
  if (r0 < rg) {
    if (MODE == 3) Vec8<T>::load(x + (int64_t)m0 * ldx + c, mu);  // the shift K
    if (MODE == 1 || MODE == 2) Vec8<float>::load(mean + c, mu);
    if (MODE == 2) Vec8<float>::load(rstd + c, rs);
    float mgv[8], mbv[8];
    if (MODE == 2 && mb) Vec8<float>::load(mg + c, mgv), Vec8<float>::load(mb + c, mbv);
    for (int m = m0 + r0; m < m1; m += rg) {
      float v[8];
      Vec8<T>::load(x + (int64_t)m * ldx + c, v);
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a0[j] += v[j];
      } else if (MODE == 3) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = v[j] - mu[j]; a0[j] += d; a1[j] += d * d; }
      } else if (MODE == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = v[j] - mu[j]; a0[j] += d * d; }
      } else {
        float g[8];
        Vec8<T>::load(dy + (int64_t)m * lddy + c, g);
        if (ym) {
          float y[8];
          Vec8<T>::load(ym + (int64_t)m * ldym + c, y);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = y[j] > 0.f ? g[j] : 0.f;
        } else if (mb) {  // ReLU mask of this BatchNorm's own output, recomputed from x
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = (v[j] - mu[j]) * rs[j] * mgv[j] + mbv[j] > 0.f ? g[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a0[j] += g[j];
          a1[j] += g[j] * (v[j] - mu[j]) * rs[j];
        }
      }
    }
  }
  // fixed-order combine of the rg row groups
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][tid * 8 + j] = a0[j];
    if (MODE >= 2) red[NACC - 1][tid * 8 + j] = a1[j];
  }
  __syncthreads();
  for (int e = tid; e < cpb; e += 256) {
    const int l = e / 8, j = e % 8;
    float sq[NACC];
#pragma unroll
    for (int q = 0; q < NACC; ++q) {
      float s = 0.f;
      for (int r = 0; r < rg; ++r) s += red[q][(r * tpr + l) * 8 + j];
      sq[q] = s;
    }
    if constexpr (MODE == 3) {  // shifted sums -> (sum x, M2 about the block mean)
      const float K = to_f32(x[(int64_t)m0 * ldx + blockIdx.x * cpb + e]), nb = (float)(m1 - m0);
      const float S = sq[0], Q = sq[1];
      sq[0] = nb * K + S;
      sq[1] = fmaxf(0.f, Q - S * (S / nb));
    }
#pragma unroll
    for (int q = 0; q < NACC; ++q) part[((int64_t)blockIdx.y * NACC + q) * C + blockIdx.x * cpb + e] = sq[q];
  }
}

// MODE 0: mean = s/M.  MODE 1: var = s/M, rstd = 1/sqrt(var+eps), running stats.
// MODE 2: dbeta = s0, dgamma = s1 -> out0/out1 (batch values for the apply pass) and
//         (+)= into the parameter gradients.
// Block = 16 columns x 64 split phases (1024 threads, finish_parts16 of common.h): each
// thread sums every 64th split partial of its column with four loads in flight, then an
// LDS reduction over the phases -- the partial matrix is read in about one memory round
// trip.  (Round 2 before: 64 columns x 16 groups with one load in flight, ~25 us per call
// x 3 calls per BatchNorm on config 2; one thread per column before that, ~300 us.)
constexpr int BNF_COLS = 16;
template <int MODE>
__global__ __launch_bounds__(1024) void bn_finish_kernel(int M, int C, int splits, const float* __restrict__ part,
                                                         float eps, float momentum, float* __restrict__ out0,
                                                         float* __restrict__ out1, float* __restrict__ run_mean,
                                                         float* __restrict__ run_var, const float* __restrict__ mean,
                                                         float* __restrict__ g0, float* __restrict__ g1,
                                                         int accumulate, int64_t* __restrict__ nbt) {
  constexpr int NACC = MODE == 2 ? 2 : 1;
  float s0 = finish_parts16(part, (int64_t)NACC * C, splits, C), s1 = 0.f;
  if (MODE == 2) {
    __syncthreads();  // finish_parts16's LDS image is reused
    s1 = finish_parts16(part + C, (int64_t)NACC * C, splits, C);
  }
  const int c = blockIdx.x * BNF_COLS + threadIdx.x;
  if (MODE == 1 && nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
  if (threadIdx.x >= BNF_COLS || c >= C) return;
  if (MODE == 0) {
    out0[c] = s0 / (float)M;
  } else if (MODE == 1) {
    const float var = s0 / (float)M;
    out1[c] = 1.0f / sqrtf(var + eps);
    if (run_mean) run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean[c];
    if (run_var) {
      const float unb = M > 1 ? s0 / (float)(M - 1) : var;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
    }
  } else {
    out0[c] = s0;
    out1[c] = s1;
    if (g0) g0[c] = accumulate ? g0[c] + s1 : s1;  // dgamma
    if (g1) g1[c] = accumulate ? g1[c] + s0 : s0;  // dbeta
  }
}

// Forward statistics from MODE-3 partials (s0_b = sum x, M2_b over n_b = min(rps, M - b*rps)
// rows), one sweep: with K = split 0's mean, M*var = sum_b [M2_b + n_b (s0_b/n_b - K)^2]
// - M (mean - K)^2 (exact; K within a few sigma / sqrt(n_0) of the mean, so nothing cancels);
// rstd, the running statistics and num_batches_tracked (+1, block 0) as nn.BatchNorm2d's
// training forward.  16 columns x 64 split phases per block as finish_parts16.
__global__ __launch_bounds__(1024) void bn_finish_stats_kernel(int M, int C, int splits, int rps,
                                                               const float* __restrict__ part, float eps,
                                                               float momentum, float* __restrict__ mean,
                                                               float* __restrict__ rstd, float* __restrict__ run_mean,
                                                               float* __restrict__ run_var, int64_t* __restrict__ nbt) {
  __shared__ float red_s[64][BNF_COLS + 1], red_q[64][BNF_COLS + 1];
  const int cc = threadIdx.x & 15, ph = threadIdx.x >> 4, i = blockIdx.x * BNF_COLS + cc;
  const int64_t ld = 2 * (int64_t)C;
  float K = 0.f, S0 = 0.f, S1 = 0.f, Q0 = 0.f, Q1 = 0.f;
  if (i < C) {
    K = part[i] / (float)min(rps, M);
    int b = ph;
    for (; b + 64 < splits; b += 128) {  // two parts in flight
      const float na = (float)min(rps, M - b * rps), nb = (float)min(rps, M - (b + 64) * rps);
      const float sa = part[b * ld + i], ma = part[b * ld + C + i];
      const float sb = part[(b + 64) * ld + i], mb = part[(b + 64) * ld + C + i];
      const float da = sa / na - K, db = sb / nb - K;
      S0 += sa, S1 += sb;
      Q0 += ma + na * da * da;
      Q1 += mb + nb * db * db;
    }
    if (b < splits) {
      const float na = (float)min(rps, M - b * rps), sa = part[b * ld + i];
      const float da = sa / na - K;
      S0 += sa;
      Q0 += part[b * ld + C + i] + na * da * da;
    }
  }
  red_s[ph][cc] = S0 + S1;
  red_q[ph][cc] = Q0 + Q1;
  __syncthreads();
  if (threadIdx.x < 64) {  // 4 lanes per column, 16 phases each, then two shuffles
    const int q = threadIdx.x >> 4;
    float ts = 0.f, tq = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) ts += red_s[q * 16 + p][cc], tq += red_q[q * 16 + p][cc];
    ts += __shfl_xor(ts, 16, 64);
    ts += __shfl_xor(ts, 32, 64);
    tq += __shfl_xor(tq, 16, 64);
    tq += __shfl_xor(tq, 32, 64);
    if (threadIdx.x < BNF_COLS && i < C) {
      const float mu = ts / (float)M, dm = mu - K;
      const float m2 = fmaxf(0.f, tq - (float)M * dm * dm), var = m2 / (float)M;
      mean[i] = mu;
      rstd[i] = 1.0f / sqrtf(var + eps);
      if (run_mean) run_mean[i] = (1.f - momentum) * run_mean[i] + momentum * mu;
      if (run_var) run_var[i] = (1.f - momentum) * run_var[i] + momentum * (M > 1 ? m2 / (float)(M - 1) : var);
    }
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
}

__global__ void bn_eval_kernel(int C, const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                               float* __restrict__ mean, float* __restrict__ rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  rstd[c] = 1.0f / sqrtf(rv[c] + eps);
}

// y = act((x - mean) * rstd * gamma + beta + residual)
template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(int M, int C, const T* __restrict__ x, int64_t ldx,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       const T* __restrict__ res, int64_t ldr, int relu,
                                                       T* __restrict__ y, int64_t ldy) {
  const int c8n = C / 8;
  const int64_t total = (int64_t)M * c8n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / c8n;
    const int c = (int)(i % c8n) * 8;
    float v[8], mu[8], rs[8], g[8], b[8];
    Vec8<T>::load(x + m * ldx + c, v);
    Vec8<float>::load(mean + c, mu);
    Vec8<float>::load(rstd + c, rs);
    Vec8<float>::load(gamma + c, g);
    Vec8<float>::load(beta + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (v[j] - mu[j]) * rs[j] * g[j] + b[j];
    if (res) {
      float r[8];
      Vec8<T>::load(res + m * ldr + c, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : 0.f;
    }
    Vec8<T>::store(y + m * ldy + c, v);
  }
}

// dx = beta_acc*dx + gamma*rstd*(dz - dbeta/M - xhat*dgamma/M); dz = dy*[y>0]; dz_out = dz
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(int M, int C, const T* __restrict__ dy, int64_t lddy,
                                                           const T* __restrict__ ym, int64_t ldym,
                                                           const T* __restrict__ x, int64_t ldx,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ sdb, const float* __restrict__ sdg,
                                                           T* __restrict__ dx, int64_t lddx, float beta_acc,
                                                           T* __restrict__ dz_out, int64_t lddz, int batch_stats,
                                                           const float* __restrict__ mb) {
  const int c8n = C / 8;
  const int64_t total = (int64_t)M * c8n;
  const float invM = 1.0f / (float)M;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / c8n;
    const int c = (int)(i % c8n) * 8;
    float g[8], v[8], mu[8], rs[8], ga[8], db[8], dg[8];
    Vec8<T>::load(dy + m * lddy + c, g);
    const bool need_x = dx || mb;
    if (need_x) {
      Vec8<T>::load(x + m * ldx + c, v);
      Vec8<float>::load(mean + c, mu);
      Vec8<float>::load(rstd + c, rs);
      Vec8<float>::load(gamma + c, ga);
    }
    if (ym) {
      float y[8];
      Vec8<T>::load(ym + m * ldym + c, y);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = y[j] > 0.f ? g[j] : 0.f;
    } else if (mb) {  // ReLU mask of this BatchNorm's own output (bn_apply's expression), from x
      float bb[8];
      Vec8<float>::load(mb + c, bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = (v[j] - mu[j]) * rs[j] * ga[j] + bb[j] > 0.f ? g[j] : 0.f;
    }
    if (dz_out) Vec8<T>::store(dz_out + m * lddz + c, g);
    if (!dx) continue;
    Vec8<float>::load(sdb + c, db);
    Vec8<float>::load(sdg + c, dg);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (v[j] - mu[j]) * rs[j];
      o[j] = batch_stats ? ga[j] * rs[j] * (g[j] - db[j] * invM - xh * dg[j] * invM) : ga[j] * rs[j] * g[j];
    }
    if (beta_acc != 0.f) {
      float p[8];
      Vec8<T>::load(dx + m * lddx + c, p);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += beta_acc * p[j];
    }
    Vec8<T>::store(dx + m * lddx + c, o);
  }
}

// ----------------------------------------------------------------- pooling --
// max-pool (KxK, stride s, pad p, -inf padding); idx[b,oh,ow,c] = window offset of the
// first maximum in (kh, kw) scan order (aten max_pool2d: `val > max || isnan(val)`).
template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(int B, int H, int W, int C, int K, int st, int pad, int OH,
                                                          int OW, const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ idx) {
  const int c8n = C / 8;
  const int64_t total = (int64_t)B * OH * OW * c8n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % c8n) * 8;
    int64_t t = i / c8n;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH), b = (int)(t / OH);
    float mx[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mx[j] = -INFINITY; am[j] = 0; }
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh * st - pad + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int iw = ow * st - pad + kw;
        if (iw < 0 || iw >= W) continue;
        float v[8];
        Vec8<T>::load(x + (((int64_t)b * H + ih) * W + iw) * C + c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[j] > mx[j] || isnan(v[j])) { mx[j] = v[j]; am[j] = kh * K + kw; }
      }
    }
    const int64_t o = (((int64_t)b * OH + oh) * OW + ow) * C + c;
    Vec8<T>::store(y + o, mx);
#pragma unroll
    for (int j = 0; j < 8; ++j) idx[o + j] = (uint8_t)am[j];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(int B, int H, int W, int C, int K, int st, int pad, int OH,
                                                          int OW, const T* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx, T* __restrict__ dx) {
  const int c8n = C / 8;
  const int64_t total = (int64_t)B * H * W * c8n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % c8n) * 8;
    int64_t t = i / c8n;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H), b = (int)(t / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int kh = 0; kh < K; ++kh) {
      const int th = h + pad - kh;
      if (th < 0 || th % st) continue;
      const int oh = th / st;
      if (oh >= OH) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int tw = w + pad - kw;
        if (tw < 0 || tw % st) continue;
        const int ow = tw / st;
        if (ow >= OW) continue;
        const int64_t o = (((int64_t)b * OH + oh) * OW + ow) * C + c;
        float g[8];
        Vec8<T>::load(dy + o, g);
        const int want = kh * K + kw;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (idx[o + j] == want) acc[j] += g[j];
      }
    }
    Vec8<T>::store(dx + (((int64_t)b * H + h) * W + w) * C + c, acc);
  }
}

// adaptive average pool (aten adaptive_avg_pool2d windows: [floor(o*I/O), ceil((o+1)*I/O)))
__device__ __forceinline__ int ap_start(int o, int I, int O) { return (int)(((int64_t)o * I) / O); }
__device__ __forceinline__ int ap_end(int o, int I, int O) { return (int)(((int64_t)(o + 1) * I + O - 1) / O); }

template <typename T>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(int B, int H, int W, int C, int OH, int OW,
                                                          const T* __restrict__ x, T* __restrict__ y, int64_t ldy) {
  const int c8n = C / 8;
  const int64_t total = (int64_t)B * OH * OW * c8n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % c8n) * 8;
    int64_t t = i / c8n;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH), b = (int)(t / OH);
    const int h0 = ap_start(oh, H, OH), h1 = ap_end(oh, H, OH);
    const int w0 = ap_start(ow, W, OW), w1 = ap_end(ow, W, OW);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) {
        float v[8];
        Vec8<T>::load(x + (((int64_t)b * H + h) * W + w) * C + c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
    const float inv = 1.0f / (float)((h1 - h0) * (w1 - w0));
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= inv;
    Vec8<T>::store(y + ((int64_t)b * OH * OW + oh * OW + ow) * ldy + c, acc);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(int B, int H, int W, int C, int OH, int OW,
                                                          const T* __restrict__ dy, int64_t lddy, T* __restrict__ dx,
                                                          float beta) {
  const int c8n = C / 8;
  const int64_t total = (int64_t)B * H * W * c8n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % c8n) * 8;
    int64_t t = i / c8n;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H), b = (int)(t / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // output windows containing h: oh with start(oh) <= h < end(oh)
    for (int oh = 0; oh < OH; ++oh) {
      const int h0 = ap_start(oh, H, OH), h1 = ap_end(oh, H, OH);
      if (h < h0 || h >= h1) continue;
      for (int ow = 0; ow < OW; ++ow) {
        const int w0 = ap_start(ow, W, OW), w1 = ap_end(ow, W, OW);
        if (w < w0 || w >= w1) continue;
        float g[8];
        Vec8<T>::load(dy + ((int64_t)b * OH * OW + oh * OW + ow) * lddy + c, g);
        const float inv = 1.0f / (float)((h1 - h0) * (w1 - w0));
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += g[j] * inv;
      }
    }
    T* p = dx + (((int64_t)b * H + h) * W + w) * C + c;
    if (beta != 0.f) {
      float o[8];
      Vec8<T>::load(p, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += beta * o[j];
    }
    Vec8<T>::store(p, acc);
  }
}

static int grid_for(int64_t work) { return (int)std::min<int64_t>(8192, std::max<int64_t>(1, (work + 255) / 256)); }

// BatchNorm split geometry: blocks of CPB columns x rows_per_split rows, ~2048 blocks.
struct BnGeom {
  int cpb, rg, col_blocks, splits, rps;
};
static BnGeom bn_geom(int M, int C) {
  BnGeom g;
  g.cpb = C < BN_MAX_CPB ? C : BN_MAX_CPB;
  g.rg = 256 / (g.cpb / 8);
  g.col_blocks = C / g.cpb;
  const int want = std::max(1, 2048 / g.col_blocks);
  int rps = cdiv(M, want);
  rps = std::max(rps, 4 * g.rg);
  rps = cdiv(rps, g.rg) * g.rg;
  g.rps = rps;
  g.splits = cdiv(M, rps);
  return g;
}
static bool bn_shape_ok(int C) { return C % 8 == 0 && (C <= BN_MAX_CPB || C % BN_MAX_CPB == 0); }

}  // namespace capk

using namespace capk;

#define DT_DISPATCH(dtype, NAME, ...)                                        \
  if ((dtype) == CAPK_BF16) { NAME(bf16, __VA_ARGS__); }                     \
  else if ((dtype) == CAPK_F32) { NAME(float, __VA_ARGS__); }                \
  else { set_error("%s: bad dtype %d", __func__, (int)(dtype)); return CAPK_EINVAL; }

extern "C" int capk_im2col(int in_dtype, int out_dtype, int B, int H, int W, int C, int64_t sb, int64_t sh,
                           int64_t sw, int64_t sc, int KH, int KW, int stride, int pad, int OH, int OW, int Kp,
                           const void* x, void* col, void* stream) {
  CAPK_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0 && KH > 0 && KW > 0 && stride > 0 && OH > 0 && OW > 0,
                 "capk_im2col: bad shape");
  CAPK_CHECK_ARG(Kp >= KH * KW * C && Kp % 8 == 0, "capk_im2col: Kp=%d must be >= KH*KW*C and a multiple of 8", Kp);
  CAPK_CHECK_ARG(OH == (H + 2 * pad - KH) / stride + 1 && OW == (W + 2 * pad - KW) / stride + 1,
                 "capk_im2col: OH/OW inconsistent with the convolution geometry");
  const bool vec = sc == 1 && C % 8 == 0 && sb % 8 == 0 && sh % 8 == 0 && sw % 8 == 0;
  hipStream_t st = S(stream);
  const int64_t M = (int64_t)B * OH * OW;
#define GO(TI, TO)                                                                                                 \
  do {                                                                                                             \
    if (vec)                                                                                                       \
      hipLaunchKernelGGL((im2col_vec_kernel<TI, TO>), dim3(grid_for(M * Kp / 8)), dim3(256), 0, st, B, H, W, C, sb, \
                         sh, sw, KH, KW, stride, pad, OH, OW, Kp, (const TI*)x, (TO*)col);                         \
    else                                                                                                           \
      hipLaunchKernelGGL((im2col_gather8_kernel<TI, TO>), dim3(grid_for(M * Kp / 8)), dim3(256), 0, st, B, H, W, C, \
                         sb, sh, sw, sc, KH, KW, stride, pad, OH, OW, Kp, (const TI*)x, (TO*)col);               \
  } while (0)
  if (in_dtype == CAPK_F32 && out_dtype == CAPK_F32) GO(float, float);
  else if (in_dtype == CAPK_F32 && out_dtype == CAPK_BF16) GO(float, bf16);
  else if (in_dtype == CAPK_BF16 && out_dtype == CAPK_BF16) GO(bf16, bf16);
  else CAPK_CHECK_ARG(false, "capk_im2col: unsupported dtype pair %d -> %d", in_dtype, out_dtype);
#undef GO
  CAPK_LAUNCH_CHECK("im2col_kernel");
  return CAPK_OK;
}

extern "C" int capk_col2im(int dtype, int B, int H, int W, int C, int KH, int KW, int stride, int pad, int OH, int OW,
                           int Kp, const void* dcol, void* dx, float beta, void* stream) {
  CAPK_CHECK_ARG(B > 0 && C % 8 == 0 && Kp % 8 == 0 && Kp >= KH * KW * C, "capk_col2im: bad shape (C %% 8 == 0)");
  CAPK_CHECK_ARG(OH == (H + 2 * pad - KH) / stride + 1 && OW == (W + 2 * pad - KW) / stride + 1,
                 "capk_col2im: OH/OW inconsistent with the convolution geometry");
  const int64_t work = (int64_t)B * H * W * C / 8;
#define L(T, _)                                                                                              \
  hipLaunchKernelGGL(col2im_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), B, H, W, C, KH, KW, \
                     stride, pad, OH, OW, Kp, (const T*)dcol, (T*)dx, beta)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("col2im_kernel");
  return CAPK_OK;
}

extern "C" size_t capk_bn_workspace(int M, int C) {
  if (M <= 0 || C <= 0 || !bn_shape_ok(C)) return 0;
  const BnGeom g = bn_geom(M, C);
  return (size_t)g.splits * 2 * C * sizeof(float) + 2 * (size_t)C * sizeof(float);
}

extern "C" int capk_bn_stats(int dtype, int M, int C, const void* x, int64_t ldx, float eps, float momentum,
                             float* mean, float* rstd, float* running_mean, float* running_var,
                             int64_t* num_batches_tracked, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(M > 0 && bn_shape_ok(C) && ldx % 8 == 0, "capk_bn_stats: bad shape M=%d C=%d", M, C);
  CAPK_CHECK_ARG(ws && ws_bytes >= capk_bn_workspace(M, C), "capk_bn_stats: workspace too small");
  const BnGeom g = bn_geom(M, C);
  float* part = (float*)ws;
  hipStream_t st = S(stream);
  dim3 grid(g.col_blocks, g.splits);
#define L(T, MODE)                                                                                                \
  hipLaunchKernelGGL((bn_reduce_kernel<T, MODE>), grid, dim3(256), 0, st, M, C, g.rps, (const T*)x, ldx,         \
                     (const T*)nullptr, (int64_t)0, (const T*)nullptr, (int64_t)0, (const float*)mean, (const float*)rstd, part, \
                     (const float*)nullptr, (const float*)nullptr)
  // one sweep (shifted per-block sums, merged exactly) unless CAPK_BN_TWOPASS=1 (the global two-pass A/B)
  static const bool two_pass = [] {
    const char* v = getenv("CAPK_BN_TWOPASS");
    return v && v[0] == '1';
  }();
  if (!two_pass) {
    DT_DISPATCH(dtype, L, 3)
    CAPK_LAUNCH_CHECK("bn_reduce_kernel<3>");
    hipLaunchKernelGGL(bn_finish_stats_kernel, dim3(cdiv(C, BNF_COLS)), dim3(1024), 0, st, M, C, g.splits, g.rps,
                       (const float*)part, eps, momentum, mean, rstd, running_mean, running_var, num_batches_tracked);
    CAPK_LAUNCH_CHECK("bn_finish_stats_kernel");
    return CAPK_OK;
  }
  DT_DISPATCH(dtype, L, 0)
  CAPK_LAUNCH_CHECK("bn_reduce_kernel<0>");
  hipLaunchKernelGGL(bn_finish_kernel<0>, dim3(cdiv(C, BNF_COLS)), dim3(1024), 0, st, M, C, g.splits, (const float*)part,
                     eps, momentum, mean, rstd, (float*)nullptr, (float*)nullptr, (const float*)nullptr,
                     (float*)nullptr, (float*)nullptr, 0, (int64_t*)nullptr);
  DT_DISPATCH(dtype, L, 1)
  CAPK_LAUNCH_CHECK("bn_reduce_kernel<1>");
#undef L
  hipLaunchKernelGGL(bn_finish_kernel<1>, dim3(cdiv(C, BNF_COLS)), dim3(1024), 0, st, M, C, g.splits, (const float*)part,
                     eps, momentum, mean, rstd, running_mean, running_var, (const float*)mean, (float*)nullptr,
                     (float*)nullptr, 0, num_batches_tracked);
  CAPK_LAUNCH_CHECK("bn_finish_kernel");
  return CAPK_OK;
}

extern "C" int capk_bn_eval_stats(int C, const float* running_mean, const float* running_var, float eps, float* mean,
                                  float* rstd, void* stream) {
  CAPK_CHECK_ARG(C > 0 && running_mean && running_var, "capk_bn_eval_stats: bad args");
  hipLaunchKernelGGL(bn_eval_kernel, dim3(cdiv(C, 256)), dim3(256), 0, S(stream), C, running_mean, running_var, eps,
                     mean, rstd);
  CAPK_LAUNCH_CHECK("bn_eval_kernel");
  return CAPK_OK;
}

extern "C" int capk_bn_apply(int dtype, int M, int C, const void* x, int64_t ldx, const float* mean, const float* rstd,
                             const float* gamma, const float* beta, const void* residual, int64_t ldr, int relu,
                             void* y, int64_t ldy, void* stream) {
  CAPK_CHECK_ARG(M > 0 && C % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && (!residual || ldr % 8 == 0),
                 "capk_bn_apply: bad shape");
  const int64_t work = (int64_t)M * C / 8;
#define L(T, _)                                                                                                   \
  hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), M, C, (const T*)x, ldx, \
                     mean, rstd, gamma, beta, (const T*)residual, ldr, relu, (T*)y, ldy)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("bn_apply_kernel");
  return CAPK_OK;
}

extern "C" int capk_bn_bwd(int dtype, int M, int C, const void* dy, int64_t lddy, const void* y_mask, int64_t ldym,
                           const void* x, int64_t ldx, const float* mean, const float* rstd, const float* gamma,
                           const float* relu_beta, float* dgamma, float* dbeta, int accumulate, void* dx,
                           int64_t lddx, float beta_acc, void* dz_out, int64_t lddz, int batch_stats, void* ws,
                           size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(!(y_mask && relu_beta), "capk_bn_bwd: y_mask and relu_beta are exclusive");
  CAPK_CHECK_ARG(M > 0 && bn_shape_ok(C) && lddy % 8 == 0 && ldx % 8 == 0, "capk_bn_bwd: bad shape M=%d C=%d", M, C);
  CAPK_CHECK_ARG(ws && ws_bytes >= capk_bn_workspace(M, C), "capk_bn_bwd: workspace too small");
  const BnGeom g = bn_geom(M, C);
  float* part = (float*)ws;
  float* sdb = part + (size_t)g.splits * 2 * C;
  float* sdg = sdb + C;
  hipStream_t st = S(stream);
  dim3 grid(g.col_blocks, g.splits);
#define L(T, _)                                                                                                   \
  hipLaunchKernelGGL((bn_reduce_kernel<T, 2>), grid, dim3(256), 0, st, M, C, g.rps, (const T*)x, ldx, (const T*)dy, \
                     lddy, (const T*)y_mask, ldym, mean, rstd, part, relu_beta ? gamma : nullptr, relu_beta)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("bn_reduce_kernel<2>");
  hipLaunchKernelGGL(bn_finish_kernel<2>, dim3(cdiv(C, BNF_COLS)), dim3(1024), 0, st, M, C, g.splits, (const float*)part,
                     0.f, 0.f, sdb, sdg, (float*)nullptr, (float*)nullptr, (const float*)nullptr, dgamma, dbeta,
                     accumulate, (int64_t*)nullptr);
  CAPK_LAUNCH_CHECK("bn_finish_kernel<2>");
  if (dx || dz_out) {
    const int64_t work = (int64_t)M * C / 8;
#define L(T, _)                                                                                                      \
  hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(grid_for(work)), dim3(256), 0, st, M, C, (const T*)dy, lddy,     \
                     (const T*)y_mask, ldym, (const T*)x, ldx, mean, rstd, gamma, (const float*)sdb,                \
                     (const float*)sdg, (T*)dx, lddx, beta_acc, (T*)dz_out, lddz, batch_stats, relu_beta)
    DT_DISPATCH(dtype, L, 0)
#undef L
    CAPK_LAUNCH_CHECK("bn_bwd_apply_kernel");
  }
  return CAPK_OK;
}

extern "C" int capk_maxpool_fwd(int dtype, int B, int H, int W, int C, int K, int stride, int pad, int OH, int OW,
                                const void* x, void* y, uint8_t* idx, void* stream) {
  CAPK_CHECK_ARG(B > 0 && C % 8 == 0 && K > 0 && K * K <= 255 && stride > 0, "capk_maxpool_fwd: bad shape");
  CAPK_CHECK_ARG(OH == (H + 2 * pad - K) / stride + 1 && OW == (W + 2 * pad - K) / stride + 1,
                 "capk_maxpool_fwd: OH/OW inconsistent");
  const int64_t work = (int64_t)B * OH * OW * C / 8;
#define L(T, _)                                                                                               \
  hipLaunchKernelGGL(maxpool_fwd_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), B, H, W, C, K,    \
                     stride, pad, OH, OW, (const T*)x, (T*)y, idx)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("maxpool_fwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_maxpool_bwd(int dtype, int B, int H, int W, int C, int K, int stride, int pad, int OH, int OW,
                                const void* dy, const uint8_t* idx, void* dx, void* stream) {
  CAPK_CHECK_ARG(B > 0 && C % 8 == 0 && K > 0 && stride > 0, "capk_maxpool_bwd: bad shape");
  CAPK_CHECK_ARG(OH == (H + 2 * pad - K) / stride + 1 && OW == (W + 2 * pad - K) / stride + 1,
                 "capk_maxpool_bwd: OH/OW inconsistent");
  const int64_t work = (int64_t)B * H * W * C / 8;
#define L(T, _)                                                                                              \
  hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), B, H, W, C, K,   \
                     stride, pad, OH, OW, (const T*)dy, idx, (T*)dx)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("maxpool_bwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_avgpool_fwd(int dtype, int B, int H, int W, int C, int OH, int OW, const void* x, void* y,
                                int64_t ldy, void* stream) {
  CAPK_CHECK_ARG(B > 0 && C % 8 == 0 && OH > 0 && OW > 0 && ldy % 8 == 0 && ldy >= C, "capk_avgpool_fwd: bad shape");
  const int64_t work = (int64_t)B * OH * OW * C / 8;
#define L(T, _)                                                                                               \
  hipLaunchKernelGGL(avgpool_fwd_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), B, H, W, C, OH,   \
                     OW, (const T*)x, (T*)y, ldy)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("avgpool_fwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_avgpool_bwd(int dtype, int B, int H, int W, int C, int OH, int OW, const void* dy, int64_t lddy,
                                void* dx, float beta, void* stream) {
  CAPK_CHECK_ARG(B > 0 && C % 8 == 0 && OH > 0 && OW > 0 && lddy % 8 == 0, "capk_avgpool_bwd: bad shape");
  const int64_t work = (int64_t)B * H * W * C / 8;
#define L(T, _)                                                                                               \
  hipLaunchKernelGGL(avgpool_bwd_kernel<T>, dim3(grid_for(work)), dim3(256), 0, S(stream), B, H, W, C, OH,   \
                     OW, (const T*)dy, lddy, (T*)dx, beta)
  DT_DISPATCH(dtype, L, 0)
#undef L
  CAPK_LAUNCH_CHECK("avgpool_bwd_kernel");
  return CAPK_OK;
}
