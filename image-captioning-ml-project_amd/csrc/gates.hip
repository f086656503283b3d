// Elementwise / per-row gate kernels of the attention modules.
//
//   ew_mul              out = a * b                      AoA info * gate (attention.py:354)
//   tanh_gate_fwd/bwd   out = g * tanh(c), c fp32         adaptive visual sentinel
//                                                         sigmoid(W[q;h]) * tanh(c) (258-262)
//   gate_mix_fwd/bwd    beta = sigmoid(w_a . [ctx; s] + b_a); out = beta ctx + (1-beta) s
//                       (attention.py:279-285) — the 2D->1 projection is a per-row dot
//                       product here instead of an N=1 GEMM; its weight gradient is
//                       accumulated over decode steps with fp32 atomics.
//   attn_probs_mean     mean over heads of softmax(q k^T * scale) rebuilt from the saved
//                       log-sum-exp: the head-averaged weights MultiHeadAttention returns
//                       (attention.py:207-210).
#include "common.h"

namespace capk {

template <typename T>
__global__ __launch_bounds__(256) void ew_mul_kernel(int rows, int cols, const T* __restrict__ a, int64_t lda,
                                                     const T* __restrict__ b, int64_t ldb, T* __restrict__ out,
                                                     int64_t ldo) {
  const int64_t n = (int64_t)rows * cols;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cols;
    const int c = (int)(e % cols);
    out[r * ldo + c] = from_f32<T>(to_f32(a[r * lda + c]) * to_f32(b[r * ldb + c]));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void tanh_gate_fwd_kernel(int rows, int cols, const float* __restrict__ c, int64_t ldc,
                                                            const T* __restrict__ g, int64_t ldg, T* __restrict__ out,
                                                            int64_t ldo) {
  const int64_t n = (int64_t)rows * cols;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cols;
    const int j = (int)(e % cols);
    out[r * ldo + j] = from_f32<T>(to_f32(g[r * ldg + j]) * tanhf(c[r * ldc + j]));
  }
}

// dg = dout * tanh(c);  dc += dout * g * (1 - tanh(c)^2)
template <typename T>
__global__ __launch_bounds__(256) void tanh_gate_bwd_kernel(int rows, int cols, const float* __restrict__ c, int64_t ldc,
                                                            const T* __restrict__ g, int64_t ldg,
                                                            const T* __restrict__ dout, int64_t lddo,
                                                            T* __restrict__ dg, int64_t lddg, float* __restrict__ dc,
                                                            int64_t lddc) {
  const int64_t n = (int64_t)rows * cols;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cols;
    const int j = (int)(e % cols);
    const float t = tanhf(c[r * ldc + j]);
    const float d = to_f32(dout[r * lddo + j]);
    dg[r * lddg + j] = from_f32<T>(d * t);
    dc[r * lddc + j] += d * to_f32(g[r * ldg + j]) * (1.f - t * t);
  }
}

// one workgroup per row
template <typename T>
__global__ __launch_bounds__(256) void gate_mix_fwd_kernel(int D, const T* __restrict__ ctx, int64_t ldx,
                                                           const T* __restrict__ s, int64_t lds,
                                                           const float* __restrict__ wa, const float* __restrict__ ba,
                                                           float* __restrict__ beta, T* __restrict__ out,
                                                           int64_t ldo) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ float red[4];
  __shared__ float sb;
  const T* x = ctx + (int64_t)b * ldx;
  const T* y = s + (int64_t)b * lds;
  float acc = 0.f;
  for (int j = tid; j < D; j += 256) acc += to_f32(x[j]) * wa[j] + to_f32(y[j]) * wa[D + j];
  acc = wave_sum(acc);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) {
    const float z = red[0] + red[1] + red[2] + red[3] + ba[0];
    sb = 1.f / (1.f + __expf(-z));
    beta[b] = sb;
  }
  __syncthreads();
  const float bt = sb;
  for (int j = tid; j < D; j += 256)
    out[(int64_t)b * ldo + j] = from_f32<T>(bt * to_f32(x[j]) + (1.f - bt) * to_f32(y[j]));
}

template <typename T>
__global__ __launch_bounds__(256) void gate_mix_bwd_kernel(int D, const T* __restrict__ ctx, int64_t ldx,
                                                           const T* __restrict__ s, int64_t lds,
                                                           const float* __restrict__ wa, const float* __restrict__ beta,
                                                           const T* __restrict__ dout, int64_t lddo,
                                                           T* __restrict__ dctx, int64_t lddx, T* __restrict__ ds,
                                                           int64_t ldds, float* __restrict__ dwa,
                                                           float* __restrict__ dba) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ float red[4];
  __shared__ float sz;
  const T* x = ctx + (int64_t)b * ldx;
  const T* y = s + (int64_t)b * lds;
  const T* g = dout + (int64_t)b * lddo;
  const float bt = beta[b];
  float acc = 0.f;
  for (int j = tid; j < D; j += 256) acc += to_f32(g[j]) * (to_f32(x[j]) - to_f32(y[j]));
  acc = wave_sum(acc);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) {
    const float dz = (red[0] + red[1] + red[2] + red[3]) * bt * (1.f - bt);  // through the sigmoid
    sz = dz;
    atomicAdd(dba, dz);
  }
  __syncthreads();
  const float dz = sz;
  for (int j = tid; j < D; j += 256) {
    const float gj = to_f32(g[j]), xj = to_f32(x[j]), yj = to_f32(y[j]);
    dctx[(int64_t)b * lddx + j] = from_f32<T>(bt * gj + dz * wa[j]);
    ds[(int64_t)b * ldds + j] = from_f32<T>((1.f - bt) * gj + dz * wa[D + j]);
    atomicAdd(dwa + j, dz * xj);
    atomicAdd(dwa + D + j, dz * yj);
  }
}

// out[b, q, s] = mean_h exp(scale * q_h . k_h,s - lse[b,h,q]) (0 for padded keys)
template <typename T>
__global__ __launch_bounds__(256) void attn_probs_mean_kernel(int H, int Nq, int Nk, int hd, float scale,
                                                              const T* __restrict__ q, int64_t q_bs, int64_t q_rs,
                                                              const T* __restrict__ k, int64_t k_bs, int64_t k_rs,
                                                              const uint8_t* __restrict__ key_pad,
                                                              const float* __restrict__ lse, float* __restrict__ out) {
  const int b = blockIdx.x / Nq, qi = blockIdx.x % Nq;
  const T* qr = q + (int64_t)b * q_bs + (int64_t)qi * q_rs;
  for (int s = threadIdx.x; s < Nk; s += blockDim.x) {
    float acc = 0.f;
    const bool pad = key_pad && key_pad[(int64_t)b * Nk + s];
    if (!pad) {
      const T* kr = k + (int64_t)b * k_bs + (int64_t)s * k_rs;
      for (int h = 0; h < H; ++h) {
        float d = 0.f;
        for (int i = 0; i < hd; ++i) d += to_f32(qr[h * hd + i]) * to_f32(kr[h * hd + i]);
        acc += __expf(d * scale - lse[((int64_t)b * H + h) * Nq + qi]);
      }
    }
    out[((int64_t)b * Nq + qi) * Nk + s] = acc / H;
  }
}

// Backward of attn_probs_mean_kernel (the head-averaged weights MultiHeadAttention returns,
// attention.py:207-211, are differentiable in the reference): with P_h = softmax(scale
// q_h.k_h) and dP_h = dW / H,
//   dscore_h[s] = P_h[s] (dP_h[s] - sum_s' P_h[s'] dP_h[s']),
//   dq_h += scale sum_s dscore_h[s] k_h[s],   dk_h[s] += scale dscore_h[s] q_h.
// One block per (image, head) walks the queries in order (dk rows are shared by the
// queries of an image): deterministic, no atomics.  dq (T) and dk (fp32) ACCUMULATE.
static constexpr int PMB_MAXK = 2048;
template <typename T>
__global__ __launch_bounds__(256) void attn_probs_mean_bwd_kernel(int H, int Nq, int Nk, int hd, float scale,
                                                                  const T* __restrict__ q, int64_t q_bs, int64_t q_rs,
                                                                  const T* __restrict__ k, int64_t k_bs, int64_t k_rs,
                                                                  const uint8_t* __restrict__ key_pad,
                                                                  const float* __restrict__ lse,
                                                                  const float* __restrict__ dw, T* __restrict__ dq,
                                                                  int64_t dq_bs, int64_t dq_rs, float* __restrict__ dk,
                                                                  int64_t dk_bs, int64_t dk_rs) {
  const int b = blockIdx.x / H, h = blockIdx.x % H, tid = threadIdx.x;
  __shared__ float ds[PMB_MAXK];
  __shared__ float red[4];
  const T* kb = k + (int64_t)b * k_bs + h * hd;
  float* dkb = dk + (int64_t)b * dk_bs + h * hd;
  const float invH = 1.f / H;
  for (int qi = 0; qi < Nq; ++qi) {
    const T* qr = q + (int64_t)b * q_bs + (int64_t)qi * q_rs + h * hd;
    const float l = lse[((int64_t)b * H + h) * Nq + qi];
    const float* g = dw + ((int64_t)b * Nq + qi) * Nk;
    float part = 0.f;
    for (int s = tid; s < Nk; s += blockDim.x) {
      float p = 0.f;
      if (!(key_pad && key_pad[(int64_t)b * Nk + s])) {
        const T* kr = kb + (int64_t)s * k_rs;
        float d = 0.f;
        for (int i = 0; i < hd; ++i) d += to_f32(qr[i]) * to_f32(kr[i]);
        p = __expf(d * scale - l);
      }
      ds[s] = p;
      part += p * g[s] * invH;
    }
    part = wave_sum(part);
    if ((tid & 63) == 0) red[tid >> 6] = part;
    __syncthreads();
    const float c = red[0] + red[1] + red[2] + red[3];
    for (int s = tid; s < Nk; s += blockDim.x) ds[s] = ds[s] * (g[s] * invH - c) * scale;
    __syncthreads();
    for (int i = tid; i < hd; i += blockDim.x) {
      float acc = 0.f;
      for (int s = 0; s < Nk; ++s) acc += ds[s] * to_f32(kb[(int64_t)s * k_rs + i]);
      T* dqr = dq + (int64_t)b * dq_bs + (int64_t)qi * dq_rs + h * hd;
      dqr[i] = from_f32<T>(to_f32(dqr[i]) + acc);
    }
    for (int e = tid; e < Nk * hd; e += blockDim.x) {
      const int s = e / hd, i = e % hd;
      dkb[(int64_t)s * dk_rs + i] += ds[s] * to_f32(qr[i]);
    }
    __syncthreads();  // ds and red are rewritten by the next query
  }
}

static int grid_e(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace capk

using namespace capk;

#define DT3(dtype, K)                                                      \
  do {                                                                     \
    if ((dtype) == CAPK_F32) { K(float); }                                 \
    else if ((dtype) == CAPK_BF16) { K(bf16); }                            \
    else { set_error("capk gates: dtype"); return CAPK_EINVAL; }           \
  } while (0)

extern "C" int capk_ew_mul(int dtype, int rows, int cols, const void* a, int64_t lda, const void* b, int64_t ldb,
                           void* out, int64_t ldo, void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols > 0, "capk_ew_mul: sizes");
#define K(T) hipLaunchKernelGGL(ew_mul_kernel<T>, dim3(grid_e((int64_t)rows * cols)), dim3(256), 0, S(stream), rows, cols, (const T*)a, lda, (const T*)b, ldb, (T*)out, ldo)
  DT3(dtype, K);
#undef K
  CAPK_LAUNCH_CHECK("ew_mul_kernel");
  return CAPK_OK;
}

extern "C" int capk_tanh_gate_fwd(int dtype, int rows, int cols, const float* c, int64_t ldc, const void* g,
                                  int64_t ldg, void* out, int64_t ldo, void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols > 0, "capk_tanh_gate_fwd: sizes");
#define K(T) hipLaunchKernelGGL(tanh_gate_fwd_kernel<T>, dim3(grid_e((int64_t)rows * cols)), dim3(256), 0, S(stream), rows, cols, c, ldc, (const T*)g, ldg, (T*)out, ldo)
  DT3(dtype, K);
#undef K
  CAPK_LAUNCH_CHECK("tanh_gate_fwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_tanh_gate_bwd(int dtype, int rows, int cols, const float* c, int64_t ldc, const void* g,
                                  int64_t ldg, const void* dout, int64_t lddo, void* dg, int64_t lddg, float* dc,
                                  int64_t lddc, void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols > 0, "capk_tanh_gate_bwd: sizes");
#define K(T) hipLaunchKernelGGL(tanh_gate_bwd_kernel<T>, dim3(grid_e((int64_t)rows * cols)), dim3(256), 0, S(stream), rows, cols, c, ldc, (const T*)g, ldg, (const T*)dout, lddo, (T*)dg, lddg, dc, lddc)
  DT3(dtype, K);
#undef K
  CAPK_LAUNCH_CHECK("tanh_gate_bwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_gate_mix_fwd(int dtype, int B, int D, const void* ctx, int64_t ldx, const void* s, int64_t lds,
                                 const float* wa, const float* ba, float* beta, void* out, int64_t ldo, void* stream) {
  CAPK_CHECK_ARG(B > 0 && D > 0, "capk_gate_mix_fwd: sizes");
#define K(T) hipLaunchKernelGGL(gate_mix_fwd_kernel<T>, dim3(B), dim3(256), 0, S(stream), D, (const T*)ctx, ldx, (const T*)s, lds, wa, ba, beta, (T*)out, ldo)
  DT3(dtype, K);
#undef K
  CAPK_LAUNCH_CHECK("gate_mix_fwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_gate_mix_bwd(int dtype, int B, int D, const void* ctx, int64_t ldx, const void* s, int64_t lds,
                                 const float* wa, const float* beta, const void* dout, int64_t lddo, void* dctx,
                                 int64_t lddx, void* ds, int64_t ldds, float* dwa, float* dba, void* stream) {
  CAPK_CHECK_ARG(B > 0 && D > 0, "capk_gate_mix_bwd: sizes");
#define K(T) hipLaunchKernelGGL(gate_mix_bwd_kernel<T>, dim3(B), dim3(256), 0, S(stream), D, (const T*)ctx, ldx, (const T*)s, lds, wa, beta, (const T*)dout, lddo, (T*)dctx, lddx, (T*)ds, ldds, dwa, dba)
  DT3(dtype, K);
#undef K
  CAPK_LAUNCH_CHECK("gate_mix_bwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_attention_probs_mean(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, const void* q,
                                         int64_t q_bs, int64_t q_rs, const void* k, int64_t k_bs, int64_t k_rs,
                                         const uint8_t* key_pad, const float* lse, float* out, void* stream) {
  CAPK_CHECK_ARG(B > 0 && H > 0 && Nq > 0 && Nk > 0 && hd > 0, "capk_attention_probs_mean: sizes");
#define K(T) hipLaunchKernelGGL(attn_probs_mean_kernel<T>, dim3(B * Nq), dim3(256), 0, S(stream), H, Nq, Nk, hd, scale, (const T*)q, q_bs, q_rs, (const T*)k, k_bs, k_rs, key_pad, lse, out)
  DT3(dtype, K);
#undef K
  CAPK_LAUNCH_CHECK("attn_probs_mean_kernel");
  return CAPK_OK;
}

extern "C" int capk_attention_probs_mean_bwd(int dtype, int B, int H, int Nq, int Nk, int hd, float scale,
                                             const void* q, int64_t q_bs, int64_t q_rs, const void* k, int64_t k_bs,
                                             int64_t k_rs, const uint8_t* key_pad, const float* lse, const float* dw,
                                             void* dq, int64_t dq_bs, int64_t dq_rs, float* dk, int64_t dk_bs,
                                             int64_t dk_rs, void* stream) {
  CAPK_CHECK_ARG(B > 0 && H > 0 && Nq > 0 && Nk > 0 && hd > 0, "capk_attention_probs_mean_bwd: sizes");
  CAPK_CHECK_ARG(Nk <= PMB_MAXK, "capk_attention_probs_mean_bwd: need Nk <= %d", PMB_MAXK);
#define K(T) hipLaunchKernelGGL(attn_probs_mean_bwd_kernel<T>, dim3(B * H), dim3(256), 0, S(stream), H, Nq, Nk, hd, scale, (const T*)q, q_bs, q_rs, (const T*)k, k_bs, k_rs, key_pad, lse, dw, (T*)dq, dq_bs, dq_rs, dk, dk_bs, dk_rs)
  DT3(dtype, K);
#undef K
  CAPK_LAUNCH_CHECK("attn_probs_mean_bwd_kernel");
  return CAPK_OK;
}
