// Legacy Show-Attend-Tell training step pieces (models/decoder.py
// + train.py).  The decoder step itself runs on the shared kernels (MFMA GEMMs, the
// additive-attention kernels of lstm.hip with the ReLU energy, the LSTM cell kernel);
// these are the loss / optimizer-side extras of train.py:92-112:
//   attn_coverage_reg  ((1 - sum_t alpha[b,t,s])^2).mean() (train.py:101, the doubly
//                      stochastic attention term) and its gradient coefficient
//   clamp              param.grad.clamp_(-grad_clip, grad_clip) (train.py:105-110)
//   mask_rows_by_length predictions[b, t] = 0 for t >= dec_len[b] (decoder.py:130-133:
//                      the predictions tensor starts as zeros and only active rows are set)
#include "common.h"

namespace capk {

// alphas t-major [T][B][S] fp32 (inactive rows zero).  One workgroup, deterministic.
__global__ __launch_bounds__(1024) void coverage_reg_kernel(int B, int T, int S, const float* __restrict__ alphas,
                                                            const float* __restrict__ grad_scale,
                                                            float* __restrict__ loss_acc, float* __restrict__ coef) {
  __shared__ float red[16];
  const int n = B * S;
  const float inv_n = 1.0f / (float)n;
  const float gs = grad_scale ? grad_scale[0] : 1.0f;
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float a = 0.f;
    for (int t = 0; t < T; ++t) a += alphas[(int64_t)t * n + i];
    const float r = 1.0f - a;
    acc += r * r;
    if (coef) coef[i] = -2.0f * r * inv_n * gs;
  }
  acc = wave_sum(acc);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0 && loss_acc) {
    float s = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += red[k];
    loss_acc[0] += s * inv_n;
  }
}

__global__ __launch_bounds__(256) void clamp_kernel(int64_t n, float* __restrict__ x, float lo, float hi) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = fminf(fmaxf(x[i], lo), hi);
}

template <typename T>
__global__ __launch_bounds__(256) void mask_rows_kernel(int B, int Tn, int cols, T* __restrict__ x, int64_t ld,
                                                        int64_t bs, const int32_t* __restrict__ len) {
  const int64_t total = (int64_t)B * Tn * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % cols);
    const int64_t r = i / cols;
    const int t = (int)(r % Tn), b = (int)(r / Tn);
    if (t >= len[b]) x[b * bs + t * ld + c] = from_f32<T>(0.f);
  }
}

static int grid_of(int64_t work) { return (int)std::min<int64_t>(8192, std::max<int64_t>(1, (work + 255) / 256)); }

}  // namespace capk

using namespace capk;

extern "C" int capk_attn_coverage_reg(int B, int T, int S, const float* alphas, const float* grad_scale,
                                      float* loss_acc, float* coef, void* stream) {
  CAPK_CHECK_ARG(B > 0 && T > 0 && S > 0 && alphas, "capk_attn_coverage_reg: bad shape");
  hipLaunchKernelGGL(coverage_reg_kernel, dim3(1), dim3(1024), 0, capk::S(stream), B, T, S, alphas, grad_scale, loss_acc,
                     coef);
  CAPK_LAUNCH_CHECK("coverage_reg_kernel");
  return CAPK_OK;
}

extern "C" int capk_clamp(int64_t n, float* x, float lo, float hi, void* stream) {
  CAPK_CHECK_ARG(n >= 0 && lo <= hi, "capk_clamp: bad args");
  if (n == 0) return CAPK_OK;
  hipLaunchKernelGGL(clamp_kernel, dim3(grid_of(n)), dim3(256), 0, S(stream), n, x, lo, hi);
  CAPK_LAUNCH_CHECK("clamp_kernel");
  return CAPK_OK;
}

extern "C" int capk_mask_rows_by_length(int dtype, int B, int T, int cols, void* x, int64_t ld, int64_t bs,
                                        const int32_t* len, void* stream) {
  CAPK_CHECK_ARG(B > 0 && T > 0 && cols > 0 && len, "capk_mask_rows_by_length: bad args");
  const int64_t work = (int64_t)B * T * cols;
  if (dtype == CAPK_BF16)
    hipLaunchKernelGGL(mask_rows_kernel<bf16>, dim3(grid_of(work)), dim3(256), 0, S(stream), B, T, cols, (bf16*)x, ld,
                       bs, len);
  else if (dtype == CAPK_F32)
    hipLaunchKernelGGL(mask_rows_kernel<float>, dim3(grid_of(work)), dim3(256), 0, S(stream), B, T, cols, (float*)x,
                       ld, bs, len);
  else
    CAPK_CHECK_ARG(false, "capk_mask_rows_by_length: dtype");
  CAPK_LAUNCH_CHECK("mask_rows_kernel");
  return CAPK_OK;
}
