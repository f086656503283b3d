// LSTM decoder step kernels.
//
// The recurrent GEMMs (gates = x W_ih^T + b_ih + h W_hh^T + b_hh) run on the MFMA
// GEMM; these kernels are the per-step elementwise / reduction parts:
//   lstm_cell_fwd / lstm_cell_bwd  torch nn.LSTM cell (aten lstm_cell: gate order
//                                  i, f, g, o; c' = f c + i g; h' = o tanh(c')), cell
//                                  state kept in fp32, inter-layer dropout fused on
//                                  the copy of h' that feeds the next layer.
//   soft_attn_fwd / soft_attn_bwd  SoftAttention (src/models/attention.py:57-118):
//                                  e = energy(tanh(q_proj(q) + key_proj(k))) / T,
//                                  masked_fill(-1e9), softmax over S, ctx = w @ v.
//                                  key_proj(k) is hoisted out of the decode loop by
//                                  the caller (same values every step).
// One workgroup per image for the attention kernels (S <= 256, D <= 1024).
#include "common.h"

namespace capk {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

template <typename T>
__global__ __launch_bounds__(256) void lstm_cell_fwd_kernel(int B, int D, const T* __restrict__ gates, int64_t ldg,
                                                            const float* __restrict__ c_prev, float* __restrict__ c_out,
                                                            T* __restrict__ h_out, int64_t ldh, T* __restrict__ h_drop,
                                                            int64_t ldhd, T* __restrict__ act, Drop drop) {
  const int64_t n = (int64_t)B * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / D), d = (int)(e % D);
    const T* g = gates + (int64_t)b * ldg;
    const float i = sigm(to_f32(g[d])), f = sigm(to_f32(g[D + d]));
    const float gg = tanhf(to_f32(g[2 * D + d])), o = sigm(to_f32(g[3 * D + d]));
    const float c = f * c_prev[e] + i * gg;
    const float h = o * tanhf(c);
    c_out[e] = c;
    h_out[(int64_t)b * ldh + d] = from_f32<T>(h);
    if (h_drop) h_drop[(int64_t)b * ldhd + d] = from_f32<T>(drop.on() ? h * drop.mul((uint64_t)e) : h);
    T* a = act + (int64_t)b * 4 * D;
    a[d] = from_f32<T>(i);
    a[D + d] = from_f32<T>(f);
    a[2 * D + d] = from_f32<T>(gg);
    a[3 * D + d] = from_f32<T>(o);
  }
}

// dh: total gradient w.r.t. h' (T), dc: in = grad w.r.t. c', out = grad w.r.t. c_prev (fp32, in place)
template <typename T>
__global__ __launch_bounds__(256) void lstm_cell_bwd_kernel(int B, int D, const T* __restrict__ act,
                                                            const float* __restrict__ c_prev, const T* __restrict__ dh,
                                                            int64_t lddh, float* __restrict__ dc,
                                                            T* __restrict__ dgates) {
  const int64_t n = (int64_t)B * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / D), d = (int)(e % D);
    const T* a = act + (int64_t)b * 4 * D;
    const float i = to_f32(a[d]), f = to_f32(a[D + d]), g = to_f32(a[2 * D + d]), o = to_f32(a[3 * D + d]);
    const float cp = c_prev[e];
    const float c = f * cp + i * g;
    const float tc = tanhf(c);
    const float gh = to_f32(dh[(int64_t)b * lddh + d]);
    const float dct = dc[e] + gh * o * (1.f - tc * tc);
    T* dg = dgates + (int64_t)b * 4 * D;
    dg[d] = from_f32<T>(dct * g * i * (1.f - i));
    dg[D + d] = from_f32<T>(dct * cp * f * (1.f - f));
    dg[2 * D + d] = from_f32<T>(dct * i * (1.f - g * g));
    dg[3 * D + d] = from_f32<T>(gh * tc * o * (1.f - o));
    dc[e] = dct * f;
  }
}

// The same cells fed by the recurrent pair product's fp32 split-K slabs (capk_gemm_pair_slabs:
// slab s of a [B, ldw] product at ws + s * B * ldw), summed here instead of by a reduce
// launch.  Forward: gates = sum_s slab[s] + bias_a + bias_b (+ res, bf16).
__global__ __launch_bounds__(256) void lstm_cell_fwd_slabs_kernel(
    int B, int D, const float* __restrict__ ws, int splits, int64_t ldw, const float* __restrict__ ba,
    const float* __restrict__ bb, const bf16* __restrict__ res, int64_t ldr, const float* __restrict__ c_prev,
    float* __restrict__ c_out, bf16* __restrict__ h_out, int64_t ldh, bf16* __restrict__ h_drop, int64_t ldhd,
    bf16* __restrict__ act, Drop drop) {
  const int64_t n = (int64_t)B * D, ss = (int64_t)B * ldw;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / D), d = (int)(e % D);
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int col = q * D + d;
      g[q] = (ba ? ba[col] : 0.f) + (bb ? bb[col] : 0.f) + (res ? to_f32(res[(int64_t)b * ldr + col]) : 0.f);
    }
    const float* w = ws + (int64_t)b * ldw + d;
    int s = 0;
    for (; s + 2 <= splits; s += 2, w += 2 * ss) {  // 8 independent loads in flight per thread
      float x[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = w[q * D], x[4 + q] = w[ss + q * D];
#pragma unroll
      for (int q = 0; q < 4; ++q) g[q] += x[q] + x[4 + q];
    }
    if (s < splits) {
#pragma unroll
      for (int q = 0; q < 4; ++q) g[q] += w[q * D];
    }
    const float i = sigm(g[0]), f = sigm(g[1]), gg = tanhf(g[2]), o = sigm(g[3]);
    const float c = f * c_prev[e] + i * gg;
    const float h = o * tanhf(c);
    c_out[e] = c;
    h_out[(int64_t)b * ldh + d] = from_f32<bf16>(h);
    if (h_drop) h_drop[(int64_t)b * ldhd + d] = from_f32<bf16>(drop.on() ? h * drop.mul((uint64_t)e) : h);
    bf16* a = act + (int64_t)b * 4 * D;
    a[d] = from_f32<bf16>(i);
    a[D + d] = from_f32<bf16>(f);
    a[2 * D + d] = from_f32<bf16>(gg);
    a[3 * D + d] = from_f32<bf16>(o);
  }
}

// sum over n slabs of one element (slab stride ss), 4 loads in flight, fixed order
__device__ __forceinline__ float slab_col_sum(const float* __restrict__ w, int n, int64_t ss) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 0;
  for (; s + 4 <= n; s += 4, w += 4 * ss) a0 += w[0], a1 += w[ss], a2 += w[2 * ss], a3 += w[3 * ss];
  for (; s < n; ++s, w += ss) a0 += *w;
  return (a0 + a1) + (a2 + a3);
}

// Backward: the gradient w.r.t. h' = dh (bf16, optional) + drop(sum_s up[s][:, 0:D]) (the layer
// above's input gradient through the forward's dropout mask, index b*D + d) + sum_s rec[s][:, colr:colr+D]
// (this layer's recurrent gradient from step t+1).
__global__ __launch_bounds__(256) void lstm_cell_bwd_slabs_kernel(
    int B, int D, const bf16* __restrict__ act, const float* __restrict__ c_prev, const bf16* __restrict__ dh,
    int64_t lddh, const float* __restrict__ wsu, int su, int64_t ldu, Drop drop, const float* __restrict__ wsr, int sr,
    int64_t ldrr, int colr, float* __restrict__ dc, bf16* __restrict__ dgates) {
  const int64_t n = (int64_t)B * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / D), d = (int)(e % D);
    float gh = dh ? to_f32(dh[(int64_t)b * lddh + d]) : 0.f;
    if (wsu) {
      const float u = slab_col_sum(wsu + (int64_t)b * ldu + d, su, (int64_t)B * ldu);
      gh += drop.on() ? u * drop.mul((uint64_t)e) : u;
    }
    if (wsr) gh += slab_col_sum(wsr + (int64_t)b * ldrr + colr + d, sr, (int64_t)B * ldrr);
    const bf16* a = act + (int64_t)b * 4 * D;
    const float i = to_f32(a[d]), f = to_f32(a[D + d]), g = to_f32(a[2 * D + d]), o = to_f32(a[3 * D + d]);
    const float cp = c_prev[e];
    const float c = f * cp + i * g;
    const float tc = tanhf(c);
    const float dct = dc[e] + gh * o * (1.f - tc * tc);
    bf16* dg = dgates + (int64_t)b * 4 * D;
    dg[d] = from_f32<bf16>(dct * g * i * (1.f - i));
    dg[D + d] = from_f32<bf16>(dct * cp * f * (1.f - f));
    dg[2 * D + d] = from_f32<bf16>(dct * i * (1.f - g * g));
    dg[3 * D + d] = from_f32<bf16>(gh * tc * o * (1.f - o));
    dc[e] = dct * f;
  }
}

// out[m][j] = sum_s ws[s][m][col0 + j] (+ res[m][j]) (slabs of a [M, ldw] product), bf16.
__global__ __launch_bounds__(256) void slab_sum_kernel(int M, int ncols, const float* __restrict__ ws, int splits,
                                                       int64_t ldw, int col0, const bf16* __restrict__ res,
                                                       int64_t ldr, bf16* __restrict__ out, int64_t ldo) {
  const int64_t n = (int64_t)M * ncols, ss = (int64_t)M * ldw;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(e / ncols), j = (int)(e % ncols);
    const float r = res ? to_f32(res[(int64_t)m * ldr + j]) : 0.f;
    out[(int64_t)m * ldo + j] = from_f32<bf16>(slab_col_sum(ws + (int64_t)m * ldw + col0 + j, splits, ss) + r);
  }
}

// ------------------------------------------------------------ soft attention --
static constexpr int SA_MAXS = 256;
// energy nonlinearity: 0 = tanh (SoftAttention, attention.py:100), 1 = ReLU (legacy
// Show-Attend-Tell attention, models/decoder.py:145-146)
template <int ACT>
__device__ __forceinline__ float energy_act(float x) { return ACT == 0 ? tanhf(x) : (x > 0.f ? x : 0.f); }
template <int ACT>
__device__ __forceinline__ float energy_act_grad(float pre, float a) { return ACT == 0 ? 1.f - a * a : (pre > 0.f ? 1.f : 0.f); }

template <typename T, int ACT>
__global__ __launch_bounds__(1024) void soft_attn_fwd_kernel(int S, int D, int Dv, const T* __restrict__ qp, int64_t ldq,
                                                            const T* __restrict__ kp, int64_t kp_bs, int64_t kp_rs,
                                                            const T* __restrict__ v, int64_t v_bs, int64_t v_rs,
                                                            const float* __restrict__ we, const float* __restrict__ be,
                                                            float inv_temp, const uint8_t* __restrict__ key_pad,
                                                            T* __restrict__ ctx, int64_t ldc, float* __restrict__ wout) {
  // 1024 threads (16 waves) per image: the per-key energies are 16 wave-dot-products in
  // flight and the context columns one per thread (4 waves left the latency exposed)
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  __shared__ float sc[SA_MAXS];
  __shared__ float red[1];
  const T* q = qp + (int64_t)b * ldq;
  const T* kb = kp + (int64_t)b * kp_bs;
  for (int s = w; s < S; s += nw) {
    const T* k = kb + (int64_t)s * kp_rs;
    float acc = 0.f;
    for (int d = lane; d < D; d += 64) acc += we[d] * energy_act<ACT>(to_f32(q[d]) + to_f32(k[d]));
    acc = wave_sum(acc);
    if (lane == 0) {
      float e = (acc + be[0]) * inv_temp;
      if (key_pad && key_pad[(int64_t)b * S + s]) e = -1e9f;
      sc[s] = e;
    }
  }
  __syncthreads();
  if (w == 0) {
    float m = -INFINITY;
    for (int s = lane; s < S; s += 64) m = fmaxf(m, sc[s]);
    m = wave_max(m);
    float l = 0.f;
    for (int s = lane; s < S; s += 64) {
      const float p = __expf(sc[s] - m);
      sc[s] = p;
      l += p;
    }
    l = wave_sum(l);
    if (lane == 0) red[0] = 1.f / l;
  }
  __syncthreads();
  const float inv = red[0];
  for (int s = tid; s < S; s += blockDim.x) {
    sc[s] *= inv;
    wout[(int64_t)b * S + s] = sc[s];
  }
  __syncthreads();
  const T* vb = v + (int64_t)b * v_bs;
  for (int d = tid; d < Dv; d += blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < S; ++s) acc += sc[s] * to_f32(vb[(int64_t)s * v_rs + d]);
    ctx[(int64_t)b * ldc + d] = from_f32<T>(acc);
  }
}

// Gradients of one step; the key/value/energy gradients ACCUMULATE (fp32) over the
// decode steps: dkp [B,S,D], dv [B,S,D], dwe_part [B,D], dbe_part [B].
template <typename T, int ACT>
__global__ __launch_bounds__(1024) void soft_attn_bwd_kernel(int S, int D, int Dv, const T* __restrict__ qp, int64_t ldq,
                                                            const T* __restrict__ kp, int64_t kp_bs, int64_t kp_rs,
                                                            const T* __restrict__ v, int64_t v_bs, int64_t v_rs,
                                                            const float* __restrict__ we, float inv_temp,
                                                            const float* __restrict__ wsave, const T* __restrict__ dctx,
                                                            int64_t lddc, const float* __restrict__ dw_in,
                                                            T* __restrict__ dqp, int64_t lddq,
                                                            float* __restrict__ dkp, float* __restrict__ dv,
                                                            float* __restrict__ dwe_part, float* __restrict__ dbe_part,
                                                            float* __restrict__ de_out, T* __restrict__ dctx_out) {
  // grid (B, column chunks of blockDim): every chunk block recomputes the step's S-vector
  // (dctx . v[s], softmax Jacobian) -- S*Dv MACs -- and owns blockDim columns of dq / dkp /
  // dwe / dv; chunk 0 also writes dbe.  (One 4-wave block per image left the latency and
  // half the CUs idle.)
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const int CH = blockDim.x, d0 = blockIdx.y * CH;
  __shared__ float ws[SA_MAXS], de[SA_MAXS];
  __shared__ float red[16];
  const T* g = dctx + (int64_t)b * lddc;
  const T* vb = v + (int64_t)b * v_bs;
  for (int s = tid; s < S; s += CH) ws[s] = wsave[(int64_t)b * S + s];
  __syncthreads();
  // dw[s] = dctx . v[s]
  for (int s = w; s < S; s += nw) {
    const T* vr = vb + (int64_t)s * v_rs;
    float acc = 0.f;
    for (int d = lane; d < Dv; d += 64) acc += to_f32(g[d]) * to_f32(vr[d]);
    acc = wave_sum(acc);
    if (lane == 0) de[s] = acc + (dw_in ? dw_in[(int64_t)b * S + s] : 0.f);
  }
  __syncthreads();
  if (w == 0) {
    float dot = 0.f;
    for (int s = lane; s < S; s += 64) dot += ws[s] * de[s];
    dot = wave_sum(dot);
    if (lane == 0) red[0] = dot;
  }
  __syncthreads();
  const float dot = red[0];
  for (int s = tid; s < S; s += CH) {
    de[s] = ws[s] * (de[s] - dot) * inv_temp;
    if (de_out && blockIdx.y == 0) de_out[(int64_t)b * S + s] = de[s];
  }
  if (dctx_out) {  // this step's output gradient, for the deferred dv
    const int Y = gridDim.y, e0 = (int)((int64_t)Dv * blockIdx.y / Y), e1 = (int)((int64_t)Dv * (blockIdx.y + 1) / Y);
    for (int d = e0 + tid; d < e1; d += CH) dctx_out[(int64_t)b * Dv + d] = g[d];
  }
  __syncthreads();
  const T* q = qp + (int64_t)b * ldq;
  const T* kb = kp + (int64_t)b * kp_bs;
  float* dkb = dkp ? dkp + (int64_t)b * S * D : nullptr;
  float dbe = 0.f;
  for (int s = tid; s < S; s += CH) dbe += de[s];
  for (int d = d0 + tid; d < D && d < d0 + CH; d += CH) {
    const float qd = to_f32(q[d]), wd = we[d];
    float dq = 0.f, dw = 0.f;
#pragma unroll 7
    for (int s = 0; s < S; ++s) {
      const float pre = qd + to_f32(kb[(int64_t)s * kp_rs + d]);
      const float a = energy_act<ACT>(pre);
      const float gr = de[s] * wd * energy_act_grad<ACT>(pre, a);
      dq += gr;
      dw += de[s] * a;
      if (dkp) dkb[(int64_t)s * D + d] += gr;
    }
    dqp[(int64_t)b * lddq + d] = from_f32<T>(dq);
    dwe_part[(int64_t)b * D + d] += dw;
  }
  if (dv) {
    float* dvb = dv + (int64_t)b * S * Dv;
    // columns [Dv * y / Y, Dv * (y + 1) / Y) of dv for chunk y of Y (Dv may differ from D)
    const int Y = gridDim.y, e0 = (int)((int64_t)Dv * blockIdx.y / Y), e1 = (int)((int64_t)Dv * (blockIdx.y + 1) / Y);
    for (int d = e0 + tid; d < e1; d += CH) {
      const float gd = to_f32(g[d]);
#pragma unroll 7
      for (int s = 0; s < S; ++s) dvb[(int64_t)s * Dv + d] += ws[s] * gd;
    }
  }
  if (blockIdx.y != 0) return;
  dbe = wave_sum(dbe);
  if (lane == 0) red[w] = dbe;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += red[i];
    dbe_part[b] += t;
  }
}

// The key / value gradients of all steps at once (the deferred form of soft_attn_bwd's per-step
// read-modify-write of two [B, S, D] fp32 buffers): dkp[b,s,d] = sum_t de_t[b,s] we[d]
// act'(qp_t[b,d] + kp[b,s,d]), dv[b,s,d] = sum_t w_t[b,s] dctx_t[b,d], t from the last step
// down -- the order (and expressions) of the per-step accumulation it replaces.  One block per
// (image, key), threads over the columns.
template <typename T, int ACT>
__global__ __launch_bounds__(256) void soft_attn_kv_grad_kernel(int steps, int B, int S, int D, int Dv,
                                                                const T* __restrict__ qp, const T* __restrict__ kp,
                                                                int64_t kp_bs, int64_t kp_rs,
                                                                const float* __restrict__ we,
                                                                const float* __restrict__ de_all,
                                                                const float* __restrict__ w_all,
                                                                const T* __restrict__ dctx_all,
                                                                float* __restrict__ dkp, float* __restrict__ dv) {
  const int b = blockIdx.x / S, s = blockIdx.x % S;
  const T* k = kp + (int64_t)b * kp_bs + (int64_t)s * kp_rs;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const float kd = to_f32(k[d]), wd = we[d];
    float acc = 0.f;
    for (int t = steps - 1; t >= 0; --t) {
      const float pre = to_f32(qp[((int64_t)t * B + b) * D + d]) + kd;
      const float a = energy_act<ACT>(pre);
      acc += de_all[((int64_t)t * B + b) * S + s] * wd * energy_act_grad<ACT>(pre, a);
    }
    dkp[((int64_t)b * S + s) * D + d] = acc;
  }
  if (!dv) return;
  for (int d = threadIdx.x; d < Dv; d += blockDim.x) {
    float acc = 0.f;
    for (int t = steps - 1; t >= 0; --t)
      acc += w_all[((int64_t)t * B + b) * S + s] * to_f32(dctx_all[((int64_t)t * B + b) * Dv + d]);
    dv[((int64_t)b * S + s) * Dv + d] = acc;
  }
}

static int grid_n(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace capk

using namespace capk;

#define DT2(dtype, KERNEL_T, ...)                                                 \
  do {                                                                           \
    if ((dtype) == CAPK_F32) { KERNEL_T(float, __VA_ARGS__); }                    \
    else if ((dtype) == CAPK_BF16) { KERNEL_T(bf16, __VA_ARGS__); }               \
    else { set_error("capk lstm: dtype"); return CAPK_EINVAL; }                   \
  } while (0)

extern "C" int capk_lstm_cell_fwd(int dtype, int B, int D, const void* gates, int64_t ldg, const float* c_prev,
                                  float* c_out, void* h_out, int64_t ldh, void* h_drop, int64_t ldhd, void* act,
                                  float drop_p, uint32_t drop_seed, void* stream) {
  CAPK_CHECK_ARG(B > 0 && D > 0 && ldg >= 4 * D && ldh >= D, "capk_lstm_cell_fwd: bad sizes");
#define K(T, _) hipLaunchKernelGGL(lstm_cell_fwd_kernel<T>, dim3(grid_n((int64_t)B * D)), dim3(256), 0, S(stream), B, D, (const T*)gates, ldg, c_prev, c_out, (T*)h_out, ldh, (T*)h_drop, ldhd, (T*)act, make_drop(drop_p, drop_seed))
  DT2(dtype, K, 0);
#undef K
  CAPK_LAUNCH_CHECK("lstm_cell_fwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_lstm_cell_bwd(int dtype, int B, int D, const void* act, const float* c_prev, const void* dh,
                                  int64_t lddh, float* dc, void* dgates, void* stream) {
  CAPK_CHECK_ARG(B > 0 && D > 0 && lddh >= D, "capk_lstm_cell_bwd: bad sizes");
#define K(T, _) hipLaunchKernelGGL(lstm_cell_bwd_kernel<T>, dim3(grid_n((int64_t)B * D)), dim3(256), 0, S(stream), B, D, (const T*)act, c_prev, (const T*)dh, lddh, dc, (T*)dgates)
  DT2(dtype, K, 0);
#undef K
  CAPK_LAUNCH_CHECK("lstm_cell_bwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_lstm_cell_fwd_slabs(int B, int D, const float* ws, int splits, int64_t ldw, const float* bias_a,
                                        const float* bias_b, const void* res, int64_t ldr, const float* c_prev,
                                        float* c_out, void* h_out, int64_t ldh, void* h_drop, int64_t ldhd, void* act,
                                        float drop_p, uint32_t drop_seed, void* stream) {
  CAPK_CHECK_ARG(B > 0 && D > 0 && ws && splits > 0 && ldw >= 4 * D && ldh >= D && (!res || ldr >= 4 * D) &&
                     c_prev && c_out && h_out && act,
                 "capk_lstm_cell_fwd_slabs: bad arguments");
  hipLaunchKernelGGL(lstm_cell_fwd_slabs_kernel, dim3(grid_n((int64_t)B * D)), dim3(256), 0, S(stream), B, D, ws,
                     splits, ldw, bias_a, bias_b, (const bf16*)res, ldr, c_prev, c_out, (bf16*)h_out, ldh,
                     (bf16*)h_drop, ldhd, (bf16*)act, make_drop(drop_p, drop_seed));
  CAPK_LAUNCH_CHECK("lstm_cell_fwd_slabs_kernel");
  return CAPK_OK;
}

extern "C" int capk_lstm_cell_bwd_slabs(int B, int D, const void* act, const float* c_prev, const void* dh,
                                        int64_t lddh, const float* ws_up, int splits_up, int64_t ld_up, float drop_p,
                                        uint32_t drop_seed, const float* ws_rec, int splits_rec, int64_t ld_rec,
                                        int col_rec, float* dc, void* dgates, void* stream) {
  CAPK_CHECK_ARG(B > 0 && D > 0 && act && c_prev && dc && dgates && (!dh || lddh >= D) &&
                     (!ws_up || (splits_up > 0 && ld_up >= D)) &&
                     (!ws_rec || (splits_rec > 0 && col_rec >= 0 && ld_rec >= col_rec + D)),
                 "capk_lstm_cell_bwd_slabs: bad arguments");
  hipLaunchKernelGGL(lstm_cell_bwd_slabs_kernel, dim3(grid_n((int64_t)B * D)), dim3(256), 0, S(stream), B, D,
                     (const bf16*)act, c_prev, (const bf16*)dh, lddh, ws_up, splits_up, ld_up,
                     make_drop(drop_p, drop_seed), ws_rec, splits_rec, ld_rec, col_rec, dc, (bf16*)dgates);
  CAPK_LAUNCH_CHECK("lstm_cell_bwd_slabs_kernel");
  return CAPK_OK;
}

extern "C" int capk_slab_sum(int M, int ncols, const float* ws, int splits, int64_t ldw, int col0, const void* res,
                             int64_t ldr, void* out, int64_t ldo, void* stream) {
  CAPK_CHECK_ARG(M > 0 && ncols > 0 && ws && out && splits > 0 && col0 >= 0 && ldw >= col0 + ncols && ldo >= ncols &&
                     (!res || ldr >= ncols),
                 "capk_slab_sum: bad arguments");
  hipLaunchKernelGGL(slab_sum_kernel, dim3(grid_n((int64_t)M * ncols)), dim3(256), 0, S(stream), M, ncols, ws, splits,
                     ldw, col0, (const bf16*)res, ldr, (bf16*)out, ldo);
  CAPK_LAUNCH_CHECK("slab_sum_kernel");
  return CAPK_OK;
}

extern "C" int capk_additive_attn_fwd(int dtype, int act, int B, int S, int D, int Dv, const void* qp, int64_t ldq,
                                      const void* kp, int64_t kp_bs, int64_t kp_rs, const void* v, int64_t v_bs,
                                      int64_t v_rs, const float* we, const float* be, float inv_temp,
                                      const uint8_t* key_pad, void* ctx, int64_t ldc, float* w_out, void* stream) {
  CAPK_CHECK_ARG(B > 0 && S > 0 && S <= SA_MAXS && D > 0 && Dv > 0, "capk_additive_attn_fwd: need 0 < S <= %d",
                 SA_MAXS);
  CAPK_CHECK_ARG(act == 0 || act == 1, "capk_additive_attn_fwd: act must be 0 (tanh) or 1 (relu)");
#define K(T, A) hipLaunchKernelGGL((soft_attn_fwd_kernel<T, A>), dim3(B), dim3(1024), 0, capk::S(stream), S, D, Dv, (const T*)qp, ldq, (const T*)kp, kp_bs, kp_rs, (const T*)v, v_bs, v_rs, we, be, inv_temp, key_pad, (T*)ctx, ldc, w_out)
  if (act == 0) DT2(dtype, K, 0); else DT2(dtype, K, 1);
#undef K
  CAPK_LAUNCH_CHECK("soft_attn_fwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_additive_attn_bwd(int dtype, int act, int B, int S, int D, int Dv, const void* qp, int64_t ldq,
                                      const void* kp, int64_t kp_bs, int64_t kp_rs, const void* v, int64_t v_bs,
                                      int64_t v_rs, const float* we, float inv_temp, const float* w, const void* dctx,
                                      int64_t lddc, const float* dw_in, void* dqp, int64_t lddq, float* dkp, float* dv,
                                      float* dwe_part, float* dbe_part, void* stream) {
  CAPK_CHECK_ARG(B > 0 && S > 0 && S <= SA_MAXS && D > 0 && Dv > 0, "capk_additive_attn_bwd: need 0 < S <= %d",
                 SA_MAXS);
  CAPK_CHECK_ARG(act == 0 || act == 1, "capk_additive_attn_bwd: act must be 0 (tanh) or 1 (relu)");
#define K(T, A) hipLaunchKernelGGL((soft_attn_bwd_kernel<T, A>), dim3(B, (D + 1023) / 1024), dim3(1024), 0, capk::S(stream), S, D, Dv, (const T*)qp, ldq, (const T*)kp, kp_bs, kp_rs, (const T*)v, v_bs, v_rs, we, inv_temp, w, (const T*)dctx, lddc, dw_in, (T*)dqp, lddq, dkp, dv, dwe_part, dbe_part, (float*)nullptr, (T*)nullptr)
  if (act == 0) DT2(dtype, K, 0); else DT2(dtype, K, 1);
#undef K
  CAPK_LAUNCH_CHECK("soft_attn_bwd_kernel");
  return CAPK_OK;
}

extern "C" int capk_soft_attn_bwd_step(int dtype, int B, int S, int D, const void* qp, int64_t ldq, const void* kp,
                                       int64_t kp_bs, int64_t kp_rs, const void* v, int64_t v_bs, int64_t v_rs,
                                       const float* we, float inv_temp, const float* w, const void* dctx,
                                       int64_t lddc, const float* dw_in, void* dqp, int64_t lddq, float* dwe_part,
                                       float* dbe_part, float* de_out, void* dctx_out, void* stream) {
  CAPK_CHECK_ARG(B > 0 && S > 0 && S <= SA_MAXS && D > 0 && de_out && dctx_out,
                 "capk_soft_attn_bwd_step: need 0 < S <= %d and the de / dctx stashes", SA_MAXS);
#define K(T, A) hipLaunchKernelGGL((soft_attn_bwd_kernel<T, A>), dim3(B, (D + 1023) / 1024), dim3(1024), 0, capk::S(stream), S, D, D, (const T*)qp, ldq, (const T*)kp, kp_bs, kp_rs, (const T*)v, v_bs, v_rs, we, inv_temp, w, (const T*)dctx, lddc, dw_in, (T*)dqp, lddq, (float*)nullptr, (float*)nullptr, dwe_part, dbe_part, de_out, (T*)dctx_out)
  DT2(dtype, K, 0);
#undef K
  CAPK_LAUNCH_CHECK("soft_attn_bwd_kernel(step)");
  return CAPK_OK;
}

extern "C" int capk_soft_attn_kv_grad(int dtype, int steps, int B, int S, int D, const void* qp, const void* kp,
                                      int64_t kp_bs, int64_t kp_rs, const float* we, const float* de_all,
                                      const float* w_all, const void* dctx_all, float* dkp, float* dv, void* stream) {
  CAPK_CHECK_ARG(steps > 0 && B > 0 && S > 0 && D > 0 && qp && kp && we && de_all && dkp && (!dv || (w_all && dctx_all)),
                 "capk_soft_attn_kv_grad: bad arguments");
#define K(T, _) hipLaunchKernelGGL((soft_attn_kv_grad_kernel<T, 0>), dim3(B * S), dim3(256), 0, capk::S(stream), steps, B, S, D, D, (const T*)qp, (const T*)kp, kp_bs, kp_rs, we, de_all, w_all, (const T*)dctx_all, dkp, dv)
  DT2(dtype, K, 0);
#undef K
  CAPK_LAUNCH_CHECK("soft_attn_kv_grad_kernel");
  return CAPK_OK;
}

extern "C" int capk_soft_attn_fwd(int dtype, int B, int S, int D, const void* qp, int64_t ldq, const void* kp,
                                  int64_t kp_bs, int64_t kp_rs, const void* v, int64_t v_bs, int64_t v_rs,
                                  const float* we, const float* be, float inv_temp, const uint8_t* key_pad, void* ctx,
                                  int64_t ldc, float* w_out, void* stream) {
  return capk_additive_attn_fwd(dtype, 0, B, S, D, D, qp, ldq, kp, kp_bs, kp_rs, v, v_bs, v_rs, we, be, inv_temp,
                                key_pad, ctx, ldc, w_out, stream);
}

extern "C" int capk_soft_attn_bwd(int dtype, int B, int S, int D, const void* qp, int64_t ldq, const void* kp,
                                  int64_t kp_bs, int64_t kp_rs, const void* v, int64_t v_bs, int64_t v_rs,
                                  const float* we, float inv_temp, const float* w, const void* dctx, int64_t lddc,
                                  const float* dw_in, void* dqp, int64_t lddq, float* dkp, float* dv, float* dwe_part,
                                  float* dbe_part, void* stream) {
  return capk_additive_attn_bwd(dtype, 0, B, S, D, D, qp, ldq, kp, kp_bs, kp_rs, v, v_bs, v_rs, we, inv_temp, w,
                                dctx, lddc, dw_in, dqp, lddq, dkp, dv, dwe_part, dbe_part, stream);
}
