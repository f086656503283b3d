// Swin window attention (SwinEncoder, src/models/encoders.py:140-182 ->
// transformers SwinAttention / eager_attention_forward, modeling_swin.py:373-468) and the
// per-sample row scaling of SwinDropPath (modeling_swin.py:42-60).
//
// Rows are in window order: window w (= b * nW + window-in-image) owns rows
// [w*N, (w+1)*N), N = ws*ws, token t = r*ws + c of the (shifted) window.  The caller
// permutes the residual stream into that order (cyclic shift + window_partition are a row
// permutation, capk_gather_rows), so the kernels see plain [rows, 3C] QKV buffers.
//
//   s_ij = scale * q_i.k_j + table[idx(i,j), h] + (label_i != label_j ? -100 : 0)
//   idx(i,j) = (r_i - r_j + ws-1) * (2ws-1) + (c_i - c_j + ws-1)   (SwinRelativePositionBias)
//   p = softmax_j(s), o_i = sum_j p_ij v_j
//
// Windows are tiny (N = 49, hd = 32 for every published Swin): one wave per (window,
// head), one lane per query row, scores in registers, K/V in LDS read as broadcasts.  The
// FLOPs are ~1 % of a Swin block's (its GEMMs run on capk_gemm), so this is a latency /
// LDS kernel, not an MFMA one.  Backward recomputes the scores from the saved LSE, keeps P
// and dS of the window in LDS, forms dK/dV with one lane per key row, and reduces dS into
// the (2ws-1)^2 relative-position bins per window in a fixed order (deterministic); a
// finish kernel sums the per-window bins (fixed order, finish_parts16).
#include <algorithm>

#include "common.h"

namespace capk {

namespace {

constexpr int NMAX = 64;  // N = ws*ws <= 64

template <typename T, int HD>
__device__ __forceinline__ void load_row(const T* __restrict__ p, float (&v)[HD]) {
#pragma unroll
  for (int d = 0; d < HD; d += 8) {
    float t[8];
    Vec8<T>::load(p + d, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[d + e] = t[e];
  }
}
template <typename T, int HD>
__device__ __forceinline__ void store_row(T* __restrict__ p, const float (&v)[HD]) {
#pragma unroll
  for (int d = 0; d < HD; d += 8) {
    float t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = v[d + e];
    Vec8<T>::store(p + d, t);
  }
}
// rows [0, N) x HD columns of a head into an fp32 LDS image [N][HD] (whole wave)
template <typename T, int HD>
__device__ __forceinline__ void stage_rows(const T* __restrict__ g, int64_t ld, int N, float* s, int lane) {
  constexpr int SEGS = HD / 8;
  for (int u = lane; u < N * SEGS; u += 64) {
    const int r = u / SEGS, d = (u % SEGS) * 8;
    float t[8];
    Vec8<T>::load(g + (int64_t)r * ld + d, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[r * HD + d + e] = t[e];
  }
}
template <int HD>
__device__ __forceinline__ float dot_lds(const float (&q)[HD], const float* k) {
  float a = 0.f;
#pragma unroll
  for (int d = 0; d < HD; d += 4) {
    const f32x4 kv = *(const f32x4*)(k + d);
    a = fmaf(q[d], kv[0], a);
    a = fmaf(q[d + 1], kv[1], a);
    a = fmaf(q[d + 2], kv[2], a);
    a = fmaf(q[d + 3], kv[3], a);
  }
  return a;
}
template <int HD>
__device__ __forceinline__ void axpy_lds(float (&o)[HD], float p, const float* v) {
#pragma unroll
  for (int d = 0; d < HD; d += 4) {
    const f32x4 vv = *(const f32x4*)(v + d);
    o[d] = fmaf(p, vv[0], o[d]);
    o[d + 1] = fmaf(p, vv[1], o[d + 1]);
    o[d + 2] = fmaf(p, vv[2], o[d + 2]);
    o[d + 3] = fmaf(p, vv[3], o[d + 3]);
  }
}

struct WinArgs {
  int nwin, nw_img, ws, H, C;
  float scale;
  const void* qkv;
  int64_t ldq;
  const float* table;    // [(2ws-1)^2, H]
  const int32_t* label;  // [nw_img, N] shift-region labels, or null (no shift mask)
  const void* o;
  int64_t ldo;
  const void* dout;
  int64_t lddo;
  float* lse;            // [nwin, H, N]
  void* dqkv;
  int64_t lddq;
  float* part;           // [nwin, NB*H] per-window bias-gradient bins
};

// scores of query row i (lane) against every key of the window: s[j], j < N
template <int HD>
__device__ __forceinline__ void window_scores(const WinArgs& a, const float (&q)[HD], const float* Ks,
                                              const float* tab, const int* lab, int i, int N, float (&s)[NMAX]) {
  const int ws = a.ws, ri = i / ws, ci = i - ri * ws, w2 = 2 * ws - 1;
  const int li = lab ? lab[i] : 0;
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    if (j < N) {
      const int rj = j / ws, cj = j - rj * ws;
      float v = a.scale * dot_lds<HD>(q, Ks + j * HD) + tab[(ri - rj + ws - 1) * w2 + (ci - cj + ws - 1)];
      if (lab && lab[j] != li) v += -100.f;
      s[j] = v;
    } else {
      s[j] = -INFINITY;
    }
  }
}

// one wave per (window, head); 4 waves per block
template <typename T, int HD>
__global__ __launch_bounds__(256) void window_attn_fwd_kernel(WinArgs a) {
  const int N = a.ws * a.ws, NB = (2 * a.ws - 1) * (2 * a.ws - 1);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __shared__ __attribute__((aligned(16))) float sK[4][NMAX * HD];
  __shared__ __attribute__((aligned(16))) float sV[4][NMAX * HD];
  __shared__ float sTab[4][225];
  __shared__ int sLab[4][NMAX];
  const int total = a.nwin * a.H;
  const bool valid = blockIdx.x * 4 + wave < total;
  const int unit = valid ? blockIdx.x * 4 + wave : total - 1;  // a spare wave recomputes the last unit, stores nothing
  const int win = unit / a.H, h = unit - win * a.H;
  const T* base = (const T*)a.qkv + (int64_t)win * N * a.ldq + h * HD;
  stage_rows<T, HD>(base + a.C, a.ldq, N, sK[wave], lane);
  stage_rows<T, HD>(base + 2 * a.C, a.ldq, N, sV[wave], lane);
  for (int b = lane; b < NB; b += 64) sTab[wave][b] = a.table[b * a.H + h];
  const int* lab = nullptr;
  if (a.label) {
    const int32_t* L = a.label + (int64_t)(win % a.nw_img) * N;
    if (lane < N) sLab[wave][lane] = L[lane];
    lab = sLab[wave];
  }
  __syncthreads();
  const int i = lane < N ? lane : N - 1;  // idle lanes recompute row N-1 and store nothing
  float q[HD];
  load_row<T, HD>(base + (int64_t)i * a.ldq, q);
  float s[NMAX];
  window_scores<HD>(a, q, sK[wave], sTab[wave], lab, i, N, s);
  float m = s[0];
#pragma unroll
  for (int j = 1; j < NMAX; ++j) m = fmaxf(m, s[j]);
  float l = 0.f;
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    s[j] = j < N ? __expf(s[j] - m) : 0.f;
    l += s[j];
  }
  const float inv = 1.f / l;
  float o[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) o[d] = 0.f;
#pragma unroll
  for (int j = 0; j < NMAX; ++j)
    if (j < N) axpy_lds<HD>(o, s[j] * inv, sV[wave] + j * HD);
  if (valid && lane < N) {
    store_row<T, HD>((T*)a.o + ((int64_t)win * N + i) * a.ldo + h * HD, o);
    a.lse[((int64_t)win * a.H + h) * N + i] = m + __logf(l);
  }
}

// one wave per (window, head), one wave per block (P and dS of the window in LDS)
template <typename T, int HD>
__global__ __launch_bounds__(64) void window_attn_bwd_kernel(WinArgs a) {
  const int N = a.ws * a.ws, ws = a.ws, w2 = 2 * ws - 1, NB = w2 * w2;
  const int lane = threadIdx.x;
  __shared__ __attribute__((aligned(16))) float sK[NMAX * HD];
  __shared__ __attribute__((aligned(16))) float sV[NMAX * HD];
  __shared__ __attribute__((aligned(16))) float sQ[NMAX * HD];
  __shared__ __attribute__((aligned(16))) float sD[NMAX * HD];  // dO rows
  __shared__ float sP[NMAX * NMAX];
  __shared__ float sS[NMAX * NMAX];  // dS
  __shared__ float sTab[225];
  __shared__ int sLab[NMAX];
  const int win = blockIdx.x / a.H, h = blockIdx.x - win * a.H;
  const T* base = (const T*)a.qkv + (int64_t)win * N * a.ldq + h * HD;
  stage_rows<T, HD>(base, a.ldq, N, sQ, lane);
  stage_rows<T, HD>(base + a.C, a.ldq, N, sK, lane);
  stage_rows<T, HD>(base + 2 * a.C, a.ldq, N, sV, lane);
  stage_rows<T, HD>((const T*)a.dout + (int64_t)win * N * a.lddo + h * HD, a.lddo, N, sD, lane);
  for (int b = lane; b < NB; b += 64) sTab[b] = a.table[b * a.H + h];
  const int* lab = nullptr;
  if (a.label) {
    const int32_t* L = a.label + (int64_t)(win % a.nw_img) * N;
    if (lane < N) sLab[lane] = L[lane];
    lab = sLab;
  }
  __syncthreads();
  const int i = lane < N ? lane : N - 1;
  float q[HD], g[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    q[d] = sQ[i * HD + d];
    g[d] = sD[i * HD + d];
  }
  float ov[HD];
  load_row<T, HD>((const T*)a.o + ((int64_t)win * N + i) * a.ldo + h * HD, ov);
  float Di = 0.f;
#pragma unroll
  for (int d = 0; d < HD; ++d) Di = fmaf(g[d], ov[d], Di);
  const float lse = a.lse[((int64_t)win * a.H + h) * N + i];
  float s[NMAX];
  window_scores<HD>(a, q, sK, sTab, lab, i, N, s);
  float dq[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) dq[d] = 0.f;
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    if (j < N) {
      const float p = __expf(s[j] - lse);
      const float dp = dot_lds<HD>(g, sV + j * HD);
      const float ds = p * (dp - Di);
      if (lane < N) {
        sP[i * N + j] = p;
        sS[i * N + j] = ds;
      }
      axpy_lds<HD>(dq, ds * a.scale, sK + j * HD);
    }
  }
  T* dbase = (T*)a.dqkv + (int64_t)win * N * a.lddq + h * HD;
  if (lane < N) store_row<T, HD>(dbase + (int64_t)i * a.lddq, dq);
  __syncthreads();
  // key rows: dK_j = scale * sum_i dS_ij q_i, dV_j = sum_i P_ij dO_i
  const int j = i;
  float dk[HD], dv[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) dk[d] = dv[d] = 0.f;
  for (int r = 0; r < N; ++r) {
    axpy_lds<HD>(dk, sS[r * N + j] * a.scale, sQ + r * HD);
    axpy_lds<HD>(dv, sP[r * N + j], sD + r * HD);
  }
  if (lane < N) {
    store_row<T, HD>(dbase + a.C + (int64_t)j * a.lddq, dk);
    store_row<T, HD>(dbase + 2 * a.C + (int64_t)j * a.lddq, dv);
  }
  // relative-position bins: bin (dr, dc) sums dS_ij over r_i - r_j = dr, c_i - c_j = dc,
  // in ascending i (fixed order)
  for (int b = lane; b < NB; b += 64) {
    const int dr = b / w2 - (ws - 1), dc = b % w2 - (ws - 1);
    float acc = 0.f;
    for (int ii = 0; ii < N; ++ii) {
      const int ri = ii / ws, ci = ii - ri * ws, rj = ri - dr, cj = ci - dc;
      if (rj >= 0 && rj < ws && cj >= 0 && cj < ws) acc += sS[ii * N + rj * ws + cj];
    }
    a.part[(int64_t)win * NB * a.H + b * a.H + h] = acc;
  }
}

__global__ __launch_bounds__(1024) void window_bias_finish_kernel(int nwin, int ncols, const float* __restrict__ part,
                                                                  float* __restrict__ out, int accumulate) {
  const float s = finish_parts16(part, ncols, nwin, ncols);
  const int c = blockIdx.x * 16 + threadIdx.x;
  if (threadIdx.x < 16 && c < ncols) out[c] = accumulate ? out[c] + s : s;
}

template <typename T>
__global__ void rowscale_add_kernel(int rows, int cols, const T* __restrict__ x, int64_t ldx,
                                    const float* __restrict__ scale, int group_rows, const T* __restrict__ res,
                                    int64_t ldr, T* __restrict__ y, int64_t ldy) {
  const int segs = cols / 8;
  const int64_t n = (int64_t)rows * segs;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(u / segs), c = (int)(u - (int64_t)r * segs) * 8;
    const float sc = scale[r / group_rows];
    float v[8];
    Vec8<T>::load(x + (int64_t)r * ldx + c, v);
    if (res) {
      float rv[8];
      Vec8<T>::load(res + (int64_t)r * ldr + c, rv);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaf(v[e], sc, rv[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= sc;
    }
    Vec8<T>::store(y + (int64_t)r * ldy + c, v);
  }
}

int check_win(int dtype, int nwin, int nw_img, int ws, int H, int hd, int C) {
  CAPK_CHECK_ARG(dtype == CAPK_F32 || dtype == CAPK_BF16, "capk_window_attn: dtype");
  CAPK_CHECK_ARG(nwin > 0 && nw_img > 0 && nwin % nw_img == 0, "capk_window_attn: nwin %% nw_img != 0");
  CAPK_CHECK_ARG(ws >= 1 && ws * ws <= NMAX && (2 * ws - 1) * (2 * ws - 1) <= 225,
                 "capk_window_attn: window %d (need ws*ws <= 64)", ws);
  CAPK_CHECK_ARG(hd == 32 && H > 0 && C == H * hd, "capk_window_attn: head dim %d (built for 32), C=%d H=%d", hd, C,
                 H);
  return CAPK_OK;
}

}  // namespace

}  // namespace capk

using namespace capk;

extern "C" int capk_window_attn_fwd(int dtype, int nwin, int nw_img, int ws, int H, int hd, float scale,
                                    const void* qkv, int64_t ldq, int C, const float* table, const int32_t* labels,
                                    void* out, int64_t ldo, float* lse, void* stream) {
  const int rc = check_win(dtype, nwin, nw_img, ws, H, hd, C);
  if (rc != CAPK_OK) return rc;
  CAPK_CHECK_ARG(qkv && table && out && lse && ldq % 8 == 0 && ldo % 8 == 0 && ldq >= 3 * C,
                 "capk_window_attn_fwd: operands / strides");
  WinArgs a{nwin, nw_img, ws, H, C, scale, qkv, ldq, table, labels, out, ldo, nullptr, 0, lse, nullptr, 0, nullptr};
  const int grid = cdiv((int64_t)nwin * H, 4);
  if (dtype == CAPK_BF16)
    hipLaunchKernelGGL((window_attn_fwd_kernel<bf16, 32>), dim3(grid), dim3(256), 0, S(stream), a);
  else
    hipLaunchKernelGGL((window_attn_fwd_kernel<float, 32>), dim3(grid), dim3(256), 0, S(stream), a);
  CAPK_LAUNCH_CHECK("window_attn_fwd_kernel");
  return CAPK_OK;
}

extern "C" size_t capk_window_attn_bwd_workspace(int nwin, int ws, int H) {
  return (size_t)nwin * (2 * ws - 1) * (2 * ws - 1) * H * sizeof(float);
}

extern "C" int capk_window_attn_bwd(int dtype, int nwin, int nw_img, int ws, int H, int hd, float scale,
                                    const void* qkv, int64_t ldq, int C, const float* table, const int32_t* labels,
                                    const void* out, int64_t ldo, const void* dout, int64_t lddo, const float* lse,
                                    void* dqkv, int64_t lddq, float* dtable, int accumulate, void* wsp,
                                    size_t ws_bytes, void* stream) {
  const int rc = check_win(dtype, nwin, nw_img, ws, H, hd, C);
  if (rc != CAPK_OK) return rc;
  CAPK_CHECK_ARG(qkv && table && out && dout && lse && dqkv && dtable, "capk_window_attn_bwd: null operand");
  CAPK_CHECK_ARG(ldq % 8 == 0 && ldo % 8 == 0 && lddo % 8 == 0 && lddq % 8 == 0 && ldq >= 3 * C && lddq >= 3 * C,
                 "capk_window_attn_bwd: strides");
  CAPK_CHECK_ARG(wsp && ws_bytes >= capk_window_attn_bwd_workspace(nwin, ws, H), "capk_window_attn_bwd: workspace");
  WinArgs a{nwin, nw_img, ws, H, C, scale, qkv, ldq, table, labels, out, ldo, dout, lddo, const_cast<float*>(lse),
            dqkv, lddq, (float*)wsp};
  const int grid = nwin * H;
  if (dtype == CAPK_BF16)
    hipLaunchKernelGGL((window_attn_bwd_kernel<bf16, 32>), dim3(grid), dim3(64), 0, S(stream), a);
  else
    hipLaunchKernelGGL((window_attn_bwd_kernel<float, 32>), dim3(grid), dim3(64), 0, S(stream), a);
  CAPK_LAUNCH_CHECK("window_attn_bwd_kernel");
  const int ncols = (2 * ws - 1) * (2 * ws - 1) * H;
  hipLaunchKernelGGL(window_bias_finish_kernel, dim3(cdiv(ncols, 16)), dim3(1024), 0, S(stream), nwin, ncols,
                     (const float*)wsp, dtable, accumulate);
  CAPK_LAUNCH_CHECK("window_bias_finish_kernel");
  return CAPK_OK;
}

extern "C" int capk_rowscale_add(int dtype, int rows, int cols, const void* x, int64_t ldx, const float* scale,
                                 int group_rows, const void* res, int64_t ldr, void* y, int64_t ldy, void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && (!res || ldr % 8 == 0) &&
                     group_rows > 0 && scale,
                 "capk_rowscale_add: shape / strides");
  const int64_t n = (int64_t)rows * (cols / 8);
  const int grid = (int)std::min<int64_t>(cdiv(n, 256), 8192);
  if (dtype == CAPK_BF16)
    hipLaunchKernelGGL(rowscale_add_kernel<bf16>, dim3(grid), dim3(256), 0, S(stream), rows, cols, (const bf16*)x, ldx,
                       scale, group_rows, (const bf16*)res, ldr, (bf16*)y, ldy);
  else if (dtype == CAPK_F32)
    hipLaunchKernelGGL(rowscale_add_kernel<float>, dim3(grid), dim3(256), 0, S(stream), rows, cols, (const float*)x,
                       ldx, scale, group_rows, (const float*)res, ldr, (float*)y, ldy);
  else
    CAPK_CHECK_ARG(false, "capk_rowscale_add: dtype");
  CAPK_LAUNCH_CHECK("rowscale_add_kernel");
  return CAPK_OK;
}
