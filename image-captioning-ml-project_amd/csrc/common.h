// Shared device/host helpers for libcapk (gfx950 only).
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "../../include/capk.h"

typedef __bf16 bf16;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace capk {

// ---------------------------------------------------------------- errors ----
void set_error(const char* fmt, ...);
int hip_status(hipError_t e, const char* what);

#define CAPK_CHECK_ARG(cond, ...)            \
  do {                                       \
    if (!(cond)) {                           \
      ::capk::set_error(__VA_ARGS__);        \
      return CAPK_EINVAL;                    \
    }                                        \
  } while (0)

#define CAPK_LAUNCH_CHECK(what)                                      \
  do {                                                               \
    hipError_t _e = hipGetLastError();                               \
    if (_e != hipSuccess) return ::capk::hip_status(_e, what);       \
  } while (0)

// ------------------------------------------------------------ conversions ---
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// vector of 8 elements of T <-> 8 floats
template <typename T> struct Vec8;
template <> struct Vec8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) {
    f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[8]) {
    f32x4 a = {v[0], v[1], v[2], v[3]}, b = {v[4], v[5], v[6], v[7]};
    *(f32x4*)p = a; *(f32x4*)(p + 4) = b;
  }
};
template <> struct Vec8<bf16> {
  __device__ __forceinline__ static void load(const bf16* p, float (&v)[8]) {
    bf16x8 a = *(const bf16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
  }
  __device__ __forceinline__ static void store(bf16* p, const float (&v)[8]) {
    bf16x8 a;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = (bf16)v[i];
    *(bf16x8*)p = a;
  }
};

// Deferred finishes (capk_finish_defer, misc.hip): while on (this host thread), the partial-sum
// finishes of the column-sum producers are queued per stream and launched together by
// capk_finish_flush -- out[n] (+)= the sum over nparts rows of part[r * ld + n], n < ncols, the
// same per-column sums as the single launches.  Returns false when deferral is off.
bool finish_enqueue(const float* part, int64_t ld, int nparts, int ncols, float* out, int accumulate, hipStream_t st);

// ------------------------------------------------------ partial-sum finish ---
// Column i of part[nparts][ld] summed over the parts ph, ph+PH, ph+2PH, ... with four
// independent accumulators (four loads in flight per thread).  The finish kernels run
// 16 columns x 64 part-phases per 1024-thread block and reduce the phases in LDS:
// deterministic, and the whole partial matrix is read in about one memory round trip.
template <int PH>
__device__ __forceinline__ float sum_parts(const float* __restrict__ part, int64_t ld, int nparts, int i, int ph) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = ph;
  for (; b + 3 * PH < nparts; b += 4 * PH) {
    s0 += part[(int64_t)b * ld + i];
    s1 += part[(int64_t)(b + PH) * ld + i];
    s2 += part[(int64_t)(b + 2 * PH) * ld + i];
    s3 += part[(int64_t)(b + 3 * PH) * ld + i];
  }
  for (; b < nparts; b += PH) s0 += part[(int64_t)b * ld + i];
  return (s0 + s1) + (s2 + s3);
}
// 1024-thread finish block: returns the column total in threads 0..15 (column blockIdx.x*16 + tid).
__device__ __forceinline__ float finish_parts16(const float* __restrict__ part, int64_t ld, int nparts, int ncols,
                                                int cb = -1) {  // cb: column block (default blockIdx.x)
  __shared__ float red[64][17];
  const int c = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int i = (cb < 0 ? (int)blockIdx.x : cb) * 16 + c;
  red[ph][c] = i < ncols ? sum_parts<64>(part, ld, nparts, i, ph) : 0.f;
  __syncthreads();
  if (threadIdx.x < 64) {  // 4 lanes per column, 16 phases each, then two shuffles
    const int cc = threadIdx.x & 15, q = threadIdx.x >> 4;
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) s += red[q * 16 + p][cc];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    return s;
  }
  return 0.f;
}

// ------------------------------------------------------------ activations ---
__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case CAPK_ACT_GELU_ERF: return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
    case CAPK_ACT_GELU_TANH: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      return 0.5f * x * (1.0f + tanhf(k0 * (x + k1 * x * x * x)));
    }
    case CAPK_ACT_QUICK_GELU: return x / (1.0f + __expf(-1.702f * x));
    case CAPK_ACT_TANH: return tanhf(x);
    case CAPK_ACT_RELU: return x > 0.f ? x : 0.f;
    case CAPK_ACT_SIGMOID: return 1.0f / (1.0f + __expf(-x));
    default: return x;
  }
}
// derivative d act(x) / dx
__device__ __forceinline__ float act_grad(int act, float x) {
  switch (act) {
    case CAPK_ACT_GELU_ERF: {
      float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
      float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
      return cdf + x * pdf;
    }
    case CAPK_ACT_GELU_TANH: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      float u = k0 * (x + k1 * x * x * x);
      float t = tanhf(u);
      return 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * k0 * (1.0f + 3.0f * k1 * x * x);
    }
    case CAPK_ACT_QUICK_GELU: {
      float s = 1.0f / (1.0f + __expf(-1.702f * x));
      return s + 1.702f * x * s * (1.0f - s);
    }
    case CAPK_ACT_TANH: { float t = tanhf(x); return 1.0f - t * t; }
    case CAPK_ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case CAPK_ACT_SIGMOID: { float sg = 1.0f / (1.0f + __expf(-x)); return sg * (1.0f - sg); }
    default: return 1.0f;
  }
}

// Fast GELU forms for the bf16 epilogues (GEMM epilogue / activation passes; the fp32 parity
// path keeps erff in act_fwd / act_grad above).  The erf-GELU is evaluated through its
// logistic (tanh) form x * sigmoid(2 sqrt(2/pi) (x + 0.044715 x^3)): one exp and one rcp,
// 7 VALU instructions (11 with the derivative) instead of 18 for Abramowitz & Stegun 7.1.26.
// It differs from x Phi(x) by <= 4.8e-4 absolute (derivative <= 8.7e-4), below the bf16
// resolution of the stored activations (2^-8 relative) -- the GELU epilogue runs while the
// CU's MFMAs idle, so its VALU count is exposed time.
constexpr float kGeluC0 = 1.5957691216057308f;               // 2 sqrt(2/pi)
constexpr float kGeluC1 = 0.0713548162726f;                  // 2 sqrt(2/pi) 0.044715
constexpr float kLog2eF = 1.4426950408889634f;
__device__ __forceinline__ float gelu_sig(float x, float u) {  // sigmoid(z), u = x^2
  // v_exp_f32 (2^t) and v_rcp_f32 (1 ulp) directly: __expf / __frcp_rn expand to range
  // reduction and a correctly rounded division (10 more instructions per element)
  const float t = x * fmaf(u, kGeluC1 * kLog2eF, kGeluC0 * kLog2eF);
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-t));
}
__device__ __forceinline__ float sig_fast(float x) {  // 1 / (1 + e^-x) on v_exp_f32 / v_rcp_f32
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x * kLog2eF));
}
// The GELU-family activations for bf16 storage: s = the logistic factor, z' = d(arg)/dx;
// act = x s, act' = s + x s (1 - s) z'.  GELU_TANH (GPT-2 gelu_new) IS this form exactly;
// GELU_ERF uses it as above; QUICK_GELU (CLIP) is x sigmoid(1.702 x).
__device__ __forceinline__ bool fast_family(int act) {
  return act == CAPK_ACT_GELU_ERF || act == CAPK_ACT_GELU_TANH || act == CAPK_ACT_QUICK_GELU;
}
__device__ __forceinline__ float fast_sig(int act, float x, float& zp) {
  if (act == CAPK_ACT_QUICK_GELU) {
    zp = 1.702f;
    return sig_fast(1.702f * x);
  }
  const float u = x * x;
  zp = fmaf(u, 3.0f * kGeluC1, kGeluC0);
  return gelu_sig(x, u);
}
// T: the storage type of the values; fp32 storage (the parity path's passes) keeps the exact
// forms (erff, tanhf, expf).
template <typename T>
__device__ __forceinline__ float act_fwd_fast(int act, float x) {
  if (!std::is_same<T, float>::value && fast_family(act)) {
    float zp;
    return x * fast_sig(act, x, zp);
  }
  return act_fwd(act, x);
}
template <typename T>
__device__ __forceinline__ float act_grad_fast(int act, float x) {
  if (!std::is_same<T, float>::value && fast_family(act)) {
    float zp;
    const float s = fast_sig(act, x, zp);
    return fmaf(x * fmaf(-s, s, s), zp, s);  // s + x s (1 - s) z'
  }
  return act_grad(act, x);
}
// Two elements at once on packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two lanes'
// worth per issue) for the GEMM epilogues, where the GELU-family math runs while the CU's
// MFMAs idle and its VALU issue count is the epilogue's time; the two transcendentals per
// element stay scalar.  Same formulas as act_fwd_fast / act_fwd_grad_fast above (bf16 storage
// only; the fp32 parity path never reaches these).
__device__ __forceinline__ f32x2 fast_sig2(int act, f32x2 x, f32x2& zp) {
  f32x2 t;
  if (act == CAPK_ACT_QUICK_GELU) {
    zp = (f32x2){1.702f, 1.702f};
    t = x * (1.702f * kLog2eF);
  } else {
    const f32x2 u = x * x;
    zp = u * (3.0f * kGeluC1) + kGeluC0;
    t = x * (u * (kGeluC1 * kLog2eF) + kGeluC0 * kLog2eF);
  }
  f32x2 e = {__builtin_amdgcn_exp2f(-t[0]), __builtin_amdgcn_exp2f(-t[1])};
  e = e + 1.0f;
  return (f32x2){__builtin_amdgcn_rcpf(e[0]), __builtin_amdgcn_rcpf(e[1])};
}
__device__ __forceinline__ f32x2 act_fwd_fast2(int act, f32x2 x) {
  f32x2 zp;
  return x * fast_sig2(act, x, zp);
}
__device__ __forceinline__ f32x2 act_fwd_grad_fast2(int act, f32x2 x, f32x2& d) {
  f32x2 zp;
  const f32x2 s = fast_sig2(act, x, zp);
  d = (x * (s - s * s)) * zp + s;  // s + x s (1 - s) z'
  return x * s;
}

// act(x) and act'(x) together (one logistic evaluation): CAPK_ACT_DERIV epilogues
template <typename T>
__device__ __forceinline__ float act_fwd_grad_fast(int act, float x, float& d) {
  if (!std::is_same<T, float>::value && fast_family(act)) {
    float zp;
    const float s = fast_sig(act, x, zp);
    d = fmaf(x * fmaf(-s, s, s), zp, s);
    return x * s;
  }
  d = act_grad(act, x);
  return act_fwd(act, x);
}

// --------------------------------------------------------------- dropout ----
// Counter-based dropout mask: keep(seed, idx) = fmix32(seed ^ mix(idx)) >= p * 2^32.
// The same (seed, idx) regenerates the identical mask in backward, so no mask tensor
// is stored.  Index conventions per site are documented in include/capk.h.
__host__ __device__ __forceinline__ uint32_t drop_hash(uint32_t seed, uint64_t idx) {
  uint32_t x = seed ^ ((uint32_t)idx * 0x9E3779B9u) ^ ((uint32_t)(idx >> 32) * 0x7FEB352Du);
  x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
  return x;
}
struct Drop {
  uint32_t thr;   // keep iff hash >= thr ; thr == 0 -> dropout off
  uint32_t seed;
  float scale;    // 1 / (1 - p)
  __device__ __forceinline__ bool on() const { return thr != 0; }
  __device__ __forceinline__ float mul(uint64_t idx) const { return drop_hash(seed, idx) >= thr ? scale : 0.f; }
};
inline Drop make_drop(float p, uint32_t seed) {
  Drop d;
  if (p <= 0.f) { d.thr = 0; d.seed = 0; d.scale = 1.f; return d; }
  double t = (double)p * 4294967296.0;
  d.thr = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  if (d.thr == 0) d.thr = 1;
  d.seed = seed;
  d.scale = 1.0f / (1.0f - p);
  return d;
}

// ------------------------------------------------------- wave reductions ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline hipStream_t S(void* s) { return (hipStream_t)s; }

}  // namespace capk
