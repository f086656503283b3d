// fp8 (OCP e4m3fn) operand quantisation for the scaled-MFMA GEMM (config 5, gemm8p.hip F8).
//
// Each output row r (an activation row, or a weight's output feature) gets one power-of-two
// scale 2^e, stored as its E8M0 code e + 127 -- the format v_mfma_scale_f32_16x16x128_f8f6f4
// takes per lane, so the GEMM applies the scales inside the MFMA and its epilogue is the
// bf16 one.  e is the smallest exponent with amax(row) * 2^-e <= 448 (e4m3fn's largest
// finite value): q = RNE_e4m3(x * 2^-e), exact scaling, no saturation needed.
//
//   rows mode       x [rows][cols] (ldx)      -> q [rows][cols] (ldq), one wave per row
//   transpose mode  x [cols][rows] (ldx)      -> q [rows][cols]: a Conv1D weight [in, out]
//                   (GPT-2) becomes the K-major [out][in] operand: column maxima (atomic max
//                   into the caller's workspace), then 64x64 tiles transposed through LDS.
//
// HBM-bound: reads 2 (bf16) or 4 (fp32) bytes and writes 1 byte per element.
#include "common.h"

namespace capk {

namespace {

// E8M0 code of the row scale for a row maximum |x| = amax (finite, >= 0).
__device__ __forceinline__ int scale_code(float amax) {
  if (!(amax > 0.f)) return 127;  // all-zero row: scale 1
  int ex;
  const float f = frexpf(amax, &ex);  // amax = f * 2^ex, f in [0.5, 1)
  // amax = (2f) * 2^(ex-1); (2f) * 2^(ex-1-e) <= 1.75 * 2^8  <=>  e >= ex - 9 (+1 if 2f > 1.75)
  const int e = ex - 9 + (f > 0.875f ? 1 : 0);
  return min(254, max(0, e + 127));
}
__device__ __forceinline__ float inv_scale(int code) { return ldexpf(1.f, 127 - code); }

__device__ __forceinline__ uint32_t pack4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&v)[8]) {
  Vec8<T>::load(p, v);
}

// rows mode: 4 waves per block, one row per wave; cols % 8 == 0.
template <typename T>
__global__ __launch_bounds__(256) void quant_rows_kernel(int rows, int cols, const T* __restrict__ x, int64_t ldx,
                                                         uint8_t* __restrict__ q, int64_t ldq,
                                                         uint8_t* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + (int64_t)row * ldx;
  float amax = 0.f;
  for (int c = lane * 8; c < cols; c += 512) {
    float v[8];
    load8(xr + c, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
  }
  amax = wave_max(amax);
  const int code = scale_code(amax);
  const float inv = inv_scale(code);
  uint8_t* qr = q + (int64_t)row * ldq;
  for (int c = lane * 8; c < cols; c += 512) {
    float v[8];
    load8(xr + c, v);
    uint2 w;
    w.x = pack4(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
    w.y = pack4(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv);
    *(uint2*)(qr + c) = w;
  }
  if (lane == 0) scale[row] = (uint8_t)code;
}

// transpose mode, pass 1: column maxima.  grid (ceil(rows/256), ceil(cols/64)); thread =
// one input column n (coalesced rows), 64 input rows; partial maxima combined with an
// atomic max on the fp32 bit pattern (non-negative floats order like their bits).
template <typename T>
__global__ __launch_bounds__(256) void amax_cols_kernel(int rows, int cols, const T* __restrict__ x, int64_t ldx,
                                                        uint32_t* __restrict__ amax) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= rows) return;
  const int k0 = blockIdx.y * 64, k1 = min(cols, k0 + 64);
  float m = 0.f;
#pragma unroll 8
  for (int k = k0; k < k1; ++k) m = fmaxf(m, fabsf(to_f32(x[(int64_t)k * ldx + n])));
  atomicMax(amax + n, __float_as_uint(m));
}

// transpose mode, pass 2: one 64 (output rows) x 64 (k) tile per block, grid
// (ceil(rows/64), ceil(cols/64)); staged through LDS and written K-contiguous (each thread
// 16 bytes = 16 k of one output row).
template <typename T>
__global__ __launch_bounds__(256) void quant_trans_kernel(int rows, int cols, const T* __restrict__ x, int64_t ldx,
                                                          const uint32_t* __restrict__ amax, uint8_t* __restrict__ q,
                                                          int64_t ldq, uint8_t* __restrict__ scale) {
  __shared__ float tile[64][65];
  __shared__ float sinv[64];
  const int tid = threadIdx.x, cl = tid & 63, rg = tid >> 6;
  const int r0 = blockIdx.x * 64;  // first output row = input column
  const int k0 = blockIdx.y * 64;
  const int n = r0 + cl;
  if (tid < 64) {
    const int code = scale_code(r0 + tid < rows ? __uint_as_float(amax[r0 + tid]) : 0.f);
    sinv[tid] = inv_scale(code);
    if (blockIdx.y == 0 && r0 + tid < rows) scale[r0 + tid] = (uint8_t)code;
  }
  __syncthreads();
  // load x[k0 + kk][r0 + cl] for kk = rg, rg+4, ...  (coalesced along n)
#pragma unroll 4
  for (int kk = rg; kk < 64; kk += 4) {
    const int k = k0 + kk;
    tile[kk][cl] = (k < cols && n < rows) ? to_f32(x[(int64_t)k * ldx + n]) * sinv[cl] : 0.f;
  }
  __syncthreads();
  const int rr = tid >> 2, c4 = tid & 3;
  const int kb = k0 + c4 * 16;
  if (r0 + rr < rows && kb < cols) {
    uint4 w;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = tile[c4 * 16 + i][rr];
    w.x = pack4(v[0], v[1], v[2], v[3]);
    w.y = pack4(v[4], v[5], v[6], v[7]);
    w.z = pack4(v[8], v[9], v[10], v[11]);
    w.w = pack4(v[12], v[13], v[14], v[15]);
    *(uint4*)(q + (int64_t)(r0 + rr) * ldq + kb) = w;
  }
}

}  // namespace
}  // namespace capk

using namespace capk;

extern "C" size_t capk_quant_fp8_workspace(int rows, int cols, int transpose) {
  (void)cols;
  return transpose ? (size_t)rows * sizeof(uint32_t) : 0;
}

extern "C" int capk_quant_fp8(int in_dtype, int rows, int cols, const void* x, int64_t ldx, int transpose, void* q,
                              int64_t ldq, void* scale, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(rows > 0 && cols > 0 && x && q && scale, "capk_quant_fp8: bad arguments");
  CAPK_CHECK_ARG(in_dtype == CAPK_BF16 || in_dtype == CAPK_F32, "capk_quant_fp8: in_dtype must be f32 or bf16");
  // rows mode stores 8 bytes per lane, transpose mode 16
  const int qa = transpose ? 16 : 8;
  CAPK_CHECK_ARG(ldq >= cols && ldq % qa == 0 && (uintptr_t)q % qa == 0,
                 "capk_quant_fp8: q must be %d-B aligned with ldq >= cols, ldq %% %d == 0", qa, qa);
  hipStream_t st = S(stream);
  if (!transpose) {
    const int esz = in_dtype == CAPK_F32 ? 4 : 2;
    CAPK_CHECK_ARG(cols % 8 == 0 && ldx >= cols && ldx % 8 == 0 && (uintptr_t)x % 16 == 0,
                   "capk_quant_fp8(rows): cols, ldx must be multiples of 8 with 16-B aligned x");
    (void)esz;
    const int grid = (rows + 3) / 4;
    if (in_dtype == CAPK_F32)
      hipLaunchKernelGGL(quant_rows_kernel<float>, dim3(grid), dim3(256), 0, st, rows, cols, (const float*)x, ldx,
                         (uint8_t*)q, ldq, (uint8_t*)scale);
    else
      hipLaunchKernelGGL(quant_rows_kernel<bf16>, dim3(grid), dim3(256), 0, st, rows, cols, (const bf16*)x, ldx,
                         (uint8_t*)q, ldq, (uint8_t*)scale);
  } else {
    CAPK_CHECK_ARG(cols % 16 == 0 && ldx >= rows, "capk_quant_fp8(transpose): cols %% 16 == 0, ldx >= rows");
    CAPK_CHECK_ARG(ws && ws_bytes >= (size_t)rows * 4 && (uintptr_t)ws % 4 == 0,
                   "capk_quant_fp8(transpose): workspace of capk_quant_fp8_workspace() bytes required");
    uint32_t* amax = (uint32_t*)ws;
    const hipError_t me = hipMemsetAsync(amax, 0, (size_t)rows * 4, st);
    if (me != hipSuccess) return hip_status(me, "capk_quant_fp8: hipMemsetAsync");
    const dim3 g1((rows + 255) / 256, (cols + 63) / 64), g2((rows + 63) / 64, (cols + 63) / 64);
    if (in_dtype == CAPK_F32) {
      hipLaunchKernelGGL(amax_cols_kernel<float>, g1, dim3(256), 0, st, rows, cols, (const float*)x, ldx, amax);
      hipLaunchKernelGGL(quant_trans_kernel<float>, g2, dim3(256), 0, st, rows, cols, (const float*)x, ldx, amax,
                         (uint8_t*)q, ldq, (uint8_t*)scale);
    } else {
      hipLaunchKernelGGL(amax_cols_kernel<bf16>, g1, dim3(256), 0, st, rows, cols, (const bf16*)x, ldx, amax);
      hipLaunchKernelGGL(quant_trans_kernel<bf16>, g2, dim3(256), 0, st, rows, cols, (const bf16*)x, ldx, amax,
                         (uint8_t*)q, ldq, (uint8_t*)scale);
    }
  }
  CAPK_LAUNCH_CHECK("capk_quant_fp8");
  return CAPK_OK;
}
