// GEMM for the captioning hot path (every nn.Linear / Conv1D / patch-conv and
// both of its backward products).  Two paths:
//
//  * bf16 (throughput): 128x128x64 block tile, 4 waves (2x2, 64x64 per wave),
//    v_mfma_f32_16x16x32_bf16, fp32 accumulation.  Operand tiles are staged
//    HBM -> LDS with global_load_lds (16 B / lane, lane-linear LDS image, XOR
//    swizzle applied on the per-lane SOURCE address).  K-major operands are read
//    with ds_read_b128, M/N-major (transposed) operands with ds_read_b64_tr_b16,
//    so dX = dY W and dW = dY^T X need no transpose kernels.  Double-buffered,
//    one barrier per K-tile.  XCD-aware block->tile remap so tiles that share an
//    A panel run on one XCD's L2.  Split-K writes fp32 slabs that a reduce
//    kernel sums (deterministic) and finishes with the same epilogue.
//  * f32 (parity): exact-f32 v_mfma_f32_16x16x4_f32, arbitrary strides, 64x64x16
//    tile; used for the fp32 parity mode that must match the CPU reference.
//
// Epilogue (both): alpha*acc + beta*C + bias[n] + residual[m,n], then forward
// activation (optionally saving the pre-activation) or the backward form
// acc * act'(aux).  bias is fp32; C/residual/preact/aux use the output dtype.
#include "common.h"

namespace capk {

struct Epi {
  void* C;
  int64_t ldc;
  float alpha, beta;
  const float* bias;
  const void* res;
  int64_t ldr;
  int act;
  void* pre;
  const void* aux;
  int64_t ldx;
  int M, N;
};

template <typename OutT>
__device__ __forceinline__ void epilogue8(const Epi& e, int m, int n, float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] *= e.alpha;
  if (e.beta != 0.f) {
    float c[8];
    Vec8<OutT>::load((const OutT*)e.C + (int64_t)m * e.ldc + n, c);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += e.beta * c[i];
  }
  if (e.bias) {
    float b[8];
    Vec8<float>::load(e.bias + n, b);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += b[i];
  }
  if (e.res) {
    float r[8];
    Vec8<OutT>::load((const OutT*)e.res + (int64_t)m * e.ldr + n, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += r[i];
  }
  if (e.act & CAPK_ACT_BWD) {
    float a[8];
    Vec8<OutT>::load((const OutT*)e.aux + (int64_t)m * e.ldx + n, a);
    const int act = e.act & 15;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] *= act_grad(act, a[i]);
  } else if (e.act) {
    if (e.pre) Vec8<OutT>::store((OutT*)e.pre + (int64_t)m * e.ldx + n, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = act_fwd(e.act, v[i]);
  }
  Vec8<OutT>::store((OutT*)e.C + (int64_t)m * e.ldc + n, v);
}

template <typename OutT>
__device__ __forceinline__ void epilogue1(const Epi& e, int m, int n, float v) {
  v *= e.alpha;
  if (e.beta != 0.f) v += e.beta * to_f32(((const OutT*)e.C)[(int64_t)m * e.ldc + n]);
  if (e.bias) v += e.bias[n];
  if (e.res) v += to_f32(((const OutT*)e.res)[(int64_t)m * e.ldr + n]);
  if (e.act & CAPK_ACT_BWD) {
    v *= act_grad(e.act & 15, to_f32(((const OutT*)e.aux)[(int64_t)m * e.ldx + n]));
  } else if (e.act) {
    if (e.pre) ((OutT*)e.pre)[(int64_t)m * e.ldx + n] = from_f32<OutT>(v);
    v = act_fwd(e.act, v);
  }
  ((OutT*)e.C)[(int64_t)m * e.ldc + n] = from_f32<OutT>(v);
}

// XCD-aware bijective remap: blocks dealt round-robin over 8 XCDs become
// contiguous chunks of the tile sequence per XCD (cdna guide T1, bijective form).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ============================================================ bf16 kernel ===
constexpr int BM = 128, BN = 128, BKT = 64;
constexpr int TILE_BYTES = BM * BKT * 2;             // 16 KiB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;          // A + B
constexpr int EPI_LD = BN + 4;                       // fp32 staging row (floats)
constexpr int EPI_BYTES = BM * EPI_LD * 4;
constexpr int SMEM_BYTES = (2 * STAGE_BYTES > EPI_BYTES) ? 2 * STAGE_BYTES : EPI_BYTES;

// K-major image [128 rows][64 k] (128-B rows): 16-B chunk c of row r stored at
// chunk c ^ ((r>>1)&7) -> conflict-free ds_read_b128 for the 16x16x32 operand.
__device__ __forceinline__ int swz_k(int r) { return (r >> 1) & 7; }
// MN-major image [64 k][128 mn] (256-B rows): chunk c of k-row r stored at
// c ^ (f(r)<<1), f(r) = (r&3) | ((r>>3)&1)<<2 -> conflict-free ds_read_b64_tr_b16.
__device__ __forceinline__ int swz_t(int r) { return (((r & 3) | (((r >> 3) & 1) << 2)) << 1); }

// Stage one 128 x 64 operand tile into LDS (16 KiB, 4 x 1-KiB pieces per wave).
// K-major operands use global_load_lds; MN-major (transposed) operands use
// range-checked buffer_load ... lds whose descriptor ends at row K, so K-tail rows
// of a split reduction (token counts that are not multiples of 64) read as 0.
template <bool KMAJ>
__device__ __forceinline__ void stage_tile(const bf16* __restrict__ X, int64_t ld, int rows, int row0,
                                           int k0, char* lds_tile, int wave, int lane, __amdgpu_buffer_rsrc_t rsrc) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ins = wave * 4 + t;
    if constexpr (KMAJ) {
      const int r = ins * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ swz_k(r);
      int gr = row0 + r;
      gr = gr < rows ? gr : rows - 1;
      const bf16* src = X + (int64_t)gr * ld + k0 + lc * 8;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds_tile + ins * 1024), 16, 0, 0);
    } else {
      const int kr = ins * 4 + (lane >> 4);
      const int lc = (lane & 15) ^ swz_t(kr);
      int gc = row0 + lc * 8;
      gc = gc + 8 <= rows ? gc : rows - 8;
      const unsigned voff = (unsigned)(((int64_t)(k0 + kr) * ld + gc) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(lds_tile + ins * 1024),
                                               16, voff, 0, 0, 0);
    }
  }
}

template <bool KMAJ>
__device__ __forceinline__ bf16x8 read_frag(const char* tile, int rbase, int s, int lane) {
  if constexpr (KMAJ) {
    const int r = rbase + (lane & 15);
    const int lc = s * 4 + (lane >> 4);
    return *(const bf16x8*)(tile + r * 128 + ((lc ^ swz_k(r)) << 4));
  } else {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
    const int lc = (rbase >> 3) + (p >> 1);
    const int kr0 = s * 32 + g * 8 + q, kr1 = kr0 + 4;
    const char* a0 = tile + kr0 * 256 + ((lc ^ swz_t(kr0)) << 4) + (p & 1) * 8;
    const char* a1 = tile + kr1 * 256 + ((lc ^ swz_t(kr1)) << 4) + (p & 1) * 8;
    bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, a0));
    bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, a1));
    bf16x8 r;
    r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
    r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
    return r;
  }
}

template <bool AK, bool BK, typename OutT>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(const bf16* __restrict__ A, int64_t lda,
                                                           const bf16* __restrict__ B, int64_t ldb,
                                                           int M, int N, int K, int splits, Epi e,
                                                           float* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN, ntiles = ntm * ntn;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles, tile = wg % ntiles;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int nk_all = (K + BKT - 1) / BKT;
  // range-checked descriptors for MN-major operands: [0, K*ld) elements are valid
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)((int64_t)K * lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)((int64_t)K * ldb * 2), 0x00020000);
  const int kt_per = (nk_all + splits - 1) / splits;
  const int kt0 = split * kt_per;
  const int kt1 = min(nk_all, kt0 + kt_per);
  const int nk = max(0, kt1 - kt0);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    stage_tile<AK>(A, lda, M, m0, kt0 * BKT, smem, wave, lane, rsA);
    stage_tile<BK>(B, ldb, N, n0, kt0 * BKT, smem + TILE_BYTES, wave, lane, rsB);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    char* sc = smem + cur * STAGE_BYTES;
    if (kt + 1 < nk) {
      char* sn = smem + (cur ^ 1) * STAGE_BYTES;
      stage_tile<AK>(A, lda, M, m0, (kt0 + kt + 1) * BKT, sn, wave, lane, rsA);
      stage_tile<BK>(B, ldb, N, n0, (kt0 + kt + 1) * BKT, sn + TILE_BYTES, wave, lane, rsB);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<AK>(sc, wm * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<BK>(sc + TILE_BYTES, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: accumulators -> LDS (fp32, row-major) -> 8-wide rows
  float* stg = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int col = wn * 64 + j * 16 + (lane & 15);
        stg[row * EPI_LD + col] = acc[i][j][r];
      }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = it * 256 + tid;
    const int row = idx >> 4, col = (idx & 15) * 8;
    const int gm = m0 + row, gn = n0 + col;
    if (gm >= M || gn >= N) continue;
    float v[8];
    Vec8<float>::load(stg + row * EPI_LD + col, v);
    if (ws) {
      Vec8<float>::store(ws + ((int64_t)split * M + gm) * N + gn, v);
    } else {
      epilogue8<OutT>(e, gm, gn, v);
    }
  }
}

// split-K finish: sum the fp32 slabs, then the regular epilogue.
template <typename OutT>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, Epi e) {
  const int64_t n8 = (int64_t)e.M * e.N / 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t off = i * 8;
    const int m = (int)(off / e.N), n = (int)(off % e.N);
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < splits; ++s) {
      float t[8];
      Vec8<float>::load(ws + (int64_t)s * e.M * e.N + off, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += t[k];
    }
    epilogue8<OutT>(e, m, n, v);
  }
}

// ============================================================= f32 kernel ===
// Exact fp32 (parity mode).  A(m,k) = A[m*sam + k*sak], B(n,k) = B[n*sbn + k*sbk].
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, int64_t sam, int64_t sak,
                                                       const float* __restrict__ B, int64_t sbn, int64_t sbk,
                                                       int M, int N, int K, Epi e) {
  __shared__ float As[16][68];
  __shared__ float Bs[16][68];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = (N + 63) / 64;
  const int m0 = (blockIdx.x / ntn) * 64, n0 = (blockIdx.x % ntn) * 64;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const bool a_kc = (sak == 1), b_kc = (sbk == 1);
  for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int eidx = tid + 256 * r;
      int mm, kk;
      if (a_kc) { mm = eidx >> 4; kk = eidx & 15; } else { mm = eidx & 63; kk = eidx >> 6; }
      const int gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < M && gk < K) ? A[(int64_t)gm * sam + (int64_t)gk * sak] : 0.f;
      int nn;
      if (b_kc) { nn = eidx >> 4; kk = eidx & 15; } else { nn = eidx & 63; kk = eidx >> 6; }
      const int gn = n0 + nn, gk2 = k0 + kk;
      Bs[kk][nn] = (gn < N && gk2 < K) ? B[(int64_t)gn * sbn + (int64_t)gk2 * sbk] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[ks * 4 + (lane >> 4)][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[ks * 4 + (lane >> 4)][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int gn = n0 + wn * 32 + j * 16 + (lane & 15);
        if (gm < M && gn < N) epilogue1<float>(e, gm, gn, acc[i][j][r]);
      }
}

static int choose_splits(int M, int N, int K) {
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  const int nk = cdiv(K, BKT);
  int s = 1;
  // aim for >= 2 waves of workgroups over 256 CUs (2 WGs/CU resident)
  while (tiles * s < 512 && s * 2 <= 16 && nk / (s * 2) >= 4) s *= 2;
  return s;
}

}  // namespace capk

using namespace capk;

extern "C" size_t capk_gemm_workspace(int in_dtype, int out_dtype, int M, int N, int K) {
  (void)out_dtype;
  if (in_dtype != CAPK_BF16) return 0;
  const int s = choose_splits(M, N, K);
  return s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
}

extern "C" int capk_gemm(int in_dtype, int out_dtype, int M, int N, int K, const void* A, int64_t lda,
                         int a_kmajor, const void* B, int64_t ldb, int b_kmajor, void* C, int64_t ldc,
                         float alpha, float beta, const float* bias, const void* residual, int64_t ldr,
                         int act, void* preact, const void* aux, int64_t ldx, void* ws, size_t ws_bytes,
                         void* stream) {
  CAPK_CHECK_ARG(M > 0 && N > 0 && K > 0, "capk_gemm: bad sizes M=%d N=%d K=%d", M, N, K);
  CAPK_CHECK_ARG(A && B && C, "capk_gemm: null operand");
  CAPK_CHECK_ARG(!(act & CAPK_ACT_BWD) || aux, "capk_gemm: backward activation needs aux");
  Epi e{C, ldc, alpha, beta, bias, residual, ldr, act, preact, aux, ldx, M, N};
  hipStream_t st = S(stream);
  if (in_dtype == CAPK_F32) {
    CAPK_CHECK_ARG(out_dtype == CAPK_F32, "capk_gemm: f32 inputs need f32 output");
    const int64_t sam = a_kmajor ? lda : 1, sak = a_kmajor ? 1 : lda;
    const int64_t sbn = b_kmajor ? ldb : 1, sbk = b_kmajor ? 1 : ldb;
    const int grid = cdiv(M, 64) * cdiv(N, 64);
    hipLaunchKernelGGL(gemm_f32_kernel, dim3(grid), dim3(256), 0, st, (const float*)A, sam, sak,
                       (const float*)B, sbn, sbk, M, N, K, e);
    CAPK_LAUNCH_CHECK("gemm_f32_kernel");
    return CAPK_OK;
  }
  CAPK_CHECK_ARG(in_dtype == CAPK_BF16, "capk_gemm: unknown in_dtype %d", in_dtype);
  CAPK_CHECK_ARG(out_dtype == CAPK_BF16 || out_dtype == CAPK_F32, "capk_gemm: unknown out_dtype");
  CAPK_CHECK_ARG(!(a_kmajor || b_kmajor) || K % BKT == 0,
                 "capk_gemm(bf16): K=%d must be a multiple of %d when an operand is K-major", K, BKT);
  CAPK_CHECK_ARG(N % 8 == 0, "capk_gemm(bf16): N=%d must be a multiple of 8", N);
  CAPK_CHECK_ARG(a_kmajor || (M % 8 == 0 && M >= 8), "capk_gemm(bf16): M-major A needs M %% 8 == 0");
  CAPK_CHECK_ARG(b_kmajor || (N % 8 == 0 && N >= 8), "capk_gemm(bf16): N-major B needs N %% 8 == 0");
  CAPK_CHECK_ARG((a_kmajor || (int64_t)K * lda * 2 < (1ll << 31)) && (b_kmajor || (int64_t)K * ldb * 2 < (1ll << 31)),
                 "capk_gemm(bf16): MN-major operand larger than 2 GiB");
  const int64_t esz = out_dtype == CAPK_F32 ? 4 : 2;
  CAPK_CHECK_ARG(((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % 8 == 0 && ldb % 8 == 0,
                 "capk_gemm(bf16): A/B must be 16-B aligned with lda, ldb %% 8 == 0");
  CAPK_CHECK_ARG(((uintptr_t)C % 16 == 0) && (ldc * esz) % 16 == 0, "capk_gemm(bf16): C alignment");
  int splits = choose_splits(M, N, K);
  if (!ws || ws_bytes < (size_t)splits * M * N * sizeof(float)) splits = 1;
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  const int grid = tiles * splits;
  float* slab = splits > 1 ? (float*)ws : nullptr;
#define LAUNCH(AK, BKM, OT)                                                                               \
  hipLaunchKernelGGL((gemm_bf16_kernel<AK, BKM, OT>), dim3(grid), dim3(256), 0, st, (const bf16*)A, lda, \
                     (const bf16*)B, ldb, M, N, K, splits, e, slab)
#define DISPATCH(OT)                          \
  if (a_kmajor && b_kmajor) LAUNCH(true, true, OT);     \
  else if (a_kmajor) LAUNCH(true, false, OT);           \
  else if (b_kmajor) LAUNCH(false, true, OT);           \
  else LAUNCH(false, false, OT);
  if (out_dtype == CAPK_BF16) { DISPATCH(bf16) } else { DISPATCH(float) }
#undef DISPATCH
#undef LAUNCH
  CAPK_LAUNCH_CHECK("gemm_bf16_kernel");
  if (splits > 1) {
    const int64_t n8 = (int64_t)M * N / 8;
    const int g = (int)std::min<int64_t>(2048, (n8 + 255) / 256);
    if (out_dtype == CAPK_BF16)
      hipLaunchKernelGGL(splitk_reduce_kernel<bf16>, dim3(g), dim3(256), 0, st, (const float*)ws, splits, e);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)ws, splits, e);
    CAPK_LAUNCH_CHECK("splitk_reduce_kernel");
  }
  return CAPK_OK;
}
