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
#include <stdlib.h>

#include "gemm_common.h"

namespace capk {
// Main loop: an NST-deep LDS ring.  Before reading K-tile kt a counted
// `s_waitcnt vmcnt` retires only that tile (the NST-2 younger ones stay in flight),
// then a raw s_barrier publishes it and the slot freed one iteration ago is refilled.
// Second operand pair of a two-segment product (PAIR instantiations; the LSTM recurrences):
// K-concatenated, C = [A | A2] [B | B2]^T with K-tiles k >= k1 read from A2 / B2 at k - k1
// (both operands K-major), or N-concatenated, columns n >= n1 of C = A B2^T (n - n1) and
// columns n < n1 = A B^T.  k1 % BKX == 0 and n1 % BN == 0, so no tile straddles the seam.
struct Seg2 {
  const bf16* A2;
  int64_t lda2;
  const bf16* B2;
  int64_t ldb2;
  int k1, n1;
};

template <int BMX, int BKX, int NST, bool AK, bool BK, typename OutT, bool PAIR = false>
__global__ __launch_bounds__(BMX / 32 * 64) void gemm_bf16_kernel(
    const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb, int M, int N, int K, int splits,
    Epi e, float* __restrict__ ws, Seg2 g2) {
  using C = Cfg<BMX, BKX, NST>;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntm = (M + BMX - 1) / BMX, ntn = (N + BN - 1) / BN, ntiles = ntm * ntn;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles, tile = wg % ntiles;
  const int m0 = (tile / ntn) * BMX, n0 = (tile % ntn) * BN;
  const int nk_all = (K + BKX - 1) / BKX;
  const int kt_per = (nk_all + splits - 1) / splits;
  const int kt0 = split * kt_per;
  const int kt1 = min(nk_all, kt0 + kt_per);
  const int nk = max(0, kt1 - kt0);
  // this tile's B operand: the N-concatenated pair's second matrix past column n1
  const bf16* Bt = B;
  int64_t ldbt = ldb;
  int nb = N, nb0 = n0;
  if constexpr (PAIR) {
    if (g2.n1 > 0) {
      if (n0 >= g2.n1) Bt = g2.B2, ldbt = g2.ldb2, nb = N - g2.n1, nb0 = n0 - g2.n1;
      else nb = g2.n1;
    }
  }
  // range-checked descriptors for MN-major operands: [0, K*ld) elements are valid
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)((int64_t)K * lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, (short)0, (int)((int64_t)K * ldbt * 2), 0x00020000);

  auto stage = [&](int kt, int slot) {
    char* base = smem + slot * C::STAGE;
    int kg = (kt0 + kt) * BKX;
    const bf16* As = A;
    const bf16* Bs = Bt;
    int64_t las = lda, lbs = ldbt;
    if constexpr (PAIR) {
      if (g2.k1 > 0 && kg >= g2.k1) As = g2.A2, las = g2.lda2, Bs = g2.B2, lbs = g2.ldb2, kg -= g2.k1;
    }
    stage_tile<AK, BMX, BKX, C::A_PIECES>(As, las, M, m0, kg, base, wave * C::A_PIECES, lane, rsA);
    stage_tile<BK, BN, BKX, C::B_PIECES>(Bs, lbs, nb, nb0, kg, base + C::A_BYTES, wave * C::B_PIECES, lane, rsB);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < nk) stage(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NST - 2 < nk) wait_vm<(NST - 2) * C::VM_PER_STAGE>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < nk) stage(kt + NST - 1, (kt + NST - 1) % NST);
    const char* sc = smem + (kt % NST) * C::STAGE;
#pragma unroll
    for (int s = 0; s < BKX / 32; ++s) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<AK, BMX, BKX>(sc, wm * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<BK, BN, BKX>(sc + C::A_BYTES, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  // (the last K-tile was waited with vmcnt(0): no operand load is outstanding here)

  // ---- epilogue, 64 rows at a time: accumulators -> LDS (fp32) -> 8-wide rows.
  // Each thread owns the same 8 columns in every row it stores (THREADS % 16 == 0).
  constexpr int ITS = 64 * BN / 8 / C::THREADS;
  const int ecol = (tid & 15) * 8, egn = n0 + ecol;
  float bias8[8];
  Raw8<OutT> side[BMX / 64][ITS];
  const bool has_side = !ws && prefetch_side<OutT, BMX / 64, ITS, C::THREADS, 16>(e, m0, egn, tid, bias8, side);
  lds_barrier();
  float* stg = (float*)smem;
#pragma unroll
  for (int h = 0; h < BMX / 64; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = i * 16 + (lane >> 4) * 4 + r;
            const int col = wn * 64 + j * 16 + (lane & 15);
            stg[row * C::EPI_LD + col] = acc[i][j][r];
          }
    }
    lds_barrier();
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
      const int row = (it * C::THREADS + tid) >> 4;
      const int gm = m0 + h * 64 + row;
      if (gm < M && egn < N) {
        float v[8];
        Vec8<float>::load(stg + row * C::EPI_LD + ecol, v);
        if (ws) Vec8<float>::store(ws + ((int64_t)split * M + gm) * N + egn, v);
        else epilogue8<OutT>(e, gm, egn, v, e.bias ? bias8 : nullptr, has_side ? &side[h][it] : nullptr);
      }
    }
    lds_barrier();
  }
}

// 64x64 tile, four waves of 32x32 (cfg 9), K-major operands, no split-K: the one-round decode
// products (M = k·B rows of a beam step).  A 128x128 tile gives each wave a 64x64 block, i.e.
// 32 MFMA 16x16x32 per 64-deep K-tile on one SIMD (~0.43 us of the measured 0.66 us per
// K-tile), and at <= 256 tiles only a quarter of the chip's SIMDs: here every wave issues 8
// MFMAs per K-tile and a 1280 x 768 product runs 240 WGs x 4 waves.
template <int NST, typename OutT>
__global__ __launch_bounds__(256) void gemm_s64_kernel(const bf16* __restrict__ A, int64_t lda,
                                                       const bf16* __restrict__ B, int64_t ldb, int M, int N, int K,
                                                       int splits, Epi e, float* __restrict__ ws) {
  constexpr int T = 64, BKX = 64, TB = T * BKX * 2, STAGE = 2 * TB, EPI_LD = T + 4;
  constexpr int SMEM = (NST * STAGE > T * EPI_LD * 4) ? NST * STAGE : T * EPI_LD * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = (N + T - 1) / T, ntiles = ((M + T - 1) / T) * ntn;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles, tile = wg % ntiles;
  const int m0 = (tile / ntn) * T, n0 = (tile % ntn) * T;
  // split-K (ws != nullptr: fp32 slabs [splits][M][N], no epilogue -- the LayerNorm sums them)
  const int nk_all = K / BKX, kt_per = (nk_all + splits - 1) / splits, kt0 = split * kt_per;
  const int nk = max(0, min(nk_all, kt0 + kt_per) - kt0);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0, 0x00020000);  // unused (K-major)
  auto stage = [&](int kt, int slot) {
    char* base = smem + slot * STAGE;
    stage_tile<true, T, BKX, 2>(A, lda, M, m0, (kt0 + kt) * BKX, base, wave * 2, lane, rs);
    stage_tile<true, T, BKX, 2>(B, ldb, N, n0, (kt0 + kt) * BKX, base + TB, wave * 2, lane, rs);
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < nk) stage(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NST - 2 < nk) wait_vm<(NST - 2) * 4>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < nk) stage(kt + NST - 1, (kt + NST - 1) % NST);
    const char* sc = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int s = 0; s < BKX / 32; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = read_frag<true, T, BKX>(sc, wm * 32 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = read_frag<true, T, BKX>(sc + TB, wn * 32 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  // epilogue: accumulators -> LDS (fp32 [64][68]) -> 8-wide rows, 8 threads per row
  constexpr int ITS = T * T / 8 / 256;
  const int ecol = (tid & 7) * 8, egn = n0 + ecol;
  float bias8[8];
  Raw8<OutT> side[1][ITS];
  const bool has_side = !ws && prefetch_side<OutT, 1, ITS, 256, 8>(e, m0, egn, tid, bias8, side);
  lds_barrier();
  float* stg = (float*)smem;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        stg[(wm * 32 + i * 16 + (lane >> 4) * 4 + r) * EPI_LD + wn * 32 + j * 16 + (lane & 15)] = acc[i][j][r];
  lds_barrier();
#pragma unroll
  for (int it = 0; it < ITS; ++it) {
    const int row = (it * 256 + tid) >> 3;
    const int gm = m0 + row;
    if (gm < M && egn < N) {
      float v[8];
      Vec8<float>::load(stg + row * EPI_LD + ecol, v);
      if (ws) Vec8<float>::store(ws + ((int64_t)split * M + gm) * N + egn, v);
      else epilogue8<OutT>(e, gm, egn, v, e.bias ? bias8 : nullptr, has_side ? &side[0][it] : nullptr);
    }
  }
}

// Activation pass after the 256x256 kernel's plain product (the split activation route):
// forward: C holds pre = acc + bias; writes act(pre) to C and pre or act'(pre)
// (CAPK_ACT_DERIV) to `pre`.  Backward: C holds dY.W; multiplies by act'(aux) or by aux
// itself (CAPK_ACT_DERIV).  One HBM pass, 8-wide segments, grid-stride.
// from_pre: the library wrote pre = acc + bias straight into `pre` (plain forward act with a
// kept pre-activation): read it there and write only act(pre) to C.
template <typename OutT>
__global__ __launch_bounds__(256) void act_pass_kernel(int M, int N, OutT* __restrict__ C, int64_t ldc,
                                                       OutT* __restrict__ pre, const OutT* __restrict__ aux,
                                                       int64_t ldx, int act, int from_pre) {
  const int nseg = N / 8;
  const int64_t total = (int64_t)M * nseg;
  const int a = act & 15;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (from_pre && ldc == N && ldx == N) {
    // dense rows (the FFN activations): flat index, two 16-B segments in flight per lane
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (; i + stride < total; i += 2 * stride) {
      float v[8], w[8];
      Vec8<OutT>::load(pre + i * 8, v);
      Vec8<OutT>::load(pre + (i + stride) * 8, w);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[k] = act_fwd_fast<OutT>(a, v[k]);
        w[k] = act_fwd_fast<OutT>(a, w[k]);
      }
      Vec8<OutT>::store(C + i * 8, v);
      Vec8<OutT>::store(C + (i + stride) * 8, w);
    }
    if (i < total) {
      float v[8];
      Vec8<OutT>::load(pre + i * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd_fast<OutT>(a, v[k]);
      Vec8<OutT>::store(C + i * 8, v);
    }
    return;
  }
  if ((act & CAPK_ACT_BWD) && ldc == N && ldx == N) {
    // dense rows (FC2 dX x act'): flat index, two segments in flight per lane
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (; i < total; i += 2 * stride) {
      const bool two = i + stride < total;
      float v[8], g[8], w[8], h[8];
      Vec8<OutT>::load(C + i * 8, v);
      Vec8<OutT>::load(aux + i * 8, g);
      if (two) {
        Vec8<OutT>::load(C + (i + stride) * 8, w);
        Vec8<OutT>::load(aux + (i + stride) * 8, h);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[k] *= (act & CAPK_ACT_DERIV) ? g[k] : act_grad_fast<OutT>(a, g[k]);
        if (two) w[k] *= (act & CAPK_ACT_DERIV) ? h[k] : act_grad_fast<OutT>(a, h[k]);
      }
      Vec8<OutT>::store(C + i * 8, v);
      if (two) Vec8<OutT>::store(C + (i + stride) * 8, w);
    }
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    const int m = (int)(i / nseg), n = (int)(i % nseg) * 8;
    float v[8];
    if (from_pre) {
      Vec8<OutT>::load(pre + (int64_t)m * ldx + n, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd_fast<OutT>(a, v[k]);
      Vec8<OutT>::store(C + (int64_t)m * ldc + n, v);
      continue;
    }
    Vec8<OutT>::load(C + (int64_t)m * ldc + n, v);
    if (act & CAPK_ACT_BWD) {
      float g[8];
      Vec8<OutT>::load(aux + (int64_t)m * ldx + n, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= (act & CAPK_ACT_DERIV) ? g[k] : act_grad_fast<OutT>(a, g[k]);
    } else if (pre && (act & CAPK_ACT_DERIV)) {
      float d[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd_grad_fast<OutT>(a, v[k], d[k]);
      Vec8<OutT>::store(pre + (int64_t)m * ldx + n, d);
    } else {
      if (pre) Vec8<OutT>::store(pre + (int64_t)m * ldx + n, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd_fast<OutT>(a, v[k]);
    }
    Vec8<OutT>::store(C + (int64_t)m * ldc + n, v);
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

// Tile configuration: the 256x128 / 3-stage ring when the grid fills the chip with one
// WG per CU, else 128x128 / 2-stage (2 WGs per CU) for small decoder-side GEMMs.
static int g_forced_cfg = -1;  // capk_gemm_force_config(): tests / A-B benches
static int cfg_override() {
  static int v = [] {
    const char* s = getenv("CAPK_GEMM_CFG");
    return s ? atoi(s) : 0;
  }();
  return g_forced_cfg >= 0 ? g_forced_cfg : v;
}
// Tile configurations (CAPK_GEMM_CFG overrides for A/B measurements):
//   1: 128x128, BK 64, 2-deep ring (64 KiB, 2 WGs/CU)
//   2: 256x128, BK 64, 3-deep ring (144 KiB, 1 WG/CU)
//   3: 128x128, BK 32, 4-deep ring (64 KiB, 2 WGs/CU)
//   4: 128x128, BK 32, 3-deep ring (48 KiB, 3 WGs/CU)
//   5: 256x256, BK 64, 8 waves, phased half-tile ring (128 KiB, 1 WG/CU)
//   6: the same tile as a persistent kernel with a register-direct epilogue (gemm8q.hip)
//   7: 128x128, BK 64, 4-deep ring (128 KiB, 1 WG/CU): grids of at most one WG per CU
//   8: 64x128, BK 64, 2-deep ring, 2 waves (48 KiB, 3 WGs/CU): K-major operands only
//   9: 64x64, BK 64, 3-deep ring, 4 waves of 32x32 (48 KiB, 3 WGs/CU): K-major operands,
//      K % 64 == 0, no split-K (gemm_s64_kernel)
static bool big_tile(int cfg) { return cfg == 5 || cfg == 6; }
static int slots_of(int cfg) {  // resident WGs
  return (cfg == 2 || cfg == 7 || big_tile(cfg)) ? 256 : (cfg == 4 || cfg == 8 || cfg == 9) ? 768 : 512;
}
static int tiles_of(int cfg, int M, int N) {
  return cdiv(M, (cfg == 2 || big_tile(cfg)) ? 256 : (cfg == 8 || cfg == 9) ? 64 : 128) *
         cdiv(N, big_tile(cfg) ? 256 : cfg == 9 ? 64 : BN);
}
// Measured per shape class (tools/gemm_bench.py, profiles/): the 3-WG/CU BK-32 ring wins when
// the epilogue carries an activation (its stores overlap other WGs' main loops) and for the
// split-K weight-gradient GEMMs whose grid fits one round; the 2-WG/CU BK-64 ring elsewhere.
static int choose_splits(int cfg, int M, int N, int K);
// One-round grids of the 128x128 ring (at most one WG per CU: the decode steps' products) take
// the 4-deep ring: three K-tiles in flight instead of one (CAPK_GEMM_DEEP=0 keeps the 2-deep
// ring, for A/B)
static bool deep_ring(int grid) {
  static const bool on = [] {
    const char* v = getenv("CAPK_GEMM_DEEP");
    return !(v && v[0] == '0');
  }();
  return on && grid <= 256;
}
static int choose_cfg(int M, int N, int K, int a_kmajor, int b_kmajor, int act) {
  int o = cfg_override();
  // K-major operands with K % 64 != 0 (e.g. Swin-T/S, C = 96): only the BK-32 rings apply
  if ((a_kmajor || b_kmajor) && K % 64) return o == 3 ? 3 : 4;
  if ((o == 2 || big_tile(o)) && M < 256) o = 1;
  if ((o == 3 || o == 4) && (a_kmajor || b_kmajor) && K % 32) o = 1;
  if (o == 7 && (int64_t)cdiv(M, 128) * cdiv(N, BN) > 256) o = 1;
  if ((o == 8 || o == 9) && !(a_kmajor && b_kmajor)) o = 1;  // the MN-major image swizzle assumes 128-row tiles
  if (o == 9 && K % 64) o = 1;
  if (o >= 1 && o <= 9) return o;
  // Huge-M products with a short K (ResNet layer-1 convolutions at bs 128: M = 401 408 rows of
  // 56x56; the 1x1 expansion forward and backward-data and the 3x3 dcol have K = 64): with one
  // K-tile per item the 256x256 kernels are store-bound at one WG per CU and the 3-WG/CU BK-32
  // ring measured 3.5-4.3x faster; on that layer's N <= 128, K <= 1024 products it is 7-13 %
  // faster than the 2-WG/CU ring (graph-replayed, profiles/round4/conv_shapes.txt).
  static const bool short_k = [] {  // CAPK_GEMM_SHORTK=0: without this rule (A/B)
    const char* v = getenv("CAPK_GEMM_SHORTK");
    return !(v && v[0] == '0');
  }();
  if (short_k && a_kmajor && K % 32 == 0 &&
      ((K <= 64 && (int64_t)cdiv(M, 128) * cdiv(N, BN) >= 1024) || (M >= 65536 && N <= 128 && K <= 1024)))
    return 4;
  // the 256x256 phased kernel (gemm8p.hip) whenever its grid (x split-K for the weight
  // gradients) fills most of the chip: measured faster than the 128-row tiles on every
  // config-3 shape of that size (tools/gemm_bench.py, profiles/round2/)
  // grids of more than one round take the persistent kernel (cfg 6, gemm8q.hip; the host
  // routes one-round grids and the epilogues it lacks to gemm8p).  CAPK_GEMM_8Q=0 keeps
  // every large grid on gemm8p (A/B: profiles/round3/gemm_shapes_*).
  static const int big = [] {
    const char* v = getenv("CAPK_GEMM_8Q");
    return v && v[0] == '0' ? 5 : 6;
  }();
  // One-round grids of K-major operands (the config-3 decoder's 5120-row QKV / FC1 / FC2-dX
  // products, 180-240 tiles) measured 30-35 % faster on the 128x64 BK-64 ring than on the
  // 256x256 kernel, with or without an activation epilogue, and the 3-WG/CU BK-32 ring lost
  // to it on every activation shape (profiles/round3/decoder_gemm_cfgs.txt); small split-K
  // weight gradients (a 768 x 768 tile grid x 16 splits) likewise.
  if (M >= 256 && N >= 256) {
    const int t5 = tiles_of(5, M, N);
    if (!a_kmajor && !b_kmajor) {
      if (t5 * choose_splits(5, M, N, K) >= 192) return big;
    } else if (t5 > 256) {
      return big;
    } else if (K >= 8192 && t5 * choose_splits(5, M, N, K) >= 192) {
      // long-K products with a small tile grid (the LM-head dX: 5120 x 768 x 50 304, 60
      // tiles): split-K on the 256x256 kernel -- the 128-row ring ran it as 240 one-WG-per-CU
      // tiles at 0.17 of peak (938 us, profiles/round4)
      return big;
    }
  }
  if (!a_kmajor && !b_kmajor && tiles_of(4, M, N) < slots_of(4)) return 1;  // split-K dW (cfg 4 measured slower)
  return 1;
}
// Split-K factor: fill one round of resident workgroups when the tile grid alone cannot
// (any integer factor; every split keeps >= 4 K-tiles).
static int choose_splits(int cfg, int M, int N, int K) {
  static const int max_split_env = [] {  // A/B control (tools/gemm_bench.py): CAPK_GEMM_MAXSPLIT=1 disables split-K
    const char* v = getenv("CAPK_GEMM_MAXSPLIT");
    return v ? std::max(1, atoi(v)) : 0;
  }();
  // very long reductions (conv weight gradients: K = B*H*W up to 4e5) with a tiny M x N
  // grid fill the chip only with more than 16 splits (each split still >= 4 K-tiles)
  // (K >= 16384: the ViT O-projection weight gradient, 768 x 768 = 9 tiles, fills 252 CUs
  // with 28 splits instead of 144 with 16)
  // (K >= 262144: ResNet layer-1 / stem weight gradients, 2-tile grids over 4e5-1.6e6 rows,
  // fill the chip with 128 splits instead of half of it with 64; the stem's 1.6e6 rows take
  // 256: 275 -> 216 us, while 256 on the 4e5-row ones lost, 89 -> 108 us)
  const int max_split = max_split_env ? max_split_env
                                      : (K >= 1048576 ? 256 : K >= 262144 ? 128 : K >= 65536 ? 64
                                         : K >= 16384 ? 32 : 16);
  const int bk = (cfg == 3 || cfg == 4) ? 32 : 64;
  const int tiles = tiles_of(cfg, M, N), slots = slots_of(cfg);
  const int nk = cdiv(K, bk);
  if (2 * tiles >= slots) return 1;
  // decode-step shapes (tools/gemm_bench.py dec*, graph-timed): with >= 128 tiles, or >= 48
  // on a short K, the separate reduce launch costs more than the split saves
  if (tiles >= 128 || (K < 2048 && tiles > 48)) return 1;
  int s = std::min(max_split, slots / tiles);
  s = std::min(s, std::max(1, nk / 4));
  return std::max(1, s);
}


}  // namespace capk

using namespace capk;

static thread_local int g_last_cfg = 0;
extern "C" int capk_gemm_last_config(void) { return g_last_cfg; }
extern "C" int capk_gemm_force_config(int cfg) {
  capk::g_forced_cfg = cfg;
  return CAPK_OK;
}

extern "C" size_t capk_gemm_workspace(int in_dtype, int out_dtype, int M, int N, int K) {
  (void)out_dtype;
  if (in_dtype != CAPK_BF16) return 0;
  // upper bound over the configurations (the launch picks one of them)
  int s = 1;
  for (int c = 1; c <= 8; ++c) s = std::max(s, choose_splits(c, M, N, K));  // (cfg 9 never splits)
  const size_t slab = s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
  // persistent grids: the split-tail hand-off area (gemm8q.hip)
  return tiles_of(6, M, N) > 256 ? std::max(slab, gemm8q_tail_workspace(M, N, K)) : slab;
}

extern "C" int capk_gemm(int in_dtype, int out_dtype, int M, int N, int K, const void* A, int64_t lda,
                         int a_kmajor, const void* B, int64_t ldb, int b_kmajor, void* C, int64_t ldc,
                         float alpha, float beta, const float* bias, const void* residual, int64_t ldr,
                         int act, void* preact, const void* aux, int64_t ldx, float drop_p, uint32_t drop_seed,
                         void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(M > 0 && N > 0 && K > 0, "capk_gemm: bad sizes M=%d N=%d K=%d", M, N, K);
  CAPK_CHECK_ARG(A && B && C, "capk_gemm: null operand");
  CAPK_CHECK_ARG(!(act & CAPK_ACT_BWD) || aux, "capk_gemm: backward activation needs aux");
  Epi e{C, ldc, alpha, beta, bias, residual, ldr, act, preact, aux, ldx, M, N, make_drop(drop_p, drop_seed)};
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
  CAPK_CHECK_ARG(!(a_kmajor || b_kmajor) || K % 32 == 0,
                 "capk_gemm(bf16): K=%d must be a multiple of 32 when an operand is K-major", K);
  CAPK_CHECK_ARG(N % 8 == 0, "capk_gemm(bf16): N=%d must be a multiple of 8", N);
  CAPK_CHECK_ARG(a_kmajor || (M % 8 == 0 && M >= 8), "capk_gemm(bf16): M-major A needs M %% 8 == 0");
  CAPK_CHECK_ARG(b_kmajor || (N % 8 == 0 && N >= 8), "capk_gemm(bf16): N-major B needs N %% 8 == 0");
  CAPK_CHECK_ARG((a_kmajor || (int64_t)K * lda * 2 < (1ll << 31)) && (b_kmajor || (int64_t)K * ldb * 2 < (1ll << 31)),
                 "capk_gemm(bf16): MN-major operand larger than 2 GiB");
  const int64_t esz = out_dtype == CAPK_F32 ? 4 : 2;
  CAPK_CHECK_ARG(((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % 8 == 0 && ldb % 8 == 0,
                 "capk_gemm(bf16): A/B must be 16-B aligned with lda, ldb %% 8 == 0");
  CAPK_CHECK_ARG(((uintptr_t)C % 16 == 0) && (ldc * esz) % 16 == 0, "capk_gemm(bf16): C alignment");
  int cfg = choose_cfg(M, N, K, a_kmajor, b_kmajor, act);
  int splits = choose_splits(cfg, M, N, K);
  if (!ws || ws_bytes < (size_t)splits * M * N * sizeof(float)) splits = 1;
  if (splits > 1) {  // effective count: every split owns >= 1 K-tile (the reduce sums exactly these)
    const int bk = (cfg == 3 || cfg == 4) ? 32 : 64, nk = cdiv(K, bk), per = cdiv(nk, splits);
    splits = cdiv(nk, per);
  }
  // gemm8q: at most one side operand and >= 2 K-tiles per item (else the 8p kernel); its
  // items all run kt_per K-tiles, so a split count that pads the last split is taken only
  // for MN-major operands (whose K rows past K read as zero; a K-major row would run on
  // into the next row)
  if (cfg == 6) {
    const int nk64 = cdiv(K, 64), per = cdiv(nk64, splits);
    const bool padded = nk64 % per != 0;
    if (!gemm8q_supports(e, out_dtype == CAPK_F32) || per < 2 || (padded && (a_kmajor || b_kmajor)) ||
        splits > 1 ||                          // split-K slabs: gemm8p + splitk_reduce
        tiles_of(6, M, N) * splits <= 256 ||  // one round: the non-persistent kernel
        ((act & 15) && !(act & CAPK_ACT_BWD) && splits == 1 && !(a_kmajor && b_kmajor)))
      cfg = 5;
  }
  if (cfg == 1 && cfg_override() == 0 && deep_ring(tiles_of(1, M, N) * splits)) cfg = 7;
  // one-round K-major products on the 64x64 four-wave tile (CAPK_GEMM_S64=0 keeps them on the
  // 4-deep 128x128 ring, =1 only when the 64x64 grid is one round, for A/B)
  static const int s64_mode = [] {
    const char* v = getenv("CAPK_GEMM_S64");
    return v ? atoi(v) : 2;
  }();
  if (cfg == 7 && cfg_override() == 0 && s64_mode && splits == 1 && a_kmajor && b_kmajor && K % 64 == 0 &&
      (s64_mode == 2 || tiles_of(9, M, N) <= slots_of(9)))
    cfg = 9;
  if (cfg == 9) splits = 1;
  g_last_cfg = cfg;
  const int tiles = tiles_of(cfg, M, N);
  const int grid = tiles * splits;
  float* slab = splits > 1 ? (float*)ws : nullptr;
#define LAUNCH1(BMX, BKX, NST, AK, BKM, OT)                                                                     \
  hipLaunchKernelGGL((gemm_bf16_kernel<BMX, BKX, NST, AK, BKM, OT>), dim3(grid), dim3(BMX / 32 * 64), 0, st, \
                     (const bf16*)A, lda, (const bf16*)B, ldb, M, N, K, splits, e, slab, Seg2{})
#define LAUNCH(AK, BKM, OT)                                    \
  do {                                                         \
    switch (cfg) {                                             \
      case 2: LAUNCH1(256, 64, 3, AK, BKM, OT); break;         \
      case 3: LAUNCH1(128, 32, 4, AK, BKM, OT); break;         \
      case 4: LAUNCH1(128, 32, 3, AK, BKM, OT); break;         \
      case 7: LAUNCH1(128, 64, 4, AK, BKM, OT); break;         \
      case 8: LAUNCH1(64, 64, 2, AK, BKM, OT); break;          \
      default: LAUNCH1(128, 64, 2, AK, BKM, OT); break;        \
    }                                                          \
  } while (0)
#define DISPATCH(OT)                          \
  if (a_kmajor && b_kmajor) LAUNCH(true, true, OT);     \
  else if (a_kmajor) LAUNCH(true, false, OT);           \
  else if (b_kmajor) LAUNCH(false, true, OT);           \
  else LAUNCH(false, false, OT);
  if (cfg == 6) {
    int tail_r0 = -1, tail_splits = 1;
    const int rc = launch_gemm8q(a_kmajor, b_kmajor, out_dtype == CAPK_F32, A, lda, B, ldb, M, N, K, splits, e, slab,
                                 st, nullptr, slab ? nullptr : ws, slab ? 0 : ws_bytes, &tail_r0, &tail_splits);
    if (rc != CAPK_OK) return rc;
    if (tail_r0 >= 0) {  // the split-K tail round's slabs -> rows [256 r0, M) with the epilogue
      // (bf16 outputs with any one side operand; fp32 outputs carry none: gemm8q_supports)
      const int64_t r = (int64_t)tail_r0 * 256, es = esz;  // row offsets in output elements
      Epi et = e;
      et.M = M - (int)r;
      et.C = (char*)e.C + r * e.ldc * es;
      if (e.res) et.res = (const char*)e.res + r * e.ldr * es;
      if (e.aux) et.aux = (const char*)e.aux + r * e.ldx * es;
      if (e.pre) et.pre = (char*)e.pre + r * e.ldx * es;
      const int64_t n8 = (int64_t)et.M * N / 8;
      const int g = (int)std::min<int64_t>(2048, (n8 + 255) / 256);
      if (out_dtype == CAPK_BF16)
        hipLaunchKernelGGL(splitk_reduce_kernel<bf16>, dim3(g), dim3(256), 0, st, (const float*)ws, tail_splits, et);
      else
        hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)ws, tail_splits, et);
      CAPK_LAUNCH_CHECK("splitk_reduce_kernel");
    }
  } else if (cfg == 5) {
    // Activation products on the 256x256 kernel: plain product (+ bias) into the kept
    // pre-activation / C, then one elementwise pass (act_pass_kernel) -- measured faster than
    // the fused activation epilogue, which runs while the CU's MFMAs idle (1 WG per CU), at
    // well below HBM bandwidth.  CAPK_GEMM_SPLIT_ACT=0 keeps the fused epilogue (A/B).
    static const bool split_act = [] {
      const char* v = getenv("CAPK_GEMM_SPLIT_ACT");
      return !(v && v[0] == '0');
    }();
    const bool split = split_act && (act & 15) && !(drop_p > 0.f) && !residual && beta == 0.f &&
                       out_dtype == CAPK_BF16 && splits == 1;
    const int from_pre = !(act & CAPK_ACT_BWD) && !(act & CAPK_ACT_DERIV) && preact != nullptr;
    Epi ep = e;
    if (split) {
      ep.act = 0;
      ep.pre = nullptr;
      ep.aux = nullptr;
      if (from_pre) {
        ep.C = preact;
        ep.ldc = ldx;
      }
      if (act & CAPK_ACT_BWD) ep.bias = nullptr;
    }
    const int rc = launch_gemm8p(a_kmajor, b_kmajor, out_dtype == CAPK_F32, grid, A, lda, B, ldb, M, N, K, splits, ep,
                                 slab, st);
    if (rc != CAPK_OK) return rc;
    if (split) {
      const int64_t segs = (int64_t)M * (N / 8);
      const bool dense = ldc == N && ldx == N && (from_pre || (act & CAPK_ACT_BWD));
      const int grid_a = (int)std::min<int64_t>(dense ? cdiv(segs, 512) : cdiv(segs, 256), dense ? (1 << 20) : 8192);
      hipLaunchKernelGGL(act_pass_kernel<bf16>, dim3(grid_a), dim3(256), 0, st, M, N, (bf16*)C, ldc, (bf16*)preact,
                         (const bf16*)aux, ldx, act, from_pre);
      CAPK_LAUNCH_CHECK("act_pass_kernel");
    }
  } else if (cfg == 9) {
    // grids past one round of the 3-deep ring (3 WGs/CU) take the 2-deep ring (32 KiB, 5 WGs/CU)
    // (CAPK_GEMM_S64_NST2=0: always 3-deep, for A/B)
    static const bool nst2_on = [] {
      const char* v = getenv("CAPK_GEMM_S64_NST2");
      return !(v && v[0] == '0');
    }();
#define S64(NS)                                                                                               \
  do {                                                                                                        \
    if (out_dtype == CAPK_BF16)                                                                               \
      hipLaunchKernelGGL((gemm_s64_kernel<NS, bf16>), dim3(grid), dim3(256), 0, st, (const bf16*)A, lda,      \
                         (const bf16*)B, ldb, M, N, K, 1, e, nullptr);                                        \
    else                                                                                                      \
      hipLaunchKernelGGL((gemm_s64_kernel<NS, float>), dim3(grid), dim3(256), 0, st, (const bf16*)A, lda,     \
                         (const bf16*)B, ldb, M, N, K, 1, e, nullptr);                                        \
  } while (0)
    if (nst2_on && grid > slots_of(9)) S64(2);
    else S64(3);
#undef S64
  } else if (out_dtype == CAPK_BF16) {
    DISPATCH(bf16)
  } else {
    DISPATCH(float)
  }
#undef DISPATCH
#undef LAUNCH
#undef LAUNCH1
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

// The LM head with the shifted cross entropy's forward folded into its epilogue: C = x W^T + b
// (bf16) and, from the same registers, per (row, column tile, wave) the (max, sum 2^(t - max))
// pair of t = log2(e) * bf16(C) over the wave's 64 columns below V -- the softmax partials that
// capk_ce_lse_fwd merges into each row's log-sum-exp, so the [rows, Vp] logits are not re-read
// for the loss.  Persistent-kernel grids only (the config-3 LM head: 20 x 197 tiles); any other
// shape runs capk_gemm and reports *done = 0 (the caller then uses capk_shifted_ce).
extern "C" size_t capk_linear_lse_part_bytes(int M, int N) { return (size_t)cdiv(N, 256) * 4 * M * 2 * sizeof(float); }

extern "C" int capk_linear_lse(int M, int N, int K, const void* x, int64_t ldx, const void* w, int64_t ldw,
                               const float* bias, void* C, int64_t ldc, int V, float* part, size_t part_bytes,
                               int* done, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(M > 0 && N > 0 && K > 0 && x && w && C && part && done && V > 0 && V <= N,
                 "capk_linear_lse: bad arguments");
  CAPK_CHECK_ARG(part_bytes >= capk_linear_lse_part_bytes(M, N), "capk_linear_lse: partials buffer too small");
  *done = 0;
  const bool fits = K % 64 == 0 && cdiv(K, 64) >= 2 && N % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0 &&
                    (uintptr_t)x % 16 == 0 && (uintptr_t)w % 16 == 0 && (uintptr_t)C % 16 == 0 &&
                    choose_cfg(M, N, K, 1, 1, 0) == 6 && tiles_of(6, M, N) > 256;
  if (!fits)
    return capk_gemm(CAPK_BF16, CAPK_BF16, M, N, K, x, ldx, 1, w, ldw, 1, C, ldc, 1.f, 0.f, bias, nullptr, 0, 0, nullptr,
                     nullptr, 0, 0.f, 0, ws, ws_bytes, stream);
  Epi e{C, ldc, 1.f, 0.f, bias, nullptr, 0, 0, nullptr, nullptr, 0, M, N, make_drop(0.f, 0)};
  g_last_cfg = 6;
  const int rc = launch_gemm8q(true, true, false, x, ldx, w, ldw, M, N, K, 1, e, nullptr, S(stream), nullptr, nullptr,
                               0, nullptr, nullptr, part, V);
  if (rc == CAPK_OK) *done = 1;
  return rc;
}

// Two-segment products into fp32 split-K slabs, no epilogue: the LSTM recurrences, whose
// consumers (the cell kernels, lstm.hip) sum the slabs themselves -- one launch per step and
// layer in place of two GEMMs and two split-K reduces.  128x128 ring tiles; splits so that
// about one round of WGs runs, every split >= CAPK_PAIR_MINKT (4) K-tiles.
// A single product (no seam: the decode steps' GEMM -> LayerNorm pairs) has no reduce launch
// to amortise -- its consumer sums the slabs -- so it splits until about two WGs per CU run
// (each split >= 4 K-tiles): the decode steps' K = 768 out-projections at 1280 rows go from 60
// one-split tiles (12 K-tiles each, latency-bound) to 3 splits.  CAPK_SLAB_SPLITS=0 keeps
// capk_gemm's own count, whose slabs are bit-identical to capk_gemm + splitk_reduce.
static int pair_splits(int M, int N, int K, bool seam) {
  static const int min_kt = [] {
    const char* v = getenv("CAPK_PAIR_MINKT");
    return v ? std::max(1, atoi(v)) : 4;
  }();
  static const bool slab_policy = [] {
    const char* v = getenv("CAPK_SLAB_SPLITS");
    return !(v && v[0] == '0');
  }();
  const int tiles = cdiv(M, 128) * cdiv(N, BN), nk = cdiv(K, 64);
  int s;
  if (seam) s = std::max(1, std::min(256 / tiles, nk / min_kt));
  else {
    s = choose_splits(1, M, N, K);
    if (slab_policy) s = std::max(s, std::min(512 / tiles, nk / min_kt));
  }
  s = std::max(1, s);
  return cdiv(nk, cdiv(nk, s));  // effective count: every split owns >= 1 K-tile
}

// The no-seam slab products with a K-major weight (the decode steps' out-projection / FFN2 ->
// LayerNorm pairs) run on the 64x64 four-wave tile (cfg 9): splits so that about one round of
// 3 WGs per CU runs, every split >= CAPK_PAIR_MINKT K-tiles (CAPK_SLAB_S64=0: the 128x128 ring
// with pair_splits' count, for A/B).
static bool slab_s64_on() {
  static const bool on = [] {
    const char* v = getenv("CAPK_SLAB_S64");
    return !(v && v[0] == '0');
  }();
  return on;
}
static int s64_slab_splits(int M, int N, int K) {
  static const int min_kt = [] {
    const char* v = getenv("CAPK_PAIR_MINKT");
    return v ? std::max(1, atoi(v)) : 4;
  }();
  const int tiles = cdiv(M, 64) * cdiv(N, 64), nk = cdiv(K, 64);
  const int s = std::max(1, std::min(slots_of(9) / tiles, nk / min_kt));
  return cdiv(nk, cdiv(nk, s));
}

extern "C" size_t capk_gemm_pair_workspace(int M, int N, int K, int* splits) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int s = pair_splits(M, N, K, true);
  if (splits) *splits = s;
  return (size_t)s * M * N * sizeof(float);
}

extern "C" size_t capk_gemm_slabs_workspace(int M, int N, int K, int* splits) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  // an upper bound over both weight layouts (capk_gemm_pair_slabs returns the count it ran)
  int s = pair_splits(M, N, K, false);
  if (slab_s64_on() && K % 64 == 0) s = std::max(s, s64_slab_splits(M, N, K));
  if (splits) *splits = s;
  return (size_t)s * M * N * sizeof(float);
}

extern "C" int capk_gemm_pair_slabs(int M, int N, int K, const void* A, int64_t lda, int a_kmajor, const void* B,
                                    int64_t ldb, int b_kmajor, const void* A2, int64_t lda2, const void* B2,
                                    int64_t ldb2, int k1, int n1, float* ws, size_t ws_bytes, int* splits_out,
                                    void* stream) {
  CAPK_CHECK_ARG(M > 0 && N > 0 && K > 0 && A && B && ws && (k1 == 0 && n1 == 0 || B2),
                 "capk_gemm_pair_slabs: bad arguments");
  CAPK_CHECK_ARG(!(k1 > 0 && n1 > 0), "capk_gemm_pair_slabs: at most one of k1 (K seam) / n1 (N seam)");
  CAPK_CHECK_ARG(a_kmajor, "capk_gemm_pair_slabs: A must be K-major");
  CAPK_CHECK_ARG(k1 == 0 || (A2 && b_kmajor && k1 % 64 == 0 && (K - k1) % 64 == 0 && k1 < K),
                 "capk_gemm_pair_slabs: K seam k1=%d needs K-major A2/B2 and k1, K-k1 multiples of 64", k1);
  CAPK_CHECK_ARG(n1 == 0 || (n1 % BN == 0 && n1 < N), "capk_gemm_pair_slabs: N seam n1=%d must be a multiple of %d",
                 n1, BN);
  CAPK_CHECK_ARG(K % 64 == 0 && N % 8 == 0, "capk_gemm_pair_slabs: K=%d %% 64, N=%d %% 8", K, N);
  CAPK_CHECK_ARG(b_kmajor || (int64_t)K * std::max(ldb, ldb2) * 2 < (1ll << 31), "capk_gemm_pair_slabs: B too large");
  CAPK_CHECK_ARG(((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && ((uintptr_t)B2 % 16 == 0) &&  // (null passes)
                     (!A2 || (uintptr_t)A2 % 16 == 0) && lda % 8 == 0 && ldb % 8 == 0 && lda2 % 8 == 0 &&
                     ldb2 % 8 == 0,
                 "capk_gemm_pair_slabs: operands must be 16-B aligned with leading dimensions %% 8 == 0");
  const bool s64 = slab_s64_on() && k1 == 0 && n1 == 0 && b_kmajor;
  const int splits = s64 ? s64_slab_splits(M, N, K) : pair_splits(M, N, K, k1 > 0 || n1 > 0);
  CAPK_CHECK_ARG(ws_bytes >= (size_t)splits * M * N * sizeof(float), "capk_gemm_pair_slabs: workspace too small");
  Epi e{nullptr, N, 1.f, 0.f, nullptr, nullptr, 0, 0, nullptr, nullptr, 0, M, N, make_drop(0.f, 0)};
  if (s64) {
    const int grid = cdiv(M, 64) * cdiv(N, 64) * splits;
    g_last_cfg = 9;
    if (grid > slots_of(9))
      hipLaunchKernelGGL((gemm_s64_kernel<2, bf16>), dim3(grid), dim3(256), 0, S(stream), (const bf16*)A, lda,
                         (const bf16*)B, ldb, M, N, K, splits, e, ws);
    else
      hipLaunchKernelGGL((gemm_s64_kernel<3, bf16>), dim3(grid), dim3(256), 0, S(stream), (const bf16*)A, lda,
                         (const bf16*)B, ldb, M, N, K, splits, e, ws);
    CAPK_LAUNCH_CHECK("gemm_s64_kernel(slabs)");
    if (splits_out) *splits_out = splits;
    return CAPK_OK;
  }
  const Seg2 g2{(const bf16*)A2, lda2, (const bf16*)B2, ldb2, k1, n1};
  const int grid = cdiv(M, 128) * cdiv(N, BN) * splits;
  const bool deep = deep_ring(grid);
  g_last_cfg = deep ? 7 : 1;
#define PAIR_LAUNCH(NST, BKM)                                                                                    \
  hipLaunchKernelGGL((gemm_bf16_kernel<128, 64, NST, true, BKM, bf16, true>), dim3(grid), dim3(256), 0, S(stream), \
                     (const bf16*)A, lda, (const bf16*)B, ldb, M, N, K, splits, e, ws, g2)
  if (deep) {
    if (b_kmajor) PAIR_LAUNCH(4, true);
    else PAIR_LAUNCH(4, false);
  } else {
    if (b_kmajor) PAIR_LAUNCH(2, true);
    else PAIR_LAUNCH(2, false);
  }
#undef PAIR_LAUNCH
  CAPK_LAUNCH_CHECK("gemm_bf16_kernel(pair)");
  if (splits_out) *splits_out = splits;
  return CAPK_OK;
}

// dX = dY W times act'(pre) with the column sums of the result (the pre-LN FFN backward:
// dPre of fc1 and fc1's bias gradient, modeling_vit.py:249-254).  Persistent grids take the
// fused kernel (gemm8q DSUM: column-sum partials from the register epilogue + one finish
// launch); others the plain product + capk_act_bwd_colsum.
extern "C" size_t capk_gemm_dx_act_colsum_workspace(int M, int N, int K) {
  const size_t g = capk_gemm_workspace(CAPK_BF16, CAPK_BF16, M, N, K);
  const size_t c = capk_colsum_workspace(M, N);
  const size_t d = (size_t)cdiv(M, 256) * 2 * N * sizeof(float);
  return std::max(g, std::max(c, d));
}

// w_kmajor: W given as its K-major copy W^T [N][K] (capk_gemm_dx_act_colsum_wt)
static int dx_act_colsum(int M, int N, int K, const void* dY, int64_t ldy, const void* W, int64_t ldw, int w_kmajor,
                         void* C, int64_t ldc, int act, const void* aux, int64_t ldx, float* db, int accumulate,
                         void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(M > 0 && N > 0 && K > 0 && dY && W && C && aux && db && (act & 15),
                 "capk_gemm_dx_act_colsum: bad arguments");
  CAPK_CHECK_ARG(ws && ws_bytes >= capk_gemm_dx_act_colsum_workspace(M, N, K),
                 "capk_gemm_dx_act_colsum: workspace too small");
  const int act_bwd = CAPK_ACT_BWD | act;
  Epi e{C, ldc, 1.f, 0.f, nullptr, nullptr, 0, act_bwd, nullptr, aux, ldx, M, N, make_drop(0.f, 0)};
  const int cfg = choose_cfg(M, N, K, 1, w_kmajor, act_bwd);
  const int splits = choose_splits(cfg, M, N, K);
  const bool fused = (cfg == 5 || cfg == 6) && splits == 1 && (act & CAPK_ACT_DERIV) && K % 32 == 0 &&
                     tiles_of(6, M, N) > 256 && gemm8q_supports(e, false) && K >= 128;
  if (fused) {
    g_last_cfg = 6;
    const int rc = launch_gemm8q(true, w_kmajor != 0, false, dY, ldy, W, ldw, M, N, K, 1, e, nullptr, S(stream),
                                 (float*)ws, nullptr, 0, nullptr, nullptr);
    if (rc != CAPK_OK) return rc;
    return launch_colsum_finish(cdiv(M, 256) * 2, N, (const float*)ws, db, accumulate, S(stream));
  }
  int rc = capk_gemm(CAPK_BF16, CAPK_BF16, M, N, K, dY, ldy, 1, W, ldw, w_kmajor, C, ldc, 1.f, 0.f, nullptr, nullptr,
                     0, 0, nullptr, nullptr, 0, 0.f, 0, ws, ws_bytes, stream);
  if (rc != CAPK_OK) return rc;
  return capk_act_bwd_colsum(CAPK_BF16, M, N, C, ldc, aux, ldx, act, db, accumulate, ws, ws_bytes, stream);
}

extern "C" int capk_gemm_dx_act_colsum(int M, int N, int K, const void* dY, int64_t ldy, const void* W, int64_t ldw,
                                       void* C, int64_t ldc, int act, const void* aux, int64_t ldx, float* db,
                                       int accumulate, void* ws, size_t ws_bytes, void* stream) {
  return dx_act_colsum(M, N, K, dY, ldy, W, ldw, 0, C, ldc, act, aux, ldx, db, accumulate, ws, ws_bytes, stream);
}

extern "C" int capk_gemm_dx_act_colsum_wt(int M, int N, int K, const void* dY, int64_t ldy, const void* WT,
                                          int64_t ldwt, void* C, int64_t ldc, int act, const void* aux, int64_t ldx,
                                          float* db, int accumulate, void* ws, size_t ws_bytes, void* stream) {
  return dx_act_colsum(M, N, K, dY, ldy, WT, ldwt, 1, C, ldc, act, aux, ldx, db, accumulate, ws, ws_bytes, stream);
}

// fp8 GEMM (config 5): C = epilogue((diag(2^sa) A8) (diag(2^sb) B8)^T), A8 [M][K], B8 [N][K]
// e4m3fn, scales E8M0 per row (capk_quant_fp8).  The 256x256 kernel only (F8 variant of
// gemm8p: 128-deep K-tiles of v_mfma_scale_f32_16x16x128_f8f6f4), split-K as for bf16.
extern "C" size_t capk_gemm_f8_workspace(int M, int N, int K) {
  const int s = choose_splits(5, M, N, K / 2);  // 128-deep K-tiles: half as many as bf16's 64
  return s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
}

extern "C" int capk_gemm_f8(int out_dtype, int M, int N, int K, const void* A, int64_t lda, const void* a_scale,
                            const void* B, int64_t ldb, const void* b_scale, void* C, int64_t ldc, float beta,
                            const float* bias, const void* residual, int64_t ldr, int act, void* preact, int64_t ldx,
                            float drop_p, uint32_t drop_seed, void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(M > 0 && N > 0 && K > 0, "capk_gemm_f8: bad sizes M=%d N=%d K=%d", M, N, K);
  CAPK_CHECK_ARG(A && B && C && a_scale && b_scale, "capk_gemm_f8: null operand");
  CAPK_CHECK_ARG(K % 128 == 0, "capk_gemm_f8: K=%d must be a multiple of 128", K);
  CAPK_CHECK_ARG(N % 8 == 0, "capk_gemm_f8: N=%d must be a multiple of 8", N);
  CAPK_CHECK_ARG(!(act & CAPK_ACT_BWD), "capk_gemm_f8: forward products only");
  CAPK_CHECK_ARG(out_dtype == CAPK_BF16 || out_dtype == CAPK_F32, "capk_gemm_f8: unknown out_dtype");
  CAPK_CHECK_ARG(((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % 16 == 0 && ldb % 16 == 0 &&
                     lda >= K && ldb >= K,
                 "capk_gemm_f8: A/B must be 16-B aligned with lda, ldb >= K and %% 16 == 0");
  const int64_t esz = out_dtype == CAPK_F32 ? 4 : 2;
  CAPK_CHECK_ARG(((uintptr_t)C % 16 == 0) && (ldc * esz) % 16 == 0, "capk_gemm_f8: C alignment");
  Epi e{C, ldc, 1.f, beta, bias, residual, ldr, act, preact, nullptr, ldx, M, N, make_drop(drop_p, drop_seed)};
  hipStream_t st = S(stream);
  int splits = choose_splits(5, M, N, K / 2);
  if (!ws || ws_bytes < (size_t)splits * M * N * sizeof(float)) splits = 1;
  const int grid = tiles_of(5, M, N) * splits;
  float* slab = splits > 1 ? (float*)ws : nullptr;
  // activation: plain product (+ bias) into preact / C, then the elementwise pass (as bf16 cfg 5)
  const bool split = (act & 15) && !(drop_p > 0.f) && !residual && beta == 0.f && out_dtype == CAPK_BF16 &&
                     splits == 1;
  const int from_pre = !(act & CAPK_ACT_DERIV) && preact != nullptr;
  Epi ep = e;
  if (split) {
    ep.act = 0;
    ep.pre = nullptr;
    if (from_pre) {
      ep.C = preact;
      ep.ldc = ldx;
    }
  }
  const int rc = launch_gemm8p_f8(out_dtype == CAPK_F32, grid, A, lda, (const uint8_t*)a_scale, B, ldb,
                                  (const uint8_t*)b_scale, M, N, K, splits, splits > 1 ? e : ep, slab, st);
  if (rc != CAPK_OK) return rc;
  if (split) {
    const int64_t segs = (int64_t)M * (N / 8);
    const bool dense = ldc == N && ldx == N && from_pre;
    const int grid_a = (int)std::min<int64_t>(dense ? cdiv(segs, 512) : cdiv(segs, 256), dense ? (1 << 20) : 8192);
    hipLaunchKernelGGL(act_pass_kernel<bf16>, dim3(grid_a), dim3(256), 0, st, M, N, (bf16*)C, ldc, (bf16*)preact,
                       (const bf16*)nullptr, ldx, act, from_pre);
    CAPK_LAUNCH_CHECK("act_pass_kernel");
  }
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
