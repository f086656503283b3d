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
  Drop drop;  // mask index m*N + n, applied after the activation (or with act'), before the residual
};

// One 8-wide row segment of an epilogue side operand (aux or residual), raw in registers.
template <typename T> struct Raw8;
template <> struct Raw8<bf16> {
  bf16x8 v;
  __device__ __forceinline__ void load(const bf16* p) { v = *(const bf16x8*)p; }
  __device__ __forceinline__ float get(int i) const { return (float)v[i]; }
};
template <> struct Raw8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) { a = *(const f32x4*)p; b = *(const f32x4*)(p + 4); }
  __device__ __forceinline__ float get(int i) const { return i < 4 ? a[i] : b[i - 4]; }
};

// bias8 / side: operands the caller loaded before its first store (nullptr: load here).
// side is aux for a backward activation, else the residual.
template <typename OutT>
__device__ __forceinline__ void epilogue8(const Epi& e, int m, int n, float (&v)[8], const float* bias8 = nullptr,
                                          const Raw8<OutT>* side = nullptr) {
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
    if (bias8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = bias8[i];
    } else {
      Vec8<float>::load(e.bias + n, b);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += b[i];
  }
  if (e.act & CAPK_ACT_BWD) {
    float a[8];
    if (side) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = side->get(i);
    } else {
      Vec8<OutT>::load((const OutT*)e.aux + (int64_t)m * e.ldx + n, a);
    }
    const int act = e.act & 15;
    if (e.act & CAPK_ACT_DERIV) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] *= a[i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] *= act_grad_fast(act, a[i]);
    }
  } else if (e.act) {
    const int act = e.act & 15;
    if (e.pre && (e.act & CAPK_ACT_DERIV)) {
      float d[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = act_fwd_grad_fast(act, v[i], d[i]);
      Vec8<OutT>::store((OutT*)e.pre + (int64_t)m * e.ldx + n, d);
    } else {
      if (e.pre) Vec8<OutT>::store((OutT*)e.pre + (int64_t)m * e.ldx + n, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = act_fwd_fast(act, v[i]);
    }
  }
  if (e.drop.on()) {
    const uint64_t base = (uint64_t)m * e.N + n;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] *= e.drop.mul(base + i);
  }
  if (e.res) {
    float r[8];
    if (side && !(e.act & CAPK_ACT_BWD)) {
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] = side->get(i);
    } else {
      Vec8<OutT>::load((const OutT*)e.res + (int64_t)m * e.ldr + n, r);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += r[i];
  }
  Vec8<OutT>::store((OutT*)e.C + (int64_t)m * e.ldc + n, v);
}

// Epilogue operand prefetch.  On gfx9 vmcnt counts stores as well as loads, in order,
// so a load issued after a store cannot be waited for without waiting for that store:
// an epilogue that loads bias / aux / residual per 8-wide segment serialises one
// store round trip per segment.  Kernels therefore load every side segment of the
// tile (and the thread's bias columns) before the first store, and separate the LDS
// staging chunks with LDS-only barriers (s_waitcnt lgkmcnt(0) + s_barrier) instead of
// __syncthreads, which would also drain the stores.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename OutT, int NH, int ITS, int THREADS, int SEGS_PER_ROW>
__device__ __forceinline__ bool prefetch_side(const Epi& e, int m0, int gn, int tid, float (&bias8)[8],
                                              Raw8<OutT> (&side)[NH][ITS]) {
  const bool bwd = e.act & CAPK_ACT_BWD;
  const OutT* sp = (const OutT*)(bwd ? e.aux : e.res);
  const int64_t sld = bwd ? e.ldx : e.ldr;
  if (gn >= e.N) return false;
  if (e.bias) Vec8<float>::load(e.bias + gn, bias8);
  if (!sp) return false;
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
      const int gm = m0 + h * 64 + (it * THREADS + tid) / SEGS_PER_ROW;
      if (gm < e.M) side[h][it].load(sp + (int64_t)gm * sld + gn);
    }
  return true;
}

template <typename OutT>
__device__ __forceinline__ void epilogue1(const Epi& e, int m, int n, float v) {
  v *= e.alpha;
  if (e.beta != 0.f) v += e.beta * to_f32(((const OutT*)e.C)[(int64_t)m * e.ldc + n]);
  if (e.bias) v += e.bias[n];
  if (e.act & CAPK_ACT_BWD) {
    const float a = to_f32(((const OutT*)e.aux)[(int64_t)m * e.ldx + n]);
    v *= (e.act & CAPK_ACT_DERIV) ? a : act_grad(e.act & 15, a);
  } else if (e.act) {
    if (e.pre)
      ((OutT*)e.pre)[(int64_t)m * e.ldx + n] = from_f32<OutT>((e.act & CAPK_ACT_DERIV) ? act_grad(e.act & 15, v) : v);
    v = act_fwd(e.act & 15, v);
  }
  if (e.drop.on()) v *= e.drop.mul((uint64_t)m * e.N + n);
  if (e.res) v += to_f32(((const OutT*)e.res)[(int64_t)m * e.ldr + n]);
  ((OutT*)e.C)[(int64_t)m * e.ldc + n] = from_f32<OutT>(v);
}

// XCD-aware bijective remap: blocks dealt round-robin over 8 XCDs become
// contiguous chunks of the tile sequence per XCD (cdna guide T1, bijective form).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ============================================================ bf16 kernel ===
// Two tile configurations of one kernel template:
//   <128, 2>: 128x128 block, 4 waves, 2-stage LDS ring (64 KiB -> 2 WGs/CU)  [small grids]
//   <256, 3>: 256x128 block, 8 waves, 3-stage LDS ring (144 KiB -> 1 WG/CU)  [large grids]
// Every wave owns a 64x64 output (4x4 16x16 blocks).  The ring keeps NST-1 K-tiles in
// flight: a counted `s_waitcnt vmcnt` retires only the tile about to be read and a raw
// s_barrier (no vmcnt(0) drain) publishes it (cdna guide §5 "Pipelining across barriers").
constexpr int BN = 128, BKT = 64;  // BKT: K granularity required of K-major operands (max BK)

// K-major image [rows][BK k]: 16-B chunk c of row r stored at chunk c ^ swz_k(r):
// conflict-free ds_read_b128 of the 16x16x32 operand for 128-B (BK=64) and 64-B (BK=32) rows.
template <int BKX>
__device__ __forceinline__ int swz_k(int r) { return BKX == 64 ? ((r >> 1) & 7) : ((r >> 1) & 3); }
// MN-major image [BK k][rows] (2*rows-B rows): chunk c of k-row r stored at
// c ^ (f(r)<<1), f(r) = (r&3) | ((r>>3)&1)<<2 -> conflict-free ds_read_b64_tr_b16.
__device__ __forceinline__ int swz_t(int r) { return (((r & 3) | (((r >> 3) & 1) << 2)) << 1); }

template <int BMX, int BKX, int NST>
struct Cfg {
  static constexpr int WAVES = BMX / 32;                 // (BMX/64) x 2 waves, 64x64 outputs each
  static constexpr int THREADS = WAVES * 64;
  static constexpr int A_BYTES = BMX * BKX * 2;
  static constexpr int B_BYTES = BN * BKX * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_PIECES = A_BYTES / 1024 / WAVES;  // 1-KiB LDS-DMA pieces per wave
  static constexpr int B_PIECES = B_BYTES / 1024 / WAVES;
  static constexpr int VM_PER_STAGE = A_PIECES + B_PIECES;
  static constexpr int EPI_LD = BN + 4;
  static constexpr int EPI_BYTES = 64 * EPI_LD * 4;       // epilogue staged 64 rows at a time
  static constexpr int SMEM = (NST * STAGE > EPI_BYTES) ? NST * STAGE : EPI_BYTES;
};

// Stage one ROWS x BKX operand tile into LDS: NP 1-KiB pieces per wave starting at piece p0.
// K-major operands use global_load_lds; MN-major (transposed) operands use
// range-checked buffer_load ... lds whose descriptor ends at row K, so K-tail rows
// of a split reduction (token counts that are not multiples of 64) read as 0.
template <bool KMAJ, int ROWS, int BKX, int NP>
__device__ __forceinline__ void stage_tile(const bf16* __restrict__ X, int64_t ld, int rows, int row0,
                                           int k0, char* lds_tile, int p0, int lane, __amdgpu_buffer_rsrc_t rsrc) {
#pragma unroll
  for (int t = 0; t < NP; ++t) {
    const int ins = p0 + t;
    if constexpr (KMAJ) {
      constexpr int CPR = BKX / 8;         // chunks per row
      constexpr int RPP = 64 / CPR;        // rows per piece
      const int r = ins * RPP + lane / CPR;
      const int lc = (lane % CPR) ^ swz_k<BKX>(r);
      int gr = row0 + r;
      gr = gr < rows ? gr : rows - 1;
      const bf16* src = X + (int64_t)gr * ld + k0 + lc * 8;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(lds_tile + ins * 1024), 16, 0, 0);
    } else {
      constexpr int CPR = ROWS / 8;          // 16-B chunks per k-row
      constexpr int RPP = 64 / CPR;          // k-rows per 1-KiB piece
      const int kr = ins * RPP + lane / CPR;
      const int lc = (lane % CPR) ^ swz_t(kr);
      int gc = row0 + lc * 8;
      gc = gc + 8 <= rows ? gc : rows - 8;
      const unsigned voff = (unsigned)(((int64_t)(k0 + kr) * ld + gc) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(lds_tile + ins * 1024),
                                               16, voff, 0, 0, 0);
    }
  }
}

template <bool KMAJ, int ROWS, int BKX>
__device__ __forceinline__ bf16x8 read_frag(const char* tile, int rbase, int s, int lane) {
  if constexpr (KMAJ) {
    const int r = rbase + (lane & 15);
    const int lc = s * 4 + (lane >> 4);
    return *(const bf16x8*)(tile + r * (BKX * 2) + ((lc ^ swz_k<BKX>(r)) << 4));
  } else {
    constexpr int RB = ROWS * 2;
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
    const int lc = (rbase >> 3) + (p >> 1);
    const int kr0 = s * 32 + g * 8 + q, kr1 = kr0 + 4;
    const char* a0 = tile + kr0 * RB + ((lc ^ swz_t(kr0)) << 4) + (p & 1) * 8;
    const char* a1 = tile + kr1 * RB + ((lc ^ swz_t(kr1)) << 4) + (p & 1) * 8;
    bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, a0));
    bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, a1));
    bf16x8 r;
    r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
    r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
    return r;
  }
}

template <int VM>
__device__ __forceinline__ void wait_vm() {
  if constexpr (VM == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (VM == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (VM == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (VM == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (VM == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (VM == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(VM == 0, "unsupported vmcnt");
}

// Main loop: an NST-deep LDS ring.  Before reading K-tile kt a counted
// `s_waitcnt vmcnt` retires only that tile (the NST-2 younger ones stay in flight),
// then a raw s_barrier publishes it and the slot freed one iteration ago is refilled.
template <int BMX, int BKX, int NST, bool AK, bool BK, typename OutT>
__global__ __launch_bounds__(BMX / 32 * 64) void gemm_bf16_kernel(
    const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb, int M, int N, int K, int splits,
    Epi e, float* __restrict__ ws) {
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
  // range-checked descriptors for MN-major operands: [0, K*ld) elements are valid
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)((int64_t)K * lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)((int64_t)K * ldb * 2), 0x00020000);

  auto stage = [&](int kt, int slot) {
    char* base = smem + slot * C::STAGE;
    stage_tile<AK, BMX, BKX, C::A_PIECES>(A, lda, M, m0, (kt0 + kt) * BKX, base, wave * C::A_PIECES, lane, rsA);
    stage_tile<BK, BN, BKX, C::B_PIECES>(B, ldb, N, n0, (kt0 + kt) * BKX, base + C::A_BYTES, wave * C::B_PIECES,
                                         lane, rsB);
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

// ====================================================== 256x256 bf16 kernel ===
// Large-grid tile: 256x256x64, 8 waves as 2 (M) x 4 (N), 128x64 outputs per wave (8x4
// 16x16 accumulators = 128 VGPRs).  Twice the FLOP per staged byte of the 128x128 tile
// (32 B/clk/CU of L2->LDS traffic at the MFMA rate instead of 64, the per-CU L2 limit),
// 2-deep LDS ring (2 x 64 KiB -> 1 WG/CU), one raw barrier per K-tile: the next tile's
// LDS-DMA is issued right after the barrier and lands under the 64 MFMAs of this one.
template <int BKX, int NST, bool AK, bool BK, typename OutT>
__global__ __launch_bounds__(512) void gemm256_kernel(const bf16* __restrict__ A, int64_t lda,
                                                      const bf16* __restrict__ B, int64_t ldb, int M, int N, int K,
                                                      int splits, Epi e, float* __restrict__ ws) {
  constexpr int BM = 256, BNN = 256;
  constexpr int A_BYTES = BM * BKX * 2, B_BYTES = BNN * BKX * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PIECES = STAGE / 1024 / 8;  // LDS-DMA pieces per wave per stage (A and B halves)
  constexpr int EPI_LD = BNN + 4;
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int ntm = (M + BM - 1) / BM, ntn = (N + BNN - 1) / BNN, ntiles = ntm * ntn;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles, tile = wg % ntiles;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BNN;
  const int nk_all = (K + BKX - 1) / BKX;
  const int kt_per = (nk_all + splits - 1) / splits;
  const int kt0 = split * kt_per;
  const int kt1 = min(nk_all, kt0 + kt_per);
  const int nk = max(0, kt1 - kt0);
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)((int64_t)K * lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)((int64_t)K * ldb * 2), 0x00020000);

  auto stage = [&](int kt, int slot) {
    char* base = smem + slot * STAGE;
    stage_tile<AK, BM, BKX, PIECES / 2>(A, lda, M, m0, (kt0 + kt) * BKX, base, wave * (PIECES / 2), lane, rsA);
    stage_tile<BK, BNN, BKX, PIECES / 2>(B, ldb, N, n0, (kt0 + kt) * BKX, base + A_BYTES, wave * (PIECES / 2), lane,
                                         rsB);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < nk) stage(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    // retire only tile kt (NST-2 younger tiles stay in flight), then publish it
    if (kt + NST - 2 < nk) wait_vm<(NST - 2) * PIECES>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < nk) stage(kt + NST - 1, (kt + NST - 1) % NST);
    const char* sc = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int s = 0; s < BKX / 32; ++s) {
      bf16x8 bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<BK, BNN, BKX>(sc + A_BYTES, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int ih = 0; ih < 2; ++ih) {
        bf16x8 af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = read_frag<AK, BM, BKX>(sc, wm * 128 + (ih * 4 + i) * 16, s, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[ih * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[ih * 4 + i][j], 0, 0, 0);
      }
    }
  }
  // (the last K-tile was waited with vmcnt(0): no operand load is outstanding here)

  // ---- epilogue, 64 rows at a time through LDS (fp32) -> 8-wide rows (fixed 8 columns per thread)
  constexpr int ITS = 64 * BNN / 8 / 512;
  const int ecol = (tid & 31) * 8, egn = n0 + ecol;
  float bias8[8];
  Raw8<OutT> side[BM / 64][ITS];
  const bool has_side = !ws && prefetch_side<OutT, BM / 64, ITS, 512, 32>(e, m0, egn, tid, bias8, side);
  lds_barrier();
  float* stg = (float*)smem;
#pragma unroll
  for (int h = 0; h < BM / 64; ++h) {
    if (wm == (h >> 1)) {
      const int ib = (h & 1) * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = i * 16 + (lane >> 4) * 4 + r;
            const int col = wn * 64 + j * 16 + (lane & 15);
            stg[row * EPI_LD + col] = acc[ib + i][j][r];
          }
    }
    lds_barrier();
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
      const int row = (it * 512 + tid) >> 5;
      const int gm = m0 + h * 64 + row;
      if (gm < M && egn < N) {
        float v[8];
        Vec8<float>::load(stg + row * EPI_LD + ecol, v);
        if (ws) Vec8<float>::store(ws + ((int64_t)split * M + gm) * N + egn, v);
        else epilogue8<OutT>(e, gm, egn, v, e.bias ? bias8 : nullptr, has_side ? &side[h][it] : nullptr);
      }
    }
    lds_barrier();
  }
}

// Activation pass after a library GEMM (the hipBLASLt route of an activation product):
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
        v[k] = act_fwd_fast(a, v[k]);
        w[k] = act_fwd_fast(a, w[k]);
      }
      Vec8<OutT>::store(C + i * 8, v);
      Vec8<OutT>::store(C + (i + stride) * 8, w);
    }
    if (i < total) {
      float v[8];
      Vec8<OutT>::load(pre + i * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd_fast(a, v[k]);
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
        v[k] *= (act & CAPK_ACT_DERIV) ? g[k] : act_grad_fast(a, g[k]);
        if (two) w[k] *= (act & CAPK_ACT_DERIV) ? h[k] : act_grad_fast(a, h[k]);
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
      for (int k = 0; k < 8; ++k) v[k] = act_fwd_fast(a, v[k]);
      Vec8<OutT>::store(C + (int64_t)m * ldc + n, v);
      continue;
    }
    Vec8<OutT>::load(C + (int64_t)m * ldc + n, v);
    if (act & CAPK_ACT_BWD) {
      float g[8];
      Vec8<OutT>::load(aux + (int64_t)m * ldx + n, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= (act & CAPK_ACT_DERIV) ? g[k] : act_grad_fast(a, g[k]);
    } else if (pre && (act & CAPK_ACT_DERIV)) {
      float d[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd_grad_fast(a, v[k], d[k]);
      Vec8<OutT>::store(pre + (int64_t)m * ldx + n, d);
    } else {
      if (pre) Vec8<OutT>::store(pre + (int64_t)m * ldx + n, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = act_fwd_fast(a, v[k]);
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
static int cfg_override() {
  static int v = [] {
    const char* s = getenv("CAPK_GEMM_CFG");
    return s ? atoi(s) : 0;
  }();
  return v;
}
// Tile configurations (CAPK_GEMM_CFG overrides for A/B measurements):
//   1: 128x128, BK 64, 2-deep ring (64 KiB, 2 WGs/CU)
//   2: 256x128, BK 64, 3-deep ring (144 KiB, 1 WG/CU)
//   3: 128x128, BK 32, 4-deep ring (64 KiB, 2 WGs/CU)
//   4: 128x128, BK 32, 3-deep ring (48 KiB, 3 WGs/CU)
static bool big_tile(int cfg) { return cfg == 5 || cfg == 6; }
static int slots_of(int cfg) { return (cfg == 2 || big_tile(cfg)) ? 256 : cfg == 4 ? 768 : 512; }  // resident WGs
static int tiles_of(int cfg, int M, int N) {
  return cdiv(M, (cfg == 2 || big_tile(cfg)) ? 256 : 128) * cdiv(N, big_tile(cfg) ? 256 : BN);
}
// Measured per shape class (tools/gemm_bench.py, profiles/): the 3-WG/CU BK-32 ring wins when
// the epilogue carries an activation (its stores overlap other WGs' main loops) and for the
// split-K weight-gradient GEMMs whose grid fits one round; the 2-WG/CU BK-64 ring elsewhere.
static int choose_cfg(int M, int N, int K, int a_kmajor, int b_kmajor, int act) {
  int o = cfg_override();
  if ((o == 2 || big_tile(o)) && M < 256) o = 1;
  if ((o == 3 || o == 4 || o == 6) && (a_kmajor || b_kmajor) && K % 32) o = 1;
  if (o >= 1 && o <= 6) return o;
  if (act && (a_kmajor || b_kmajor) && K % 32 == 0) return 4;
  if (!a_kmajor && !b_kmajor && tiles_of(4, M, N) < slots_of(4)) return 1;  // split-K dW (cfg 4 measured slower)
  return 1;
}
// Split-K factor: fill one round of resident workgroups when the tile grid alone cannot
// (any integer factor; every split keeps >= 4 K-tiles).
static int choose_splits(int cfg, int M, int N, int K) {
  const int bk = (cfg == 3 || cfg == 4 || cfg == 6) ? 32 : 64;
  const int tiles = tiles_of(cfg, M, N), slots = slots_of(cfg);
  const int nk = cdiv(K, bk);
  if (2 * tiles >= slots) return 1;
  int s = std::min(16, slots / tiles);
  s = std::min(s, std::max(1, nk / 4));
  return std::max(1, s);
}

// blaslt.cpp
bool lt_enabled();
bool lt_gemm(int out_f32, int M, int N, int K, const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb,
             int b_kmajor, void* C, int64_t ldc, float alpha, float beta, const float* bias, const void* residual,
             int64_t ldr, void* ws, size_t ws_bytes, hipStream_t st);
size_t lt_workspace_bytes();

}  // namespace capk

using namespace capk;

static thread_local int g_last_route = 0;
extern "C" int capk_gemm_last_route(void) { return g_last_route; }

extern "C" size_t capk_gemm_workspace(int in_dtype, int out_dtype, int M, int N, int K) {
  (void)out_dtype;
  if (in_dtype != CAPK_BF16) return 0;
  // upper bound over the configurations (the launch picks one of them)
  int s = 1;
  for (int c = 1; c <= 6; ++c) s = std::max(s, choose_splits(c, M, N, K));
  const size_t slabs = s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
  return lt_enabled() ? std::max(slabs, lt_workspace_bytes()) : slabs;
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
  // plain products with a K-major A (forward Linear without activation, dX) -> hipBLASLt
  // (K >= 32768, the LM-head dX, measured no faster there)
  if (lt_enabled() && act == 0 && !(drop_p > 0.f) && a_kmajor && K < 32768 &&
      lt_gemm(out_dtype == CAPK_F32, M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, alpha, beta, bias, residual,
              ldr, ws, ws_bytes, st)) {
    g_last_route = 1;
    return CAPK_OK;
  }
  // activation products (bias + act with its side output, or x act'): library GEMM for the
  // product, then one elementwise pass -- measured faster than the fused epilogue on the
  // FFN shapes because the library main loop is faster than gemm_bf16_kernel's
  // (a plain forward act that keeps pre writes the product straight into preact: one stream less)
  const int from_pre = !(act & CAPK_ACT_BWD) && !(act & CAPK_ACT_DERIV) && preact != nullptr;
  if (lt_enabled() && (act & 15) && !(drop_p > 0.f) && a_kmajor && K < 32768 && !residual && beta == 0.f &&
      out_dtype == CAPK_BF16 &&
      lt_gemm(0, M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, from_pre ? preact : C, from_pre ? ldx : ldc, alpha, 0.f,
              (act & CAPK_ACT_BWD) ? nullptr : bias, nullptr, 0, ws, ws_bytes, st)) {
    const int64_t segs = (int64_t)M * (N / 8);
    // dense rows: one launch-wide pass, each lane a pair of segments (flat paths in act_pass_kernel)
    const bool dense = ldc == N && ldx == N && (from_pre || (act & CAPK_ACT_BWD));
    const int grid_a = (int)std::min<int64_t>(dense ? cdiv(segs, 512) : cdiv(segs, 256), dense ? (1 << 20) : 8192);
    hipLaunchKernelGGL(act_pass_kernel<bf16>, dim3(grid_a), dim3(256), 0, st, M, N, (bf16*)C, ldc, (bf16*)preact,
                       (const bf16*)aux, ldx, act, from_pre);
    CAPK_LAUNCH_CHECK("act_pass_kernel");
    g_last_route = 1;
    return CAPK_OK;
  }
  g_last_route = 0;
  const int cfg = choose_cfg(M, N, K, a_kmajor, b_kmajor, act);
  int splits = choose_splits(cfg, M, N, K);
  if (!ws || ws_bytes < (size_t)splits * M * N * sizeof(float)) splits = 1;
  const int tiles = tiles_of(cfg, M, N);
  const int grid = tiles * splits;
  float* slab = splits > 1 ? (float*)ws : nullptr;
#define LAUNCH1(BMX, BKX, NST, AK, BKM, OT)                                                                     \
  hipLaunchKernelGGL((gemm_bf16_kernel<BMX, BKX, NST, AK, BKM, OT>), dim3(grid), dim3(BMX / 32 * 64), 0, st, \
                     (const bf16*)A, lda, (const bf16*)B, ldb, M, N, K, splits, e, slab)
#define LAUNCH(AK, BKM, OT)                                    \
  do {                                                         \
    switch (cfg) {                                             \
      case 5:                                                  \
        hipLaunchKernelGGL((gemm256_kernel<64, 2, AK, BKM, OT>), dim3(grid), dim3(512), 0, st, (const bf16*)A, \
                           lda, (const bf16*)B, ldb, M, N, K, splits, e, slab); \
        break;                                                 \
      case 6:                                                  \
        hipLaunchKernelGGL((gemm256_kernel<32, 4, AK, BKM, OT>), dim3(grid), dim3(512), 0, st, (const bf16*)A, \
                           lda, (const bf16*)B, ldb, M, N, K, splits, e, slab); \
        break;                                                 \
      case 2: LAUNCH1(256, 64, 3, AK, BKM, OT); break;         \
      case 3: LAUNCH1(128, 32, 4, AK, BKM, OT); break;         \
      case 4: LAUNCH1(128, 32, 3, AK, BKM, OT); break;         \
      default: LAUNCH1(128, 64, 2, AK, BKM, OT); break;        \
    }                                                          \
  } while (0)
#define DISPATCH(OT)                          \
  if (a_kmajor && b_kmajor) LAUNCH(true, true, OT);     \
  else if (a_kmajor) LAUNCH(true, false, OT);           \
  else if (b_kmajor) LAUNCH(false, true, OT);           \
  else LAUNCH(false, false, OT);
  if (out_dtype == CAPK_BF16) { DISPATCH(bf16) } else { DISPATCH(float) }
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
