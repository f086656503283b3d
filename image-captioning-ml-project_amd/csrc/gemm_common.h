// Shared pieces of the bf16 GEMM kernels (gemm.hip: 128-row tiles + dispatch;
// gemm8p.hip: the 256x256 phased kernel): epilogue, LDS staging of operand tiles,
// fragment reads.  See gemm.hip for the design notes.
#pragma once
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
      for (int i = 0; i < 8; ++i) v[i] *= act_grad_fast<OutT>(act, a[i]);
    }
  } else if (e.act) {
    const int act = e.act & 15;
    if (e.pre && (e.act & CAPK_ACT_DERIV)) {
      float d[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = act_fwd_grad_fast<OutT>(act, v[i], d[i]);
      Vec8<OutT>::store((OutT*)e.pre + (int64_t)m * e.ldx + n, d);
    } else {
      if (e.pre) Vec8<OutT>::store((OutT*)e.pre + (int64_t)m * e.ldx + n, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = act_fwd_fast<OutT>(act, v[i]);
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
  // Unconditional loads with clamped rows / columns (tail lanes load a valid segment they
  // never store): a branch per load makes every value a phi, and hipcc then waits
  // vmcnt(0) behind each load to copy it -- one memory round trip per segment.
  const int gnc = gn < e.N ? gn : e.N - 8;
  if (e.bias) Vec8<float>::load(e.bias + gnc, bias8);
  if (!sp) return false;
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
      const int gm = m0 + h * 64 + (it * THREADS + tid) / SEGS_PER_ROW;
      side[h][it].load(sp + (int64_t)(gm < e.M ? gm : e.M - 1) * sld + gnc);
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
  else if constexpr (VM == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if constexpr (VM == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else static_assert(VM == 0, "unsupported vmcnt");
}

// ---- pieces shared by the 256x256 kernels (gemm8p.hip, gemm8q.hip) ----
template <int VM>
__device__ __forceinline__ void wait_vmc() {
  static_assert(VM >= 0 && VM <= 16 && VM % 2 == 0, "unsupported vmcnt");
  if constexpr (VM == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (VM == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (VM == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (VM == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (VM == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (VM == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (VM == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (VM == 14) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Per-lane byte offset of LDS-DMA piece `ins` (0..15) of a 128-row half-tile whose first
// row (K-major) / column (MN-major) is row0; k0 = 0.  K-major image [128 rows][64 k]
// (chunk c of row r at c ^ swz_k<64>(r)); MN-major image [64 k][128 cols] (chunk c of
// k-row r at c ^ swz_t(r)).
template <bool KMAJ, int ESZ = 2>
__device__ __forceinline__ uint32_t piece_voff(int ins, int lane, int row0, int rows, int64_t ld) {
  if constexpr (KMAJ) {
    const int r = ins * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ swz_k<64>(r);
    return (uint32_t)((int64_t)(row0 + r) * ld * ESZ + lc * 16);
  } else {
    const int kr = ins * 4 + (lane >> 4);
    const int lc = (lane & 15) ^ swz_t(kr);
    int gc = row0 + lc * 8;
    gc = gc + 8 <= rows ? gc : rows - 8;
    return (uint32_t)(((int64_t)kr * ld + gc) * 2);
  }
}

// One 16x16x32 operand fragment from a half-tile image.  K-major: ds_read_b128 (as
// read_frag).  MN-major: two ds_read_b64_tr_b16 issued as inline asm -- hipcc treats the
// transpose-read builtin as aliasing every LDS-DMA in flight and drains vmcnt(0) before it,
// which would serialise the load pipeline; the caller waits lgkmcnt itself (every phase
// boundary has `s_waitcnt lgkmcnt(0)` before the first MFMA that consumes a fragment).
template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag(const char* half, int rbase, int s, int lane) {
  if constexpr (KMAJ) {
    return read_frag<true, 128, 64>(half, rbase, s, lane);
  } else {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
    const int lc = (rbase >> 3) + (p >> 1);
    const int kr0 = s * 32 + g * 8 + q;  // kr0 + 4 has the same swizzle: +1024 bytes
    const uint32_t a = (uint32_t)(uintptr_t)LDS_PTR(char, half + kr0 * 256 + ((lc ^ swz_t(kr0)) << 4) + (p & 1) * 8);
    bf16x4 x0, x1;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(x0) : "v"(a));
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:1024" : "=v"(x1) : "v"(a));
    bf16x8 r;
    r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
    r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
    return r;
  }
}

// gemm8p.hip: launch the 256x256 phased kernel (grid = tiles * splits)
int launch_gemm8p(bool a_kmajor, bool b_kmajor, bool out_f32, int grid, const void* A, int64_t lda, const void* B,
                  int64_t ldb, int M, int N, int K, int splits, const Epi& e, float* slab, hipStream_t st);
// fp8 e4m3 x e4m3 (both K-major, K % 128 == 0) with per-row E8M0 scales (gemm8p.hip)
int launch_gemm8p_f8(bool out_f32, int grid, const void* A, int64_t lda, const uint8_t* scA, const void* B,
                     int64_t ldb, const uint8_t* scB, int M, int N, int K, int splits, const Epi& e, float* slab,
                     hipStream_t st);
// gemm8q.hip: the persistent 256x256 kernel (grid = min(tiles * splits, 256))
bool gemm8q_supports(const Epi& e, bool out_f32);
// misc.hip: out[n] (+)= sum over `parts` partial rows part[r][n] (fixed order)
int launch_colsum_finish(int parts, int N, const float* part, float* out, int accumulate, hipStream_t st);

// dsum != nullptr: the dX x act' product also writes per-(tile row, wave row) column-sum
// partials [2 * cdiv(M, 256)][N] fp32 there (capk_gemm_dx_act_colsum)
// lse_part != nullptr (plain K-major bf16 products; no tail round): also the softmax partials of
// the stored C over columns < lse_v, [cdiv(N, 256) * 4][M] (max, sum exp) pairs in the log2
// domain (capk_linear_lse)
// tail_r0 != nullptr and ws of gemm8q_tail_workspace() bytes: the split-K tail round when
// gemm8q_tail_plan() picks one -- then, unless the launch combines the slabs itself (tail mode
// 2), *tail_r0 >= 0 and the caller must reduce the fp32 slabs ws[*tail_splits][M - 256
// *tail_r0][N] into rows [256 *tail_r0, M) with the epilogue (splitk_reduce_kernel);
// otherwise *tail_r0 = -1 and the launch wrote every row
int launch_gemm8q(bool a_kmajor, bool b_kmajor, bool out_f32, const void* A, int64_t lda, const void* B, int64_t ldb,
                  int M, int N, int K, int splits, const Epi& e, float* slab, hipStream_t st, float* dsum = nullptr,
                  void* ws = nullptr, size_t ws_bytes = 0, int* tail_r0 = nullptr, int* tail_splits = nullptr,
                  float* lse_part = nullptr, int lse_v = 0);
bool gemm8q_tail_plan(int M, int N, int K, int* r0, int* splits);
size_t gemm8q_tail_workspace(int M, int N, int K);

}  // namespace capk
