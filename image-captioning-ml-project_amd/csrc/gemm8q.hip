// Persistent 256x256 bf16 GEMM (round 3) -- the large-grid kernel of capk_gemm for grids
// of more than one round.  The main loop is gemm8p.hip's: 256x256x64 tiles, 8 waves (2 x 4),
// four 16-KiB half-tiles per K-tile staged by LDS-DMA through two 64-KiB stages, two phases
// of 32 v_mfma_f32_16x16x32_bf16 per K-tile, waves 4-7 one barrier behind waves 0-3, static
// vmcnt counts.  What changes is everything around it:
//
//  * Persistent grid of 256 workgroups (one per CU).  WG b takes items first + 256 j with
//    first = (b & 7) * 32 + (b >> 3): the 32 WGs of an XCD work on 32 consecutive items of
//    the row-major tile order at a time, so that XCD's L2 holds the A rows and B columns
//    they share.  Every item has the same number of K-tiles nk (>= 2).
//  * ONE continuous K-tile sequence over all of the WG's items (step u = item j's K-tile
//    u - j nk): the LDS-DMA schedule of gemm8p (phase Q1 of step u issues half A1 of step
//    u+1, Q2 issues A0/B0/B1 of step u+2) runs across item boundaries, so the next item's
//    first two K-tiles are loaded under the current item's last two and only the WG's
//    first item pays a prologue.
//  * Register-direct epilogue (no LDS staging: the stages hold the next item's K-tiles).
//    The MFMAs take the B fragment first, so a lane's accumulator holds 4 consecutive
//    columns of one row; one v_permlane16_swap per register pair turns the two 16-column
//    blocks of a 32-column strip into 8 consecutive columns per lane, written by one 16-B
//    buffer store (16 rows x 64 contiguous bytes per store instruction).  The item's bias
//    (the wave's 64 columns) is LDS-DMA-ed with the item's first K-tile into a per-wave
//    slot; a side operand (residual / aux / C) is loaded per half by 8 buffer loads.
//    Rows and columns past M / N go through the buffer descriptors' range checks, so every
//    wave issues the same memory instructions.
//  * The epilogue's stores are left in flight: they drain while the next item's first
//    K-tile computes.  vmcnt counts loads, LDS-DMA and stores together in issue order, so
//    the two waits after an epilogue add its store count S (a compile-time function of the
//    instantiation and the run-time output kind); every other wait is gemm8p's count (+1
//    where the phase issued a bias DMA).  Too small a count is safe (it only waits longer),
//    so the run-time counts are rounded down to the encodings wait_le() has.
//
//  * Split-K tail round (round 4, TAIL: grids whose last round is partly empty, e.g. the
//    591 items = 2.31 rounds of a 50 432 x 768 product, when K is long enough): only the
//    row blocks [0, r0) run as whole items (r0 * ntn <= 256 * rounds), and the remaining
//    row blocks run as S K-splits per tile in one extra round (T * S <= 256 parts), each
//    part writing its fp32 accumulators to its own slab; the host then launches the split-K
//    reduce + epilogue over those rows (tail mode 1, default; gemm.hip: splitk_reduce_kernel).
//    Tail mode 2 (round 6, opt-in) combines inside the launch instead: each part draws an
//    arrival ticket for its tile (slab stores drained, one agent-scope release); the part
//    drawing the last one takes one agent-scope acquire, sums the tile's slabs in split order
//    and runs the item's register epilogue -- bit-identical to mode 1, but measured 30-33 us
//    SLOWER per ViT product (profiles/round6/gemm_tail_combine_ab.txt): one WG per tail tile
//    reads its 3 x 256 KiB of slabs at ~30 GB/s, where the reduce launch spreads the same
//    bytes over the whole chip (round 4's pairwise hand-off through an sc1 workspace lost
//    the same way, profiles/round4/ab_round4.md).  Contiguous-range stream-K was measured
//    slower (profiles/round4/streamk_contiguous_ab.txt: concurrent WGs no longer shared A
//    row blocks in L2).
//
// Epilogue (compile-time forms, gemm8q_supports): bias, a forward GELU-family / ReLU
// activation with act'(pre) (DV) or pre kept, OR one side operand -- the backward multiply by
// aux = act'(pre), a residual, or beta*C -- and optionally (DSUM) the column sums of the
// result.  alpha != 1, dropout and split-K run on gemm8p.
#include <atomic>
#include <ctime>
#include <map>
#include <mutex>
#include <type_traits>

#include "gemm_common.h"

namespace capk {

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long gu64;  // hand-off flag words: global, never flat
typedef __attribute__((address_space(1))) unsigned gu32;

// One segment of the side operand (8 elements of one row) loaded by an asm buffer load that
// hipcc does not count; the epilogue waits for all of them with one vmcnt(0) statement that
// names every destination.
template <typename T> struct SideSeg;
template <> struct SideSeg<bf16> {
  i32x4 a;
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(a) : "v"(off), "s"(rs) : "memory");
  }
  __device__ __forceinline__ float get(int i) const {
    const bf16x8 v = __builtin_bit_cast(bf16x8, a);
    return (float)v[i];
  }
};
template <> struct SideSeg<float> {
  i32x4 a, b;
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(a) : "v"(off), "s"(rs) : "memory");
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:16" : "=v"(b) : "v"(off), "s"(rs) : "memory");
  }
  __device__ __forceinline__ float get(int i) const {
    const int x = i < 4 ? a[i] : b[i - 4];
    return __int_as_float(x);
  }
};

// 8 results of one row segment -> one (bf16) or two (fp32) 16-byte buffer stores
__device__ __forceinline__ void store8(__amdgpu_buffer_rsrc_t rs, uint32_t off, const float (&v)[8], bf16*) {
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, o), rs, off, 0, 0);
}
__device__ __forceinline__ void store8(__amdgpu_buffer_rsrc_t rs, uint32_t off, const float (&v)[8], float*) {
  const i32x4 a = {__float_as_int(v[0]), __float_as_int(v[1]), __float_as_int(v[2]), __float_as_int(v[3])};
  const i32x4 b = {__float_as_int(v[4]), __float_as_int(v[5]), __float_as_int(v[6]), __float_as_int(v[7])};
  __builtin_amdgcn_raw_buffer_store_b128(a, rs, off, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(b, rs, off + 16, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(bytes < 0x7FFFFFFF ? bytes : 0x7FFFFFFF),
                                           0x00020000);
}

constexpr uint32_t OOR = 0x80000000u;  // a buffer offset past every descriptor's range: dropped / reads 0
constexpr float kLog2eG = 1.4426950408889634f;
// 2^x on v_exp_f32 (x <= 0 or -inf -> 0; NaN only from -inf - -inf, which the callers exclude)
__device__ __forceinline__ float fexp2s(float x) { return __builtin_amdgcn_exp2f(x); }

// side operand kind (at most one per launch: gemm8q_supports)
enum { SIDE_NONE = 0, SIDE_AUX = 1, SIDE_RES = 2, SIDE_C = 3 };

// The epilogue as the kernel sees it (built from Epi on the host: the side operand is already
// chosen, so every field is a plain wave-uniform value).
struct Epi8q {
  void* C;
  const void* side;
  void* pre;
  const float* bias;
  int64_t ldc, lds, ldp;
  float beta;
  float* dsum;  // DSUM kernels: column-sum partials [2 * tile rows][N]
  float* tail_ws;  // TAIL kernels: fp32 slabs [splits][M - 256 tail_r0][N] of the tail row blocks
  int tail_r0, tail_splits;
  int* tail_cnt;   // TAIL kernels, in-launch combine: one arrival ticket per tail tile (zero on entry,
                   // zeroed again by the tile's last arriver); nullptr: the host launches the reduce
  float* lse_part;  // LSEP kernels: softmax partials [ntn * 4][M] of (max, sum exp) pairs (float2)
  int lse_v;        // LSEP: columns >= lse_v are padding (excluded from the partials)
  int group;  // grouped raster: tiles of the whole-item rows in groups of `group` row blocks, column-major
              // inside a group (0: row-major); host: gemm8q_group()
  unsigned long long* trace;  // CAPK_DIAG_TRACE builds only: per-item timestamps
};


// s_waitcnt vmcnt(<= n) for a wave-uniform run-time n: the largest encoded count <= n
__device__ __forceinline__ void wait_le(int n) {
#define CAPK_W(N) \
  if (n >= N) { asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); return; }
  CAPK_W(40) CAPK_W(39) CAPK_W(38) CAPK_W(34) CAPK_W(33) CAPK_W(32) CAPK_W(24) CAPK_W(23) CAPK_W(22)
  CAPK_W(18) CAPK_W(17) CAPK_W(16) CAPK_W(15) CAPK_W(14) CAPK_W(10) CAPK_W(9) CAPK_W(8) CAPK_W(7) CAPK_W(6)
  CAPK_W(4) CAPK_W(3) CAPK_W(2) CAPK_W(1)
#undef CAPK_W
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ACT: the forward activation the epilogue evaluates (CAPK_ACT_* kind, 0 = none), a template
// parameter so each of the 16 unrolled epilogue segments carries only its own code.
// SIDE: the epilogue reads a side operand (residual / aux / C).
// DSUM: also the column sums of the final values (the bias gradient of the Linear whose
// output gradient this dX is): per (tile row, wm) partial rows [2 ntm][N] into e.dsum,
// summed in a fixed order by colsum_finish (capk_gemm_dx_act_colsum).
template <bool AK, bool BK, typename OutT, int ACT, bool DV, int SK, bool DSUM = false, bool TAIL = false,
          bool LSEP = false, bool TCOMB = false>
__global__ __launch_bounds__(512) void gemm8q_kernel(const void* __restrict__ A, int64_t lda,
                                                     const void* __restrict__ B, int64_t ldb, int M, int N, int K,
                                                     int splits, Epi8q e) {
  constexpr int HALF = 128 * 64 * 2, STAGE = 4 * HALF, BIAS0 = 2 * STAGE;
  // two stages + bias slots [item parity][wave] of 64 fp32 (the wave's columns)
#if defined(CAPK_DIAG_TRACE)  // diagnostic build: per-item timestamps of waves 0 and 4 (LDS, then e.trace)
  constexpr int TR_ITEMS = 64, TR_BYTES = 2 * TR_ITEMS * 4 * 8;
#else
  constexpr int TR_BYTES = 0;
#endif
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 2 * 8 * 256 + 16 + TR_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool lag = wave >= 4;  // waves 4-7 run one barrier behind
  const int ntn = (N + 255) / 256, ntiles = ((M + 255) / 256) * ntn, items = ntiles * splits;
  const int nk = ((K + 63) / 64 + splits - 1) / splits;  // K-tiles per item (>= 2: host)
  const int first = (blockIdx.x & 7) * 32 + (blockIdx.x >> 3);  // grid = 256
  // segments: whole items first + 256 j (< W), then (TAIL) one K-split part of a tail tile:
  // part p = first (< T * S) is split p / T of tail tile p % T, so the WGs of an XCD run one
  // split of neighbouring tiles (shared A row-block slices in its L2)
  const int W = TAIL ? e.tail_r0 * ntn : items, T = items - W, TS = TAIL ? e.tail_splits : 1;
  const bool hasTail = TAIL && first < T * TS;
  const int tsplit = hasTail ? first / T : 0, ttile = hasTail ? first % T : 0;
  const int tk0 = tsplit * nk / TS, tk1 = (tsplit + 1) * nk / TS;
  const int nwhole = first < W ? (W - first + 255) >> 8 : 0;
  const int nseg = nwhole + hasTail;
  if (nseg == 0) return;
  const int total = nwhole * nk + (hasTail ? tk1 - tk0 : 0);  // K-tile steps of this WG

  const __amdgpu_buffer_rsrc_t rsA = rsrc_of(A, (AK ? (int64_t)M * lda : (int64_t)K * lda) * 2);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_of(B, (BK ? (int64_t)N * ldb : (int64_t)K * ldb) * 2);
  const uint32_t kstepA = AK ? 128u : (uint32_t)(64 * lda * 2);
  const uint32_t kstepB = BK ? 128u : (uint32_t)(64 * ldb * 2);
  const uint32_t rowA = AK ? (uint32_t)(lda * 2) : 2u, rowB = BK ? (uint32_t)(ldb * 2) : 2u;

  struct Item {
    int m0, n0, kb;  // tile origin, first K-tile of the item's split
    int k0, k1;      // K-tiles [k0, k1) of the item this segment runs
  };
  auto item_at = [&](int j) -> Item {
    int it = first + (j << 8), k0 = 0, k1 = nk;
    if (TAIL && hasTail && j == nseg - 1) {  // this WG's K-split part of a tail tile
      it = W + ttile;
      k0 = tk0;
      k1 = tk1;
    }
    const int sp = it / ntiles, tile = it - sp * ntiles;
    int tm, tn;
    if (e.group > 0 && tile < W) {  // grouped raster over the whole-item rows [0, W / ntn)
      const int gsz = e.group * ntn, g = tile / gsz, r = tile - g * gsz;
      const int rows = min(e.group, W / ntn - g * e.group);
      tn = r / rows;
      tm = g * e.group + (r - tn * rows);
    } else {
      tm = tile / ntn;
      tn = tile - tm * ntn;
    }
    return Item{tm * 256, tn * 256, sp * nk, k0, k1};
  };

  // per-lane byte offsets of this wave's two 1-KiB pieces of each half (h: A0 A1 B0 B1) at
  // row / column 0, k 0 (no clamp: rows / columns past M / N only feed outputs that are
  // never stored, and the descriptor range check zeroes reads past the operand)
  uint32_t vo[4][2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    vo[0][p] = piece_voff<AK, 2>(wave * 2 + p, lane, 0, 1 << 30, lda);
    vo[1][p] = piece_voff<AK, 2>(wave * 2 + p, lane, 128, 1 << 30, lda);
    vo[2][p] = piece_voff<BK, 2>(wave * 2 + p, lane, 0, 1 << 30, ldb);
    vo[3][p] = piece_voff<BK, 2>(wave * 2 + p, lane, 128, 1 << 30, ldb);
  }
  // piece p (0, 1) of this wave's share of half h of K-tile k of item `it` into stage u & 1
  auto load_piece = [&](int h, const Item& it, int k, int u, int p) {
    char* dst = smem + (u & 1) * STAGE + h * HALF;
#if defined(CAPK_DIAG_ROW0)  // diagnostic build: every item reads the A rows of tile row 0 (L2-resident)
    const uint32_t so = h < 2 ? (uint32_t)(it.kb + k) * kstepA : (uint32_t)it.n0 * rowB + (uint32_t)(it.kb + k) * kstepB;
#else
    const uint32_t so = h < 2 ? (uint32_t)it.m0 * rowA + (uint32_t)(it.kb + k) * kstepA
                              : (uint32_t)it.n0 * rowB + (uint32_t)(it.kb + k) * kstepB;
#endif
    __builtin_amdgcn_raw_ptr_buffer_load_lds(h < 2 ? rsA : rsB,
                                             (__attribute__((address_space(3))) void*)(dst + (wave * 2 + p) * 1024),
                                             16, vo[h][p] + so, 0, 0, 0);
  };
  auto load = [&](int h, const Item& it, int k, int u) {
    load_piece(h, it, k, u, 0);
    load_piece(h, it, k, u, 1);
  };
  const bool has_bias = e.bias != nullptr;
  // the wave's 64 bias columns of item j (lane l: column (l >> 5) * 128 + wn * 32 + (l & 31))
  auto bias_dma = [&](const Item& it, int j) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsrc_of(e.bias, (int64_t)N * 4),
        (__attribute__((address_space(3))) void*)(smem + BIAS0 + ((j & 1) * 8 + wave) * 256), 4,
        (uint32_t)(it.n0 + (lane >> 5) * 128 + wn * 32 + (lane & 31)) * 4u, 0, 0, 0);
  };
  constexpr bool SIDE = SK != SIDE_NONE;
  const bool has_pre = ACT != 0 && e.pre != nullptr;

  // ---- fragments and MFMAs (B fragment first: lane = row, registers = 4 consecutive columns)
  auto half = [&](int u, int h) -> const char* { return smem + (u & 1) * STAGE + h * HALF; };
  auto readA = [&](bf16x8 (&f)[2][4], int u, int h) {
    const char* base = half(u, h);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) f[s][i] = frag<AK>(base, wm * 64 + i * 16, s, lane);
  };
  auto readB = [&](bf16x8 (&f)[2][2], int u, int h) {
    const char* base = half(u, h);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j) f[s][j] = frag<BK>(base, wn * 32 + j * 16, s, lane);
  };
  f32x4 acc[2][2][4][2];
  auto zero_acc = [&] {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  };
  auto mma = [&](const bf16x8 (&fa)[2][4], const bf16x8 (&fb)[2][2], f32x4 (&c)[4][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[s][j], fa[s][i], c[i][j], 0, 0, 0);
  };
  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
  // MFMA clusters at wave priority 1 (the lagging group at priority 1 throughout, or no
  // priority changes at all, measured the same: profiles/round5/gemm_prio_ab.txt)
  auto prio_mfma = [] { __builtin_amdgcn_s_setprio(1); };
  auto prio_load = [] { __builtin_amdgcn_s_setprio(0); };
  auto bar = [&] {
    fence();
    raw_barrier();
    fence();
  };
  auto lds_done = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fence();
  };
#if defined(CAPK_DIAG_TRACE)
  // stamp s (0: item's MFMAs done, 1: epilogue done, 2: next item's first data wait done,
  // 3: next item's first MFMA phase entered) of item jx, waves 0 and 4 only
  unsigned long long* const trs = (unsigned long long*)(smem + 2 * STAGE + 2 * 8 * 256 + 16);
  auto stamp = [&](int jx, int st) {
    if ((wave & 3) == 0 && lane == 0 && jx < TR_ITEMS)
      trs[((wave >> 2) * TR_ITEMS + jx) * 4 + st] = __builtin_amdgcn_s_memrealtime();
  };
  if ((wave & 3) == 0)  // unstamped entries read as 0 (the same wave copies them out at the end)
    for (int x = lane; x < TR_ITEMS * 4; x += 64) trs[(wave >> 2) * TR_ITEMS * 4 + x] = 0ull;
#else
  auto stamp = [](int, int) {};
#endif

  // ---- epilogue (register-direct); returns the memory instructions it leaves in flight ----
  const int g4 = lane >> 4, qq = ((g4 & 1) << 1) | (g4 >> 1);  // lane's 8-column group after the swap
  const int lrow = wm * 64 + (lane & 15), lcol = wn * 32 + qq * 8;  // in a 128 x 128 quadrant (+16 i)
  constexpr int ESZ = (int)sizeof(OutT);

  // lane byte offset of (row m0 + lrow, column n0 + qn*128 + lcol) in a [rows][ld] matrix of
  // element size es; columns past N -> OOR (rows past M fail the range check by themselves)
  auto this_lane_off = [&](const Item& c, int64_t ld, int es, int qn) -> uint32_t {
    const int n = c.n0 + qn * 128 + lcol;
    return n < N ? (uint32_t)(((int64_t)(c.m0 + lrow) * ld + n) * es) : OOR;
  };
  // the segment (qm, i) adds (qm*128 + i*16) rows: one v_add of a wave-uniform constant
  auto seg_add = [&](int64_t ld, int es, int qm, int i) -> uint32_t { return (uint32_t)((qm * 128 + i * 16) * ld * es); };
  // One half of an item's epilogue: the 8 segments of quadrant row QM (acc[QM]).
  // Lean per-segment work (the epilogue runs while the CU's MFMAs idle): the accumulator
  // swap, bias (zeros when absent), the compile-time side operand / activation, the store.
  // Out-of-range rows / columns keep the OOR offset (+ a segment offset < 2^26 stays past
  // every descriptor range), so there is no per-segment select.
  auto epi_body = [&](const Item& c, int j, const SideSeg<OutT> (&side)[2][2][4], float (&cs)[2][8],
                      auto qmc) -> int {
    constexpr int QM = decltype(qmc)::value;
    auto lane_off = [&](int64_t ld, int es, int qn) -> uint32_t { return this_lane_off(c, ld, es, qn); };
    // this item's bias (the wave's slot of item parity j & 1): the lane's 8 columns per quadrant
    f32x4 bias[2][2];
    if (has_bias) {
      const float* slot = (const float*)(smem + BIAS0 + ((j & 1) * 8 + wave) * 256);
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
        bias[qn][0] = *(const f32x4*)(slot + qn * 32 + qq * 8);
        bias[qn][1] = *(const f32x4*)(slot + qn * 32 + qq * 8 + 4);
      }
    } else {
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) bias[qn][0] = bias[qn][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    const __amdgpu_buffer_rsrc_t rsC = rsrc_of(e.C, (int64_t)M * e.ldc * ESZ);
    const uint32_t o0 = lane_off(e.ldc, ESZ, 0), o1 = lane_off(e.ldc, ESZ, 1);
    // LSEP: per row i of the lane, running (max, sum exp) over its columns, in the log2 domain
    // (values scaled by log2 e), of the stored (bf16-rounded) logits
    float lm[4], ls[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lm[i] = -INFINITY;
      ls[i] = 0.f;
    }
    const uint32_t p0 = has_pre ? lane_off(e.ldp, ESZ, 0) : OOR, p1 = has_pre ? lane_off(e.ldp, ESZ, 1) : OOR;
    // one 16-row x 32-column segment (qm, qn, i), unrolled by hand (the 16 bodies exceed the
    // unroller's budget, and a rolled loop would index the accumulators dynamically)
    auto segment = [&](auto qmc2, auto qnc, auto ic) {
      constexpr int qm = decltype(qmc2)::value, qn = decltype(qnc)::value, i = decltype(ic)::value;
      // blocks j = 0, 1 (columns 0-15, 16-31 of the strip): lane has columns 4*g4 + r of each;
      // one swap of rows 1,3 of X with rows 0,2 of Y gives 8 consecutive columns
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // (no __builtin_bit_cast of a vector-element expression: ROCm 7.2's clang folds
        // bit_cast(acc[r]) to element 0 for every r)
        const float x = acc[qm][qn][i][0][r], y = acc[qm][qn][i][1][r];
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
        const unsigned sx = sw[0], sy = sw[1];
        v[r] = __uint_as_float(sx) + bias[qn][0][r];
        v[4 + r] = __uint_as_float(sy) + bias[qn][1][r];
      }
      const SideSeg<OutT>& sd = side[qm][qn][i];
      if constexpr (SK == SIDE_C) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = fmaf(e.beta, sd.get(k), v[k]);
      }
      float pre[8];
      if constexpr (SK == SIDE_AUX) {  // backward activation: aux holds act'(pre) (CAPK_ACT_DERIV)
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= sd.get(k);
      } else if constexpr (ACT != 0) {
        constexpr bool PK = std::is_same<OutT, bf16>::value &&
                            (ACT == CAPK_ACT_GELU_ERF || ACT == CAPK_ACT_GELU_TANH || ACT == CAPK_ACT_QUICK_GELU);
        if constexpr (PK) {  // packed fp32 pairs (common.h act_*_fast2)
#pragma unroll
          for (int k = 0; k < 8; k += 2) {
            const f32x2 x = {v[k], v[k + 1]};
            f32x2 y, d;
            if constexpr (DV) y = act_fwd_grad_fast2(ACT, x, d);
            else {
              d = x;
              y = act_fwd_fast2(ACT, x);
            }
            v[k] = y[0]; v[k + 1] = y[1];
            pre[k] = d[0]; pre[k + 1] = d[1];
          }
        } else if constexpr (DV) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = act_fwd_grad_fast<OutT>(ACT, v[k], pre[k]);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            pre[k] = v[k];
            v[k] = act_fwd_fast<OutT>(ACT, v[k]);
          }
        }
      }
      if constexpr (SK == SIDE_RES) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += sd.get(k);
      }
      if constexpr (DSUM) {  // rows past M hold bias / zero-operand values: not summed
        const bool row_ok = c.m0 + qm * 128 + i * 16 + lrow < M;
#pragma unroll
        for (int k = 0; k < 8; ++k) cs[qn][k] += row_ok ? v[k] : 0.f;
      }
      if constexpr (LSEP) {
        const int n = c.n0 + qn * 128 + lcol;
        float t[8], mx = lm[i];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          t[k] = n + k < e.lse_v ? (float)(bf16)v[k] * kLog2eG : -INFINITY;
          mx = fmaxf(mx, t[k]);
        }
        if (mx != -INFINITY) {  // (a lane whose columns are all padding keeps (-inf, 0))
          float sm = ls[i] * fexp2s(lm[i] - mx);
#pragma unroll
          for (int k = 0; k < 8; ++k) sm += fexp2s(t[k] - mx);
          lm[i] = mx;
          ls[i] = sm;
        }
      }
#if defined(CAPK_DIAG_NOSTORE)  // diagnostic build: the stores issue but are dropped (range check)
      store8(rsC, OOR, v, (OutT*)nullptr);
#else
      store8(rsC, (qn ? o1 : o0) + seg_add(e.ldc, ESZ, qm, i), v, (OutT*)nullptr);
#endif
      if constexpr (ACT != 0) {
        const __amdgpu_buffer_rsrc_t rsPre = rsrc_of(e.pre, (int64_t)M * e.ldp * ESZ);
        store8(rsPre, (qn ? p1 : p0) + seg_add(e.ldp, ESZ, qm, i), pre, (OutT*)nullptr);
      }
    };
#define CAPK_SEG(QN, I) \
  segment(qmc, std::integral_constant<int, QN>{}, std::integral_constant<int, I>{});
    CAPK_SEG(0, 0) CAPK_SEG(0, 1) CAPK_SEG(0, 2) CAPK_SEG(0, 3)
    CAPK_SEG(1, 0) CAPK_SEG(1, 1) CAPK_SEG(1, 2) CAPK_SEG(1, 3)
#undef CAPK_SEG
    // memory instructions issued after the last wait (the stores): per segment one (bf16) or
    // two (fp32) for C, the same again for the pre-activation (dropped when not kept)
    constexpr int per = ESZ == 2 ? 1 : 2;
    int nst = 8 * per * (ACT != 0 ? 2 : 1);
    if constexpr (LSEP) {
      // the lane's rows (i) now hold (max, sum exp) over its 16 columns; merge the four column
      // groups of the wave (lanes l ^ 16, l ^ 32), then lanes 0-15 store the wave's partial for
      // its 64 columns: part[(tn * 4 + wn) * M + row]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int x = 16; x <= 32; x <<= 1) {
          const float mo = __shfl_xor(lm[i], x, 64), so = __shfl_xor(ls[i], x, 64);
          const float mn = fmaxf(lm[i], mo);
          ls[i] = mn == -INFINITY ? 0.f : ls[i] * fexp2s(lm[i] - mn) + so * fexp2s(mo - mn);
          lm[i] = mn;
        }
        const int row = c.m0 + QM * 128 + wm * 64 + i * 16 + (lane & 15);
        const int64_t pidx = (int64_t)((c.n0 >> 8) * 4 + wn) * M + row;
        const uint32_t off = (lane < 16 && row < M) ? (uint32_t)(pidx * 8) : OOR;
        const __amdgpu_buffer_rsrc_t rsP = rsrc_of(e.lse_part, (int64_t)((N + 255) / 256) * 4 * M * 8);
        __builtin_amdgcn_raw_buffer_store_b64(
            (__attribute__((ext_vector_type(2))) unsigned){__float_as_uint(lm[i]), __float_as_uint(ls[i])}, rsP, off, 0, 0);
      }
      nst += 4;
    }
    return nst;
  };
  // The item's epilogue, one quadrant row (half) at a time; a side operand (residual / aux /
  // C) is loaded per half, 8 segments in flight, one wait (the first also retires the next
  // item's operand loads issued before it, the second the first half's stores).  Returns the
  // memory instructions it leaves in flight (the second half's stores, + the first's without
  // a side operand).
  auto epilogue = [&](const Item& c, int j) -> int {
#if defined(CAPK_DIAG_NOEPI)  // diagnostic build: no epilogue at all (accumulators kept live)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) asm volatile("" ::"v"(acc[a][b][i][jj]));
    return 0;
#endif
    // Both halves' side segments are requested at once (the A / B fragment registers of the
    // main loop are dead here): the second half's loads fly while the first half computes, so
    // an item pays one side-operand round trip, not two.  Waits: vmcnt <= 8 leaves exactly
    // the second half's 8 loads (the first) / the first half's 8 stores (the second) younger.
    SideSeg<OutT> side[2][2][4];
    auto issue_side = [&](auto qmc) {
      constexpr int QM = decltype(qmc)::value;
      if constexpr (SIDE && ESZ == 2) {
        const __amdgpu_buffer_rsrc_t rsSide = rsrc_of(e.side, (int64_t)M * e.lds * ESZ);
        const uint32_t s0 = this_lane_off(c, e.lds, ESZ, 0), s1 = this_lane_off(c, e.lds, ESZ, 1);
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int i = 0; i < 4; ++i) side[QM][qn][i].load(rsSide, (qn ? s1 : s0) + seg_add(e.lds, ESZ, QM, i));
      }
    };
    auto wait_side = [&](auto qmc) {
      constexpr int QM = decltype(qmc)::value;
      if constexpr (SIDE && ESZ == 2) {
        asm volatile("s_waitcnt vmcnt(8)"
                     : "+v"(side[QM][0][0].a), "+v"(side[QM][0][1].a), "+v"(side[QM][0][2].a), "+v"(side[QM][0][3].a),
                       "+v"(side[QM][1][0].a), "+v"(side[QM][1][1].a), "+v"(side[QM][1][2].a), "+v"(side[QM][1][3].a)
                     :
                     : "memory");
        fence();
      }
    };
    using QA = std::integral_constant<int, 0>;
    using QB = std::integral_constant<int, 1>;
    float cs[2][8];
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int k = 0; k < 8; ++k) cs[qn][k] = 0.f;
    issue_side(QA{});
    issue_side(QB{});
    wait_side(QA{});
    const int n0 = epi_body(c, j, side, cs, QA{});
    wait_side(QB{});
    const int n1 = epi_body(c, j, side, cs, QB{});
    int nd = 0;
    if constexpr (DSUM) {
      // the lane's 8 columns summed over its 8 rows; now over the 16 lanes of its column
      // group (lane & 15 = row), then one 8-column partial per (tile row, wm) and quadrant
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float x = cs[qn][k];
          x += __shfl_xor(x, 1, 16);
          x += __shfl_xor(x, 2, 16);
          x += __shfl_xor(x, 4, 16);
          x += __shfl_xor(x, 8, 16);
          cs[qn][k] = x;
        }
      const __amdgpu_buffer_rsrc_t rsD = rsrc_of(e.dsum, (int64_t)((M + 255) / 256) * 2 * N * 4);
      const int64_t prow = (int64_t)(c.m0 / 256) * 2 + wm;
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
        const int n = c.n0 + qn * 128 + lcol;
        const uint32_t off = ((lane & 15) == 0 && n < N) ? (uint32_t)((prow * N + n) * 4) : OOR;
        store8(rsD, off, cs[qn], (float*)nullptr);
      }
      nd = 4;  // two 16-B stores per quadrant column
    }
    return n0 + n1 + nd;
  };

  // ---- TAIL: this WG's K-split part of a tail tile -> fp32 slab tsplit (no bias / epilogue:
  // the reduce applies them once); rows past M and columns past N are not written (a row past
  // the slab's rows would land in the next split's slab).  Returns the stores left in flight.
  auto tail_store = [&](const Item& c) -> int {
    const int64_t Mt = (int64_t)M - (int64_t)e.tail_r0 * 256;
    const __amdgpu_buffer_rsrc_t rsW = rsrc_of(e.tail_ws + (size_t)tsplit * Mt * N, Mt * N * 4);
    auto seg = [&](auto qmc, auto qnc, auto ic) {
      constexpr int qm = decltype(qmc)::value, qn = decltype(qnc)::value, i = decltype(ic)::value;
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = acc[qm][qn][i][0][r], y = acc[qm][qn][i][1][r];
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
        v[r] = __uint_as_float(sw[0]);
        v[4 + r] = __uint_as_float(sw[1]);
      }
      const int64_t row = (int64_t)c.m0 - (int64_t)e.tail_r0 * 256 + qm * 128 + i * 16 + lrow;
      const int n = c.n0 + qn * 128 + lcol;
      const uint32_t off = row < Mt && n < N ? (uint32_t)((row * N + n) * 4) : OOR;
      store8(rsW, off, v, (float*)nullptr);
    };
#define CAPK_TSEG(QM, QN, I) \
  seg(std::integral_constant<int, QM>{}, std::integral_constant<int, QN>{}, std::integral_constant<int, I>{});
    CAPK_TSEG(0, 0, 0) CAPK_TSEG(0, 0, 1) CAPK_TSEG(0, 0, 2) CAPK_TSEG(0, 0, 3)
    CAPK_TSEG(0, 1, 0) CAPK_TSEG(0, 1, 1) CAPK_TSEG(0, 1, 2) CAPK_TSEG(0, 1, 3)
    CAPK_TSEG(1, 0, 0) CAPK_TSEG(1, 0, 1) CAPK_TSEG(1, 0, 2) CAPK_TSEG(1, 0, 3)
    CAPK_TSEG(1, 1, 0) CAPK_TSEG(1, 1, 1) CAPK_TSEG(1, 1, 2) CAPK_TSEG(1, 1, 3)
#undef CAPK_TSEG
    return 32;  // two 16-B stores per segment
  };

  // ---- main loop: gemm8p's two phases per K-tile over the continuous step sequence ----
  //   phase  quadrants          ds_read (L)           LDS-DMA issued (L)              wait (L)
  //   Q1     (0,0) (0,1)        A0(u) B0(u) B1(u)     A1(u+1)                         A1(u)
  //   Q2     (1,1) (1,0)        A1(u)                 A0 B0 B1 (+bias) (u+2)          A0 B0 B1 (+bias) (u+1)
  // Step u is K-tile k of item j (u = j nk + k); steps u+1, u+2 lie in item j or j+1 (nk >= 2).
  // Wait counts: Q1(u) leaves Q2(u-1)'s loads (6, +1 with a bias DMA) younger, Q2(u) leaves
  // Q1(u)'s 2; both + S when the epilogue of item j-1 ran since the awaited issue (k == 0).
  // TAIL: the last segment starts at K-tile cur.k0 and ends at cur.k1 (>= 4 K-tiles: host)
  Item cur = item_at(0), nxt = item_at(nseg > 1 ? 1 : 0);
  int j = 0, k = TAIL ? cur.k0 : 0;
  zero_acc();
  bf16x8 fa[2][4], fb0[2][2], fb1[2][2];
  // prologue: A0 B0 B1 (+bias) of step 0, A1 of step 0, A0 B0 B1 of step 1
  load(0, cur, k, 0);
  load(2, cur, k, 0);
  load(3, cur, k, 0);
  if (has_bias) bias_dma(cur, 0);
  load(1, cur, k, 0);
  load(0, cur, k + 1, 1);
  load(2, cur, k + 1, 1);
  load(3, cur, k + 1, 1);
  wait_vmc<8>();  // A0 B0 B1 (+bias) of step 0: A1(0) and step 1's three halves younger
  bar();
  if (lag) bar();  // waves 4-7 fall one barrier behind
  int S = 0;        // stores left in flight by the last epilogue (k == 0 phases only)
  int q2prev = 6;   // loads issued by the previous Q2 (prologue: step 1's three halves)

  for (int u = 0;; ++u) {
    const bool has1 = u + 1 < total, has2 = u + 2 < total;
    // Q1: (0,0), (0,1).  L: read A0, B0, B1 (u); wait A1 (u); issue A1 (u+1)
    readA(fa, u, 0);
    readB(fb0, u, 2);
    readB(fb1, u, 3);
    const int kend = TAIL ? cur.k1 : nk, kbn = TAIL ? nxt.k0 : 0;  // this segment's end, the next's start
    const int k0c = TAIL ? cur.k0 : 0;
    const int e1 = k == k0c ? S : 0;
    {
      const int n1 = q2prev + e1;  // steady state: 6, +1 with a bias DMA in that phase
      if (n1 == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else if (n1 == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else wait_le(n1);
    }
    if (k == k0c) stamp(j, 2);
    const Item& t1 = k + 1 < kend ? cur : nxt;
    const int k1n = k + 1 < kend ? k + 1 : kbn;
    if (has1) load(1, t1, k1n, u + 1);
    lds_done();
    bar();
    if (k == k0c) stamp(j, 3);
    prio_mfma();
    mma(fa, fb0, acc[0][0]);
    mma(fa, fb1, acc[0][1]);
    prio_load();
    bar();
    // Q2: (1,1), (1,0).  L: read A1 (u); wait A0 B0 B1 (+bias) (u+1); issue A0 B0 B1 (+bias) (u+2)
    readA(fa, u, 1);
    const int q1n = has1 ? 2 : 0;
    if (q1n + e1 == 2) wait_vmc<2>();
    else wait_le(q1n + e1);
    q2prev = 0;
    const bool same2 = k + 2 < kend;
    const int k2 = same2 ? k + 2 : kbn + (k + 2 - kend);
    const Item& t2 = same2 ? cur : nxt;
    if (has2) {
      load(0, t2, k2, u + 2);
      load(2, t2, k2, u + 2);
      load(3, t2, k2, u + 2);
      q2prev = 6;
      if ((TAIL ? !same2 && k + 2 == kend : k2 == 0) && has_bias) {  // the next segment's first K-tile
        bias_dma(t2, j + 1);
        q2prev = 7;
      }
    }
    lds_done();
    bar();
    prio_mfma();
    mma(fa, fb1, acc[1][1]);
    mma(fa, fb0, acc[1][0]);
    prio_load();
    bar();
    if (++k == kend) {  // the segment's last K-tile: epilogue, stores left in flight
      stamp(j, 0);
      fence();
      {
        S = (TAIL && hasTail && j == nseg - 1) ? tail_store(cur) : epilogue(cur, j);
        zero_acc();
        fence();
        stamp(j, 1);
        if (++j == nseg) break;
      }
      cur = nxt;
      k = TAIL ? cur.k0 : 0;
      nxt = item_at(j + 1 < nseg ? j + 1 : j);
    }
  }
  if (!lag) bar();  // realign the two groups (every barrier is matched)
  if constexpr (TAIL && TCOMB) {
    // ---- in-launch split-K combine of the tail tile (e.tail_cnt): every part has stored its
    // slab (tail_store); the part drawing the tile's last ticket sums the slabs in split order
    // (0 + s0 + s1 + ..., splitk_reduce_kernel's order: the same bits) and runs the item's
    // register epilogue.  Publish: every wave drains its slab stores, the barrier, then ONE
    // agent-scope release before the ticket; the reducer takes ONE agent-scope acquire before
    // its plain slab loads (correct for any placement of a tile's parts over the XCDs).
    if (hasTail && e.tail_cnt != nullptr) {
      int* const last_flag = (int*)(smem + BIAS0 + 2 * 8 * 256);  // the 16 spare bytes of smem
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gu32* const cnt = (gu32*)(e.tail_cnt + ttile);  // a global (never flat) agent-scope word
        const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == (unsigned)(TS - 1);
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        *last_flag = last;
      }
      __syncthreads();
      if (*last_flag == 0) return;
      // the slabs, summed segment by segment in tail_store's (swapped) layout into acc, then
      // swapped back (the swap is an involution) for the epilogue
      const int64_t Mt = (int64_t)M - (int64_t)e.tail_r0 * 256;
      zero_acc();
      // one quadrant row at a time (16 segments of 2 loads in flight, no spills)
      auto combine = [&](auto qmc) {
        constexpr int qm = decltype(qmc)::value;
        uint32_t off[2][4];
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int64_t row = (int64_t)cur.m0 - (int64_t)e.tail_r0 * 256 + qm * 128 + i * 16 + lrow;
            const int n = cur.n0 + qn * 128 + lcol;
            off[qn][i] = row < Mt && n < N ? (uint32_t)((row * N + n) * 4) : OOR;
          }
        for (int s = 0; s < TS; ++s) {
          const __amdgpu_buffer_rsrc_t rsW = rsrc_of(e.tail_ws + (size_t)s * Mt * N, Mt * N * 4);
#pragma unroll
          for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const i32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rsW, off[qn][i], 0, 0);
              const i32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rsW, off[qn][i] + 16, 0, 0);
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                acc[qm][qn][i][0][r] += __int_as_float(a[r]);
                acc[qm][qn][i][1][r] += __int_as_float(b[r]);
              }
            }
        }
      };
      combine(std::integral_constant<int, 0>{});
      combine(std::integral_constant<int, 1>{});
#pragma unroll
      for (int qm = 0; qm < 2; ++qm)
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[qm][qn][i][0][r]),
                                                               __float_as_uint(acc[qm][qn][i][1][r]), false, false);
              acc[qm][qn][i][0][r] = __uint_as_float(sw[0]);
              acc[qm][qn][i][1][r] = __uint_as_float(sw[1]);
            }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      fence();
      epilogue(cur, nseg - 1);
    }
  }
#if defined(CAPK_DIAG_TRACE)
  if ((wave & 3) == 0 && e.trace) {  // this wave's stamps -> e.trace [blockIdx][group][item][4]
    unsigned long long* dst = e.trace + ((size_t)blockIdx.x * 2 + (wave >> 2)) * TR_ITEMS * 4;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int x = lane; x < TR_ITEMS * 4; x += 64) dst[x] = trs[(wave >> 2) * TR_ITEMS * 4 + x];
  }
#endif
}

}  // namespace

bool gemm8q_supports(const Epi& e, bool out_f32) {
  const int sides = ((e.act & CAPK_ACT_BWD) ? 1 : 0) + (e.res ? 1 : 0) + (e.beta != 0.f ? 1 : 0);
  const int a = e.act & 15;
  const bool fwd_act = a && !(e.act & CAPK_ACT_BWD);
  if (e.alpha != 1.0f || e.drop.thr != 0) return false;  // (dropout: gemm8p)
  if (fwd_act && a != CAPK_ACT_GELU_ERF && a != CAPK_ACT_GELU_TANH && a != CAPK_ACT_QUICK_GELU && a != CAPK_ACT_RELU)
    return false;  // (tanh / sigmoid epilogues: pooler-sized products, the 8p kernel)
  if (fwd_act && (sides || out_f32)) return false;
  // backward activations only in the multiply-by-aux form (CAPK_ACT_DERIV: aux = act'(pre));
  // fp32 outputs take no side operand (16 segments of 8 fp32 would need 128 VGPRs)
  return sides <= (out_f32 ? 0 : 1) && (!(e.act & CAPK_ACT_BWD) || (e.act & CAPK_ACT_DERIV));
}


#if defined(CAPK_DIAG_TRACE)
static size_t diag_trace_bytes() { return (size_t)256 * 2 * 64 * 4 * 8; }
static void* diag_trace_buf() {
  static void* buf = nullptr;
  if (!buf && hipMalloc(&buf, diag_trace_bytes()) != hipSuccess) buf = nullptr;
  return buf;
}
#endif

// The split-K tail round: after the whole rounds, the row blocks [r0, ntm) as S K-splits per
// tile in one more round (T tail tiles, T * S <= 256).  It pays when the tail round is long
// enough that cutting it to 1/S plus the reduce launch (~12 us for the ViT shapes) wins: K >=
// 1536 (24 K-tiles), S >= 2, each split >= 8 K-tiles.  capk_gemm_set_tail / CAPK_GEMM_TAIL=0
// turn it off (A/B).
static int g_tail_mode = -1;
static int tail_mode() {
  static const int env_mode = [] {
    const char* v = getenv("CAPK_GEMM_TAIL");
    return v ? atoi(v) : 1;
  }();
  return g_tail_mode >= 0 ? g_tail_mode : env_mode;
}
bool gemm8q_tail_plan(int M, int N, int K, int* r0, int* splits) {
  const int mode = tail_mode();
  const int ntm = cdiv(M, 256), ntn = cdiv(N, 256), items = ntm * ntn, nk = cdiv(K, 64);
  const int rounds = items >> 8;
  if (mode == 0 || rounds < 1 || (items & 255) == 0 || nk < 24) return false;
  const int rr0 = (rounds * 256) / ntn, T = (ntm - rr0) * ntn;
  if (rr0 < 1 || T <= 0) return false;
  const int S = std::min(256 / T, nk / 8);
  if (S < 2) return false;
  *r0 = rr0;
  *splits = S;
  return true;
}
// Arrival tickets of the in-launch tail combine: a pool of zeroed 256-int blocks per device,
// allocated on the first tail launch outside a stream capture; each (device, stream) takes its
// own block on first use (no allocation then, so a stream being captured can take one too).
// Every launch leaves its tickets at zero (the last arriver of each tile resets its own), so
// launches on one stream -- graph replays included -- reuse the block, and concurrent streams
// never share one.  No block (first use inside a capture, pool exhausted): the launch reduces
// with the separate kernel instead.
static int* tail_tickets(hipStream_t st) {
  constexpr int kBlocks = 64, kInts = 256;
  static std::mutex mu;
  static std::map<int, int*> pools;
  static std::map<std::pair<int, hipStream_t>, int*> taken;
  static std::map<int, int> used;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_pair(dev, st);
  auto it = taken.find(key);
  if (it != taken.end()) return it->second;
  auto pit = pools.find(dev);
  if (pit == pools.end()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    int* p = nullptr;
    if (hipMalloc(&p, (size_t)kBlocks * kInts * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, (size_t)kBlocks * kInts * sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    pit = pools.emplace(dev, p).first;
  }
  int& n = used[dev];
  if (n >= kBlocks) return nullptr;
  int* b = pit->second + (size_t)(n++) * kInts;
  taken[key] = b;
  return b;
}

size_t gemm8q_tail_workspace(int M, int N, int K) {
  int r0, S;
  if (!gemm8q_tail_plan(M, N, K, &r0, &S)) return 0;
  return (size_t)S * (size_t)(M - r0 * 256) * N * sizeof(float);
}

// Grouped raster (Epi8q::group).  WG b runs items (b & 7) * 32 + (b >> 3) + 256 j, so the 32
// WGs of one XCD work on 32 consecutive items at a time, and the operand blocks they read
// (one 256-row A block per tile row, one 256-column B block per tile column, each
// 256 x K bf16) come through that XCD's 4 MiB L2: with the 32 WGs in near lockstep, a
// (block, K-tile) misses once per chunk, so the L2 miss share of the LDS-DMA stream is about
// distinct blocks / 64.  Row-major order makes a 32-item chunk of a wide product touch 1-3 row
// blocks and up to 32 column blocks (the LM head: 2 + 32; FC1: 3 + 12, QKV 4 + 9); groups of
// g row blocks walked column-major make it g rows x 32/g columns.  Measured in one process
// (tools/gemm_ab.py, profiles/round5/raster_ab.txt): g = 8 on the ViT's wide products (QKV
// 168.7 -> 163.8 us, FC1 + GELU + act' 309.9 -> 300.4, FC2 dX x act' 287.0 -> 277.9), g = 4 on
// the 20-row LM head (409.9 -> 371.8), row-major on the N = 768 products (3 column blocks:
// already 11 rows + 3 columns per chunk; grouping measured neutral to -1 %).
static int g_group_mode = -2;
int gemm8q_group(int ntm, int ntn) {
  static const int env_mode = [] {
    const char* v = getenv("CAPK_GEMM_GROUP");
    return v ? atoi(v) : -1;
  }();
  const int mode = g_group_mode >= -1 ? g_group_mode : env_mode;
  if (mode >= 0) return mode;
  if (ntn <= 4 || ntm < 8) return 0;
  return ntm <= 32 ? 4 : 8;
}

int launch_gemm8q(bool a_kmajor, bool b_kmajor, bool out_f32, const void* A, int64_t lda, const void* B, int64_t ldb,
                  int M, int N, int K, int splits, const Epi& e, float* slab, hipStream_t st, float* dsum,
                  void* ws, size_t ws_bytes, int* tail_r0, int* tail_splits, float* lse_part, int lse_v) {
  CAPK_CHECK_ARG((a_kmajor ? (int64_t)M * lda : (int64_t)K * lda) * 2 < (1ll << 31) &&
                     (b_kmajor ? (int64_t)N * ldb : (int64_t)K * ldb) * 2 < (1ll << 31),
                 "capk_gemm(bf16, 256x256): operand larger than 2 GiB");
  CAPK_CHECK_ARG(gemm8q_supports(e, out_f32) && splits == 1 && !slab, "capk_gemm(gemm8q): unsupported epilogue");
  const int64_t esz = out_f32 ? 4 : 2;
  Epi8q p{};
  p.C = e.C;
  p.ldc = e.ldc;
  p.beta = e.beta;
  p.bias = e.bias;
  const int a = e.act & 15;
  const bool fwd_act = a && !(e.act & CAPK_ACT_BWD);
  const bool dv = fwd_act && (e.act & CAPK_ACT_DERIV);
  if (fwd_act) {
    p.pre = e.pre;
    p.ldp = e.ldx;
  }
  int sk = SIDE_NONE;
  if (e.act & CAPK_ACT_BWD) {
    sk = SIDE_AUX;
    p.side = e.aux;
    p.lds = e.ldx;
  } else if (e.res) {
    sk = SIDE_RES;
    p.side = e.res;
    p.lds = e.ldr;
  } else if (e.beta != 0.f) {
    sk = SIDE_C;
    p.side = e.C;
    p.lds = e.ldc;
  }
  CAPK_CHECK_ARG((int64_t)M * e.ldc * esz < (1ll << 31) && (!p.pre || (int64_t)M * p.ldp * esz < (1ll << 31)) &&
                     (!p.side || (int64_t)M * p.lds * esz < (1ll << 31)),
                 "capk_gemm(bf16, 256x256): output or side operand larger than 2 GiB");
  const int items = cdiv(M, 256) * cdiv(N, 256);
  CAPK_CHECK_ARG(items > 256, "capk_gemm(gemm8q): persistent kernel for grids of more than 256 items");
  // the split-K tail round (not the DSUM form): the caller reduces the slabs
  if (tail_r0) *tail_r0 = -1;
  {
    int r0, S;
    if (tail_r0 && ws && !dsum && !lse_part && gemm8q_tail_plan(M, N, K, &r0, &S) &&
        ws_bytes >= (size_t)S * (size_t)(M - r0 * 256) * N * sizeof(float)) {
      p.tail_ws = (float*)ws;
      p.tail_r0 = r0;
      p.tail_splits = S;
      // mode 2: the parts combine in the launch (tickets), else the caller's reduce launch
      p.tail_cnt = tail_mode() == 2 ? tail_tickets(st) : nullptr;
      *tail_r0 = p.tail_cnt ? -1 : r0;
      *tail_splits = S;
    }
  }
  CAPK_CHECK_ARG(!fwd_act || (a_kmajor && b_kmajor), "capk_gemm(gemm8q): forward activations need K-major operands");
  // grouped raster over the whole-item rows (all rows, or [0, r0) with a tail round)
  p.group = gemm8q_group(p.tail_ws ? p.tail_r0 : cdiv(M, 256), cdiv(N, 256));
#if defined(CAPK_DIAG_TRACE)
  p.trace = (unsigned long long*)diag_trace_buf();
  CAPK_CHECK_ARG(p.trace != nullptr, "capk_gemm(gemm8q, trace build): no trace buffer");
  hipMemsetAsync(p.trace, 0, diag_trace_bytes(), st);
#endif
  const dim3 grid(256), block(512);
#define L8(AK, BKM, OT, ACTK, DVK, SKK, DS)                                                                        \
  do {                                                                                                          \
    constexpr bool TAILV = !DS;                                                                                 \
    if (TAILV && p.tail_ws && p.tail_cnt)                                                                       \
      hipLaunchKernelGGL((gemm8q_kernel<AK, BKM, OT, ACTK, DVK, SKK, DS, TAILV, false, true>), grid, block, 0, st, \
                         A, lda, B, ldb, M, N, K, 1, p);                                                        \
    else if (TAILV && p.tail_ws)                                                                                \
      hipLaunchKernelGGL((gemm8q_kernel<AK, BKM, OT, ACTK, DVK, SKK, DS, TAILV>), grid, block, 0, st, A, lda, B, \
                         ldb, M, N, K, 1, p);                                                                   \
    else                                                                                                        \
      hipLaunchKernelGGL((gemm8q_kernel<AK, BKM, OT, ACTK, DVK, SKK, DS, false>), grid, block, 0, st, A, lda, B, \
                         ldb, M, N, K, 1, p);                                                                   \
  } while (0)
#define L8SK(AK, BKM)                                      \
  switch (sk) {                                            \
    case SIDE_AUX: L8(AK, BKM, bf16, 0, false, SIDE_AUX, false); break; \
    case SIDE_RES: L8(AK, BKM, bf16, 0, false, SIDE_RES, false); break; \
    case SIDE_C: L8(AK, BKM, bf16, 0, false, SIDE_C, false); break;     \
    default: L8(AK, BKM, bf16, 0, false, SIDE_NONE, false); break;      \
  }
#define L8ACT(ACTK)                                        \
  if (dv) L8(true, true, bf16, ACTK, true, SIDE_NONE, false); \
  else L8(true, true, bf16, ACTK, false, SIDE_NONE, false);
  if (lse_part) {  // the LM head with the shifted CE's softmax partials (capk_linear_lse)
    CAPK_CHECK_ARG(a_kmajor && b_kmajor && !out_f32 && sk == SIDE_NONE && !fwd_act && !dsum,
                   "capk_gemm(gemm8q): softmax partials only on a plain K-major bf16 product");
    p.lse_part = lse_part;
    p.lse_v = lse_v;
    hipLaunchKernelGGL((gemm8q_kernel<true, true, bf16, 0, false, SIDE_NONE, false, false, true>), grid, block, 0, st,
                       A, lda, B, ldb, M, N, K, 1, p);
  } else if (dsum) {  // dX with the backward-activation multiply + column sums (capk_gemm_dx_act_colsum)
    CAPK_CHECK_ARG(a_kmajor && !out_f32 && sk == SIDE_AUX,
                   "capk_gemm(gemm8q): column sums only on the dX x act' product");
    p.dsum = dsum;
    if (b_kmajor) L8(true, true, bf16, 0, false, SIDE_AUX, true);  // (the weight's K-major copy)
    else L8(true, false, bf16, 0, false, SIDE_AUX, true);
  } else if (out_f32) {  // fp32 outputs: no activation, no side operand (gemm8q_supports)
    if (a_kmajor && b_kmajor) L8(true, true, float, 0, false, SIDE_NONE, false);
    else if (a_kmajor) L8(true, false, float, 0, false, SIDE_NONE, false);
    else if (b_kmajor) L8(false, true, float, 0, false, SIDE_NONE, false);
    else L8(false, false, float, 0, false, SIDE_NONE, false);
  } else if (fwd_act) {
    switch (a) {
      case CAPK_ACT_GELU_ERF: L8ACT(CAPK_ACT_GELU_ERF) break;
      case CAPK_ACT_GELU_TANH: L8ACT(CAPK_ACT_GELU_TANH) break;
      case CAPK_ACT_QUICK_GELU: L8ACT(CAPK_ACT_QUICK_GELU) break;
      default: L8ACT(CAPK_ACT_RELU) break;
    }
  } else if (a_kmajor && b_kmajor) {
    L8SK(true, true)
  } else if (a_kmajor) {
    L8SK(true, false)
  } else if (b_kmajor) {
    L8SK(false, true)
  } else {
    L8SK(false, false)
  }
#undef L8ACT
#undef L8SK
#undef L8
  CAPK_LAUNCH_CHECK("gemm8q_kernel");
  return CAPK_OK;
}

}  // namespace capk

#if defined(CAPK_DIAG_TRACE)
// diagnostic build only: the last gemm8q launch's timestamps (s_memrealtime, 100 MHz) as
// uint64 [256 WGs][2 wave groups][64 items][4 stamps] (see stamp() in the kernel)
extern "C" int capk_gemm_diag_trace(void* host_dst, size_t bytes) {
  void* b = capk::diag_trace_buf();
  if (!b || bytes < capk::diag_trace_bytes()) return CAPK_EINVAL;
  return hipMemcpy(host_dst, b, capk::diag_trace_bytes(), hipMemcpyDeviceToHost) == hipSuccess ? CAPK_OK : CAPK_EINVAL;
}
#endif

extern "C" int capk_gemm_set_group(int rows) {
  CAPK_CHECK_ARG(rows >= -2 && rows <= 64, "capk_gemm_set_group: rows must be -2 (environment), -1 (auto) or 0..64");
  capk::g_group_mode = rows;
  return CAPK_OK;
}

extern "C" int capk_gemm_set_tail(int mode) {
  CAPK_CHECK_ARG(mode >= -1 && mode <= 2, "capk_gemm_set_tail: mode must be -1 (environment), 0, 1 or 2");
  capk::g_tail_mode = mode;
  return CAPK_OK;
}
