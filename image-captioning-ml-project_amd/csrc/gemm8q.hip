// Persistent 256x256 bf16 GEMM with a register-direct epilogue (round 3) — the large-grid
// kernel of capk_gemm.  Same tile, waves, LDS images and phased main loop as gemm8p.hip;
// what changes is everything around the main loop:
//
//  * Persistent grid: min(tiles x splits, 256) workgroups, one per CU; WG b takes items
//    j*256 + (b & 7)*32 + (b >> 3) (j = 0, 1, ...) -- every XCD works on 32 consecutive items
//    of the row-major tile order at a time, so an XCD's L2 holds the A rows and B columns
//    they share.
//  * One continuous K-tile pipeline over ALL of the WG's items: the loads of item j+1's first
//    two K-tiles are issued during item j's last two K-tiles (exactly where the steady-state
//    schedule issues them), so no item pays a prologue; only the WG's first item does.
//  * Register-direct epilogue: no LDS staging.  The MFMAs run with the operands swapped
//    (B fragment first), so a lane's accumulator holds 4 consecutive columns of one row;
//    one v_permlane16_swap per register pair turns the two 16-column blocks of a 32-column
//    strip into 8 consecutive columns per lane, stored as one 16-byte buffer store (each
//    store instruction writes 16 rows x 64 contiguous bytes).  Bias comes from a 1-KiB LDS
//    slot filled by LDS-DMA when the item's first K-tile is loaded; the side operand
//    (residual / aux / C) by 16 buffer loads.  Out-of-range rows and columns go through the
//    buffer descriptors' range checks (no branches: every wave issues the same number of
//    memory instructions, which the vmcnt ledger below relies on).
//  * The epilogue's stores are NOT waited for: they drain while the next item's first K-tile
//    computes (its operands were loaded before the stores were issued).  vmcnt counts loads,
//    LDS-DMA and stores together in issue order, so every wait is computed at run time from a
//    per-wave ledger of issued memory instructions (`ops` and the issue marks of each group)
//    instead of the fixed counts of gemm8p.
//
// Epilogue: alpha, bias, forward activation (+ pre-activation or act' side output), backward
// activation (x act'(aux) or x aux), dropout, residual, beta*C -- with at most ONE of
// aux / residual / C (gemm8q_supports); split-K items write fp32 slabs that
// splitk_reduce_kernel finishes.
#include <type_traits>

#include "gemm_common.h"

namespace capk {

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));

// s_waitcnt vmcnt(n) for a run-time, wave-uniform n (clamped to the field's 63)
__device__ __forceinline__ void vm_wait_switch(int n);
__device__ __forceinline__ void vm_wait(int n) {
#if defined(CAPK_DIAG_VM0)  // diagnostic build: drain every wait
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return;
#endif
  // the steady-state counts inline; the rest (the two phases after an epilogue, the tail)
  // through the full switch
  if (n == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else vm_wait_switch(n);
}
__device__ __forceinline__ void vm_wait_switch(int n) {
  n = n > 63 ? 63 : n;
  switch (n) {
#define CAPK_VMW(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    CAPK_VMW(0) CAPK_VMW(1) CAPK_VMW(2) CAPK_VMW(3) CAPK_VMW(4) CAPK_VMW(5) CAPK_VMW(6) CAPK_VMW(7)
    CAPK_VMW(8) CAPK_VMW(9) CAPK_VMW(10) CAPK_VMW(11) CAPK_VMW(12) CAPK_VMW(13) CAPK_VMW(14) CAPK_VMW(15)
    CAPK_VMW(16) CAPK_VMW(17) CAPK_VMW(18) CAPK_VMW(19) CAPK_VMW(20) CAPK_VMW(21) CAPK_VMW(22) CAPK_VMW(23)
    CAPK_VMW(24) CAPK_VMW(25) CAPK_VMW(26) CAPK_VMW(27) CAPK_VMW(28) CAPK_VMW(29) CAPK_VMW(30) CAPK_VMW(31)
    CAPK_VMW(32) CAPK_VMW(33) CAPK_VMW(34) CAPK_VMW(35) CAPK_VMW(36) CAPK_VMW(37) CAPK_VMW(38) CAPK_VMW(39)
    CAPK_VMW(40) CAPK_VMW(41) CAPK_VMW(42) CAPK_VMW(43) CAPK_VMW(44) CAPK_VMW(45) CAPK_VMW(46) CAPK_VMW(47)
    CAPK_VMW(48) CAPK_VMW(49) CAPK_VMW(50) CAPK_VMW(51) CAPK_VMW(52) CAPK_VMW(53) CAPK_VMW(54) CAPK_VMW(55)
    CAPK_VMW(56) CAPK_VMW(57) CAPK_VMW(58) CAPK_VMW(59) CAPK_VMW(60) CAPK_VMW(61) CAPK_VMW(62)
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
#undef CAPK_VMW
  }
}

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
  float alpha, beta;
  int side_kind, act;  // act: CAPK_ACT_* kind | CAPK_ACT_BWD | CAPK_ACT_DERIV
  Drop drop;
  int dropN;  // Epi::N (the dropout mask index is m * dropN + n)
};

// ACT: the forward activation the epilogue evaluates (CAPK_ACT_* kind, 0 = none), a template
// parameter so each of the 16 unrolled epilogue segments carries only its own code
// SIDE: the epilogue reads a side operand (residual / aux / C); a template parameter so the
// kernels without one do not reserve its 64 registers
template <bool AK, bool BK, typename OutT, int ACT, bool SIDE>
__global__ __launch_bounds__(512) void gemm8q_kernel(const void* __restrict__ A, int64_t lda,
                                                     const void* __restrict__ B, int64_t ldb, int M, int N, int K,
                                                     int splits, Epi8q e, float* __restrict__ ws) {
  constexpr int HALF = 128 * 64 * 2, STAGE = 4 * HALF, BIAS0 = 2 * STAGE;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 4 * 1024];  // stages + 4 bias slots
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool lag = wave >= 4;  // waves 4-7 run one barrier behind
  const int ntm = (M + 255) / 256, ntn = (N + 255) / 256, ntiles = ntm * ntn, items = ntiles * splits;
  const int nk_all = (K + 63) / 64, kt_per = (nk_all + splits - 1) / splits;
  const int G = gridDim.x, bid = blockIdx.x;

  const __amdgpu_buffer_rsrc_t rsA = rsrc_of(A, (AK ? (int64_t)M * lda : (int64_t)K * lda) * 2);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_of(B, (BK ? (int64_t)N * ldb : (int64_t)K * ldb) * 2);
  const uint32_t kstepA = AK ? 128u : (uint32_t)(64 * lda * 2);
  const uint32_t kstepB = BK ? 128u : (uint32_t)(64 * ldb * 2);

  // ---- work items: (split, tile), each kt_per K-tiles (the last split's K-tiles past K read
  // zeros: split-K runs on MN-major operands only, whose K rows end at the descriptor range)
  const int nk = kt_per;  // >= 2 (the host routes shorter reductions to gemm8p)
  struct Item {
    int m0, n0, split;  // split < 0: no such item
  };
  auto item_at = [&](int j) -> Item {
    int it;
    if (items <= G) it = j == 0 ? xcd_remap(bid, G) : -1;
    else {
      it = j * G + (bid & 7) * (G >> 3) + (bid >> 3);
      it = it < items ? it : -1;
    }
    if (it < 0) return Item{0, 0, -1};
    const int split = it / ntiles, tile = it - split * ntiles;
    return Item{(tile / ntn) * 256, (tile % ntn) * 256, split};
  };

  // per-lane byte offsets of this wave's two 1-KiB pieces of each half (h: A0 A1 B0 B1) at
  // row0 = 0, k0 = 0; an item's rows / columns and the K-tile enter as the scalar offset
  uint32_t vo[4][2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    vo[0][p] = piece_voff<AK, 2>(wave * 2 + p, lane, 0, 1 << 30, lda);
    vo[1][p] = piece_voff<AK, 2>(wave * 2 + p, lane, 128, 1 << 30, lda);
    vo[2][p] = piece_voff<BK, 2>(wave * 2 + p, lane, 0, 1 << 30, ldb);
    vo[3][p] = piece_voff<BK, 2>(wave * 2 + p, lane, 128, 1 << 30, ldb);
  }
  const uint32_t rowA = AK ? (uint32_t)(lda * 2) : 2u, rowB = BK ? (uint32_t)(ldb * 2) : 2u;  // bytes per row / col
  // K-tile (item it, local k) -> stage slot of global step t; h = 0..3
  auto dma = [&](auto hc, const Item& it, int k, int t) {
    constexpr int h = decltype(hc)::value;
    char* dst = smem + (t & 1) * STAGE + h * HALF;
    // the whole offset goes in the VGPR operand: the descriptor's range check (rows past M /
    // N, K rows past K read as zero) must see it
    const uint32_t so = (h < 2 ? (uint32_t)it.m0 * rowA : (uint32_t)it.n0 * rowB) +
                        (uint32_t)(it.split * kt_per + k) * (h < 2 ? kstepA : kstepB);
#pragma unroll
    for (int p = 0; p < 2; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h < 2 ? rsA : rsB,
                                               (__attribute__((address_space(3))) void*)(dst + (wave * 2 + p) * 1024),
                                               16, vo[h][p] + so, 0, 0, 0);
  };
  using H0 = std::integral_constant<int, 0>;
  using H1 = std::integral_constant<int, 1>;
  using H2 = std::integral_constant<int, 2>;
  using H3 = std::integral_constant<int, 3>;
  // bias of an item: 256 fp32 columns = one 16-B-per-lane LDS-DMA by wave 0 into slot j & 3
  auto bias_dma = [&](const Item& it, int j) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsrc_of(e.bias, (int64_t)N * 4), (__attribute__((address_space(3))) void*)(smem + BIAS0 + (j & 3) * 1024), 16,
        (uint32_t)lane * 16u + (uint32_t)it.n0 * 4u, 0, 0, 0);
  };
  const bool has_bias = e.bias != nullptr && ws == nullptr;
  const int side_kind = (!SIDE || ws) ? SIDE_NONE : e.side_kind;
  const bool has_pre = ACT != 0 && !ws && e.pre != nullptr;

  // ---- fragments and MFMAs (B fragment first: lane = row, registers = 4 consecutive columns)
  auto half = [&](int t, int h) -> const char* { return smem + (t & 1) * STAGE + h * HALF; };
  auto readA = [&](bf16x8 (&f)[2][4], int t, int h) {
    const char* base = half(t, h);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) f[s][i] = frag<AK>(base, wm * 64 + i * 16, s, lane);
  };
  auto readB = [&](bf16x8 (&f)[2][2], int t, int h) {
    const char* base = half(t, h);
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
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[s][j], fa[s][i], c[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
  auto bar = [&] {
    fence();
    raw_barrier();
    fence();
  };
  auto lds_done = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fence();
  };

  // ---- epilogue (register-direct); returns the memory instructions it leaves in flight ----
  const int g4 = lane >> 4, qq = ((g4 & 1) << 1) | (g4 >> 1);  // lane's 8-column group after the swap
  const int lrow = wm * 64 + (lane & 15), lcol = wn * 32 + qq * 8;  // in a 128 x 128 quadrant (+16 i)
  constexpr int ESZ = (int)sizeof(OutT);

  // lane byte offset of (row m0 + lrow, column n0 + qn*128 + lcol) in a [rows][ld] matrix of
  // element size es; columns past N -> OOR (rows past M fail the range check by themselves)
  auto this_lane_off = [&](const Item& c, int64_t ld, int es, int qn) -> uint32_t {
#if defined(CAPK_DIAG_L2STORE)  // diagnostic build: every item stores over tile (0, 0) (L2-resident)
    const int n = qn * 128 + lcol;
    return n < N ? (uint32_t)(((int64_t)lrow * ld + n) * es) : OOR;
#else
    const int n = c.n0 + qn * 128 + lcol;
    return n < N ? (uint32_t)(((int64_t)(c.m0 + lrow) * ld + n) * es) : OOR;
#endif
  };
  // the segment (qm, i) adds (qm*128 + i*16) rows: one v_add of a wave-uniform constant
  auto seg_add = [&](int64_t ld, int es, int qm, int i) -> uint32_t { return (uint32_t)((qm * 128 + i * 16) * ld * es); };
  // One half of an item's epilogue: the 8 segments of quadrant row QM (acc[QM]).
  auto epi_body = [&](const Item& c, int j, const SideSeg<OutT> (&side)[2][2][4], auto qmc) -> int {
    constexpr int QM = decltype(qmc)::value;
    auto lane_off = [&](int64_t ld, int es, int qn) -> uint32_t { return this_lane_off(c, ld, es, qn); };
    // this item's bias (LDS slot j & 3): the lane's 8 columns of each column quadrant
    f32x4 bias[2][2];
    if (has_bias) {
      const float* slot = (const float*)(smem + BIAS0 + (j & 3) * 1024);
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
        bias[qn][0] = *(const f32x4*)(slot + qn * 128 + lcol);
        bias[qn][1] = *(const f32x4*)(slot + qn * 128 + lcol + 4);
      }
    }
    const __amdgpu_buffer_rsrc_t rsC = ws ? rsrc_of(ws, (int64_t)splits * M * N * 4) : rsrc_of(e.C, (int64_t)M * e.ldc * ESZ);
    const __amdgpu_buffer_rsrc_t rsPre = rsrc_of(e.pre, (int64_t)M * e.ldp * ESZ);
    // split-K slab rows: split * M + m of [splits * M][N] fp32 (rows past M must not land in
    // the next split's slab: OOR)
    const int64_t ldo = ws ? N : e.ldc;
    const int eso = ws ? 4 : ESZ;
    uint32_t o0 = lane_off(ldo, eso, 0), o1 = lane_off(ldo, eso, 1);
    if (ws) {
      const uint32_t sl = (uint32_t)((int64_t)c.split * M * N * 4);
      o0 = o0 == OOR ? OOR : o0 + sl;
      o1 = o1 == OOR ? OOR : o1 + sl;
    }
    const uint32_t p0 = has_pre ? lane_off(e.ldp, ESZ, 0) : 0u, p1 = has_pre ? lane_off(e.ldp, ESZ, 1) : 0u;
    const bool unit_alpha = e.alpha == 1.0f;
    // one 16-row x 32-column segment (qm, qn, i), unrolled by hand (the 16 bodies exceed the
    // unroller's budget, and a rolled loop would index the accumulators dynamically)
    auto segment = [&](auto qmc, auto qnc, auto ic) {
      constexpr int qm = decltype(qmc)::value, qn = decltype(qnc)::value, i = decltype(ic)::value;
      // blocks j = 0, 1 (columns 0-15, 16-31 of the strip): lane has columns 4*g4 + r of each;
      // one swap of rows 1,3 of X with rows 0,2 of Y gives 8 consecutive columns
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // (no __builtin_bit_cast of a vector-element expression: ROCm 7.2's clang folds
        // bit_cast(acc[r]) to element 0 for every r -- tools/gemm_layout_probe.py found it)
        const float x = acc[qm][qn][i][0][r], y = acc[qm][qn][i][1][r];
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
        const unsigned sx = sw[0], sy = sw[1];
        v[r] = __uint_as_float(sx);
        v[4 + r] = __uint_as_float(sy);
      }
      const uint32_t ob = qn ? o1 : o0;
      const bool row_ok = c.m0 + qm * 128 + i * 16 + lrow < M;  // (split slabs only: rows past M)
      if (ws) {  // split-K slab: raw fp32 partial sums
        store8(rsC, (row_ok && ob != OOR) ? ob + seg_add(N, 4, qm, i) : OOR, v, (float*)nullptr);
        return;
      }
      if (!unit_alpha) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= e.alpha;
      }
      const SideSeg<OutT>& sd = side[qm][qn][i];
      if (SIDE && side_kind == SIDE_C) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += e.beta * sd.get(k);
      }
      if (has_bias) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] += bias[qn][0][k];
          v[4 + k] += bias[qn][1][k];
        }
      }
      float pre[8];
      if (SIDE && side_kind == SIDE_AUX) {  // backward activation: aux holds act'(pre) (CAPK_ACT_DERIV)
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= sd.get(k);
      } else if constexpr (ACT != 0) {
        if (e.act & CAPK_ACT_DERIV) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = act_fwd_grad_fast(ACT, v[k], pre[k]);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            pre[k] = v[k];
            v[k] = act_fwd_fast(ACT, v[k]);
          }
        }
      }
      if (e.drop.on()) {
        const int m = c.m0 + qm * 128 + i * 16 + lrow, n = c.n0 + qn * 128 + lcol;
        const uint64_t base = (uint64_t)m * e.dropN + n;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= e.drop.mul(base + k);
      }
      if (SIDE && side_kind == SIDE_RES) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += sd.get(k);
      }
      store8(rsC, ob == OOR ? OOR : ob + seg_add(e.ldc, ESZ, qm, i), v, (OutT*)nullptr);
      if (ACT != 0 && has_pre) {
        const uint32_t pb = qn ? p1 : p0;
        store8(rsPre, pb == OOR ? OOR : pb + seg_add(e.ldp, ESZ, qm, i), pre, (OutT*)nullptr);
      }
    };
#define CAPK_SEG(QN, I) \
  segment(qmc, std::integral_constant<int, QN>{}, std::integral_constant<int, I>{});
    CAPK_SEG(0, 0) CAPK_SEG(0, 1) CAPK_SEG(0, 2) CAPK_SEG(0, 3)
    CAPK_SEG(1, 0) CAPK_SEG(1, 1) CAPK_SEG(1, 2) CAPK_SEG(1, 3)
#undef CAPK_SEG
    // memory instructions issued after the last wait (the stores): per segment one (bf16) or
    // two (fp32) for C, the same again for the pre-activation
    constexpr int per = ESZ == 2 ? 1 : 2;
    return ws ? 8 * 2 : 8 * per * ((ACT != 0 && has_pre) ? 2 : 1);
  };
  // The item's epilogue, one quadrant row (half) at a time; a side operand (residual / aux /
  // C) is loaded per half, 8 segments in flight, one wait (the first also retires the next
  // item's operand loads issued before it, the second the first half's stores).  Returns the
  // memory instructions it leaves in flight (the second half's stores, + the first's without
  // a side operand).
  auto epilogue = [&](const Item& c, int j) -> int {
    SideSeg<OutT> side[2][2][4];
    auto load_side = [&](auto qmc) {
      constexpr int QM = decltype(qmc)::value;
      if constexpr (SIDE && ESZ == 2) {
        if (side_kind != SIDE_NONE) {
          const __amdgpu_buffer_rsrc_t rsSide = rsrc_of(e.side, (int64_t)M * e.lds * ESZ);
          const uint32_t s0 = this_lane_off(c, e.lds, ESZ, 0), s1 = this_lane_off(c, e.lds, ESZ, 1);
#pragma unroll
          for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int i = 0; i < 4; ++i) side[QM][qn][i].load(rsSide, (qn ? s1 : s0) + seg_add(e.lds, ESZ, QM, i));
          asm volatile("s_waitcnt vmcnt(0)"
                       : "+v"(side[QM][0][0].a), "+v"(side[QM][0][1].a), "+v"(side[QM][0][2].a), "+v"(side[QM][0][3].a),
                         "+v"(side[QM][1][0].a), "+v"(side[QM][1][1].a), "+v"(side[QM][1][2].a), "+v"(side[QM][1][3].a)
                       :
                       : "memory");
          fence();
        }
      }
    };
    using QA = std::integral_constant<int, 0>;
    using QB = std::integral_constant<int, 1>;
    load_side(QA{});
    const int n0 = epi_body(c, j, side, QA{});
    load_side(QB{});
    const int n1 = epi_body(c, j, side, QB{});
    return (SIDE && ESZ == 2 && side_kind != SIDE_NONE) ? n1 : n0 + n1;
  };
  auto zero_half = [&](auto qmc) {
    constexpr int QM = decltype(qmc)::value;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[QM][b][i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
  };

  // ---- main loop: four phases per K-tile, one C quadrant (16 MFMAs) each ----
  //   phase  quadrant  ds_read (L)       LDS-DMA issued (L)   waits for (L, read next phase)
  //   P1     (0,0)     A0(t) B0(t)       A1(t+1)              B1(t)
  //   P2     (0,1)     B1(t)             A0(t+2)              A1(t)
  //   P3     (1,1)     A1(t)             B0(t+2)              -
  //   P4     (1,0)     - (B0 kept)       B1(t+2)              A0(t+1) B0(t+1)
  // A half is refilled in the phase after its last read (LDS WAR), waited for one phase before
  // its first read (RAW: wait, barrier, read); in steady state each wait leaves the four
  // younger groups (8 instructions) in flight.  Step t of this WG is K-tile k = t mod nk of
  // its item j = t / nk; `cur` is item j, `nxt` item j+1 (nk >= 2: steps t+1, t+2 lie in one
  // of the two).  Every wait is computed from the per-wave ledger (ops, issue marks).
  int j = 0, k = 0;
  Item cur = item_at(0), nxt = item_at(1);
  if (cur.split < 0) return;  // (the host never launches an idle WG)
  zero_acc();
  int ops = 0;  // memory instructions this wave has issued (loads, LDS-DMA, stores), in order
  // issue half h of K-tile `ahead` steps after (item cur, local k); returns the issue mark
  auto issue = [&](auto hc, int ahead, int t) -> int {
    const bool same = k + ahead < nk;
    const Item& it = same ? cur : nxt;
    if (it.split >= 0) {
      const int kk = same ? k + ahead : k + ahead - nk;
      dma(hc, it, kk, t + ahead);
      ops += 2;
      if (decltype(hc)::value == 2 && kk == 0 && has_bias && wave == 0) {  // the item's bias, with B0 of its first K-tile
        bias_dma(it, (t + ahead) / nk);
        ops += 1;
      }
    }
    return ops;
  };
  // prologue: A0 B0 B1 A1 of K-tile 0, A0 B0 B1 of K-tile 1
  issue(H0{}, 0, 0);
  int mB0 = issue(H2{}, 0, 0);  // (B0(t) and A0(t) are read together: one mark)
  int mB1 = issue(H3{}, 0, 0);
  int mA1 = issue(H1{}, 0, 0);
  issue(H0{}, 1, 0);
  int mB0n = issue(H2{}, 1, 0);
  int mB1n = issue(H3{}, 1, 0);
  vm_wait(ops - mB0);
  bar();
  if (lag) bar();  // waves 4-7 fall one barrier behind

  bf16x8 fa[2][4], fb0[2][2], fb1[2][2];
  for (int t = 0;; ++t) {
    // P1: (0,0).  L: [epilogue of the previous item] read A0, B0 (t); wait B1 (t); issue A1 (t+1)
    readA(fa, t, 0);
    readB(fb0, t, 2);
    vm_wait(ops - mB1);
    const int mA1n = issue(H1{}, 1, t);
    lds_done();
    bar();
    mma(fa, fb0, acc[0][0]);
    bar();
    // P2: (0,1).  L: read B1 (t); wait A1 (t); issue A0 (t+2)
    readB(fb1, t, 3);
    vm_wait(ops - mA1);
    issue(H0{}, 2, t);
    lds_done();
    bar();
    mma(fa, fb1, acc[0][1]);
    bar();
    // P3: (1,1).  L: read A1 (t); issue B0 (t+2)
    readA(fa, t, 1);
    const int mB0nn = issue(H2{}, 2, t);
    lds_done();
    bar();
    mma(fa, fb1, acc[1][1]);
    bar();
    // P4: (1,0).  L: wait A0 B0 (t+1); issue B1 (t+2)
    vm_wait(ops - mB0n);
    const int mB1nn = issue(H3{}, 2, t);
    fence();
    bar();
    mma(fa, fb0, acc[1][0]);
    bar();
    mB1 = mB1n;
    mB1n = mB1nn;
    mB0n = mB0nn;
    mA1 = mA1n;
    if (++k == nk) {  // the item's last K-tile: epilogue, stores left in flight
      fence();
      ops += epilogue(cur, j);
      zero_acc();
      fence();
      k = 0;
      ++j;
      cur = nxt;
      if (cur.split < 0) break;
      nxt = item_at(j + 1);
    }
  }
  if (!lag) bar();  // realign the two groups (every barrier is matched)
}

}  // namespace

bool gemm8q_supports(const Epi& e, bool out_f32) {
  const int sides = ((e.act & CAPK_ACT_BWD) ? 1 : 0) + (e.res ? 1 : 0) + (e.beta != 0.f ? 1 : 0);
  const int a = e.act & 15;
  if (a && !(e.act & CAPK_ACT_BWD) && a != CAPK_ACT_GELU_ERF && a != CAPK_ACT_GELU_TANH && a != CAPK_ACT_QUICK_GELU &&
      a != CAPK_ACT_RELU)
    return false;  // (tanh / sigmoid epilogues: pooler-sized products, the 8p kernel)
  // backward activations only in the multiply-by-aux form (CAPK_ACT_DERIV: aux = act'(pre))
  // (fp32 outputs take no side operand and no activation here: 16 segments of 8 fp32 would
  // need 128 VGPRs)
  if (out_f32 && (a && !(e.act & CAPK_ACT_BWD))) return false;
  return sides <= (out_f32 ? 0 : 1) && (!(e.act & CAPK_ACT_BWD) || (e.act & CAPK_ACT_DERIV));
}

int launch_gemm8q(bool a_kmajor, bool b_kmajor, bool out_f32, const void* A, int64_t lda, const void* B, int64_t ldb,
                  int M, int N, int K, int splits, const Epi& e, float* slab, hipStream_t st) {
  CAPK_CHECK_ARG((a_kmajor ? (int64_t)M * lda : (int64_t)K * lda) * 2 < (1ll << 31) &&
                     (b_kmajor ? (int64_t)N * ldb : (int64_t)K * ldb) * 2 < (1ll << 31),
                 "capk_gemm(bf16, 256x256): operand larger than 2 GiB");
  CAPK_CHECK_ARG(gemm8q_supports(e, out_f32), "capk_gemm(gemm8q): unsupported epilogue");
  const int64_t esz = out_f32 ? 4 : 2;
  Epi8q p{};
  p.C = e.C;
  p.ldc = e.ldc;
  p.alpha = e.alpha;
  p.beta = e.beta;
  p.bias = e.bias;
  p.act = e.act;
  p.drop = e.drop;
  p.dropN = e.N;
  const bool fwd_act = (e.act & 15) && !(e.act & CAPK_ACT_BWD);
  if (fwd_act && e.pre) {
    p.pre = e.pre;
    p.ldp = e.ldx;
  }
  if (e.act & CAPK_ACT_BWD) {
    p.side_kind = SIDE_AUX;
    p.side = e.aux;
    p.lds = e.ldx;
  } else if (e.res) {
    p.side_kind = SIDE_RES;
    p.side = e.res;
    p.lds = e.ldr;
  } else if (e.beta != 0.f) {
    p.side_kind = SIDE_C;
    p.side = e.C;
    p.lds = e.ldc;
  }
  CAPK_CHECK_ARG((slab ? (int64_t)splits * M * N * 4 : (int64_t)M * e.ldc * esz) < (1ll << 31) &&
                     (!p.pre || (int64_t)M * p.ldp * esz < (1ll << 31)) &&
                     (!p.side || (int64_t)M * p.lds * esz < (1ll << 31)),
                 "capk_gemm(bf16, 256x256): output or side operand larger than 2 GiB");
  const int items = cdiv(M, 256) * cdiv(N, 256) * splits;
  const int grid = items <= 256 ? items : 256;
#define L8(AK, BKM, OT, ACTK, SD)                                                                                 \
  hipLaunchKernelGGL((gemm8q_kernel<AK, BKM, OT, ACTK, SD>), dim3(grid), dim3(512), 0, st, A, lda, B, ldb, M, N, K, \
                     splits, p, slab)
#define L8S(AK, BKM, OT, ACTK)          \
  if (side) L8(AK, BKM, OT, ACTK, true); \
  else L8(AK, BKM, OT, ACTK, false);
#define L8D(OT)                                                                    \
  if (a_kmajor && b_kmajor) {                                                       \
    switch (fwd_act && !slab ? (e.act & 15) : 0) {                                  \
      case CAPK_ACT_GELU_ERF: L8S(true, true, OT, CAPK_ACT_GELU_ERF) break;         \
      case CAPK_ACT_GELU_TANH: L8S(true, true, OT, CAPK_ACT_GELU_TANH) break;       \
      case CAPK_ACT_QUICK_GELU: L8S(true, true, OT, CAPK_ACT_QUICK_GELU) break;     \
      case CAPK_ACT_RELU: L8S(true, true, OT, CAPK_ACT_RELU) break;                 \
      default: L8S(true, true, OT, 0) break;                                        \
    }                                                                               \
  } else if (a_kmajor) {                                                            \
    L8S(true, false, OT, 0)                                                         \
  } else if (b_kmajor) {                                                            \
    L8S(false, true, OT, 0)                                                         \
  } else {                                                                          \
    L8S(false, false, OT, 0)                                                        \
  }
  CAPK_CHECK_ARG(!fwd_act || slab || (a_kmajor && b_kmajor), "capk_gemm(gemm8q): forward activations need K-major operands");
  const bool side = !slab && p.side_kind != SIDE_NONE;
  if (out_f32) {
    // fp32 outputs: no activation, no side operand (gemm8q_supports)
    if (a_kmajor && b_kmajor) L8(true, true, float, 0, false);
    else if (a_kmajor) L8(true, false, float, 0, false);
    else if (b_kmajor) L8(false, true, float, 0, false);
    else L8(false, false, float, 0, false);
  } else {
    L8D(bf16)
  }
#undef L8D
#undef L8S
#undef L8
  CAPK_LAUNCH_CHECK("gemm8q_kernel");
  return CAPK_OK;
}

}  // namespace capk
