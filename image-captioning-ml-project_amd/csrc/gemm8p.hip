// 256x256 phased bf16 GEMM — the large-grid kernel of capk_gemm (shared pieces in
// gemm_common.h, dispatch in gemm.hip).
//
// Tile 256x256x64, 8 waves (2 in M x 4 in N), one WG per CU.  Operands are staged in
// 16-KiB half-tiles -- A0 (tile rows 0-127), A1 (128-255), B0 (tile cols 0-127), B1
// (128-255) of one 64-deep K-tile -- through two 64-KiB LDS stages (half h of K-tile t at
// stage t & 1).  Wave (wm, wn) owns the four 64x32 output quadrants (qm, qn) at rows
// qm*128 + wm*64, cols qn*128 + wn*32, so quadrant (qm, qn) reads only A_qm and B_qn.  A
// K-tile runs as two phases, Q1 = quadrants (0,0) + (0,1) on A0 and Q2 = (1,1) + (1,0) on
// A1 (32 v_mfma_f32_16x16x32_bf16 each).  Every phase is two segments separated by
// workgroup barriers: L (ds_read the phase's fragments, wait for landed halves, issue
// LDS-DMA, lgkmcnt(0)) and M (the 32 MFMAs).  Waves 4-7 run one barrier behind waves 0-3
// (one extra s_barrier before the loop, cdna guide §5 template / MI355X_MICROARCH "two
// waves per SIMD" item 9): the two waves sharing a SIMD alternate L and M, so one wave's
// LDS / DMA issue overlaps its partner's MFMAs.
//
//   phase   ds_read (L)              LDS-DMA issued (L)           vmcnt wait (L, for next phase)
//   Q1      A0(t), B0(t), B1(t)      A1(t+1)                      A1(t)              vmcnt(6)
//   Q2      A1(t)                    A0(t+2), B0(t+2), B1(t+2)    A0/B0/B1(t+1)      vmcnt(2)
//
// With the groups one barrier apart, a half is published to every wave by waiting for it
// one phase before its first read (each wave waits for its own LDS-DMA pieces, and a
// barrier of both groups lies between every wait and every read), and a stage slot may be
// refilled from the phase after its last read (every L ends with lgkmcnt(0) before the
// next barrier) -- two phases (four MFMA segments) between a half's LDS-DMA and its wait.
// The schedule, RAW / WAR safety and every wait count were checked by simulation over
// K-tile counts 1..14 (tail waits are computed from the same schedule at run time).
// Operand addresses are 32-bit buffer offsets computed once per lane (8 VGPRs); rows past
// the operand's end and K rows past K read as zero through the descriptor range check.
#include <type_traits>

#include "gemm_common.h"

namespace capk {

namespace {

// fp8 (F8): one 16x16x128 operand half-fragment -- 16-B chunk 2*(lane>>4) + s of row
// rbase + (lane&15) of a K-major [128 rows][128 B] image, i.e. the lane's 32 k-bytes
// 32*(lane>>4) .. +31 split in two (s = 0, 1); the same swizzled image as bf16.
__device__ __forceinline__ bf16x8 frag8(const char* half, int rbase, int s, int lane) {
  const int r = rbase + (lane & 15);
  const int lc = 2 * (lane >> 4) + s;
  return *(const bf16x8*)(half + r * 128 + ((lc ^ swz_k<64>(r)) << 4));
}
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x8 cat8(const bf16x8& lo, const bf16x8& hi) {
  const i32x4 a = __builtin_bit_cast(i32x4, lo), b = __builtin_bit_cast(i32x4, hi);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
// E8M0 scale bytes of 4 fragment rows row0 + 16*i + (lane & 15), i = 0..3, packed (byte i);
// rows past `rows` take the last row's code (their data read as zero)
__device__ __forceinline__ uint32_t scale_word(const uint8_t* sc, int row0, int rows, int lane) {
  uint32_t w = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = row0 + 16 * i + (lane & 15);
    w |= (uint32_t)sc[r < rows ? r : rows - 1] << (8 * i);
  }
  return w;
}

__device__ __forceinline__ void pin(const Raw8<bf16>& r) { asm volatile("" ::"v"(r.v)); }
__device__ __forceinline__ void pin(const Raw8<float>& r) { asm volatile("" ::"v"(r.a), "v"(r.b)); }

template <bool AK, bool BK, typename OutT, bool F8 = false>
__global__ __launch_bounds__(512) void gemm8p_kernel(const void* __restrict__ A, int64_t lda,
                                                     const void* __restrict__ B, int64_t ldb, int M, int N, int K,
                                                     int splits, Epi e, float* __restrict__ ws,
                                                     const uint8_t* __restrict__ scA, const uint8_t* __restrict__ scB) {
  static_assert(!F8 || (AK && BK), "fp8 operands are K-major");
  constexpr int ESZ = F8 ? 1 : 2, BKE = F8 ? 128 : 64;  // element bytes, K elements per K-tile
  constexpr int HALF = 128 * 64 * 2, STAGE = 4 * HALF;
  constexpr int EPI_LD = 256 + 4;
  constexpr int SMEM = (2 * STAGE > 128 * EPI_LD * 4) ? 2 * STAGE : 128 * EPI_LD * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool lag = wave >= 4;  // waves 4-7 run one barrier behind
  const int ntm = (M + 255) / 256, ntn = (N + 255) / 256, ntiles = ntm * ntn;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles, tile = wg % ntiles;
  const int m0 = (tile / ntn) * 256, n0 = (tile % ntn) * 256;
  const int nk_all = (K + BKE - 1) / BKE;
  const int kt_per = (nk_all + splits - 1) / splits;
  const int kt0 = split * kt_per;
  const int nk = max(0, min(nk_all, kt0 + kt_per) - kt0);
  // descriptor ranges: K-major operands end at row M (N); MN-major ones at k row K
  const int bytesA = (int)((AK ? (int64_t)M * lda : (int64_t)K * lda) * ESZ);
  const int bytesB = (int)((BK ? (int64_t)N * ldb : (int64_t)K * ldb) * ESZ);
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, bytesA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, bytesB, 0x00020000);
  // per-lane offsets of this wave's two pieces in each half (k0 = 0); h: 0 = A0, 1 = A1,
  // 2 = B0, 3 = B1
  uint32_t vo[4][2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    vo[0][p] = piece_voff<AK, ESZ>(wave * 2 + p, lane, m0, M, lda);
    vo[1][p] = piece_voff<AK, ESZ>(wave * 2 + p, lane, m0 + 128, M, lda);
    vo[2][p] = piece_voff<BK, ESZ>(wave * 2 + p, lane, n0, N, ldb);
    vo[3][p] = piece_voff<BK, ESZ>(wave * 2 + p, lane, n0 + 128, N, ldb);
  }
  // byte step of one K-tile: 64 k along a K-major row, 64 k rows of an MN-major operand
  const uint32_t kstepA = AK ? 128u : (uint32_t)(64 * lda * 2);
  const uint32_t kstepB = BK ? 128u : (uint32_t)(64 * ldb * 2);

  auto half = [&](int t, int h) -> char* { return smem + (t & 1) * STAGE + h * HALF; };
  auto ex = [&](int t) { return t >= 0 && t < nk; };
  auto load = [&](int t, int h) {
    if (!ex(t)) return;
    char* dst = half(t, h);
#if defined(CAPK_DIAG_NOKSTEP)  // diagnostic build: every K-tile re-reads K-tile 0 (L2-resident)
    const uint32_t koff = 0u * (uint32_t)(kt0 + t);
#else
    const uint32_t koff = (uint32_t)(kt0 + t) * (h < 2 ? kstepA : kstepB);
#endif
#if defined(CAPK_V_GLDS)  // diagnostic: flat global_load_lds (no range check: full tiles only)
    const char* gbase = (const char*)(h < 2 ? (const void*)A : (const void*)B);
#pragma unroll
    for (int p = 0; p < 2; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(gbase + vo[h][p] + koff),
                                       (__attribute__((address_space(3))) void*)(dst + (wave * 2 + p) * 1024), 16, 0, 0);
#else
#pragma unroll
    for (int p = 0; p < 2; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h < 2 ? rsA : rsB,
                                               (__attribute__((address_space(3))) void*)(dst + (wave * 2 + p) * 1024),
                                               16, vo[h][p] + koff, 0, 0, 0);
#endif
  };
  // LDS-DMA schedule by global phase ph = 2u + j (j = 0: Q1, 1: Q2 of K-tile u):
  //   Q1: A1(u+1)   Q2: A0(u+2), B0(u+2), B1(u+2)
  auto issue = [&](int ph) {
    const int u = ph >> 1, j = ph & 1;
    if (j == 0) {
      load(u + 1, 1);
    } else {
      load(u + 2, 0);
      load(u + 2, 2);
      load(u + 2, 3);
    }
  };
  auto nload = [&](int ph) {  // LDS-DMA instructions issued in phase ph
    const int u = ph >> 1, j = ph & 1;
    return j == 0 ? 2 * ex(u + 1) : 6 * ex(u + 2);
  };
  auto younger = [&](int ph_a, int ph_b) {  // instructions issued in phases (ph_a, ph_b)
    int c = 0;
    for (int ph = ph_a + 1; ph < ph_b; ++ph) c += nload(ph);
    return c;
  };
  auto wait_n = [](int n) {  // s_waitcnt vmcnt(<= n)
    if (n >= 16) wait_vmc<16>();
    else if (n >= 14) wait_vmc<14>();
    else if (n >= 12) wait_vmc<12>();
    else if (n >= 10) wait_vmc<10>();
    else if (n >= 8) wait_vmc<8>();
    else if (n >= 6) wait_vmc<6>();
    else if (n >= 4) wait_vmc<4>();
    else if (n >= 2) wait_vmc<2>();
    else wait_vmc<0>();
  };
  auto readA = [&](bf16x8 (&f)[2][4], int t, int h) {
    const char* base = half(t, h);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (F8) f[s][i] = frag8(base, wm * 64 + i * 16, s, lane);
        else f[s][i] = frag<AK>(base, wm * 64 + i * 16, s, lane);
      }
  };
  auto readB = [&](bf16x8 (&f)[2][2], int t, int h) {
    const char* base = half(t, h);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (F8) f[s][j] = frag8(base, wn * 32 + j * 16, s, lane);
        else f[s][j] = frag<BK>(base, wn * 32 + j * 16, s, lane);
      }
  };
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // fp8: E8M0 row scales of this wave's fragment rows, applied inside the scaled MFMA
  // (byte i of sa[qm]: A rows qm*128 + wm*64 + 16i + (lane&15); byte 2qn+j of sb: B rows
  // qn*128 + wn*32 + 16j + (lane&15))
  uint32_t sa[2] = {0u, 0u}, sb = 0u;
  if constexpr (F8) {
    sa[0] = scale_word(scA, m0 + wm * 64, M, lane);
    sa[1] = scale_word(scA, m0 + 128 + wm * 64, M, lane);
    const uint32_t b0 = scale_word(scB, n0 + wn * 32, N, lane), b1 = scale_word(scB, n0 + 128 + wn * 32, N, lane);
    sb = (b0 & 0xFFFFu) | (b1 << 16);
  }
  auto mma = [&](const bf16x8 (&fa)[2][4], const bf16x8 (&fb)[2][2], f32x4 (&c)[4][2], auto qmc, auto qnc) {
    constexpr int QM = decltype(qmc)::value, QN = decltype(qnc)::value;
#if !defined(CAPK_V_NOPRIO) && !defined(CAPK_V_STATICPRIO)
    __builtin_amdgcn_s_setprio(1);
#endif
#if defined(CAPK_DIAG_NOMFMA)  // diagnostic build: keep the fragments live, skip the MFMAs
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(fa[s][i]), "v"(fb[s][j]));
#else
    if constexpr (F8) {
      const int sA = (int)sa[QM], sB = (int)sb;
#define F8MMA(I, J)                                                                                              \
  c[I][J] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(cat8(fa[0][I], fa[1][I]), cat8(fb[0][J], fb[1][J]), \
                                                             c[I][J], 0, 0, I, sA, 2 * QN + J, sB)
      F8MMA(0, 0); F8MMA(0, 1); F8MMA(1, 0); F8MMA(1, 1);
      F8MMA(2, 0); F8MMA(2, 1); F8MMA(3, 0); F8MMA(3, 1);
#undef F8MMA
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s][i], fb[s][j], c[i][j], 0, 0, 0);
    }
#endif
#if !defined(CAPK_V_NOPRIO) && !defined(CAPK_V_STATICPRIO)
    __builtin_amdgcn_s_setprio(0);
#endif
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

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  bf16x8 fa[2][4], fb0[2][2], fb1[2][2];
  // prologue: K-tiles 0 and 1 in the order the steady-state phases -3 .. -1 would issue
  // them (A0/B0/B1(0), A1(0), A0/B0/B1(1)), then wait for A0/B0/B1(0) (read in phase 0)
#pragma unroll
  for (int ph = -3; ph < 0; ++ph) issue(ph);
  wait_n(younger(-3, 0));
  bar();
#if defined(CAPK_V_STATICPRIO)
  if (lag) __builtin_amdgcn_s_setprio(1);
#endif
#if !defined(CAPK_V_NOSTAGGER)
  if (lag) bar();  // waves 4-7 fall one barrier behind
#endif
  for (int u = 0; u < nk; ++u) {
    const int ph = 2 * u;
    const bool steady = u + 2 < nk;
    // Q1: quadrants (0,0), (0,1).  L: read A0(u), B0(u), B1(u); wait A1(u) (phase 2u-2)
    readA(fa, u, 0);
    readB(fb0, u, 2);
    readB(fb1, u, 3);
    if (steady) wait_vmc<6>(); else wait_n(younger(ph - 2, ph));
    issue(ph);
    lds_done();
    bar();
    mma(fa, fb0, acc[0][0], I0{}, I0{});
    mma(fa, fb1, acc[0][1], I0{}, I1{});
    bar();
    // Q2: quadrants (1,1), (1,0).  L: read A1(u); wait A0/B0/B1(u+1) (phase 2u-1)
    readA(fa, u, 1);
    if (steady) wait_vmc<2>(); else wait_n(younger(ph - 1, ph + 1));
    issue(ph + 1);
    lds_done();
    bar();
    mma(fa, fb1, acc[1][1], I1{}, I1{});
    mma(fa, fb0, acc[1][0], I1{}, I0{});
    bar();
  }
#if !defined(CAPK_V_NOSTAGGER)
  if (!lag) bar();  // realign the two groups before the epilogue
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if defined(CAPK_DIAG_NOSTORE)  // diagnostic build: main loop only (accumulators kept live, no epilogue)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[a][b][i][j]));
  return;
#endif

  // ---- epilogue: two 128-row halves through LDS (fp32); each thread owns 8 fixed columns
  constexpr int ITS = 256 * 256 / 8 / 512;  // 16 row segments per thread over the tile
  const int ecol = (tid & 31) * 8, egn = n0 + ecol;
  float bias8[8];
  Raw8<OutT> side[4][ITS / 4];
  bool has_side;
  // Side operand (aux of a backward activation, else the residual): all 16 segments are
  // loaded up front and pinned by one empty asm use after the first LDS barrier, so they
  // share one memory round trip that overlaps the accumulator staging.  (Unpinned, the
  // compiler sinks each load to its first use, behind the previous segments' stores --
  // vmcnt counts stores too -- serialising one round trip per segment: +180 us on a
  // 50432 x 3072 epilogue.)
  has_side = !ws && prefetch_side<OutT, 4, ITS / 4, 512, 32>(e, m0, egn, tid, bias8, side);
  lds_barrier();
  float* stg = (float*)smem;
#pragma unroll
  for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
            const int col = qn * 128 + wn * 32 + j * 16 + (lane & 15);
            stg[row * EPI_LD + col] = acc[qm][qn][i][j][r];
          }
    lds_barrier();
    if (qm == 0 && has_side) {
#pragma unroll
      for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int it = 0; it < ITS / 4; ++it) pin(side[h][it]);
    }
#pragma unroll
    for (int it = 0; it < ITS / 2; ++it) {
      const int row = (it * 512 + tid) >> 5;  // 0..127 within this half
      const int gm = m0 + qm * 128 + row;
      if (gm < M && egn < N) {
        float v[8];
        Vec8<float>::load(stg + row * EPI_LD + ecol, v);
        if (ws) Vec8<float>::store(ws + ((int64_t)split * M + gm) * N + egn, v);
        else epilogue8<OutT>(e, gm, egn, v, e.bias ? bias8 : nullptr, has_side ? &side[qm * 2 + (it >> 2)][it & 3] : nullptr);
      }
    }
    lds_barrier();
  }
}

}  // namespace

int launch_gemm8p(bool a_kmajor, bool b_kmajor, bool out_f32, int grid, const void* A, int64_t lda, const void* B,
                  int64_t ldb, int M, int N, int K, int splits, const Epi& e, float* slab, hipStream_t st) {
  CAPK_CHECK_ARG((a_kmajor ? (int64_t)M * lda : (int64_t)K * lda) * 2 < (1ll << 31) &&
                     (b_kmajor ? (int64_t)N * ldb : (int64_t)K * ldb) * 2 < (1ll << 31),
                 "capk_gemm(bf16, 256x256): operand larger than 2 GiB");
#define L8(AK, BKM, OT)                                                                                            \
  hipLaunchKernelGGL((gemm8p_kernel<AK, BKM, OT>), dim3(grid), dim3(512), 0, st, A, lda, B, ldb, M, N, K, splits, \
                     e, slab, nullptr, nullptr)
#define L8D(OT)                                  \
  if (a_kmajor && b_kmajor) L8(true, true, OT);   \
  else if (a_kmajor) L8(true, false, OT);         \
  else if (b_kmajor) L8(false, true, OT);         \
  else L8(false, false, OT);
  if (out_f32) { L8D(float) } else { L8D(bf16) }
#undef L8D
#undef L8
  CAPK_LAUNCH_CHECK("gemm8p_kernel");
  return CAPK_OK;
}

int launch_gemm8p_f8(bool out_f32, int grid, const void* A, int64_t lda, const uint8_t* scA, const void* B,
                     int64_t ldb, const uint8_t* scB, int M, int N, int K, int splits, const Epi& e, float* slab,
                     hipStream_t st) {
  CAPK_CHECK_ARG((int64_t)M * lda < (1ll << 31) && (int64_t)N * ldb < (1ll << 31),
                 "capk_gemm_f8: operand larger than 2 GiB");
  if (out_f32)
    hipLaunchKernelGGL((gemm8p_kernel<true, true, float, true>), dim3(grid), dim3(512), 0, st, A, lda, B, ldb, M, N, K,
                       splits, e, slab, scA, scB);
  else
    hipLaunchKernelGGL((gemm8p_kernel<true, true, bf16, true>), dim3(grid), dim3(512), 0, st, A, lda, B, ldb, M, N, K,
                       splits, e, slab, scA, scB);
  CAPK_LAUNCH_CHECK("gemm8p_kernel<f8>");
  return CAPK_OK;
}

}  // namespace capk
