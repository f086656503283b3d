// Fused multi-head attention forward/backward for short sequences
// (ViT N=197, CLIP N=50, decoder T=20 self / T x 196 cross).  One workgroup per
// (batch, head); the whole K/V (fwd) or Q/K/V/dO (bwd) of that head is staged
// in LDS once, so S = QK^T never reaches HBM.
//
// bf16 path (v_mfma_f32_16x16x32_bf16):
//  fwd: each wave owns 16-query tiles and computes S^T = K Q^T so that every
//       lane holds one query's scores (column = lane&15); row max / sum need
//       only two xor-shuffles (16, 32).  P^T stays in registers and is the B
//       operand of O^T = V^T P^T with the k (=key) order permuted to match the
//       accumulator layout; V is staged row-major and its V^T fragments are read
//       with ds_read_b64_tr_b16.  LSE is saved for backward.
//  bwd: phase A (waves own 16-key blocks): S, dP, dS recomputed with the key on
//       the lane; dV^T += dO^T P and dK^T += Q^T dS take dO^T / Q^T from the
//       row-major LDS images via ds_read_b64_tr_b16.  Phase B (waves own 16-query
//       blocks): S^T, dP^T recomputed; dQ^T += K^T dS^T (K^T by tr reads).  No
//       atomics: every output element has one owner.
// f32 path (parity): straightforward per-query / per-key loops, exact fp32.
#include <stdlib.h>

#include "common.h"

namespace capk {

struct AttnArgs {
  int B, H, Nq, Nk, hd, causal;
  float scale;
  const void *q, *k, *v, *o, *dout;
  int64_t q_bs, q_rs, k_bs, k_rs, v_bs, v_rs, o_bs, o_rs, do_bs, do_rs;
  const uint8_t* key_pad;
  void* out;
  int64_t out_bs, out_rs;
  float* lse;
  const float* lse_in;
  void *dq, *dk, *dv;
  int64_t dq_bs, dq_rs, dk_bs, dk_rs, dv_bs, dv_rs;
  Drop drop;  // attention-probability dropout, mask index ((b*H + h)*Nq + q)*Nk + key
  // decode with a beam-history table (capk_attention_decode_rows): key j < Nk-1 of batch row b
  // lives in K/V row kv_rows[b * kv_rows_ld + j], the last key (the step's own token) in row b
  const int* kv_rows;
  int64_t kv_rows_ld;
  // backward, optional (split kernels): per-image column sums of dQ / dK / dV -- the fused QKV
  // bias gradient of capk_attention_bwd_bias.  Row b of [B][ld]: dQ sums at h*hd + d, dK at
  // H*hd + h*hd + d, dV at 2*H*hd + h*hd + d (one colsum_finish launch sums the images).
  // rsum: [B*H][2][Nq] scratch of the dQ kernel (per-query sums over the keys of dS and P).
  float* dbias_part;
  int64_t dbias_ld;
  float* rsum;
  int b_base;  // batch index of this launch's first image (a batch slice): dropout mask index
  // XCD-chunked block order (xcd_bh): set by the host when the grid is B * H blocks, B * H % 8 == 0
  int xcd_chunk;
  // stage the swizzled 64-wide head images by LDS DMA (stage_dma_sw), bit 0 forward, 1 dQ, 2 dK/dV
  int dma_stage;
};

// (batch, head) of this workgroup.  Workgroups are dispatched round-robin over the 8 XCDs
// (block i runs on XCD i % 8), so with the plain order the H heads of one image run on H
// different XCDs.  With hd = 96 a head's slice of a K / V row is 192 B and shares 128-B lines
// with its neighbours, so every XCD fetched each line of the row through its own L2.  With
// xcd_chunk, XCD x takes the contiguous logical blocks [x n / 8, (x + 1) n / 8) in order: the
// heads of an image run back to back on one XCD and read the shared lines once.
__device__ __forceinline__ int xcd_bh(const AttnArgs& a) {
  const int i = blockIdx.x;
  return a.xcd_chunk ? (i & 7) * (int)(gridDim.x >> 3) + (i >> 3) : i;
}


// the K / V batch row holding key j of batch row b
__device__ __forceinline__ int64_t kv_row(const AttnArgs& a, int b, int j) {
  return (a.kv_rows && j < a.Nk - 1) ? (int64_t)a.kv_rows[(int64_t)b * a.kv_rows_ld + j] : (int64_t)b;
}
__device__ __forceinline__ uint64_t drop_idx(const AttnArgs& a, int b, int h, int q, int key) {
  return (((uint64_t)(b + a.b_base) * a.H + h) * a.Nq + q) * a.Nk + key;
}
__device__ __forceinline__ float pdrop(const AttnArgs& a, int b, int h, int q, int key) {
  return a.drop.mul(drop_idx(a, b, h, q, key));
}
// Drop::mul(idx0 + off) for a run of a lane's scores from one base index (the same values as
// pdrop: drop_hash's low-word product is (lo + off) C1 = lo C1 + off C1 mod 2^32, and a carry
// out of the low word adds C2 to the high word's): per score two adds, a compare and the
// finaliser, instead of the 64-bit index product and two more 32-bit multiplies.
struct DropRun {
  uint32_t lo, lo_c1, hi_c2;
  __device__ __forceinline__ explicit DropRun(uint64_t idx0)
      : lo((uint32_t)idx0), lo_c1((uint32_t)idx0 * 0x9E3779B9u), hi_c2((uint32_t)(idx0 >> 32) * 0x7FEB352Du) {}
  __device__ __forceinline__ float mul(const Drop& d, uint32_t off) const {
    const uint32_t l = lo + off;
    uint32_t x = d.seed ^ (lo_c1 + off * 0x9E3779B9u) ^ (hi_c2 + (l < off ? 0x7FEB352Du : 0u));
    x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
    return x >= d.thr ? d.scale : 0.f;
  }
};

__device__ __forceinline__ bool key_ok(const AttnArgs& a, int b, int key, int q) {
  if (key >= a.Nk) return false;
  if (a.causal && key > q + (a.Nk - a.Nq)) return false;  // bottom-right aligned (prefix / KV cache)
  if (a.key_pad && a.key_pad[(int64_t)b * a.Nk + key]) return false;
  return true;
}

// a 16-key block with no causal / padding / tail mask (wave-uniform test)
__device__ __forceinline__ bool full_kb(const AttnArgs& a, int kb) {
  return !a.causal && !a.key_pad && (kb + 1) * 16 <= a.Nk;
}
constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;

// Compile-time launch modes of the bf16 kernels: MODE bit 0 = probability dropout, bit 1 =
// causal / key-padding masks.  The common ViT / cross-attention launch (mode 0) has no
// per-score branches: only the last key block is tested, against Nk.
constexpr int AM_DROP = 1, AM_MASK = 2;
template <int MODE>
__device__ __forceinline__ bool kok(const AttnArgs& a, int b, int key, int q) {
  if constexpr (MODE & AM_MASK) return key_ok(a, b, key, q);
  else return key < a.Nk;
}
template <int MODE>
__device__ __forceinline__ bool fullk(const AttnArgs& a, int kb) {
  if constexpr (MODE & AM_MASK) return full_kb(a, kb);
  else return (kb + 1) * 16 <= a.Nk;
}
template <int MODE>
constexpr bool dropm() { return (MODE & AM_DROP) != 0; }
// v_exp_f32 directly: arguments are <= 0 or -inf (-> 0); no denormal range reduction
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *(const bf16x8*)p; }
__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}
__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (bf16)a[0]; r[1] = (bf16)a[1]; r[2] = (bf16)a[2]; r[3] = (bf16)a[3];
  r[4] = (bf16)b[0]; r[5] = (bf16)b[1]; r[6] = (bf16)b[2]; r[7] = (bf16)b[3];
  return r;
}
__device__ __forceinline__ void store4(bf16* p, const f32x4& v, float s) {
  bf16x4 r;
  r[0] = (bf16)(v[0] * s); r[1] = (bf16)(v[1] * s); r[2] = (bf16)(v[2] * s); r[3] = (bf16)(v[3] * s);
  *(bf16x4*)p = r;
}
// transposed 4x16 block read: rows r0..r0+3 (lane-group local), columns c0..c0+15
__device__ __forceinline__ bf16x4 tr_read(const bf16* img, int st, int r0, int c0, int lane) {
  const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const bf16* a = img + (r0 + q) * st + c0 + 4 * p;
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, a));
}
__device__ __forceinline__ bf16x8 tr_read8(const bf16* img, int st, int r0, int c0, int lane) {
  // logical k = 8g + j  <->  rows r0 + 4g + j (j<4), r0 + 16 + 4g + (j-4) (j>=4)
  const int g = lane >> 4;
  bf16x4 x0 = tr_read(img, st, r0 + 4 * g, c0, lane);
  bf16x4 x1 = tr_read(img, st, r0 + 16 + 4 * g, c0, lane);
  bf16x8 r;
  r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
  r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
  return r;
}

// Swizzled head image (HDP 64): unpadded 128-B rows, 16-B chunk c of row r stored at chunk
// c ^ (r & 6).  Bank rule (MI355X_MICROARCH §LDS): ds_read_b128 is serviced in the 16-lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32), ds_read_b64_tr_b16 in 32-lane halves,
// 64 banks of 4 B.  Fragment reads (lane l: row l & 15, chunk 4s + (l >> 4)) and transposed
// reads (8 rows x 2 adjacent chunks per half) are both conflict-free with this mask
// (exhaustive search over XOR-linear masks of the row bits); the GEMM's c ^ ((r >> 1) & 7)
// left every transposed read 2-way conflicted (25 % of the forward kernel's LDS cycles).
// 12 % less LDS than 8-element padding: a ViT head's K/V take 52 KiB, three WGs per CU.
__device__ __forceinline__ int swz_f(int r) { return r & 6; }
__device__ __forceinline__ int swz_off(int r, int col) {
  return r * 64 + ((((col >> 3) ^ swz_f(r))) << 3) + (col & 7);
}
__device__ __forceinline__ bf16x4 tr_read_sw(const bf16* img, int r0, int c0, int lane) {
  const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, img + swz_off(r0 + q, c0 + 4 * p)));
}
// tr_read8 on a swizzled image; hi = false: the upper 16 rows lie past the image (zeros)
__device__ __forceinline__ bf16x8 tr_read8_sw(const bf16* img, int r0, int c0, int lane, bool hi) {
  const int g = lane >> 4;
  bf16x4 x0 = tr_read_sw(img, r0 + 4 * g, c0, lane);
  bf16x4 x1 = {(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
  if (hi) x1 = tr_read_sw(img, r0 + 16 + 4 * g, c0, lane);
  bf16x8 r;
  r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
  r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
  return r;
}

// Stage up to NIMG row-major [NP x HDP] head images into LDS (row stride HDP+16: 2*HDP+32 bytes
// puts both the b128 fragment reads and the transposed reads on distinct banks for HDP 32..128;
// the former +8 pad left both 2-way conflicted).
// Every global load of every image is issued before the first LDS write, so a
// workgroup pays one memory round trip for its whole staging, not one per chunk.
struct StageSrc {
  bf16* img;
  const bf16* src;  // already offset to batch b and head column h*hd
  int64_t rs;
  int n, NP;
};
template <int HDP, int NIMG, int MINTHR, bool SWZ = false>
__device__ __forceinline__ void stage_images(const StageSrc (&S)[NIMG], int hd) {
  static_assert(!SWZ || HDP == 64, "swizzled images are 64 wide");
  constexpr int NCH = HDP / 8;
  constexpr int ST = HDP + 16;
  constexpr int MAXIT = (256 * NCH + MINTHR - 1) / MINTHR;  // NP <= 256
  bf16x8 v[NIMG][MAXIT];
#pragma unroll
  for (int im = 0; im < NIMG; ++im)
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      const int c = threadIdx.x + it * blockDim.x;
      const int r = c / NCH, dc = c % NCH;
      v[im][it] = (r < S[im].n && dc * 8 < hd) ? ld8(S[im].src + (int64_t)r * S[im].rs + dc * 8) : zero8();
    }
#pragma unroll
  for (int im = 0; im < NIMG; ++im)
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      const int c = threadIdx.x + it * blockDim.x;
      const int r = c / NCH, dc = c % NCH;
      if (r < S[im].NP) *(bf16x8*)(S[im].img + (SWZ ? swz_off(r, dc * 8) : r * ST + dc * 8)) = v[im][it];
    }
}

// stage_images for any blockDim: rounds of R 16-B chunks per image per thread (all loads
// of a round issued before its LDS writes).
template <int HDP, int NIMG, bool SWZ>
__device__ __forceinline__ void stage_images_rt(const StageSrc (&S)[NIMG], int hd) {
  constexpr int NCH = HDP / 8, ST = HDP + 16, R = 4;
  int total = 0;
#pragma unroll
  for (int im = 0; im < NIMG; ++im) total = max(total, S[im].NP * NCH);
  for (int base = 0; base < total; base += R * (int)blockDim.x) {
    bf16x8 v[NIMG][R];
#pragma unroll
    for (int im = 0; im < NIMG; ++im)
#pragma unroll
      for (int it = 0; it < R; ++it) {
        const int c = base + threadIdx.x + it * blockDim.x;
        const int r = c / NCH, dc = c % NCH;
        v[im][it] = (r < S[im].n && dc * 8 < hd) ? ld8(S[im].src + (int64_t)r * S[im].rs + dc * 8) : zero8();
      }
#pragma unroll
    for (int im = 0; im < NIMG; ++im)
#pragma unroll
      for (int it = 0; it < R; ++it) {
        const int c = base + threadIdx.x + it * blockDim.x;
        const int r = c / NCH, dc = c % NCH;
        if (r < S[im].NP) *(bf16x8*)(S[im].img + (SWZ ? swz_off(r, dc * 8) : r * ST + dc * 8)) = v[im][it];
      }
  }
}

// Swizzled 64-wide head images (swz_off layout) staged by LDS DMA (global_load_lds, 16 B per
// lane): 1-KiB pieces of 8 rows; lane l of a piece writes row 8p + l/8, chunk slot l%8, which
// holds source chunk (l%8) ^ ((l/8) & 6) -- the swizzle moves to the source address, and no
// VGPR, address select or LDS store is spent on the copy.  Rows n..NP-1 read row n - 1 (the
// kernels mask or zero-weight them).  The caller waits vmcnt(0) and barriers before reading.
template <int NIMG>
__device__ __forceinline__ void stage_dma_sw(const StageSrc (&S)[NIMG], int wave, int nwaves, int lane) {
  const int rl = lane >> 3, csrc = ((lane & 7) ^ (rl & 6)) * 8;
#pragma unroll
  for (int im = 0; im < NIMG; ++im) {
    const int pieces = S[im].NP >> 3;
    for (int p = wave; p < pieces; p += nwaves) {
      const int r = min(p * 8 + rl, S[im].n - 1);
      __builtin_amdgcn_global_load_lds((const void*)(S[im].src + (int64_t)r * S[im].rs + csrc),
                                       (__attribute__((address_space(3))) void*)(S[im].img + p * 512), 16, 0, 0);
    }
  }
}

template <int HDP>
__device__ __forceinline__ void load_q_frags(const AttnArgs& a, const bf16* qsrc, int qt, int lane, bf16x8 (&qf)[HDP / 32]) {
  const int qi = qt * 16 + (lane & 15);
#pragma unroll
  for (int s = 0; s < HDP / 32; ++s) {
    const int d = s * 32 + 8 * (lane >> 4);
    qf[s] = (qi < a.Nq && d < a.hd) ? ld8(qsrc + (int64_t)qi * a.q_rs + d) : zero8();
  }
}

// One 16-query tile of the forward: S^T = K Q^T from the staged K image, online softmax over
// 32-key chunks, O^T = V^T P^T, O and lse stored.
template <int HDP, int MODE>
__device__ __forceinline__ void fwd_qtile(const AttnArgs& a, int b, int h, int qt, int lane, const bf16x8 (&qf)[HDP / 32],
                                          const bf16* Ks, const bf16* Vs, int NKP) {
  constexpr bool SW = HDP == 64;
  constexpr int ST = SW ? 64 : HDP + 16;
  const int hoff = h * a.hd;
  const float sl2 = a.scale * kLog2e;  // scores kept in the log2 domain: exp2(s*scale*log2e - max)
  // Online softmax over 32-key chunks (two 16-key S blocks = one PV MFMA step): only one
  // chunk of scores is live, so the wave stays far below 128 VGPRs and two workgroups
  // share a CU (the whole-row version held 16 score blocks and spilled).
  const int qi = qt * 16 + (lane & 15);
  // Scores are kept as t = s * sl2 - mref (log2 domain, against a per-query reference
  // mref).  The reference is set from the first chunk holding a valid key and only moves
  // when some score exceeds it by more than 8 (p = 2^t <= 256 otherwise): the common chunk
  // costs one fma + max per score and a wave ballot -- no cross-lane shuffles; the rare
  // move path reduces the chunk maximum over the query's four lane groups and rescales.
  // Without dropout the row sum l comes from the PV MFMA itself (an all-ones A operand
  // against the same bf16 P^T), so no per-score adds either.
  constexpr bool MFMA_L = !dropm<MODE>();
  bool have = false;  // the query has a reference (uniform over its lane groups)
  float mref = 0.f, l = 0.f;
  f32x4 o[HDP / 16], lacc = {0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.f;
#pragma unroll
  for (int db = 0; db < HDP / 16; ++db) o[db] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t * 32 < NKP; ++t) {
    f32x4 sc[2];
    const bool hi = (2 * t + 1) * 16 < NKP;  // the chunk's upper 16 keys are staged
    float lm = -INFINITY;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int kb = 2 * t + c;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (c == 0 || hi) {
#pragma unroll
        for (int s = 0; s < HDP / 32; ++s) {
          const int row = kb * 16 + (lane & 15), col = s * 32 + 8 * (lane >> 4);
          bf16x8 kf = *(const bf16x8*)(Ks + (SW ? swz_off(row, col) : row * ST + col));
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], acc, 0, 0, 0);
        }
      }
      if (!fullk<MODE>(a, kb)) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb * 16 + (lane >> 4) * 4 + r;
          acc[r] = kok<MODE>(a, b, key, qi) ? acc[r] : -INFINITY;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc[r] = fmaf(acc[r], sl2, -mref);
        lm = fmaxf(lm, acc[r]);
      }
      sc[c] = acc;
    }
    if (__builtin_amdgcn_ballot_w64(lm > 8.f || (!have && lm > -INFINITY))) {
      float cm = lm;
      cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
      cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
      const bool move = cm > 8.f || (!have && cm > -INFINITY);
      if (move) {  // new reference mref + cm: rescale what was accumulated against the old one
        const float alpha = have ? fexp2(-cm) : 0.f;
        mref += cm;
        have = true;
        l *= alpha;
        lacc *= alpha;
#pragma unroll
        for (int db = 0; db < HDP / 16; ++db) o[db] *= alpha;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) sc[c][r] -= cm;
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = fexp2(sc[c][r]);
        if constexpr (!MFMA_L) {
          l += p;  // the normaliser excludes dropout
          sc[c][r] = p * pdrop(a, b, h, qi, (2 * t + c) * 16 + (lane >> 4) * 4 + r);
        } else {
          sc[c][r] = p;
        }
      }
    const bf16x8 pb = pack8(sc[0], sc[1]);
#pragma unroll
    for (int db = 0; db < HDP / 16; ++db)  // O^T += V^T P^T, V^T fragments by transposed LDS reads
      o[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
          SW ? tr_read8_sw(Vs, 32 * t, db * 16, lane, hi) : tr_read8(Vs, ST, 32 * t, db * 16, lane), pb, o[db], 0, 0, 0);
    if constexpr (MFMA_L) lacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb, lacc, 0, 0, 0);
  }
  if constexpr (MFMA_L) {
    l = lacc[0];  // every row of the ones product holds the query's sum over all keys
  } else {
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
  }
  if (qi < a.Nq) {
    const float inv = 1.f / l;
    bf16* orow = (bf16*)a.out + (int64_t)b * a.out_bs + (int64_t)qi * a.out_rs + hoff;
#pragma unroll
    for (int db = 0; db < HDP / 16; ++db) {
      const int d0 = db * 16 + (lane >> 4) * 4;
      if (d0 < a.hd) store4(orow + d0, o[db], inv);
    }
    if ((lane >> 4) == 0) a.lse[((int64_t)b * a.H + h) * a.Nq + qi] = (mref + __log2f(l)) * kLn2;
  }
}

// 8 waves over the 16-query tiles; HDP 64 is held to 80 VGPRs so that three workgroups
// (52 KiB of swizzled K/V each) share a CU.  (Measured: one wave per tile -- 13-wave
// workgroups, two per CU -- 130 us vs 101 us on the ViT layer: fewer, longer-staging
// workgroups overlap less.)
template <int HDP, int MODE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(HDP == 64 ? 6 : 1))) void attn_fwd_bf16(
    AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  constexpr bool SW = HDP == 64;  // swizzled 16-row-granular images (swz_off)
  const int NKP = SW ? (a.Nk + 15) & ~15 : (a.Nk + 31) & ~31;
  constexpr int ST = SW ? 64 : HDP + 16;
  bf16* Ks = (bf16*)smem;
  bf16* Vs = Ks + NKP * ST;
  const int hoff = h * a.hd;
  const bf16* qsrc = (const bf16*)a.q + (int64_t)b * a.q_bs + hoff;
  // issue this wave's first Q tile before the K/V staging so the latencies overlap
  bf16x8 qf[HDP / 32];
  load_q_frags<HDP>(a, qsrc, wave, lane, qf);
  {
    const StageSrc S[2] = {{Ks, (const bf16*)a.k + (int64_t)b * a.k_bs + hoff, a.k_rs, a.Nk, NKP},
                           {Vs, (const bf16*)a.v + (int64_t)b * a.v_bs + hoff, a.v_rs, a.Nk, NKP}};
    if (SW && a.hd == 64 && (a.dma_stage & 1)) {
      stage_dma_sw<2>(S, wave, nwaves, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      stage_images_rt<HDP, 2, SW>(S, a.hd);
    }
  }
  __syncthreads();

  for (int qt = wave; qt * 16 < a.Nq; qt += nwaves) {
    if (qt != wave) load_q_frags<HDP>(a, qsrc, qt, lane, qf);
    fwd_qtile<HDP, MODE>(a, b, h, qt, lane, qf, Ks, Vs, NKP);
  }
}

template <int HDP, int MODE>
__global__ __launch_bounds__(512) void attn_bwd_bf16(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int NQP = (a.Nq + 31) & ~31, NKP = (a.Nk + 31) & ~31;
  constexpr int ST = HDP + 16;
  bf16* Qs = (bf16*)smem;
  bf16* dOs = Qs + NQP * ST;
  bf16* Ks = dOs + NQP * ST;
  bf16* Vs = Ks + NKP * ST;
  float* lse_s = (float*)(Vs + NKP * ST);
  float* del_s = lse_s + NQP;
  const int hoff = h * a.hd;
  {
    const StageSrc S[4] = {{Qs, (const bf16*)a.q + (int64_t)b * a.q_bs + hoff, a.q_rs, a.Nq, NQP},
                           {dOs, (const bf16*)a.dout + (int64_t)b * a.do_bs + hoff, a.do_rs, a.Nq, NQP},
                           {Ks, (const bf16*)a.k + (int64_t)b * a.k_bs + hoff, a.k_rs, a.Nk, NKP},
                           {Vs, (const bf16*)a.v + (int64_t)b * a.v_bs + hoff, a.v_rs, a.Nk, NKP}};
    stage_images<HDP, 4, 512>(S, a.hd);
  }
  // lse and delta_q = sum_d dO*O (fp32): 16-B vector loads of O, dO from LDS,
  // per-chunk partial dots -> LDS -> one thread per query sums them.
  constexpr int NCH = HDP / 8;
  float* part = del_s + NQP;  // [NQP][NCH]
  for (int q = threadIdx.x; q < NQP; q += blockDim.x)
    lse_s[q] = q < a.Nq ? a.lse_in[((int64_t)b * a.H + h) * a.Nq + q] * kLog2e : 0.f;  // log2 domain
  const float sl2 = a.scale * kLog2e;
  for (int idx = threadIdx.x; idx < NQP * NCH; idx += blockDim.x) {
    const int q = idx / NCH, c = idx % NCH;
    float s = 0.f;
    if (q < a.Nq && c * 8 < a.hd) {
      const bf16x8 ov = ld8((const bf16*)a.o + (int64_t)b * a.o_bs + (int64_t)q * a.o_rs + hoff + c * 8);
      const bf16x8 dv = *(const bf16x8*)(dOs + q * ST + c * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += (float)ov[i] * (float)dv[i];
    }
    part[idx] = s;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < NQP; q += blockDim.x) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += part[q * NCH + c];
    del_s[q] = s;
  }
  __syncthreads();

  // ---- phase A: dK, dV (waves own 16-key blocks)
  const int nwaves = blockDim.x >> 6;
  for (int kb = wave; kb < NKP / 16; kb += nwaves) {
    const int keyl = kb * 16 + (lane & 15);
    f32x4 dvt[HDP / 16], dkt[HDP / 16];
#pragma unroll
    for (int db = 0; db < HDP / 16; ++db) dvt[db] = dkt[db] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < NQP / 32; ++t) {
      f32x4 p[2], ds[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int qa = t * 32 + c * 16 + (lane & 15);
        f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < HDP / 32; ++s) {
          const int d = s * 32 + 8 * (lane >> 4);
          s_acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(Qs + qa * ST + d),
                                                          *(const bf16x8*)(Ks + keyl * ST + d), s_acc, 0, 0, 0);
          dp_acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(dOs + qa * ST + d),
                                                           *(const bf16x8*)(Vs + keyl * ST + d), dp_acc, 0, 0, 0);
        }
        const DropRun dr(dropm<MODE>() ? drop_idx(a, b, h, t * 32 + c * 16 + (lane >> 4) * 4, keyl) : 0);  // + r Nk
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = t * 32 + c * 16 + (lane >> 4) * 4 + r;
          const bool ok = q < a.Nq && (fullk<MODE>(a, kb) || kok<MODE>(a, b, keyl, q));
          const float pv = ok ? fexp2(s_acc[r] * sl2 - lse_s[q]) : 0.f;
          const float mk = dropm<MODE>() && q < a.Nq ? dr.mul(a.drop, (uint32_t)(r * a.Nk)) : 1.f;
          p[c][r] = pv * mk;
          ds[c][r] = pv * (dp_acc[r] * mk - del_s[q]);
        }
      }
      const bf16x8 pb = pack8(p[0], p[1]), dsb = pack8(ds[0], ds[1]);
#pragma unroll
      for (int db = 0; db < HDP / 16; ++db) {
        dvt[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_read8(dOs, ST, t * 32, db * 16, lane), pb, dvt[db], 0, 0, 0);
        dkt[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_read8(Qs, ST, t * 32, db * 16, lane), dsb, dkt[db], 0, 0, 0);
      }
    }
    if (keyl < a.Nk) {
      bf16* dkrow = (bf16*)a.dk + (int64_t)b * a.dk_bs + (int64_t)keyl * a.dk_rs + hoff;
      bf16* dvrow = (bf16*)a.dv + (int64_t)b * a.dv_bs + (int64_t)keyl * a.dv_rs + hoff;
#pragma unroll
      for (int db = 0; db < HDP / 16; ++db) {
        const int d0 = db * 16 + (lane >> 4) * 4;
        if (d0 < a.hd) {
          store4(dkrow + d0, dkt[db], a.scale);
          store4(dvrow + d0, dvt[db], 1.f);
        }
      }
    }
  }

  // ---- phase B: dQ (waves own 16-query blocks)
  for (int qb = wave; qb < NQP / 16; qb += nwaves) {
    const int ql = qb * 16 + (lane & 15);
    const float lq = lse_s[ql], dq_del = del_s[ql];
    f32x4 dqt[HDP / 16];
#pragma unroll
    for (int db = 0; db < HDP / 16; ++db) dqt[db] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < NKP / 32; ++t) {
      f32x4 ds[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int ka = t * 32 + c * 16 + (lane & 15);
        f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < HDP / 32; ++s) {
          const int d = s * 32 + 8 * (lane >> 4);
          s_acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(Ks + ka * ST + d),
                                                          *(const bf16x8*)(Qs + ql * ST + d), s_acc, 0, 0, 0);
          dp_acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(Vs + ka * ST + d),
                                                           *(const bf16x8*)(dOs + ql * ST + d), dp_acc, 0, 0, 0);
        }
        const DropRun dr(dropm<MODE>() ? drop_idx(a, b, h, ql, t * 32 + c * 16 + (lane >> 4) * 4) : 0);  // + r
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = t * 32 + c * 16 + (lane >> 4) * 4 + r;
          const bool ok = ql < a.Nq && (fullk<MODE>(a, 2 * t + c) || kok<MODE>(a, b, key, ql));
          const float pv = ok ? fexp2(s_acc[r] * sl2 - lq) : 0.f;
          const float mk = dropm<MODE>() && ok ? dr.mul(a.drop, r) : 1.f;
          ds[c][r] = pv * (dp_acc[r] * mk - dq_del);
        }
      }
      const bf16x8 dsb = pack8(ds[0], ds[1]);
#pragma unroll
      for (int db = 0; db < HDP / 16; ++db)
        dqt[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_read8(Ks, ST, t * 32, db * 16, lane), dsb, dqt[db], 0, 0, 0);
    }
    if (ql < a.Nq) {
      bf16* dqrow = (bf16*)a.dq + (int64_t)b * a.dq_bs + (int64_t)ql * a.dq_rs + hoff;
#pragma unroll
      for (int db = 0; db < HDP / 16; ++db) {
        const int d0 = db * 16 + (lane >> 4) * 4;
        if (d0 < a.hd) store4(dqrow + d0, dqt[db], a.scale);
      }
    }
  }
}

// Backward split in two kernels so that each holds only two head images in LDS (two
// workgroups per CU instead of one): dK/dV with Q, dO staged and the wave's own K/V rows
// in registers; dQ with K, V staged and the wave's own Q/dO rows in registers.  Same
// arithmetic as attn_bwd_bf16 phases A and B (which remains for reference shapes that
// do not fit this split's launch checks).
// BIAS: also the per-image column sums of dQ (AttnArgs::dbias_part), as
// sum_k dQ[k, :] = scale * sum_k (sum_q dS[q, k]) K[k, :]: the per-key sums of the dS this
// kernel forms anyway go to LDS, then one pass over the head's K rows (L2-resident).
template <int HDP, int WPE, int MODE, bool BIAS = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE))) void attn_bwd_kv_bf16(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const int NQP = (a.Nq + 31) & ~31, NKP = (a.Nk + 31) & ~31;
  constexpr bool SW = HDP == 64;  // swizzled Q / dO images (swz_off)
  constexpr int ST = SW ? 64 : HDP + 16;
  constexpr int NCH = HDP / 8;
  bf16* Qs = (bf16*)smem;
  bf16* dOs = Qs + NQP * ST;
  float* lse_s = (float*)(dOs + NQP * ST);
  float* del_s = lse_s + NQP;
  const int hoff = h * a.hd;
  const bf16* kbase = (const bf16*)a.k + (int64_t)b * a.k_bs + hoff;
  const bf16* vbase = (const bf16*)a.v + (int64_t)b * a.v_bs + hoff;
  // the wave's own K / V rows; the next key block's are loaded while this one computes
  auto load_rows = [&](int kb, bf16x8 (&kf)[HDP / 32], bf16x8 (&vf)[HDP / 32]) {
    const int keyl = kb * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < HDP / 32; ++s) {
      const int d = s * 32 + 8 * (lane >> 4);
      const bool in = keyl < a.Nk && d < a.hd;
      kf[s] = in ? ld8(kbase + (int64_t)keyl * a.k_rs + d) : zero8();
      vf[s] = in ? ld8(vbase + (int64_t)keyl * a.v_rs + d) : zero8();
    }
  };
  // Prologue: every global load of the workgroup's set-up -- the first key block's K / V
  // rows, lse, the O chunks of delta and the Q / dO staging -- is issued before the first
  // wait, so the workgroup pays one memory round trip instead of three (stage, then O,
  // then K / V).  8 lanes per query for delta (chunks c8, c8 + 8, ...); NQP * 8 is a
  // multiple of 64, so every wave runs whole iterations (shuffles see all lanes).
  bf16x8 kf[HDP / 32], vf[HDP / 32];
  if (wave < NKP / 16) load_rows(wave, kf, vf);
  const float lse_r = threadIdx.x < a.Nq ? a.lse_in[((int64_t)b * a.H + h) * a.Nq + threadIdx.x] * kLog2e : 0.f;
  constexpr int DIT = (256 * 8 + 511) / 512, DCH = (NCH + 7) / 8;  // NQP <= 256, blockDim 512
  bf16x8 ov[DIT][DCH];
#pragma unroll
  for (int it = 0; it < DIT; ++it)
#pragma unroll
    for (int j = 0; j < DCH; ++j) {
      const int idx = threadIdx.x + it * 512, q = idx >> 3, c = (idx & 7) + 8 * j;
      ov[it][j] = (q < a.Nq && c < NCH && c * 8 < a.hd)
                      ? ld8((const bf16*)a.o + (int64_t)b * a.o_bs + (int64_t)q * a.o_rs + hoff + c * 8)
                      : zero8();
    }
  {
    const StageSrc S[2] = {{Qs, (const bf16*)a.q + (int64_t)b * a.q_bs + hoff, a.q_rs, a.Nq, NQP},
                           {dOs, (const bf16*)a.dout + (int64_t)b * a.do_bs + hoff, a.do_rs, a.Nq, NQP}};
    if (SW && a.hd == 64 && (a.dma_stage & 4)) {  // rows Nq..NQP-1 repeat row Nq-1: P = dS = 0 there
      stage_dma_sw<2>(S, wave, nwaves, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      stage_images<HDP, 2, 512, SW>(S, a.hd);
    }
  }
  if (threadIdx.x < NQP) lse_s[threadIdx.x] = lse_r;  // log2 domain
  float* ksum_s = del_s + NQP;  // BIAS: [NKP] sum_q dS[q, key]
  __syncthreads();
#pragma unroll
  for (int it = 0; it < DIT; ++it) {
    const int idx = threadIdx.x + it * 512, q = idx >> 3;
    if (it * 512 >= NQP * 8) break;  // uniform over the block
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < DCH; ++j) {
      const int c = (idx & 7) + 8 * j;
      if (q < NQP && c < NCH) {
        const bf16x8 dv = *(const bf16x8*)(dOs + (SW ? swz_off(q, c * 8) : q * ST + c * 8));
#pragma unroll
        for (int i = 0; i < 8; ++i) s += (float)ov[it][j][i] * (float)dv[i];
      }
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if ((idx & 7) == 0 && q < NQP) del_s[q] = s;
  }
  __syncthreads();
  // delta for the dQ kernel, which then needs no O: stashed as fp32 in the first 4 bytes of
  // each (image, query, head) slot of dQ, which that kernel reads before overwriting it
  for (int q = threadIdx.x; q < a.Nq; q += blockDim.x)
    *(float*)((bf16*)a.dq + (int64_t)b * a.dq_bs + (int64_t)q * a.dq_rs + hoff) = del_s[q];
  const float sl2 = a.scale * kLog2e;
  for (int kb = wave; kb < NKP / 16; kb += nwaves) {
    const int keyl = kb * 16 + (lane & 15);
    bf16x8 kn[HDP / 32], vn[HDP / 32];
    if (kb + nwaves < NKP / 16) load_rows(kb + nwaves, kn, vn);
    f32x4 dvt[HDP / 16], dkt[HDP / 16];
#pragma unroll
    for (int db = 0; db < HDP / 16; ++db) dvt[db] = dkt[db] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float dsum = 0.f;  // BIAS: this lane's share of sum_q dS[q, key]
    for (int t = 0; t < NQP / 32; ++t) {
      f32x4 p[2], ds[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int qa = t * 32 + c * 16 + (lane & 15);
        f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < HDP / 32; ++s) {
          const int d = s * 32 + 8 * (lane >> 4);
          const int qo = SW ? swz_off(qa, d) : qa * ST + d;
          s_acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(Qs + qo), kf[s], s_acc, 0, 0, 0);
          dp_acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(dOs + qo), vf[s], dp_acc, 0, 0, 0);
        }
        const DropRun dr(dropm<MODE>() ? drop_idx(a, b, h, t * 32 + c * 16 + (lane >> 4) * 4, keyl) : 0);  // + r Nk
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = t * 32 + c * 16 + (lane >> 4) * 4 + r;
          const bool ok = q < a.Nq && (fullk<MODE>(a, kb) || kok<MODE>(a, b, keyl, q));
          const float pv = ok ? fexp2(s_acc[r] * sl2 - lse_s[q]) : 0.f;
          const float mk = dropm<MODE>() && q < a.Nq ? dr.mul(a.drop, (uint32_t)(r * a.Nk)) : 1.f;
          p[c][r] = pv * mk;
          ds[c][r] = pv * (dp_acc[r] * mk - del_s[q]);
          if constexpr (BIAS) dsum += ds[c][r];
        }
      }
      const bf16x8 pb = pack8(p[0], p[1]), dsb = pack8(ds[0], ds[1]);
#pragma unroll
      for (int db = 0; db < HDP / 16; ++db) {
        const bf16x8 dot = SW ? tr_read8_sw(dOs, t * 32, db * 16, lane, true) : tr_read8(dOs, ST, t * 32, db * 16, lane);
        const bf16x8 qt = SW ? tr_read8_sw(Qs, t * 32, db * 16, lane, true) : tr_read8(Qs, ST, t * 32, db * 16, lane);
        dvt[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dot, pb, dvt[db], 0, 0, 0);
        dkt[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qt, dsb, dkt[db], 0, 0, 0);
      }
    }
    if (keyl < a.Nk) {
      bf16* dkrow = (bf16*)a.dk + (int64_t)b * a.dk_bs + (int64_t)keyl * a.dk_rs + hoff;
      bf16* dvrow = (bf16*)a.dv + (int64_t)b * a.dv_bs + (int64_t)keyl * a.dv_rs + hoff;
#pragma unroll
      for (int db = 0; db < HDP / 16; ++db) {
        const int d0 = db * 16 + (lane >> 4) * 4;
        if (d0 < a.hd) {
          store4(dkrow + d0, dkt[db], a.scale);
          store4(dvrow + d0, dvt[db], 1.f);
        }
      }
    }
    if constexpr (BIAS) {  // (keys past Nk: zeros)
      dsum += __shfl_xor(dsum, 16, 64);
      dsum += __shfl_xor(dsum, 32, 64);
      if (lane < 16) ksum_s[keyl] = dsum;
    }
#pragma unroll
    for (int s = 0; s < HDP / 32; ++s) {
      kf[s] = kn[s];
      vf[s] = vn[s];
    }
  }
  if constexpr (BIAS) {  // dQ column sums: G key-strided partials per column, then summed in order
    __syncthreads();  // ksum_s complete; the Q image is free for the partials
    constexpr int G = 512 / HDP;
    float* part = (float*)smem;  // [G][HDP]
    const int g = threadIdx.x / HDP, d = threadIdx.x % HDP;
    if (g < G) {
      float t = 0.f;
      if (d < a.hd)
        for (int k = g; k < a.Nk; k += G) t += ksum_s[k] * (float)kbase[(int64_t)k * a.k_rs + d];
      part[g * HDP + d] = t;
    }
    __syncthreads();
    if (threadIdx.x < a.hd) {
      float t = 0.f;
#pragma unroll
      for (int g2 = 0; g2 < G; ++g2) t += part[g2 * HDP + threadIdx.x];
      a.dbias_part[(int64_t)b * a.dbias_ld + hoff + threadIdx.x] = t * a.scale;
    }
  }
}

// Fused single-pass backward for 64-wide heads (the ViT layers, N = 197): one workgroup per
// (image, head) with one wave per 16-key block (13 for N = 197, up to 16) holds Q, dO and K in
// LDS (LDS-DMA), forms P and dS once per (query, key) and produces dK, dV and dQ.  The split
// pair (attn_bwd_kv_bf16 + attn_bwd_q_bf16) formed P and dS twice and read every operand twice.
//  * key waves: the attn_bwd_kv_bf16 loop over 32-query chunks (their K / V rows in registers,
//    dV += dO^T P, dK += Q^T dS in registers), and each chunk's dS^T block goes to an LDS
//    image [keys][32 queries] (double-buffered, one barrier per chunk);
//  * after the barrier, waves 0-7 each form one 16 x 16 block of the chunk's dQ^T = K^T dS^T
//    over all keys (transposed reads of the K image and of the dS^T image, the same key order
//    on both sides) and store it -- every key has contributed, so no dQ accumulator survives
//    the chunk.
// Same expressions as the split pair (P, dS, delta, masks, dropout index).  Requires hd == 64,
// NKP = Nk rounded to 16 <= 256, LDS (2 NQP + NKP) x 128 B + the dS^T images <= 160 KiB.
// BIAS (round 6): also the per-(image, head) column sums of the dQ, dK and dV it stores (the
// bf16 values, summed in fp32 in a fixed order) into AttnArgs::dbias_part [B][3 H 64]: the QKV
// bias gradient of the fused projection without a column-sum pass over the 232 MB dQKV.
template <int MODE, bool BIAS = false>
__global__ __launch_bounds__(1024) void attn_bwd_fused64(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int HDP = 64, DSST = 48;  // dS^T image row stride: 32 queries + 16 (conflict-free transposed reads)
  const int b = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int NQP = (a.Nq + 31) & ~31, NKP = (a.Nk + 15) & ~15, NKB = NKP / 16, NKC = (NKP + 31) / 32;
  bf16* Qs = (bf16*)smem;      // [NQP][64], swz_off layout
  bf16* dOs = Qs + NQP * 64;   // [NQP][64]
  bf16* Ks = dOs + NQP * 64;   // [NKP][64]
  bf16* dST = Ks + NKP * 64;   // [2][NKC * 32][DSST]
  const int DSB = NKC * 32 * DSST;
  float* lse_s = (float*)(dST + 2 * DSB);
  float* del_s = lse_s + NQP;
  const int hoff = h * HDP;
  const bool kw = wave < NKB;  // a key wave: key block kb = wave
  const int kb = wave, keyl = kb * 16 + i16;
  const bf16* kbase = (const bf16*)a.k + (int64_t)b * a.k_bs + hoff;
  const bf16* vbase = (const bf16*)a.v + (int64_t)b * a.v_bs + hoff;
  // ---- prologue: the wave's K / V rows, lse, O rows for delta, and the Q / dO / K images by DMA
  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int d = s * 32 + 8 * g;
    const bool in = kw && keyl < a.Nk;
    kf[s] = in ? ld8(kbase + (int64_t)keyl * a.k_rs + d) : zero8();
    vf[s] = in ? ld8(vbase + (int64_t)keyl * a.v_rs + d) : zero8();
  }
  const float lse_r = threadIdx.x < a.Nq ? a.lse_in[((int64_t)b * a.H + h) * a.Nq + threadIdx.x] * kLog2e : 0.f;
  bf16x8 ov[2];  // 8 lanes per query, 8 dims each: queries threadIdx.x / 8 (+ 128 per pass)
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = threadIdx.x + it * (int)blockDim.x, q = idx >> 3, c = idx & 7;
    ov[it] = q < a.Nq ? ld8((const bf16*)a.o + (int64_t)b * a.o_bs + (int64_t)q * a.o_rs + hoff + c * 8) : zero8();
  }
  {
    const StageSrc S[3] = {{Qs, (const bf16*)a.q + (int64_t)b * a.q_bs + hoff, a.q_rs, a.Nq, NQP},
                           {dOs, (const bf16*)a.dout + (int64_t)b * a.do_bs + hoff, a.do_rs, a.Nq, NQP},
                           {Ks, kbase, a.k_rs, a.Nk, NKP}};
    stage_dma_sw<3>(S, wave, nwaves, lane);
  }
  // dS^T rows past NKP are read by the last key chunk's transposed reads: zero, both buffers
  for (int e = threadIdx.x; e < 2 * (NKC * 32 - NKP) * DSST; e += blockDim.x) {
    const int bi = e / ((NKC * 32 - NKP) * DSST), rem = e - bi * (NKC * 32 - NKP) * DSST;
    dST[bi * DSB + NKP * DSST + rem] = (bf16)0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // lse and delta for EVERY padded query row q < NQP (rows past Nq: 0), whatever blockDim is:
  // the key waves read lse_s / del_s of the padded rows too (ds = 0 * (dp - del_s[q]) there,
  // so a stale LDS word would turn into NaN)
  for (int q = threadIdx.x; q < NQP; q += blockDim.x)
    lse_s[q] = q == (int)threadIdx.x ? lse_r : (q < a.Nq ? a.lse_in[((int64_t)b * a.H + h) * a.Nq + q] * kLog2e : 0.f);
  for (int it = 0; it * (int)blockDim.x < NQP * 8; ++it) {  // delta = rowsum(dO * O), the attn_bwd_kv_bf16 order
    const int idx = threadIdx.x + it * (int)blockDim.x, q = idx >> 3, c = idx & 7;
    // (uniform loop bound over the block: every wave runs whole iterations for the shuffles)
    const bf16x8 o8 = it == 0 ? ov[0] : it == 1 ? ov[1]
                    : (q < a.Nq ? ld8((const bf16*)a.o + (int64_t)b * a.o_bs + (int64_t)q * a.o_rs + hoff + c * 8) : zero8());
    float sum = 0.f;
    if (q < NQP) {
      const bf16x8 dv = *(const bf16x8*)(dOs + swz_off(q, c * 8));
#pragma unroll
      for (int i = 0; i < 8; ++i) sum += (float)o8[i] * (float)dv[i];
    }
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    sum += __shfl_xor(sum, 4, 64);
    if (c == 0 && q < NQP) del_s[q] = sum;
  }
  __syncthreads();
  const float sl2 = a.scale * kLog2e;
  f32x4 dvt[4], dkt[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) dvt[db] = dkt[db] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 qsum = {0.f, 0.f, 0.f, 0.f};  // BIAS: this lane's query column of the stored dQ, over the chunks
  // the key waves' LDS element offsets at chunk 0: the swizzle reads row bits 1-2 only, which a
  // chunk's 32 rows and a 16-row half leave alone, so chunk t is + t * 2048 and the upper half
  // + 1024 (swz_off / tr_read8_sw values, without their per-read address arithmetic)
  int fo[2], tro[4];
#pragma unroll
  for (int s = 0; s < 2; ++s) fo[s] = swz_off(i16, s * 32 + 8 * g);
#pragma unroll
  for (int db = 0; db < 4; ++db) tro[db] = swz_off(4 * g + (i16 >> 2), db * 16 + 4 * (i16 & 3));
  auto tr8 = [](const bf16* p) -> bf16x8 {  // tr_read8_sw at a precomputed offset (both halves)
    const bf16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, p));
    const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4, p + 1024));
    bf16x8 r;
    r[0] = x0[0]; r[1] = x0[1]; r[2] = x0[2]; r[3] = x0[3];
    r[4] = x1[0]; r[5] = x1[1]; r[6] = x1[2]; r[7] = x1[3];
    return r;
  };
  for (int t = 0; t < NQP / 32; ++t) {
    bf16* dsi = dST + (t & 1) * DSB;
    if (kw) {
      const bf16* Qt = Qs + t * 2048;
      const bf16* dOt = dOs + t * 2048;
      f32x4 p[2], ds[2], s_acc[2], dp_acc[2], l4[2], d4[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        s_acc[c] = dp_acc[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          s_acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(Qt + c * 1024 + fo[s]), kf[s], s_acc[c], 0, 0, 0);
          dp_acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(dOt + c * 1024 + fo[s]), vf[s], dp_acc[c], 0, 0, 0);
        }
        // lse / delta of the lane's 4 queries (one 16-B read each)
        l4[c] = *(const f32x4*)(lse_s + t * 32 + c * 16 + 4 * g);
        d4[c] = *(const f32x4*)(del_s + t * 32 + c * 16 + 4 * g);
      }
      // P and dS without branches: exp2 of every entry, masked entries selected to 0 afterwards
      // (the same values); a chunk of 32 real queries against a full key block (no dropout)
      // takes the form without any mask
      if (!dropm<MODE>() && t * 32 + 32 <= a.Nq && fullk<MODE>(a, kb)) {
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = fexp2(s_acc[c][r] * sl2 - l4[c][r]);
            p[c][r] = e;
            ds[c][r] = e * (dp_acc[c][r] - d4[c][r]);
          }
      } else {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const DropRun dr(dropm<MODE>() ? drop_idx(a, b, h, t * 32 + c * 16 + g * 4, keyl) : 0);  // + r Nk
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int q = t * 32 + c * 16 + g * 4 + r;
            const bool ok = q < a.Nq && (fullk<MODE>(a, kb) || kok<MODE>(a, b, keyl, q));
            const float e = fexp2(s_acc[c][r] * sl2 - l4[c][r]);
            const float pv = ok ? e : 0.f;
            const float mk = dropm<MODE>() && q < a.Nq ? dr.mul(a.drop, (uint32_t)(r * a.Nk)) : 1.f;
            p[c][r] = pv * mk;
            ds[c][r] = pv * (dp_acc[c][r] * mk - d4[c][r]);
          }
        }
      }
      const bf16x8 pb = pack8(p[0], p[1]), dsb = pack8(ds[0], ds[1]);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16x8 dot = tr8(dOt + tro[db]);
        const bf16x8 qt = tr8(Qt + tro[db]);
        dvt[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dot, pb, dvt[db], 0, 0, 0);
        dkt[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qt, dsb, dkt[db], 0, 0, 0);
      }
      // this key row's dS for the chunk's queries c * 16 + 4g .. + 3 (the bf16 values dK used)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        bf16x4 w;
        w[0] = dsb[4 * c + 0]; w[1] = dsb[4 * c + 1]; w[2] = dsb[4 * c + 2]; w[3] = dsb[4 * c + 3];
        *(bf16x4*)(dsi + keyl * DSST + c * 16 + 4 * g) = w;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the chunk's dS^T image is complete
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (wave < 8) {  // dQ^T block (dims db * 16.., queries qb * 16..) of the chunk, over every key
      const int qb = wave >> 2, db = wave & 3;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (NKC == 7) {  // the ViT shape (N = 197): transposed reads four key chunks ahead of the MFMA chain
        bf16x8 kt[4], dst[4];
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
          kt[kc] = tr_read8_sw(Ks, kc * 32, db * 16, lane, true);
          dst[kc] = tr_read8(dsi, DSST, kc * 32, qb * 16, lane);
        }
#pragma unroll
        for (int kc = 0; kc < 7; ++kc) {
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt[kc & 3], dst[kc & 3], acc, 0, 0, 0);
          if (kc + 4 < 7) {
            kt[kc & 3] = tr_read8_sw(Ks, (kc + 4) * 32, db * 16, lane, (kc + 4) * 32 + 16 < NKP);
            dst[kc & 3] = tr_read8(dsi, DSST, (kc + 4) * 32, qb * 16, lane);
          }
        }
      } else {
        for (int kc = 0; kc < NKC; ++kc) {
          const bool hi = kc * 32 + 16 < NKP;
          const bf16x8 kt = tr_read8_sw(Ks, kc * 32, db * 16, lane, hi);
          const bf16x8 dst = tr_read8(dsi, DSST, kc * 32, qb * 16, lane);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt, dst, acc, 0, 0, 0);
        }
      }
      const int q = t * 32 + qb * 16 + i16;
      if (q < a.Nq) store4((bf16*)a.dq + (int64_t)b * a.dq_bs + (int64_t)q * a.dq_rs + hoff + db * 16 + 4 * g, acc, a.scale);
      if constexpr (BIAS) {
#pragma unroll
        for (int r = 0; r < 4; ++r) qsum[r] += q < a.Nq ? (float)(bf16)(acc[r] * a.scale) : 0.f;
      }
    }
  }
  if constexpr (BIAS) {
    // per wave: the sums over its 16 lanes of a row group (keys of a key wave, queries of a dQ
    // wave) by xor shuffles, then per dimension over the waves in wave order through LDS.  The
    // partials overwrite the Q image, which no wave reads once it has passed the last chunk's
    // barrier (the dQ phase reads K and dS^T only); the barrier below waits for LDS only, not
    // for the dQ stores in flight, and the dK / dV stores are issued after it.
    float* kpart = (float*)smem;      // [16 waves][64] dK sums
    float* vpart = kpart + 16 * 64;   // [16][64] dV sums
    float* qpart = vpart + 16 * 64;   // [2 query blocks][64] dQ sums
    auto lanesum = [](float v) {
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      return v;
    };
    if (kw) {
      const bool in = keyl < a.Nk;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float ks = lanesum(in ? (float)(bf16)(dkt[db][r] * a.scale) : 0.f);
          const float vs = lanesum(in ? (float)(bf16)dvt[db][r] : 0.f);
          if (i16 == 0) {
            kpart[wave * 64 + db * 16 + 4 * g + r] = ks;
            vpart[wave * 64 + db * 16 + 4 * g + r] = vs;
          }
        }
    }
    if (wave < 8) {
      const int qb = wave >> 2, db = wave & 3;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float qs = lanesum(qsum[r]);
        if (i16 == 0) qpart[qb * 64 + db * 16 + 4 * g + r] = qs;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (threadIdx.x < 64) {
      const int d = threadIdx.x;
      float ks = 0.f, vs = 0.f;
      for (int w = 0; w < NKB; ++w) {
        ks += kpart[w * 64 + d];
        vs += vpart[w * 64 + d];
      }
      float* out = a.dbias_part + (int64_t)b * a.dbias_ld + hoff + d;
      const int64_t D = (int64_t)a.H * 64;
      out[0] = qpart[d] + qpart[64 + d];
      out[D] = ks;
      out[2 * D] = vs;
    }
  }
  if (kw && keyl < a.Nk) {
    bf16* dkrow = (bf16*)a.dk + (int64_t)b * a.dk_bs + (int64_t)keyl * a.dk_rs + hoff;
    bf16* dvrow = (bf16*)a.dv + (int64_t)b * a.dv_bs + (int64_t)keyl * a.dv_rs + hoff;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int d0 = db * 16 + g * 4;
      store4(dkrow + d0, dkt[db], a.scale);
      store4(dvrow + d0, dvt[db], 1.f);
    }
  }
}

// dQ kernel; HDP 64: swizzled 16-row K/V images and <= 80 VGPRs (three workgroups per CU),
// as the forward kernel.
// BIAS: also the per-image column sums of dK and dV (AttnArgs::dbias_part), as
// sum_k dK[k, :] = scale * sum_q (sum_k dS[q, k]) Q[q, :] and sum_k dV[k, :] =
// sum_q (sum_k P~[q, k]) dO[q, :]: per-query sums of the dS / dropped-P rows this kernel forms
// go to the rsum scratch, then one pass over the head's Q and dO rows (L2-resident).
template <int HDP, int MODE, bool BIAS = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(HDP == 64 ? 6 : 1))) void attn_bwd_q_bf16(
    AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  constexpr bool SW = HDP == 64;
  const int NQP = (a.Nq + 31) & ~31, NKP = SW ? (a.Nk + 15) & ~15 : (a.Nk + 31) & ~31;
  constexpr int ST = SW ? 64 : HDP + 16;
  bf16* Ks = (bf16*)smem;
  bf16* Vs = Ks + NKP * ST;
  const int hoff = h * a.hd;
  const bf16* qbase = (const bf16*)a.q + (int64_t)b * a.q_bs + hoff;
  const bf16* dobase = (const bf16*)a.dout + (int64_t)b * a.do_bs + hoff;
  const bf16* dqbase = (const bf16*)a.dq + (int64_t)b * a.dq_bs + hoff;
  // the wave's query block operands: Q, dO rows (fragment layout), lse and delta_q =
  // sum_d dO * O (from the dK/dV kernel, stashed in this query's dQ slot)
  bf16x8 qf[HDP / 32], dof[HDP / 32];
  float lq = 0.f, dd = 0.f;
  auto load_q = [&](int qb) {
    const int ql = qb * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < HDP / 32; ++s) {
      const int d = s * 32 + 8 * (lane >> 4);
      const bool in = ql < a.Nq && d < a.hd;
      qf[s] = in ? ld8(qbase + (int64_t)ql * a.q_rs + d) : zero8();
      dof[s] = in ? ld8(dobase + (int64_t)ql * a.do_rs + d) : zero8();
    }
    lq = ql < a.Nq ? a.lse_in[((int64_t)b * a.H + h) * a.Nq + ql] * kLog2e : 0.f;
    dd = ql < a.Nq ? *(const float*)(dqbase + (int64_t)ql * a.dq_rs) : 0.f;
  };
  // the first block's Q / dO / lse / delta are requested before the K / V staging
  if (wave < NQP / 16) load_q(wave);
  {
    const StageSrc S[2] = {{Ks, (const bf16*)a.k + (int64_t)b * a.k_bs + hoff, a.k_rs, a.Nk, NKP},
                           {Vs, (const bf16*)a.v + (int64_t)b * a.v_bs + hoff, a.v_rs, a.Nk, NKP}};
    if (SW && a.hd == 64 && (a.dma_stage & 2)) {
      stage_dma_sw<2>(S, wave, nwaves, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      stage_images_rt<HDP, 2, SW>(S, a.hd);
    }
  }
  __syncthreads();
  const float sl2 = a.scale * kLog2e;
  for (int qb = wave; qb < NQP / 16; qb += nwaves) {
    const int ql = qb * 16 + (lane & 15);
    if (qb != wave) load_q(qb);
    f32x4 dqt[HDP / 16];
#pragma unroll
    for (int db = 0; db < HDP / 16; ++db) dqt[db] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float dsr = 0.f, pr = 0.f;  // BIAS: this lane's share of sum_k dS[ql, k], sum_k P~[ql, k]
    for (int t = 0; t * 32 < NKP; ++t) {
      f32x4 ds[2];
      const bool hi = (2 * t + 1) * 16 < NKP;  // the chunk's upper 16 keys are staged
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int ka = t * 32 + c * 16 + (lane & 15);
        f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = {0.f, 0.f, 0.f, 0.f};
        if (c == 0 || hi) {
#pragma unroll
          for (int s = 0; s < HDP / 32; ++s) {
            const int d = s * 32 + 8 * (lane >> 4);
            const int ko = SW ? swz_off(ka, d) : ka * ST + d;
            s_acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(Ks + ko), qf[s], s_acc, 0, 0, 0);
            dp_acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(Vs + ko), dof[s], dp_acc, 0, 0, 0);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = t * 32 + c * 16 + (lane >> 4) * 4 + r;
          const bool ok = ql < a.Nq && (fullk<MODE>(a, 2 * t + c) || kok<MODE>(a, b, key, ql));
          const float pv = ok ? fexp2(s_acc[r] * sl2 - lq) : 0.f;
          const float mk = dropm<MODE>() && ok ? pdrop(a, b, h, ql, key) : 1.f;
          ds[c][r] = pv * (dp_acc[r] * mk - dd);
          if constexpr (BIAS) {
            dsr += ds[c][r];
            pr += pv * mk;
          }
        }
      }
      const bf16x8 dsb = pack8(ds[0], ds[1]);
#pragma unroll
      for (int db = 0; db < HDP / 16; ++db)
        dqt[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            SW ? tr_read8_sw(Ks, t * 32, db * 16, lane, hi) : tr_read8(Ks, ST, t * 32, db * 16, lane), dsb, dqt[db], 0, 0, 0);
    }
    if (ql < a.Nq) {
      bf16* dqrow = (bf16*)a.dq + (int64_t)b * a.dq_bs + (int64_t)ql * a.dq_rs + hoff;
#pragma unroll
      for (int db = 0; db < HDP / 16; ++db) {
        const int d0 = db * 16 + (lane >> 4) * 4;
        if (d0 < a.hd) store4(dqrow + d0, dqt[db], a.scale);
      }
    }
    if constexpr (BIAS) {
      dsr += __shfl_xor(dsr, 16, 64);
      dsr += __shfl_xor(dsr, 32, 64);
      pr += __shfl_xor(pr, 16, 64);
      pr += __shfl_xor(pr, 32, 64);
      float* rs = a.rsum + (int64_t)blockIdx.x * 2 * a.Nq;
      if (lane < 16 && ql < a.Nq) {
        rs[ql] = dsr;
        rs[a.Nq + ql] = pr;
      }
    }
  }
  if constexpr (BIAS) {  // dK | dV column sums: G query-strided partials per column, then summed in order
    __syncthreads();  // rsum rows visible to the workgroup; the K / V images are free for the partials
    constexpr int NC = 2 * HDP, G = 512 / NC;
    const float* rs = a.rsum + (int64_t)blockIdx.x * 2 * a.Nq;
    float* part = (float*)smem;  // [G][NC]
    const int g = threadIdx.x / NC, col = threadIdx.x % NC, kind = col / HDP, d = col % HDP;
    if (g < G) {
      float t = 0.f;
      if (d < a.hd) {
        const bf16* x = kind ? dobase : qbase;
        const int64_t xrs = kind ? a.do_rs : a.q_rs;
        for (int q = g; q < a.Nq; q += G) t += rs[kind * a.Nq + q] * (float)x[(int64_t)q * xrs + d];
      }
      part[g * NC + col] = t;
    }
    __syncthreads();
    if (threadIdx.x < NC) {
      const int kd = threadIdx.x / HDP, dd2 = threadIdx.x % HDP;
      if (dd2 < a.hd) {
        float t = 0.f;
#pragma unroll
        for (int g2 = 0; g2 < G; ++g2) t += part[g2 * NC + threadIdx.x];
        a.dbias_part[(int64_t)b * a.dbias_ld + (int64_t)(1 + kd) * a.H * a.hd + hoff + dd2] = kd ? t : t * a.scale;
      }
    }
  }
}

// ------------------------------------------------------------ f32 parity path
template <int HD>
__global__ __launch_bounds__(64) void attn_fwd_f32(AttnArgs a) {
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int q = blockIdx.y * 64 + threadIdx.x;
  if (q >= a.Nq) return;
  const int hoff = h * HD;
  const float* qr = (const float*)a.q + (int64_t)b * a.q_bs + (int64_t)q * a.q_rs + hoff;
  float qv[HD], o[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) { qv[d] = qr[d]; o[d] = 0.f; }
  auto krow = [&](int j) { return (const float*)a.k + kv_row(a, b, j) * a.k_bs + hoff + (int64_t)j * a.k_rs; };
  auto vrow = [&](int j) { return (const float*)a.v + kv_row(a, b, j) * a.v_bs + hoff + (int64_t)j * a.v_rs; };
  float mx = -INFINITY;
  for (int j = 0; j < a.Nk; ++j) {
    if (!key_ok(a, b, j, q)) continue;
    const float* kr = krow(j);
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) s += qv[d] * kr[d];
    mx = fmaxf(mx, s * a.scale);
  }
  float l = 0.f;
  for (int j = 0; j < a.Nk; ++j) {
    if (!key_ok(a, b, j, q)) continue;
    const float* kr = krow(j);
    const float* vr = vrow(j);
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) s += qv[d] * kr[d];
    const float p = expf(s * a.scale - mx);
    l += p;
    const float pd = a.drop.on() ? p * pdrop(a, b, h, q, j) : p;
#pragma unroll
    for (int d = 0; d < HD; ++d) o[d] += pd * vr[d];
  }
  float* orow = (float*)a.out + (int64_t)b * a.out_bs + (int64_t)q * a.out_rs + hoff;
#pragma unroll
  for (int d = 0; d < HD; ++d) orow[d] = o[d] / l;
  a.lse[((int64_t)b * a.H + h) * a.Nq + q] = mx + logf(l);
}

template <int HD>
__global__ __launch_bounds__(64) void attn_bwd_dq_f32(AttnArgs a) {
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int q = blockIdx.y * 64 + threadIdx.x;
  if (q >= a.Nq) return;
  const int hoff = h * HD;
  const float* qr = (const float*)a.q + (int64_t)b * a.q_bs + (int64_t)q * a.q_rs + hoff;
  const float* orow = (const float*)a.o + (int64_t)b * a.o_bs + (int64_t)q * a.o_rs + hoff;
  const float* dorow = (const float*)a.dout + (int64_t)b * a.do_bs + (int64_t)q * a.do_rs + hoff;
  const float* kb = (const float*)a.k + (int64_t)b * a.k_bs + hoff;
  const float* vb = (const float*)a.v + (int64_t)b * a.v_bs + hoff;
  float qv[HD], dov[HD], dq[HD];
  float del = 0.f;
#pragma unroll
  for (int d = 0; d < HD; ++d) { qv[d] = qr[d]; dov[d] = dorow[d]; dq[d] = 0.f; del += dov[d] * orow[d]; }
  const float lse = a.lse_in[((int64_t)b * a.H + h) * a.Nq + q];
  for (int j = 0; j < a.Nk; ++j) {
    if (!key_ok(a, b, j, q)) continue;
    float s = 0.f, dp = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) {
      s += qv[d] * kb[(int64_t)j * a.k_rs + d];
      dp += dov[d] * vb[(int64_t)j * a.v_rs + d];
    }
    const float p = expf(s * a.scale - lse);
    const float mk = a.drop.on() ? pdrop(a, b, h, q, j) : 1.f;
    const float ds = p * (dp * mk - del);
#pragma unroll
    for (int d = 0; d < HD; ++d) dq[d] += ds * kb[(int64_t)j * a.k_rs + d];
  }
  float* dqrow = (float*)a.dq + (int64_t)b * a.dq_bs + (int64_t)q * a.dq_rs + hoff;
#pragma unroll
  for (int d = 0; d < HD; ++d) dqrow[d] = dq[d] * a.scale;
}

template <int HD>
__global__ __launch_bounds__(64) void attn_bwd_dkv_f32(AttnArgs a) {
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int j = blockIdx.y * 64 + threadIdx.x;
  if (j >= a.Nk) return;
  const int hoff = h * HD;
  const float* krow = (const float*)a.k + (int64_t)b * a.k_bs + (int64_t)j * a.k_rs + hoff;
  const float* vrow = (const float*)a.v + (int64_t)b * a.v_bs + (int64_t)j * a.v_rs + hoff;
  float kv[HD], vv[HD], dk[HD], dv[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) { kv[d] = krow[d]; vv[d] = vrow[d]; dk[d] = 0.f; dv[d] = 0.f; }
  for (int q = 0; q < a.Nq; ++q) {
    if (!key_ok(a, b, j, q)) continue;
    const float* qr = (const float*)a.q + (int64_t)b * a.q_bs + (int64_t)q * a.q_rs + hoff;
    const float* orow = (const float*)a.o + (int64_t)b * a.o_bs + (int64_t)q * a.o_rs + hoff;
    const float* dorow = (const float*)a.dout + (int64_t)b * a.do_bs + (int64_t)q * a.do_rs + hoff;
    float s = 0.f, dp = 0.f, del = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) {
      s += qr[d] * kv[d];
      dp += dorow[d] * vv[d];
      del += dorow[d] * orow[d];
    }
    const float p = expf(s * a.scale - a.lse_in[((int64_t)b * a.H + h) * a.Nq + q]);
    const float mk = a.drop.on() ? pdrop(a, b, h, q, j) : 1.f;
    const float ds = p * (dp * mk - del);
#pragma unroll
    for (int d = 0; d < HD; ++d) {
      dv[d] += p * mk * dorow[d];
      dk[d] += ds * qr[d];
    }
  }
  float* dkrow = (float*)a.dk + (int64_t)b * a.dk_bs + (int64_t)j * a.dk_rs + hoff;
  float* dvrow = (float*)a.dv + (int64_t)b * a.dv_bs + (int64_t)j * a.dv_rs + hoff;
#pragma unroll
  for (int d = 0; d < HD; ++d) { dkrow[d] = dk[d] * a.scale; dvrow[d] = dv[d]; }
}

static size_t fwd_smem(int Nk, int hdp) {
  const int NKP = (Nk + 31) & ~31;
  return (size_t)2 * NKP * (hdp + 16) * 2;
}
// attn_fwd_bf16: hdp 64 uses swizzled unpadded images at 16-row granularity
static size_t fwd_kernel_smem(int Nk, int hdp) {
  if (hdp != 64) return fwd_smem(Nk, hdp);
  return (size_t)2 * ((Nk + 15) & ~15) * 64 * 2;
}
static size_t bwd_kv_smem(int Nq, int hdp) {  // Q, dO images (hdp 64: swizzled, unpadded) + lse, delta
  const int NQP = (Nq + 31) & ~31;
  return (size_t)2 * NQP * (hdp == 64 ? 64 : hdp + 16) * 2 + (size_t)2 * NQP * 4;
}
static size_t bwd_smem(int Nq, int Nk, int hdp) {
  const int NQP = (Nq + 31) & ~31, NKP = (Nk + 31) & ~31;
  return (size_t)(2 * NQP + 2 * NKP) * (hdp + 16) * 2 + (size_t)2 * NQP * 4 + (size_t)NQP * (hdp / 8) * 4;
}

template <typename K>
static int launch_dyn(K kernel, dim3 grid, dim3 block, size_t shm, hipStream_t st, const AttnArgs& a,
                      const char* name) {
  if (shm > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return hip_status(e, name);
  }
  hipLaunchKernelGGL(kernel, grid, block, shm, st, a);
  CAPK_LAUNCH_CHECK(name);
  return CAPK_OK;
}


// ------------------------------------------------------------ decode (small Nq) ---
// Incremental-decode attention (KV-cached beam / greedy steps): Nq <= 8 queries per
// (batch, head) — one new token per beam for self-attention, or the k beams of one
// image against its shared memory keys for cross-attention.  HBM-bound on the K/V
// stream, so VALU (fp32) instead of MFMA: 16 lanes own one key row (8 dims each,
// 16-B loads, a 192-B contiguous row segment at hd 96), 4 keys per wave, 16 per
// block iteration; scores go to LDS, softmax per query by one wave, then P·V with
// the same key ownership and a cross-wave LDS reduction.  No dropout / causal
// (decode never needs either); key padding honoured.
template <int NQ>
__global__ __launch_bounds__(256) void attn_decode_bf16(AttnArgs a) {
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, grp = lane >> 4, c = lane & 15;
  const bool act = c * 8 < a.hd;
  const int hoff = h * a.hd + c * 8;
  __shared__ float sc[NQ][257];
  __shared__ float red[4][NQ][128];
  __shared__ float inv_l[NQ];
  const float qs = a.scale * kLog2e;
  float qv[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    bf16x8 t = (act && q < a.Nq) ? ld8((const bf16*)a.q + (int64_t)b * a.q_bs + (int64_t)q * a.q_rs + hoff) : zero8();
#pragma unroll
    for (int i = 0; i < 8; ++i) qv[q][i] = (float)t[i] * qs;
  }
  const bf16* kb = (const bf16*)a.k + (int64_t)b * a.k_bs + hoff;
  const bf16* vb = (const bf16*)a.v + (int64_t)b * a.v_bs + hoff;
  // phase 1: scores (log2 domain).  Every K and V row segment this lane will touch is
  // requested up front (<= 16 keys per lane at Nk <= 256) so the whole block's K/V
  // stream is in flight at once instead of one dependent load per loop trip.
  constexpr int KIT = 16;
  bf16x8 kr[KIT], vr[KIT];
  const int j0 = w * 4 + grp;
#pragma unroll
  for (int it = 0; it < KIT; ++it) {
    const int j = j0 + 16 * it;
    kr[it] = (act && j < a.Nk) ? ld8(kb + (int64_t)j * a.k_rs) : zero8();
  }
#pragma unroll
  for (int it = 0; it < KIT; ++it) {
    const int j = j0 + 16 * it;
    vr[it] = (act && j < a.Nk) ? ld8(vb + (int64_t)j * a.v_rs) : zero8();
  }
#pragma unroll
  for (int it = 0; it < KIT; ++it) {
    const int j = j0 + 16 * it;
    if (16 * it >= a.Nk) break;
    float kf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) kf[i] = (float)kr[it][i];
    const bool ok = j < a.Nk && (!a.key_pad || !a.key_pad[(int64_t)b * a.Nk + j]);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d = fmaf(qv[q][i], kf[i], d);
      d += __shfl_xor(d, 8, 64);
      d += __shfl_xor(d, 4, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 1, 64);
      if (c == 0 && j < a.Nk) sc[q][j] = ok ? d : -INFINITY;
    }
  }
  __syncthreads();
  // phase 2: softmax per query (wave w owns queries w, w+4)
  for (int q = w; q < a.Nq; q += 4) {
    float m = -INFINITY;
    for (int j = lane; j < a.Nk; j += 64) m = fmaxf(m, sc[q][j]);
    m = wave_max(m);
    float l = 0.f;
    for (int j = lane; j < a.Nk; j += 64) {
      const float p = (m == -INFINITY) ? 0.f : exp2f(sc[q][j] - m);
      sc[q][j] = p;
      l += p;
    }
    l = wave_sum(l);
    if (lane == 0) {
      inv_l[q] = l > 0.f ? 1.f / l : 0.f;
      a.lse[((int64_t)b * a.H + h) * a.Nq + q] = l > 0.f ? (m + __log2f(l)) * kLn2 : -INFINITY;
    }
  }
  __syncthreads();
  // phase 3: O = P V
  float acc[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[q][i] = 0.f;
#pragma unroll
  for (int it = 0; it < KIT; ++it) {
    const int j = j0 + 16 * it;
    if (16 * it >= a.Nk) break;
    if (j < a.Nk) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const float p = sc[q][j];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[q][i] = fmaf(p, (float)vr[it][i], acc[q][i]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float x = acc[q][i];
      x += __shfl_xor(x, 16, 64);
      x += __shfl_xor(x, 32, 64);
      acc[q][i] = x;
    }
  if (grp == 0 && act) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[w][q][c * 8 + i] = acc[q][i];
  }
  __syncthreads();
  for (int e = tid; e < a.Nq * a.hd; e += 256) {
    const int q = e / a.hd, d = e % a.hd;
    const float o = (red[0][q][d] + red[1][q][d] + red[2][q][d] + red[3][q][d]) * inv_l[q];
    ((bf16*)a.out)[(int64_t)b * a.out_bs + (int64_t)q * a.out_rs + h * a.hd + d] = (bf16)o;
  }
}

// ------------------------------------------ cross-attention: short query block vs memory ---
// The <= 32 queries of one (image, head) against its <= 256 memory keys on MFMA: the beam
// cross-attention step (config-3 beam-5: Nq = 5, Nk = 196, hd 96; 114 launches per 256-image
// batch) and, round 4, the training decoder's cross-attention forward (Nq = T = 20 caption
// positions, attention dropout, nn.TransformerDecoderLayer.multihead_attn via
// src/models/decoders.py:421-428).  The step is a K / V stream (K/V 154 MB at bs 256), so what
// costs is round trips, not FLOPs; the VALU decode kernels spent ~1000 VALU issues per wave on
// 5 x 196 x 96 dot products (88 us per step, 1.9 TB/s):
//  * 4 waves per (batch, head), each owning 64 keys (Nk <= 256): S^T = K Q^T with K
//    fragments loaded straight from global memory (16 keys x 32 dims per MFMA, 16-B lane
//    loads of K rows) and the queries as the B operand (NQT 16-query tiles);
//  * the wave's V rows staged in its own LDS image (row stride HDP + 16) and read as V^T
//    fragments by ds_read_b64_tr_b16 for O^T = V^T P^T, P^T packed from the S^T registers
//    (the attn_fwd_bf16 layout: no shuffles between the two products);
//  * every K, V and Q load of the wave issued before the first wait (one round trip);
//  * per-wave softmax (m, l, O^T) merged across the 4 waves in LDS with the flash-decoding
//    rescale; the row sum l excludes dropout (dropout(softmax) V), the mask is the training
//    kernels' pdrop index, so attn_bwd recomputes the same keep decisions.  No causal mask;
//    key padding honoured.  lse (natural log) written for the backward.
template <int HDP, int MODE, int NQT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HDP == 96 ? 3 : 1, 8))) void attn_xdec_bf16(
    AttnArgs a) {
  constexpr int NW = 4, KPW = 64, ST = HDP + (HDP == 96 ? 8 : 16), NCH = HDP / 8, NS = HDP / 32, ND = HDP / 16, NQ = 16 * NQT;
  constexpr int OPS = HDP + 1;  // fp32 partial-O row stride: an odd word count spreads the 16 query rows of a
                                // store over the banks (HDP words put them on 2 bank groups: 8-way conflicts)
  static_assert(NQ * OPS * 4 <= KPW * ST * 2, "the fp32 partial O of a wave fits its V image");
  __shared__ __attribute__((aligned(16))) bf16 vimg[NW][KPW * ST];
  __shared__ float mm[NW][NQ], ll[NW][NQ];
  const int bh = xcd_bh(a), b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const int hoff = h * a.hd;
  const int k0 = w * KPW;  // the wave's first key
  const bf16* kbase = (const bf16*)a.k + (int64_t)b * a.k_bs + hoff;
  const bf16* vbase = (const bf16*)a.v + (int64_t)b * a.v_bs + hoff;
  // Q^T fragments (B operand): query 16 qt + c16, dims s*32 + 8g
  bf16x8 qf[NQT][NS];
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int d = s * 32 + 8 * g, q = 16 * qt + c16;
      qf[qt][s] = (q < a.Nq && d < a.hd) ? ld8((const bf16*)a.q + (int64_t)b * a.q_bs + (int64_t)q * a.q_rs + hoff + d)
                                         : zero8();
    }
  // K fragments (A operand): key k0 + 16 kb + c16, dims s*32 + 8g
  bf16x8 kf[KPW / 16][NS];
#pragma unroll
  for (int kb = 0; kb < KPW / 16; ++kb)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int key = k0 + kb * 16 + c16, d = s * 32 + 8 * g;
      kf[kb][s] = (key < a.Nk && d < a.hd) ? ld8(kbase + (int64_t)key * a.k_rs + d) : zero8();
    }
  // V rows of the wave -> registers -> its LDS image (chunk ch = lane + 64 i: row ch / NCH)
  constexpr int VIT = KPW * NCH / 64;
  bf16x8 vr[VIT];
#pragma unroll
  for (int i = 0; i < VIT; ++i) {
    const int ch = lane + 64 * i, row = ch / NCH, col = (ch % NCH) * 8;
    const int key = k0 + row;
    vr[i] = (key < a.Nk && col < a.hd) ? ld8(vbase + (int64_t)key * a.v_rs + col) : zero8();
  }
  bf16* Vs = vimg[w];
#pragma unroll
  for (int i = 0; i < VIT; ++i) {
    const int ch = lane + 64 * i, row = ch / NCH, col = (ch % NCH) * 8;
    *(bf16x8*)(Vs + row * ST + col) = vr[i];
  }
  // S^T = K Q^T per query tile, scores in the log2 domain; keys past Nk / padded -> -inf
  const float sl2 = a.scale * kLog2e;
  f32x4 sc[NQT][KPW / 16];
  float m[NQT], l[NQT];
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt) {
    m[qt] = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < KPW / 16; ++kb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kb][s], qf[qt][s], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + kb * 16 + 4 * g + r;
        const bool ok = (MODE & AM_MASK) ? key_ok(a, b, key, 16 * qt + c16) : key < a.Nk;
        acc[r] = ok ? acc[r] * sl2 : -INFINITY;
        m[qt] = fmaxf(m[qt], acc[r]);
      }
      sc[qt][kb] = acc;
    }
    m[qt] = fmaxf(m[qt], __shfl_xor(m[qt], 16, 64));
    m[qt] = fmaxf(m[qt], __shfl_xor(m[qt], 32, 64));
    l[qt] = 0.f;
    const DropRun dr(dropm<MODE>() ? drop_idx(a, b, h, 16 * qt + c16, k0 + 4 * g) : 0);  // + 16 kb + r
#pragma unroll
    for (int kb = 0; kb < KPW / 16; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = m[qt] == -INFINITY ? 0.f : fexp2(sc[qt][kb][r] - m[qt]);
        l[qt] += p;  // the normaliser excludes dropout
        sc[qt][kb][r] = dropm<MODE>() && 16 * qt + c16 < a.Nq ? p * dr.mul(a.drop, kb * 16 + r) : p;
      }
    l[qt] += __shfl_xor(l[qt], 16, 64);
    l[qt] += __shfl_xor(l[qt], 32, 64);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own V image is written
  // O^T = V^T P^T over two 32-key chunks
  f32x4 o[NQT][ND];
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
    for (int db = 0; db < ND; ++db) o[qt][db] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < KPW / 32; ++t)
#pragma unroll
    for (int db = 0; db < ND; ++db) {
      const bf16x8 vt = tr_read8(Vs, ST, 32 * t, db * 16, lane);
#pragma unroll
      for (int qt = 0; qt < NQT; ++qt)
        o[qt][db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vt, pack8(sc[qt][2 * t], sc[qt][2 * t + 1]), o[qt][db], 0, 0, 0);
    }
  // merge the 4 waves: (m, l) per query, O^T partials into the (now free) V images as fp32
  __syncthreads();  // every wave is done reading its V image
  float* op = (float*)vimg[w];  // [NQ queries][OPS] fp32 (fits in the wave's image)
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int r = 0; r < 4; ++r) op[(16 * qt + c16) * OPS + db * 16 + 4 * g + r] = o[qt][db][r];
  if (g == 0) {
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) {
      mm[w][16 * qt + c16] = m[qt];
      ll[w][16 * qt + c16] = l[qt];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < a.Nq * a.hd; e += blockDim.x) {
    const int q = e / a.hd, d = e % a.hd;
    float mt = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) mt = fmaxf(mt, mm[ww][q]);
    float num = 0.f, den = 0.f;
    if (mt > -INFINITY) {
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) {
        const float f = mm[ww][q] == -INFINITY ? 0.f : fexp2(mm[ww][q] - mt);
        num += f * ((const float*)vimg[ww])[q * OPS + d];
        den += f * ll[ww][q];
      }
    }
    ((bf16*)a.out)[(int64_t)b * a.out_bs + (int64_t)q * a.out_rs + hoff + d] = (bf16)(den > 0.f ? num / den : 0.f);
    if (d == 0) a.lse[((int64_t)b * a.H + h) * a.Nq + q] = den > 0.f ? (mt + __log2f(den)) * kLn2 : -INFINITY;
  }
}

// ------------------------------------ cross-attention backward: short query block ---
// Backward of attn_xdec_bf16's training launch (the decoder's cross-attention: Nq = 20
// caption positions against Nk = 196 memory keys, hd 96, dropout; <= 32 queries, <= 256 keys).
// The data is K / V in and dK / dV out (2 x 154 MB at bs 256); Q, dO, O are 20 rows per
// (image, head).  4 waves per (batch, head), each owning 64 keys in two 32-key chunks:
//  * per 16-key block: S = Q K^T and dP = dO V^T with the KEY on the lane (Q / dO fragments
//    from the staged images as the A operand, K / V fragments straight from global memory as
//    the B operand), P = exp2(S - lse), dS = P (dP m - D) (m: the pdrop keep factor);
//  * dV^T += dO^T (P m), dK^T += Q^T dS with the query as the MFMA k dimension: dO^T / Q^T by
//    transposed reads of the zero-padded 32-row images, P / dS packed from the score registers
//    (attn_fwd_bf16's k permutation on both sides); dK / dV rows written once (no reduction);
//  * dQ = dS K needs the key on the k dimension: the chunk's dS (bf16) and K rows go to the
//    wave's own LDS images and both are read transposed; the 4 waves' dQ partials are summed
//    in LDS in a fixed order (deterministic).
template <int HDP, int MODE, int NQT>
__global__ __launch_bounds__(256) void attn_xbwd_bf16(AttnArgs a) {
  constexpr int NW = 4, KPW = 64, ST = HDP + 16, NS = HDP / 32, ND = HDP / 16, NQ = 16 * NQT;
  constexpr int DST = 32 + 8;  // dS image [32 keys][32 queries] row stride (bf16)
  __shared__ __attribute__((aligned(16))) bf16 kimg[NW][32 * ST];  // the wave's 32-key chunk of K
  __shared__ __attribute__((aligned(16))) bf16 qimg[32 * ST], doimg[32 * ST];  // rows >= Nq are zero
  __shared__ __attribute__((aligned(16))) bf16 dsimg[NW][32 * DST];
  __shared__ float lse_s[32], del_s[32];
  static_assert(2 * NQ * HDP * 4 <= (int)sizeof(kimg), "two fp32 dQ partials fit the K images");
  const int bh = xcd_bh(a), b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const int hoff = h * a.hd;
  const bf16* kbase = (const bf16*)a.k + (int64_t)b * a.k_bs + hoff;
  const bf16* vbase = (const bf16*)a.v + (int64_t)b * a.v_bs + hoff;
  // ---- prologue: Q / dO images (32 rows, zero past Nq), lse, D = rowsum(dO * O)
  for (int e = threadIdx.x; e < 32 * (HDP / 8); e += blockDim.x) {
    const int r = e / (HDP / 8), c = (e % (HDP / 8)) * 8;
    const bool in = r < a.Nq && c < a.hd;
    *(bf16x8*)(qimg + r * ST + c) = in ? ld8((const bf16*)a.q + (int64_t)b * a.q_bs + (int64_t)r * a.q_rs + hoff + c) : zero8();
    *(bf16x8*)(doimg + r * ST + c) =
        in ? ld8((const bf16*)a.dout + (int64_t)b * a.do_bs + (int64_t)r * a.do_rs + hoff + c) : zero8();
  }
  if (threadIdx.x < 32) {
    const int q = threadIdx.x;
    lse_s[q] = q < a.Nq ? a.lse_in[((int64_t)b * a.H + h) * a.Nq + q] * kLog2e : INFINITY;  // exp2(s - inf) = 0
  }
  __syncthreads();
  // D[q]: 8 lanes per query row (the dO row from LDS, O from global)
  for (int e = threadIdx.x; e < 32 * 8; e += blockDim.x) {
    const int q = e >> 3, c8 = e & 7;
    float d = 0.f;
    if (q < a.Nq)
      for (int c = c8 * 8; c < a.hd; c += 64) {
        const bf16x8 ov = ld8((const bf16*)a.o + (int64_t)b * a.o_bs + (int64_t)q * a.o_rs + hoff + c);
        const bf16x8 dv = *(const bf16x8*)(doimg + q * ST + c);
#pragma unroll
        for (int i = 0; i < 8; ++i) d += (float)ov[i] * (float)dv[i];
      }
    d += __shfl_xor(d, 1, 64);
    d += __shfl_xor(d, 2, 64);
    d += __shfl_xor(d, 4, 64);
    if (c8 == 0) del_s[q] = d;
  }
  // Q / dO fragments (A operand: query 16 qt + c16, dims s*32 + 8g)
  bf16x8 qf[NQT][NS], dof[NQT][NS];
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[qt][s] = *(const bf16x8*)(qimg + (16 * qt + c16) * ST + s * 32 + 8 * g);
      dof[qt][s] = *(const bf16x8*)(doimg + (16 * qt + c16) * ST + s * 32 + 8 * g);
    }
  __syncthreads();  // del_s
  float lq[NQT][4], dq_[NQT][4];
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      lq[qt][r] = lse_s[16 * qt + 4 * g + r];
      dq_[qt][r] = del_s[16 * qt + 4 * g + r];
    }
  const float sl2 = a.scale * kLog2e;
  f32x4 dqa[NQT][ND];  // dQ[q][d] partial: lane = d (c16), rows q = 4g + r
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
    for (int db = 0; db < ND; ++db) dqa[qt][db] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16* Kc = kimg[w];
  bf16* dSc = dsimg[w];
  for (int ch = 0; ch < KPW / 32; ++ch) {
    const int kc0 = w * KPW + ch * 32;  // the chunk's first key
    if (kc0 >= a.Nk) break;             // (wave-uniform)
    // K / V fragments of the chunk's two 16-key blocks (B operand: key c16, dims s*32 + 8g)
    bf16x8 kf[2][NS], vf[2][NS];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int key = kc0 + kb * 16 + c16, d = s * 32 + 8 * g;
        const bool in = key < a.Nk && d < a.hd;
        kf[kb][s] = in ? ld8(kbase + (int64_t)key * a.k_rs + d) : zero8();
        vf[kb][s] = in ? ld8(vbase + (int64_t)key * a.v_rs + d) : zero8();
      }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < NS; ++s) *(bf16x8*)(Kc + (kb * 16 + c16) * ST + s * 32 + 8 * g) = kf[kb][s];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int key = kc0 + kb * 16 + c16;
      f32x4 p[NQT], ds[NQT];
#pragma unroll
      for (int qt = 0; qt < NQT; ++qt) {
        f32x4 sa = {0.f, 0.f, 0.f, 0.f}, dpa = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          sa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[qt][s], kf[kb][s], sa, 0, 0, 0);
          dpa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dof[qt][s], vf[kb][s], dpa, 0, 0, 0);
        }
        const DropRun dr(dropm<MODE>() ? drop_idx(a, b, h, 16 * qt + 4 * g, key) : 0);  // + r Nk
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = 16 * qt + 4 * g + r;
          const bool ok = (MODE & AM_MASK) ? key_ok(a, b, key, q) : key < a.Nk;
          const float pv = ok ? fexp2(sa[r] * sl2 - lq[qt][r]) : 0.f;
          const float mk = dropm<MODE>() && q < a.Nq ? dr.mul(a.drop, (uint32_t)(r * a.Nk)) : 1.f;
          p[qt][r] = pv * mk;
          ds[qt][r] = pv * (dpa[r] * mk - dq_[qt][r]);
        }
        // dS -> the chunk's image, row = key, columns = queries 16 qt + 4g .. + 3
        bf16x4 d4;
        d4[0] = (bf16)ds[qt][0]; d4[1] = (bf16)ds[qt][1]; d4[2] = (bf16)ds[qt][2]; d4[3] = (bf16)ds[qt][3];
        *(bf16x4*)(dSc + (kb * 16 + c16) * DST + 16 * qt + 4 * g) = d4;
      }
      if constexpr (NQT == 1) {  // queries 16..31 of the images are zero rows; the dS columns too
        const bf16x4 z = {(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
        *(bf16x4*)(dSc + (kb * 16 + c16) * DST + 16 + 4 * g) = z;
      }
      const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
      const bf16x8 pb = pack8(p[0], NQT > 1 ? p[NQT - 1] : zero4);
      const bf16x8 dsb = pack8(ds[0], NQT > 1 ? ds[NQT - 1] : zero4);
      // dV^T = dO^T (P m), dK^T = Q^T dS over the (permuted) 32 queries: lane = key, rows = dims
      // (the transposed reads run with every lane active, as the ISA requires; only the stores
      // are per lane)
      bf16* dkrow = (bf16*)a.dk + (int64_t)b * a.dk_bs + (int64_t)key * a.dk_rs + hoff;
      bf16* dvrow = (bf16*)a.dv + (int64_t)b * a.dv_bs + (int64_t)key * a.dv_rs + hoff;
#pragma unroll
      for (int db = 0; db < ND; ++db) {
        f32x4 dv4 = {0.f, 0.f, 0.f, 0.f}, dk4 = {0.f, 0.f, 0.f, 0.f};
        dv4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_read8(doimg, ST, 0, db * 16, lane), pb, dv4, 0, 0, 0);
        dk4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_read8(qimg, ST, 0, db * 16, lane), dsb, dk4, 0, 0, 0);
        const int d0 = db * 16 + 4 * g;
        if (key < a.Nk && d0 < a.hd) {
          store4(dkrow + d0, dk4, a.scale);
          store4(dvrow + d0, dv4, 1.f);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the chunk's K and dS images are written (wave-private)
    // dQ[q][d] += dS[q][keys] K[keys][d]: A = dS (lane = query), B = K (lane = dim), k = the
    // chunk's 32 keys in tr_read8's order on both sides
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) {
      const bf16x8 af = tr_read8(dSc, DST, 0, 16 * qt, lane);
#pragma unroll
      for (int db = 0; db < ND; ++db)
        dqa[qt][db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, tr_read8(Kc, ST, 0, db * 16, lane), dqa[qt][db], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next chunk rewrites the images
  }
  // ---- dQ: the 4 waves' partials summed in a fixed order through two fp32 buffers over kimg
  __syncthreads();
  // row stride RS = HDP + 4 words: a store's 4 row groups (4g) land 16 banks apart (HDP words
  // put them on the same 16 banks: 4-way conflicts)
  constexpr int RS = HDP + 4;
  static_assert(2 * NQ * RS * 4 <= (int)sizeof(kimg), "two padded fp32 dQ partials fit the K images");
  float* red = (float*)&kimg[0][0];  // [2][NQ][RS]
  auto put = [&](float* buf, bool add) {
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
      for (int db = 0; db < ND; ++db)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* x = buf + (16 * qt + 4 * g + r) * RS + db * 16 + c16;
          *x = add ? *x + dqa[qt][db][r] : dqa[qt][db][r];
        }
  };
  if (w < 2) put(red + w * NQ * RS, false);
  __syncthreads();
  if (w >= 2) put(red + (w - 2) * NQ * RS, true);
  __syncthreads();
  for (int e = threadIdx.x; e < a.Nq * a.hd; e += blockDim.x) {
    const int q = e / a.hd, d = e % a.hd;
    ((bf16*)a.dq)[(int64_t)b * a.dq_bs + (int64_t)q * a.dq_rs + hoff + d] =
        (bf16)((red[q * RS + d] + red[NQ * RS + q * RS + d]) * a.scale);
  }
}

// --------------------------------------------- short sequences: one wave per (batch, head) ---
// The decoder's causal self-attention (T = 20 caption positions, hd 96, key-padding mask of the
// caption pads, probability dropout; nn.TransformerDecoderLayer.self_attn via
// src/models/decoders.py:421-428): <= 32 queries x <= 32 keys per (batch, head) is a handful of
// MFMAs, so the 8-wave per-(batch, head) kernels spent their time on set-up and barriers.  Here
// one wave owns a (batch, head): S^T = K Q^T from global fragments (the xdec layout, query on
// the lane), softmax over the 32 keys in registers (two xor-shuffles), O^T = V^T P^T with V^T
// by transposed reads of the wave's own LDS image; no barriers.  WG = SW_WAVES waves.
constexpr int SW_WAVES = 4;
template <int HDP, int MODE>
__global__ __launch_bounds__(64 * SW_WAVES) void attn_short_fwd_bf16(AttnArgs a) {
  constexpr int ST = HDP + 16, NCH = HDP / 8, NS = HDP / 32, ND = HDP / 16;
  __shared__ __attribute__((aligned(16))) bf16 vimg[SW_WAVES][32 * ST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const int bh = blockIdx.x * SW_WAVES + w;
  if (bh >= a.B * a.H) return;  // (wave-uniform; no barriers below)
  const int b = bh / a.H, h = bh % a.H, hoff = h * a.hd;
  const bf16* kbase = (const bf16*)a.k + (int64_t)b * a.k_bs + hoff;
  const bf16* vbase = (const bf16*)a.v + (int64_t)b * a.v_bs + hoff;
  bf16x8 qf[2][NS], kf[2][NS];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int r = 16 * t + c16, d = s * 32 + 8 * g;
      qf[t][s] = (r < a.Nq && d < a.hd) ? ld8((const bf16*)a.q + (int64_t)b * a.q_bs + (int64_t)r * a.q_rs + hoff + d)
                                        : zero8();
      kf[t][s] = (r < a.Nk && d < a.hd) ? ld8(kbase + (int64_t)r * a.k_rs + d) : zero8();
    }
  bf16* Vs = vimg[w];
  constexpr int VIT = 32 * NCH / 64;
#pragma unroll
  for (int i = 0; i < VIT; ++i) {
    const int ch = lane + 64 * i, row = ch / NCH, col = (ch % NCH) * 8;
    *(bf16x8*)(Vs + row * ST + col) = (row < a.Nk && col < a.hd) ? ld8(vbase + (int64_t)row * a.v_rs + col) : zero8();
  }
  const float sl2 = a.scale * kLog2e;
  f32x4 sc[2][2];  // [query tile][key block]: lane = query 16 qt + c16, keys 16 kb + 4g + r
  f32x4 o[2][ND];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = 16 * qt + c16;
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kb][s], qf[qt][s], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * kb + 4 * g + r;
        const bool ok = (MODE & AM_MASK) ? key_ok(a, b, key, q) : key < a.Nk;
        acc[r] = ok ? acc[r] * sl2 : -INFINITY;
        m = fmaxf(m, acc[r]);
      }
      sc[qt][kb] = acc;
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
    const DropRun dr(dropm<MODE>() ? drop_idx(a, b, h, q, 4 * g) : 0);  // + 16 kb + r
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = m == -INFINITY ? 0.f : fexp2(sc[qt][kb][r] - m);
        l += p;  // the normaliser excludes dropout
        sc[qt][kb][r] = dropm<MODE>() && q < a.Nq ? p * dr.mul(a.drop, 16 * kb + r) : p;
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (q < a.Nq && g == 0) a.lse[((int64_t)b * a.H + h) * a.Nq + q] = l > 0.f ? (m + __log2f(l)) * kLn2 : -INFINITY;
    const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) sc[qt][kb] *= inv;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's V image is written
#pragma unroll
  for (int db = 0; db < ND; ++db) {
    const bf16x8 vt = tr_read8(Vs, ST, 0, db * 16, lane);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      o[qt][db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vt, pack8(sc[qt][0], sc[qt][1]), z, 0, 0, 0);
    }
  }
  // O^T fragments: lane = query, rows = dims 16 db + 4g + r -> 8-B row stores
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = 16 * qt + c16;
    if (q < a.Nq) {
      bf16* orow = (bf16*)a.out + (int64_t)b * a.out_bs + (int64_t)q * a.out_rs + hoff;
#pragma unroll
      for (int db = 0; db < ND; ++db) {
        const int d0 = db * 16 + 4 * g;
        if (d0 < a.hd) store4(orow + d0, o[qt][db], 1.f);
      }
    }
  }
}

// Backward of attn_short_fwd_bf16: one wave per (batch, head), attn_xbwd_bf16's products for
// one 32-key chunk (dV^T = dO^T (P m), dK^T = Q^T dS with the key on the lane; dQ^T = K^T dS^T
// through the wave's transposed K and dS images, so dQ rows are stored directly).
constexpr int SB_WAVES = 2;
template <int HDP, int MODE>
__global__ __launch_bounds__(64 * SB_WAVES) void attn_short_bwd_bf16(AttnArgs a) {
  constexpr int ST = HDP + 16, NS = HDP / 32, ND = HDP / 16, NCH = HDP / 8, DST = 32 + 8;
  __shared__ __attribute__((aligned(16))) bf16 qimg[SB_WAVES][32 * ST], doimg[SB_WAVES][32 * ST];
  __shared__ __attribute__((aligned(16))) bf16 kimg[SB_WAVES][32 * ST], dsimg[SB_WAVES][32 * DST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const int bh = blockIdx.x * SB_WAVES + w;
  if (bh >= a.B * a.H) return;  // (wave-uniform; no barriers below)
  const int b = bh / a.H, h = bh % a.H, hoff = h * a.hd;
  bf16 *Qi = qimg[w], *dOi = doimg[w], *Ki = kimg[w], *dSi = dsimg[w];
  // images: rows 0..31 (zero past Nq / Nk), 16-B chunks round-robin over the wave
  constexpr int IT = 32 * NCH / 64;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int ch = lane + 64 * i, r = ch / NCH, c = (ch % NCH) * 8;
    const bool iq = r < a.Nq && c < a.hd, ik = r < a.Nk && c < a.hd;
    *(bf16x8*)(Qi + r * ST + c) = iq ? ld8((const bf16*)a.q + (int64_t)b * a.q_bs + (int64_t)r * a.q_rs + hoff + c) : zero8();
    *(bf16x8*)(dOi + r * ST + c) =
        iq ? ld8((const bf16*)a.dout + (int64_t)b * a.do_bs + (int64_t)r * a.do_rs + hoff + c) : zero8();
    *(bf16x8*)(Ki + r * ST + c) = ik ? ld8((const bf16*)a.k + (int64_t)b * a.k_bs + (int64_t)r * a.k_rs + hoff + c) : zero8();
  }
  // D[q] = rowsum(dO * O) for the lane's 4 queries 4g + r of each tile (O from global, dO
  // from the image once it is written), lse
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float lq[2][4], dd[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = 16 * qt + 4 * g + r;
      lq[qt][r] = q < a.Nq ? a.lse_in[((int64_t)b * a.H + h) * a.Nq + q] * kLog2e : INFINITY;
      // 16 lanes (c16) share the row: each sums hd / 16 columns, then xor-reduce over c16
      float d = 0.f;
      if (q < a.Nq)
        for (int c = c16 * 8; c < a.hd; c += 128) {
          const bf16x8 ov = ld8((const bf16*)a.o + (int64_t)b * a.o_bs + (int64_t)q * a.o_rs + hoff + c);
          const bf16x8 dv = *(const bf16x8*)(dOi + q * ST + c);
#pragma unroll
          for (int i = 0; i < 8; ++i) d += (float)ov[i] * (float)dv[i];
        }
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 4, 64);
      d += __shfl_xor(d, 8, 64);
      dd[qt][r] = d;
    }
  bf16x8 qf[2][NS], dof[2][NS], kf[2][NS], vf[2][NS];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int r = 16 * t + c16, d = s * 32 + 8 * g;
      qf[t][s] = *(const bf16x8*)(Qi + r * ST + d);
      dof[t][s] = *(const bf16x8*)(dOi + r * ST + d);
      kf[t][s] = *(const bf16x8*)(Ki + r * ST + d);
      vf[t][s] = (r < a.Nk && d < a.hd) ? ld8((const bf16*)a.v + (int64_t)b * a.v_bs + (int64_t)r * a.v_rs + hoff + d)
                                        : zero8();
    }
  const float sl2 = a.scale * kLog2e;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int key = 16 * kb + c16;
    f32x4 p[2], ds[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x4 sa = {0.f, 0.f, 0.f, 0.f}, dpa = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[qt][s], kf[kb][s], sa, 0, 0, 0);
        dpa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dof[qt][s], vf[kb][s], dpa, 0, 0, 0);
      }
      const DropRun dr(dropm<MODE>() ? drop_idx(a, b, h, 16 * qt + 4 * g, key) : 0);  // + r Nk
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = 16 * qt + 4 * g + r;
        const bool ok = (MODE & AM_MASK) ? key_ok(a, b, key, q) : key < a.Nk;
        const float pv = ok ? fexp2(sa[r] * sl2 - lq[qt][r]) : 0.f;
        const float mk = dropm<MODE>() && q < a.Nq ? dr.mul(a.drop, (uint32_t)(r * a.Nk)) : 1.f;
        p[qt][r] = pv * mk;
        ds[qt][r] = pv * (dpa[r] * mk - dd[qt][r]);
      }
      bf16x4 d4;
      d4[0] = (bf16)ds[qt][0]; d4[1] = (bf16)ds[qt][1]; d4[2] = (bf16)ds[qt][2]; d4[3] = (bf16)ds[qt][3];
      *(bf16x4*)(dSi + key * DST + 16 * qt + 4 * g) = d4;
    }
    const bf16x8 pb = pack8(p[0], p[1]), dsb = pack8(ds[0], ds[1]);
    bf16* dkrow = (bf16*)a.dk + (int64_t)b * a.dk_bs + (int64_t)key * a.dk_rs + hoff;
    bf16* dvrow = (bf16*)a.dv + (int64_t)b * a.dv_bs + (int64_t)key * a.dv_rs + hoff;
#pragma unroll
    for (int db = 0; db < ND; ++db) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 dv4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_read8(dOi, ST, 0, db * 16, lane), pb, z, 0, 0, 0);
      const f32x4 dk4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_read8(Qi, ST, 0, db * 16, lane), dsb, z, 0, 0, 0);
      const int d0 = db * 16 + 4 * g;
      if (key < a.Nk && d0 < a.hd) {
        store4(dkrow + d0, dk4, a.scale);
        store4(dvrow + d0, dv4, 1.f);
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the dS image is written
  // dQ^T[d][q] = K^T dS^T over the 32 keys (tr_read8's k order on both sides): lane = query
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const bf16x8 dst = tr_read8(dSi, DST, 0, 16 * qt, lane);
    const int q = 16 * qt + c16;
    bf16* dqrow = (bf16*)a.dq + (int64_t)b * a.dq_bs + (int64_t)q * a.dq_rs + hoff;
#pragma unroll
    for (int db = 0; db < ND; ++db) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 dq4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_read8(Ki, ST, 0, db * 16, lane), dst, z, 0, 0, 0);
      const int d0 = db * 16 + 4 * g;
      if (q < a.Nq && d0 < a.hd) store4(dqrow + d0, dq4, a.scale);
    }
  }
}

// ---------------------------------------------------------------- decode v2 ---
// KV-cached decode attention (Nq <= 8 queries per (batch, head): one beam row's query, or the
// k beams of one image against its shared memory K/V).  The step is HBM-bound on the K/V
// stream and tiny per (batch, head), so what costs is instructions and round trips, not
// FLOPs; attn_decode_bf16 above spends ~2000 VALU + ~400 cross-lane shuffles per lane on a
// 196-key cross step (96 us for 154 MB: 1.6 TB/s).  Here:
//  * LPR lanes own one key row (LPR = hd / 8 rounded up to 8 or 16: one 16-B chunk each),
//    KPP = 64 / LPR keys per pass, every K and V chunk of the wave's <= MAXP passes requested
//    before the first use (one round trip per wave);
//  * the dot product is reduced inside the key's lane group by DPP (quad_perm,
//    row_half_mirror, row_mirror: no LDS traffic), so every lane of the group holds the score;
//  * each wave runs its own softmax over its keys (max / sum across the KPP groups: two to
//    three xor shuffles per query) and accumulates P V for its chunk; waves of a workgroup
//    (W = ceil(passes / MAXP), 1 for self-attention steps) merge their (m, l, acc) in LDS
//    with the flash-decoding rescale.
// No dropout / causal (decode never needs either); key padding honoured.
template <int LPR>
__device__ __forceinline__ float grp_sum(float x) {  // sum over the lane's LPR-lane group (LPR 8 / 16)
#define CAPK_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false))
  x += CAPK_DPP(x, 0xB1);   // quad_perm [1,0,3,2]
  x += CAPK_DPP(x, 0x4E);   // quad_perm [2,3,0,1]
  x += CAPK_DPP(x, 0x141);  // row_half_mirror: lane i <-> 7 - i of its 8
  if constexpr (LPR == 16) x += CAPK_DPP(x, 0x140);  // row_mirror: lane i <-> 15 - i of its 16
#undef CAPK_DPP
  return x;
}
template <int LPR, int NQ, int MAXP>
__global__ __launch_bounds__(512) void attn_decode2_bf16(AttnArgs a, int passes_per_wave) {
  constexpr int KPP = 64 / LPR;
  const int bh = xcd_bh(a), b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, W = blockDim.x >> 6;
  const int g = lane / LPR, c = lane % LPR;
  const bool act = c * 8 < a.hd;
  const int hoff = h * a.hd + c * 8;
  const int p0 = w * passes_per_wave;  // the wave's first pass (key j = pass * KPP + g)
  const bf16* kb = (const bf16*)a.k + hoff;
  const bf16* vb = (const bf16*)a.v + hoff;
  bf16x8 kr[MAXP], vr[MAXP];
  float qf[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const bf16x8 t = (act && q < a.Nq) ? ld8((const bf16*)a.q + (int64_t)b * a.q_bs + (int64_t)q * a.q_rs + hoff) : zero8();
#pragma unroll
    for (int i = 0; i < 8; ++i) qf[q][i] = (float)t[i];
  }
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int j = (p0 + p) * KPP + g;
    const bool in = act && p < passes_per_wave && j < a.Nk;
    if (a.kv_rows) {  // (wave-uniform) beam-history table: the row per key
      const int64_t rb = in ? kv_row(a, b, j) : 0;
      kr[p] = in ? ld8(kb + rb * a.k_bs + (int64_t)j * a.k_rs) : zero8();
      vr[p] = in ? ld8(vb + rb * a.v_bs + (int64_t)j * a.v_rs) : zero8();
    } else {
      kr[p] = in ? ld8(kb + (int64_t)b * a.k_bs + (int64_t)j * a.k_rs) : zero8();
      vr[p] = in ? ld8(vb + (int64_t)b * a.v_bs + (int64_t)j * a.v_rs) : zero8();
    }
  }
  const float qs = a.scale * kLog2e;
  float s[MAXP][NQ];
  float m[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) m[q] = -INFINITY;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int j = (p0 + p) * KPP + g;
    const bool ok = p < passes_per_wave && j < a.Nk && (!a.key_pad || !a.key_pad[(int64_t)b * a.Nk + j]);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d = fmaf(qf[q][i], (float)kr[p][i], d);
      d = grp_sum<LPR>(d) * qs;
      s[p][q] = ok ? d : -INFINITY;
      m[q] = fmaxf(m[q], s[p][q]);
    }
  }
  // the wave's max / sum over its KPP key groups (xor over the group index bits)
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) m[q] = fmaxf(m[q], __shfl_xor(m[q], o, 64));
  float l[NQ], acc[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    l[q] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[q][i] = 0.f;
  }
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    float vf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) vf[i] = (float)vr[p][i];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const float pv = m[q] == -INFINITY ? 0.f : fexp2(s[p][q] - m[q]);
      l[q] += pv;  // every lane of the group holds the same pv: the group sum is counted once below
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[q][i] = fmaf(pv, vf[i], acc[q][i]);
    }
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) {
      l[q] += __shfl_xor(l[q], o, 64);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[q][i] += __shfl_xor(acc[q][i], o, 64);
    }
  }
  // every lane of chunk c now holds the wave's (m, l, acc) for c; lanes of group 0 publish
  if (W == 1) {
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q >= a.Nq) break;
        const float inv = l[q] > 0.f ? 1.f / l[q] : 0.f;
        if (act) {
          bf16x8 o;
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = (bf16)(acc[q][i] * inv);
          *(bf16x8*)((bf16*)a.out + (int64_t)b * a.out_bs + (int64_t)q * a.out_rs + hoff) = o;
        }
        if (c == 0) a.lse[((int64_t)b * a.H + h) * a.Nq + q] = l[q] > 0.f ? (m[q] + __log2f(l[q])) * kLn2 : -INFINITY;
      }
    }
    return;
  }
  // (m, l) per wave and query, then acc [w][q][128]: dynamic LDS, none for W == 1 launches
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  float(*sm)[NQ] = (float(*)[NQ])dsm;
  float(*sl)[NQ] = (float(*)[NQ])(dsm + 8 * NQ);
  float(*sacc)[NQ][128] = (float(*)[NQ][128])(dsm + 16 * NQ);
  if (g == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (c == 0) { sm[w][q] = m[q]; sl[w][q] = l[q]; }
      if (act) {
#pragma unroll
        for (int i = 0; i < 8; ++i) sacc[w][q][c * 8 + i] = acc[q][i];
      }
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < a.Nq * a.hd; e += blockDim.x) {
    const int q = e / a.hd, d = e % a.hd;
    float mt = -INFINITY;
    for (int ww = 0; ww < W; ++ww) mt = fmaxf(mt, sm[ww][q]);
    float num = 0.f, den = 0.f;
    if (mt > -INFINITY) {
      for (int ww = 0; ww < W; ++ww) {
        const float f = sm[ww][q] == -INFINITY ? 0.f : fexp2(sm[ww][q] - mt);
        num += f * sacc[ww][q][d];
        den += f * sl[ww][q];
      }
    }
    ((bf16*)a.out)[(int64_t)b * a.out_bs + (int64_t)q * a.out_rs + h * a.hd + d] = (bf16)(den > 0.f ? num / den : 0.f);
    if (d == 0) a.lse[((int64_t)b * a.H + h) * a.Nq + q] = den > 0.f ? (mt + __log2f(den)) * kLn2 : -INFINITY;
  }
}

// xcd_chunk for a grid of nblk (batch, head) workgroups (CAPK_ATTN_XCD=0: the plain order, for A/B)
static int attn_xcd(int nblk) {
  static const bool on = [] { const char* e = getenv("CAPK_ATTN_XCD"); return !(e && e[0] == '0'); }();
  return on && nblk % 8 == 0 ? 1 : 0;
}

// launch the v2 decode kernel: LPR by head width, W waves so that each wave has <= MAXP passes
template <int NQ>
static int launch_decode2(AttnArgs a, hipStream_t st) {
  a.xcd_chunk = attn_xcd(a.B * a.H);
  constexpr int MAXP = 8;
  const int lpr = a.hd <= 64 ? 8 : 16, kpp = 64 / lpr;
  const int npass = cdiv(a.Nk, kpp);
  const int W = std::min(8, cdiv(npass, MAXP)), ppw = cdiv(npass, W);
  const dim3 g(a.B * a.H), blk(64 * W);
  const size_t shm = W > 1 ? (size_t)(16 * NQ + 8 * NQ * 128) * sizeof(float) : 0;
  if (lpr == 8) hipLaunchKernelGGL((attn_decode2_bf16<8, NQ, MAXP>), g, blk, shm, st, a, ppw);
  else hipLaunchKernelGGL((attn_decode2_bf16<16, NQ, MAXP>), g, blk, shm, st, a, ppw);
  CAPK_LAUNCH_CHECK("attn_decode2_bf16");
  return CAPK_OK;
}

static int hdp_of(int hd) { return hd <= 32 ? 32 : hd <= 64 ? 64 : hd <= 96 ? 96 : 128; }

static int check_common(int dtype, int B, int H, int Nq, int Nk, int hd) {
  CAPK_CHECK_ARG(B > 0 && H > 0 && Nq > 0 && Nk > 0, "capk_attention: bad sizes");
  CAPK_CHECK_ARG(Nq <= 256 && Nk <= 256, "capk_attention: Nq, Nk <= 256 (got %d, %d)", Nq, Nk);
  CAPK_CHECK_ARG(hd % 8 == 0 && hd <= 128, "capk_attention: hd=%d must be a multiple of 8, <= 128", hd);
  CAPK_CHECK_ARG(dtype == CAPK_BF16 || dtype == CAPK_F32, "capk_attention: dtype");
  return CAPK_OK;
}

#define F32_HD_DISPATCH(KERNEL, grid, ...)                                                           \
  switch (a.hd) {                                                                                   \
    case 8: hipLaunchKernelGGL(KERNEL<8>, grid, dim3(64), 0, st, a); break;                         \
    case 16: hipLaunchKernelGGL(KERNEL<16>, grid, dim3(64), 0, st, a); break;                       \
    case 32: hipLaunchKernelGGL(KERNEL<32>, grid, dim3(64), 0, st, a); break;                       \
    case 64: hipLaunchKernelGGL(KERNEL<64>, grid, dim3(64), 0, st, a); break;                       \
    case 96: hipLaunchKernelGGL(KERNEL<96>, grid, dim3(64), 0, st, a); break;                       \
    case 128: hipLaunchKernelGGL(KERNEL<128>, grid, dim3(64), 0, st, a); break;                     \
    default: set_error("capk_attention(f32): hd=%d unsupported", a.hd); return CAPK_EUNSUPPORTED;   \
  }

int launch_colsum_finish(int parts, int N, const float* part, float* out, int accumulate, hipStream_t st);  // misc.hip

}  // namespace capk

using namespace capk;

static int attn_dma_env() {  // CAPK_ATTN_DMA: bit 0 forward, bit 1 dQ, bit 2 dK/dV kernel (default 7; A/B)
  static const int v = [] { const char* e = getenv("CAPK_ATTN_DMA"); return e ? atoi(e) & 7 : 7; }();
  return v;
}

extern "C" int capk_attention_fwd(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, int causal,
                                  const void* q, int64_t q_bs, int64_t q_rs, const void* k, int64_t k_bs,
                                  int64_t k_rs, const void* v, int64_t v_bs, int64_t v_rs, const uint8_t* key_pad,
                                  void* o, int64_t o_bs, int64_t o_rs, float* lse, float drop_p, uint32_t drop_seed,
                                  void* stream) {
  int rc = check_common(dtype, B, H, Nq, Nk, hd);
  if (rc) return rc;
  AttnArgs a{};
  a.B = B; a.H = H; a.Nq = Nq; a.Nk = Nk; a.hd = hd; a.causal = causal; a.scale = scale;
  a.q = q; a.k = k; a.v = v; a.q_bs = q_bs; a.q_rs = q_rs; a.k_bs = k_bs; a.k_rs = k_rs; a.v_bs = v_bs; a.v_rs = v_rs;
  a.key_pad = key_pad; a.out = o; a.out_bs = o_bs; a.out_rs = o_rs; a.lse = lse;
  a.drop = make_drop(drop_p, drop_seed);
  a.dma_stage = attn_dma_env();
  hipStream_t st = S(stream);
  if (dtype == CAPK_F32) {
    dim3 grid(B * H, cdiv(Nq, 64));
    F32_HD_DISPATCH(attn_fwd_f32, grid);
    CAPK_LAUNCH_CHECK("attn_fwd_f32");
    return CAPK_OK;
  }
  CAPK_CHECK_ARG(q_rs % 8 == 0 && k_rs % 8 == 0 && v_rs % 8 == 0 && o_rs % 4 == 0 && q_bs % 8 == 0 &&
                     k_bs % 8 == 0 && v_bs % 8 == 0,
                 "capk_attention_fwd(bf16): strides must allow 16-B vector access");
  static const bool decode_v1 = [] { const char* e = getenv("CAPK_DECODE_V1"); return e && e[0] == '1'; }();
  // short sequences (the decoder / GPT-2 / QFormer self-attention: 8 < Nq <= 32, Nk <= 32): one
  // wave per (batch, head) (CAPK_SHORT_ATTN=0: the per-(batch, head) 8-wave kernel, for A/B)
  static const bool short_on = [] { const char* e = getenv("CAPK_SHORT_ATTN"); return !(e && e[0] == '0'); }();
  if (short_on && Nq > 8 && Nq <= 32 && Nk <= 32 && (hd == 64 || hd == 96 || hd == 128)) {
    const dim3 g(cdiv(B * H, SW_WAVES)), blk(64 * SW_WAVES);
    const int sm = (causal || key_pad ? AM_MASK : 0) | (drop_p > 0.f ? AM_DROP : 0);
#define SFM(HD)                                                                                    \
  switch (sm) {                                                                                    \
    case 0: hipLaunchKernelGGL((attn_short_fwd_bf16<HD, 0>), g, blk, 0, st, a); break;               \
    case AM_DROP: hipLaunchKernelGGL((attn_short_fwd_bf16<HD, AM_DROP>), g, blk, 0, st, a); break;   \
    case AM_MASK: hipLaunchKernelGGL((attn_short_fwd_bf16<HD, AM_MASK>), g, blk, 0, st, a); break;   \
    default: hipLaunchKernelGGL((attn_short_fwd_bf16<HD, AM_MASK | AM_DROP>), g, blk, 0, st, a); break; \
  }
    if (hd == 64) { SFM(64) } else if (hd == 96) { SFM(96) } else { SFM(128) }
#undef SFM
    CAPK_LAUNCH_CHECK("attn_short_fwd_bf16");
    return CAPK_OK;
  }
  // short query blocks against memory keys (beam cross-attention steps: k beams of an image;
  // the training decoder's cross-attention: T = 20 positions, with dropout): the MFMA xdec
  // kernel (CAPK_XDEC=0 keeps the beam steps on the VALU decode kernel and the training
  // launches on attn_fwd_bf16, for A/B)
  static const bool xdec_on = [] { const char* e = getenv("CAPK_XDEC"); return !(e && e[0] == '0'); }();
  if (xdec_on && !decode_v1 && Nq >= 2 && Nq <= 32 && Nk > 64 && Nk <= 256 && !causal &&
      (hd == 64 || hd == 96 || hd == 128)) {
    const dim3 g(B * H), blk(256);
    a.xcd_chunk = attn_xcd(B * H);
    const int xm = (key_pad ? AM_MASK : 0) | (drop_p > 0.f ? AM_DROP : 0);
#define XDQ(HD, M)                                                                  \
  if (Nq <= 16) hipLaunchKernelGGL((attn_xdec_bf16<HD, M, 1>), g, blk, 0, st, a);   \
  else hipLaunchKernelGGL((attn_xdec_bf16<HD, M, 2>), g, blk, 0, st, a);
#define XD(HD)                                                                      \
  switch (xm) {                                                                     \
    case 0: XDQ(HD, 0) break;                                                       \
    case AM_DROP: XDQ(HD, AM_DROP) break;                                           \
    case AM_MASK: XDQ(HD, AM_MASK) break;                                           \
    default: XDQ(HD, AM_MASK | AM_DROP) break;                                      \
  }
    if (hd == 64) { XD(64) } else if (hd == 96) { XD(96) } else { XD(128) }
#undef XD
#undef XDQ
    CAPK_LAUNCH_CHECK("attn_xdec_bf16");
    return CAPK_OK;
  }
  if (Nq <= 8 && !causal && !(drop_p > 0.f) && !decode_v1 && o_rs % 8 == 0 && o_bs % 8 == 0) {
    switch (Nq) {
      case 1: return launch_decode2<1>(a, st);
      case 2: return launch_decode2<2>(a, st);
      case 3: return launch_decode2<3>(a, st);
      case 4: return launch_decode2<4>(a, st);
      case 5: return launch_decode2<5>(a, st);
      case 6: return launch_decode2<6>(a, st);
      case 7: return launch_decode2<7>(a, st);
      default: return launch_decode2<8>(a, st);
    }
  }
  if (Nq <= 8 && !causal && !(drop_p > 0.f)) {  // CAPK_DECODE_V1=1: the first decode kernel (A/B)
    const dim3 g(B * H), blk(256);
    switch (Nq) {
      case 1: hipLaunchKernelGGL(attn_decode_bf16<1>, g, blk, 0, st, a); break;
      case 2: hipLaunchKernelGGL(attn_decode_bf16<2>, g, blk, 0, st, a); break;
      case 3: hipLaunchKernelGGL(attn_decode_bf16<3>, g, blk, 0, st, a); break;
      case 4: hipLaunchKernelGGL(attn_decode_bf16<4>, g, blk, 0, st, a); break;
      case 5: hipLaunchKernelGGL(attn_decode_bf16<5>, g, blk, 0, st, a); break;
      case 6: hipLaunchKernelGGL(attn_decode_bf16<6>, g, blk, 0, st, a); break;
      case 7: hipLaunchKernelGGL(attn_decode_bf16<7>, g, blk, 0, st, a); break;
      default: hipLaunchKernelGGL(attn_decode_bf16<8>, g, blk, 0, st, a); break;
    }
    CAPK_LAUNCH_CHECK("attn_decode_bf16");
    return CAPK_OK;
  }
  const int hdp = hdp_of(hd);
  const size_t shm = fwd_kernel_smem(Nk, hdp);
  const dim3 grid(B * H), block(512);
  const int mode = (drop_p > 0.f ? AM_DROP : 0) | ((causal || key_pad) ? AM_MASK : 0);
#define FWD_M(HD)                                                                                        \
  switch (mode) {                                                                                        \
    case 0: return launch_dyn(attn_fwd_bf16<HD, 0>, grid, block, shm, st, a, "attn_fwd_bf16");           \
    case 1: return launch_dyn(attn_fwd_bf16<HD, 1>, grid, block, shm, st, a, "attn_fwd_bf16");           \
    case 2: return launch_dyn(attn_fwd_bf16<HD, 2>, grid, block, shm, st, a, "attn_fwd_bf16");           \
    default: return launch_dyn(attn_fwd_bf16<HD, 3>, grid, block, shm, st, a, "attn_fwd_bf16");          \
  }
  switch (hdp) {
    case 32: FWD_M(32)
    case 64: FWD_M(64)
    case 96: FWD_M(96)
    default: FWD_M(128)
  }
#undef FWD_M
}

extern "C" int capk_attention_decode_rows(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, const void* q,
                                          int64_t q_bs, int64_t q_rs, const void* k, int64_t k_bs, int64_t k_rs,
                                          const void* v, int64_t v_bs, int64_t v_rs, const int32_t* kv_rows,
                                          int64_t kv_rows_ld, void* o, int64_t o_bs, int64_t o_rs, float* lse,
                                          void* stream) {
  int rc = check_common(dtype, B, H, Nq, Nk, hd);
  if (rc) return rc;
  CAPK_CHECK_ARG(Nq <= 8 && kv_rows && kv_rows_ld >= Nk - 1, "capk_attention_decode_rows: Nq <= 8 and a history table");
  AttnArgs a{};
  a.B = B; a.H = H; a.Nq = Nq; a.Nk = Nk; a.hd = hd; a.causal = 0; a.scale = scale;
  a.q = q; a.k = k; a.v = v; a.q_bs = q_bs; a.q_rs = q_rs; a.k_bs = k_bs; a.k_rs = k_rs; a.v_bs = v_bs; a.v_rs = v_rs;
  a.out = o; a.out_bs = o_bs; a.out_rs = o_rs; a.lse = lse;
  a.drop = make_drop(0.f, 0);
  a.kv_rows = kv_rows; a.kv_rows_ld = kv_rows_ld;
  hipStream_t st = S(stream);
  if (dtype == CAPK_F32) {
    dim3 grid(B * H, cdiv(Nq, 64));
    F32_HD_DISPATCH(attn_fwd_f32, grid);
    CAPK_LAUNCH_CHECK("attn_fwd_f32");
    return CAPK_OK;
  }
  CAPK_CHECK_ARG(q_rs % 8 == 0 && k_rs % 8 == 0 && v_rs % 8 == 0 && o_rs % 8 == 0 && q_bs % 8 == 0 &&
                     k_bs % 8 == 0 && v_bs % 8 == 0 && o_bs % 8 == 0,
                 "capk_attention_decode_rows(bf16): strides must allow 16-B vector access");
  switch (Nq) {
    case 1: return launch_decode2<1>(a, st);
    case 2: return launch_decode2<2>(a, st);
    case 3: return launch_decode2<3>(a, st);
    case 4: return launch_decode2<4>(a, st);
    case 5: return launch_decode2<5>(a, st);
    case 6: return launch_decode2<6>(a, st);
    case 7: return launch_decode2<7>(a, st);
    default: return launch_decode2<8>(a, st);
  }
}

static int g_bwd_slice = -1;  // capk_attention_set_bwd_slice (-1: CAPK_ATTN_BWD_SLICE)
static int g_fused_bwd = -1;  // capk_attention_set_fused_bwd (-1: CAPK_ATTN_FUSED_BWD, default on)

// bias_part != nullptr: the split kernels also write per-image dQ / dK / dV column sums
// ([B][3*H*hd], AttnArgs::dbias_part) and *bias_fused is set; other routes leave it false.
static int attention_bwd_impl(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, int causal,
                              const void* q, int64_t q_bs, int64_t q_rs, const void* k, int64_t k_bs,
                              int64_t k_rs, const void* v, int64_t v_bs, int64_t v_rs, const uint8_t* key_pad,
                              const void* o, int64_t o_bs, int64_t o_rs, const void* dout, int64_t do_bs,
                              int64_t do_rs, const float* lse, void* dq, int64_t dq_bs, int64_t dq_rs, void* dk,
                              int64_t dk_bs, int64_t dk_rs, void* dv, int64_t dv_bs, int64_t dv_rs,
                              float drop_p, uint32_t drop_seed, void* stream, float* bias_part, bool* bias_fused) {
  if (bias_fused) *bias_fused = false;
  int rc = check_common(dtype, B, H, Nq, Nk, hd);
  if (rc) return rc;
  AttnArgs a{};
  a.B = B; a.H = H; a.Nq = Nq; a.Nk = Nk; a.hd = hd; a.causal = causal; a.scale = scale;
  a.q = q; a.k = k; a.v = v; a.q_bs = q_bs; a.q_rs = q_rs; a.k_bs = k_bs; a.k_rs = k_rs; a.v_bs = v_bs; a.v_rs = v_rs;
  a.key_pad = key_pad; a.o = o; a.o_bs = o_bs; a.o_rs = o_rs; a.dout = dout; a.do_bs = do_bs; a.do_rs = do_rs;
  a.lse_in = lse; a.dq = dq; a.dq_bs = dq_bs; a.dq_rs = dq_rs; a.dk = dk; a.dk_bs = dk_bs; a.dk_rs = dk_rs;
  a.dv = dv; a.dv_bs = dv_bs; a.dv_rs = dv_rs;
  a.drop = make_drop(drop_p, drop_seed);
  a.dma_stage = attn_dma_env();
  hipStream_t st = S(stream);
  if (dtype == CAPK_F32) {
    {
      dim3 grid(B * H, cdiv(Nq, 64));
      F32_HD_DISPATCH(attn_bwd_dq_f32, grid);
      CAPK_LAUNCH_CHECK("attn_bwd_dq_f32");
    }
    {
      dim3 grid(B * H, cdiv(Nk, 64));
      F32_HD_DISPATCH(attn_bwd_dkv_f32, grid);
      CAPK_LAUNCH_CHECK("attn_bwd_dkv_f32");
    }
    return CAPK_OK;
  }
  CAPK_CHECK_ARG(q_rs % 8 == 0 && k_rs % 8 == 0 && v_rs % 8 == 0 && do_rs % 8 == 0 && dq_rs % 4 == 0 &&
                     dk_rs % 4 == 0 && dv_rs % 4 == 0,
                 "capk_attention_bwd(bf16): strides must allow vector access");
  const int hdp = hdp_of(hd);
  const dim3 grid(B * H), block(512);
  const int mode = (drop_p > 0.f ? AM_DROP : 0) | ((causal || key_pad) ? AM_MASK : 0);
#define BY_MODE(CALL)        \
  switch (mode) {            \
    case 0: CALL(0); break;  \
    case 1: CALL(1); break;  \
    case 2: CALL(2); break;  \
    default: CALL(3); break; \
  }
#define BY_HDP(CALL2, M)          \
  switch (hdp) {                  \
    case 32: CALL2(32, M); break; \
    case 64: CALL2(64, M); break; \
    case 96: CALL2(96, M); break; \
    default: CALL2(128, M); break; \
  }
  int rc2 = CAPK_OK;
  static const bool short_on = [] { const char* e = getenv("CAPK_SHORT_ATTN"); return !(e && e[0] == '0'); }();
  if (short_on && Nq > 8 && Nq <= 32 && Nk <= 32 && (hd == 64 || hd == 96 || hd == 128)) {
    const dim3 g(cdiv(B * H, SB_WAVES)), blk(64 * SB_WAVES);
    const int sm = (causal || key_pad ? AM_MASK : 0) | (drop_p > 0.f ? AM_DROP : 0);
#define SBM(HD)                                                                                    \
  switch (sm) {                                                                                    \
    case 0: hipLaunchKernelGGL((attn_short_bwd_bf16<HD, 0>), g, blk, 0, st, a); break;               \
    case AM_DROP: hipLaunchKernelGGL((attn_short_bwd_bf16<HD, AM_DROP>), g, blk, 0, st, a); break;   \
    case AM_MASK: hipLaunchKernelGGL((attn_short_bwd_bf16<HD, AM_MASK>), g, blk, 0, st, a); break;   \
    default: hipLaunchKernelGGL((attn_short_bwd_bf16<HD, AM_MASK | AM_DROP>), g, blk, 0, st, a); break; \
  }
    if (hd == 64) { SBM(64) } else if (hd == 96) { SBM(96) } else { SBM(128) }
#undef SBM
    CAPK_LAUNCH_CHECK("attn_short_bwd_bf16");
    return CAPK_OK;
  }
  // short query blocks against memory keys (the training decoder's cross-attention): the
  // MFMA xbwd kernel, the backward of attn_xdec_bf16 (CAPK_XDEC=0: the fused kernel below)
  static const bool xbwd_on = [] { const char* e = getenv("CAPK_XDEC"); return !(e && e[0] == '0'); }();
  if (xbwd_on && Nq >= 2 && Nq <= 32 && Nk > 64 && Nk <= 256 && !causal && (hd == 64 || hd == 96 || hd == 128)) {
    const dim3 g(B * H), blk(256);
    a.xcd_chunk = attn_xcd(B * H);
    const int xm = (key_pad ? AM_MASK : 0) | (drop_p > 0.f ? AM_DROP : 0);
#define XBQ(HD, M)                                                                  \
  if (Nq <= 16) hipLaunchKernelGGL((attn_xbwd_bf16<HD, M, 1>), g, blk, 0, st, a);   \
  else hipLaunchKernelGGL((attn_xbwd_bf16<HD, M, 2>), g, blk, 0, st, a);
#define XB(HD)                                                                      \
  switch (xm) {                                                                     \
    case 0: XBQ(HD, 0) break;                                                       \
    case AM_DROP: XBQ(HD, AM_DROP) break;                                           \
    case AM_MASK: XBQ(HD, AM_MASK) break;                                           \
    default: XBQ(HD, AM_MASK | AM_DROP) break;                                      \
  }
    if (hd == 64) { XB(64) } else if (hd == 96) { XB(96) } else { XB(128) }
#undef XB
#undef XBQ
    CAPK_LAUNCH_CHECK("attn_xbwd_bf16");
    return CAPK_OK;
  }
  // 64-wide heads without the bias sums: the fused single-pass kernel (attn_bwd_fused64)
  // CAPK_ATTN_FUSED_BWD: 0 the split pair, 1 (default) attn_bwd_fused64
  static const int fused_env = [] { const char* e = getenv("CAPK_ATTN_FUSED_BWD"); return !(e && e[0] == '0'); }();
  const int fmode = g_fused_bwd >= 0 ? g_fused_bwd : fused_env;
  if (fmode >= 1 && hd == 64 && Nq > 32 && Nk <= 256) {
    const int nqp = (Nq + 31) & ~31, nkp = (Nk + 15) & ~15, nkc = (nkp + 31) / 32;
    const size_t shm = (size_t)(2 * nqp + nkp) * 128 + (size_t)2 * nkc * 32 * 48 * 2 + (size_t)2 * nqp * 4;
    if (shm <= 160 * 1024) {  // (>= 8.5 KiB: the BIAS partials reuse the images)
      const dim3 fg(B * H), fb(64 * std::max(8, nkp / 16));
      if (bias_part) {  // the QKV bias gradient's per-(image, head) column sums, [B][3 H 64]
        a.dbias_part = bias_part;
        a.dbias_ld = (int64_t)3 * H * hd;
        *bias_fused = true;
        switch (mode) {
          case 0: return launch_dyn(attn_bwd_fused64<0, true>, fg, fb, shm, st, a, "attn_bwd_fused64");
          case 1: return launch_dyn(attn_bwd_fused64<1, true>, fg, fb, shm, st, a, "attn_bwd_fused64");
          case 2: return launch_dyn(attn_bwd_fused64<2, true>, fg, fb, shm, st, a, "attn_bwd_fused64");
          default: return launch_dyn(attn_bwd_fused64<3, true>, fg, fb, shm, st, a, "attn_bwd_fused64");
        }
      }
      switch (mode) {
        case 0: return launch_dyn(attn_bwd_fused64<0>, fg, fb, shm, st, a, "attn_bwd_fused64");
        case 1: return launch_dyn(attn_bwd_fused64<1>, fg, fb, shm, st, a, "attn_bwd_fused64");
        case 2: return launch_dyn(attn_bwd_fused64<2>, fg, fb, shm, st, a, "attn_bwd_fused64");
        default: return launch_dyn(attn_bwd_fused64<3>, fg, fb, shm, st, a, "attn_bwd_fused64");
      }
    }
  }
  {
    // split backward: dK/dV kernel, then dQ kernel (two head images in LDS each)
    static const int wpe = [] { const char* e = getenv("CAPK_ATTN_WPE"); return e ? atoi(e) : 4; }();
    // the bias sums ride on the dK/dV kernel (<= 128-VGPR build only): per-wave rows after the images
    const bool bias = bias_part && wpe == 4 && hdp <= 128;
    const size_t s1 = bwd_kv_smem(Nq, hdp) + (bias ? (size_t)((Nk + 31) & ~31) * sizeof(float) : 0);
    const size_t s2 = fwd_kernel_smem(Nk, hdp);
    // (measured: ViT N=197 bwd 554 -> 460 us; for Nq <= 32 the second launch costs more than it saves)
    if (Nq > 32 && s1 <= 80 * 1024 && s2 <= 80 * 1024) {
      if (bias) {
        a.dbias_part = bias_part;
        a.dbias_ld = (int64_t)3 * H * hd;
        a.rsum = bias_part + (size_t)B * 3 * H * hd;
        *bias_fused = true;
      }
#define KV4(HD, M) rc2 = launch_dyn(attn_bwd_kv_bf16<HD, 4, M>, grid, block, s1, st, a, "attn_bwd_kv_bf16")
#define KV4B(HD, M) rc2 = launch_dyn(attn_bwd_kv_bf16<HD, 4, M, true>, grid, block, s1, st, a, "attn_bwd_kv_bf16")
#define KV2(HD, M) rc2 = launch_dyn(attn_bwd_kv_bf16<HD, 2, M>, grid, block, s1, st, a, "attn_bwd_kv_bf16")
#define QK(HD, M) rc2 = launch_dyn(attn_bwd_q_bf16<HD, M>, grid, block, s2, st, a, "attn_bwd_q_bf16")
#define QKB(HD, M) rc2 = launch_dyn(attn_bwd_q_bf16<HD, M, true>, grid, block, s2, st, a, "attn_bwd_q_bf16")
#define KV4M(M) BY_HDP(KV4, M)
#define KV4BM(M) BY_HDP(KV4B, M)
#define KV2M(M) BY_HDP(KV2, M)
#define QKM(M) BY_HDP(QK, M)
#define QKBM(M) BY_HDP(QKB, M)
      // CAPK_ATTN_BWD_SLICE=n: the two kernels alternate over slices of n images, so the dQ
      // kernel re-reads a slice's Q / K / V / O / dO while the Infinity Cache still holds them
      static const int env_slice = [] { const char* e = getenv("CAPK_ATTN_BWD_SLICE"); return e ? atoi(e) : 0; }();
      const int slice = g_bwd_slice >= 0 ? g_bwd_slice : env_slice;
      const int sl = slice > 0 && slice < B ? slice : B;
      const size_t es = 2;  // bf16
      const AttnArgs base = a;
      for (int b0 = 0; b0 < B; b0 += sl) {
        const int nb = std::min(sl, B - b0);
        AttnArgs a = base;
        const dim3 grid(nb * H);
        a.B = nb;
        a.b_base = b0;
        a.q = (const char*)base.q + (size_t)b0 * q_bs * es;
        a.k = (const char*)base.k + (size_t)b0 * k_bs * es;
        a.v = (const char*)base.v + (size_t)b0 * v_bs * es;
        a.o = (const char*)base.o + (size_t)b0 * o_bs * es;
        a.dout = (const char*)base.dout + (size_t)b0 * do_bs * es;
        a.dq = (char*)base.dq + (size_t)b0 * dq_bs * es;
        a.dk = (char*)base.dk + (size_t)b0 * dk_bs * es;
        a.dv = (char*)base.dv + (size_t)b0 * dv_bs * es;
        a.lse_in = base.lse_in + (size_t)b0 * H * Nq;
        if (base.key_pad) a.key_pad = base.key_pad + (size_t)b0 * Nk;
        if (bias) {
          a.dbias_part = base.dbias_part + (size_t)b0 * base.dbias_ld;
          a.rsum = base.rsum + (size_t)b0 * H * 2 * Nq;
        }
        if (bias) {
          BY_MODE(KV4BM)
        } else if (wpe == 4) {  // <= 128 VGPRs: two workgroups per CU
          BY_MODE(KV4M)
        } else {
          BY_MODE(KV2M)
        }
        if (rc2) return rc2;
        if (bias) {
          BY_MODE(QKBM)
        } else {
          BY_MODE(QKM)
        }
        if (rc2) return rc2;
      }
      return rc2;
    }
  }
  const size_t shm = bwd_smem(Nq, Nk, hdp);
  CAPK_CHECK_ARG(shm <= 160 * 1024, "capk_attention_bwd: LDS %zu > 160 KiB", shm);
#define FB(HD, M) rc2 = launch_dyn(attn_bwd_bf16<HD, M>, grid, block, shm, st, a, "attn_bwd_bf16")
#define FBM(M) BY_HDP(FB, M)
  BY_MODE(FBM)
  return rc2;
#undef FB
#undef FBM
#undef KV4
#undef KV4B
#undef KV2
#undef QK
#undef QKB
#undef QKBM
#undef KV4M
#undef KV4BM
#undef KV2M
#undef QKM
#undef BY_HDP
#undef BY_MODE
}


extern "C" int capk_attention_bwd(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, int causal,
                                  const void* q, int64_t q_bs, int64_t q_rs, const void* k, int64_t k_bs,
                                  int64_t k_rs, const void* v, int64_t v_bs, int64_t v_rs, const uint8_t* key_pad,
                                  const void* o, int64_t o_bs, int64_t o_rs, const void* dout, int64_t do_bs,
                                  int64_t do_rs, const float* lse, void* dq, int64_t dq_bs, int64_t dq_rs, void* dk,
                                  int64_t dk_bs, int64_t dk_rs, void* dv, int64_t dv_bs, int64_t dv_rs,
                                  float drop_p, uint32_t drop_seed, void* stream) {
  return attention_bwd_impl(dtype, B, H, Nq, Nk, hd, scale, causal, q, q_bs, q_rs, k, k_bs, k_rs, v, v_bs, v_rs,
                            key_pad, o, o_bs, o_rs, dout, do_bs, do_rs, lse, dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv,
                            dv_bs, dv_rs, drop_p, drop_seed, stream, nullptr, nullptr);
}

extern "C" int capk_attention_set_fused_bwd(int mode) {
  CAPK_CHECK_ARG(mode >= -1 && mode <= 1, "capk_attention_set_fused_bwd: mode must be -1, 0 or 1");
  g_fused_bwd = mode;
  return CAPK_OK;
}

// Test support: every CU's LDS filled with one 32-bit pattern (e.g. a NaN or -inf), so that
// a following kernel that reads LDS words it never wrote shows it (LDS is not cleared between
// workgroups).  4 x 256 workgroups of 40 KiB each (four per CU), plain vector LDS stores.
__global__ __launch_bounds__(256) void debug_fill_lds_kernel(uint32_t pattern) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* w = (uint32_t*)smem;
  for (int i = threadIdx.x; i < 40 * 1024 / 4; i += blockDim.x) w[i] = pattern;
  __syncthreads();
  const uint32_t back = w[(threadIdx.x * 37) % (40 * 1024 / 4)];
  asm volatile("" ::"v"(back));  // a live read keeps the stores
}

extern "C" int capk_debug_fill_lds(uint32_t pattern, void* stream) {
  hipLaunchKernelGGL(debug_fill_lds_kernel, dim3(4 * 256), dim3(256), 40 * 1024, S(stream), pattern);
  CAPK_LAUNCH_CHECK("debug_fill_lds_kernel");
  return CAPK_OK;
}

extern "C" int capk_attention_set_bwd_slice(int images) {
  CAPK_CHECK_ARG(images >= -1, "capk_attention_set_bwd_slice: images must be >= -1");
  g_bwd_slice = images;
  return CAPK_OK;
}

extern "C" size_t capk_attention_bwd_bias_workspace(int B, int H, int Nq, int Nk, int hd) {
  const int D = H * hd;
  const size_t fused = ((size_t)B * 3 * D + (size_t)B * H * 2 * Nq) * sizeof(float);
  const size_t sep = capk_colsum_workspace(B * std::max(Nq, Nk), D);
  return std::max(fused, sep);
}

extern "C" int capk_attention_bwd_bias(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, int causal,
                                       const void* q, int64_t q_bs, int64_t q_rs, const void* k, int64_t k_bs,
                                       int64_t k_rs, const void* v, int64_t v_bs, int64_t v_rs, const uint8_t* key_pad,
                                       const void* o, int64_t o_bs, int64_t o_rs, const void* dout, int64_t do_bs,
                                       int64_t do_rs, const float* lse, void* dq, int64_t dq_bs, int64_t dq_rs,
                                       void* dk, int64_t dk_bs, int64_t dk_rs, void* dv, int64_t dv_bs,
                                       int64_t dv_rs, float drop_p, uint32_t drop_seed, float* dbias, int accumulate,
                                       void* ws, size_t ws_bytes, void* stream) {
  CAPK_CHECK_ARG(dbias != nullptr, "capk_attention_bwd_bias: dbias is NULL");
  const int D = H * hd;
  CAPK_CHECK_ARG(ws && ws_bytes >= capk_attention_bwd_bias_workspace(B, H, Nq, Nk, hd),
                 "capk_attention_bwd_bias: workspace too small");
  bool fused = false;
  int rc = attention_bwd_impl(dtype, B, H, Nq, Nk, hd, scale, causal, q, q_bs, q_rs, k, k_bs, k_rs, v, v_bs, v_rs,
                              key_pad, o, o_bs, o_rs, dout, do_bs, do_rs, lse, dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv,
                              dv_bs, dv_rs, drop_p, drop_seed, stream, (float*)ws, &fused);
  if (rc) return rc;
  if (fused) return launch_colsum_finish(B, 3 * D, (const float*)ws, dbias, accumulate, S(stream));
  // other routes: column sums of the three gradient views (row-uniform: batch stride = rows * row stride)
  CAPK_CHECK_ARG(dq_bs == (int64_t)Nq * dq_rs && dk_bs == (int64_t)Nk * dk_rs && dv_bs == (int64_t)Nk * dv_rs,
                 "capk_attention_bwd_bias: gradient views must be row-uniform ([B*N, ld])");
  rc = capk_colsum(dtype, B * Nq, D, dq, dq_rs, dbias, accumulate, ws, ws_bytes, stream);
  if (!rc) rc = capk_colsum(dtype, B * Nk, D, dk, dk_rs, dbias + D, accumulate, ws, ws_bytes, stream);
  if (!rc) rc = capk_colsum(dtype, B * Nk, D, dv, dv_rs, dbias + 2 * D, accumulate, ws, ws_bytes, stream);
  return rc;
}
