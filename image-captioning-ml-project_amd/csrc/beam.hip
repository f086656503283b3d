// Beam search on the device.
//
// Semantics: transformers 5.15 GenerationMixin._beam_search
// (transformers/generation/utils.py:3208-3535), decoder-only, prompt length 1,
// one EOS id, MaxLength + EOS stopping — the search GPT2Decoder.generate reaches
// (src/models/decoders.py:645-654) and, per SURVEY D16, the one applied to every
// decoder through a per-step logits callback.
//
// One step = two kernels:
//   beam_rows_kernel   grid = B*k rows, 256 threads.  Streams one row of logits
//                      (V valid columns of a padded row) once from HBM: online
//                      max / sum-exp (log_softmax statistics) and the row's top-2k
//                      logits.  Within a row log_softmax(x) + running_score is
//                      monotone in x, so the image's top-2k over [k*V] is contained
//                      in the union of its rows' top-2k.
//   beam_update_kernel grid = B, one wave.  Candidate scores
//                      ((x - max) - logsum) + running_score exactly as torch
//                      log_softmax + add, top-2k (score desc, flat index asc),
//                      EOS / max-length hits, next running beams (top-k after the
//                      -1e9 penalty), finished-beam merge with the length penalty,
//                      early-stop heuristic, and the cache-reorder indices.
// All search state (running/finished sequences, scores, beam indices, flags)
// lives in one device buffer; the host reads 3 flag words per step to decide
// whether to continue (HF's batch-global stopping rule).
#include "common.h"

namespace capk {

static constexpr int BEAM_KMAX = 8;            // num_beams <= 8
static constexpr int BEAM_K2MAX = 2 * BEAM_KMAX;
static constexpr int BEAM_LMAX = 256;          // max_length <= 256
static constexpr int ROWS_THREADS = 256;

struct BeamState {
  int* flags;      // [4]: any improvement possible, any batch not all finished, any valid continuation
  int* rseq;       // [B][k][L] running sequences
  float* rscore;   // [B][k]
  int* rbi;        // [B][k][L-1] running beam indices
  int* seq;        // [B][k][L] finished sequences
  float* score;    // [B][k]
  int* bi;         // [B][k][L-1]
  int* fin;        // [B][k]
  int* unsat;      // [B]
};

__host__ __device__ inline size_t al64(size_t x) { return (x + 63) & ~(size_t)63; }

__host__ __device__ inline size_t beam_layout(int B, int k, int L, char* base, BeamState* s) {
  size_t off = 0;
  auto take = [&](size_t bytes) { char* p = base + off; off += al64(bytes); return p; };
  const size_t Bk = (size_t)B * k;
  char* p;
  p = take(16);                          if (s) s->flags = (int*)p;
  p = take(Bk * L * 4);                  if (s) s->rseq = (int*)p;
  p = take(Bk * 4);                      if (s) s->rscore = (float*)p;
  p = take(Bk * (L - 1) * 4);            if (s) s->rbi = (int*)p;
  p = take(Bk * L * 4);                  if (s) s->seq = (int*)p;
  p = take(Bk * 4);                      if (s) s->score = (float*)p;
  p = take(Bk * (L - 1) * 4);            if (s) s->bi = (int*)p;
  p = take(Bk * 4);                      if (s) s->fin = (int*)p;
  p = take((size_t)B * 4);               if (s) s->unsat = (int*)p;
  // per-row candidates written by beam_rows_kernel
  return off;
}

// candidate scratch after the state: [B*k][K2] values + tokens, [B*k] max, logsum
__host__ __device__ inline size_t beam_scratch_bytes(int B, int k) {
  const size_t Bk = (size_t)B * k;
  return al64(Bk * 2 * k * 4) * 2 + al64(Bk * 4) * 2;
}

// order-preserving float -> uint32 (larger float -> larger key)
__device__ __forceinline__ uint32_t fkey(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float funkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}
// (value desc, index asc) as one u64 maximised
__device__ __forceinline__ uint64_t ckey(float v, int idx) {
  return ((uint64_t)fkey(v) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)idx);
}
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int o) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = __shfl_xor(lo, o, 64);
  hi = __shfl_xor(hi, o, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = shfl_xor_u64(v, o);
    v = w > v ? w : v;
  }
  return v;
}

// merge (m, s) log-sum-exp partials; m = -inf means empty
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; s = s2; return; }
  if (m2 > m) { s = s * __expf(m - m2) + s2; m = m2; }
  else s += s2 * __expf(m2 - m);
}

// Per-wave candidate filter: a wave streams 512 contiguous logits per iteration (8 per
// lane, 16-B loads); an element enters the wave's LDS candidate buffer only if its
// (value, -index) key is >= the wave threshold (the K2-th best key seen so far), which
// makes appends rare after the first chunk; the buffer is compacted to its K2 best
// (rank counting) when it could overflow.  All control flow on the filter is
// wave-uniform (ballots), so there is no per-lane insertion divergence.
static constexpr int WAVE_CAP = 128;
static constexpr int RPD = 4;  // logits chunk loads in flight per wave

template <typename T> struct RawRow8;
template <> struct RawRow8<bf16> {
  bf16x8 a;
  __device__ __forceinline__ void load(const bf16* p) { a = *(const bf16x8*)p; }
  __device__ __forceinline__ void cvt(float (&v)[8]) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)a[j];
  }
};
template <> struct RawRow8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) { a = *(const f32x4*)p; b = *(const f32x4*)(p + 4); }
  __device__ __forceinline__ void cvt(float (&v)[8]) const {
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  }
};

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// keep the K2 best of wb[0..cnt) in wb[0..K2) sorted descending; returns new count
__device__ __forceinline__ int wave_compact(uint64_t* wb, int cnt, int K2, int lane) {
  const uint64_t a0 = lane < cnt ? wb[lane] : 0, a1 = lane + 64 < cnt ? wb[lane + 64] : 0;
  int r0 = 0, r1 = 0;
  for (int e = 0; e < cnt; ++e) {
    const uint64_t x = wb[e];
    r0 += x > a0;
    r1 += x > a1;
  }
  __builtin_amdgcn_wave_barrier();
  if (a0 && r0 < K2) wb[r0] = a0;
  if (a1 && r1 < K2) wb[r1] = a1;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return cnt < K2 ? cnt : K2;
}

template <typename T>
__global__ __launch_bounds__(ROWS_THREADS) void beam_rows_kernel(const T* __restrict__ logits, int64_t ld, int V,
                                                                 int K2, int* flags, float* cand_val, int* cand_tok,
                                                                 float* row_max, float* row_logsum, int cur_len,
                                                                 int early_true) {
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (r == 0 && tid == 0) {
    // HF's batch-global stopping rule on the previous step's flags, made sticky in flags[3]:
    // a replayed chunk of steps (capk/graphs.py) that runs past the host's stop point then
    // leaves the search state untouched (beam_update_kernel returns at once).
    if (cur_len > 1 && !(flags[0] && !(early_true && !flags[1]) && flags[2])) flags[3] = 1;
    flags[0] = flags[1] = flags[2] = 0;
  }
  const T* x = logits + (int64_t)r * ld;
  __shared__ uint64_t wbuf[4][WAVE_CAP];
  __shared__ float sm[4], ss[4];
  uint64_t* wb = wbuf[w];
  float m = -INFINITY, s = 0.f;
  // thr: the K2-th best (value, -index) key buffered so far; thr_f its value, a float
  // pre-filter (v >= thr_f keeps every key >= thr; offer() applies the exact test)
  uint64_t thr = 0;
  float thr_f = -INFINITY;
  auto set_thr = [&](uint64_t t) {
    thr = t;
    thr_f = t ? funkey((uint32_t)(t >> 32)) : -INFINITY;
  };
  int cnt = 0;
  auto offer = [&](uint64_t key) {  // wave-uniform call
    bool p = key != 0 && key >= thr;
    uint64_t mask = __ballot(p);
    if (!mask) return;
    if (cnt + 64 > WAVE_CAP) {
      cnt = wave_compact(wb, cnt, K2, lane);
      if (cnt == K2) set_thr(wb[K2 - 1]);
      p = key != 0 && key >= thr;
      mask = __ballot(p);
      if (!mask) return;
    }
    if (p) wb[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0))] = key;
    cnt += __popcll(mask);
  };
  const int V8 = V & ~7;
  bool first = true;
  // One 512-logit chunk (8 per lane at column i).  FULL: every lane in range (all chunks but
  // a row's last), so the -inf masking and the validity exec mask are compiled out.  Keys are
  // built only for the wave's first chunk (threshold seed) and for elements that pass the
  // float pre-filter; each pass of the offer loop takes one such element per lane.
  auto process = [&](auto full_tag, float (&v)[8], int i) {
    constexpr bool FULL = decltype(full_tag)::value;
    const bool valid = FULL || i < V8;
    if (!FULL && !valid) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = -INFINITY;
    }
    float cm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) cm = fmaxf(cm, v[j]);
    if (valid) {
      if (cm > m) { s = (m == -INFINITY) ? 0.f : s * __expf(m - cm); m = cm; }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
    }
    if (first) {  // threshold from the K2-th best lane maximum of the first chunk
      first = false;
      uint64_t kmax = 0;
      if (valid) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { const uint64_t kk = ckey(v[j], i + j); kmax = kk > kmax ? kk : kmax; }
      }
      int rank = 0;
      for (int o = 0; o < 64; ++o) rank += readlane_u64(kmax, o) > kmax;
      const uint64_t ball = __ballot(kmax != 0 && rank == K2 - 1);
      set_thr(ball ? readlane_u64(kmax, __builtin_ctzll(ball)) : 0);
    }
    // offer() raises the threshold only after a compaction, and a key it then drops is below
    // K2 buffered keys, so filtering against the threshold of the moment is exact
    if (__ballot(valid && cm >= thr_f)) {
      uint32_t qm = 0;
      if (valid) {
#pragma unroll
        for (int j = 0; j < 8; ++j) qm |= v[j] >= thr_f ? (1u << j) : 0u;
      }
      while (__ballot(qm != 0)) {
        const int jq = qm ? __builtin_ctz(qm) : 0;
        float vq = v[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) vq = j == jq ? v[j] : vq;
        const uint64_t key = qm ? ckey(vq, i + jq) : 0;
        qm &= qm - 1;
        offer(key);
      }
    }
  };
  // Chunk q of wave w covers [w*512 + q*2048, +512).  RPD chunk loads stay in flight per
  // wave: raw 16-B registers, issued unconditionally (lanes past V8 read the row start and
  // are masked after the load), so no exec-masked branch forces a wait right after the load.
  const int c_first = __builtin_amdgcn_readfirstlane(w) * 512;  // wave-uniform (scalar loop control)
  const int nq = c_first < V8 ? (V8 - c_first + 2047) / 2048 : 0;
  RawRow8<T> buf[RPD];
  auto issue = [&](int q, RawRow8<T>& d) {
    const int i = c_first + q * 2048 + lane * 8;
    d.load(x + (i < V8 ? i : 0));
  };
  // the chunk count is rounded up to a multiple of RPD: chunks past the row are all-invalid
  // (their loads hit the row's first line), which keeps every load unconditional
  // (a row shorter than one chunk, V8 == 0, issues nothing: a 16-B load at the row start would
  // read past a short last row)
  if (V8 > 0) {
#pragma unroll
    for (int sl = 0; sl < RPD; ++sl) issue(sl, buf[sl]);
  }
  for (int q0 = 0; q0 < nq; q0 += RPD) {
#pragma unroll
    for (int sl = 0; sl < RPD; ++sl) {
      const int q = q0 + sl;
      const int c0 = c_first + q * 2048;
      float v[8];
      buf[sl].cvt(v);
      issue(q + RPD, buf[sl]);
      if (c0 + 512 <= V8) process(std::true_type{}, v, c0 + lane * 8);
      else if (c0 < V8) process(std::false_type{}, v, c0 + lane * 8);
    }
  }
  for (int t0 = V8 + w * 64; t0 < V; t0 += 256) {  // tail (< 8 elements, one wave-uniform pass)
    const int i = t0 + lane;
    uint64_t key = 0;
    if (i < V) {
      const float v = to_f32(x[i]);
      if (v > m) { s = (m == -INFINITY) ? 0.f : s * __expf(m - v); m = v; }
      s += __expf(v - m);
      key = ckey(v, i);
    }
    offer(key);
  }
  cnt = wave_compact(wb, cnt, K2, lane);
  for (int j = cnt + lane; j < K2; j += 64) wb[j] = 0;
  // log-sum-exp statistics: wave, then block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
  if (lane == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (w == 0) {
    float M = sm[0], Ssum = ss[0];
    for (int q = 1; q < 4; ++q) lse_merge(M, Ssum, sm[q], ss[q]);
    // final top-K2 of the 4*K2 wave candidates by rank counting
    const int nc = 4 * K2;
    uint64_t mine = lane < nc ? wbuf[lane / K2][lane % K2] : 0;
    int rank = 0;
    for (int c = 0; c < nc; ++c) rank += wbuf[c / K2][c % K2] > mine;
    if (lane < nc && rank < K2 && mine != 0) {
      cand_val[(int64_t)r * K2 + rank] = funkey((uint32_t)(mine >> 32));
      cand_tok[(int64_t)r * K2 + rank] = (int)(0xFFFFFFFFu - (uint32_t)mine);
    }
    if (lane == 0) { row_max[r] = M; row_logsum[r] = logf(Ssum); }
  }
}

// ---------------------------------------------------------------- update ----
__global__ __launch_bounds__(64) void beam_update_kernel(BeamState st, int k, int L, int V, int cur_len, int eos,
                                                         float fin_div, float best_div, int early_true,
                                                         const float* __restrict__ cand_val,
                                                         const int* __restrict__ cand_tok,
                                                         const float* __restrict__ row_max,
                                                         const float* __restrict__ row_logsum, int* reorder,
                                                         int64_t* next_ids) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (st.flags[3]) return;  // the search already stopped (see beam_rows_kernel)
  const int K2 = 2 * k, Lb = L - 1;
  extern __shared__ int sh[];
  int* o_rseq = sh;                       // [k][L]
  int* o_rbi = o_rseq + k * L;            // [k][L-1]
  int* o_seq = o_rbi + k * Lb;            // [k][L]
  int* o_bi = o_seq + k * L;              // [k][L-1]
  __shared__ float t_lp[BEAM_K2MAX];      // top-2k accumulated log-probs
  __shared__ int t_beam[BEAM_K2MAX], t_tok[BEAM_K2MAX], t_hit[BEAM_K2MAX];
  __shared__ int nxt[BEAM_KMAX];          // running selection (index into top-2k)
  __shared__ int msel[BEAM_KMAX];         // finished selection (index into merged k + 2k)
  __shared__ float m_score[BEAM_KMAX + BEAM_K2MAX];
  __shared__ int m_fin[BEAM_KMAX + BEAM_K2MAX];
  __shared__ float n_rscore[BEAM_KMAX];
  __shared__ float t_trl[BEAM_K2MAX];
  const size_t sb = (size_t)b * k;
  // 0. stash the old sequences / indices of this image
  for (int e = lane; e < k * L; e += 64) { o_rseq[e] = st.rseq[sb * L + e]; o_seq[e] = st.seq[sb * L + e]; }
  for (int e = lane; e < k * Lb; e += 64) { o_rbi[e] = st.rbi[sb * Lb + e]; o_bi[e] = st.bi[sb * Lb + e]; }
  const int unsat_old = st.unsat[b];
  const int fin_l = lane < k ? st.fin[sb + lane] : 1;
  // 1. candidates: k rows x K2, score = ((x - max) - logsum) + running (torch log_softmax + add)
  const int nc = k * K2;  // <= 128
  float cs[2];
  uint64_t ck[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = lane + 64 * h;
    ck[h] = 0;
    cs[h] = 0.f;
    if (c < nc) {
      const int rr = c / K2;
      const int64_t row = (int64_t)sb + rr;
      const float xv = cand_val[row * K2 + (c % K2)];
      const int tok = cand_tok[row * K2 + (c % K2)];
      const float lp = (xv - row_max[row]) - row_logsum[row];
      cs[h] = lp + st.rscore[row];
      ck[h] = ckey(cs[h], rr * V + tok);
    }
  }
  // rank-count over all candidates (keys unique: flat index unique); the other lanes' keys
  // are read with v_readlane (uniform lane index), not a permute round trip per candidate
  int rk[2] = {0, 0};
  for (int c2 = 0; c2 < (nc < 64 ? nc : 64); ++c2) {
    const uint64_t o = readlane_u64(ck[0], c2);
    rk[0] += (o > ck[0]) ? 1 : 0;
    rk[1] += (o > ck[1]) ? 1 : 0;
  }
  for (int c2 = 64; c2 < nc; ++c2) {
    const uint64_t o = readlane_u64(ck[1], c2 - 64);
    rk[0] += (o > ck[0]) ? 1 : 0;
    rk[1] += (o > ck[1]) ? 1 : 0;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int rank = rk[h];
    const int c = lane + 64 * h;
    if (c < nc && rank < K2) {
      const int flat = (int)(0xFFFFFFFFu - (uint32_t)ck[h]);
      t_lp[rank] = cs[h];
      t_beam[rank] = flat / V;
      t_tok[rank] = flat % V;
    }
  }
  __syncthreads();
  // 2. stopping criteria per continuation; running log-probs with the -1e9 penalty
  const int full = __ballot(fin_l == 0) == 0;  // all k finished slots of this image taken
  if (lane < K2) {
    const int hit = (t_tok[lane] == eos) || (cur_len + 1 >= L);
    t_hit[lane] = hit;
    t_trl[lane] = t_lp[lane] + (hit ? -1.0e9f : -0.0f);
    // finished-candidate score: lp / len^lp, + full, + !unsat, + !just_finished penalties (utils.py:3175-3190)
    float sc = t_lp[lane] / fin_div;
    sc += (full && early_true) ? -1.0e9f : -0.0f;
    sc += unsat_old ? -0.0f : -1.0e9f;
    const int jf = hit && (lane < k);
    sc += jf ? -0.0f : -1.0e9f;
    m_score[k + lane] = sc;
    m_fin[k + lane] = jf;
  }
  if (lane < k) { m_score[lane] = st.score[sb + lane]; m_fin[lane] = fin_l; }
  __syncthreads();
  // 3. top-k running (ties: lower position first) and top-k finished over the merged list
  {
    const int nm = k + K2;
    const uint64_t me_r = lane < K2 ? ckey(t_trl[lane], lane) : 0;
    const uint64_t me_m = lane < nm ? ckey(m_score[lane], lane) : 0;
    int rank_r = 0, rank_m = 0;
    for (int j = 0; j < K2; ++j) rank_r += (readlane_u64(me_r, j) > me_r) ? 1 : 0;
    for (int j = 0; j < nm; ++j) rank_m += (readlane_u64(me_m, j) > me_m) ? 1 : 0;
    if (lane < K2 && rank_r < k) { nxt[rank_r] = lane; n_rscore[rank_r] = t_trl[lane]; }
    if (lane < nm && rank_m < k) msel[rank_m] = lane;
  }
  __syncthreads();
  // 4. write the new running state
  for (int e = lane; e < k * L; e += 64) {
    const int i = e / L, p = e % L, j = nxt[i];
    st.rseq[sb * L + e] = (p == cur_len) ? t_tok[j] : o_rseq[t_beam[j] * L + p];
  }
  for (int e = lane; e < k * Lb; e += 64) {
    const int i = e / Lb, p = e % Lb, j = nxt[i];
    st.rbi[sb * Lb + e] = (p == cur_len - 1) ? (int)sb + t_beam[j] : o_rbi[t_beam[j] * Lb + p];
  }
  if (lane < k) {
    const int j = nxt[lane];
    st.rscore[sb + lane] = n_rscore[lane];
    reorder[sb + lane] = (int)sb + t_beam[j];
    next_ids[sb + lane] = t_tok[j];
  }
  // 5. finished state from the merged selection
  for (int e = lane; e < k * L; e += 64) {
    const int i = e / L, p = e % L, mi = msel[i];
    int v;
    if (mi < k) v = o_seq[mi * L + p];
    else {
      const int j = mi - k;
      v = (p == cur_len) ? t_tok[j] : o_rseq[t_beam[j] * L + p];
    }
    st.seq[sb * L + e] = v;
  }
  for (int e = lane; e < k * Lb; e += 64) {
    const int i = e / Lb, p = e % Lb, mi = msel[i];
    int v;
    if (mi < k) v = o_bi[mi * Lb + p];
    else {
      const int j = mi - k;
      v = (p == cur_len - 1) ? (int)sb + t_beam[j] : o_rbi[t_beam[j] * Lb + p];
    }
    st.bi[sb * Lb + e] = v;
  }
  __syncthreads();
  if (lane == 0) {
    // 6. finished scores/flags, early-stop heuristic (utils.py:3008-3053), global flags
    float worst = 3.4e38f;
    int all_fin = 1;
    float nsc[BEAM_KMAX];
    int nfin[BEAM_KMAX];
    for (int i = 0; i < k; ++i) {
      nsc[i] = m_score[msel[i]];
      nfin[i] = m_fin[msel[i]];
      st.score[sb + i] = nsc[i];
      st.fin[sb + i] = nfin[i];
      worst = fminf(worst, nsc[i]);
      all_fin &= nfin[i];
    }
    const float best_running = n_rscore[0] / best_div;
    int any = 0;
    for (int i = 0; i < k; ++i) any |= best_running > (nfin[i] ? worst : -1.0e9f);
    const int unsat_new = unsat_old && any;
    st.unsat[b] = unsat_new;
    int any_valid = 0;
    for (int j = 0; j < K2; ++j) any_valid |= !t_hit[j];
    if (unsat_new) atomicOr(&st.flags[0], 1);
    if (!all_fin) atomicOr(&st.flags[1], 1);
    if (any_valid) atomicOr(&st.flags[2], 1);
  }
}

__global__ void beam_init_kernel(BeamState st, int B, int k, int L, const int64_t* prompt, int fill) {
  const int64_t n = (int64_t)B * k * L;
  if (blockIdx.x == 0 && threadIdx.x < 4) st.flags[threadIdx.x] = 0;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(e % L);
    const int b = (int)(e / ((int64_t)k * L));
    const int v = p == 0 ? (int)prompt[b] : fill;
    st.rseq[e] = v;
    st.seq[e] = v;
    const int64_t row = e / L;
    if (p < L - 1) { st.rbi[row * (L - 1) + p] = -1; st.bi[row * (L - 1) + p] = -1; }
    if (p == 0) {
      st.rscore[row] = (row % k) == 0 ? 0.f : -1.0e9f;
      st.score[row] = -1.0e9f;
      st.fin[row] = 0;
      if (row % k == 0) st.unsat[b] = 1;
    }
  }
}

__global__ void beam_finalize_kernel(BeamState st, int B, int k, int L, int64_t* sequences, float* scores,
                                     int* beam_indices) {
  const int64_t n = (int64_t)B * k * L;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    sequences[e] = st.seq[e];
    const int p = (int)(e % L);
    const int64_t row = e / L;
    if (p < L - 1) beam_indices[row * (L - 1) + p] = st.bi[row * (L - 1) + p];
    if (p == 0) scores[row] = st.score[row];
  }
}

template <typename T>
__global__ void gather_rows_kernel(int G, int R, int cols, const int* __restrict__ idx, const T* __restrict__ x,
                                   int64_t ldx, int64_t gsx, T* __restrict__ y, int64_t ldy, int64_t gsy) {
  const int c8 = cols / 8;
  const int64_t n = (int64_t)G * R * c8;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % c8) * 8;
    const int64_t gr = e / c8;
    const int r = (int)(gr % R), g = (int)(gr / R);
    float v[8];
    Vec8<T>::load(x + g * gsx + (int64_t)idx[r] * ldx + c, v);
    Vec8<T>::store(y + g * gsy + (int64_t)r * ldy + c, v);
  }
}


// Row-wise argmax over the V valid columns of a padded row (greedy decoding:
// logits.argmax(dim=-1), first index on ties like torch).
template <typename T>
__global__ __launch_bounds__(256) void argmax_rows_kernel(const T* __restrict__ x, int64_t ld, int V,
                                                          int64_t* __restrict__ out, int64_t out_stride) {
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const T* row = x + (int64_t)r * ld;
  uint64_t best = 0;
  for (int i = tid; i < V; i += 256) {
    const uint64_t k = ckey(to_f32(row[i]), i);
    best = k > best ? k : best;
  }
  best = wave_max_u64(best);
  __shared__ uint64_t sb[4];
  if (lane == 0) sb[w] = best;
  __syncthreads();
  if (tid == 0) {
    uint64_t b = sb[0];
    for (int q = 1; q < 4; ++q) b = sb[q] > b ? sb[q] : b;
    out[(int64_t)r * out_stride] = (int64_t)(0xFFFFFFFFu - (uint32_t)b);
  }
}


// Categorical sampling from softmax(logits[r, :V]) by inverse CDF with a counter-based
// uniform u = hash(seed, step<<32 | r) (SCST sampler, trainer.py:383-438 restated: the
// distribution of torch.distributions.Categorical(softmax(logits)), a reproducible RNG
// stream instead of torch.multinomial's).  Thread t owns the contiguous columns
// [t*chunk, (t+1)*chunk); the CDF is the in-order sum of exp(x - max) over threads'
// chunks (block exclusive scan), so the oracle can restate it exactly.
__global__ __launch_bounds__(256) void sample_rows_kernel_f32(const float* __restrict__ x0, int64_t ld, int V,
                                                              uint32_t seed, int step, int64_t* __restrict__ out,
                                                              int64_t out_stride, float* __restrict__ logp,
                                                              int is_bf16, const uint32_t* __restrict__ seedp) {
  if (seedp) seed = *seedp;
  const int r = blockIdx.x, tid = threadIdx.x;
  const int chunk = (V + 255) / 256;
  const int lo = tid * chunk, hi = min(V, lo + chunk);
  const float* xf = x0 + (is_bf16 ? 0 : (int64_t)r * ld);
  const bf16* xb = (const bf16*)x0 + (is_bf16 ? (int64_t)r * ld : 0);
  auto X = [&](int i) { return is_bf16 ? (float)xb[i] : xf[i]; };
  __shared__ float red[4];
  __shared__ float pre[257];
  float m = -INFINITY;
  for (int i = lo; i < hi; ++i) m = fmaxf(m, X(i));
  m = wave_max(m);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  const float M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sl = 0.f;
  for (int i = lo; i < hi; ++i) sl += __expf(X(i) - M);
  pre[tid + 1] = sl;
  __syncthreads();
  if (tid == 0) {
    pre[0] = 0.f;
    for (int t = 1; t <= 256; ++t) pre[t] += pre[t - 1];
  }
  __syncthreads();
  const float S = pre[256];
  const uint32_t h = drop_hash(seed, ((uint64_t)(uint32_t)step << 32) | (uint32_t)r);
  const float target = (float)(h >> 8) * (1.0f / 16777216.0f) * S;
  // the owning thread: pre[t] <= target < pre[t+1]; rounding past the end -> last non-empty chunk
  const bool own = (pre[tid] <= target && target < pre[tid + 1]) ||
                   (tid == min(255, (V - 1) / chunk) && target >= pre[tid + 1]);
  if (own && lo < hi) {
    float cum = pre[tid];
    int tok = hi - 1;
    for (int i = lo; i < hi; ++i) {
      cum += __expf(X(i) - M);
      if (cum > target) { tok = i; break; }
    }
    out[(int64_t)r * out_stride] = tok;
    if (logp) logp[r] = (X(tok) - M) - logf(S);
  }
}

// bf16 rows up to SAMPLE_LDS_MAX elements: the same arithmetic (per-thread contiguous chunks
// summed in order) on a row staged once in LDS with coalesced 16-B loads -- the chunk-owner
// layout reads global memory 197 elements apart per lane, and three passes re-read it.
constexpr int SAMPLE_LDS_MAX = 65536;  // 128 KiB of LDS
__global__ __launch_bounds__(256) void sample_rows_lds_kernel(const bf16* __restrict__ x0, int64_t ld, int V,
                                                              uint32_t seed, int step, int64_t* __restrict__ out,
                                                              int64_t out_stride, float* __restrict__ logp,
                                                              const uint32_t* __restrict__ seedp) {
  if (seedp) seed = *seedp;
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  bf16* row = (bf16*)dyn;
  const int r = blockIdx.x, tid = threadIdx.x;
  const bf16* xr = x0 + (int64_t)r * ld;
  const int v8 = V & ~7;
  for (int i = tid * 8; i < v8; i += 256 * 8) *(bf16x8*)(row + i) = *(const bf16x8*)(xr + i);
  for (int i = v8 + tid; i < V; i += 256) row[i] = xr[i];
  __syncthreads();
  const int chunk = (V + 255) / 256;
  const int lo = tid * chunk, hi = min(V, lo + chunk);
  __shared__ float red[4];
  __shared__ float pre[257];
  float m = -INFINITY;
  for (int i = lo; i < hi; ++i) m = fmaxf(m, (float)row[i]);
  m = wave_max(m);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  const float M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sl = 0.f;
  for (int i = lo; i < hi; ++i) sl += __expf((float)row[i] - M);
  pre[tid + 1] = sl;
  __syncthreads();
  if (tid == 0) {
    pre[0] = 0.f;
    for (int t = 1; t <= 256; ++t) pre[t] += pre[t - 1];
  }
  __syncthreads();
  const float S = pre[256];
  const uint32_t h = drop_hash(seed, ((uint64_t)(uint32_t)step << 32) | (uint32_t)r);
  const float target = (float)(h >> 8) * (1.0f / 16777216.0f) * S;
  const bool own = (pre[tid] <= target && target < pre[tid + 1]) ||
                   (tid == min(255, (V - 1) / chunk) && target >= pre[tid + 1]);
  if (own && lo < hi) {
    float cum = pre[tid];
    int tok = hi - 1;
    for (int i = lo; i < hi; ++i) {
      cum += __expf((float)row[i] - M);
      if (cum > target) { tok = i; break; }
    }
    out[(int64_t)r * out_stride] = tok;
    if (logp) logp[r] = ((float)row[tok] - M) - logf(S);
  }
}

static int grid_of(int64_t work) {
  int64_t g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace capk

using namespace capk;

extern "C" size_t capk_beam_state_bytes(int B, int num_beams, int max_length) {
  if (B <= 0 || num_beams <= 0 || max_length < 2) return 0;
  return beam_layout(B, num_beams, max_length, nullptr, nullptr) + beam_scratch_bytes(B, num_beams);
}

static int check_dims(int B, int k, int L, const char* who) {
  CAPK_CHECK_ARG(B > 0 && k >= 1 && k <= BEAM_KMAX && L >= 2 && L <= BEAM_LMAX, "%s: need B>0, 1<=num_beams<=%d, "
                 "2<=max_length<=%d (got B=%d k=%d L=%d)", who, BEAM_KMAX, BEAM_LMAX, B, k, L);
  return CAPK_OK;
}

extern "C" int capk_beam_init(int B, int num_beams, int max_length, const int64_t* prompt, int64_t fill, void* state,
                              size_t state_bytes, void* stream) {
  if (int rc = check_dims(B, num_beams, max_length, "capk_beam_init")) return rc;
  CAPK_CHECK_ARG(state && prompt && state_bytes >= capk_beam_state_bytes(B, num_beams, max_length),
                 "capk_beam_init: state buffer too small");
  BeamState st;
  beam_layout(B, num_beams, max_length, (char*)state, &st);
  hipLaunchKernelGGL(beam_init_kernel, dim3(grid_of((int64_t)B * num_beams * max_length)), dim3(256), 0, S(stream),
                     st, B, num_beams, max_length, prompt, (int)fill);
  CAPK_LAUNCH_CHECK("beam_init_kernel");
  return CAPK_OK;
}

extern "C" int capk_beam_step(int dtype, int B, int num_beams, int max_length, int V, int64_t ld, const void* logits,
                              int cur_len, int64_t eos, float fin_div, float best_div, int early_stopping,
                              void* state, size_t state_bytes, int32_t* reorder, int64_t* next_ids, void* stream) {
  if (int rc = check_dims(B, num_beams, max_length, "capk_beam_step")) return rc;
  const int k = num_beams, L = max_length;
  CAPK_CHECK_ARG(state && state_bytes >= capk_beam_state_bytes(B, k, L), "capk_beam_step: state buffer too small");
  CAPK_CHECK_ARG(V >= 2 * k && ld >= V && ld % 8 == 0 && cur_len >= 1 && cur_len < L && fin_div > 0.f &&
                 best_div > 0.f && (int64_t)k * V < 0x7FFFFFFF, "capk_beam_step: bad V/ld/cur_len/penalty");
  CAPK_CHECK_ARG(dtype == CAPK_F32 || dtype == CAPK_BF16, "capk_beam_step: dtype");
  BeamState st;
  const size_t sz = beam_layout(B, k, L, (char*)state, &st);
  char* scr = (char*)state + sz;
  const size_t Bk = (size_t)B * k;
  float* cand_val = (float*)scr;
  int* cand_tok = (int*)(scr + al64(Bk * 2 * k * 4));
  float* row_max = (float*)(scr + 2 * al64(Bk * 2 * k * 4));
  float* row_logsum = (float*)(scr + 2 * al64(Bk * 2 * k * 4) + al64(Bk * 4));
  hipStream_t s = S(stream);
  if (dtype == CAPK_F32)
    hipLaunchKernelGGL(beam_rows_kernel<float>, dim3((unsigned)Bk), dim3(ROWS_THREADS), 0, s, (const float*)logits,
                       ld, V, 2 * k, st.flags, cand_val, cand_tok, row_max, row_logsum, cur_len,
                       early_stopping == 1 ? 1 : 0);
  else
    hipLaunchKernelGGL(beam_rows_kernel<bf16>, dim3((unsigned)Bk), dim3(ROWS_THREADS), 0, s, (const bf16*)logits,
                       ld, V, 2 * k, st.flags, cand_val, cand_tok, row_max, row_logsum, cur_len,
                       early_stopping == 1 ? 1 : 0);
  CAPK_LAUNCH_CHECK("beam_rows_kernel");
  const size_t lds = (size_t)(2 * k * L + 2 * k * (L - 1)) * sizeof(int);
  hipLaunchKernelGGL(beam_update_kernel, dim3(B), dim3(64), lds, s, st, k, L, V, cur_len, (int)eos, fin_div,
                     best_div, early_stopping == 1 ? 1 : 0, cand_val, cand_tok, row_max, row_logsum, reorder,
                     next_ids);
  CAPK_LAUNCH_CHECK("beam_update_kernel");
  return CAPK_OK;
}

extern "C" int capk_beam_finalize(int B, int num_beams, int max_length, const void* state, int64_t* sequences,
                                  float* scores, int32_t* beam_indices, void* stream) {
  if (int rc = check_dims(B, num_beams, max_length, "capk_beam_finalize")) return rc;
  BeamState st;
  beam_layout(B, num_beams, max_length, (char*)state, &st);
  hipLaunchKernelGGL(beam_finalize_kernel, dim3(grid_of((int64_t)B * num_beams * max_length)), dim3(256), 0,
                     S(stream), st, B, num_beams, max_length, sequences, scores, beam_indices);
  CAPK_LAUNCH_CHECK("beam_finalize_kernel");
  return CAPK_OK;
}

extern "C" int capk_beam_flags(const void* state, int32_t* flags_out, void* stream) {
  CAPK_CHECK_ARG(state && flags_out, "capk_beam_flags: null");
  hipError_t e = hipMemcpyAsync(flags_out, state, 3 * sizeof(int32_t), hipMemcpyDeviceToHost, S(stream));
  if (e != hipSuccess) return hip_status(e, "capk_beam_flags");
  e = hipStreamSynchronize(S(stream));
  if (e != hipSuccess) return hip_status(e, "capk_beam_flags");
  return CAPK_OK;
}

extern "C" int capk_gather_rows(int dtype, int groups, int rows, int cols, const int32_t* idx, const void* x,
                                int64_t ldx, int64_t gsx, void* y, int64_t ldy, int64_t gsy, void* stream) {
  CAPK_CHECK_ARG(groups > 0 && rows > 0 && cols > 0 && cols % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 &&
                 gsx % 8 == 0 && gsy % 8 == 0, "capk_gather_rows: need cols/strides multiples of 8");
  const int64_t work = (int64_t)groups * rows * (cols / 8);
  if (dtype == CAPK_F32)
    hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(grid_of(work)), dim3(256), 0, S(stream), groups, rows, cols,
                       idx, (const float*)x, ldx, gsx, (float*)y, ldy, gsy);
  else if (dtype == CAPK_BF16)
    hipLaunchKernelGGL(gather_rows_kernel<bf16>, dim3(grid_of(work)), dim3(256), 0, S(stream), groups, rows, cols,
                       idx, (const bf16*)x, ldx, gsx, (bf16*)y, ldy, gsy);
  else CAPK_CHECK_ARG(false, "capk_gather_rows: dtype");
  CAPK_LAUNCH_CHECK("gather_rows_kernel");
  return CAPK_OK;
}

extern "C" int capk_argmax_rows(int dtype, int rows, int V, int64_t ld, const void* x, int64_t* out, int64_t out_stride,
                                void* stream) {
  CAPK_CHECK_ARG(rows > 0 && V > 0 && ld >= V, "capk_argmax_rows: bad sizes");
  if (dtype == CAPK_F32)
    hipLaunchKernelGGL(argmax_rows_kernel<float>, dim3(rows), dim3(256), 0, S(stream), (const float*)x, ld, V, out,
                       out_stride);
  else if (dtype == CAPK_BF16)
    hipLaunchKernelGGL(argmax_rows_kernel<bf16>, dim3(rows), dim3(256), 0, S(stream), (const bf16*)x, ld, V, out,
                       out_stride);
  else CAPK_CHECK_ARG(false, "capk_argmax_rows: dtype");
  CAPK_LAUNCH_CHECK("argmax_rows_kernel");
  return CAPK_OK;
}

static int sample_rows_launch(int dtype, int rows, int V, int64_t ld, const void* logits, uint32_t seed,
                              const uint32_t* seedp, int step, int64_t* out, int64_t out_stride, float* logp,
                              void* stream) {
  CAPK_CHECK_ARG(rows > 0 && V > 0 && ld >= V && (dtype == CAPK_F32 || dtype == CAPK_BF16),
                 "capk_sample_rows: bad arguments");
  if (dtype == CAPK_BF16 && V <= SAMPLE_LDS_MAX && ld % 8 == 0 && (uintptr_t)logits % 16 == 0) {
    const size_t lds = (size_t)((V + 7) & ~7) * sizeof(bf16);
    static const hipError_t attr = hipFuncSetAttribute((const void*)sample_rows_lds_kernel,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       SAMPLE_LDS_MAX * (int)sizeof(bf16));
    if (attr != hipSuccess) return hip_status(attr, "capk_sample_rows: hipFuncSetAttribute");
    hipLaunchKernelGGL(sample_rows_lds_kernel, dim3(rows), dim3(256), lds, S(stream), (const bf16*)logits, ld, V, seed,
                       step, out, out_stride, logp, seedp);
  } else {
    hipLaunchKernelGGL(sample_rows_kernel_f32, dim3(rows), dim3(256), 0, S(stream), (const float*)logits, ld, V, seed,
                       step, out, out_stride, logp, dtype == CAPK_BF16 ? 1 : 0, seedp);
  }
  CAPK_LAUNCH_CHECK("sample_rows_kernel");
  return CAPK_OK;
}

extern "C" int capk_sample_rows(int dtype, int rows, int V, int64_t ld, const void* logits, uint32_t seed, int step,
                                int64_t* out, int64_t out_stride, float* logp, void* stream) {
  return sample_rows_launch(dtype, rows, V, ld, logits, seed, nullptr, step, out, out_stride, logp, stream);
}

extern "C" int capk_sample_rows_dev(int dtype, int rows, int V, int64_t ld, const void* logits, const uint32_t* seed,
                                    int step, int64_t* out, int64_t out_stride, float* logp, void* stream) {
  CAPK_CHECK_ARG(seed != nullptr, "capk_sample_rows_dev: null seed");
  return sample_rows_launch(dtype, rows, V, ld, logits, 0u, seed, step, out, out_stride, logp, stream);
}
