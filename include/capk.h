/* capk — MI355X (gfx950) compute backend for the image-captioning hot path.
 *
 * C ABI of libcapk.so.  Plain pointers, sizes and strides; no torch types.
 * The reference (thromel/Image-Captioning-ML-Project) is pure Python whose
 * arithmetic runs inside torch / HF transformers modules; each entry point
 * below names the reference call site it replaces (file:line).
 *
 * Conventions
 *  - Return 0 on success, a negative CAPK_E* code on failure; the message of the
 *    last failure on this thread is capk_last_error().
 *  - dtype codes: CAPK_F32 (fp32 storage, fp32 arithmetic: the parity path) and
 *    CAPK_BF16 (bf16 storage, fp32 accumulation: the throughput path).
 *  - Strides are in ELEMENTS.  `stream` is a hipStream_t passed as void*.
 *  - The caller owns every buffer (inputs, outputs, workspaces).  No entry point
 *    allocates or frees device memory, synchronises the device or the stream,
 *    so every call is hipGraph-capturable.
 */
#ifndef CAPK_H
#define CAPK_H
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define CAPK_OK 0
#define CAPK_EINVAL (-1)      /* bad shape / stride / dtype / alignment          */
#define CAPK_EHIP (-2)        /* a HIP runtime call failed (message has details) */
#define CAPK_EUNSUPPORTED (-3)/* combination not implemented                     */

#define CAPK_F32 0
#define CAPK_BF16 1

/* epilogue activations (act argument of capk_gemm) */
#define CAPK_ACT_NONE 0
#define CAPK_ACT_GELU_ERF 1   /* HF "gelu" / torch F.gelu (ViT, nn.TransformerDecoderLayer) */
#define CAPK_ACT_GELU_TANH 2  /* HF "gelu_new" (GPT-2)                                      */
#define CAPK_ACT_QUICK_GELU 3 /* CLIP quick_gelu x*sigmoid(1.702x)                          */
#define CAPK_ACT_TANH 4       /* ViT pooler                                                 */
#define CAPK_ACT_RELU 5
#define CAPK_ACT_SIGMOID 6    /* AoA info gate, adaptive sentinel gate (attention.py:258,318) */
/* backward forms: out = acc * act'(aux) where aux is the saved pre-activation */
#define CAPK_ACT_BWD 16
#define CAPK_ACT_DERIV 32 /* forward: preact receives act'(pre) instead of pre; with CAPK_ACT_BWD:
                           aux already holds act'(pre), so v = pre * aux[m,n] (no activation math) */

const char* capk_last_error(void);
int capk_version(void);
int capk_device_arch(char* buf, int len); /* writes gcnArchName of the current device */

/* --------------------------------------------------------------- dropout ----
 * Dropout masks are never stored: keep(seed, idx) = fmix32(seed ^ mix(idx)) >= p*2^32
 * is recomputed wherever needed, scale 1/(1-p).  drop_p = 0 disables.  Index per site:
 *   GEMM epilogue: m*N + n of the output;  LN backward masked copy: row*cols + col;
 *   attention probabilities: ((b*H + h)*Nq + q)*Nk + key;  embedding: (b*T + t)*D + d.
 * capk_dropout_mask() materialises a mask for tests. */
int capk_dropout_mask(int64_t n, uint64_t offset, float p, uint32_t seed, uint8_t* out, void* stream);

/* ---------------------------------------------------------------- GEMM -----
 * pre[m,n] = alpha * sum_k A(m,k) * B(n,k) + beta * C[m,n] + bias[n]   (bias fp32, optional)
 * then  act:  CAPK_ACT_x              -> preact (optional) = pre, v = act(pre)
 *             CAPK_ACT_BWD|CAPK_ACT_x -> v = pre * act'(aux[m,n])
 *             CAPK_ACT_NONE           -> v = pre
 * C[m,n] = dropout(v) + residual[m,n]   (dropout and residual optional)
 * A(m,k) = a_kmajor ? A[m*lda + k] : A[k*lda + m]
 * B(n,k) = b_kmajor ? B[n*ldb + k] : B[k*ldb + n]
 * Replaces every nn.Linear / Conv1D / patch-conv GEMM (and its two backward
 * GEMMs) on the hot path: modeling_vit.py:60-69,216-218,236,249-254;
 * torch/nn/modules/transformer.py (in_proj/out_proj/linear1/linear2);
 * src/models/decoders.py:390,431 (visual_projection, output_layer).
 * in_dtype applies to A and B; out_dtype to C, residual, preact, aux.
 * Workspace (split-K partial slabs, fp32) — query with capk_gemm_workspace();
 * pass ws=NULL/ws_bytes=0 to disable split-K. */
size_t capk_gemm_workspace(int in_dtype, int out_dtype, int M, int N, int K);
/* Tile configuration of the calling thread's last hand-written capk_gemm (gemm.hip
 * choose_cfg: 1-4 = 128-row tiles, 5 = the 256x256 phased kernel, 6 = the persistent
 * 256x256 kernel, 7 = the 4-deep 128x128 ring of one-WG-per-CU grids, 8 = the 64x128
 * two-wave tile, 9 = the 64x64 four-wave tile of one-round K-major products). */
int capk_gemm_last_config(void);
/* Test / benchmark control: force the tile configuration (cfg 1..9; 0 = automatic choice;
 * -1 = CAPK_GEMM_CFG environment value) for every later capk_gemm call.  7 falls back to 1
 * on grids of more than 256 tiles, 8 and 9 to 1 unless both operands are K-major (9 also
 * needs K % 64 == 0 and never splits K). */
int capk_gemm_force_config(int cfg);
/* Split-K tail round of the persistent 256x256 kernel (grids of more than 256 items with a
 * partial last round and K >= 1536: the row blocks past the whole rounds run as 2+ K-splits
 * per tile into fp32 slabs in capk_gemm's workspace): 1 (default) one reduce + epilogue
 * launch after the GEMM, 2 the split arriving last at a tail tile sums the slabs in split
 * order and runs the epilogue inside the launch (arrival tickets per stream; bit-identical
 * to 1, measured slower), 0 off, -1 back to CAPK_GEMM_TAIL. */
int capk_gemm_set_tail(int mode);
/* Tile raster of the persistent 256x256 kernel: tiles in groups of `rows` row blocks,
 * column-major inside a group, so the 32 tiles an XCD runs at a time share fewer operand
 * blocks in its L2.  -1: automatic (default: 8 row blocks for products of more than 4
 * column blocks, 4 when the grid has <= 32 row blocks, row-major for narrower products),
 * 0: row-major, n > 0: groups of n row blocks; -2: back to CAPK_GEMM_GROUP. */
int capk_gemm_set_group(int rows);
int capk_gemm(int in_dtype, int out_dtype, int M, int N, int K,
              const void* A, int64_t lda, int a_kmajor,
              const void* B, int64_t ldb, int b_kmajor,
              void* C, int64_t ldc, float alpha, float beta,
              const float* bias, const void* residual, int64_t ldr,
              int act, void* preact, const void* aux, int64_t ldx,
              float drop_p, uint32_t drop_seed,
              void* ws, size_t ws_bytes, void* stream);

/* Two-segment bf16 product into fp32 split-K slabs, no epilogue (the LSTM recurrences of
 * decoders.py:199 / nn.LSTM: one launch per step and layer instead of the x W_ih^T and
 * h W_hh^T GEMMs with their reduces; the cell kernels below sum the slabs).
 *   k1 > 0 (K seam): C = [A | A2] [B | B2]^T, A (M x k1), A2 (M x (K - k1)), B / B2 K-major
 *     (N x k1 / N x (K - k1)); k1 and K - k1 multiples of 64.
 *   n1 > 0 (N seam): C[:, :n1] = A B^T, C[:, n1:] = A B2^T (B / B2 as b_kmajor says, n1 % 128 == 0).
 *   A K-major.  Slab s = ws + s*M*N ([M][N] fp32), s < *splits_out; capk_gemm_pair_workspace
 *   returns the bytes and the split count for (M, N, K). */
size_t capk_gemm_pair_workspace(int M, int N, int K, int* splits);
/* The same entry with k1 = n1 = 0 (A2 / B2 unused) is a plain product C = A B^T whose split
 * count is capk_gemm's own for the shape (capk_gemm_slabs_workspace): its slabs, summed in
 * order, are bit-identical to capk_gemm's split-K partials (consumer: capk_layernorm_fwd_slabs). */
size_t capk_gemm_slabs_workspace(int M, int N, int K, int* splits);
int capk_gemm_pair_slabs(int M, int N, int K, const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb,
                         int b_kmajor, const void* A2, int64_t lda2, const void* B2, int64_t ldb2, int k1, int n1,
                         float* ws, size_t ws_bytes, int* splits_out, void* stream);

/* ------------------------------------------------- fp8 (config 5) --------
 * The forward Linear / Conv1D products of BASELINE config 5 ("fp8 MFMA") on OCP e4m3fn
 * operands with one power-of-two scale per row, stored as its E8M0 code (2^(code-127)):
 * the code format v_mfma_scale_f32_16x16x128_f8f6f4 applies per lane, so scaling costs
 * nothing in the GEMM.  Replaces the fp16-autocast nn.Linear / Conv1D forward of the
 * reference's CLIP (modeling_clip.py:273-276,322-325) and GPT-2 (modeling_gpt2.py:
 * 267,281,559-561, pytorch_utils.Conv1D) under src/train/trainer.py:224-226 autocast.
 *
 * capk_quant_fp8: q = RNE_e4m3(x * 2^-e) per output row, e the smallest exponent with
 *   amax(row) * 2^-e <= 448; scale[row] = e + 127 (0x7F for an all-zero row).
 *   transpose = 0: x [rows][cols] (ldx >= cols, cols % 8 == 0);
 *   transpose = 1: x [cols][rows] (ldx >= rows; a Conv1D weight [in][out]), q [rows][cols].
 *   q [rows][ldq] bytes, ldq % 8 == 0 (rows) / % 16 == 0 (transpose).  in_dtype CAPK_F32 or CAPK_BF16.
 * capk_gemm_f8: C[M,N] = epilogue(sum_k A[m,k] 2^sa[m] * B[n,k] 2^sb[n]) with fp32
 *   accumulation; A [M][lda], B [N][ldb] e4m3fn K-major, K % 128 == 0; same epilogue
 *   arguments and meaning as capk_gemm (forward activations only). */
size_t capk_quant_fp8_workspace(int rows, int cols, int transpose); /* transpose: rows * 4 bytes */
int capk_quant_fp8(int in_dtype, int rows, int cols, const void* x, int64_t ldx, int transpose,
                   void* q, int64_t ldq, void* scale, void* ws, size_t ws_bytes, void* stream);
size_t capk_gemm_f8_workspace(int M, int N, int K);
int capk_gemm_f8(int out_dtype, int M, int N, int K, const void* A, int64_t lda, const void* a_scale,
                 const void* B, int64_t ldb, const void* b_scale, void* C, int64_t ldc, float beta,
                 const float* bias, const void* residual, int64_t ldr, int act, void* preact, int64_t ldx,
                 float drop_p, uint32_t drop_seed, void* ws, size_t ws_bytes, void* stream);

/* -------------------------------------------------------- LayerNorm -------
 * y = (x - mean) * rstd * w + b over the last `cols` elements of each row;
 * mean/rstd (fp32, [rows]) saved for backward.  LN eps 1e-12 (ViT), 1e-5
 * (nn.TransformerDecoderLayer, CLIP, GPT-2).  Replaces F.layer_norm at
 * modeling_vit.py:270,278,348 and transformer.py:1148-1153. */
int capk_layernorm_fwd(int dtype, int rows, int cols, const void* x, int64_t ldx,
                       const float* w, const float* b, float eps,
                       void* y, int64_t ldy, float* mean, float* rstd, void* stream);
/* y = LayerNorm(x), x = bf16(sum_s ws[s] + bias + res) from the no-seam slabs of
 * capk_gemm_pair_slabs ([rows][cols] fp32 each, in order); x_out (optional) keeps x.  bf16,
 * bit-identical to capk_gemm (+ bias + residual) followed by capk_layernorm_fwd: the decode
 * steps' out-projection / MLP-projection -> LayerNorm pairs (GPT-2 modeling_gpt2.py:
 * 324-331,397-409 / nn.TransformerDecoderLayer norm1..3) in one launch after the GEMM. */
int capk_layernorm_fwd_slabs(int rows, int cols, const float* ws, int splits, const float* bias, const void* res,
                             int64_t ldr, void* x_out, int64_t ldxo, const float* w, const float* b, float eps,
                             void* y, int64_t ldy, void* stream);
/* dx = LN'(dy) (+ dres if non-NULL); dw/db (fp32 [cols]) = sum over rows
 * (accumulate into existing dw/db when accumulate != 0); dsum (optional, fp32 [cols])
 * (+)= the column sums of dx -- the bias gradient of the Linear whose output gradient dx
 * is (the residual-stream producers of a pre-LN block), fused instead of a capk_colsum.  If dx_drop != NULL it also
 * receives LN'(dy) * dropout-mask (the gradient of a dropped residual branch, e.g.
 * nn.TransformerDecoderLayer dropout1..3).  ws: capk_layernorm_bwd_workspace. */
size_t capk_layernorm_bwd_workspace(int rows, int cols);
int capk_layernorm_bwd(int dtype, int rows, int cols, const void* dy, int64_t lddy,
                       const void* x, int64_t ldx, const float* w,
                       const float* mean, const float* rstd,
                       void* dx, int64_t lddx, const void* dres, int64_t ldres,
                       float* dw, float* db, float* dsum, int accumulate,
                       float drop_p, uint32_t drop_seed, void* dx_drop, int64_t lddx_drop,
                       void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------- Attention --------
 * Fused multi-head scaled-dot-product attention, one (batch, head) per
 * workgroup, Q/K/V/dO staged in LDS, softmax by wavefront shuffles.
 * Token t of batch b, head h lives at  X + b*x_bs + t*x_rs + h*hd.
 * key_pad (optional, [B, Nk] uint8, 1 = padded key) and causal masks follow
 * nn.MultiheadAttention (-inf).  The causal mask is bottom-right aligned: key j is
 * visible to query i iff j <= i + (Nk - Nq) (square: j <= i; GPT-2 with a 10-slot
 * prefix cache: the prefix is always visible, modeling_gpt2.py causal mask with
 * past_key_values).  lse (fp32 [B,H,Nq]) is saved for backward.
 * Nk <= 256, Nq <= 256, hd % 8 == 0, hd <= 128 (fp32 path: hd in {8,16,32,64,96,128}).
 * Nq <= 8 without causal/dropout (decode steps) runs a VALU kernel streaming K/V once.
 * Replaces ViT/CLIP SDPA (modeling_vit.py:164-189,219-235), the self/cross
 * attention of nn.TransformerDecoderLayer (transformer.py _sa_block/_mha_block)
 * and GPT2Attention (modeling_gpt2.py:144-226). */
int capk_attention_fwd(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, int causal,
                       const void* q, int64_t q_bs, int64_t q_rs,
                       const void* k, int64_t k_bs, int64_t k_rs,
                       const void* v, int64_t v_bs, int64_t v_rs,
                       const uint8_t* key_pad,
                       void* o, int64_t o_bs, int64_t o_rs, float* lse,
                       float drop_p, uint32_t drop_seed, void* stream);
/* KV-cached decode step over a beam-history table instead of a reordered cache (HF
 * Cache.reorder_cache, generation/utils.py:3479-3489, without moving the cache): key j <
 * Nk-1 of batch row b is read from K/V batch row kv_rows[b*kv_rows_ld + j] (int32), the
 * last key (this step's token, written in place) from row b.  Same arithmetic as
 * capk_attention_fwd on the reordered cache, bit for bit.  Nq <= 8, no masks / dropout;
 * bf16 or fp32. */
int capk_attention_decode_rows(int dtype, int B, int H, int Nq, int Nk, int hd, float scale,
                               const void* q, int64_t q_bs, int64_t q_rs,
                               const void* k, int64_t k_bs, int64_t k_rs,
                               const void* v, int64_t v_bs, int64_t v_rs,
                               const int32_t* kv_rows, int64_t kv_rows_ld,
                               void* o, int64_t o_bs, int64_t o_rs, float* lse, void* stream);
int capk_attention_bwd(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, int causal,
                       const void* q, int64_t q_bs, int64_t q_rs,
                       const void* k, int64_t k_bs, int64_t k_rs,
                       const void* v, int64_t v_bs, int64_t v_rs,
                       const uint8_t* key_pad,
                       const void* o, int64_t o_bs, int64_t o_rs,
                       const void* dout, int64_t do_bs, int64_t do_rs, const float* lse,
                       void* dq, int64_t dq_bs, int64_t dq_rs,
                       void* dk, int64_t dk_bs, int64_t dk_rs,
                       void* dv, int64_t dv_bs, int64_t dv_rs,
                       float drop_p, uint32_t drop_seed, void* stream);
/* The self-attention split backward (Nq > 32) alternates its dK/dV and dQ kernels over
 * slices of `images` batch entries (0 = one launch each over the whole batch; -1 = the
 * CAPK_ATTN_BWD_SLICE environment value), so the dQ kernel re-reads a slice's operands while
 * they are still in the Infinity Cache.  Results are identical for every slice size. */
int capk_attention_set_bwd_slice(int images);
/* 64-wide heads with Nq > 32 (the ViT layers; not the bias-sum variant) take a fused
 * single-pass backward: one workgroup per (image, head) forms P and dS once and writes dQ, dK
 * and dV.  mode 1: on, 0: the split pair above, -1: back to CAPK_ATTN_FUSED_BWD (default on). */
int capk_attention_set_fused_bwd(int mode);
/* Test support (no reference counterpart): fills every CU's LDS with a 32-bit pattern, so that a
 * following kernel reading LDS words it never wrote sees that pattern (e.g. a NaN). */
int capk_debug_fill_lds(uint32_t pattern, void* stream);
/* capk_attention_bwd plus the bias gradient of the fused QKV projection that produced q, k, v
 * (in_proj / c_attn / ViT query,key,value biases: autograd's sum of dQ, dK, dV over the tokens,
 * modeling_vit.py:205-216 through F.linear): dbias[3*H*hd] fp32 (+)= [colsum dQ | colsum dK |
 * colsum dV].  The split backward kernels (self-attention, Nq > 32) emit per-image column sums
 * and one finish pass sums the images in a fixed order; other routes run capk_colsum on the
 * three gradient views, which must then be row-uniform (batch stride = rows * row stride).
 * ws: capk_attention_bwd_bias_workspace(B, H, Nq, Nk, hd) bytes. */
size_t capk_attention_bwd_bias_workspace(int B, int H, int Nq, int Nk, int hd);
int capk_attention_bwd_bias(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, int causal,
                            const void* q, int64_t q_bs, int64_t q_rs,
                            const void* k, int64_t k_bs, int64_t k_rs,
                            const void* v, int64_t v_bs, int64_t v_rs,
                            const uint8_t* key_pad,
                            const void* o, int64_t o_bs, int64_t o_rs,
                            const void* dout, int64_t do_bs, int64_t do_rs, const float* lse,
                            void* dq, int64_t dq_bs, int64_t dq_rs,
                            void* dk, int64_t dk_bs, int64_t dk_rs,
                            void* dv, int64_t dv_bs, int64_t dv_rs,
                            float drop_p, uint32_t drop_seed, float* dbias, int accumulate,
                            void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------- Embedding / patches ----
 * ViT patchify (im2col of Conv2d k=s=P, modeling_vit.py:60-69): images fp32
 * [B,C,H,W] -> out [B*(H/P)*(W/P), C*P*P] in out_dtype, column = c*P*P+kh*P+kw. */
int capk_patchify(int out_dtype, int B, int C, int H, int W, int P,
                  const float* images, void* out, void* stream);
/* x[b,0,:] = cls + pos[0];  x[b,1+p,:] = patch_out[b*Np+p,:] + pos[1+p]
 * (ViTEmbeddings.forward modeling_vit.py:146-157). cls/pos fp32. */
int capk_vit_assemble(int dtype, int B, int Np, int D, const void* patch_out,
                      const float* cls, const float* pos, void* x, void* stream);
/* backward: dpatch[b*Np+p] = dx[b,1+p];  dcls = sum_b dx[b,0];  dpos = sum_b dx[b]
 * (fp32, overwrite).  ws >= capk_vit_assemble_bwd_workspace(). */
size_t capk_vit_assemble_bwd_workspace(int B, int Np, int D);
int capk_vit_assemble_bwd(int dtype, int B, int Np, int D, const void* dx, void* dpatch,
                          float* dcls, float* dpos, void* ws, size_t ws_bytes, void* stream);
/* token + position embedding:  out[b*T+t] = table[ids[b*T+t]] + pos[pos_offset+t]
 * (decoders.py:409-414; GPT-2 wte+wpe).  pos may be NULL. */
int capk_embedding_fwd(int dtype, int B, int T, int D, const int64_t* ids, const float* table,
                       const float* pos, int pos_offset, float drop_p, uint32_t drop_seed,
                       void* out, void* stream);
/* dtable[ids] += dout (rows whose id == padding_idx skipped, nn.Embedding
 * padding_idx semantics, decoders.py:337-339); dpos[pos_offset+t] += sum_b dout.
 * dtable/dpos fp32, accumulated (caller zeroes). */
int capk_embedding_bwd(int dtype, int B, int T, int D, const int64_t* ids, const void* dout,
                       int padding_idx, float* dtable, float* dpos, int pos_offset,
                       float drop_p, uint32_t drop_seed, void* stream);

/* --------------------------------------------------- Loss ------------------
 * Shifted cross entropy (CombinedLoss, src/train/losses.py:236-247):
 * logits [B*T, ld] (row b*T+t, first V columns valid) vs targets[b, t+1] for
 * t < T-1, ignore_index = pad.  If loss_out != NULL: loss_out[0] = mean over
 * counted tokens (fp32), loss_out[1] = count.  If dlogits != NULL it receives
 * d(loss)/d(logits) * (*grad_scale) (grad_scale: DEVICE pointer to the upstream
 * gradient, NULL = 1; rows t = T-1, ignored rows and columns >= V are zeroed);
 * dlogits may alias logits. */
size_t capk_shifted_ce_workspace(int B, int T);
int capk_shifted_ce(int dtype, int B, int T, int V, int64_t ld, const void* logits,
                    const int64_t* targets, int ignore_index, const float* grad_scale,
                    float* loss_out, void* dlogits, void* ws, size_t ws_bytes, void* stream);
/* Same with a per-sample weight w[b] on every counted row: loss = sum w_b (-log p) / count,
 * d logits scaled by w_b — the SCST policy-gradient loss -mean(logp * advantage) over the
 * unmasked sampled tokens (trainer.py:367-374 with D8: per-sample advantage, masked after
 * EOS via ignore_index targets). */
int capk_shifted_ce_weighted(int dtype, int B, int T, int V, int64_t ld, const void* logits,
                             const int64_t* targets, int ignore_index, const float* row_weight,
                             const float* grad_scale, float* loss_out, void* dlogits, void* ws, size_t ws_bytes,
                             void* stream);
/* The shifted cross entropy with its forward folded into the LM head (config-3 training, bf16):
 * capk_linear_lse computes C = x W^T + b (src/models/decoders.py:431, output_layer) and, from
 * the epilogue registers, softmax partials part[P = 4 cdiv(N, 256)][M] of (max, sum 2^(t - max))
 * over t = log2(e) * bf16(C[row, n]), n < V (capk_linear_lse_part_bytes); *done = 0 when the
 * shape does not take the persistent kernel (C is then plain capk_gemm output and the caller
 * uses capk_shifted_ce).  capk_ce_lse_fwd merges the partials: lse_out[row] (natural log) and
 * loss_out = (mean, count) as capk_shifted_ce.  capk_ce_lse_bwd writes d(loss)/d(logits) *
 * (*grad_scale) from the logits and lse in one pass (count: DEVICE pointer, loss_out + 1), and,
 * if dbias != NULL, the column sums of that gradient over its ld columns (the LM-head bias
 * gradient, written, not accumulated).  capk_ce_lse_workspace bounds both calls; the forward
 * needs only (4 + B*T) floats of it. */
size_t capk_linear_lse_part_bytes(int M, int N);
int capk_linear_lse(int M, int N, int K, const void* x, int64_t ldx, const void* w, int64_t ldw,
                    const float* bias, void* C, int64_t ldc, int V, float* part, size_t part_bytes,
                    int* done, void* ws, size_t ws_bytes, void* stream);
size_t capk_ce_lse_workspace(int B, int T, int64_t ld);
int capk_ce_lse_fwd(int B, int T, int V, int64_t ld, const void* logits, const int64_t* targets,
                    int ignore_index, const float* part, int nparts, float* lse_out, float* loss_out,
                    void* ws, size_t ws_bytes, void* stream);
int capk_ce_lse_bwd(int dtype, int B, int T, int V, int64_t ld, const void* logits, const int64_t* targets,
                    int ignore_index, const float* lse, const float* cnt, const float* grad_scale,
                    void* dlogits, float* dbias, void* ws, size_t ws_bytes, void* stream);
/* Zero rows b * rpb + j (S <= j < rpb, row < rows; row_bytes from each row start, rows ld_bytes
 * apart) -- the gap rows of a strided per-image view (the cross-attention K / V gradient of
 * src/models/decoders.py:421-428 over the ViT sequence minus its CLS rows). */
int capk_zero_gap_rows(void* base, int64_t ld_bytes, int64_t row_bytes, int B, int rpb, int S, int rows,
                       void* stream);
/* hipMemsetAsync(ptr, 0, bytes) on the stream (gradient buffers that are scatter-added). */
int capk_zero(void* ptr, size_t bytes, void* stream);

/* --------------------------------------------------- Reductions ------------
 * Deferred finishes (round 6): with capk_finish_defer(1) on a host thread, the last step of
 * the column-sum reductions below and of capk_layernorm_bwd (summing the per-workgroup
 * partial rows into db / dw / dsum) is queued per stream instead of launched, and
 * capk_finish_flush(stream) / capk_finish_flush_all() launch every queued finish of this thread
 * in one kernel -- the same per-column sums, bit-identical outputs.  The workspaces passed to
 * the queued calls must stay allocated until the flush is enqueued; a queued finish whose
 * output overlaps an earlier one's flushes the queue first.  The backward of a model layer
 * (src/models/encoders.py ViT layer, decoders.py:421-428 decoder layer) issues 4-9 such
 * finishes: one launch instead of 4-9 launches of a few workgroups each.  Off by default. */
int capk_finish_defer(int on);
int capk_finish_flush(void* stream);
int capk_finish_flush_all(void);
/* db[n] (+)= sum_m dy[m, n]   (bias gradients; fp32 out). */
size_t capk_colsum_workspace(int M, int N);
int capk_colsum(int dtype, int M, int N, const void* dy, int64_t ldy, float* db, int accumulate,
                void* ws, size_t ws_bytes, void* stream);
/* C <- C * act'(aux) (CAPK_ACT_DERIV: C * aux) in place and db (+)= its column sums: the
 * backward activation of an FFN product fused with the bias gradient of the Linear that
 * produced the activation's input (ViTMLP fc1.bias, modeling_vit.py:249-254).
 * ws: capk_colsum_workspace(M, N). */
int capk_act_bwd_colsum(int dtype, int M, int N, void* C, int64_t ldc, const void* aux, int64_t ldx, int act,
                        float* db, int accumulate, void* ws, size_t ws_bytes, void* stream);
/* C[M,N] = (dY[M,K] W[K,N]) * act'(pre) (act | CAPK_ACT_DERIV: * aux) and db (+)= the column
 * sums of C -- the FFN backward of a pre-LN block in one call: fc2's dX product, the GELU
 * backward and fc1's bias gradient (ViTMLP, modeling_vit.py:249-254).  bf16
 * operands (dY K-major with ldy, W [K][N] with ldw), bf16 C / aux, fp32 db.  Large grids run
 * the persistent GEMM with the column sums taken from its register epilogue; others the
 * product + capk_act_bwd_colsum.  ws: capk_gemm_dx_act_colsum_workspace(M, N, K). */
size_t capk_gemm_dx_act_colsum_workspace(int M, int N, int K);
int capk_gemm_dx_act_colsum(int M, int N, int K, const void* dY, int64_t ldy, const void* W, int64_t ldw, void* C,
                            int64_t ldc, int act, const void* aux, int64_t ldx, float* db, int accumulate, void* ws,
                            size_t ws_bytes, void* stream);
/* The same with W given as its K-major copy WT = W^T [N][K] (ldwt): capk_transpose_bf16_batch. */
int capk_gemm_dx_act_colsum_wt(int M, int N, int K, const void* dY, int64_t ldy, const void* WT, int64_t ldwt,
                               void* C, int64_t ldc, int act, const void* aux, int64_t ldx, float* db, int accumulate,
                               void* ws, size_t ws_bytes, void* stream);
/* elementwise casts / copies */
int capk_cast(int in_dtype, int out_dtype, int64_t n, const void* x, void* y, void* stream);
int capk_copy_rows(int dtype, int rows, int cols, const void* x, int64_t ldx, void* y, int64_t ldy, void* stream);
/* Batched bf16 transposes (round 6): dst[c][r] = src[r][c] for every descriptor, all in one
 * launch per 64 descriptors.  The backward's dX products read the weight W [N_out][K_in]
 * N-major; a K-major copy W^T [K_in][N_out], refreshed once per optimizer step for every
 * weight the dX products use (capk/ops.py WeightT), runs them on the K-major GEMM paths
 * (nn.Linear backward, torch autograd; the reference's decoders.py / ViT layers).  rows, cols,
 * ld_src and ld_dst multiples of 8; src / dst 16-B aligned. */
typedef struct capk_transpose_desc {
  const void* src;
  void* dst;
  int64_t ld_src, ld_dst;
  int32_t rows, cols;
} capk_transpose_desc;
int capk_transpose_bf16_batch(int n, const capk_transpose_desc* descs, void* stream);

/* y = x * dropout-mask(p, seed, index r*cols + c) — the GEMM-epilogue mask of an
 * [rows, cols] output re-applied to its gradient (GPT-2 resid_dropout backward,
 * modeling_gpt2.py:224,243). */
int capk_dropout_apply(int dtype, int rows, int cols, const void* x, int64_t ldx, float p, uint32_t seed,
                       void* y, int64_t ldy, void* stream);
/* y[g][r][c] (+)= sum_{s<nseg} x[g][r][s*seg_stride + c]   (y fp32): e.g. the GPT-2
 * prefix gradient dP = sum over layers of dK + dV of the 10 prefix slots (K = V =
 * prefix; decoders.py:597-617). */
int capk_add_rows(int dtype, int groups, int rows, int cols, const void* x, int64_t gsx, int64_t ldx, int nseg,
                  int64_t seg_stride, float* y, int64_t gsy, int64_t ldy, int accumulate, void* stream);

/* out = dy * act'(aux) elementwise (activation backward outside a GEMM, e.g. the
 * ViT pooler tanh, modeling_vit.py:295-301). */
int capk_act_bwd(int dtype, int64_t n, int act, const void* dy, const void* aux, void* out, void* stream);

/* --------------------------------------------------- Optimizer -------------
 * torch.optim.AdamW step (decoupled weight decay; trainer.py:131-134) over a
 * flat fp32 segment; optional bf16 shadow copy of the updated parameters for
 * the throughput path.  bc1 = 1-beta1^t, bc2 = 1-beta2^t computed by the host. */
int capk_adamw(int64_t n, float* param, const float* grad, float* m, float* v,
               void* param_bf16, float lr, float weight_decay, float beta1, float beta2,
               float eps, float bc1, float bc2, void* stream);

/* --------------------------------------------------- Beam search (A14) -----
 * transformers 5.15 GenerationMixin._beam_search (generation/utils.py:3208-3535)
 * as reached by GPT2Decoder.generate (src/models/decoders.py:645-654; SURVEY D16:
 * the same search for every decoder).  Prompt length 1, one EOS id, MaxLength +
 * EOS stopping.  All search state lives in one device buffer of
 * capk_beam_state_bytes(B, num_beams, max_length) bytes (num_beams <= 8,
 * max_length <= 256).  Per decode step the caller produces logits [B*k, ld]
 * (V valid columns; rows b*k..b*k+k-1 are image b's beams) and calls
 * capk_beam_step with cur_len = current sequence length (1 at the first step),
 * fin_div = float((cur_len+1-1) ** length_penalty) and best_div = the
 * early-stop heuristic's float(best_len ** length_penalty) (utils.py:3008-3053,
 * 3175); early_stopping 0 = False, 1 = True, 2 = "never".  It writes the next
 * token of every running beam (next_ids [B*k] int64) and the cache-reorder
 * index (reorder [B*k]: row b*k+i continues from row reorder[b*k+i];
 * utils.py:3479-3489).  capk_beam_flags copies the three batch-global flags
 * (any improvement possible, any image with an unfinished slot, any valid
 * continuation) to host memory and synchronises the stream; HF stops when
 * !(f0 && !(early_stopping==True && !f1) && f2) (utils.py:3055-3075).
 * capk_beam_finalize writes finished sequences [B,k,L] int64 (unfilled = fill),
 * scores [B,k] and beam indices [B,k,L-1] int32 (-1 = not generated). */
size_t capk_beam_state_bytes(int B, int num_beams, int max_length);
int capk_beam_init(int B, int num_beams, int max_length, const int64_t* prompt, int64_t fill, void* state,
                   size_t state_bytes, void* stream);
int capk_beam_step(int dtype, int B, int num_beams, int max_length, int V, int64_t ld, const void* logits,
                   int cur_len, int64_t eos, float fin_div, float best_div, int early_stopping, void* state,
                   size_t state_bytes, int32_t* reorder, int64_t* next_ids, void* stream);
int capk_beam_flags(const void* state, int32_t* flags_out, void* stream);
int capk_beam_finalize(int B, int num_beams, int max_length, const void* state, int64_t* sequences,
                       float* scores, int32_t* beam_indices, void* stream);
/* out[r * out_stride] = argmax over the V valid columns of row r (first index on ties,
 * torch.argmax): greedy decoding (decoders.py:308-309, 480). */
int capk_argmax_rows(int dtype, int rows, int V, int64_t ld, const void* x, int64_t* out, int64_t out_stride,
                     void* stream);
/* Categorical sample from softmax(logits[r, :V]) by inverse CDF with the counter-based
 * uniform u = (hash(seed, step<<32 | r) >> 8) / 2^24 (same hash as dropout); out[r*out_stride]
 * = token, logp[r] (optional) = its log-probability.  SCST sampler (trainer.py:383-438). */
int capk_sample_rows(int dtype, int rows, int V, int64_t ld, const void* logits, uint32_t seed, int step,
                     int64_t* out, int64_t out_stride, float* logp, void* stream);
/* ------------------------------------------------------ input pipeline -----
 * The reference's torchvision transforms on PIL images (src/main.py:139-153;
 * src/data/dataset.py:105-112): per image of a packed uint8 RGB HWC buffer, crop
 * (cy, cx, ch, cw) -> Pillow-exact antialiased bilinear resize to (rh, rw) -> the size x size
 * window at (oy, ox) -> optional horizontal flip -> x / 255 -> (x - mean) / std, written
 * [B, 3, size, size] (out_dtype CAPK_F32 / CAPK_BF16).  desc = B packed descriptors
 * {int64 offset; int32 H, W, cy, cx, ch, cw, rh, rw, oy, ox, flip} of
 * capk_image_desc_bytes() bytes each; downscale per axis <= 31x. */
size_t capk_image_desc_bytes(void);
int capk_resize_normalize(int out_dtype, int B, int size, const void* images, const void* desc,
                          const float* mean, const float* stdv, void* out, void* stream);
/* capk_sample_rows with the seed read from device memory (a replayed HIP graph of the
 * sampling loop keeps its kernel arguments; capk/graphs.py writes the seed before replay). */
int capk_sample_rows_dev(int dtype, int rows, int V, int64_t ld, const void* logits, const uint32_t* seed,
                         int step, int64_t* out, int64_t out_stride, float* logp, void* stream);
/* y[g][r] = x[g][idx[r]] row gather over G groups (KV-cache reorder after a beam
 * step, all layers in one launch; HF Cache.reorder_cache = index_select on dim 0). */
int capk_gather_rows(int dtype, int groups, int rows, int cols, const int32_t* idx, const void* x, int64_t ldx,
                     int64_t gsx, void* y, int64_t ldy, int64_t gsy, void* stream);

/* --------------------------------------------------- LSTM decoder (A6/A7) ---
 * nn.LSTM cell (gate order i, f, g, o; aten lstm_cell) on pre-activation gates
 * [B, 4D] (= x W_ih^T + b_ih + h W_hh^T + b_hh from two GEMMs).  Cell state fp32.
 * h_drop (optional) receives dropout(h') (inter-layer dropout of nn.LSTM, index
 * b*D + d) for the next layer's input; act [B, 4D] saves i, f, g, o for backward.
 * capk_lstm_cell_bwd: dh = total grad w.r.t. h'; dc in = grad w.r.t. c', out = grad
 * w.r.t. c_prev (in place); dgates = pre-activation gate gradients [B, 4D].
 * Replaces torch.nn.LSTM (decoders.py:97-103, 199) one step at a time. */
int capk_lstm_cell_fwd(int dtype, int B, int D, const void* gates, int64_t ldg, const float* c_prev, float* c_out,
                       void* h_out, int64_t ldh, void* h_drop, int64_t ldhd, void* act, float drop_p,
                       uint32_t drop_seed, void* stream);
int capk_lstm_cell_bwd(int dtype, int B, int D, const void* act, const float* c_prev, const void* dh, int64_t lddh,
                       float* dc, void* dgates, void* stream);
/* The cells fed by capk_gemm_pair_slabs' slabs (bf16, slab s of a [B, ld] product at
 * ws + s*B*ld).  Forward: gates = sum_s ws[s] + bias_a + bias_b (+ res [B, 4D] bf16; biases
 * fp32, optional).  Backward: grad w.r.t. h' = dh (optional bf16) + dropout(sum_s
 * ws_up[s][:, 0:D]) (the layer above's input gradient, mask of the forward's h_drop, index
 * b*D + d) + sum_s ws_rec[s][:, col_rec:col_rec+D] (the recurrent gradient from step t+1);
 * either slab set optional.  capk_slab_sum: out[m][j] = bf16(sum_s ws[s][m][col0 + j] + res[m][j])
 * (res bf16, optional). */
int capk_lstm_cell_fwd_slabs(int B, int D, const float* ws, int splits, int64_t ldw, const float* bias_a,
                             const float* bias_b, const void* res, int64_t ldr, const float* c_prev, float* c_out,
                             void* h_out, int64_t ldh, void* h_drop, int64_t ldhd, void* act, float drop_p,
                             uint32_t drop_seed, void* stream);
int capk_lstm_cell_bwd_slabs(int B, int D, const void* act, const float* c_prev, const void* dh, int64_t lddh,
                             const float* ws_up, int splits_up, int64_t ld_up, float drop_p, uint32_t drop_seed,
                             const float* ws_rec, int splits_rec, int64_t ld_rec, int col_rec, float* dc,
                             void* dgates, void* stream);
int capk_slab_sum(int M, int ncols, const float* ws, int splits, int64_t ldw, int col0, const void* res, int64_t ldr,
                  void* out, int64_t ldo, void* stream);
/* SoftAttention (src/models/attention.py:57-118) for one decode step, one query per
 * image: e[b,s] = (sum_d we[d] tanh(qp[b,d] + kp[b,s,d]) + be) * inv_temp, key_pad ->
 * -1e9, w = softmax_s(e), ctx[b] = sum_s w[b,s] v[b,s] (w_out fp32 [B,S]).  kp is the
 * hoisted key_proj(keys).  Backward ACCUMULATES (fp32) dkp, dv [B,S,D], dwe_part [B,D],
 * dbe_part [B] over steps and writes dqp; dw_in (optional fp32 [B,S]) is a gradient on
 * the returned weights.  S <= 256. */
int capk_soft_attn_fwd(int dtype, int B, int S, int D, const void* qp, int64_t ldq, const void* kp, int64_t kp_bs,
                       int64_t kp_rs, const void* v, int64_t v_bs, int64_t v_rs, const float* we, const float* be,
                       float inv_temp, const uint8_t* key_pad, void* ctx, int64_t ldc, float* w_out, void* stream);
int capk_soft_attn_bwd(int dtype, int B, int S, int D, const void* qp, int64_t ldq, const void* kp, int64_t kp_bs,
                       int64_t kp_rs, const void* v, int64_t v_bs, int64_t v_rs, const float* we, float inv_temp,
                       const float* w, const void* dctx, int64_t lddc, const float* dw_in, void* dqp, int64_t lddq,
                       float* dkp, float* dv, float* dwe_part, float* dbe_part, void* stream);
/* The deferred form: capk_soft_attn_bwd_step writes dqp, accumulates dwe_part / dbe_part and
 * stashes the step's softmax-Jacobian energies de_out [B,S] (fp32) and output gradient
 * dctx_out [B,D] instead of updating dkp / dv; after the last step capk_soft_attn_kv_grad WRITES
 * dkp, dv [B,S,D] (fp32) from the stashes of all steps ([steps,B,S] / [steps,B,D], qp
 * [steps,B,D], w_all = the forward weights [steps,B,S]), summing t from the last step down as
 * the per-step accumulation does -- two [B,S,D] read-modify-writes per step become one write. */
int capk_soft_attn_bwd_step(int dtype, int B, int S, int D, const void* qp, int64_t ldq, const void* kp,
                            int64_t kp_bs, int64_t kp_rs, const void* v, int64_t v_bs, int64_t v_rs, const float* we,
                            float inv_temp, const float* w, const void* dctx, int64_t lddc, const float* dw_in,
                            void* dqp, int64_t lddq, float* dwe_part, float* dbe_part, float* de_out, void* dctx_out,
                            void* stream);
int capk_soft_attn_kv_grad(int dtype, int steps, int B, int S, int D, const void* qp, const void* kp, int64_t kp_bs,
                           int64_t kp_rs, const float* we, const float* de_all, const float* w_all,
                           const void* dctx_all, float* dkp, float* dv, void* stream);

/* ------------------------------------------- attention-module gates (A8-A10) ----
 * capk_ew_mul: out = a * b (AoA info * gate, attention.py:354).
 * capk_tanh_gate_fwd/bwd: out = g * tanh(c) with c fp32 (adaptive visual sentinel,
 * attention.py:258-262); bwd: dg = dout * tanh(c), dc += dout * g * (1 - tanh(c)^2).
 * capk_gate_mix_fwd/bwd: beta[b] = sigmoid(wa[:D].ctx[b] + wa[D:].s[b] + ba),
 * out = beta ctx + (1 - beta) s (attention.py:279-285); bwd writes dctx, ds and
 * ACCUMULATES dwa [2D], dba [1] (fp32 atomics).
 * capk_attention_probs_mean: out[b,q,s] = mean_h softmax weights rebuilt from the lse
 * of capk_attention_fwd (MultiHeadAttention's returned weights, attention.py:207-210).
 * capk_attention_probs_mean_bwd: gradient of those weights, dw fp32 [B, Nq, Nk]:
 *   ACCUMULATES dq (dtype, [B, Nq, H*hd] view) and dk (fp32 [B, Nk, H*hd] view); one
 *   block per (image, head), queries in order (deterministic).  Nk <= 2048. */
int capk_ew_mul(int dtype, int rows, int cols, const void* a, int64_t lda, const void* b, int64_t ldb, void* out,
                int64_t ldo, void* stream);
int capk_tanh_gate_fwd(int dtype, int rows, int cols, const float* c, int64_t ldc, const void* g, int64_t ldg,
                       void* out, int64_t ldo, void* stream);
int capk_tanh_gate_bwd(int dtype, int rows, int cols, const float* c, int64_t ldc, const void* g, int64_t ldg,
                       const void* dout, int64_t lddo, void* dg, int64_t lddg, float* dc, int64_t lddc, void* stream);
int capk_gate_mix_fwd(int dtype, int B, int D, const void* ctx, int64_t ldx, const void* s, int64_t lds,
                      const float* wa, const float* ba, float* beta, void* out, int64_t ldo, void* stream);
int capk_gate_mix_bwd(int dtype, int B, int D, const void* ctx, int64_t ldx, const void* s, int64_t lds,
                      const float* wa, const float* beta, const void* dout, int64_t lddo, void* dctx, int64_t lddx,
                      void* ds, int64_t ldds, float* dwa, float* dba, void* stream);
int capk_attention_probs_mean(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, const void* q,
                              int64_t q_bs, int64_t q_rs, const void* k, int64_t k_bs, int64_t k_rs,
                              const uint8_t* key_pad, const float* lse, float* out, void* stream);
int capk_attention_probs_mean_bwd(int dtype, int B, int H, int Nq, int Nk, int hd, float scale, const void* q,
                                  int64_t q_bs, int64_t q_rs, const void* k, int64_t k_bs, int64_t k_rs,
                                  const uint8_t* key_pad, const float* lse, const float* dw, void* dq, int64_t dq_bs,
                                  int64_t dq_rs, float* dk, int64_t dk_bs, int64_t dk_rs, void* stream);

/* ------------------------------------------------ convolutional encoder (A3) ----
 * Channels-last activations [B, H, W, C] (row m = (b*H + h)*W + w, C contiguous).
 * capk_im2col: col[m, k] of a KHxKW / stride / pad convolution, m = (b, oh, ow),
 *   k = (kh*KW + kw)*C + c, zero for padding taps and for KH*KW*C <= k < Kp; input
 *   element (b,h,w,c) at x[b*sb + h*sh + w*sw + c*sc] (so NCHW fp32 images feed the
 *   stem directly).  in/out dtype pairs: f32->f32, f32->bf16, bf16->bf16.
 *   Replaces the im2col inside nn.Conv2d (transformers ResNetConvLayer /
 *   ResNetShortCut, modeling_resnet.py:39-110; torchvision resnet101 convs).
 * capk_col2im: dx = beta*dx + the adjoint of capk_im2col (gather-sum, deterministic).
 * capk_bn_stats: training-mode nn.BatchNorm2d statistics over the M rows of [M, C]:
 *   mean, rstd = 1/sqrt(biased var + eps); running_mean/var (nullable) updated with
 *   `momentum` (running_var from the unbiased variance), num_batches_tracked (nullable,
 *   int64) += 1; one sweep over x: per-block sums and squared deviations about the block
 *   mean, merged exactly (CAPK_BN_TWOPASS=1: two global passes).  capk_bn_eval_stats: mean,
 *   rstd from the running buffers (eval mode).
 * capk_bn_apply: y = [relu]((x - mean)*rstd*gamma + beta [+ residual]).
 * capk_bn_bwd: dz = dy * [y_mask > 0] (y_mask nullable: the ReLU output; or, with relu_beta
 *   (the BatchNorm's beta) instead, the mask of this BatchNorm's own ReLU output recomputed
 *   from x as capk_bn_apply computes it, so y is not re-read), dgamma,
 *   dbeta = column sums (written, or added with accumulate), dx (nullable) =
 *   beta_acc*dx + gamma*rstd*(dz - mean(dz) - xhat*mean(dz*xhat)); dz_out (nullable)
 *   receives dz.  batch_stats = 0: statistics were the running buffers (eval mode),
 *   dx = beta_acc*dx + gamma*rstd*dz.  Workspace capk_bn_workspace(M, C) bytes.
 *   C % 8 == 0 and (C <= 2048 or C % 2048 == 0).
 * capk_maxpool_fwd/bwd: KxK max pool, -inf padding, idx = first-max window offset
 *   (nn.MaxPool2d, ResNetEmbeddings.pooler modeling_resnet.py:83).
 * capk_avgpool_fwd/bwd: adaptive average pool to OHxOW (aten window rule); y rows
 *   b*OH*OW + oh*OW + ow with row stride ldy (ResNetModel pooler
 *   AdaptiveAvgPool2d((1,1)); legacy models/encoder.py:10 AdaptiveAvgPool2d((14,14))). */
int capk_im2col(int in_dtype, int out_dtype, int B, int H, int W, int C, int64_t sb, int64_t sh, int64_t sw,
                int64_t sc, int KH, int KW, int stride, int pad, int OH, int OW, int Kp, const void* x, void* col,
                void* stream);
int capk_col2im(int dtype, int B, int H, int W, int C, int KH, int KW, int stride, int pad, int OH, int OW, int Kp,
                const void* dcol, void* dx, float beta, void* stream);
size_t capk_bn_workspace(int M, int C);
int capk_bn_stats(int dtype, int M, int C, const void* x, int64_t ldx, float eps, float momentum, float* mean,
                  float* rstd, float* running_mean, float* running_var, int64_t* num_batches_tracked, void* ws,
                  size_t ws_bytes, void* stream);
int capk_bn_eval_stats(int C, const float* running_mean, const float* running_var, float eps, float* mean,
                       float* rstd, void* stream);
int capk_bn_apply(int dtype, int M, int C, const void* x, int64_t ldx, const float* mean, const float* rstd,
                  const float* gamma, const float* beta, const void* residual, int64_t ldr, int relu, void* y,
                  int64_t ldy, void* stream);
int capk_bn_bwd(int dtype, int M, int C, const void* dy, int64_t lddy, const void* y_mask, int64_t ldym,
                const void* x, int64_t ldx, const float* mean, const float* rstd, const float* gamma,
                const float* relu_beta, float* dgamma, float* dbeta, int accumulate, void* dx, int64_t lddx,
                float beta_acc, void* dz_out, int64_t lddz, int batch_stats, void* ws, size_t ws_bytes,
                void* stream);
int capk_maxpool_fwd(int dtype, int B, int H, int W, int C, int K, int stride, int pad, int OH, int OW,
                     const void* x, void* y, uint8_t* idx, void* stream);
int capk_maxpool_bwd(int dtype, int B, int H, int W, int C, int K, int stride, int pad, int OH, int OW,
                     const void* dy, const uint8_t* idx, void* dx, void* stream);
int capk_avgpool_fwd(int dtype, int B, int H, int W, int C, int OH, int OW, const void* x, void* y, int64_t ldy,
                     void* stream);
int capk_avgpool_bwd(int dtype, int B, int H, int W, int C, int OH, int OW, const void* dy, int64_t lddy, void* dx,
                     float beta, void* stream);

/* ------------------------------------------- legacy Show-Attend-Tell (A11) ----
 * capk_additive_attn_fwd/bwd: capk_soft_attn_* generalised to the legacy decoder's
 * attention (models/decoder.py:141-151): energy nonlinearity act (0 = tanh,
 * 1 = ReLU) and a value width Dv != D (alpha-weighted sum of 2048-wide encoder
 * pixels with 512-wide attention projections).  dv may be NULL (no value gradient).
 * capk_attn_coverage_reg: alphas t-major [T, B, S] fp32 (inactive rows 0);
 * loss_acc[0] += mean_{b,s} (1 - sum_t alphas)^2 (train.py:101) when non-NULL;
 * coef[b, s] (nullable) = d/d alpha[b,t,s] * (*grad_scale, NULL = 1).
 * capk_clamp: x = min(max(x, lo), hi) in place (train.py:105-110 grad clamp).
 * capk_mask_rows_by_length: x[b*bs + t*ld + c] = 0 for t >= len[b] (device int32). */
int capk_additive_attn_fwd(int dtype, int act, int B, int S, int D, int Dv, const void* qp, int64_t ldq,
                           const void* kp, int64_t kp_bs, int64_t kp_rs, const void* v, int64_t v_bs, int64_t v_rs,
                           const float* we, const float* be, float inv_temp, const uint8_t* key_pad, void* ctx,
                           int64_t ldc, float* w_out, void* stream);
int capk_additive_attn_bwd(int dtype, int act, int B, int S, int D, int Dv, const void* qp, int64_t ldq,
                           const void* kp, int64_t kp_bs, int64_t kp_rs, const void* v, int64_t v_bs, int64_t v_rs,
                           const float* we, float inv_temp, const float* w, const void* dctx, int64_t lddc,
                           const float* dw_in, void* dqp, int64_t lddq, float* dkp, float* dv, float* dwe_part,
                           float* dbe_part, void* stream);
int capk_attn_coverage_reg(int B, int T, int S, const float* alphas, const float* grad_scale, float* loss_acc,
                           float* coef, void* stream);
int capk_clamp(int64_t n, float* x, float lo, float hi, void* stream);
int capk_mask_rows_by_length(int dtype, int B, int T, int cols, void* x, int64_t ld, int64_t bs, const int32_t* len,
                             void* stream);

/* ------------------------------------------------- Swin encoder (§8f-4) ----
 * Window attention of transformers SwinAttention (modeling_swin.py:401-468, reached from
 * SwinEncoder.forward, src/models/encoders.py:165-182), rows in window order: window w
 * (= b*nw_img + window-in-image) owns rows [w*N, (w+1)*N), N = ws*ws <= 64, token
 * t = r*ws + c.  q / k / v of head h are columns h*hd, C + h*hd, 2C + h*hd of qkv
 * (row stride ldq); hd = 32.  s_ij = scale*q_i.k_j + table[idx(i,j)*H + h]
 * (+ -100 where labels[w % nw_img][i] != labels[..][j]; labels = null for an unshifted
 * block), idx(i,j) = (r_i-r_j+ws-1)*(2ws-1) + (c_i-c_j+ws-1) (SwinRelativePositionBias);
 * out = softmax(s) v per head into columns h*hd of out; lse [nwin, H, N] fp32.
 * capk_window_attn_bwd: dq/dk/dv into the same column layout of dqkv (every element of
 * the 3C columns written); dtable [(2ws-1)^2, H] fp32 (+)= sum over windows of dS binned
 * by idx (fixed-order reduction through the caller's workspace).
 * capk_rowscale_add: y[r, :] = res[r, :] + x[r, :] * scale[r / group_rows] (res may be
 * null) -- SwinDropPath's per-sample keep/(1-p) factor (modeling_swin.py:42-60). */
int capk_window_attn_fwd(int dtype, int nwin, int nw_img, int ws, int H, int hd, float scale, const void* qkv,
                         int64_t ldq, int C, const float* table, const int32_t* labels, void* out, int64_t ldo,
                         float* lse, void* stream);
size_t capk_window_attn_bwd_workspace(int nwin, int ws, int H);
int capk_window_attn_bwd(int dtype, int nwin, int nw_img, int ws, int H, int hd, float scale, const void* qkv,
                         int64_t ldq, int C, const float* table, const int32_t* labels, const void* out, int64_t ldo,
                         const void* dout, int64_t lddo, const float* lse, void* dqkv, int64_t lddq, float* dtable,
                         int accumulate, void* work, size_t work_bytes, void* stream);
int capk_rowscale_add(int dtype, int rows, int cols, const void* x, int64_t ldx, const float* scale, int group_rows,
                      const void* res, int64_t ldr, void* y, int64_t ldy, void* stream);

/* ------------------------------------------------------ CIDEr-D (host) ----
 * SCST reward: replaces src/evaluate/metrics.py:46-110 (pycocoevalcap
 * CiderD, via CaptioningTrainer._calculate_rewards, src/train/trainer.py:440-484) with a
 * per-sample score.  HOST code (no device memory, no stream): token-id sentences as
 * CSR arrays — candidate i = cand_tok[cand_off[i] .. cand_off[i+1]); reference r =
 * ref_tok[ref_off[r] .. ref_off[r+1]); the references of candidate i are r in
 * [ref_img[i], ref_img[i+1]).  Document frequencies are taken over this corpus (one
 * entry per candidate).  n_max = 4, sigma = 6 for CIDEr-D; scores[i] in the
 * scorer's x10 scale.  threads <= 0: all hardware threads. */
int capk_cider_d(int n_cand, const int32_t* cand_tok, const int64_t* cand_off, const int32_t* ref_tok,
                 const int64_t* ref_off, const int64_t* ref_img, int n_max, double sigma, int threads,
                 double* scores);

#ifdef __cplusplus
}
#endif
#endif /* CAPK_H */
