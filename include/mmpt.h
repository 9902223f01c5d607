/*
 * mmpt.h — C-ABI of the MI355X-native pre-training step library (libmmpt.so).
 *
 * The reference (tttyuntian/multimodal_llm_pretraining) has no native code and
 * no FFI: every op below replaces an ATen / DeepSpeed kernel that HF
 * transformers launches on the reference's behalf inside
 * `ManualTrainer.manual_training_step` / `manual_optimization_step`
 * (src/benchmarking/utils.py:61-80).  Each declaration cites the reference-side
 * interface it replaces.  `tf:` = transformers source.
 *
 * Conventions:
 *   - plain pointers + sizes, no torch types; all memory is caller-owned
 *     (PyTorch's caching allocator); the library never allocates on the hot path;
 *   - every call takes the caller's HIP stream as `void* stream` (hipStream_t);
 *   - return 0 on success, <0 for argument / unsupported errors, >0 = hipError_t;
 *     the message is in mmpt_last_error() (thread-local);
 *   - bf16 tensors are passed as `void*` (uint16 storage), fp32 as `float*`;
 *   - leading dimensions (`ld*`) are in elements.
 */
#ifndef MMPT_H_
#define MMPT_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMPT_ABI_VERSION 14

enum mmpt_status { MMPT_OK = 0, MMPT_ERR_ARG = -1, MMPT_ERR_UNSUPPORTED = -2 };

int mmpt_abi_version(void);
const char* mmpt_last_error(void);
/* Number of compute units / clock of the current device (for roofline maths). */
int mmpt_device_info(int* cus, int* clock_khz, int* arch_gfx);
/* Test / measurement hook (ABI 9): kernel-variant switches are read ONCE from the
 * environment (MMPT_ATTN_PAIR: D = 256 dK/dV wave-pair kernel, MMPT_ATTN_DS: dQ through dS
 * tiles, MMPT_ATTN_NATIVE80: head_dim 80 computed over 80 dims; default 1 each; ABI 11:
 * MMPT_GEMM_KREV, gemm4p's odd tiles per workgroup walk K last-to-first, default 2 =
 * by shape; MMPT_GEMM_TAIL, the tail split, default 1; MMPT_GEMM_TAIL128 (round 6), tails of
 * <= 128 rows on the 128-row kernel, default 1; MMPT_GEMM_WTAIL (round 6), the weight-gradient
 * tail split, default 1 (2: tail tile columns only); MMPT_CE_REG, the register-resident
 * cross entropy, default 1); this overrides one for the rest of
 * the process.  value ∈ {0, 1} (2: KREV, WTAIL);
 * returns the previous value, MMPT_ERR_ARG for an unknown name. */
int mmpt_set_switch(const char* name, int value);

/* ------------------------------------------------------------------------
 * K1  nn.Linear → aten::addmm / mm (bf16 autocast).  tf:models/gpt_neox/
 * modeling_gpt_neox.py:38-49,176-177,190; tf:models/vit/modeling_vit.py:203-206,
 * 244-246; tf:models/llava/modeling_llava.py:92-100; lm_head :384.
 *
 * C[M,N] = op(A)[M,K] · op(B)[K,N], bf16 operands, fp32 accumulation.
 *   layout_a: MMPT_ROWS_K → A stored [M][K] (K contiguous, lda ≥ K)
 *             MMPT_K_ROWS → A stored [K][M] (M contiguous, lda ≥ M)
 *   layout_b: MMPT_ROWS_K → B stored [N][K] (K contiguous: nn.Linear weight)
 *             MMPT_K_ROWS → B stored [K][N] (N contiguous)
 * Forward Y = X·Wᵀ is (ROWS_K, ROWS_K); dX = dY·W is (ROWS_K, K_ROWS);
 * dW = dYᵀ·X is (K_ROWS, K_ROWS).
 * ---------------------------------------------------------------------- */
enum mmpt_layout { MMPT_ROWS_K = 0, MMPT_K_ROWS = 1 };
enum mmpt_epilogue {
  MMPT_EPI_BF16 = 0,       /* C(bf16) = bf16(acc + bias)                              */
  MMPT_EPI_BF16_GELU = 1,  /* C(bf16) = pre = bf16(acc + bias); C2(bf16) = bf16(gelu(pre)) */
  MMPT_EPI_BF16_DGELU = 2, /* C(bf16) = bf16(bf16(acc) * gelu'(aux))   [aux = pre, bf16] */
  MMPT_EPI_F32_ACC = 3,    /* C(f32) += f32(bf16(acc))   (weight-grad accumulation)     */
  MMPT_EPI_F32_STORE = 4,  /* C(f32)  = f32(bf16(acc))                                 */
  MMPT_EPI_F32_RESID = 5,  /* v = bf16(acc+bias); if aux: v = bf16(v + aux);
                              C(f32) = C2(f32 resid, may alias C) + v   (residual add)  */
  MMPT_EPI_BF16_DGELU_COLSUM = 6, /* as BF16_DGELU, plus per-tile column sums of the bf16
                              result into C2 (f32 [mmpt_gemm_colsum_rows][N]); finish with
                              mmpt_colsum_f32 -> the bias gradient of the layer whose
                              input gradient C is (fused addmm grad_bias)            */
  /* quick-GELU (x·sigmoid(1.702x), CLIP's hidden_act, tf:activations.py:70-123) forms of
     the three GELU epilogues, with autocast's bf16 roundings between its ops        */
  MMPT_EPI_BF16_QGELU = 7,
  MMPT_EPI_BF16_DQGELU = 8,
  MMPT_EPI_BF16_DQGELU_COLSUM = 9,
  /* SwiGLU MLP (LlamaMLP: down(silu(gate(x)) * up(x)), tf:models/llama/modeling_llama.py),
     with the fused gate|up projection stored BLOCKED: weight rows [256k, 256k+128) are
     gate rows f = 128k.., rows [256k+128, 256k+256) the up rows of the same features.
     SWIGLU (fwd, N = 2F, F % 128 == 0, no bias): C(bf16 [M][2F]) = the gate|up outputs in
     that blocked order; C2(bf16 [M][F]) = bf16(bf16(silu(gate)) * up).
     DSWIGLU (bwd, N = F): d = bf16(acc) is the act gradient; aux = the forward's C; writes
     C(bf16 [M][2F], blocked) = d gate, d up — autograd's bf16 mul / silu_backward. */
  MMPT_EPI_BF16_SWIGLU = 10,
  MMPT_EPI_BF16_DSWIGLU = 11,
  /* (ABI 12) weight + bias gradient in one pass: as F32_ACC, plus the sums over K of op(A)'s
     rows — Σ_k dY[k, m], addmm backward's grad_bias when A = dY (K_ROWS: [tokens][out]) — into
     C2 (f32 [mmpt_gemm_acc_colsum_rows][ldc2 ≥ M]: one partial row per K split and 256-column
     tile, each column summing its share of the K-tiles); finish with
     mmpt_colsum_f32(rows, M, C2, dbias, ...).  Both layouts K_ROWS, problems the big-tile
     kernel takes (mmpt_gemm_acc_colsum_rows > 0; since ABI 13 any K: token counts K % 64 != 0
     run the K-tail form); else MMPT_ERR_UNSUPPORTED. */
  MMPT_EPI_F32_ACC_COLSUM = 12
};
/* Rows of the column-sum partial buffer an EPI_BF16_DGELU_COLSUM call writes. */
int64_t mmpt_gemm_colsum_rows(int64_t M, int64_t N, int64_t K);
/* (ABI 12) Rows of the partial buffer an EPI_F32_ACC_COLSUM call writes (K splits x
 * ceil(N / 256), with a workspace of mmpt_gemm_workspace_bytes; rows a call with less workspace
 * leaves are zeroed),
 * or 0: the fused form does not take this problem (run F32_ACC + mmpt_colsum_bf16). */
int64_t mmpt_gemm_acc_colsum_rows(int64_t M, int64_t N, int64_t K);
/* Weight-gradient GEMMs (F32_ACC / F32_STORE) with K >> M·N are split along K into
 * fp32 slabs (workspace ≥ mmpt_gemm_workspace_bytes) summed in fixed order by a second
 * kernel — deterministic.  workspace may be NULL (then no split, same numerics). */
int64_t mmpt_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K, int epilogue);
int mmpt_gemm_bf16(int layout_a, int layout_b, int epilogue, int64_t M, int64_t N, int64_t K,
                   const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc,
                   const void* bias_bf16, const void* aux_bf16, int64_t ld_aux, void* C2,
                   int64_t ldc2, void* workspace, int64_t workspace_bytes, void* stream);
/* Plan query (measurement / diagnostics): the tile edge (256 → the big-tile kernel,
 * gemm4p_kernel, when it takes the problem — else gemm128_kernel; 128 → gemm128_kernel) and
 * the split-K count that mmpt_gemm_bf16 would use for this problem given `workspace_bytes`. */
int mmpt_gemm_plan(int64_t M, int64_t N, int64_t K, int epilogue, int64_t workspace_bytes,
                   int* tile, int* splits);
/* The exact kernel (as rocprofv3 names it, without the namespace) mmpt_gemm_bf16 launches
 * for this problem: "gemm4p_kernel<LA, LB, E>" (4-wave pipelined, 256x256 tiles) or
 * "gemm128_kernel<LA, LB, E>" (E = 100: split-K slabs), for 16-B aligned operands.  (Round 5:
 * the 8-wave gemm256 kernel is retired; gemm4p's K-tail form is "gemm4p_kt_kernel<LA, LB, E>" in
 * mmpt_gemm_last_kernel_name.)  NUL-terminated into buf. */
int mmpt_gemm_kernel_name(int layout_a, int layout_b, int epilogue, int64_t M, int64_t N,
                          int64_t K, int64_t workspace_bytes, char* buf, int len);
/* (ABI 11) The kernel the calling thread's most recent mmpt_gemm_bf16 call launched (its
 * choice also depends on operand alignment, which mmpt_gemm_kernel_name assumes 16-B). */
int mmpt_gemm_last_kernel_name(char* buf, int len);
/* (ABI 11) Rows of the calling thread's most recent mmpt_gemm_bf16 call that ran as a "tail
 * split" (0: none): with the plain or residual epilogue on 256x256 tiles, the bottom tile rows
 * that would run as a partial last round of the persistent launch are computed as a split-K
 * GEMM over the caller's workspace (counted in mmpt_gemm_workspace_bytes) followed by an
 * epilogue kernel; MMPT_GEMM_TAIL=0 disables it.  The probe event (below) then marks the end of
 * the main launch, before the tail. */
int64_t mmpt_gemm_last_tail_rows(void);
/* Measurement hook (bench.py): the next mmpt_gemm_bf16 call on this thread records
 * `hip_event` (a hipEvent_t) on its stream right after the main GEMM kernel, before
 * the split-K reduce, so the main kernel can be timed alone.  One-shot. */
void mmpt_gemm_probe_event(void* hip_event);

/* Bias gradient: dbias[n] (+)= f32(bf16(Σ_rows dy[r, n]))  — addmm backward's
 * grad_bias (sum over rows) under autocast. Deterministic two-stage reduction.
 * dbias2 (nullable) receives the same value (two biases fed by one gradient, e.g.
 * GPTNeoX dense.bias and dense_4h_to_h.bias under the parallel residual).
 * `workspace` ≥ mmpt_colsum_workspace_bytes(rows, cols). */
int64_t mmpt_colsum_workspace_bytes(int64_t rows, int64_t cols);
/* dbias[n] (+)= f32(bf16(Σ_r part[r, n])) over an fp32 [rows][cols] partial-sum matrix
 * (e.g. the C2 output of EPI_BF16_DGELU_COLSUM); deterministic (fixed order). */
int mmpt_colsum_f32(int64_t rows, int64_t cols, const float* part, float* dbias, float* dbias2,
                    int accumulate, void* stream);
int mmpt_colsum_bf16(int64_t rows, int64_t cols, const void* dy, int64_t ld, float* dbias,
                     float* dbias2, int accumulate, void* workspace, void* stream);

/* ------------------------------------------------------------------------
 * K4  nn.LayerNorm (fp32 under autocast), tf:modeling_gpt_neox.py:245-246
 * (two LNs on the same input: input_layernorm / post_attention_layernorm),
 * tf:modeling_vit.py:261-262,274,281.
 * y1 = bf16(LN(x; w1, b1)); optional y2 = bf16(LN(x; w2, b2)) sharing μ, rstd.
 * ---------------------------------------------------------------------- */
int mmpt_layernorm_fwd(int64_t rows, int64_t h, float eps, const float* x, int64_t ldx,
                       const float* w1, const float* b1, void* y1, const float* w2,
                       const float* b2, void* y2, float* mean, float* rstd, void* stream);
/* dx = dresid + LN'(dy1; w1) + LN'(dy2; w2)  (dresid / dy2 optional, dx may alias dresid);
 * dw*, db* accumulate (+=) into fp32 grads. `workspace` ≥ mmpt_layernorm_bwd_workspace_bytes. */
int64_t mmpt_layernorm_bwd_workspace_bytes(int64_t rows, int64_t h);
int mmpt_layernorm_bwd(int64_t rows, int64_t h, const float* x, int64_t ldx, const float* mean,
                       const float* rstd, const void* dy1, const float* w1, const void* dy2,
                       const float* w2, const float* dresid, float* dx, float* dw1, float* db1,
                       float* dw2, float* db2, void* workspace, void* stream);

/* Same backward with one workgroup per row (the fast path) and two optional fused
 * outputs: dx_bf16 (nullable) = bf16(dx), the operand of the next backward GEMMs
 * (replaces a separate cast); dsum (nullable, needs dx_bf16) += f32(bf16(Σ_rows
 * bf16(dx))) — the bias gradient autocast's addmm backward computes from that bf16
 * tensor (replaces a column sum); dsum2 (nullable) receives the same value.
 * `workspace` ≥ mmpt_layernorm_bwd_ex_workspace_bytes. */
int64_t mmpt_layernorm_bwd_ex_workspace_bytes(int64_t rows, int64_t h);
int mmpt_layernorm_bwd_ex(int64_t rows, int64_t h, const float* x, int64_t ldx, const float* mean,
                          const float* rstd, const void* dy1, const float* w1, const void* dy2,
                          const float* w2, const float* dresid, float* dx, void* dx_bf16,
                          float* dw1, float* db1, float* dw2, float* db2, float* dsum,
                          float* dsum2, void* workspace, void* stream);
/* fp32-output LayerNorm — CLIP's pre_layrnorm, whose output is the fp32 residual stream
 * (tf:models/clip/modeling_clip.py CLIPVisionTransformer.forward).  y, dy, dx fp32 [rows][h];
 * dw/db accumulate (+=); workspace = mmpt_layernorm_bwd_workspace_bytes(rows, h). */
int mmpt_layernorm_f32_fwd(int64_t rows, int64_t h, float eps, const float* x, const float* w,
                           const float* b, float* y, float* mean, float* rstd, void* stream);
int mmpt_layernorm_f32_bwd(int64_t rows, int64_t h, const float* x, const float* mean,
                           const float* rstd, const float* dy, const float* w, float* dx,
                           float* dw, float* db, void* workspace, void* stream);

/* RMSNorm (LlamaRMSNorm, tf:models/llama/modeling_llama.py, fp32 under autocast):
 * y = bf16(w · (x · rstd)), rstd = 1/sqrt(mean(x²) + eps).  Backward: dx = dresid +
 * RMS'(dy; w) (dresid optional, may alias dx), dw += Σ dy·x̂, optional dx_bf16 = bf16(dx);
 * deterministic two-stage dw reduction.  workspace ≥ mmpt_rmsnorm_bwd_workspace_bytes. */
int mmpt_rmsnorm_fwd(int64_t rows, int64_t h, float eps, const float* x, int64_t ldx,
                     const float* w, void* y, float* rstd, void* stream);
int64_t mmpt_rmsnorm_bwd_workspace_bytes(int64_t rows, int64_t h);
int mmpt_rmsnorm_bwd(int64_t rows, int64_t h, const float* x, int64_t ldx, const float* rstd,
                     const void* dy, const float* w, const float* dresid, float* dx,
                     void* dx_bf16, float* dw, void* workspace, void* stream);

/* ------------------------------------------------------------------------
 * K6  partial rotary embedding, tf:modeling_gpt_neox.py:93-151 (rotate_half on the
 * first rot_dims of each head, fp32 cos/sin tables [seq][rot_dims]), applied in place
 * to the q and k parts of a fused qkv buffer.  inverse=1 applies the transpose
 * rotation (backward of the forward rotation).
 * qkv element (token t, head h, part p∈{q,k,v}, dim d) lives at
 *   qkv[t*ld + h*head_stride + p*part_stride + d]   (K7 layout, tf:...:204-207)
 * ---------------------------------------------------------------------- */
int mmpt_rope_inplace(int64_t tokens, int64_t seq, int64_t heads, int64_t head_dim,
                      int64_t rot_dims, void* qkv, int64_t ld, int64_t head_stride,
                      int64_t part_stride, int64_t parts, const float* cos, const float* sin,
                      int inverse, void* stream);

/* ------------------------------------------------------------------------
 * K2/K3  scaled-dot-product attention (torch SDPA, causal for GPTNeoX
 * tf:modeling_gpt_neox.py:214-229, non-causal for ViT tf:modeling_vit.py:221-232).
 * q/k/v are read in place from the fused qkv buffer (layout above);
 * out [tokens][heads*head_dim] bf16 (row stride ld_out), lse fp32 [batch*heads*seq].
 * ---------------------------------------------------------------------- */
int mmpt_attention_fwd(int64_t batch, int64_t seq, int64_t heads, int64_t head_dim,
                       const void* qkv, int64_t ld, int64_t head_stride, int64_t part_stride,
                       int causal, float scale, void* out, int64_t ld_out, float* lse,
                       void* stream);
/* dqkv has the same layout as qkv. `workspace` ≥ mmpt_attention_bwd_workspace_bytes. */
int64_t mmpt_attention_bwd_workspace_bytes(int64_t batch, int64_t seq, int64_t heads,
                                           int64_t head_dim);
int mmpt_attention_bwd(int64_t batch, int64_t seq, int64_t heads, int64_t head_dim,
                       const void* qkv, int64_t ld, int64_t head_stride, int64_t part_stride,
                       int causal, float scale, const void* out, const void* dout,
                       int64_t ld_out, const float* lse, void* dqkv, void* workspace,
                       void* stream);
/* K3 + K4 backward (ABI 10): mmpt_attention_bwd followed by the inverse rotation of the q and
 * k parts (= mmpt_rope_inplace(..., parts = 2, inverse = 1) on dqkv: the backward of
 * `apply_rotary_pos_emb`, tf:models/gpt_neox/modeling_gpt_neox.py:204-207).  head_dim 256 with
 * 64 rotary dims (Pythia) rotates inside the dK / dQ epilogues, bitwise the same as the two
 * calls; other shapes run them one after the other.  Same workspace as mmpt_attention_bwd. */
int mmpt_attention_bwd_rope(int64_t batch, int64_t seq, int64_t heads, int64_t head_dim,
                            const void* qkv, int64_t ld, int64_t head_stride, int64_t part_stride,
                            int causal, float scale, const void* out, const void* dout,
                            int64_t ld_out, const float* lse, void* dqkv, void* workspace,
                            int64_t rot_dims, const float* cos, const float* sin, void* stream);
/* K17  grouped-query attention (Llama-3: LlamaAttention + repeat_kv, tf:models/llama/
 * modeling_llama.py; SDPA with enable_gqa): query head h at qkv[t*ld + h*head_stride + d],
 * its kv head j = h / (heads / kv_heads) at qkv[t*ld + k_offset + j*head_stride + d] and
 * qkv[t*ld + v_offset + j*head_stride + d] (Llama's fused q|k|v projection: k_offset =
 * heads*head_dim, v_offset = k_offset + kv_heads*head_dim).  dqkv has the same layout; dK/dV
 * are summed over the query heads of the group inside one workgroup (no atomics).
 * mmpt_attention_fwd/bwd are the kv_heads = heads case (k_offset = part_stride,
 * v_offset = 2*part_stride). */
int mmpt_attention_gqa_fwd(int64_t batch, int64_t seq, int64_t heads, int64_t kv_heads,
                           int64_t head_dim, const void* qkv, int64_t ld, int64_t head_stride,
                           int64_t k_offset, int64_t v_offset, int causal, float scale, void* out,
                           int64_t ld_out, float* lse, void* stream);
int mmpt_attention_gqa_bwd(int64_t batch, int64_t seq, int64_t heads, int64_t kv_heads,
                           int64_t head_dim, const void* qkv, int64_t ld, int64_t head_stride,
                           int64_t k_offset, int64_t v_offset, int causal, float scale,
                           const void* out, const void* dout, int64_t ld_out, const float* lse,
                           void* dqkv, void* workspace, void* stream);

/* ------------------------------------------------------------------------
 * K12  ForCausalLMLoss (tf:loss/loss_utils.py:32-68): fp32 upcast, CE with
 * ignore_index, reduction sum / num_items.  labels are ALREADY shifted (label of row r
 * is the target for logits row r).  Writes per-row loss (0 for ignored rows) and,
 * if dlogits != NULL, dlogits = (softmax - onehot) * grad_scale in bf16
 * (dlogits may alias logits: fused fwd+bwd, one read of the logits).
 * ---------------------------------------------------------------------- */
int mmpt_cross_entropy(int64_t rows, int64_t vocab, int64_t vocab_valid, const void* logits,
                       int64_t ld, const int64_t* labels, int64_t ignore_index, float grad_scale,
                       float* loss_rows, void* dlogits, int64_t ld_d, void* stream);
/* out[0] = Σ x[i] (deterministic).  workspace ≥ mmpt_sum_workspace_bytes(n). */
int64_t mmpt_sum_workspace_bytes(int64_t n);
int mmpt_sum_f32(int64_t n, const float* x, float* out, void* workspace, void* stream);

/* Loss-row compaction: the lm_head and the cross-entropy run only over rows whose
 * (shifted) label is not ignore_index (ForCausalLMLoss ignores the others: their logits are
 * never consumed and their gradient is exactly zero, so skipping them changes no result).
 * gather: dst[r] = src[idx[r]]; expand: dst[r] = map[r] >= 0 ? src[map[r]] : 0.  bf16 rows. */
int mmpt_gather_rows_bf16(int64_t rows, int64_t h, const int32_t* idx, const void* src,
                          int64_t ld_src, void* dst, int64_t ld_dst, void* stream);
int mmpt_expand_rows_bf16(int64_t rows, int64_t h, const int32_t* map, const void* src,
                          int64_t ld_src, void* dst, int64_t ld_dst, void* stream);

/* ------------------------------------------------------------------------
 * K8/K9  embedding gather + LLaVA image-token merge
 * (tf:modeling_gpt_neox.py:338; tf:models/llava/modeling_llava.py:243-248).
 * out[r] = img_map[r] >= 0 ? f32(img[img_map[r]]) : table[ids[r]]     (f32 rows)
 * bwd (aten::embedding_dense_backward, deterministic): the text rows sorted by id
 * (stable) form nseg segments; segment s covers perm[seg_off[s] .. seg_off[s+1]) and
 * dtable[seg_id[s]] += Σ (in position order, fp32) dout[perm[r]] — one writer per
 * table row, no atomics.  dimg[img_map[r]] = bf16(dout[r]) for image rows.  h % 8 == 0.
 * ---------------------------------------------------------------------- */
int mmpt_embed_fwd(int64_t rows, int64_t h, const int64_t* ids, const float* table,
                   const int32_t* img_map, const void* img, float* out, void* stream);
int mmpt_embed_bwd(int64_t rows, int64_t h, int64_t nseg, const int32_t* seg_id,
                   const int32_t* seg_off, const int32_t* perm, const int32_t* img_map,
                   const float* dout, float* dtable, void* dimg, void* stream);

/* Device-side segment build for the embedding backward (ABI 8; replaces round 2's host
 * numpy argsort behind the same semantics): key[r] = ids[r] (rows with id == skip_id — the
 * LLaVA image slots, pass -1 for none — and out-of-range ids are excluded), stable counting
 * sort of (key, row) (hand-written LSD radix sort, linear in rows; ABI 9) → perm[0 .. text rows); segments as above with seg_id/seg_off sized [rows] / [rows+1]
 * and the segment count written to DEVICE memory *nseg; *bad = 1 iff some id lies outside
 * [0, vocab) and is not skip_id.  Workspace from mmpt_embed_segments_workspace_bytes (-1 on
 * bad sizes).  Replaces the CPU side of aten::embedding_dense_backward's index sort
 * (torch/nn/functional.py embedding → tf:modeling_gpt_neox.py:338 embed_in). */
int64_t mmpt_embed_segments_workspace_bytes(int64_t rows, int64_t vocab);
int mmpt_embed_segments(int64_t rows, const int64_t* ids, int64_t vocab, int64_t skip_id,
                        int32_t* seg_id, int32_t* seg_off, int32_t* perm, int32_t* nseg,
                        int32_t* bad, void* workspace, int64_t ws_bytes, void* stream);
/* mmpt_embed_bwd with the segment count read from device memory (grid sized by max_seg,
 * an upper bound such as the number of text rows). */
int mmpt_embed_bwd_dev(int64_t rows, int64_t h, int64_t max_seg, const int32_t* nseg,
                       const int32_t* seg_id, const int32_t* seg_off, const int32_t* perm,
                       const int32_t* img_map, const float* dout, float* dtable, void* dimg,
                       void* stream);

/* ABI 13: mmpt_embed_bwd_dev with segments longer than 1024 rows (one id padding most of a
 * batch, src/data/llava_data.py:95) split over 256-row chunks of the sorted order: each chunk
 * sums its piece of a long segment in position order, the pieces are added in chunk order
 * (deterministic; a different fp32 association than one serial loop for those segments only —
 * every segment of <= 1024 rows is summed bitwise as mmpt_embed_bwd_dev does).  max_seg <= rows
 * bounds the text rows; workspace from mmpt_embed_bwd_split_workspace_bytes(max_seg, h). */
int64_t mmpt_embed_bwd_split_workspace_bytes(int64_t rows, int64_t h);
int mmpt_embed_bwd_split(int64_t rows, int64_t h, int64_t max_seg, const int32_t* nseg,
                         const int32_t* seg_id, const int32_t* seg_off, const int32_t* perm,
                         const int32_t* img_map, const float* dout, float* dtable, void* dimg,
                         void* workspace, int64_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * K10  ViT patch embedding (Conv2d k=s=patch, tf:modeling_vit.py:42-69) as
 * im2col (bf16, k-order = (c, ky, kx) = Conv2d weight flattening) + GEMM, then
 * CLS concat + position embedding (tf:modeling_vit.py:129-160).
 * ---------------------------------------------------------------------- */
int mmpt_im2col_patches(int64_t batch, int64_t channels, int64_t image, int64_t patch,
                        const float* pixels, void* cols, void* stream);
/* any patch size (CLIP-L/14: 14): cols [B·(S/p)²][ld_cols] bf16, ld_cols >= C·p·p, the
 * columns past C·p·p zero-filled (16-B GEMM rows; the patch weight carries zero columns). */
int mmpt_im2col_patches_ex(int64_t batch, int64_t channels, int64_t image, int64_t patch,
                           const float* pixels, void* cols, int64_t ld_cols, void* stream);
/* out[b, 0] = cls + pos[0];  out[b, 1+i] = f32(patch_out[b*np+i]) + pos[1+i]   (f32) */
int mmpt_vit_embed_fwd(int64_t batch, int64_t num_patches, int64_t h, const void* patch_out,
                       const float* cls, const float* pos, float* out, void* stream);
/* dcls += Σ_b dout[b,0]; dpos += Σ_b dout[b,:]; dpatch = bf16(dout[b, 1:]) */
int mmpt_vit_embed_bwd(int64_t batch, int64_t num_patches, int64_t h, const float* dout,
                       float* dcls, float* dpos, void* dpatch, void* stream);
/* LLaVA feature select (vision_feature_select_strategy="default": drop CLS,
 * tf:modeling_llava.py:163-166):  out[b*np+i] = bf16(x[b*(np+1)+1+i]). */
int mmpt_select_patches_fwd(int64_t batch, int64_t num_patches, int64_t h, const float* x,
                            void* out, void* stream);
/* dx[b*(np+1)+1+i] (+)= f32(dout[b*np+i]); dx[b*(np+1)] (+)= 0 */
int mmpt_select_patches_bwd(int64_t batch, int64_t num_patches, int64_t h, const void* dout,
                            float* dx, int accumulate, void* stream);

/* ------------------------------------------------------------------------
 * K13/K14  clip_grad_norm_ + Adam / AdamW step over one flat fp32 parameter
 * buffer (src/benchmarking/utils.py:66-76; torch.optim.Adam(W) single-tensor
 * semantics; DeepSpeed FusedAdam csrc/adam/multi_tensor_adam.cu).
 * Writes the bf16 shadow copy (autocast weight cast, K15) in the same pass.
 * ---------------------------------------------------------------------- */
int64_t mmpt_l2norm_workspace_bytes(int64_t n);
/* out[0] = Σ x[i]^2 (fp32, deterministic) */
int mmpt_sumsq_f32(int64_t n, const float* x, float* out, void* workspace, void* stream);
/* grad_scale_ptr (device, nullable): multiply g by *grad_scale_ptr (clip coefficient). */
int mmpt_adam_step(int64_t n, float* param, const float* grad, float* exp_avg,
                   float* exp_avg_sq, void* param_bf16, float lr, float beta1, float beta2,
                   float eps, float weight_decay, int adamw, int64_t step,
                   const float* grad_scale_ptr, void* stream);
/* ABI 13: the same update, and the gradient zeroed as it is consumed (zero_grad fused: the
 * step's last read of g and the next step's zero are one pass; the optimizer overlapped with
 * the next forward runs it per parameter unit on its own stream).  16-B aligned buffers.
 * max_blocks > 0 caps the grid (256-thread workgroups, grid-stride): the overlapped update
 * runs one workgroup per CU beside the forward's persistent GEMMs. */
int mmpt_adam_step_zero_grad(int64_t n, float* param, float* grad, float* exp_avg,
                             float* exp_avg_sq, void* param_bf16, float lr, float beta1,
                             float beta2, float eps, float weight_decay, int adamw, int64_t step,
                             const float* grad_scale, int max_blocks, void* stream);
/* clip coefficient from Σg²: coef = min(1, max_norm / (sqrt(sumsq) + 1e-6)) (device scalar) */
int mmpt_clip_coef(const float* sumsq, float max_norm, float* coef, void* stream);

/* elementwise helpers */
int mmpt_cast_f32_bf16(int64_t n, const float* src, void* dst, void* stream);
/* dst[c][r] = src[r][c] (bf16): the transposed weight shadow W^T that lets every
 * input-gradient GEMM dX = dY·W read both operands K-contiguous (refreshed once per
 * optimizer step, after the Adam kernel wrote the bf16 shadow). */
int mmpt_transpose_bf16(int64_t rows, int64_t cols, const void* src, int64_t ld_src, void* dst,
                        int64_t ld_dst, void* stream);
/* ABI 14: every W^T of a parameter store in one launch.  desc: DEVICE int64 [n][4] =
 * {offset, rows, cols, first_tile} per weight — src + offset holds [rows][cols] (dense),
 * dst + offset receives [cols][rows]; first_tile = the sum of ceil(rows/64)·ceil(cols/64)
 * over the weights before it, total_tiles the sum over all.  rows, cols, offsets multiples
 * of 8; the same bits as mmpt_transpose_bf16 per weight. */
int mmpt_transpose_bf16_batched(int64_t n, const int64_t* desc, int64_t total_tiles,
                                const void* src, void* dst, void* stream);


/* ------------------------------------------------------------------------
 * ZeRO++ quantized communication (sharding = "zero_3++"): replaces DeepSpeed's
 * `zero_quantized_weights` / `zero_quantized_gradients` kernels that
 * src/train.py:196-201 switches on.  Blockwise symmetric quantization, 256-element
 * blocks that never straddle a part (a rank's shard of `n_part` elements, a multiple
 * of 4), one fp32 scale per block, scales laid out [part][block].
 *   quant_int8: q = rint(x·127/absmax) ∈ [-127, 127], scale = absmax/127 (bf16 in);
 *   dequant_int8: y = bf16(q·scale);
 *   quant_int4: q = rint(x·7/absmax) ∈ [-7, 7], two per byte (low nibble = even
 *               element), scale = absmax/7 (fp32 in);
 *   dequant_int4_sum: dst[i] += Σ_{r<parts} q_r[i]·scale_r (rank order, fp32).
 * ---------------------------------------------------------------------- */
int64_t mmpt_quant_blocks(int64_t n_part);
int mmpt_quant_int8(int64_t n_part, int64_t parts, const void* src_bf16, void* dst_i8,
                    float* scales, void* stream);
int mmpt_dequant_int8(int64_t n_part, int64_t parts, const void* src_i8, const float* scales,
                      void* dst_bf16, void* stream);
int mmpt_quant_int4(int64_t n_part, int64_t parts, const float* src, void* dst_u8,
                    float* scales, void* stream);
int mmpt_dequant_int4_sum(int64_t n_part, int64_t parts, const void* src_u8, const float* scales,
                          float* dst, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MMPT_H_ */
