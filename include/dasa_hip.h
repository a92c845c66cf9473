/*
 * dasa_hip.h — C-ABI of libdasa_hip.so, the MI355X (gfx950) kernel library behind the
 * DASA per-step navigation policy (agent_dg rollout).
 *
 * Conventions (every entry point):
 *   - pointers are device pointers to fp32 (or int32/int64/uint8 where named) owned by the caller;
 *   - no allocation and no host synchronisation inside a call, so every call is hipGraph-capturable;
 *   - `stream` is a hipStream_t passed as void*; work is enqueued on it;
 *   - the return value is a hipError_t (0 == hipSuccess); shape/alignment violations return
 *     hipErrorInvalidValue (1) before anything is launched;
 *   - row-major storage; "ld" is the row stride in elements.
 *
 * Each entry point names the reference code it replaces (paths relative to the DASA repo).
 */
#ifndef DASA_HIP_H
#define DASA_HIP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- library ------------------------------------------------------------------------------- */
int dasa_version(void);                 /* ABI version, bumped on any signature change */
const char* dasa_build_info(void);      /* "gfx950 ..." */
const char* dasa_error_string(int err); /* hipGetErrorString of a returned code */

/* ---- GEMM (MFMA f32 32x32x2) -----------------------------------------------------------------
 * C[b] = epilogue( alpha * opA(A[b]) @ opB(B[b]) ) (+ beta * C[b])
 *   opA: 0 = A stored [M][K] (lda >= K), 1 = A stored [K][M] (lda >= M)
 *   opB: 0 = B stored [K][N] (ldb >= N), 1 = B stored [N][K] (ldb >= K)   (nn.Linear weight = opB 1)
 * Epilogue order: v = alpha*acc; v += bias[n]; v = act(v); v = v*aux[m,n] (gate); v *= colscale[n];
 *                 v += beta*C[m,n].
 * 16-B aligned operands with ld % 4 == 0 stream with dwordx4 loads; others take a scalar-load variant.
 * Replaces every nn.Linear / torch.bmm on the hot path (model.py:263-313, vilmodel.py:179-309,
 * agent_dg.py:1519 DGAdaChannel.a_fc, r2rmodel.py:2241-2251 LSTM input projections).       */
enum dasa_act {
  DASA_ACT_NONE = 0, DASA_ACT_RELU = 1, DASA_ACT_GELU = 2, DASA_ACT_TANH = 3, DASA_ACT_SIGMOID = 4
};
typedef struct dasa_gemm_desc {
  int32_t M, N, K, batch;
  int32_t opA, opB;
  const float* A; int64_t lda; int64_t strideA;
  const float* B; int64_t ldb; int64_t strideB;
  float* C;       int64_t ldc; int64_t strideC;
  const float* bias;       /* [N] or NULL */
  int32_t act;             /* enum dasa_act */
  const float* aux;        /* gate multiplier [M][ld_aux] or NULL (DGAdaChannel: sigmoid(.)*f) */
  int64_t ld_aux; int64_t strideAux;
  const float* colscale;   /* [N] or NULL (shared env-drop noise, agent_dg.py:780-785) */
  float alpha, beta;
} dasa_gemm_desc;
/* One block of a batched strided copy (dasa_copy_segments): n0 x n1 rows of row_bytes contiguous bytes,
   row (i0, i1) at src + i0*src_s0 + i1*src_s1 (bytes), written to dst + i0*dst_s0 + i1*dst_s1. */
typedef struct dasa_copy_seg {
  const void* src; void* dst;
  int64_t n0, n1, row_bytes;
  int64_t src_s0, src_s1, dst_s0, dst_s1;
} dasa_copy_seg;
#define DASA_COPY_MAX_SEGS 16
/* Workspace bytes for this descriptor: 64 KiB of stream-K arrival counters, then split-K partials
 * (the skinny M <= 32 decoder GEMMs' split-K partials) or stream-K partial-tile slabs (mid-size GEMMs that do not fill the CUs).
 * The buffer must be ZERO-FILLED when first allocated; every call leaves the counters zero again,
 * so one buffer can be reused by consecutive calls on one stream (never by overlapping calls).
 * Passing ws == NULL (or too small) runs the GEMM without split-K / stream-K instead. */
int64_t dasa_gemm_f32_workspace(const dasa_gemm_desc* d);
/* Tuning hook: pin tile configuration `cfg % 64` (and, when cfg >= 64, split-K = cfg / 64) for
 * subsequent calls (-1 = automatic choice).
 * Returns the number of configurations. Host-only; not thread-safe with concurrent GEMM planning. */
int dasa_gemm_force_config(int cfg);
/* A/B hook for the bf16x6 plan (dasa_gemm_f32x6): split-K on many-tile problems to fill the last round of
 * tiles; 0 = off (the default; DASA_X6_BALANCE=1/2 in the environment starts on), 1 = 2- or 3-way,
 * 2 = 2-way only. Host-only setting. */
int dasa_gemm_x6_set_balance(int32_t mode);
/* Tuning hook for the skinny (M <= 32) weight-streaming GEMMs: target wave count of the plan (0 = do
 * not use the skinny kernels, -1 = default) and a pinned K-steps-per-wave (1/2/4/8, -1 = plan);
 * ks + 16 (16 = plan's KS) also turns the 17..20-row hybrid MFMA + VALU form off. Host-only; returns 0. */
int dasa_gemm_skinny_tune(int target_waves, int ks);
int dasa_gemm_f32(const dasa_gemm_desc* d, void* ws, int64_t ws_bytes, void* stream);
/* bf16-operand nn.Linear forward for BASELINE configs[4] (B = 256, bf16 with fp32 accumulation):
 * C = epilogue(A . B^T) with A fp32 [M][lda] rounded to bf16 (RNE) on load and B a bf16 weight copy
 * [N][ldb] (pass its address as d->B), fp32 accumulation, the same fused epilogue as dasa_gemm_f32.
 * Only opA = 0, opB = 1; K % 64 == 0, lda % 4 == 0, ldb % 8 == 0, 16-B aligned A and B.
 * Replaces the nn.Linear forwards of model.py / vilmodel.py / agent_dg.py:1519 in that config. */
int dasa_gemm_bf16(const dasa_gemm_desc* d, void* stream);
/* dasa_gemm_bf16 with bf16 activations (configs[4]'s FFN: the GELU output is stored as bf16 by the
   FFN-up GEMM and read as bf16 by the FFN-down GEMM; the values equal the fp32-A path's, which rounds A
   on load the same way). flags: DASA_BF16_A = A is bf16 (lda, strideA in bf16 elements, lda % 8 == 0),
   DASA_BF16_C = C is written as bf16, round to nearest even (ldc, strideC in bf16 elements; beta 0). */
#define DASA_BF16_A 1
#define DASA_BF16_C 2
int dasa_gemm_bf16_ex(const dasa_gemm_desc* d, int32_t flags, void* stream);
/* LDS-DMA probe form of the bf16 GEMM with a bf16 A (both operands by global_load_lds, a 3-stage ring): 1 on,
 * 0 off (default; DASA_BF16_DMA=1 starts it on), < 0 only queries. Returns the previous setting. Host-only. */
int dasa_gemm_bf16_dma(int32_t on);
/* y[i] = bf16(x[i]) (round to nearest even), n even; weight copies for dasa_gemm_bf16. */
int dasa_f32_to_bf16(const float* x, uint16_t* y, int64_t n, void* stream);
/* fp32 nn.Linear forward at fp32 accuracy on the bf16 matrix cores ("bf16x6"): every fp32 operand is
 * split exactly into bf16 planes hi + mid + lo, and C = epilogue(sum of the six products hh, hm, mh, hl,
 * lh, mm) with fp32 accumulation — the dropped terms are below 2^-25 of each product, under fp32's own
 * rounding. A fp32 [M][lda] is split on load; B = the weight pre-split by dasa_f32_split3_bf16: pass
 * the hi plane as d->B with d->ldb its row stride, the mid / lo planes `plane` elements further on.
 * Only opA = 0, opB = 1; K % 32 == 0, lda % 4 == 0, ldb % 8 == 0, plane % 8 == 0, 16-B aligned A / B.
 * Same fused epilogue as dasa_gemm_f32. Replaces the nn.Linear forwards (vilmodel.py BERT / LXRT
 * projections and FFN, model.py decoder linears, agent_dg.py:1519 DGAdaChannel.a_fc). */
int dasa_gemm_f32x6(const dasa_gemm_desc* d, int64_t plane, void* stream);
/* The same with a workspace (ws: zero-initialised once, >= dasa_gemm_f32x6_workspace(d) bytes; its
 * leading counters are re-armed by every call, so one buffer serves every call on one stream): problems
 * with few output tiles (< 128 of 128x128) split K over several workgroups per tile, reduced in-kernel
 * by the last split to arrive in a fixed order (deterministic). Workspace 0 = no split needed. */
int64_t dasa_gemm_f32x6_workspace(const dasa_gemm_desc* d);
int dasa_gemm_f32x6_ws(const dasa_gemm_desc* d, int64_t plane, void* ws, int64_t ws_bytes, void* stream);
/* Many-tile problems whose last round of workgroups would leave most CUs idle (12800 x 768: 2.34 rounds of
 * 128 x 128 tiles) run as two launches over row bands when the workspace allows it: whole rounds of the
 * planned form, then the remaining rows with K split to fill one round (DASA_X6_TAIL=0: off). This returns
 * how many kernels dasa_gemm_f32x6_ws launches for `d` with a workspace of ws_bytes (profiling: per-kernel
 * durations -> per-call rates). */
int dasa_gemm_f32x6_kernels(const dasa_gemm_desc* d, int64_t ws_bytes);
/* Test / A/B hook for that tail plan: 1 = on where the cost model takes it (the default unless DASA_X6_TAIL=0),
 * 0 = every call one launch. Host-only setting; returns 0 (hipErrorInvalidValue outside {0, 1}). */
int dasa_gemm_x6_set_tail(int32_t on);
/* fp32-accurate TN GEMM on the bf16 matrix cores (bf16x6, gemm_tn.hip) for long-K weight gradients:
 * C = epilogue(alpha * A^T B) (+ beta C) with A fp32 [K][lda] (M contiguous) and B fp32 [K][ldb] (N contiguous),
 * both split into bf16 planes on their way into LDS — the six products and accumulation order of
 * dasa_gemm_f32x6. Only opA = 1, opB = 0, batch 1; M, N, lda, ldb even, 8-B aligned A / B; any K >= 1.
 * Few-tile problems split K over workgroups (ws: zero-initialised once, >= dasa_gemm_f32x6_tn_workspace(d)
 * bytes, counters re-armed by every call; without it one workgroup per tile). Replaces the weight-gradient
 * products dW = dY^T X of the bi-LSTM (r2rmodel.py:2339-2343 nn.LSTM weight_ih / weight_hh) and of the
 * decoder / critic linears (model.py) in the backward of agent_dg.py:1389-1405. */
int dasa_gemm_f32x6_tn(const dasa_gemm_desc* d, void* ws, int64_t ws_bytes, void* stream);
int64_t dasa_gemm_f32x6_tn_workspace(const dasa_gemm_desc* d);
/* Sweep / test hook of that kernel: form (-1 plan, 0 one LDS stage with two workgroups per CU, 1 two stages)
 * and split count (-1 plan, 1..16). Host-only setting; returns 0. */
int dasa_gemm_x6_tn_config(int32_t form, int32_t splitk);
/* bf16x6 NT GEMM with A ALSO pre-split into three bf16 planes (gemm_x6p.hip; the producer writes the planes):
 * every operand byte goes to LDS by LDS-DMA, the MFMA loop is dasa_gemm_f32x6's (bitwise equal to its
 * one-launch 128 x 128 form). d->A / d->B = the hi planes (bf16 elements, strides lda / ldb), the mid / lo
 * planes aplane / wplane elements further on; form 3 = 128 x 128 tiles and a three-stage DMA ring, form 2 =
 * 256 x 128 and two stages. K % 32 == 0, lda / ldb / planes % 8 == 0, 16-B aligned, batch 1. */
int dasa_gemm_f32x6_pp(const dasa_gemm_desc* d, int64_t wplane, int64_t aplane, int32_t form, void* stream);
/* bf16x6 NT GEMM with 64-deep K steps (gemm_k64.hip): one LDS stage holds a 64-deep slab, so every wave runs
 * twice the MFMAs between barriers; bitwise equal to dasa_gemm_f32x6's one-launch 128 x 128 form. Same operands
 * as dasa_gemm_f32x6 (A fp32, W pre-split with plane stride `plane`); form 1 = 128 x 128 tiles (one workgroup
 * per CU), 2 = 128 x 64, 3 = 64 x 128 (two per CU). K % 64 == 0. Probe entry (measured 0.70-0.80x the
 * dasa_gemm_f32x6 plan; no plan routes here) for the same nn.Linear calls (vilmodel.py:179-309). */
int dasa_gemm_f32x6_k64(const dasa_gemm_desc* d, int64_t plane, int32_t form, void* stream);
/* x [rows][ldx] fp32 -> y = three bf16 planes [3][rows][cols] (hi, mid, lo; plane stride rows*cols),
 * x = hi + mid + lo exactly for normal fp32 values; cols % 8 == 0, 16-B aligned x and y. */
int dasa_f32_split3_bf16(const float* x, int64_t ldx, uint16_t* y, int32_t rows, int32_t cols, void* stream);

/* ---- elementwise / reductions ---------------------------------------------------------------- */
/* y = LayerNorm(dropout_p(x) + res) over N columns (eps), optionally saving mean/rstd [M] and the
 * pre-norm sum xsum [M][N] for backward (each may be NULL; res may be NULL).
 * vilmodel.py:239-250, 296-309 (BertSelfOutput/BertOutput), 1067-1095 (VisionEncoder).      */
int dasa_layernorm_fwd(const float* x, const float* res, const float* gamma, const float* beta,
                       float* y, float* mean, float* rstd, float* xsum, int32_t M, int32_t N, float eps,
                       float drop_p, uint64_t seed, void* stream);
/* The same, also writing ybf = bf16(y) (RNE; 8-B aligned, [M][N]): configs[4]'s bf16 mode hands it to the next
 * bf16 GEMM as its A operand — bitwise what that GEMM would round y to on load, at half the A bytes.       */
int dasa_layernorm_fwd_bf16(const float* x, const float* res, const float* gamma, const float* beta,
                            float* y, uint16_t* ybf, float* mean, float* rstd, float* xsum, int32_t M, int32_t N,
                            float eps, float drop_p, uint64_t seed, void* stream);
/* dx = dLN/d(xsum) (= grad of both x-after-dropout and res); dgamma/dbeta accumulated (+=) by a
 * fixed-order column reduction in the same launch (deterministic, no atomics). */
int dasa_layernorm_bwd(const float* dy, const float* xsum, const float* gamma, const float* mean,
                       const float* rstd, float* dx, float* dgamma, float* dbeta,
                       int32_t M, int32_t N, void* stream);

/* BertEmbeddings.forward (vilmodel.py:161-176): word[ids] + pos[t] + type[0] -> LN -> dropout. */
int dasa_bert_embed_fwd(const int64_t* ids, const float* word, const float* pos, const float* type0,
                        const float* gamma, const float* beta, float* out,
                        int32_t B, int32_t L, int32_t H, float eps, float drop_p, uint64_t seed,
                        void* stream);

/* Masked multi-head attention core (BertSelfAttention / BertOutAttention, vilmodel.py:214-236,
 * 481-506): ctx = softmax(Q K^T * scale + addmask[b, k]) V per head; Q/K/V/out row-major with
 * heads interleaved as [.., heads*dh]. addmask: [B][Lk] additive (-10000 for pads) or NULL.
 * dh = 64, Lq <= 128, Lk <= 128; Q/K/V 16-B aligned with ld % 4 == 0.                       */
int dasa_mha_fwd(const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* V, int64_t ldv,
                 const float* addmask, float* out, int64_t ldo, float* probs,
                 int32_t B, int32_t heads, int32_t Lq, int32_t Lk, int32_t dh, float scale,
                 float drop_p, uint64_t seed, void* stream);
/* The same attention core with bf16 Q/K/V (BASELINE configs[4]'s bf16 mode, forward only): bf16 operands
 * on v_mfma_f32_32x32x16_bf16, fp32 accumulation / scale / mask / softmax, P rounded to bf16 (RNE) for
 * P V. Q/K/V/out are bf16 element pointers with ld in elements (ld % 8 == 0, 16-B aligned); out is bf16
 * (RNE) when out_bf16 != 0, else fp32. No saved probabilities (no backward).                          */
int dasa_mha_fwd_bf16(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv,
                      const float* addmask, void* out, int64_t ldo, int32_t out_bf16, int32_t B, int32_t heads,
                      int32_t Lq, int32_t Lk, int32_t dh, float scale, float drop_p, uint64_t seed, void* stream);
/* Backward; probs are the forward's saved pre-dropout softmax [B][heads][Lq][Lk], the dropout mask
 * is regenerated from (drop_p, seed). dQ/dK/dV are written with the ld of Q/K/V. Lq, Lk <= 80 with
 * 16-B aligned dQ/dK/dV take the LDS-staged form (no atomics); larger shapes the row-streaming one. */
int dasa_mha_bwd(const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* V, int64_t ldv,
                 const float* probs, const float* dout, int64_t lddo,
                 float* dQ, float* dK, float* dV, int32_t B, int32_t heads, int32_t Lq, int32_t Lk,
                 int32_t dh, float scale, float drop_p, uint64_t seed, void* stream);
/* Workgroups per (batch, head) of the LDS-staged backward (Lq, Lk <= 80): each recomputes the whole dS
 * and writes its share of dQ / dK / dV rows (bitwise equal for every count). 0 = automatic (up to 4
 * while B x heads x parts <= 256; the finetune's B = 2), n >= 1 forced (at most 16), < 0 only
 * queries. Returns the previous setting. Host-only.                                               */
int dasa_mha_bwd_split(int32_t parts);
/* Diagnosis: the LDS-staged backward records workgroup 0's shader clock (s_memtime) at its 9 phase boundaries
 * into buf (9 uint64, device memory; NULL stops). Returns the record length. Host-only.                    */
int dasa_mha_bwd_stamps(void* buf);

/* ---- SoftDot / ShiftSoftDot attention (model.py:253-353) ------------------------------------
 * q [B][D] is linear_in(h) (computed by dasa_gemm_f32); ctx [B][N][ldn] (ldn >= D, batch stride
 * N*ldn, D <= 4096); mask [B][N] uint8 (1 = masked -> -inf) or NULL. Outputs any of scores [B][N]
 * (raw logits, output_prob=False), probs [B][N], wctx [B][D].
 * ws: dasa_attn_workspace(B, N, D) bytes, 16-B aligned, shared by the four calls below (B <= 32768);
 * its first 65536 32-bit words are arrival counters that must be ZERO on entry (calls leave them
 * zero) and the next 33 x 1024 are monotonic group-barrier counters (zero once), so a caller zeroes
 * the buffer once and reuses it on one stream for calls of any shape.
 * Implementations, same results to fp32 rounding: row-split (a batch row's rows over workgroups,
 * online-softmax merge by the last workgroup); forward with B >= 128 and N <= 36 (shift) / N <= 84
 * (SoftDot), whole-row (one
 * workgroup streams a batch row); backward with N <= 80, D % 128 == 0 and B * D/128 <= 1024 (the
 * decision step's B = 20), D-split (a batch row's 128-float column chunks over D/128 workgroups that
 * meet at a bounded group barrier; a timeout NaN-poisons the outputs and ORs 4 into the error word,
 * dasa_set_error_word); shift-attention forward with B < 128: two-launch D-split (row-dot partials,
 * then softmax + context per column chunk); candidate scores (no probs / wctx): one workgroup per
 * row at every B; SoftDot with probs / wctx at every B the whole-row form does not take: row-split
 * (mode 2: the two-launch D-split form for N <= 80, D % 128 == 0). Every kernel is built without
 * packed-FP32 VALU (r05: their results were corrupted beside starting MFMA-dense workgroups of another
 * kernel, the r04 row-split failure), and every form is bitwise reproducible under that load.
 * dasa_attn_set_mode: 0 = automatic (the default; DASA_ATTN_SPLIT=0 in the environment starts in
 * mode 1), 1 = row-split only, 2 = 0 with the D-split SoftDot forward, 3 = row-split only with
 * the r04 per-row-address loads (diagnosis, tools/rowsplit_diag.py), 4 = 0 with the shift forward on
 * the row-split kernel as well (A/B, tools/attn_mode_ab.py). Host-only setting.                     */
int64_t dasa_attn_workspace(int32_t B, int32_t N, int32_t D);
int dasa_attn_set_mode(int32_t mode);
/* Diagnosis hook (r05, tools/rowsplit_diag.py): arm a device buffer of `bytes` (16-B aligned) that the
 * NEXT row-split forward launch (attn_fwd_kernel, mode 1) fills with one record of
 * dasa_attn_debug_record_floats() floats per workgroup — HW_ID / XCC_ID / block index, every thread's 16
 * row partials, its q checksum, the wave partials as written to LDS and the summed row dots — and then
 * disarms. buf = NULL disarms. Host-only setting; not capture-safe; not used by the product path.   */
int dasa_attn_debug_buffer(float* buf, int64_t bytes);
int64_t dasa_attn_debug_record_floats(void);
int dasa_softdot_fwd(const float* q, const float* ctx, int64_t ldn, const uint8_t* mask,
                     float* scores, float* probs, float* wctx,
                     int32_t B, int32_t N, int32_t D, float* ws, void* stream);
/* Backward. dwctx [B][D] and/or dscores [B][N] (grad of raw logits); writes dq [B][D] and
 * dctx [B][N][ldn] (dctx += if accumulate; either may be NULL). probs are the forward's saved
 * softmax (for output_prob=False callers pass the softmax anyway; only dscores flows then).     */
int dasa_softdot_bwd(const float* q, const float* ctx, int64_t ldn, const float* probs,
                     const float* dwctx, const float* dscores, float* dq, float* dctx,
                     int32_t accumulate, int32_t B, int32_t N, int32_t D, float* ws, void* stream);
/* ShiftSoftDotAttention (model.py:318-353): 36 views as 3 elevation rows of 12 headings;
 * a = softmax(ctx.q); w = softmax(shift_logits) over K taps; a'[r][j] = sum_k w_k a[r][(j+k-K/2) mod 12];
 * wctx = sum_v a'_v ctx_v. Returns attn (pre-shift a), shifted a' and w for backward. */
int dasa_shift_attn_fwd(const float* q, const float* ctx, int64_t ldn, const float* shift_logits,
                        float* attn, float* shifted, float* wsm, float* wctx,
                        int32_t B, int32_t D, int32_t K, float* ws, void* stream);
int dasa_shift_attn_bwd(const float* q, const float* ctx, int64_t ldn, const float* attn,
                        const float* shifted, const float* wsm, const float* dwctx,
                        float* dq, float* dctx, float* dshift_logits, int32_t accumulate,
                        int32_t B, int32_t D, int32_t K, float* ws, void* stream);

/* ---- LSTM (model.py:437 nn.LSTMCell, r2rmodel.py:2241 nn.LSTM) ------------------------------ */
/* gates [B][4H] = x W_ih^T + b_ih + h W_hh^T + b_hh (PyTorch order i,f,g,o) -> h, c.
 * act_save [B][4H] holds sigmoid/tanh-activated gates for backward (may be NULL in eval). */
int dasa_lstm_cell_fwd(const float* gates, const float* c_prev, float* h, float* c, float* act_save,
                       int32_t B, int32_t H, void* stream);
int dasa_lstm_cell_bwd(const float* act_save, const float* c_prev, const float* c, const float* dh,
                       const float* dc, float* dgates, float* dc_prev, int32_t B, int32_t H, void* stream);

/* Packed bidirectional single-layer LSTM recurrence (pack_padded_sequence semantics,
 * r2rmodel.py:2339-2343). xproj [B][L][2][4H] = x W_ih^T + b_ih + b_hh for both directions;
 * whh_fwd/whh_bwd [4H][H] (weight_hh_l0 / weight_hh_l0_reverse); lengths [B] int32 (any order).
 * Writes out [B][L][2H] ([fwd,bwd]),
 * h_n/c_n [2][B][H], and (if save != NULL) save = {act [L][2][B][4H], c [L][2][B][H]}.
 * ws: dasa_bilstm_workspace(B, H) bytes (ping-pong state; + recurrent gates when B > 32; + the converted
 * W_hh of the step path, dasa_bilstm_fwd_bf16).                                                   */
int64_t dasa_bilstm_workspace(int32_t B, int32_t H);
int dasa_bilstm_fwd(const float* xproj, const float* whh_fwd, const float* whh_bwd,
                    const int32_t* lengths, float* out, float* h_n, float* c_n, float* save_act,
                    float* save_c, int32_t B, int32_t L, int32_t H, float* ws, void* stream);
/* BPTT: dout [B][L][2H], dh_n/dc_n [2][B][H] (may be NULL) -> dgates [B][L][2][4H] (time-major
 * grads of the pre-activation gates; zero at padded steps). B <= 32, H % 64 == 0.
 * ws: dasa_bilstm_bwd_workspace(B, H) bytes (carries + W_hh^T of both directions).              */
int64_t dasa_bilstm_bwd_workspace(int32_t B, int32_t H);
int dasa_bilstm_bwd(const float* whh_fwd, const float* whh_bwd, const int32_t* lengths,
                    const float* save_act, const float* save_c,
                    const float* dout, const float* dh_n, const float* dc_n, float* dgates,
                    int32_t B, int32_t L, int32_t H, float* ws, void* stream);
/* hprev [2][B][L][H]: the recurrent input each step saw (fwd: out[b][t-1][:H], bwd: out[b][t+1][H:]),
 * zero at the sequence ends — the right operand of dW_hh = sum_t dgates_t^T hprev_t.            */
/* Recurrence implementation for dasa_bilstm_fwd/bwd: 0 = automatic (one persistent launch
 * per sequence when B <= 32 and H is a multiple of 256 up to 1024, else one launch per timestep),
 * 1 = per-timestep launches only, 2 = persistent only (error when not eligible). Host-only setting. */
int dasa_bilstm_set_mode(int mode);
/* Forward step path at B > 32 (one launch per timestep: B > 192, e.g. configs[4]'s B = 256, or mode 1): the
 * recurrent product of both directions is one batched GEMM per timestep on W_hh converted once per call in
 * the workspace — the bf16x6 fp32 GEMM (dasa_bilstm_fwd_x6 on, the default) or, with on = 1 here, bf16
 * W_hh and h (rounded on load) with fp32 accumulation (configs[4]'s bf16 mode; ops.bf16_matmul sets it).
 * < 0 only queries. Returns the previous setting. Host-only.                                      */
int dasa_bilstm_fwd_bf16(int32_t on);
/* B > 32 BPTT recurrent product (dgates_prev . W_hh per timestep): 1 = the bf16x6 fp32 GEMM on W_hh^T
 * pre-split per call (default; env DASA_BPTT_X6=0 or DASA_GEMM_EMU=0 start at 0), 0 = dasa_gemm_f32;
 * < 0 only queries. Returns the previous setting. Host-only.                                     */
int dasa_bilstm_bptt_x6(int32_t on);
/* Persistent BPTT (B <= 32) at H = 1024, B <= 16: 1 = one 16-row tile of the recurrent product (half the
 * hand-off loads and MFMAs of the two-tile form, the same products in the same order: bitwise equal;
 * default; env DASA_BPTT_ONE_TILE=0 starts at 0), 0 = the two-tile form; < 0 only queries. Returns the
 * previous setting. Host-only.                                                                     */
int dasa_bilstm_bptt_one_tile(int32_t on);
/* Persistent forward recurrence at H = 1024, B <= 64: 1 = recurrent product as bf16x6 (three exact bf16 planes of
 * h and W_hh, six products on bf16 MFMA; fp32-accurate; default; env DASA_LSTM_X6=0 or DASA_GEMM_EMU=0
 * start at 0), 0 = native fp32 MFMA; < 0 only queries. Returns the previous setting. Host-only.   */
int dasa_bilstm_fwd_x6(int32_t on);
/* Error word for failures that a kernel can only detect on the device (no host sync inside a call):
 * a persistent bi-LSTM launch whose inter-workgroup barrier times out (a workgroup was not
 * co-resident) ORs 1 (forward) / 2 (BPTT) into *dev_word and fills its outputs with NaN; a D-split
 * attention group barrier (dasa_softdot_*, dasa_shift_attn_*) ORs 4. The host reads the word at its
 * own sync points. NULL disables the report (the NaN poisoning stays). Host-only setting.
 * dasa_persist_force_timeout(1) is a test hook: every such barrier times out. */
int dasa_set_error_word(uint32_t* dev_word);
int dasa_persist_force_timeout(int32_t on);
/* Diagnostic: buf (device, >= 8 * L uint64 words) != NULL makes workgroup 0 of every persistent bi-LSTM
 * forward launch record s_memtime clocks per timestep s at buf[8s + i] (i = 0 step start, 1 after the
 * recurrent MFMAs, 2 after the partial-sum exchange, 3 after the cell update, 4 after the barrier);
 * NULL turns it off. Host-only setting, not used by the product path. */
int dasa_persist_stamps(uint64_t* buf);
int dasa_bilstm_hprev(const float* out, float* hprev, int32_t B, int32_t L, int32_t H, void* stream);

/* ---- AdaIN mu/sigma (model.py:1822-1840, adaIn_type default) ---------------------------------
 * out = (c - mean_c)/std_c * std_s + mean_s per row of N channels (unbiased var + eps, sqrt). */
int dasa_adain_musigma_fwd(const float* content, int64_t ldc_, const float* style, int64_t lds,
                           float* out, int64_t ldo, float* stats, int32_t M, int32_t N, float eps,
                           void* stream);
/* Backward of the above (autograd of model.py:1822-1840): dout -> dcontent, dstyle (either may be
 * NULL); the row statistics are recomputed from content / style. */
int dasa_adain_musigma_bwd(const float* content, int64_t ldc_, const float* style, int64_t lds,
                           const float* dout, int64_t ldg, float* dcontent, int64_t lddc, float* dstyle,
                           int64_t ldds, int32_t M, int32_t N, float eps, void* stream);

/* ---- training-path elementwise ------------------------------------------------------------------
 * DGAdaChannel with saved gate (agent_dg.py:1537-1547): out = s*f*noise[c]; backward gives the grad
 * of the a_fc pre-activation dz = dout*f*noise*s*(1-s). noise may be NULL.                        */
int dasa_ada_gate_fwd(const float* s, int64_t lds, const float* f, int64_t ldf, const float* noise,
                      float* out, int64_t ldo, int32_t rows, int32_t cols, void* stream);
int dasa_ada_gate_bwd(const float* dout, int64_t lddo, const float* s, int64_t lds, const float* f,
                      int64_t ldf, const float* noise, float* dz, int64_t ldz, int32_t rows, int32_t cols,
                      void* stream);
int dasa_act_fwd(const float* x, float* y, int64_t n, int32_t act, void* stream);
/* dx = dy * act'(.) from the activation output (relu/tanh/sigmoid) or input (gelu); n elements. */
int dasa_act_bwd(const float* y_or_x, const float* dy, float* dx, int64_t n, int32_t act, void* stream);
int dasa_add2d(const float* a, int64_t lda, const float* b, int64_t ldb, float* out, int64_t ldo,
               int32_t rows, int32_t cols, void* stream);
int dasa_copy2d(const float* x, int64_t ldx, float* out, int64_t ldo, int32_t rows, int32_t cols,
                void* stream);
/* out = x * scale[col] (shared env-drop noise on the RGB columns, agent_dg.py:731-736, 780-785). */
int dasa_colscale(const float* x, int64_t ldx, const float* scale, float* out, int64_t ldo, int32_t rows,
                  int32_t cols, void* stream);

/* ---- observation pipeline (agent_dg.py:286-323, env.py:317-360 on a device-resident store) -----
 * out[r] = [ta[ia[r]] (Fa floats; zeros if ia[r] < 0) | tb[ib[r]] (Fb floats; zeros if ib == NULL or
 * ib[r] < 0)]: panorama blocks [B][36][2048+128] and candidate blocks [B][C][2176] in one gather.  */
/* Up to DASA_COPY_MAX_SEGS strided block copies in ONE launch (no reference counterpart: the static-buffer
   traffic around replayed hipGraphs, dasa_amd/graph.py). Segments must not overlap each other's
   destinations or alias their own source; n == 0 is a no-op. */
int dasa_copy_segments(const dasa_copy_seg* segs, int32_t n, void* stream);
int dasa_gather_rows(const float* ta, const int32_t* ia, int32_t Fa, const float* tb, const int32_t* ib,
                     int32_t Fb, float* out, int32_t R, void* stream);

/* ---- small helpers --------------------------------------------------------------------------- */
/* Reverse the first lengths[b] rows of x [B][L][H] into out (rest zero), r2rmodel.py:2326-2330. */
int dasa_reverse_valid(const float* x, const int32_t* lengths, float* out, int32_t B, int32_t L,
                       int32_t H, void* stream);
/* ---- policy head (agent_dg.py:832-886) ------------------------------------------------------- */
enum dasa_policy_mode { DASA_POLICY_TEACHER = 0, DASA_POLICY_ARGMAX = 1, DASA_POLICY_SAMPLE = 2,
                        DASA_POLICY_FORCED = 3, DASA_POLICY_SAMPLE_ARGMAX = 4 };
/* One decision step's loss/action stage on logit [B][C] (row stride ld): candidates c >= cand_len[b]
 * are masked (-inf); logp [B][C] = masked log-softmax (saved for backward); ce_sum[0] = sum over rows
 * with target != ignore_index of -logp[target] (CrossEntropyLoss(reduction='sum')); mode ARGMAX:
 * action = first argmax; mode SAMPLE: action ~ Categorical(softmax) by inverse CDF on the counter RNG
 * (seed, row); ent [B] = entropy, logp_a [B] = logp[action] (each optional). target may be NULL (no
 * CE, ce_sum = 0). C <= 256. ws: B floats of scratch. One launch, deterministic.
 * Mode FORCED is mode SAMPLE with the draw replaced by the caller's action[b] (an INPUT, 0 <= action[b]
 * < cand_len[b]): entropy and logp_a as in SAMPLE. It pins the sampled rollout's loss stage against a
 * reference run whose Categorical.sample returns the same actions (tests/test_policy_gpu.py).
 * Mode SAMPLE_ARGMAX is mode SAMPLE with the draw replaced by the first argmax (a reference run whose
 * Categorical.sample is replaced by probs.argmax: the golden fixtures' sampled rollouts). */
int dasa_policy_head_fwd(const float* logit, int64_t ld, const int32_t* cand_len, const int64_t* target,
                         int32_t B, int32_t C, int32_t mode, int32_t ignore_index, uint64_t seed,
                         float* logp, float* ce_sum, float* ent, float* logp_a, int64_t* action,
                         float* ws, void* stream);
/* In modes SAMPLE / FORCED, ent and logp_a follow torch.distributions.Categorical(probs): the log-pmf
 * is l = log(clamp(p, FLT_EPSILON, 1 - FLT_EPSILON)), ent = -sum p l, logp_a = l[action]; in mode
 * ARGMAX logp_a is the exact log-softmax (F.log_softmax(...).gather).
 * Backward, `mode` as in the forward: dlogit[b][c] (row stride ldd) = d_ce * (p - onehot(target))
 *   + d_logp_a[b] * u_a * (onehot(action) - p) + d_ent[b] * p_c * (g_c - sum_j p_j g_j),
 *   g = -(l + u), u = 1 where the clamp is inactive (always in ARGMAX / TEACHER), over unmasked c, 0
 *   where masked; each d_* may be NULL. */
int dasa_policy_head_bwd(const float* logp, const int32_t* cand_len, const int64_t* target,
                         const int64_t* action, const float* ent, const float* d_ce,
                         const float* d_logp_a, const float* d_ent, float* dlogit, int64_t ldd,
                         int32_t B, int32_t C, int32_t mode, int32_t ignore_index, void* stream);

/* Device seed source for hipGraph capture. While a counter is set (dev_counter != NULL), every
 * forward dropout launch (layernorm, embeddings, attention probabilities, dropout) records it, and
 * its mask seed becomes seed ^ mix(*dev_counter) read at run time: a captured graph that starts with
 * dasa_seed_bump(dev_counter) draws fresh masks on every replay; the Categorical draw of the policy
 * head (mode SAMPLE) is keyed the same way. Backward dropout kernels (dropout, layernorm, attention
 * probabilities) launched while the same counter is set regenerate the replay's masks: a captured
 * TRAINING step runs its eager backward with its counter set (dasa_amd/graph.py AutogradGraphs).
 * Host-only setting, not thread-safe. */
int dasa_set_seed_source(const uint64_t* dev_counter);
int dasa_seed_bump(uint64_t* dev_counter, void* stream);

/* y[i] = x[i] * keep(seed, i) / (1-p) for a [rows][cols] block with row stride ld (in place ok). */
int dasa_dropout_fwd(const float* x, int64_t ldx, float* y, int64_t ldy, int32_t rows, int32_t cols,
                     float p, uint64_t seed, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DASA_HIP_H */
