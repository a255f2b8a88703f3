/*
 * recblr_hip.h — C-ABI of the MI355X (gfx950) RecBLR sequence-encoder kernels.
 *
 * This is the drop-in boundary beneath the Python mirror of the reference API
 * (datamining_recblr_amd.parallel_scan / GatedRecurrentLayer).  Every entry
 * point takes raw device pointers, int64 sizes/row strides and a hipStream_t
 * passed as void*.  Nothing here allocates, synchronises or keeps mutable
 * global state, so every call is capturable into a hipGraph and reentrant per
 * stream.  All tensors are fp32.
 *
 * Return value: 0 on success; RB_EINVAL (-1) for a bad argument (shape,
 * stride, alignment, null pointer); a positive hipError_t when the launch
 * failed.  rb_last_error_string() describes the last failure of the calling
 * thread.
 *
 * Reference interfaces replaced (paths relative to the reference repo root):
 *   rb_scan_fwd        parallel_scan.py:44-60  (forward_scan Triton kernel)
 *                      + parallel_scan.py:84-95 (Scan.forward)
 *   rb_scan_bwd        parallel_scan.py:63-80  (backward_scan Triton kernel)
 *                      + parallel_scan.py:97-114 (Scan.backward glue: shifted
 *                      gates, reverse scan, d_gates = h_{t-1} * d_t)
 *   rb_conv_silu_fwd   RecBLR.py:182-193 (causal depthwise conv1d + SiLU on
 *                      the left-padded sequence; causal_conv1d_fn or the
 *                      F.conv1d fallback at :185)
 *   rb_conv_silu_bwd   autograd of RecBLR.py:185 (dx, dW, dbias)
 *   rb_gate_scan_fwd   RecBLR.py:196-206 minus the GEMMs: alpha/beta gates
 *                      (:197-199), parallel_scan (:200), truncation (:203-204)
 *                      and the silu(z)*h merge (:206)
 *   rb_gate_scan_bwd   autograd of the same span (Scan.backward + gate math)
 *
 * Layout (channel-last, "rows" = (batch, time) pairs):
 *   element (b, t, c) of a [B, L, *] activation lives at
 *   ptr[(b * L + t) * row_stride + c]; row_stride >= H.
 *
 * Packed variable-length sequences (seq_offsets != NULL; the conv and gate
 * scan entry points): seq_offsets is a device int64 array [B + 1]; sequence b
 * occupies rows seq_offsets[b] .. seq_offsets[b+1] - 1 (length in [0, L]), so
 * element (b, t, c) lives at ptr[(seq_offsets[b] + t) * row_stride + c]; L is
 * the maximum length (it sizes the carry checkpoint [B, ceil(L/RB_TILE), H]
 * and the grid).  This is RecBole's right-padded batch without its padding:
 * the recurrence is causal, so positions past a sequence's length never reach
 * RecBLR.forward's output (gather_indexes at len - 1, RecBLR.py:84).
 * seq_offsets = NULL: the dense layout above.
 */
#ifndef RECBLR_HIP_H
#define RECBLR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RB_EINVAL (-1)

/* bf16 activation storage (raw bits); kernels compute in fp32. */
typedef uint16_t rb_bf16;

/* Time-tile length of the fused gate/scan kernels: rb_gate_scan_fwd writes one
 * carry (the recurrent state entering the tile) per (b, tile, c) and
 * rb_gate_scan_bwd reads them back.  carries has B * ceil(L / RB_TILE) * H
 * floats. */
#define RB_TILE 16

/* ABI version; bumped on any signature change. */
int rb_version(void);

/* Human-readable description of the last error on the calling thread. */
const char* rb_last_error_string(void);

/* Number of device kernels compiled into the library for gfx950 (sanity). */
int rb_num_kernels(void);

/* parallel_scan forward on the reference layout [B, C, T], T contiguous:
 *   states[b,c,t] = gates[b,c,t] * states[b,c,t-1] + tokens[b,c,t],
 *   states[b,c,-1] = 0.
 * Any T >= 1 (the reference needs a power of two; this does not). */
int rb_scan_fwd(const float* gates, const float* tokens, float* states,
                int64_t B, int64_t C, int64_t T, void* stream);

/* parallel_scan backward (parallel_scan.py:97-114):
 *   d[t]       = grad[t] + gates[t+1] * d[t+1],  d[T] = 0
 *   d_gates[t] = states[t-1] * d[t]  (states[-1] = 0)
 *   d_tokens   = d                                              */
int rb_scan_bwd(const float* gates, const float* states, const float* grad,
                float* d_gates, float* d_tokens,
                int64_t B, int64_t C, int64_t T, void* stream);

/* Causal depthwise conv (kernel K, zero history) + bias + SiLU:
 *   xc[b,t,c] = silu(bias[c] + sum_k w[c,k] * x[b, t-K+1+k, c])
 * x: [B, L, H] view with row stride x_rs (e.g. the first half of the
 * in-projection output [B, L, 2H]); w: [H, K] contiguous; xc: [B, L, H]
 * with row stride xc_rs.  1 <= K <= 8. */
int rb_conv_silu_fwd(const float* x, int64_t x_rs, const float* w,
                     const float* bias, float* xc, int64_t xc_rs,
                     int64_t B, int64_t L, int64_t H, int64_t K, const int64_t* seq_offsets, void* stream);

/* rb_conv_silu_fwd on packed sequences, tiled over the packed rows
 * [0, ntok) instead of per sequence (no work past a sequence's end):
 * row_pos is a device int64 array [ntok], row_pos[r] = position of row r
 * inside its sequence (r - seq_offsets[b] for the sequence b holding r); the
 * tap at lag l reaches row r only when l <= row_pos[r] (zero history).  Same
 * values as rb_conv_silu_fwd with the matching seq_offsets.  Replaces
 * RecBLR.py:182-193 like rb_conv_silu_fwd. */
int rb_conv_silu_fwd_rows(const float* x, int64_t x_rs, const float* w, const float* bias,
                          float* xc, int64_t xc_rs, int64_t ntok, int64_t H, int64_t K,
                          const int64_t* row_pos, void* stream);

/* Backward of rb_conv_silu_fwd.  dxc = g1 + g2 (g2 may be NULL), both
 * [B, L, H] contiguous.  Writes dx (row stride dx_rs) and per-batch partial
 * sums dw_part[b, k, c] (B*K*H floats) and db_part[b, c] (B*H floats); the
 * caller sums the partials over b (deterministic, no atomics).  db_part NULL
 * selects the folded layout: dw_part holds B rows of (K+1)*H floats, dW[c, k]
 * at c*K + k then dbias[c] at K*H + c, so one column sum over the rows gives
 * both gradients in parameter layout. */
int rb_conv_silu_bwd(const float* x, int64_t x_rs, const float* w,
                     const float* bias, const float* g1, const float* g2,
                     float* dx, int64_t dx_rs, float* dw_part, float* db_part,
                     int64_t B, int64_t L, int64_t H, int64_t K, const int64_t* seq_offsets, void* stream);

/* Fused BD-LRU forward (everything between the gates GEMM and the output
 * GEMM):
 *   alpha = exp(-softplus(lam[c]) * sigmoid(r)),
 *   beta  = sqrt(1 - alpha^2 + 1e-8) * sigmoid(i),
 *   h_t   = alpha_t * h_{t-1} + beta_t * xc_t,   h_{-1} = h0[c] (0 if NULL),
 *   y     = silu(z) * h.
 * rg: [B, L, 2H] view (r = columns [0,H), i = columns [H,2H)), row stride
 * rg_rs, to which gate_b [2H] is added when non-NULL (the gates bias, folded
 * here rather than into the GEMM; drg is the gradient w.r.t. rg + gate_b); xc, z, y: [B, L, H] views with their own row strides; lam, h0: [H].
 * carries: B * ceil(L/RB_TILE) * H floats (written, consumed by the bwd);
 * may be NULL for inference (no checkpoints written). */
int rb_gate_scan_fwd(const float* rg, int64_t rg_rs, const float* xc,
                     int64_t xc_rs, const float* z, int64_t z_rs,
                     const float* lam, const float* gate_b, const float* h0,
                     int64_t h0_bs, float* y, int64_t y_rs, float* carries,
                     int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets, void* stream);

/* Backward of rb_gate_scan_fwd given dy = dL/dy ([B, L, H] contiguous).
 * Writes drg ([B, L, 2H] view: dr | di, row stride drg_rs), dxc (the gate
 * path's share of dL/dxc, row stride dxc_rs), dz (row stride dz_rs),
 * part[3, B, H] = per-batch sums over t of {dlam, dr, di} and
 * dh0_part[B, H] = dL/dh_{-1} per batch row (caller sums over b). */
int rb_gate_scan_bwd(const float* rg, int64_t rg_rs, const float* xc,
                     int64_t xc_rs, const float* z, int64_t z_rs,
                     const float* lam, const float* gate_b, const float* carries,
                     const float* dy,
                     float* drg, int64_t drg_rs, float* dxc, int64_t dxc_rs,
                     float* dz, int64_t dz_rs, float* part, float* dh0_part,
                     int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets, void* stream);

/* rb_gate_scan_fwd / _bwd when only each sequence's LAST position of y is
 * used downstream (RecBLR.forward's gather_indexes(seq_output, len - 1),
 * RecBLR.py:84, on the last layer): the forward writes y_last [B, H]
 * contiguous (row b = y at position L-1, or at seq_offsets[b+1]-1 packed)
 * instead of y; the backward takes dy_last [B, H] with dy = 0 at every other
 * position (no [B, L, H] dy is materialised or read).  fp32.
 * batch_row (int64 [B], a permutation of 0..B-1, or NULL): sequence b's row
 * of y_last / dy_last is batch_row[b] instead of b — packed sequences run
 * longest first, so the last layer's output lands in batch order without a
 * gather (and its gradient is read without a scatter). */
int rb_gate_scan_fwd_last(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                          const float* z, int64_t z_rs, const float* lam, const float* gate_b,
                          const float* h0, int64_t h0_bs, float* y_last, float* carries,
                          int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets,
                          const int64_t* batch_row, void* stream);
int rb_gate_scan_bwd_last(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                          const float* z, int64_t z_rs, const float* lam, const float* gate_b,
                          const float* carries, const float* dy_last, float* drg,
                          int64_t drg_rs, float* dxc, int64_t dxc_rs, float* dz, int64_t dz_rs,
                          float* part, float* dh0_part, int64_t B, int64_t L, int64_t H,
                          const int64_t* seq_offsets, const int64_t* batch_row, void* stream);

/* The state the power-of-two left padding leaves in the recurrence
 * (RecBLR.py:176-179: F.pad of x by P zero steps before conv + scan), without
 * materialising the padding.  Pad steps see the per-channel constants
 * xc_p = silu(conv_b), (r_p, i_p) = gate_w xc_p + gate_b,
 * s = softplus(lam) sigmoid(r_p), alpha = exp(-s),
 * b_p = sqrt(1 - alpha^2 + 1e-8) sigmoid(i_p) xc_p, so after P steps
 *   h0 = b_p expm1(-P s) / expm1(-s)            (s clamped at 1e-20).
 * gate_w: [2H, H] row-major; h0: [n_rows, H]; row b uses pad[b] (pad != NULL)
 * or pad_len.  Feeds rb_gate_scan_fwd's h0 (h0_bs = 0 for one row, H for
 * per-row pad lengths).  workspace: 5H floats of scratch; H <= 4096. */
int rb_pad_prefix_fwd(const float* conv_b, const float* gate_w, const float* gate_b,
                      const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                      int64_t H, float* h0, float* workspace, void* stream);

/* Backward of rb_pad_prefix_fwd for dh0 [n_rows, H] (rows summed in order):
 * dconv_b [H], dgate_w [2H, H], dgate_b [2H], dlam [H] are overwritten
 * (accumulate = 0) or have this contribution added to what they hold
 * (accumulate = 1: the other gradient contributions of the same parameters,
 * so no separate add launches). */
int rb_pad_prefix_bwd(const float* conv_b, const float* gate_w, const float* gate_b,
                      const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                      int64_t H, const float* dh0, float* dconv_b, float* dgate_w,
                      float* dgate_b, float* dlam, float* workspace, int accumulate,
                      void* stream);

/* ---- blocks around the BD-LRU (RecurrentLayer / FeedForward / embedding) ---- */

/* Dropout in the row kernels (nn.Dropout(p), train mode): element e is kept
 * with probability 1-p and scaled by 1/(1-p).  The keep flags come from
 * `mask` (uint8 {0,1}, laid out like the data) when it is non-NULL, otherwise
 * from a Philox4x32-10 stream keyed by `seed` with counter e/4 — regenerated
 * bit-identically by the backward.  p = 0 and mask = NULL: no dropout.
 * Row widths (d, cols) must be one of 16, 32, 64, 128, 256, 512, 1024. */

/* Fused dropout + residual + LayerNorm over rows of d floats
 * (RecBLR.py:77-78 and :142, and FeedForward's :223-225):
 *   A[row] = idx ? a[clamp(idx[row], 0, n_idx_rows-1)] : a[row]   (gather)
 *   s      = dropout(A[row]) + (r ? r[row] : 0)
 *   y      = (s - mean) / sqrt(var + eps) * gamma + beta
 * s_out, mean, rstd (saved for the backward) are all given or all NULL. */
int rb_add_ln_fwd(const float* a, const int64_t* idx, int64_t n_idx_rows,
                  const uint8_t* mask, uint64_t seed, float p, const float* r,
                  const float* gamma, const float* beta, float eps, float* y,
                  float* s_out, float* mean, float* rstd, int64_t rows,
                  int64_t d, void* stream);

/* Rows of the per-block column partial-sum buffers the row backward kernels
 * write ([n_parts, width]; the caller sums them over n_parts). */
int64_t rb_row_num_parts(int64_t rows, int64_t width);

/* Backward of rb_add_ln_fwd: ds = dL/ds (the residual's gradient),
 * da = dropout-backward(ds) (the dropped input's gradient) and dbias_part =
 * column partials of da (the bias gradient of the GEMM that produced a);
 * any of the three may be NULL.  dgamma_part / dbeta_part: [n_parts, d]. */
int rb_add_ln_bwd(const float* dy, const float* s, const float* gamma,
                  const float* mean, const float* rstd, const uint8_t* mask,
                  uint64_t seed, float p, float* ds, float* da,
                  float* dgamma_part, float* dbeta_part, float* dbias_part,
                  int64_t n_parts, int64_t rows, int64_t d, void* stream);
/* rb_add_ln_bwd with the output's gradient given as two terms, dy + dy2
 * (dy2 may be NULL): autograd's sum of the gradients of a LayerNorm output
 * read by two consumers (the next projection's input gradient and a
 * residual branch), added while loading instead of in a separate pass. */
int rb_add_ln_bwd2(const float* dy, const float* dy2, const float* s, const float* gamma,
                   const float* mean, const float* rstd, const uint8_t* mask,
                   uint64_t seed, float p, float* ds, float* da,
                   float* dgamma_part, float* dbeta_part, float* dbias_part,
                   int64_t n_parts, int64_t rows, int64_t d, void* stream);

/* FeedForward's inner activation (RecBLR.py:220-221) on [rows, cols]:
 * u = dropout(silu(a + bias)) (bias [cols] may be NULL: the w_1 bias folded
 * in here instead of into the GEMM); backward
 * da = dropout-backward(du) * silu'(a + bias) with optional column partials
 * of da (the w_1 bias gradient). */
int rb_silu_dropout_fwd(const float* a, const float* bias, const uint8_t* mask,
                        uint64_t seed, float p, float* u, int64_t rows,
                        int64_t cols, void* stream);
int rb_silu_dropout_bwd(const float* a, const float* bias, const uint8_t* mask,
                        uint64_t seed, float p, const float* du, float* da,
                        float* dbias_part, int64_t n_parts, int64_t rows,
                        int64_t cols, void* stream);

/* Materialise the keep-mask of a Philox dropout stream (n % 4 == 0). */
int rb_dropout_mask(uint64_t seed, float p, uint8_t* out, int64_t n,
                    void* stream);

/* Item-embedding backward (RecBLR.py:76, nn.Embedding(padding_idx=0)):
 * dweight[v] = sum_{p : idx[p] == v} grad[p], dweight[padding_idx] = 0,
 * deterministic (stable sort + fixed-order segment sums, no atomics).
 * Ids outside [0, V) are ignored.  workspace: rb_embedding_bwd_workspace()
 * bytes, caller-allocated. */
int64_t rb_embedding_bwd_workspace(int64_t M, int64_t V, int64_t d);
int rb_embedding_bwd(const int64_t* idx, const float* grad, int64_t M, int64_t d,
                     int64_t V, int64_t padding_idx, float* dweight,
                     void* workspace, int64_t workspace_bytes, void* stream);

/* rb_embedding_bwd in two halves: the plan (stable sort of the ids, segment
 * and chunk offsets; depends on idx only, so it can run during the forward on
 * another stream) and the apply (fixed-order segment sums of grad).  Same
 * workspace, untouched between the two calls. */
int rb_embedding_bwd_plan(const int64_t* idx, int64_t M, int64_t d, int64_t V,
                          void* workspace, int64_t workspace_bytes, void* stream);
int rb_embedding_bwd_apply(const float* grad, int64_t M, int64_t d, int64_t V,
                           int64_t padding_idx, float* dweight, void* workspace,
                           int64_t workspace_bytes, void* stream);

/* Fixed-order column sums of partials: out[m*C + c] = sum over p < P of
 * in[m*ms + p*rs + c] for m < M, summed as RG interleaved partials
 * (p = g, g+RG, ... in increasing order; RG = 4 for P <= 256, else 16)
 * combined in order g = 0..RG-1.  Turns the per-block / per-split partials
 * the backward kernels write (no atomics) into gradients; deterministic. */
int rb_colsum(const float* in, int64_t M, int64_t P, int64_t C, int64_t rs, int64_t ms,
              float* out, void* stream);

/* rb_colsum for few columns and many rows in one launch: the rows of each of
 * the M matrices (contiguous: matrix m starts at in + m*P*rs) are summed in
 * chunks of `chunk_rows` (64, 128 or 256; P % chunk_rows == 0), each chunk
 * as rb_colsum(P = chunk_rows) does, then the chunk sums as
 * rb_colsum(P = P / chunk_rows) does — bitwise the two-launch result.  part:
 * [M, P / chunk_rows, C] fp32 workspace; counters: M * ceil(C / 64) uint32
 * tickets, zero on the first call and left zero by every call (the last
 * workgroup of a column block resets its ticket); calls sharing counters must
 * be ordered on one stream. */
int rb_colsum_chunked(const float* in, int64_t M, int64_t P, int64_t C, int64_t rs,
                      int64_t chunk_rows, float* part, uint32_t* counters, int64_t n_counters,
                      float* out, void* stream);

/* ---- item scoring (RecBLR.py:86-122), fp32 MFMA, no [B, V] logits ----
 * seq: [B, d] sequence representations (RecBLR.forward's output), items:
 * [V, d] item table (item_embedding.weight), both contiguous and 16-B
 * aligned; target: [B] int64 item ids.  d must be 16, 32, 64, 128 or 256.
 * Deterministic (per-split partials summed in a fixed order). */

/* Workspace bytes of rb_item_ce_fwd / rb_item_ce_bwd (one size serves both). */
int64_t rb_item_ce_workspace(int64_t B, int64_t V, int64_t d);

/* Softmax cross-entropy over all V items, mean over the batch
 * (RecBLR.py:100-102: logits = seq @ items^T; nn.CrossEntropyLoss()):
 *   lse[b] = log sum_v exp(seq[b] . items[v]),
 *   loss[0] = mean_b (lse[b] - seq[b] . items[target[b]]).
 * An out-of-range target makes loss NaN. */
int rb_item_ce_fwd(const float* seq, const float* items, const int64_t* target, int64_t B,
                   int64_t V, int64_t d, float* lse, float* loss, void* workspace,
                   int64_t workspace_bytes, void* stream);

/* Backward of rb_item_ce_fwd for the upstream gradient dloss[0] (a device
 * scalar): with P[b][v] = (softmax_v(seq[b] . items) - [v == target[b]]) *
 * dloss / B, dseq = P items and ditems = P^T seq.  The logits are recomputed
 * tile by tile; either output may be NULL. */
int rb_item_ce_bwd(const float* seq, const float* items, const int64_t* target, const float* lse,
                   const float* dloss, int64_t B, int64_t V, int64_t d, float* dseq,
                   float* ditems, void* workspace, int64_t workspace_bytes, void* stream);

/* The logits' gradient of rb_item_ce_fwd for a slice of the item table:
 * items points at rows [item_offset, item_offset + V) of the table,
 *   probs[b][v] = (softmax(seq[b] . table)[item_offset + v]
 *                  - [item_offset + v == target[b]]) * dloss / B
 * written with row stride ld >= V (lse from rb_item_ce_fwd).  With it the
 * backward is two GEMMs, dseq += probs items and ditems = probs^T seq, at
 * library speed; the slice bounds the [B, V] buffer for large tables.  The
 * fully fused rb_item_ce_bwd needs no such buffer. */
int rb_item_ce_probs(const float* seq, const float* items, const int64_t* target,
                     const float* lse, const float* dloss, int64_t B, int64_t V, int64_t d,
                     int64_t item_offset, float* probs, int64_t ld, void* stream);

/* ---- the same CE on the f16 MFMA pipe (the training step's default) ----
 * fp32-level accuracy from two-part split operands: each row x of seq and of
 * the item table is scaled by 2^(14 - e) (e = frexp exponent of max|x|) and
 * split into x0 = f16(x'), x1 = f16(x' - x0); a score is x0.y0 + x0.y1 + x1.y0
 * in fp32 on v_mfma_f32_32x32x16_f16, un-scaled exactly.
 * rb_item_split_h: x [n, d] fp32 (16-B aligned) -> image [n, 2d] fp16
 * (row: d halfs x0 | d halfs x1, 16-B aligned) and exps [n] int32;
 * group_max (float [ceil(n/32)], or NULL): max |x| over each 32-row group —
 * rb_group_absmax's output, for the weight-gradient GEMM on the same x. */
int rb_item_split_h(const float* x, int64_t n, int64_t d, void* image, int* exps,
                    float* group_max, void* stream);

/* rb_item_ce_fwd on split images (workspace: rb_item_ce_workspace). */
int rb_item_ce_fwd_h(const void* seq_img, const int* seq_exp, const void* item_img,
                     const int* item_exp, const int64_t* target, int64_t B, int64_t V, int64_t d,
                     float* lse, float* loss, void* workspace, int64_t workspace_bytes,
                     void* stream);

/* rb_item_ce_probs on split images: item_img / item_exp point at image rows
 * [item_offset, item_offset + V); lse from rb_item_ce_fwd_h on the same
 * images (bit-identical logits in both kernels). */
int rb_item_ce_probs_h(const void* seq_img, const int* seq_exp, const void* item_img,
                       const int* item_exp, const int64_t* target, const float* lse,
                       const float* dloss, int64_t B, int64_t V, int64_t d, int64_t item_offset,
                       float* probs, int64_t ld, void* stream);

/* rb_item_ce_probs_h transposed: probs_t [V, ldt] = P^T (ldt >= B, a
 * multiple of 4, 16-B aligned) and group_max [ceil(V/32)] = max |P| over
 * each 32-item group (atomic max: zeroed by the caller) — the operands of
 * dL/dseq = P W and dL/ditems = P^T seq (RecBLR.py:100-102's backward) as
 * the f16x3 weight-gradient / NT GEMMs (rb_gemm_tn_h, rb_gemm_nt_h). */
int rb_item_ce_probs_h_t(const void* seq_img, const int* seq_exp, const void* item_img,
                         const int* item_exp, const int64_t* target, const float* lse,
                         const float* dloss, int64_t B, int64_t V, int64_t d, int64_t item_offset,
                         float* probs_t, int64_t ldt, float* group_max, void* stream);

/* Both layouts in one pass: probs [B, ld] = P (as rb_item_ce_probs_h) and
 * probs_t [V, ldt] = P^T with item_group_max (as rb_item_ce_probs_h_t), plus
 * row_group_max [ceil(B/32)] = max |P| over each 32-row group (atomic max:
 * both maxima zeroed by the caller).  dL/ditems = P^T seq then runs as the
 * weight-gradient GEMM over P's rows and dL/dseq = P W over P^T's rows
 * (rb_gemm_tn_h, RecBLR.py:100-102's backward) with no library GEMM. */
int rb_item_ce_probs_h_both(const void* seq_img, const int* seq_exp, const void* item_img,
                            const int* item_exp, const int64_t* target, const float* lse,
                            const float* dloss, int64_t B, int64_t V, int64_t d,
                            int64_t item_offset, float* probs, int64_t ld, float* probs_t,
                            int64_t ldt, float* row_group_max, float* item_group_max,
                            void* stream);

/* out [ceil(n/32)] = max |x| over each 32-row group of x [n, c] (row stride
 * ld): rb_gemm_tn_h's operand scales for a tensor no f16 GEMM has read. */
int rb_group_absmax(const float* x, int64_t n, int64_t c, int64_t ld, float* out, void* stream);

/* Workspace bytes of rb_item_rank. */
int64_t rb_item_rank_workspace(int64_t B, int64_t V, int64_t d);

/* Full-sort ranking of each row's target (the full_sort_predict evaluation,
 * RecBLR.py:114-122 with RecBole's scores[:, 0] = -inf, and
 * run_with_unseen.py:229-265): over items v in [first_item, V), v != target,
 *   n_greater[b] = #{score(b, v) > score(b, target)},
 *   n_equal[b]   = #{score(b, v) == score(b, target)}   (n_equal may be NULL).
 * Hit@k = n_greater < k; NDCG@k and MRR follow from the rank.  The target's
 * score is bit-identical to the tile's score for it.  -1 for an out-of-range
 * target. */
int rb_item_rank(const float* seq, const float* items, const int64_t* target, int64_t B,
                 int64_t V, int64_t d, int64_t first_item, int64_t* n_greater, int64_t* n_equal,
                 void* workspace, int64_t workspace_bytes, void* stream);

/* scores[b][v] = seq[b] . items[v] (full_sort_predict, RecBLR.py:114-122), same
 * fma chain as the kernels above; scores [B, V] contiguous. */
int rb_item_scores(const float* seq, const float* items, int64_t B, int64_t V, int64_t d,
                   float* scores, void* stream);

/* ---- bf16 storage variants (BASELINE config 5: L = 2048, d = 256, bf16) ----
 * Same semantics, arguments and checks as the fp32 entry points above, with
 * the [B, L, *] / [B, C, T] activations stored as bf16 (loaded to fp32,
 * every recurrence, gate and accumulation in fp32 registers, the outputs
 * rounded to bf16 once, RNE); per-channel parameters (w, bias, lam, gate_b),
 * the carry checkpoint, h0 and all partial sums stay fp32.  alpha is never
 * stored (alpha ~ 0.9995 would round to 1 in bf16: SURVEY §7).  The reference
 * has no bf16 scan (parallel_scan.py:19,27-28 are fp32-only); these replace
 * the same interfaces as their fp32 forms. */
int rb_scan_fwd_bf16(const rb_bf16* gates, const rb_bf16* tokens, rb_bf16* states, int64_t B,
                     int64_t C, int64_t T, void* stream);
int rb_scan_bwd_bf16(const rb_bf16* gates, const rb_bf16* states, const rb_bf16* grad,
                     rb_bf16* d_gates, rb_bf16* d_tokens, int64_t B, int64_t C, int64_t T,
                     void* stream);
int rb_conv_silu_fwd_bf16(const rb_bf16* x, int64_t x_rs, const float* w, const float* bias,
                          rb_bf16* xc, int64_t xc_rs, int64_t B, int64_t L, int64_t H, int64_t K,
                          const int64_t* seq_offsets, void* stream);
int rb_conv_silu_fwd_rows_bf16(const rb_bf16* x, int64_t x_rs, const float* w, const float* bias,
                               rb_bf16* xc, int64_t xc_rs, int64_t ntok, int64_t H, int64_t K,
                               const int64_t* row_pos, void* stream);
int rb_conv_silu_bwd_bf16(const rb_bf16* x, int64_t x_rs, const float* w, const float* bias,
                          const rb_bf16* g1, const rb_bf16* g2, rb_bf16* dx, int64_t dx_rs,
                          float* dw_part, float* db_part, int64_t B, int64_t L, int64_t H,
                          int64_t K, const int64_t* seq_offsets, void* stream);
int rb_gate_scan_fwd_bf16(const rb_bf16* rg, int64_t rg_rs, const rb_bf16* xc, int64_t xc_rs,
                          const rb_bf16* z, int64_t z_rs, const float* lam, const float* gate_b,
                          const float* h0, int64_t h0_bs, rb_bf16* y, int64_t y_rs,
                          float* carries, int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets, void* stream);
int rb_gate_scan_bwd_bf16(const rb_bf16* rg, int64_t rg_rs, const rb_bf16* xc, int64_t xc_rs,
                          const rb_bf16* z, int64_t z_rs, const float* lam, const float* gate_b,
                          const float* carries, const rb_bf16* dy, rb_bf16* drg, int64_t drg_rs,
                          rb_bf16* dxc, int64_t dxc_rs, rb_bf16* dz, int64_t dz_rs, float* part,
                          float* dh0_part, int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets, void* stream);

/* Packed-sequence plan (RecBLR.forward on RecBole's right-padded batch,
 * RecBLR.py:75, run on each sequence's first len_b positions only): item_seq
 * [B, L] int64 (row stride seq_rs), seq_offsets [B+1] and order [B] (packed
 * sequence s is batch row order[s], rows seq_offsets[s] .. seq_offsets[s+1])
 * -> ids[r] = item_seq[order[s], t] and row_pos[r] = t for r =
 * seq_offsets[s] + t (ntok = seq_offsets[B] entries each), inv[order[s]] = s,
 * last[order[s]] = seq_offsets[s+1] - 1.  All device int64. */
int rb_pack_plan(const int64_t* item_seq, int64_t seq_rs, const int64_t* seq_offsets,
                 const int64_t* order, int64_t B, int64_t L, int64_t* ids, int64_t* row_pos,
                 int64_t* inv, int64_t* last, void* stream);

/* One Adam step (torch.optim.Adam semantics, L2 weight decay, no amsgrad)
 * over up to RB_MAX_ADAM_JOBS fp32 tensors in one launch — the optimizer of
 * the reference's training loop (run.py: RecBole's Trainer, learner
 * 'adam').  jobs: a HOST array; param / grad / exp_avg / exp_avg_sq of each
 * job are n contiguous floats, 16-B aligned.  bc1 = 1 - beta1^t and bc2 =
 * 1 - beta2^t for the step t being taken (t >= 1).  The scalars are the
 * host's doubles: lr / bc1, 1 - beta and sqrt(bc2) are formed in double and
 * rounded to fp32 once, as torch's Adam does. */
#define RB_MAX_ADAM_JOBS 48
typedef struct {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n;
} rb_adam_job;
int rb_adam_step(const rb_adam_job* jobs, int64_t n, double lr, double beta1, double beta2,
                 double eps, double weight_decay, double bc1, double bc2, void* stream);

/* ---- projection GEMMs (RecBLR.py:162,165,167,213,214: nn.Linear, fp32) ----
 * fp32 GEMMs on the f16 pipe, two-part split (csrc/gemm_half.hip).
 * Every fp32 operand is scaled by an exact power of two and split into two
 * fp16 parts, x = 2^-s (x0 + x1) (22 significant bits); the three products
 * a0b0 + a0b1 + a1b0 accumulate in fp32 (error vs fp64 within a few fp32
 * units, tests/test_gpu_gemm.py).  Weights: one scale per output column;
 * A rows: one scale per row (the weight-stationary kernel: from the row's
 * exact max; the persistent kernel: chosen online).
 *
 * Bytes of the f16 weight image of Bm [C, R]: the persistent kernel's two
 * planes, C exponents, then (R % 32 == 0) the weight-stationary kernel's two
 * planes (csrc/gemm_ws.hip). */
int64_t rb_gemm_h_weight_bytes(int64_t C, int64_t R);

/* Build the f16 weight images of up to RB_MAX_SPLIT_JOBS weights in one
 * launch (jobs: a HOST array of n descriptors; Bm = W (transpose = 0; W [C,
 * R], row stride ldw) or Bm = W^T (transpose = 1; W [R, C]); C % 32 == 0,
 * R % 16 == 0; each Wf 16-B aligned, rb_gemm_h_weight_bytes(C, R) bytes).
 * The host side refreshes every image a training step made stale (the
 * optimizer changed the weights) at once.  Replaces the weight operand of
 * F.linear (forward: Bm = W) and of its input gradient (Bm = W^T). */
#define RB_MAX_SPLIT_JOBS 32
typedef struct {
  const float* W;
  int64_t ldw;
  int64_t C;
  int64_t R;
  int64_t transpose;
  void* Wf;
} rb_split_job;
int rb_gemm_h_split_weights(const rb_split_job* jobs, int64_t n, void* stream);

/* out[m, c] = sum_r A[m, r] Bm[c, r] (+ bias[c] if bias), m < M, c < C, on
 * the f16 image Wf of Bm: F.linear's forward (A = x, Bm = W) and input
 * gradient (A = dy, Bm = W^T).  A row stride lda (multiple of 4, A 16-B
 * aligned), out row stride ldo; R % 32 == 0, C % 32 == 0, C <= 1024;
 * accumulate must be 0.  rmax (optional, [ceil(M/32)] floats): max |A| over each
 * 32-row group, the operand scale of rb_gemm_tn_h on the same rows.  Replaces
 * nn.Linear's forward / input-gradient GEMM (RecBLR.py:162,165,167,213,214).
 * From 16,384 rows with R in {128, 256, 512}, C % 128 == 0, A and out 16-B
 * aligned and lda, ldo multiples of 4: the weight-stationary kernel
 * (csrc/gemm_ws.hip; rb_gemm_nt_h_mode).  Otherwise whole rounds of 256-row
 * tiles run on the persistent kernel; the rows past the last whole round,
 * and every row when M is below one round (the gathered last-layer tail, B
 * rows) or C % 128 != 0, on the few-rows kernel (csrc/gemm_small.hip: exact
 * per-row scales). */
int rb_gemm_nt_h(const float* A, int64_t lda, int64_t M, int64_t R, const void* Wf, int64_t C,
                 const float* bias, float* out, int64_t ldo, int accumulate, float* rmax,
                 void* stream);

/* Which kernel takes rb_gemm_nt_h's calls from 16,384 rows: mode 1 the
 * weight-stationary kernel (default), 0 the persistent 256-row tiles (A/B);
 * any other value only queries.  Returns the previous mode.  Process-wide
 * host setting (not per stream). */
int rb_gemm_nt_h_mode(int mode);

/* rb_gemm_nt_h with the residual + dropout + LayerNorm that follows a
 * projection to d = 128 in its epilogue (RecBLR.py:142 after the
 * out-projection, :225-227 after the FeedForward's w_2): with
 * out = A Bm^T + bias (never stored), s = out * keep * scale + resid and
 * y = (s - mean) * rstd * gamma + beta — rb_add_ln_fwd(out, resid, ...)'s
 * outputs, s bit for bit (the same Philox keep-flags per element), mean and
 * rstd from a fixed-order combination of per-column-group moments (fp32
 * rounding apart from rb_add_ln_fwd's).  C = 128, R in {128, 256, 512};
 * resid, y and s_out [M, 128] at row stride ldo; all 16-B aligned; the
 * weight-stationary kernel only (rb_gemm_nt_h_mode 1, any M); mean and
 * rstd [M]; rmax as rb_gemm_nt_h.  Replaces nn.Linear + dropout + residual
 * + nn.LayerNorm's forward. */
int rb_gemm_nt_h_ln(const float* A, int64_t lda, int64_t M, int64_t R, const void* Wf, int64_t C,
                    const float* bias, const float* resid, const float* gamma, const float* beta,
                    float eps, uint64_t seed, float p, float* y, float* s_out, float* mean,
                    float* rstd, int64_t ldo, float* rmax, void* stream);

/* rb_gemm_nt_h with the FeedForward's activation in its epilogue
 * (RecBLR.py:219-221, w_1 then dropout(silu(.))): out = A Bm^T + bias and
 * act = dropout(silu(out)), both [M, C] with row stride ldo — act equals
 * rb_silu_dropout_fwd(out, NULL, NULL, seed, p) bit for bit (same Philox
 * flags per element).  Taken only where every row runs on a wide-epilogue
 * launch: out and act 16-B aligned, ldo % 4 == 0, C % 256 == 0, R <= 1024 and
 * not (M <= 4096 and (R > 256 or C < 256)); other shapes fail (use
 * rb_gemm_nt_h + rb_silu_dropout_fwd). */
int rb_gemm_nt_h_act(const float* A, int64_t lda, int64_t M, int64_t R, const void* Wf, int64_t C,
                     const float* bias, float* out, int64_t ldo, float* rmax, float* act,
                     uint64_t seed, float p, void* stream);

/* The backward of rb_gemm_nt_h_act's activation fused into the FeedForward's
 * input-gradient GEMM dU = dA2 W_2 (RecBLR.py:219-222 backward): dU is not
 * stored; out = dropout-backward(dU) * silu'(pre) — rb_silu_dropout_bwd(pre,
 * NULL, NULL, seed, p, dU) bit for bit — with pre the activation's input
 * (rb_gemm_nt_h_act's out), [M, C] at row stride ldo like out; dpart
 * [n_parts, C] receives column sums of out per workgroup in a fixed order
 * (the w_1 bias gradient's partials; sum them, e.g. rb_colsum; unused rows
 * zeroed).  n_parts >= rb_gemm_nt_h_dact_parts().  Shape contract of
 * rb_gemm_nt_h_act, C <= 512; no bias. */
int64_t rb_gemm_nt_h_dact_parts(void);
int rb_gemm_nt_h_dact(const float* A, int64_t lda, int64_t M, int64_t R, const void* Wf, int64_t C,
                      float* out, int64_t ldo, float* rmax, const float* pre, uint64_t seed,
                      float p, float* dpart, int64_t n_parts, void* stream);

/* Weight gradient of F.linear, dW = dY^T X, as `splits` fixed-order row-chunk
 * partials on the f16 pipe (two-part split, three products):
 * parts[s][n, k] = sum over the rows m of chunk s of dY[m, n] X[m, k]
 * (rows split into `splits` chunks of a multiple of 32 rows; parts [splits,
 * N, K] fp32, every slot written; sum them in order, e.g. rb_colsum).
 * ymax / xmax [ceil(M/32)]: max |dY| / |X| over each 32-row group — the rmax
 * side outputs of the rb_gemm_nt_h calls that read the same operands (the
 * operand scales).  N % 128 == 0, K % 128 == 0, splits >= 1, row strides
 * multiples of 4, operands 16-B aligned.  A row chunk (ceil(ceil(M/splits)/32)
 * * 32 rows) must span < 2 GiB of either operand, max(ldy, ldx) * 4 bytes per
 * row: the kernel addresses a chunk with 32-bit offsets; pass more splits
 * otherwise (an argument error, never a silent wrap). */
int rb_gemm_tn_h(const float* dY, int64_t ldy, const float* X, int64_t ldx, int64_t M, int64_t N,
                 int64_t K, const float* ymax, const float* xmax, float* parts, int64_t splits,
                 void* stream);

/* ---- bf16 activations (BASELINE configs[4]: L = 2048, d = 256) ----------
 * The same Linears (RecBLR.py:162,165,167 and their autograd) when the
 * activations are bf16: bf16 operands on the bf16 MFMA pipe (NT:
 * v_mfma_f32_16x16x32_bf16, TN: 32x32x16), fp32 accumulation
 * (csrc/gemm_bf16.hip).  Replace torch.addmm / mm / bmm on
 * bf16 tensors (hipBLASLt).
 *
 * The weight image: Bm [C, R] = W (transpose = 0; W row stride ldw) or W^T
 * (transpose = 1), rounded to bf16 (nearest even) in 16x16x32 fragment
 * order (fragment (16-column block cb, k32 block kb) = 64 lanes x 8 bf16,
 * lane l: column 16 cb + l % 16, k 32 kb + 8 (l / 16) ..); img holds C * R
 * bf16 (2 C R bytes, 16-byte aligned); C % 16 == 0, R % 32 == 0. */
int rb_gemm_bf16_weight_image(const float* W, int64_t ldw, int64_t C, int64_t R, int transpose,
                              void* img, void* stream);

/* out[M, C] (bf16, row stride ldo) = A[M, R] (bf16, row stride lda) . Bm^T
 * (+ bias[C], fp32, added before the one rounding to bf16).  R % 64 == 0,
 * C % 256 == 0, lda % 8 == 0, ldo % 8 == 0; A, img, out, bias 16-byte
 * aligned (16-B result stores). */
int rb_gemm_nt_bf16(const void* A, int64_t lda, int64_t M, int64_t R, const void* img, int64_t C,
                    const float* bias, void* out, int64_t ldo, void* stream);

/* dW (+)= dY^T X for few rows M (F.linear's weight gradient on the gathered
 * last-layer tail, RecBLR.py:167,213,214 at B rows; any M up to 2^24, fastest
 * below ~16k): dW [N, K] row-major fp32, written (accumulate = 0) or added to
 * (accumulate = 1); f16 two-part split with exact per-column scales over each
 * eighth of the rows (no rmax needed); N % 32 == 0, K % 32 == 0; any row
 * strides and alignment.  Deterministic (fixed-order partial sums). */
int rb_gemm_tn_hs(const float* dY, int64_t ldy, const float* X, int64_t ldx, int64_t M, int64_t N,
                  int64_t K, float* dw, int accumulate, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RECBLR_HIP_H */
