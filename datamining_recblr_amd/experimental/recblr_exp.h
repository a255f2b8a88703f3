/* recblr_exp.h — opt-in experimental kernels (libdmrecblr_exp.so).
 *
 * Not in the product library: these measured slower than the default path
 * and stay opt-in (RECBLR_FUSED_GRL=1, RECBLR_FUSED_GRL_BWD=1), tested against
 * the oracle in the whole step (tests/test_gpu_e2e.py) and against the
 * three-launch path (tests/test_gpu_fused.py).  Same conventions as the
 * boundary (include/recblr_hip.h): raw device pointers, int status (0 = ok,
 * RB_EINVAL = -1 for a bad argument), rb_exp_last_error_string() for the
 * message, stream as void*. */
#ifndef RECBLR_EXP_H
#define RECBLR_EXP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of the experimental library (the product ABI it pairs with). */
int rb_exp_version(void);
const char* rb_exp_last_error_string(void);

/* GatedRecurrentLayer's core in one launch (RecBLR.py:182-206 between the
 * in- and out-projections), forward, packed sequences, fp32, H == 256:
 * xc = silu(causal depthwise conv(x) + b) (conv_w [H, kc], kc in 2..4),
 * rg = xc W_g^T (W_g's f16 image: rb_gemm_h_split_weights, C = 2H, R = H;
 * three fp16 products, fp32 accumulate) + gate_b, alpha / beta gates, the
 * BD-LRU scan from h0 ([H], shared; NULL = zeros) and y = silu(z) h.
 * xz [ntok, 2H] (x | z), row stride xz_rs.  pieces: int32 [3B + G + 1] =
 * each work piece's start row, length and packed sequence index (whole
 * sequences, B of them), then G + 1 offsets into the piece list, one span
 * per workgroup.  Outputs: y [ntok, H] (y_rs) or y_last [B, H] (each
 * sequence's last row, packed order) — exactly one; optional xc [ntok, H],
 * rg [ntok, 2H] (the GEMM without gate_b), carries [B, n_tiles, H] (the
 * state entering every 16-step tile: rb_gate_scan_bwd's checkpoints) and
 * xc_rmax [ceil(ntok/32)] (max |xc| per 32-row group, the caller zeroes
 * it).  tile_carries [G, max_tiles, H] (optional): the state entering each
 * of a workgroup's 64-row tiles, the checkpoints of rb_grl_bwd.  Replaces
 * the reference's conv / gates Linear / gate math / parallel_scan chain
 * (RecBLR.py:173-206, parallel_scan.py:117). */
int rb_grl_fwd(const float* xz, int64_t xz_rs, const float* conv_w, int64_t kc,
               const float* conv_b, const void* wg_img, const float* gate_b, const float* lam,
               const float* h0, const int32_t* pieces, int64_t B, int64_t G, int64_t ntok,
               int64_t H, float* y, int64_t y_rs, float* y_last, float* xc, float* rg,
               float* carries, int64_t n_tiles, float* xc_rmax, float* tile_carries,
               int64_t max_tiles, void* stream);

/* Backward of rb_grl_fwd in one launch (autograd of RecBLR.py:182-206 and
 * parallel_scan.py:117's backward): the same pieces and 64-row tiles walked
 * in reverse; conv, gates GEMM and the forward scan recomputed from xz and
 * the forward's tile_carries; dy [ntok, H] or dy_last [B, H] (exactly one).
 * Writes dxz [ntok, 2H] (dx | dz; row stride dxz_rs), drg [ntok, 2H] (the
 * gates GEMM's output gradient), xc [ntok, H] (its input, for the weight
 * gradient drg^T xc), optional drg_rmax / xc_rmax [ceil(ntok/32)] (32-row
 * group maxima, zeroed by the caller), part [G, 4, H] (per workgroup:
 * dLambda, d gate_b r and i halves, dh0) and cpart [8G, H kc + H] (per
 * wave: d conv_w in [H, kc] order, d conv_b); column sums of part and cpart
 * are the parameter gradients.  dxc = drg W_g runs inside on W_g^T's f16
 * image (wgt_img: rb_gemm_h_split_weights of W_g^T, C = H, R = 2H). */
int rb_grl_bwd(const float* xz, int64_t xz_rs, const float* conv_w, int64_t kc,
               const float* conv_b, const void* wg_img, const void* wgt_img, const float* gate_b,
               const float* lam, const float* h0, const int32_t* pieces, int64_t B, int64_t G,
               int64_t ntok, int64_t H, const float* tile_carries, int64_t max_tiles,
               const float* dy, const float* dy_last, float* dxz, int64_t dxz_rs, float* drg,
               float* xc, float* drg_rmax, float* xc_rmax, float* part, float* cpart,
               void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RECBLR_EXP_H */
