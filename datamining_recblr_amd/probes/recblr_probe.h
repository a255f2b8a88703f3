/* recblr_probe.h — measurement aids for bench.py (libdmrecblr_probe.so).
 *
 * Not part of the drop-in boundary (include/recblr_hip.h): no reference
 * interface corresponds to these; they time the access patterns of the
 * product kernels with trivial arithmetic so the bench can report each
 * kernel against the rate the memory system grants its pattern.  Same
 * conventions as the boundary: raw device pointers, int status (0 = ok),
 * rb_probe_last_error_string() for the message, stream as void*. */
#ifndef RECBLR_PROBE_H
#define RECBLR_PROBE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* rb_probe_last_error_string(void);

/* Measurement aid (bench.py gemm.pattern; not on the model's path): the HBM
 * bytes of out[M, C] = a[M, R] W^T without the product — every row of a
 * (contiguous, R % 4 == 0) read once, C floats per row written (C % 4 == 0),
 * 16-B accesses, both 16-B aligned.  Replaces no reference interface. */
int rb_probe_gemm_pattern(const float* a, int64_t M, int64_t R, float* out, int64_t C,
                          void* stream);

/* Measurement aid (bench.py, not the model's path; no reference counterpart):
 * the memory access pattern of rb_gate_scan_bwd (fp32) — the same reads of
 * r, i, xc, z, dy and writes of dr, di, dxc, dz with the same row strides,
 * wave/lane layout, sequence pairing and reverse tile order — with one
 * product per output instead of the BD-LRU backward arithmetic.  Its rate is
 * the ceiling the memory system grants that pattern; outputs are
 * meaningless. */
int rb_probe_gate_bwd_pattern(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                              const float* z, int64_t z_rs, const float* dy, float* drg,
                              int64_t drg_rs, float* dxc, int64_t dxc_rs, float* dz,
                              int64_t dz_rs, int64_t B, int64_t L, int64_t H,
                              const int64_t* seq_offsets, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RECBLR_PROBE_H */
