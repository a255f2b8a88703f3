// capi.hip — the extern "C" boundary declared in include/recblr_hip.h:
// argument validation, error reporting, dispatch to the kernel launchers.
#include "common.h"

#include <atomic>

namespace rb {

namespace {
thread_local std::string g_last_error;
}

int fail(const char* msg) {
  g_last_error = msg;
  return RB_EINVAL;
}

int num_cus() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return static_cast<int>(e);
  }
  return 0;
}

namespace {

// Per-lane offsets inside one batch row are 32-bit: L * row_stride must fit.
int check_dims(const char* fn, int64_t B, int64_t L, int64_t H, int64_t max_rs) {
  (void)fn;
  if (B <= 0 || L <= 0 || H <= 0) return fail("B, L and H must be positive");
  if (L * max_rs + max_rs >= (int64_t(1) << 31)) return fail("L * row_stride exceeds 2^31");
  if (B * ((H + 15) / 16) / 4 + 1 > 0x7fffffffLL) return fail("grid too large");
  return 0;
}

int64_t max4(int64_t a, int64_t b, int64_t c = 0, int64_t d = 0) {
  return std::max(std::max(a, b), std::max(c, d));
}

}  // namespace

DropSpec make_drop(const uint8_t* mask, uint64_t seed, float p) {
  DropSpec d{};
  d.mask = mask;
  d.scale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  d.key0 = (uint32_t)seed;
  d.key1 = (uint32_t)(seed >> 32);
  const double keep = 1.0 - (double)p;
  d.keep_thresh = keep >= 1.0 ? 0xFFFFFFFFu : (uint32_t)(keep * 4294967296.0);
  d.mode = mask ? 1 : (p > 0.0f ? 2 : 0);
  return d;
}
}  // namespace rb

using namespace rb;

extern "C" {

int rb_version(void) { return 44; }

const char* rb_last_error_string(void) { return g_last_error.c_str(); }

int rb_num_kernels(void) { return 24; }

int rb_scan_fwd(const float* gates, const float* tokens, float* states, int64_t B, int64_t C,
                int64_t T, void* stream) {
  if (!gates || !tokens || !states) return fail("rb_scan_fwd: null pointer");
  if (B <= 0 || C <= 0 || T <= 0) return fail("rb_scan_fwd: B, C, T must be positive");
  const int64_t rows = B * C;
  if ((rows + 3) / 4 > 0x7fffffffLL) return fail("rb_scan_fwd: too many rows");
  return launch_scan_fwd(gates, tokens, states, rows, T, reinterpret_cast<hipStream_t>(stream));
}

int rb_scan_bwd(const float* gates, const float* states, const float* grad, float* d_gates,
                float* d_tokens, int64_t B, int64_t C, int64_t T, void* stream) {
  if (!gates || !states || !grad || !d_gates || !d_tokens)
    return fail("rb_scan_bwd: null pointer");
  if (B <= 0 || C <= 0 || T <= 0) return fail("rb_scan_bwd: B, C, T must be positive");
  const int64_t rows = B * C;
  if ((rows + 3) / 4 > 0x7fffffffLL) return fail("rb_scan_bwd: too many rows");
  return launch_scan_bwd(gates, states, grad, d_gates, d_tokens, rows, T,
                         reinterpret_cast<hipStream_t>(stream));
}

int rb_conv_silu_fwd(const float* x, int64_t x_rs, const float* w, const float* bias, float* xc,
                     int64_t xc_rs, int64_t B, int64_t L, int64_t H, int64_t K, const int64_t* seq_offsets, void* stream) {
  if (!x || !w || !bias || !xc) return fail("rb_conv_silu_fwd: null pointer");
  if (K < 1 || K > 8) return fail("rb_conv_silu_fwd: kernel size K must be in [1, 8]");
  if (x_rs < H || xc_rs < H) return fail("rb_conv_silu_fwd: row stride < H");
  if (int r = check_dims("rb_conv_silu_fwd", B, L, H, max4(x_rs, xc_rs))) return r;
  return launch_conv_fwd(x, x_rs, w, bias, xc, xc_rs, B, L, H, K,
                         seq_offsets, reinterpret_cast<hipStream_t>(stream));
}

int rb_conv_silu_fwd_rows(const float* x, int64_t x_rs, const float* w, const float* bias,
                          float* xc, int64_t xc_rs, int64_t ntok, int64_t H, int64_t K,
                          const int64_t* row_pos, void* stream) {
  if (!x || !w || !bias || !xc || !row_pos) return fail("rb_conv_silu_fwd_rows: null pointer");
  if (K < 1 || K > 8) return fail("rb_conv_silu_fwd_rows: kernel size K must be in [1, 8]");
  if (x_rs < H || xc_rs < H) return fail("rb_conv_silu_fwd_rows: row stride < H");
  if (int r = check_dims("rb_conv_silu_fwd_rows", ntok, 1, H, max4(x_rs, xc_rs))) return r;
  return launch_conv_fwd_rows(x, x_rs, w, bias, xc, xc_rs, ntok, H, K, row_pos,
                              reinterpret_cast<hipStream_t>(stream));
}

int rb_conv_silu_bwd(const float* x, int64_t x_rs, const float* w, const float* bias,
                     const float* g1, const float* g2, float* dx, int64_t dx_rs, float* dw_part,
                     float* db_part, int64_t B, int64_t L, int64_t H, int64_t K, const int64_t* seq_offsets, void* stream) {
  if (!x || !w || !bias || !g1 || !dx || !dw_part)   // db_part NULL: folded layout
    return fail("rb_conv_silu_bwd: null pointer");
  if (K < 1 || K > 8) return fail("rb_conv_silu_bwd: kernel size K must be in [1, 8]");
  if (x_rs < H || dx_rs < H) return fail("rb_conv_silu_bwd: row stride < H");
  if (int r = check_dims("rb_conv_silu_bwd", B, L, H, max4(x_rs, dx_rs, H))) return r;
  return launch_conv_bwd(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, K,
                         seq_offsets, reinterpret_cast<hipStream_t>(stream));
}

int rb_gate_scan_fwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                     const float* z, int64_t z_rs, const float* lam, const float* gate_b,
                     const float* h0, int64_t h0_bs, float* y, int64_t y_rs, float* carries,
                     int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets, void* stream) {
  if (!rg || !xc || !z || !lam || !y) return fail("rb_gate_scan_fwd: null pointer");
  if (h0_bs != 0 && h0_bs < H) return fail("rb_gate_scan_fwd: h0 batch stride must be 0 or >= H");
  if (rg_rs < 2 * H || xc_rs < H || z_rs < H || y_rs < H)
    return fail("rb_gate_scan_fwd: row stride too small");
  if (int r = check_dims("rb_gate_scan_fwd", B, L, H, max4(rg_rs, xc_rs, z_rs, y_rs))) return r;
  return launch_gate_fwd(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gate_b, h0, h0_bs, y, y_rs, carries,
                         B, L, H, seq_offsets, reinterpret_cast<hipStream_t>(stream));
}

int rb_gate_scan_fwd_last(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                          const float* z, int64_t z_rs, const float* lam, const float* gate_b,
                          const float* h0, int64_t h0_bs, float* y_last, float* carries,
                          int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets,
                          const int64_t* batch_row, void* stream) {
  if (!rg || !xc || !z || !lam || !y_last) return fail("rb_gate_scan_fwd_last: null pointer");
  if (h0_bs != 0 && h0_bs < H)
    return fail("rb_gate_scan_fwd_last: h0 batch stride must be 0 or >= H");
  if (rg_rs < 2 * H || xc_rs < H || z_rs < H)
    return fail("rb_gate_scan_fwd_last: row stride too small");
  if (int r = check_dims("rb_gate_scan_fwd_last", B, L, H, max4(rg_rs, xc_rs, z_rs, H))) return r;
  return launch_gate_fwd(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gate_b, h0, h0_bs, nullptr, H,
                         carries, B, L, H, seq_offsets, reinterpret_cast<hipStream_t>(stream),
                         y_last, batch_row);
}

int rb_gate_scan_bwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                     const float* z, int64_t z_rs, const float* lam, const float* gate_b,
                     const float* carries,
                     const float* dy, float* drg, int64_t drg_rs, float* dxc, int64_t dxc_rs,
                     float* dz, int64_t dz_rs, float* part, float* dh0_part, int64_t B,
                     int64_t L, int64_t H, const int64_t* seq_offsets, void* stream) {
  if (!rg || !xc || !z || !lam || !carries || !dy || !drg || !dxc || !dz || !part || !dh0_part)
    return fail("rb_gate_scan_bwd: null pointer");
  if (rg_rs < 2 * H || xc_rs < H || z_rs < H || drg_rs < 2 * H || dxc_rs < H || dz_rs < H)
    return fail("rb_gate_scan_bwd: row stride too small");
  if (int r = check_dims("rb_gate_scan_bwd", B, L, H,
                         max4(max4(rg_rs, xc_rs, z_rs, drg_rs), dz_rs, dxc_rs, H)))
    return r;
  return launch_gate_bwd(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gate_b, carries, dy, drg, drg_rs, dxc,
                         dxc_rs, dz, dz_rs, part, dh0_part, B, L, H,
                         seq_offsets, reinterpret_cast<hipStream_t>(stream));
}

// ---- bf16 storage variants (fp32 arithmetic; same checks as the fp32 forms) ----
#define BF(p) reinterpret_cast<const bf16_t*>(p)
#define BFW(p) reinterpret_cast<bf16_t*>(p)

int rb_gate_scan_bwd_last(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                          const float* z, int64_t z_rs, const float* lam, const float* gate_b,
                          const float* carries, const float* dy_last, float* drg,
                          int64_t drg_rs, float* dxc, int64_t dxc_rs, float* dz, int64_t dz_rs,
                          float* part, float* dh0_part, int64_t B, int64_t L, int64_t H,
                          const int64_t* seq_offsets, const int64_t* batch_row, void* stream) {
  if (!rg || !xc || !z || !lam || !carries || !dy_last || !drg || !dxc || !dz || !part ||
      !dh0_part)
    return fail("rb_gate_scan_bwd_last: null pointer");
  if (rg_rs < 2 * H || xc_rs < H || z_rs < H || drg_rs < 2 * H || dxc_rs < H || dz_rs < H)
    return fail("rb_gate_scan_bwd_last: row stride too small");
  if (int r = check_dims("rb_gate_scan_bwd_last", B, L, H,
                         max4(max4(rg_rs, xc_rs, z_rs, drg_rs), dz_rs, dxc_rs, H)))
    return r;
  return launch_gate_bwd(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gate_b, carries, nullptr, drg,
                         drg_rs, dxc, dxc_rs, dz, dz_rs, part, dh0_part, B, L, H, seq_offsets,
                         reinterpret_cast<hipStream_t>(stream), dy_last, batch_row);
}

int rb_scan_fwd_bf16(const rb_bf16* gates, const rb_bf16* tokens, rb_bf16* states, int64_t B,
                     int64_t C, int64_t T, void* stream) {
  if (!gates || !tokens || !states) return fail("rb_scan_fwd_bf16: null pointer");
  if (B <= 0 || C <= 0 || T <= 0) return fail("rb_scan_fwd_bf16: B, C, T must be positive");
  const int64_t rows = B * C;
  if ((rows + 3) / 4 > 0x7fffffffLL) return fail("rb_scan_fwd_bf16: too many rows");
  return launch_scan_fwd_bf16(BF(gates), BF(tokens), BFW(states), rows, T,
                              reinterpret_cast<hipStream_t>(stream));
}

int rb_scan_bwd_bf16(const rb_bf16* gates, const rb_bf16* states, const rb_bf16* grad,
                     rb_bf16* d_gates, rb_bf16* d_tokens, int64_t B, int64_t C, int64_t T,
                     void* stream) {
  if (!gates || !states || !grad || !d_gates || !d_tokens)
    return fail("rb_scan_bwd_bf16: null pointer");
  if (B <= 0 || C <= 0 || T <= 0) return fail("rb_scan_bwd_bf16: B, C, T must be positive");
  const int64_t rows = B * C;
  if ((rows + 3) / 4 > 0x7fffffffLL) return fail("rb_scan_bwd_bf16: too many rows");
  return launch_scan_bwd_bf16(BF(gates), BF(states), BF(grad), BFW(d_gates), BFW(d_tokens), rows,
                              T, reinterpret_cast<hipStream_t>(stream));
}

int rb_conv_silu_fwd_bf16(const rb_bf16* x, int64_t x_rs, const float* w, const float* bias,
                          rb_bf16* xc, int64_t xc_rs, int64_t B, int64_t L, int64_t H, int64_t K,
                          const int64_t* seq_offsets, void* stream) {
  if (!x || !w || !bias || !xc) return fail("rb_conv_silu_fwd_bf16: null pointer");
  if (K < 1 || K > 8) return fail("rb_conv_silu_fwd_bf16: kernel size K must be in [1, 8]");
  if (x_rs < H || xc_rs < H) return fail("rb_conv_silu_fwd_bf16: row stride < H");
  if (int r = check_dims("rb_conv_silu_fwd_bf16", B, L, H, max4(x_rs, xc_rs))) return r;
  return launch_conv_fwd_bf16(BF(x), x_rs, w, bias, BFW(xc), xc_rs, B, L, H, K,
                              seq_offsets, reinterpret_cast<hipStream_t>(stream));
}

int rb_conv_silu_fwd_rows_bf16(const rb_bf16* x, int64_t x_rs, const float* w, const float* bias,
                               rb_bf16* xc, int64_t xc_rs, int64_t ntok, int64_t H, int64_t K,
                               const int64_t* row_pos, void* stream) {
  if (!x || !w || !bias || !xc || !row_pos)
    return fail("rb_conv_silu_fwd_rows_bf16: null pointer");
  if (K < 1 || K > 8) return fail("rb_conv_silu_fwd_rows_bf16: kernel size K must be in [1, 8]");
  if (x_rs < H || xc_rs < H) return fail("rb_conv_silu_fwd_rows_bf16: row stride < H");
  if (int r = check_dims("rb_conv_silu_fwd_rows_bf16", ntok, 1, H, max4(x_rs, xc_rs))) return r;
  return launch_conv_fwd_rows_bf16(BF(x), x_rs, w, bias, BFW(xc), xc_rs, ntok, H, K, row_pos,
                                   reinterpret_cast<hipStream_t>(stream));
}

int rb_conv_silu_bwd_bf16(const rb_bf16* x, int64_t x_rs, const float* w, const float* bias,
                          const rb_bf16* g1, const rb_bf16* g2, rb_bf16* dx, int64_t dx_rs,
                          float* dw_part, float* db_part, int64_t B, int64_t L, int64_t H,
                          int64_t K, const int64_t* seq_offsets, void* stream) {
  if (!x || !w || !bias || !g1 || !dx || !dw_part)   // db_part NULL: folded layout
    return fail("rb_conv_silu_bwd_bf16: null pointer");
  if (K < 1 || K > 8) return fail("rb_conv_silu_bwd_bf16: kernel size K must be in [1, 8]");
  if (x_rs < H || dx_rs < H) return fail("rb_conv_silu_bwd_bf16: row stride < H");
  if (int r = check_dims("rb_conv_silu_bwd_bf16", B, L, H, max4(x_rs, dx_rs, H))) return r;
  return launch_conv_bwd_bf16(BF(x), x_rs, w, bias, BF(g1), g2 ? BF(g2) : nullptr, BFW(dx),
                              dx_rs, dw_part, db_part, B, L, H, K,
                              seq_offsets, reinterpret_cast<hipStream_t>(stream));
}

int rb_gate_scan_fwd_bf16(const rb_bf16* rg, int64_t rg_rs, const rb_bf16* xc, int64_t xc_rs,
                          const rb_bf16* z, int64_t z_rs, const float* lam, const float* gate_b,
                          const float* h0, int64_t h0_bs, rb_bf16* y, int64_t y_rs,
                          float* carries, int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets, void* stream) {
  if (!rg || !xc || !z || !lam || !y) return fail("rb_gate_scan_fwd_bf16: null pointer");
  if (h0_bs != 0 && h0_bs < H)
    return fail("rb_gate_scan_fwd_bf16: h0 batch stride must be 0 or >= H");
  if (rg_rs < 2 * H || xc_rs < H || z_rs < H || y_rs < H)
    return fail("rb_gate_scan_fwd_bf16: row stride too small");
  if (int r = check_dims("rb_gate_scan_fwd_bf16", B, L, H, max4(rg_rs, xc_rs, z_rs, y_rs)))
    return r;
  return launch_gate_fwd_bf16(BF(rg), rg_rs, BF(xc), xc_rs, BF(z), z_rs, lam, gate_b, h0, h0_bs,
                              BFW(y), y_rs, carries, B, L, H,
                              seq_offsets, reinterpret_cast<hipStream_t>(stream));
}

int rb_gate_scan_bwd_bf16(const rb_bf16* rg, int64_t rg_rs, const rb_bf16* xc, int64_t xc_rs,
                          const rb_bf16* z, int64_t z_rs, const float* lam, const float* gate_b,
                          const float* carries, const rb_bf16* dy, rb_bf16* drg, int64_t drg_rs,
                          rb_bf16* dxc, int64_t dxc_rs, rb_bf16* dz, int64_t dz_rs, float* part,
                          float* dh0_part, int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets, void* stream) {
  if (!rg || !xc || !z || !lam || !carries || !dy || !drg || !dxc || !dz || !part || !dh0_part)
    return fail("rb_gate_scan_bwd_bf16: null pointer");
  if (rg_rs < 2 * H || xc_rs < H || z_rs < H || drg_rs < 2 * H || dxc_rs < H || dz_rs < H)
    return fail("rb_gate_scan_bwd_bf16: row stride too small");
  if (int r = check_dims("rb_gate_scan_bwd_bf16", B, L, H,
                         max4(max4(rg_rs, xc_rs, z_rs, drg_rs), dz_rs, dxc_rs, H)))
    return r;
  return launch_gate_bwd_bf16(BF(rg), rg_rs, BF(xc), xc_rs, BF(z), z_rs, lam, gate_b, carries,
                              BF(dy), BFW(drg), drg_rs, BFW(dxc), dxc_rs, BFW(dz), dz_rs, part,
                              dh0_part, B, L, H, seq_offsets, reinterpret_cast<hipStream_t>(stream));
}

#undef BF
#undef BFW

int rb_add_ln_fwd(const float* a, const int64_t* idx, int64_t n_idx_rows, const uint8_t* mask,
                  uint64_t seed, float p, const float* r, const float* gamma, const float* beta,
                  float eps, float* y, float* s_out, float* mean, float* rstd, int64_t rows,
                  int64_t d, void* stream) {
  if (!a || !gamma || !beta || !y) return fail("rb_add_ln_fwd: null pointer");
  if (rows <= 0 || d <= 0) return fail("rb_add_ln_fwd: rows and d must be positive");
  if (idx && n_idx_rows <= 0) return fail("rb_add_ln_fwd: empty gather table");
  if (!(p >= 0.0f && p < 1.0f)) return fail("rb_add_ln_fwd: dropout p must be in [0, 1)");
  if ((s_out == nullptr) != (mean == nullptr) || (mean == nullptr) != (rstd == nullptr))
    return fail("rb_add_ln_fwd: s_out, mean and rstd must be given together");
  return launch_add_ln_fwd(a, idx, n_idx_rows, make_drop(mask, seed, p), r, gamma, beta, eps, y,
                           s_out, mean, rstd, rows, d, reinterpret_cast<hipStream_t>(stream));
}

int64_t rb_row_num_parts(int64_t rows, int64_t width) {
  if (rows <= 0 || width <= 0) return 0;
  return ln_num_parts(rows, width);
}

int rb_add_ln_bwd2(const float* dy, const float* dy2, const float* s, const float* gamma,
                   const float* mean, const float* rstd, const uint8_t* mask, uint64_t seed,
                   float p, float* ds, float* da, float* dgamma_part, float* dbeta_part,
                   float* dbias_part, int64_t n_parts, int64_t rows, int64_t d, void* stream) {
  if (!dy || !s || !gamma || !mean || !rstd || !dgamma_part || !dbeta_part)
    return fail("rb_add_ln_bwd: null pointer");
  if (!ds && !da && !dbias_part) return fail("rb_add_ln_bwd: nothing to write");
  if (rows <= 0 || d <= 0) return fail("rb_add_ln_bwd: rows and d must be positive");
  if (!(p >= 0.0f && p < 1.0f)) return fail("rb_add_ln_bwd: dropout p must be in [0, 1)");
  if (n_parts != ln_num_parts(rows, d)) return fail("rb_add_ln_bwd: n_parts != rb_row_num_parts");
  return launch_add_ln_bwd(dy, dy2, s, gamma, mean, rstd, make_drop(mask, seed, p), ds, da,
                           dgamma_part, dbeta_part, dbias_part, n_parts, rows, d,
                           reinterpret_cast<hipStream_t>(stream));
}

int rb_add_ln_bwd(const float* dy, const float* s, const float* gamma, const float* mean,
                  const float* rstd, const uint8_t* mask, uint64_t seed, float p, float* ds,
                  float* da, float* dgamma_part, float* dbeta_part, float* dbias_part,
                  int64_t n_parts, int64_t rows, int64_t d, void* stream) {
  return rb_add_ln_bwd2(dy, nullptr, s, gamma, mean, rstd, mask, seed, p, ds, da, dgamma_part,
                        dbeta_part, dbias_part, n_parts, rows, d, stream);
}

int rb_silu_dropout_fwd(const float* a, const float* bias, const uint8_t* mask, uint64_t seed,
                        float p, float* u, int64_t rows, int64_t cols, void* stream) {
  if (!a || !u) return fail("rb_silu_dropout_fwd: null pointer");
  if (bias && !aligned16(bias)) return fail("rb_silu_dropout_fwd: misaligned bias");
  if (rows <= 0 || cols <= 0) return fail("rb_silu_dropout_fwd: rows and cols must be positive");
  if (!(p >= 0.0f && p < 1.0f)) return fail("rb_silu_dropout_fwd: dropout p must be in [0, 1)");
  if (!aligned16(a) || !aligned16(u) || (mask && (reinterpret_cast<uintptr_t>(mask) & 3)))
    return fail("rb_silu_dropout_fwd: misaligned buffer");
  return launch_silu_dropout_fwd(a, bias, make_drop(mask, seed, p), u, rows, cols,
                                 reinterpret_cast<hipStream_t>(stream));
}

int rb_silu_dropout_bwd(const float* a, const float* bias, const uint8_t* mask, uint64_t seed,
                        float p, const float* du, float* da, float* dbias_part, int64_t n_parts,
                        int64_t rows, int64_t cols, void* stream) {
  if (!a || !du || !da) return fail("rb_silu_dropout_bwd: null pointer");
  if (bias && !aligned16(bias)) return fail("rb_silu_dropout_bwd: misaligned bias");
  if (rows <= 0 || cols <= 0) return fail("rb_silu_dropout_bwd: rows and cols must be positive");
  if (!(p >= 0.0f && p < 1.0f)) return fail("rb_silu_dropout_bwd: dropout p must be in [0, 1)");
  if (!aligned16(a) || !aligned16(du) || !aligned16(da) ||
      (mask && (reinterpret_cast<uintptr_t>(mask) & 3)))
    return fail("rb_silu_dropout_bwd: misaligned buffer");
  if (dbias_part && n_parts != ln_num_parts(rows, cols))
    return fail("rb_silu_dropout_bwd: n_parts != rb_row_num_parts");
  return launch_silu_dropout_bwd(a, bias, make_drop(mask, seed, p), du, da, dbias_part,
                                 ln_num_parts(rows, cols), rows, cols,
                                 reinterpret_cast<hipStream_t>(stream));
}

int rb_dropout_mask(uint64_t seed, float p, uint8_t* out, int64_t n, void* stream) {
  if (!out) return fail("rb_dropout_mask: null pointer");
  if (n <= 0 || n % 4) return fail("rb_dropout_mask: n must be a positive multiple of 4");
  if (!(p >= 0.0f && p < 1.0f)) return fail("rb_dropout_mask: dropout p must be in [0, 1)");
  return launch_dropout_mask(make_drop(nullptr, seed, p), out, n,
                             reinterpret_cast<hipStream_t>(stream));
}

int64_t rb_embedding_bwd_workspace(int64_t M, int64_t V, int64_t d) {
  if (M <= 0 || V <= 0 || d <= 0) return 0;
  return emb_workspace_bytes(M, V, d);
}

int rb_embedding_bwd_plan(const int64_t* idx, int64_t M, int64_t d, int64_t V, void* workspace,
                          int64_t workspace_bytes, void* stream) {
  if (!idx || !workspace) return fail("rb_embedding_bwd_plan: null pointer");
  if (M <= 0 || d <= 0 || V <= 0) return fail("rb_embedding_bwd_plan: M, d, V must be positive");
  if (M >= (int64_t(1) << 31) || V >= (int64_t(1) << 30))
    return fail("rb_embedding_bwd_plan: M or V too large");
  return launch_embedding_plan(idx, M, d, V, workspace, workspace_bytes,
                               reinterpret_cast<hipStream_t>(stream));
}

int rb_embedding_bwd_apply(const float* grad, int64_t M, int64_t d, int64_t V,
                           int64_t padding_idx, float* dweight, void* workspace,
                           int64_t workspace_bytes, void* stream) {
  if (!grad || !dweight || !workspace) return fail("rb_embedding_bwd_apply: null pointer");
  if (M <= 0 || d <= 0 || V <= 0) return fail("rb_embedding_bwd_apply: M, d, V must be positive");
  if (M >= (int64_t(1) << 31) || V >= (int64_t(1) << 30))
    return fail("rb_embedding_bwd_apply: M or V too large");
  return launch_embedding_apply(grad, M, d, V, padding_idx, dweight, workspace, workspace_bytes,
                                reinterpret_cast<hipStream_t>(stream));
}

int rb_embedding_bwd(const int64_t* idx, const float* grad, int64_t M, int64_t d, int64_t V,
                     int64_t padding_idx, float* dweight, void* workspace,
                     int64_t workspace_bytes, void* stream) {
  if (!idx || !grad || !dweight || !workspace) return fail("rb_embedding_bwd: null pointer");
  if (M <= 0 || d <= 0 || V <= 0) return fail("rb_embedding_bwd: M, d, V must be positive");
  if (M >= (int64_t(1) << 31) || V >= (int64_t(1) << 30))
    return fail("rb_embedding_bwd: M or V too large");
  return launch_embedding_bwd(idx, grad, M, d, V, padding_idx, dweight, workspace,
                              workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}

namespace {
int check_items(const char* fn, const float* seq, const float* items, int64_t B, int64_t V,
                int64_t d) {
  (void)fn;
  if (!seq || !items) return fail("item scores: null pointer");
  if (B <= 0 || V <= 0) return fail("item scores: B and V must be positive");
  if (d != 16 && d != 32 && d != 64 && d != 128 && d != 256)
    return fail("item scores: d must be 16, 32, 64, 128 or 256");
  if (!aligned16(seq) || !aligned16(items)) return fail("item scores: operands must be 16-B aligned");
  if (B >= (int64_t(1) << 31) || V >= (int64_t(1) << 31)) return fail("item scores: B or V too large");
  return 0;
}
}  // namespace

int64_t rb_item_ce_workspace(int64_t B, int64_t V, int64_t d) {
  if (B <= 0 || V <= 0 || d <= 0) return 0;
  return item_ce_workspace_bytes(B, V, d);
}

int rb_item_ce_fwd(const float* seq, const float* items, const int64_t* target, int64_t B,
                   int64_t V, int64_t d, float* lse, float* loss, void* workspace,
                   int64_t workspace_bytes, void* stream) {
  if (int rc = check_items("rb_item_ce_fwd", seq, items, B, V, d)) return rc;
  if (!target || !lse || !loss || !workspace) return fail("rb_item_ce_fwd: null pointer");
  return launch_item_ce_fwd(seq, items, target, B, V, d, lse, loss, workspace, workspace_bytes,
                            reinterpret_cast<hipStream_t>(stream));
}

int rb_item_ce_bwd(const float* seq, const float* items, const int64_t* target, const float* lse,
                   const float* dloss, int64_t B, int64_t V, int64_t d, float* dseq,
                   float* ditems, void* workspace, int64_t workspace_bytes, void* stream) {
  if (int rc = check_items("rb_item_ce_bwd", seq, items, B, V, d)) return rc;
  if (!target || !lse || !dloss || !workspace) return fail("rb_item_ce_bwd: null pointer");
  return launch_item_ce_bwd(seq, items, target, lse, dloss, B, V, d, dseq, ditems, workspace,
                            workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}

int64_t rb_item_rank_workspace(int64_t B, int64_t V, int64_t d) {
  if (B <= 0 || V <= 0 || d <= 0) return 0;
  return item_rank_workspace_bytes(B, V);
}

int rb_item_rank(const float* seq, const float* items, const int64_t* target, int64_t B,
                 int64_t V, int64_t d, int64_t first_item, int64_t* n_greater, int64_t* n_equal,
                 void* workspace, int64_t workspace_bytes, void* stream) {
  if (int rc = check_items("rb_item_rank", seq, items, B, V, d)) return rc;
  if (!target || !n_greater || !workspace) return fail("rb_item_rank: null pointer");
  if (first_item < 0) return fail("rb_item_rank: first_item must be >= 0");
  return launch_item_rank(seq, items, target, B, V, d, first_item, n_greater, n_equal, workspace,
                          workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}

int rb_item_ce_probs(const float* seq, const float* items, const int64_t* target,
                     const float* lse, const float* dloss, int64_t B, int64_t V, int64_t d,
                     int64_t item_offset, float* probs, int64_t ld, void* stream) {
  if (int rc = check_items("rb_item_ce_probs", seq, items, B, V, d)) return rc;
  if (!target || !lse || !dloss || !probs) return fail("rb_item_ce_probs: null pointer");
  if (ld < V) return fail("rb_item_ce_probs: ld < V");
  return launch_item_ce_probs(seq, items, target, lse, dloss, B, V, d, item_offset, V, probs, ld,
                              reinterpret_cast<hipStream_t>(stream));
}

int rb_item_split_h(const float* x, int64_t n, int64_t d, void* image, int* exps,
                    float* group_max, void* stream) {
  if (!x || !image || !exps) return fail("rb_item_split_h: null pointer");
  if (n <= 0) return fail("rb_item_split_h: n must be positive");
  if (d != 16 && d != 32 && d != 64 && d != 128 && d != 256)
    return fail("rb_item_split_h: d must be 16, 32, 64, 128 or 256");
  if (!aligned16(x) || !aligned16(image)) return fail("rb_item_split_h: operands must be 16-B aligned");
  if (n >= (int64_t(1) << 31)) return fail("rb_item_split_h: n too large");
  return launch_item_split_h(x, n, d, image, exps, group_max,
                             reinterpret_cast<hipStream_t>(stream));
}

namespace {
int check_items_h(const void* seq_img, const int* seq_exp, const void* item_img,
                  const int* item_exp, int64_t B, int64_t V, int64_t d) {
  if (!seq_exp || !item_exp) return fail("item scores (f16): null exponent pointer");
  return check_items("item scores (f16)", reinterpret_cast<const float*>(seq_img),
                     reinterpret_cast<const float*>(item_img), B, V, d);
}
}  // namespace

int rb_item_ce_fwd_h(const void* seq_img, const int* seq_exp, const void* item_img,
                     const int* item_exp, const int64_t* target, int64_t B, int64_t V, int64_t d,
                     float* lse, float* loss, void* workspace, int64_t workspace_bytes,
                     void* stream) {
  if (int rc = check_items_h(seq_img, seq_exp, item_img, item_exp, B, V, d)) return rc;
  if (!target || !lse || !loss || !workspace) return fail("rb_item_ce_fwd_h: null pointer");
  return launch_item_ce_fwd_h(seq_img, seq_exp, item_img, item_exp, target, B, V, d, lse, loss,
                              workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}

int rb_item_ce_probs_h(const void* seq_img, const int* seq_exp, const void* item_img,
                       const int* item_exp, const int64_t* target, const float* lse,
                       const float* dloss, int64_t B, int64_t V, int64_t d, int64_t item_offset,
                       float* probs, int64_t ld, void* stream) {
  if (int rc = check_items_h(seq_img, seq_exp, item_img, item_exp, B, V, d)) return rc;
  if (!target || !lse || !dloss || !probs) return fail("rb_item_ce_probs_h: null pointer");
  if (ld < V) return fail("rb_item_ce_probs_h: ld < V");
  return launch_item_ce_probs_h(seq_img, seq_exp, item_img, item_exp, target, lse, dloss, B, V, d,
                                item_offset, probs, ld, nullptr, nullptr, 0, nullptr,
                                reinterpret_cast<hipStream_t>(stream));
}

int rb_item_ce_probs_h_t(const void* seq_img, const int* seq_exp, const void* item_img,
                         const int* item_exp, const int64_t* target, const float* lse,
                         const float* dloss, int64_t B, int64_t V, int64_t d, int64_t item_offset,
                         float* probs_t, int64_t ldt, float* group_max, void* stream) {
  if (int rc = check_items_h(seq_img, seq_exp, item_img, item_exp, B, V, d)) return rc;
  if (!target || !lse || !dloss || !probs_t || !group_max)
    return fail("rb_item_ce_probs_h_t: null pointer");
  if (ldt < B || ldt % 4 || reinterpret_cast<uintptr_t>(probs_t) % 16)
    return fail("rb_item_ce_probs_h_t: probs_t must be 16-B aligned with ldt >= B, ldt % 4 == 0");
  return launch_item_ce_probs_h(seq_img, seq_exp, item_img, item_exp, target, lse, dloss, B, V, d,
                                item_offset, probs_t, ldt, group_max, nullptr, 0, nullptr,
                                reinterpret_cast<hipStream_t>(stream));
}

int rb_item_ce_probs_h_both(const void* seq_img, const int* seq_exp, const void* item_img,
                            const int* item_exp, const int64_t* target, const float* lse,
                            const float* dloss, int64_t B, int64_t V, int64_t d,
                            int64_t item_offset, float* probs, int64_t ld, float* probs_t,
                            int64_t ldt, float* row_group_max, float* item_group_max,
                            void* stream) {
  if (int rc = check_items_h(seq_img, seq_exp, item_img, item_exp, B, V, d)) return rc;
  if (!target || !lse || !dloss || !probs || !probs_t || !row_group_max || !item_group_max)
    return fail("rb_item_ce_probs_h_both: null pointer");
  if (ld < V) return fail("rb_item_ce_probs_h_both: ld < V");
  if (ldt < B || ldt % 4 || reinterpret_cast<uintptr_t>(probs_t) % 16)
    return fail("rb_item_ce_probs_h_both: probs_t must be 16-B aligned with ldt >= B, ldt % 4 == 0");
  return launch_item_ce_probs_h(seq_img, seq_exp, item_img, item_exp, target, lse, dloss, B, V, d,
                                item_offset, probs_t, ldt, item_group_max, probs, ld,
                                row_group_max, reinterpret_cast<hipStream_t>(stream));
}

int rb_group_absmax(const float* x, int64_t n, int64_t c, int64_t ld, float* out, void* stream) {
  if (!x || !out) return fail("rb_group_absmax: null pointer");
  if (n <= 0 || c <= 0 || ld < c) return fail("rb_group_absmax: bad shape");
  return launch_group_absmax(x, n, c, ld, out, reinterpret_cast<hipStream_t>(stream));
}

int rb_item_scores(const float* seq, const float* items, int64_t B, int64_t V, int64_t d,
                   float* scores, void* stream) {
  if (int rc = check_items("rb_item_scores", seq, items, B, V, d)) return rc;
  if (!scores) return fail("rb_item_scores: null pointer");
  return launch_item_scores(seq, items, B, V, d, scores, reinterpret_cast<hipStream_t>(stream));
}

int rb_pad_prefix_fwd(const float* conv_b, const float* gate_w, const float* gate_b,
                      const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                      int64_t H, float* h0, float* workspace, void* stream) {
  if (!conv_b || !gate_w || !gate_b || !lam || !h0 || !workspace)
    return fail("rb_pad_prefix_fwd: null pointer");
  if (H <= 0 || H > 4096 || n_rows <= 0 || pad_len < 0)
    return fail("rb_pad_prefix_fwd: need 0 < H <= 4096, n_rows > 0, pad_len >= 0");
  return launch_pad_prefix_fwd(conv_b, gate_w, gate_b, lam, pad, pad_len, n_rows, H, h0,
                               workspace, reinterpret_cast<hipStream_t>(stream));
}

int rb_pad_prefix_bwd(const float* conv_b, const float* gate_w, const float* gate_b,
                      const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                      int64_t H, const float* dh0, float* dconv_b, float* dgate_w,
                      float* dgate_b, float* dlam, float* workspace, int accumulate,
                      void* stream) {
  if (!conv_b || !gate_w || !gate_b || !lam || !dh0 || !dconv_b || !dgate_w || !dgate_b || !dlam ||
      !workspace)
    return fail("rb_pad_prefix_bwd: null pointer");
  if (H <= 0 || H > 4096 || n_rows <= 0 || pad_len < 0)
    return fail("rb_pad_prefix_bwd: need 0 < H <= 4096, n_rows > 0, pad_len >= 0");
  return launch_pad_prefix_bwd(conv_b, gate_w, gate_b, lam, pad, pad_len, n_rows, H, dh0,
                               dconv_b, dgate_w, dgate_b, dlam, workspace, accumulate,
                               reinterpret_cast<hipStream_t>(stream));
}

int rb_colsum(const float* in, int64_t M, int64_t P, int64_t C, int64_t rs, int64_t ms,
              float* out, void* stream) {
  if (!in || !out) return fail("rb_colsum: null pointer");
  if (M <= 0 || P <= 0 || C <= 0 || rs < C || (M > 1 && ms < P * rs))
    return fail("rb_colsum: bad shape or strides");
  if (M * ((C + 63) / 64) > 0x7fffffffLL) return fail("rb_colsum: grid too large");
  return launch_colsum(in, M, P, C, rs, ms, out, reinterpret_cast<hipStream_t>(stream));
}

int rb_colsum_chunked(const float* in, int64_t M, int64_t P, int64_t C, int64_t rs,
                      int64_t chunk_rows, float* part, uint32_t* counters, int64_t n_counters,
                      float* out, void* stream) {
  if (!in || !out || !part || !counters) return fail("rb_colsum_chunked: null pointer");
  if (M <= 0 || P <= 0 || C <= 0 || rs < C ||
      (chunk_rows != 64 && chunk_rows != 128 && chunk_rows != 256) || P % chunk_rows)
    return fail("rb_colsum_chunked: bad shape, stride or chunk size");
  const int64_t cblocks = (C + 63) / 64;
  if (n_counters < M * cblocks) return fail("rb_colsum_chunked: too few counters");
  if (M * cblocks * (P / chunk_rows) > 0x7fffffffLL || M * P * rs >= ((int64_t)1 << 40))
    return fail("rb_colsum_chunked: grid too large");
  return launch_colsum_chunked(in, M, P, C, rs, (int)chunk_rows, part,
                               reinterpret_cast<unsigned*>(counters), out,
                               reinterpret_cast<hipStream_t>(stream));
}

int rb_pack_plan(const int64_t* item_seq, int64_t seq_rs, const int64_t* seq_offsets,
                 const int64_t* order, int64_t B, int64_t L, int64_t* ids, int64_t* row_pos,
                 int64_t* inv, int64_t* last, void* stream) {
  if (!item_seq || !seq_offsets || !order || !ids || !row_pos || !inv || !last)
    return fail("rb_pack_plan: null pointer");
  if (B < 1 || L < 1 || seq_rs < L) return fail("rb_pack_plan: bad shape or row stride");
  if ((B + 3) / 4 > 0x7fffffffLL) return fail("rb_pack_plan: grid too large");
  return launch_pack_plan(item_seq, seq_rs, seq_offsets, order, B, ids, row_pos, inv, last,
                          reinterpret_cast<hipStream_t>(stream));
}

int64_t rb_gemm_h_weight_bytes(int64_t C, int64_t R) {
  // + the weight-stationary kernel's planes where it can run (R % 32 == 0)
  return ws_image_offset(C, R) + (R % 32 == 0 ? C * R * 4 : 0);
}
int rb_gemm_nt_h_mode(int mode) { return gemm_nt_h_mode(mode); }

int rb_gemm_nt_h_ln(const float* A, int64_t lda, int64_t M, int64_t R, const void* Wf, int64_t C,
                    const float* bias, const float* resid, const float* gamma, const float* beta,
                    float eps, uint64_t seed, float p, float* y, float* s_out, float* mean,
                    float* rstd, int64_t ldo, float* rmax, void* stream) {
  if (!A || !Wf || !resid || !gamma || !beta || !y || !s_out || !mean || !rstd)
    return fail("rb_gemm_nt_h_ln: null pointer");
  if (M <= 0 || R <= 0 || C != 128) return fail("rb_gemm_nt_h_ln: C must be 128, M and R positive");
  if (R != 128 && R != 256 && R != 512) return fail("rb_gemm_nt_h_ln: R must be 128, 256 or 512");
  if (lda < R || lda % 4 || ldo < C || ldo % 4) return fail("rb_gemm_nt_h_ln: bad row strides");
  if (!aligned16(A) || !aligned16(Wf) || !aligned16(resid) || !aligned16(y) || !aligned16(s_out) ||
      !aligned16(gamma) || !aligned16(beta) || (bias && !aligned16(bias)))
    return fail("rb_gemm_nt_h_ln: A, Wf, resid, y, s_out, gamma, beta and bias must be 16-byte aligned");
  if (!(p >= 0.0f && p < 1.0f)) return fail("rb_gemm_nt_h_ln: dropout p must be in [0, 1)");
  if (!(eps > 0.0f)) return fail("rb_gemm_nt_h_ln: eps must be positive");
  if ((M + 31) / 32 > 0x3fffffffLL) return fail("rb_gemm_nt_h_ln: grid too large");
  if (gemm_nt_h_mode(-1) != 1) return fail("rb_gemm_nt_h_ln: needs the weight-stationary kernel (rb_gemm_nt_h_mode 1)");
  return launch_gemm_nt_ws_ln(A, lda, M, (int)R, Wf, (int)C, bias, resid, make_drop(nullptr, seed, p),
                              gamma, beta, eps, y, s_out, mean, rstd, ldo, rmax,
                              reinterpret_cast<hipStream_t>(stream));
}

int rb_gemm_h_split_weights(const rb_split_job* jobs, int64_t n, void* stream) {
  if (!jobs || n < 1 || n > RB_MAX_SPLIT_JOBS)
    return fail("rb_gemm_h_split_weights: need 1..RB_MAX_SPLIT_JOBS jobs");
  for (int64_t j = 0; j < n; ++j) {
    const rb_split_job& b = jobs[j];
    if (!b.W || !b.Wf) return fail("rb_gemm_h_split_weights: null pointer");
    if (b.C <= 0 || b.R <= 0 || b.C % 32 || b.R % 16 || b.C > (1 << 20) || b.R > (1 << 20))
      return fail("rb_gemm_h_split_weights: C must be a multiple of 32 and R of 16");
    if (b.ldw < (b.transpose ? b.C : b.R)) return fail("rb_gemm_h_split_weights: bad row stride");
    if (!aligned16(b.Wf)) return fail("rb_gemm_h_split_weights: Wf must be 16-byte aligned");
  }
  return launch_split_weights_h(jobs, (int)n, reinterpret_cast<hipStream_t>(stream));
}

int rb_gemm_nt_h(const float* A, int64_t lda, int64_t M, int64_t R, const void* Wf, int64_t C,
                 const float* bias, float* out, int64_t ldo, int accumulate, float* rmax,
                 void* stream) {
  if (!A || !Wf || !out) return fail("rb_gemm_nt_h: null pointer");
  if (M <= 0 || R <= 0 || C <= 0) return fail("rb_gemm_nt_h: empty shape");
  if (accumulate) return fail("rb_gemm_nt_h: accumulate is not supported (add the residual in its consumer)");
  if (R % 32 || C % 32 || R > (1 << 16) || C > 1024)
    return fail("rb_gemm_nt_h: R and C must be multiples of 32 (C <= 1024)");
  if (lda < R || lda % 4 || ldo < C || ldo % 2) return fail("rb_gemm_nt_h: bad row strides");
  if (!aligned16(A) || !aligned16(Wf) || (reinterpret_cast<uintptr_t>(out) & 7))
    return fail("rb_gemm_nt_h: A and Wf must be 16-byte aligned, out 8-byte aligned");
  if ((M + 31) / 32 > 0x7fffffffLL) return fail("rb_gemm_nt_h: grid too large");
  return launch_gemm_nt_h(A, lda, M, (int)R, Wf, (int)C, bias, out, ldo, accumulate, rmax,
                          reinterpret_cast<hipStream_t>(stream));
}

int rb_gemm_nt_h_act(const float* A, int64_t lda, int64_t M, int64_t R, const void* Wf, int64_t C,
                     const float* bias, float* out, int64_t ldo, float* rmax, float* act,
                     uint64_t seed, float p, void* stream) {
  if (!A || !Wf || !out || !act) return fail("rb_gemm_nt_h_act: null pointer");
  if (M <= 0 || R <= 0 || C <= 0) return fail("rb_gemm_nt_h_act: empty shape");
  if (R % 32 || C % 32 || R > 1024 || C > 1024)
    return fail("rb_gemm_nt_h_act: R and C must be multiples of 32 (R, C <= 1024)");
  if (lda < R || lda % 4 || ldo < C || ldo % 4) return fail("rb_gemm_nt_h_act: bad row strides");
  if (!aligned16(A) || !aligned16(Wf) || !aligned16(out) || !aligned16(act) ||
      (bias && !aligned16(bias)))
    return fail("rb_gemm_nt_h_act: A, Wf, out, act and bias must be 16-byte aligned");
  if (!(p >= 0.0f && p < 1.0f)) return fail("rb_gemm_nt_h_act: dropout p must be in [0, 1)");
  if ((M + 31) / 32 > 0x7fffffffLL) return fail("rb_gemm_nt_h_act: grid too large");
  return launch_gemm_nt_h_act(A, lda, M, (int)R, Wf, (int)C, bias, out, ldo, rmax, act,
                              make_drop(nullptr, seed, p), reinterpret_cast<hipStream_t>(stream));
}

int rb_adam_step(const rb_adam_job* jobs, int64_t n, double lr, double beta1, double beta2,
                 double eps, double weight_decay, double bc1, double bc2, void* stream) {
  if (!jobs || n <= 0 || n > RB_MAX_ADAM_JOBS) return fail("rb_adam_step: 1..RB_MAX_ADAM_JOBS jobs");
  int64_t blocks = 0;
  for (int64_t j = 0; j < n; ++j) {
    const rb_adam_job& b = jobs[j];
    if (!b.param || !b.grad || !b.exp_avg || !b.exp_avg_sq || b.n <= 0)
      return fail("rb_adam_step: null pointer or empty tensor");
    if (!aligned16(b.param) || !aligned16(b.grad) || !aligned16(b.exp_avg) ||
        !aligned16(b.exp_avg_sq))
      return fail("rb_adam_step: tensors must be 16-byte aligned");
    blocks += (b.n + 1023) / 1024;
  }
  if (blocks > 0x7fffffffLL) return fail("rb_adam_step: too many elements");
  if (!(bc1 > 0.0 && bc2 > 0.0)) return fail("rb_adam_step: bias corrections must be > 0");
  return launch_adam(jobs, (int)n, lr, beta1, beta2, eps, weight_decay, bc1, bc2,
                     reinterpret_cast<hipStream_t>(stream));
}

int64_t rb_gemm_nt_h_dact_parts(void) { return nt_h_dact_parts(); }

int rb_gemm_nt_h_dact(const float* A, int64_t lda, int64_t M, int64_t R, const void* Wf, int64_t C,
                      float* out, int64_t ldo, float* rmax, const float* pre, uint64_t seed,
                      float p, float* dpart, int64_t n_parts, void* stream) {
  if (!A || !Wf || !out || !pre || !dpart) return fail("rb_gemm_nt_h_dact: null pointer");
  if (M <= 0 || R <= 0 || C <= 0) return fail("rb_gemm_nt_h_dact: empty shape");
  if (R % 32 || C % 32 || R > 1024 || C > 512)
    return fail("rb_gemm_nt_h_dact: R and C must be multiples of 32 (R <= 1024, C <= 512)");
  if (lda < R || lda % 4 || ldo < C || ldo % 4) return fail("rb_gemm_nt_h_dact: bad row strides");
  if (!aligned16(A) || !aligned16(Wf) || !aligned16(out) || !aligned16(pre) || !aligned16(dpart))
    return fail("rb_gemm_nt_h_dact: A, Wf, out, pre and dpart must be 16-byte aligned");
  if (!(p >= 0.0f && p < 1.0f)) return fail("rb_gemm_nt_h_dact: dropout p must be in [0, 1)");
  if ((M + 31) / 32 > 0x7fffffffLL) return fail("rb_gemm_nt_h_dact: grid too large");
  return launch_gemm_nt_h_dact(A, lda, M, (int)R, Wf, (int)C, out, ldo, rmax, pre,
                               make_drop(nullptr, seed, p), dpart, n_parts,
                               reinterpret_cast<hipStream_t>(stream));
}

int rb_gemm_tn_h(const float* dY, int64_t ldy, const float* X, int64_t ldx, int64_t M, int64_t N,
                 int64_t K, const float* ymax, const float* xmax, float* parts, int64_t splits,
                 void* stream) {
  if (!dY || !X || !ymax || !xmax || !parts) return fail("rb_gemm_tn_h: null pointer");
  if (M <= 0 || N <= 0 || K <= 0) return fail("rb_gemm_tn_h: empty shape");
  if (N % 128 || K % 128 || N > 65536 || K > 65536)
    return fail("rb_gemm_tn_h: N and K must be multiples of 128 (<= 65536)");
  if (splits < 1 || splits > 65536) return fail("rb_gemm_tn_h: splits must be in [1, 65536]");
  if (ldy < N || ldx < K || ldy % 4 || ldx % 4) return fail("rb_gemm_tn_h: bad row strides");
  if (!aligned16(dY) || !aligned16(X)) return fail("rb_gemm_tn_h: dY and X must be 16-byte aligned");
  if ((N / 128) * (K / 128) * splits > 0x7fffffffLL) return fail("rb_gemm_tn_h: grid too large");
  // the kernel reads a row chunk through a buffer descriptor: 32-bit record
  // count and lane offsets over the chunk's bytes (launch_gemm_tn_h's chunk)
  const int64_t mk = ((M + splits - 1) / splits + 31) / 32 * 32;
  if (mk * (ldy > ldx ? ldy : ldx) * 4 >= 0x7fffffffLL)
    return fail("rb_gemm_tn_h: a row chunk spans 2 GiB or more (use more splits)");
  return launch_gemm_tn_h(dY, ldy, X, ldx, M, (int)N, (int)K, ymax, xmax, parts, (int)splits,
                          reinterpret_cast<hipStream_t>(stream));
}

int rb_gemm_bf16_weight_image(const float* W, int64_t ldw, int64_t C, int64_t R, int transpose,
                              void* img, void* stream) {
  if (!W || !img) return fail("rb_gemm_bf16_weight_image: null pointer");
  if (C <= 0 || R <= 0 || C % 16 || R % 32 || C > 65536 || R > 65536)
    return fail("rb_gemm_bf16_weight_image: C % 16 == 0 and R % 32 == 0 required (<= 65536)");
  if (ldw < (transpose ? C : R)) return fail("rb_gemm_bf16_weight_image: bad row stride");
  if (!aligned16(img)) return fail("rb_gemm_bf16_weight_image: img must be 16-byte aligned");
  return launch_bf16_weight_image(W, ldw, (int)C, (int)R, transpose ? 1 : 0, img,
                                  reinterpret_cast<hipStream_t>(stream));
}

int rb_gemm_nt_bf16(const void* A, int64_t lda, int64_t M, int64_t R, const void* img, int64_t C,
                    const float* bias, void* out, int64_t ldo, void* stream) {
  if (!A || !img || !out) return fail("rb_gemm_nt_bf16: null pointer");
  if (M <= 0 || R <= 0 || C <= 0) return fail("rb_gemm_nt_bf16: empty shape");
  if (R % 64 || C % 256 || R > 16384 || C > 65536)
    return fail("rb_gemm_nt_bf16: R % 64 == 0 (<= 16384) and C % 256 == 0 required");
  if (lda < R || lda % 8 || lda > (1 << 20) || ldo < C || ldo % 8)
    return fail("rb_gemm_nt_bf16: bad row strides (lda % 8 == 0, ldo % 8 == 0)");
  if (!aligned16(A) || !aligned16(img) || !aligned16(out) || (bias && !aligned16(bias)))
    return fail("rb_gemm_nt_bf16: A, img, out and bias must be 16-byte aligned");
  if ((M + 255) / 256 > 0x7fffffffLL / (C / 256) / 2) return fail("rb_gemm_nt_bf16: too many tiles");
  return launch_gemm_nt_bf16(A, lda, M, (int)R, img, (int)C, bias, out, ldo,
                             reinterpret_cast<hipStream_t>(stream));
}

int rb_gemm_tn_hs(const float* dY, int64_t ldy, const float* X, int64_t ldx, int64_t M, int64_t N,
                  int64_t K, float* dw, int accumulate, void* stream) {
  if (!dY || !X || !dw) return fail("rb_gemm_tn_hs: null pointer");
  if (M <= 0 || N <= 0 || K <= 0) return fail("rb_gemm_tn_hs: empty shape");
  if (N % 32 || K % 32 || N > 65536 || K > 65536)
    return fail("rb_gemm_tn_hs: N and K must be multiples of 32");
  if (M > (1 << 24)) return fail("rb_gemm_tn_hs: M too large for the few-rows kernel");
  if (ldy < N || ldx < K) return fail("rb_gemm_tn_hs: bad row strides");
  return launch_gemm_tn_hs(dY, ldy, X, ldx, M, (int)N, (int)K, dw, accumulate,
                           reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
