// exp_capi.hip — the extern "C" entry points of the experimental library
// (recblr_exp.h): argument checks, then the launchers in grl_fused.hip.
// Built with hidden visibility, so its error helpers (rb::fail,
// rb::launch_status, rb::num_cus) are its own and never interpose the
// product library's.
#include "../csrc/common.h"
#include "recblr_exp.h"

#include <atomic>
#include <string>

namespace rb {

namespace {
thread_local std::string g_exp_error;
}

int fail(const char* msg) {
  g_exp_error = msg;
  return RB_EINVAL;
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_exp_error = std::string(what) + ": " + hipGetErrorString(e);
    return static_cast<int>(e);
  }
  return 0;
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

int launch_grl_fwd(const float* xz, int64_t xz_rs, const float* conv_w, int KC,
                   const float* conv_b, const void* wf, const float* gate_b, const float* lam,
                   const float* h0, const int* pieces, int64_t B, int64_t G, int64_t ntok,
                   float* y, int64_t y_rs, float* y_last, float* xc_out, float* rg_out,
                   float* carries, int64_t nTc, float* xc_rmax, float* tile_carries,
                   int64_t max_tiles, hipStream_t st);
int launch_grl_bwd(const float* xz, int64_t xz_rs, const float* conv_w, int KC,
                   const float* conv_b, const void* wf, const void* wft, const float* gate_b,
                   const float* lam, const float* h0, const int* pieces, int64_t B, int64_t G,
                   int64_t ntok, const float* tile_carries, int64_t max_tiles, const float* dy,
                   const float* dy_last, float* dxz, int64_t dxz_rs, float* drg, float* xc_out,
                   float* drg_rmax, float* xc_rmax, float* part, float* cpart, hipStream_t st);
}  // namespace rb

using namespace rb;

namespace {
constexpr int RB_EXP_ABI = 44;   // = the product library's rb_version() it pairs with
}  // namespace

extern "C" {

#define RB_EXPORT __attribute__((visibility("default")))

RB_EXPORT int rb_exp_version(void) { return RB_EXP_ABI; }

RB_EXPORT const char* rb_exp_last_error_string(void) { return g_exp_error.c_str(); }

RB_EXPORT int rb_grl_fwd(const float* xz, int64_t xz_rs, const float* conv_w, int64_t kc,
               const float* conv_b, const void* wg_img, const float* gate_b, const float* lam,
               const float* h0, const int32_t* pieces, int64_t B, int64_t G, int64_t ntok,
               int64_t H, float* y, int64_t y_rs, float* y_last, float* xc, float* rg,
               float* carries, int64_t n_tiles, float* xc_rmax, float* tile_carries,
               int64_t max_tiles, void* stream) {
  if (!xz || !conv_w || !conv_b || !wg_img || !gate_b || !lam || !pieces)
    return fail("rb_grl_fwd: null pointer");
  if (tile_carries && (max_tiles <= 0 || G * max_tiles * H >= (1LL << 40)))
    return fail("rb_grl_fwd: tile_carries need max_tiles");
  if (H != 256) return fail("rb_grl_fwd: the fused kernel is built for H = 256");
  if (kc < 2 || kc > 4) return fail("rb_grl_fwd: conv kernel size must be 2, 3 or 4");
  if (B <= 0 || G <= 0 || ntok <= 0 || ntok >= (1LL << 31) || G > (1 << 20))
    return fail("rb_grl_fwd: bad sizes");
  if (!y == !y_last) return fail("rb_grl_fwd: exactly one of y / y_last");
  if (xz_rs < 2 * H || xz_rs % 4 || !aligned16(xz)) return fail("rb_grl_fwd: xz layout");
  if (y && (y_rs < H || y_rs % 4 || !aligned16(y))) return fail("rb_grl_fwd: y layout");
  if (ntok * (y && y_rs > xz_rs ? y_rs : xz_rs) >= (1LL << 31))   // 32-bit element offsets
    return fail("rb_grl_fwd: ntok * row stride must be < 2^31");
  if (carries && n_tiles <= 0) return fail("rb_grl_fwd: carries need n_tiles");
  if ((xc && !aligned16(xc)) || !aligned16(wg_img)) return fail("rb_grl_fwd: alignment");
  return launch_grl_fwd(xz, xz_rs, conv_w, (int)kc, conv_b, wg_img, gate_b, lam, h0,
                        reinterpret_cast<const int*>(pieces), B, G, ntok, y, y_rs, y_last, xc,
                        rg, carries, n_tiles, xc_rmax, tile_carries, max_tiles,
                        reinterpret_cast<hipStream_t>(stream));
}

RB_EXPORT int rb_grl_bwd(const float* xz, int64_t xz_rs, const float* conv_w, int64_t kc,
               const float* conv_b, const void* wg_img, const void* wgt_img, const float* gate_b,
               const float* lam, const float* h0, const int32_t* pieces, int64_t B, int64_t G,
               int64_t ntok, int64_t H, const float* tile_carries, int64_t max_tiles,
               const float* dy, const float* dy_last, float* dxz, int64_t dxz_rs, float* drg,
               float* xc, float* drg_rmax, float* xc_rmax, float* part, float* cpart,
               void* stream) {
  if (!xz || !conv_w || !conv_b || !wg_img || !wgt_img || !gate_b || !lam || !pieces ||
      !tile_carries || !dxz || !drg || !xc || !part || !cpart)
    return fail("rb_grl_bwd: null pointer");
  if (H != 256) return fail("rb_grl_bwd: the fused kernel is built for H = 256");
  if (kc < 2 || kc > 4) return fail("rb_grl_bwd: conv kernel size must be 2, 3 or 4");
  if (B <= 0 || G <= 0 || ntok <= 0 || G > (1 << 20) || max_tiles <= 0)
    return fail("rb_grl_bwd: bad sizes");
  if (!dy == !dy_last) return fail("rb_grl_bwd: exactly one of dy / dy_last");
  if (xz_rs < 2 * H || xz_rs % 4 || !aligned16(xz)) return fail("rb_grl_bwd: xz layout");
  if (dxz_rs < 2 * H || dxz_rs % 4 || !aligned16(dxz)) return fail("rb_grl_bwd: dxz layout");
  // 32-bit element offsets inside the kernel
  if (ntok * (xz_rs > dxz_rs ? xz_rs : dxz_rs) >= (1LL << 31))
    return fail("rb_grl_bwd: ntok * row stride must be < 2^31");
  if (!aligned16(xc) || !aligned16(wg_img) || !aligned16(wgt_img))
    return fail("rb_grl_bwd: alignment");
  return launch_grl_bwd(xz, xz_rs, conv_w, (int)kc, conv_b, wg_img, wgt_img, gate_b, lam, h0,
                        reinterpret_cast<const int*>(pieces), B, G, ntok, tile_carries,
                        max_tiles, dy, dy_last, dxz, dxz_rs, drg, xc, drg_rmax, xc_rmax, part,
                        cpart, reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
