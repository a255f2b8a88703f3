// probe_capi.hip — the extern "C" entry points of the probe library
// (recblr_probe.h): argument checks, then the launchers in probe.hip.  The
// library is built with hidden visibility, so its error helpers (rb::fail,
// rb::launch_status) are its own and never interpose the product library's.
#include "../csrc/common.h"
#include "recblr_probe.h"

#include <algorithm>
#include <string>

namespace rb {

namespace {
thread_local std::string g_probe_error;

int64_t max4(int64_t a, int64_t b, int64_t c = 0, int64_t d = 0) {
  return std::max(std::max(a, b), std::max(c, d));
}

int check_dims(int64_t B, int64_t L, int64_t H, int64_t max_rs) {
  if (B <= 0 || L <= 0 || H <= 0) return fail("B, L and H must be positive");
  if (L * max_rs + max_rs >= (int64_t(1) << 31)) return fail("L * row_stride exceeds 2^31");
  if (B * ((H + 15) / 16) / 4 + 1 > 0x7fffffffLL) return fail("grid too large");
  return 0;
}
}  // namespace

int fail(const char* msg) {
  g_probe_error = msg;
  return RB_EINVAL;
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_probe_error = std::string(what) + ": " + hipGetErrorString(e);
    return static_cast<int>(e);
  }
  return 0;
}

int launch_probe_gemm_pattern(const float* A, int64_t M, int64_t R, float* out, int64_t C,
                              hipStream_t st);
int launch_probe_gate_bwd_pattern(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                                  const float* z, int64_t z_rs, const float* dy, float* drg,
                                  int64_t drg_rs, float* dxc, int64_t dxc_rs, float* dz,
                                  int64_t dz_rs, int64_t B, int64_t L, int64_t H,
                                  const int64_t* offs, hipStream_t st);
}  // namespace rb

using namespace rb;

extern "C" {

__attribute__((visibility("default"))) const char* rb_probe_last_error_string(void) {
  return g_probe_error.c_str();
}

__attribute__((visibility("default"))) int rb_probe_gemm_pattern(const float* a, int64_t M,
                                                                 int64_t R, float* out, int64_t C,
                                                                 void* stream) {
  if (!a || !out) return fail("rb_probe_gemm_pattern: null pointer");
  if (M <= 0 || R <= 0 || C <= 0 || R % 4 || C % 4 || R > (1 << 20) || C > (1 << 20))
    return fail("rb_probe_gemm_pattern: M, R, C must be positive, R and C multiples of 4");
  if (!aligned16(a) || !aligned16(out))
    return fail("rb_probe_gemm_pattern: operands must be 16-B aligned");
  return launch_probe_gemm_pattern(a, M, R, out, C, reinterpret_cast<hipStream_t>(stream));
}

__attribute__((visibility("default"))) int rb_probe_gate_bwd_pattern(
    const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs, const float* z, int64_t z_rs,
    const float* dy, float* drg, int64_t drg_rs, float* dxc, int64_t dxc_rs, float* dz,
    int64_t dz_rs, int64_t B, int64_t L, int64_t H, const int64_t* seq_offsets, void* stream) {
  if (!rg || !xc || !z || !dy || !drg || !dxc || !dz)
    return fail("rb_probe_gate_bwd_pattern: null pointer");
  if (rg_rs < 2 * H || xc_rs < H || z_rs < H || drg_rs < 2 * H || dxc_rs < H || dz_rs < H)
    return fail("rb_probe_gate_bwd_pattern: row stride too small");
  if (H % 4 || rg_rs % 4 || xc_rs % 4 || z_rs % 4 || drg_rs % 4 || dxc_rs % 4 || dz_rs % 4 ||
      !aligned16(rg) || !aligned16(xc) || !aligned16(z) || !aligned16(dy) || !aligned16(drg) ||
      !aligned16(dxc) || !aligned16(dz))
    return fail("rb_probe_gate_bwd_pattern: 16-B aligned rows of a multiple of 4 floats only");
  if (int r = check_dims(B, L, H, max4(max4(rg_rs, xc_rs, z_rs, drg_rs), dz_rs, dxc_rs, H)))
    return r;
  return launch_probe_gate_bwd_pattern(rg, rg_rs, xc, xc_rs, z, z_rs, dy, drg, drg_rs, dxc, dxc_rs,
                                       dz, dz_rs, B, L, H, seq_offsets,
                                       reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
