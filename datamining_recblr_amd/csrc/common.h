// common.h — shared device helpers for the RecBLR gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/recblr_hip.h"

namespace rb {

constexpr int kWave = 64;

// ---- error reporting (host) -------------------------------------------------
int fail(const char* msg);
int launch_status(const char* what);
// compute units of the current device (cached per device)
int num_cus();

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ---- scalar math, following torch's definitions ------------------------------
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }
// torch.nn.functional.softplus(beta=1, threshold=20)
__device__ __forceinline__ float softplus_f(float x) { return x > 20.0f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float dsoftplus_f(float x) { return x > 20.0f ? 1.0f : sigm(x); }
__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }
// d/dx silu(x) = s (1 + x (1 - s)), s = sigmoid(x)
__device__ __forceinline__ float dsilu_f(float x) {
  const float s = sigm(x);
  return s * (1.0f + x * (1.0f - s));
}

// ---- hardware transcendentals (v_exp_f32 / v_rcp_f32 / v_sqrt_f32, ~1 ulp) ----
// The libm forms above expand to ~10-15 instructions each (range reduction,
// IEEE division); in the [B, L, H] kernels they made the VALU co-bound with
// HBM.  The native forms keep every quantity within a few ulp, which stays
// far inside the 1e-4 parity budget: the one cancellation-prone value,
// 1 - alpha^2 with alpha -> 0.999, depends on alpha's absolute error (~ulp(1))
// exactly as it does with expf.
constexpr float kLog2e = 1.4426950408889634f;
__device__ __forceinline__ float fexp(float x) { return __builtin_amdgcn_exp2f(x * kLog2e); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float fsigm(float x) { return frcp(1.0f + fexp(-x)); }
__device__ __forceinline__ float fsilu(float x) { return x * fsigm(x); }
__device__ __forceinline__ float fdsilu(float x) {
  const float s = fsigm(x);
  return s * (1.0f + x * (1.0f - s));
}

// ---- VEC-wide loads/stores (VEC = 4 -> one 16-B access per lane) -------------
// Every [B, L, H] stream is read or written once per kernel, so the accesses
// carry the nontemporal hint (global_load/store ... nt): on this chip a plain
// 1R+1W float4 copy runs at 0.76 of 8 TB/s with default-policy accesses and
// 0.83 with nt ones (tools/copyprobe2.hip, profiles/r01_copyprobe2.log).
typedef float rb_f32x4 __attribute__((ext_vector_type(4)));
typedef float rb_f32x2v __attribute__((ext_vector_type(2)));
typedef uint32_t rb_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t rb_u32x2 __attribute__((ext_vector_type(2)));

template <bool NT, typename T>
__device__ __forceinline__ T ld_pol(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st_pol(T v, T* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
constexpr bool kNT = true;

// ldv / stv: once-touched activation streams (nt); ldc / stc: default policy,
// for small operands many workgroups re-read (parameters, carries) and for
// inputs that neighbouring tiles re-read (the conv's halo rows).
template <bool NT, int V>
__device__ __forceinline__ void ld_f32(float (&o)[V], const float* p) {
  if constexpr (V == 4) {
    const rb_f32x4 t = ld_pol<NT>(reinterpret_cast<const rb_f32x4*>(p));
    o[0] = t[0]; o[1] = t[1]; o[2] = t[2]; o[3] = t[3];
  } else if constexpr (V == 2) {
    const rb_f32x2v t = ld_pol<NT>(reinterpret_cast<const rb_f32x2v*>(p));
    o[0] = t[0]; o[1] = t[1];
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) o[v] = ld_pol<NT>(p + v);
  }
}

template <bool NT, int V>
__device__ __forceinline__ void st_f32(float* p, const float (&o)[V]) {
  if constexpr (V == 4) {
    st_pol<NT>(rb_f32x4{o[0], o[1], o[2], o[3]}, reinterpret_cast<rb_f32x4*>(p));
  } else if constexpr (V == 2) {
    st_pol<NT>(rb_f32x2v{o[0], o[1]}, reinterpret_cast<rb_f32x2v*>(p));
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) st_pol<NT>(o[v], p + v);
  }
}

template <int V>
__device__ __forceinline__ void ldv(float (&o)[V], const float* p) { ld_f32<kNT>(o, p); }
template <int V>
__device__ __forceinline__ void stv(float* p, const float (&o)[V]) { st_f32<kNT>(p, o); }
template <int V>
__device__ __forceinline__ void ldc(float (&o)[V], const float* p) { ld_f32<false>(o, p); }
template <int V>
__device__ __forceinline__ void stc(float* p, const float (&o)[V]) { st_f32<false>(p, o); }

// ---- bf16 storage (fp32 arithmetic): VEC bf16 per lane, RNE on store ---------
typedef __bf16 bf16_t;
typedef __bf16 rb_bf16x2 __attribute__((ext_vector_type(2)));
typedef float rb_f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void unpack2(uint32_t u, float& a, float& b) {
  a = __uint_as_float(u << 16);
  b = __uint_as_float(u & 0xffff0000u);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(rb_f32x2{a, b}, rb_bf16x2));
}

template <bool NT, int V>
__device__ __forceinline__ void ld_b16(float (&o)[V], const bf16_t* p) {
  if constexpr (V == 8) {
    const rb_u32x4 t = ld_pol<NT>(reinterpret_cast<const rb_u32x4*>(p));
    unpack2(t[0], o[0], o[1]); unpack2(t[1], o[2], o[3]);
    unpack2(t[2], o[4], o[5]); unpack2(t[3], o[6], o[7]);
  } else if constexpr (V == 4) {
    const rb_u32x2 t = ld_pol<NT>(reinterpret_cast<const rb_u32x2*>(p));
    unpack2(t[0], o[0], o[1]); unpack2(t[1], o[2], o[3]);
  } else if constexpr (V == 2) {
    unpack2(ld_pol<NT>(reinterpret_cast<const uint32_t*>(p)), o[0], o[1]);
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) o[v] = (float)p[v];
  }
}

template <bool NT, int V>
__device__ __forceinline__ void st_b16(bf16_t* p, const float (&o)[V]) {
  if constexpr (V == 8) {
    st_pol<NT>(rb_u32x4{pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7])},
               reinterpret_cast<rb_u32x4*>(p));
  } else if constexpr (V == 4) {
    st_pol<NT>(rb_u32x2{pack2(o[0], o[1]), pack2(o[2], o[3])}, reinterpret_cast<rb_u32x2*>(p));
  } else if constexpr (V == 2) {
    st_pol<NT>(pack2(o[0], o[1]), reinterpret_cast<uint32_t*>(p));
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) p[v] = (bf16_t)o[v];
  }
}

template <int V>
__device__ __forceinline__ void ldv(float (&o)[V], const bf16_t* p) { ld_b16<kNT>(o, p); }
template <int V>
__device__ __forceinline__ void stv(bf16_t* p, const float (&o)[V]) { st_b16<kNT>(p, o); }
template <int V>
__device__ __forceinline__ void ldc(float (&o)[V], const bf16_t* p) { ld_b16<false>(o, p); }
template <int V>
__device__ __forceinline__ void stc(bf16_t* p, const float (&o)[V]) { st_b16<false>(p, o); }

// raw (storage-format) register image of V elements: fp32 as is, bf16 as
// packed pairs, unpacked to fp32 only when used (prefetch buffers)
template <typename T, int V>
struct RawVec {
  float w[V];
};
template <int V>
struct RawVec<bf16_t, V> {
  static_assert(V % 2 == 0, "packed bf16 needs an even width");
  uint32_t w[V / 2];
};
template <>
struct RawVec<bf16_t, 1> {
  float w[1];
};

template <bool NT = kNT, int V>
__device__ __forceinline__ void ld_raw(RawVec<float, V>& o, const float* p) { ld_f32<NT>(o.w, p); }
template <int V>
__device__ __forceinline__ void unpack_raw(float (&o)[V], const RawVec<float, V>& r) {
#pragma unroll
  for (int v = 0; v < V; ++v) o[v] = r.w[v];
}
template <typename T, int V>
__device__ __forceinline__ void zero_raw(RawVec<T, V>& o) {
#pragma unroll
  for (int k = 0; k < (int)(sizeof(o.w) / sizeof(o.w[0])); ++k) o.w[k] = 0;
}

template <bool NT = kNT, int V>
__device__ __forceinline__ void ld_raw(RawVec<bf16_t, V>& o, const bf16_t* p) {
  if constexpr (V == 8) {
    const rb_u32x4 t = ld_pol<NT>(reinterpret_cast<const rb_u32x4*>(p));
    o.w[0] = t[0]; o.w[1] = t[1]; o.w[2] = t[2]; o.w[3] = t[3];
  } else if constexpr (V == 4) {
    const rb_u32x2 t = ld_pol<NT>(reinterpret_cast<const rb_u32x2*>(p));
    o.w[0] = t[0]; o.w[1] = t[1];
  } else if constexpr (V == 2) {
    o.w[0] = ld_pol<NT>(reinterpret_cast<const uint32_t*>(p));
  } else {
    o.w[0] = (float)p[0];
  }
}
template <int V>
__device__ __forceinline__ void unpack_raw(float (&o)[V], const RawVec<bf16_t, V>& r) {
  if constexpr (V == 1) {
    o[0] = r.w[0];
  } else {
#pragma unroll
    for (int k = 0; k < V / 2; ++k) unpack2(r.w[k], o[2 * k], o[2 * k + 1]);
  }
}

// channels h0 .. h0 + VH - 1 of a raw image (h0 even for packed bf16), and
// the reverse: VH results into a storage-format image (bf16: RNE pairs, as
// stv); stv_raw stores a whole image with stv's policy
template <int VH, typename T, int V>
__device__ __forceinline__ void unpack_part(float (&o)[VH], const RawVec<T, V>& r, int h0) {
  if constexpr (VH == V) {
    unpack_raw(o, r);
  } else if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int v = 0; v < VH; ++v) o[v] = r.w[h0 + v];
  } else {
#pragma unroll
    for (int k = 0; k < VH / 2; ++k) unpack2(r.w[h0 / 2 + k], o[2 * k], o[2 * k + 1]);
  }
}
template <int VH, typename T, int V>
__device__ __forceinline__ void pack_part(RawVec<T, V>& r, const float (&o)[VH], int h0) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int v = 0; v < VH; ++v) r.w[h0 + v] = o[v];
  } else {
    static_assert(VH % 2 == 0, "packed bf16 pairs");
#pragma unroll
    for (int k = 0; k < VH / 2; ++k) r.w[h0 / 2 + k] = pack2(o[2 * k], o[2 * k + 1]);
  }
}
// the words of channels h0 .. h0 + VH - 1 through an empty volatile asm (an
// ordering point for the compiler; no instruction)
template <int VH, typename T, int V>
__device__ __forceinline__ void opaque_part(RawVec<T, V>& r, int h0) {
  constexpr int per = sizeof(T) == 2 && V > 1 ? 2 : 1;   // channels per word
#pragma unroll
  for (int k = 0; k < VH / per; ++k) asm volatile("" : "+v"(r.w[h0 / per + k]));
}
template <int V>
__device__ __forceinline__ void stv_raw(float* p, const RawVec<float, V>& r) { st_f32<kNT>(p, r.w); }
template <int V>
__device__ __forceinline__ void stv_raw(bf16_t* p, const RawVec<bf16_t, V>& r) {
  if constexpr (V == 8) {
    st_pol<kNT>(rb_u32x4{r.w[0], r.w[1], r.w[2], r.w[3]}, reinterpret_cast<rb_u32x4*>(p));
  } else if constexpr (V == 4) {
    st_pol<kNT>(rb_u32x2{r.w[0], r.w[1]}, reinterpret_cast<rb_u32x2*>(p));
  } else {
    static_assert(V == 2, "packed bf16 image");
    st_pol<kNT>(r.w[0], reinterpret_cast<uint32_t*>(p));
  }
}

// ---- dropout keep-flags ------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11): counter = element index / 4, key =
// 64-bit seed, 4 uniform u32 per call -> keep flags of 4 consecutive elements.
// (each round's two 32 x 32 -> 64 products as one v_mad_u64_u32 each, not a
// v_mul_lo_u32 + v_mul_hi_u32 pair: the same bits in half the quarter-rate
// instructions — the dropout epilogues are bound by this VALU work)
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Dropout of one tensor: no-op, an explicit uint8 keep-mask laid out like the
// data, or a Philox stream regenerated on demand (forward and backward see
// the same flags for the same element index).  mode is launch-uniform.
struct DropSpec {
  const uint8_t* mask;
  uint32_t key0, key1, keep_thresh;
  float scale;
  int mode;   // 0 none, 1 mask, 2 philox

  // multipliers (0 or scale) for elements e .. e+3, e % 4 == 0
  __device__ __forceinline__ void get4(int64_t e, float (&m)[4]) const {
    if (mode == 0) {
      m[0] = m[1] = m[2] = m[3] = 1.0f;
    } else if (mode == 1) {
      const uchar4 t = *reinterpret_cast<const uchar4*>(mask + e);
      m[0] = t.x * scale; m[1] = t.y * scale; m[2] = t.z * scale; m[3] = t.w * scale;
    } else {
      const uint64_t g = (uint64_t)e >> 2;
      const uint4 r = philox4x32_10(make_uint4((uint32_t)g, (uint32_t)(g >> 32), 0u, 0u), key0,
                                    key1);
      m[0] = r.x < keep_thresh ? scale : 0.0f;
      m[1] = r.y < keep_thresh ? scale : 0.0f;
      m[2] = r.z < keep_thresh ? scale : 0.0f;
      m[3] = r.w < keep_thresh ? scale : 0.0f;
    }
  }
};

DropSpec make_drop(const uint8_t* mask, uint64_t seed, float p);

// ---- channel-last wave layout ---------------------------------------------------
// The [B, L, H] kernels give each wave one batch row b and a span of G*VEC
// channels.  Lane = q * G + g: g picks VEC consecutive channels (so the G lanes
// of one chunk read one contiguous G*VEC*4-byte segment of a row), q picks one
// of Q consecutive time chunks of TC steps inside a tile of Q*TC steps.
// Summaries of the Q chunks are combined across lanes with shuffles at stride
// G; no LDS and no barriers.

// host launch helpers (defined in the .hip files)
int launch_pack_plan(const int64_t* seq, int64_t seq_rs, const int64_t* offs,
                     const int64_t* order, int64_t B, int64_t* ids, int64_t* pos, int64_t* inv,
                     int64_t* last, hipStream_t st);
int launch_conv_fwd(const float* x, int64_t x_rs, const float* w, const float* bias, float* xc,
                    int64_t xc_rs, int64_t B, int64_t L, int64_t H, int64_t K, const int64_t* offs, hipStream_t st);
int launch_conv_bwd(const float* x, int64_t x_rs, const float* w, const float* bias,
                    const float* g1, const float* g2, float* dx, int64_t dx_rs, float* dw_part,
                    float* db_part, int64_t B, int64_t L, int64_t H, int64_t K, const int64_t* offs, hipStream_t st);
int launch_gate_fwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                    const float* z, int64_t z_rs, const float* lam, const float* gb,
                    const float* h0, int64_t h0_bs, float* y, int64_t y_rs, float* carries,
                    int64_t B, int64_t L, int64_t H, const int64_t* offs, hipStream_t st,
                    float* y_last = nullptr, const int64_t* order = nullptr);
int launch_gate_bwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                    const float* z, int64_t z_rs, const float* lam, const float* gb,
                    const float* carries, const float* dy, float* drg, int64_t drg_rs, float* dxc,
                    int64_t dxc_rs, float* dz, int64_t dz_rs, float* part, float* dh0_part,
                    int64_t B, int64_t L, int64_t H, const int64_t* offs, hipStream_t st,
                    const float* dy_last = nullptr, const int64_t* order = nullptr);
int launch_scan_fwd_bf16(const bf16_t* gates, const bf16_t* tokens, bf16_t* states,
                         int64_t rows, int64_t T, hipStream_t st);
int launch_scan_bwd_bf16(const bf16_t* gates, const bf16_t* states, const bf16_t* grad,
                         bf16_t* d_gates, bf16_t* d_tokens, int64_t rows, int64_t T,
                         hipStream_t st);
int launch_conv_fwd_rows(const float* x, int64_t x_rs, const float* w, const float* bias,
                         float* xc, int64_t xc_rs, int64_t ntok, int64_t H, int64_t K,
                         const int64_t* pos, hipStream_t st);
int launch_conv_fwd_rows_bf16(const bf16_t* x, int64_t x_rs, const float* w, const float* bias,
                              bf16_t* xc, int64_t xc_rs, int64_t ntok, int64_t H, int64_t K,
                              const int64_t* pos, hipStream_t st);
int launch_conv_fwd_bf16(const bf16_t* x, int64_t x_rs, const float* w, const float* bias,
                         bf16_t* xc, int64_t xc_rs, int64_t B, int64_t L, int64_t H, int64_t K,
                         const int64_t* offs, hipStream_t st);
int launch_conv_bwd_bf16(const bf16_t* x, int64_t x_rs, const float* w, const float* bias,
                         const bf16_t* g1, const bf16_t* g2, bf16_t* dx, int64_t dx_rs,
                         float* dw_part, float* db_part, int64_t B, int64_t L, int64_t H,
                         int64_t K, const int64_t* offs, hipStream_t st);
int launch_gate_fwd_bf16(const bf16_t* rg, int64_t rg_rs, const bf16_t* xc, int64_t xc_rs,
                         const bf16_t* z, int64_t z_rs, const float* lam, const float* gb,
                         const float* h0, int64_t h0_bs, bf16_t* y, int64_t y_rs, float* carries,
                         int64_t B, int64_t L, int64_t H, const int64_t* offs, hipStream_t st);
int launch_gate_bwd_bf16(const bf16_t* rg, int64_t rg_rs, const bf16_t* xc, int64_t xc_rs,
                         const bf16_t* z, int64_t z_rs, const float* lam, const float* gb,
                         const float* carries, const bf16_t* dy, bf16_t* drg, int64_t drg_rs,
                         bf16_t* dxc, int64_t dxc_rs, bf16_t* dz, int64_t dz_rs, float* part,
                         float* dh0_part, int64_t B, int64_t L, int64_t H, const int64_t* offs, hipStream_t st);
int launch_add_ln_fwd(const float* a, const int64_t* idx, int64_t nidx, const DropSpec& drop,
                      const float* r, const float* gamma, const float* beta, float eps, float* y,
                      float* s_out, float* mean, float* rstd, int64_t rows, int64_t d,
                      hipStream_t st);
int launch_add_ln_bwd(const float* dy, const float* dy2, const float* s, const float* gamma,
                      const float* mean, const float* rstd, const DropSpec& drop, float* ds,
                      float* da, float* dgp, float* dbp, float* dbiasp, int64_t nparts,
                      int64_t rows, int64_t d, hipStream_t st);
int64_t ln_num_parts(int64_t rows, int64_t d);
int launch_silu_dropout_fwd(const float* a, const float* bias, const DropSpec& drop, float* u,
                            int64_t rows, int64_t cols, hipStream_t st);
int launch_silu_dropout_bwd(const float* a, const float* bias, const DropSpec& drop,
                            const float* du, float* da, float* dbias_part, int64_t nparts,
                            int64_t rows, int64_t cols, hipStream_t st);
int launch_dropout_mask(const DropSpec& drop, uint8_t* out, int64_t n, hipStream_t st);
int launch_split_weights_h(const rb_split_job* jobs, int n, hipStream_t st);
int launch_bf16_weight_image(const float* W, int64_t ldw, int C, int R, int transpose, void* img,
                             hipStream_t st);
int launch_gemm_nt_bf16(const void* A, int64_t lda, int64_t M, int R, const void* img, int C,
                        const float* bias, void* out, int64_t ldo, hipStream_t st);
int launch_gemm_tn_h(const float* Y, int64_t ldy, const float* X, int64_t ldx, int64_t M, int N,
                     int K, const float* ymax, const float* xmax, float* parts, int S,
                     hipStream_t st);
// byte offset of the weight-stationary kernel's planes inside an f16 weight
// image of Bm [C, K] (after the persistent kernel's planes and the exponents)
__host__ __device__ inline int64_t ws_image_offset(int64_t C, int64_t K) {
  return C * K * 4 + ((C * 4 + 15) / 16) * 16;
}
bool nt_ws_ok(int64_t M, int K, int C, const float* A, int64_t lda, const float* out, int64_t ldo);
int launch_gemm_nt_ws(const float* A, int64_t lda, int64_t M, int K, const void* Wf, int C,
                      const float* bias, float* out, int64_t ldo, float* rmax, hipStream_t st);
int gemm_nt_h_mode(int mode);
bool nt_ws_act_ok(int64_t M, int K, int C, const float* A, int64_t lda, const float* out,
                  const float* other, int64_t ldo);
int launch_gemm_nt_ws_act(const float* A, int64_t lda, int64_t M, int K, const void* Wf, int C,
                          const float* bias, float* out, int64_t ldo, float* rmax, float* act,
                          DropSpec drop, hipStream_t st);
int launch_gemm_nt_ws_dact(const float* A, int64_t lda, int64_t M, int K, const void* Wf, int C,
                           float* out, int64_t ldo, float* rmax, const float* pre, DropSpec drop,
                           float* dpart, int64_t n_parts, hipStream_t st);
bool nt_ws_ln_ok(int64_t M, int K, int C, const float* A, int64_t lda, const float* y,
                 const float* s_out, const float* resid, int64_t ldo);
int launch_gemm_nt_ws_ln(const float* A, int64_t lda, int64_t M, int K, const void* Wf, int C,
                         const float* bias, const float* resid, DropSpec drop, const float* gamma,
                         const float* beta, float eps, float* y, float* s_out, float* mean,
                         float* rstd, int64_t ldo, float* rmax, hipStream_t st);
int launch_gemm_nt_h(const float* A, int64_t lda, int64_t M, int R, const void* Wf, int C,
                     const float* bias, float* out, int64_t ldo, int accumulate, float* rmax,
                     hipStream_t st);
int launch_gemm_nt_h_act(const float* A, int64_t lda, int64_t M, int R, const void* Wf, int C,
                         const float* bias, float* out, int64_t ldo, float* rmax, float* act,
                         DropSpec drop, hipStream_t st);
int64_t nt_h_dact_parts();
int launch_gemm_nt_h_dact(const float* A, int64_t lda, int64_t M, int R, const void* Wf, int C,
                          float* out, int64_t ldo, float* rmax, const float* pre, DropSpec drop,
                          float* dpart, int64_t n_parts, hipStream_t st);
int launch_adam(const rb_adam_job* jobs, int n, double lr, double beta1, double beta2, double eps,
                double weight_decay, double bc1, double bc2, hipStream_t st);
int launch_gemm_nt_hs(const float* A, int64_t lda, int64_t M, int R, const void* Wf, int C,
                      const float* bias, float* out, int64_t ldo, float* rmax, hipStream_t st);
int launch_gemm_tn_hs(const float* Y, int64_t ldy, const float* X, int64_t ldx, int64_t M, int N,
                      int K, float* dw, int accumulate, hipStream_t st);
int64_t emb_workspace_bytes(int64_t M, int64_t V, int64_t d);
int launch_embedding_plan(const int64_t* idx, int64_t M, int64_t d, int64_t V, void* workspace,
                          int64_t ws_bytes, hipStream_t st);
int launch_embedding_apply(const float* grad, int64_t M, int64_t d, int64_t V,
                           int64_t padding_idx, float* dw, void* workspace, int64_t ws_bytes,
                           hipStream_t st);
int launch_embedding_bwd(const int64_t* idx, const float* grad, int64_t M, int64_t d, int64_t V,
                         int64_t padding_idx, float* dw, void* workspace, int64_t ws_bytes,
                         hipStream_t st);
int64_t item_ce_workspace_bytes(int64_t B, int64_t V, int64_t D);
int64_t item_rank_workspace_bytes(int64_t B, int64_t V);
int launch_item_ce_fwd(const float* E, const float* W, const int64_t* tgt, int64_t B, int64_t V,
                       int64_t D, float* lse, float* loss, void* ws, int64_t ws_bytes,
                       hipStream_t st);
int launch_item_ce_bwd(const float* E, const float* W, const int64_t* tgt, const float* lse,
                       const float* dloss, int64_t B, int64_t V, int64_t D, float* dE, float* dW,
                       void* ws, int64_t ws_bytes, hipStream_t st);
int launch_item_rank(const float* E, const float* W, const int64_t* tgt, int64_t B, int64_t V,
                     int64_t D, int64_t first, int64_t* n_gt, int64_t* n_eq, void* ws,
                     int64_t ws_bytes, hipStream_t st);
int launch_item_ce_probs(const float* E, const float* W, const int64_t* tgt, const float* lse,
                         const float* dloss, int64_t B, int64_t V, int64_t D, int64_t v_off,
                         int64_t n_total, float* out, int64_t ld, hipStream_t st);
int launch_item_scores(const float* E, const float* W, int64_t B, int64_t V, int64_t D,
                       float* out, hipStream_t st);
int launch_item_split_h(const float* X, int64_t N, int64_t D, void* img, int* ex, float* gmax,
                        hipStream_t st);
int launch_item_ce_fwd_h(const void* Ei, const int* Ee, const void* Wi, const int* We,
                         const int64_t* tgt, int64_t B, int64_t V, int64_t D, float* lse,
                         float* loss, void* ws, int64_t ws_bytes, hipStream_t st);
int launch_item_ce_probs_h(const void* Ei, const int* Ee, const void* Wi, const int* We,
                           const int64_t* tgt, const float* lse, const float* dloss, int64_t B,
                           int64_t V, int64_t D, int64_t v_off, float* out, int64_t ld,
                           float* gmax, float* out2, int64_t ld2, float* bmax, hipStream_t st);
int launch_group_absmax(const float* x, int64_t n, int64_t c, int64_t ld, float* out,
                        hipStream_t st);
int launch_pad_prefix_fwd(const float* conv_b, const float* gw, const float* gb,
                          const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                          int64_t H, float* h0, float* ws, hipStream_t st);
int launch_pad_prefix_bwd(const float* conv_b, const float* gw, const float* gb,
                          const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                          int64_t H, const float* dh0, float* dconv_b, float* dgw, float* dgb,
                          float* dlam, float* ws, int accumulate, hipStream_t st);
int launch_colsum(const float* in, int64_t M, int64_t P, int64_t C, int64_t rs, int64_t ms,
                  float* out, hipStream_t st);
int launch_colsum_chunked(const float* in, int64_t M, int64_t P, int64_t C, int64_t rs, int CH,
                          float* part, unsigned* cnt, float* out, hipStream_t st);
int launch_scan_fwd(const float* gates, const float* tokens, float* states, int64_t rows,
                    int64_t T, hipStream_t st);
int launch_scan_bwd(const float* gates, const float* states, const float* grad, float* d_gates,
                    float* d_tokens, int64_t rows, int64_t T, hipStream_t st);

}  // namespace rb
