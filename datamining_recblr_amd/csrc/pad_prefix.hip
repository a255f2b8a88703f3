// pad_prefix.hip — the recurrent state the reference's power-of-two left
// padding leaves behind (RecBLR.py:176-179), forward and backward, each as
// one single-workgroup launch.
//
// Pad positions carry zeros into the causal conv, so every pad step sees the
// per-channel constants xc_p = silu(conv.bias), (r_p, i_p) = W_g xc_p + b_g,
// s = softplus(Lambda) sigmoid(r_p), alpha = exp(-s),
// beta = sqrt(1 - alpha^2 + 1e-8) sigmoid(i_p), b_p = beta xc_p, and after P
// such steps the state is h0 = b_p E(P, s), E = expm1(-P s) / expm1(-s)
// (= sum_{k<P} alpha^k without cancellation).  This replaces ~20 [H]-sized
// torch kernels in the forward and ~40 in the backward per layer, each a
// separate ~5 us launch at these sizes.
//
// Rows: h0 has n_rows rows; row b uses pad length pad[b] (pad != NULL) or
// pad_len.  The backward sums the per-row gradients in row order.
#include <cmath>

#include "common.h"

namespace rb {
namespace {

constexpr int kPT = 1024;  // threads of the single workgroup

struct PadConsts {
  float xc, sg_r, sg_i, sp, s, alpha, q, beta, b;
  bool clamped;
};

__device__ __forceinline__ float expm1_ratio(float P, float s) {  // E(P, s)
  return expm1f(-P * s) / expm1f(-s);
}

// dE/ds = (-P e^{-Ps} expm1(-s) + expm1(-Ps) e^{-s}) / expm1(-s)^2
__device__ __forceinline__ float expm1_ratio_ds(float P, float s) {
  const float d = expm1f(-s);
  return (-P * expf(-P * s) * d + expm1f(-P * s) * expf(-s)) / (d * d);
}

// per-channel constants from the gate pre-activations rg (LDS)
__device__ __forceinline__ PadConsts consts(int c, int H, const float* xc, const float* rg,
                                            const float* lam) {
  PadConsts k;
  k.xc = xc[c];
  k.sg_r = sigm(rg[c]);
  k.sg_i = sigm(rg[H + c]);
  k.sp = softplus_f(lam[c]);
  const float s = k.sp * k.sg_r;
  k.clamped = !(s > 1e-20f);
  k.s = k.clamped ? 1e-20f : s;
  k.alpha = expf(-s);
  k.q = sqrtf(1.0f - k.alpha * k.alpha + 1e-8f);
  k.beta = k.q * k.sg_i;
  k.b = k.beta * k.xc;
  return k;
}

// xc_p into LDS, then rg = W_g xc_p + b_g: one wave per output row, lanes
// along the row (coalesced), fixed-order butterfly reduction
__device__ void gates_of_pad(const float* conv_b, const float* gw, const float* gb, int H,
                             float* xc, float* rg) {
  for (int c = threadIdx.x; c < H; c += kPT) xc[c] = silu_f(conv_b[c]);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int o = wave; o < 2 * H; o += kPT / 64) {
    const float* w = gw + (int64_t)o * H;
    float acc = 0.0f;
    for (int k = lane; k < H; k += 64) acc = fmaf(w[k], xc[k], acc);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) rg[o] = acc + gb[o];
  }
  __syncthreads();
}

__global__ __launch_bounds__(kPT) void k_pad_prefix_fwd(const float* __restrict__ conv_b,
                                                        const float* __restrict__ gw,
                                                        const float* __restrict__ gb,
                                                        const float* __restrict__ lam,
                                                        const int64_t* __restrict__ pad,
                                                        int64_t pad_len, int64_t n_rows, int H,
                                                        float* __restrict__ h0) {
  extern __shared__ float sh[];
  float* xc = sh;
  float* rg = sh + H;
  gates_of_pad(conv_b, gw, gb, H, xc, rg);
  for (int c = threadIdx.x; c < H; c += kPT) {
    const PadConsts k = consts(c, H, xc, rg, lam);
    for (int64_t r = 0; r < n_rows; ++r) {
      const float P = (float)(pad ? pad[r] : pad_len);
      h0[r * H + c] = k.b * expm1_ratio(P, k.s);
    }
  }
}

__global__ __launch_bounds__(kPT) void k_pad_prefix_bwd(
    const float* __restrict__ conv_b, const float* __restrict__ gw, const float* __restrict__ gb,
    const float* __restrict__ lam, const int64_t* __restrict__ pad, int64_t pad_len,
    int64_t n_rows, int H, const float* __restrict__ dh0, float* __restrict__ dconv_b,
    float* __restrict__ dgw, float* __restrict__ dgb, float* __restrict__ dlam) {
  extern __shared__ float sh[];
  float* xc = sh;
  float* rg = sh + H;
  float* drg = sh + 3 * H;    // [2H]
  float* dxb = sh + 5 * H;    // [H] d xc_p through b_p
  gates_of_pad(conv_b, gw, gb, H, xc, rg);
  for (int c = threadIdx.x; c < H; c += kPT) {
    const PadConsts k = consts(c, H, xc, rg, lam);
    float gb_ = 0.0f, gs = 0.0f;   // dL/db_p, dL/ds
    for (int64_t r = 0; r < n_rows; ++r) {
      const float P = (float)(pad ? pad[r] : pad_len);
      const float g = dh0[r * H + c];
      gb_ = fmaf(g, expm1_ratio(P, k.s), gb_);
      gs = fmaf(g * k.b, expm1_ratio_ds(P, k.s), gs);
    }
    if (k.clamped) gs = 0.0f;                        // clamp_min(1e-20) passes no gradient
    // b = beta xc; beta = q sg_i; q = sqrt(1 - alpha^2 + 1e-8); alpha = exp(-s)
    const float dbeta = gb_ * k.xc;
    dxb[c] = gb_ * k.beta;
    const float dq = dbeta * k.sg_i;
    const float dsg_i = dbeta * k.q;
    const float dalpha = dq * (-k.alpha / k.q);
    // alpha = exp(-s_raw) (the unclamped s, as torch computes alpha)
    const float ds = gs + dalpha * (-k.alpha);
    // s = sp * sg_r
    dlam[c] = ds * k.sg_r * dsoftplus_f(lam[c]);
    const float dsg_r = ds * k.sp;
    drg[c] = dsg_r * k.sg_r * (1.0f - k.sg_r);
    drg[H + c] = dsg_i * k.sg_i * (1.0f - k.sg_i);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < 2 * H; o += kPT) dgb[o] = drg[o];
  // dW_g = drg (x) xc_p, written row by row (threads along the row)
  for (int o = 0; o < 2 * H; ++o)
    for (int c = threadIdx.x; c < H; c += kPT) dgw[(int64_t)o * H + c] = drg[o] * xc[c];
  // d xc_p = W_g^T drg + (through b_p), then silu'
  for (int c = threadIdx.x; c < H; c += kPT) {
    float acc = 0.0f;
    for (int o = 0; o < 2 * H; ++o) acc = fmaf(gw[(int64_t)o * H + c], drg[o], acc);
    dconv_b[c] = (acc + dxb[c]) * dsilu_f(conv_b[c]);
  }
}

}  // namespace

int launch_pad_prefix_fwd(const float* conv_b, const float* gw, const float* gb,
                          const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                          int64_t H, float* h0, hipStream_t st) {
  hipLaunchKernelGGL(k_pad_prefix_fwd, dim3(1), dim3(kPT), (size_t)3 * H * sizeof(float), st,
                     conv_b, gw, gb, lam, pad, pad_len, n_rows, (int)H, h0);
  return launch_status("rb_pad_prefix_fwd");
}

int launch_pad_prefix_bwd(const float* conv_b, const float* gw, const float* gb,
                          const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                          int64_t H, const float* dh0, float* dconv_b, float* dgw, float* dgb,
                          float* dlam, hipStream_t st) {
  hipLaunchKernelGGL(k_pad_prefix_bwd, dim3(1), dim3(kPT), (size_t)6 * H * sizeof(float), st,
                     conv_b, gw, gb, lam, pad, pad_len, n_rows, (int)H, dh0, dconv_b, dgw, dgb,
                     dlam);
  return launch_status("rb_pad_prefix_bwd");
}

}  // namespace rb
