// pad_prefix.hip — the recurrent state the reference's power-of-two left
// padding leaves behind (RecBLR.py:176-179), forward (1 small launch) and
// backward (2).
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
// pad_len.  The backward sums the per-row gradients in row order.  ws: 5H
// floats of caller scratch (rg, drg, dxb).
#include <cmath>

#include "common.h"

namespace rb {
namespace {

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

// per-channel constants from the gate pre-activations (r, i) of channel c
__device__ __forceinline__ PadConsts consts(int c, float r, float i, float xc, const float* lam) {
  PadConsts k;
  k.xc = xc;
  k.sg_r = sigm(r);
  k.sg_i = sigm(i);
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

// the gate pre-activation of row o: W_g[o] . silu(conv_b) + b_g[o], lanes
// along the row (coalesced), fixed-order butterfly; lane 0's sum (the
// butterfly's association differs per lane)
__device__ __forceinline__ float pad_gate(const float* __restrict__ conv_b,
                                          const float* __restrict__ gw,
                                          const float* __restrict__ gb, int H, int o, int lane) {
  const float* w = gw + (int64_t)o * H;
  float acc = 0.0f;
#pragma unroll 4   // H = 256: all four loads of the row in flight at once
  for (int k = lane; k < H; k += 64) acc = fmaf(w[k], silu_f(conv_b[k]), acc);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  return __shfl(acc, 0) + gb[o];
}

// forward: one wave per channel c — its two gate pre-activations (rows c and
// H + c of W_g; many workgroups, so the 2H row reads are in flight together:
// a single workgroup is load-latency bound), the constants, then h0 of every
// row (lanes over rows)
__global__ __launch_bounds__(256) void k_pad_prefix_fwd(const float* __restrict__ conv_b,
                                                        const float* __restrict__ gw,
                                                        const float* __restrict__ gb,
                                                        const float* __restrict__ lam,
                                                        const int64_t* __restrict__ pad,
                                                        int64_t pad_len, int64_t n_rows, int H,
                                                        float* __restrict__ h0) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= H) return;
  const float r = pad_gate(conv_b, gw, gb, H, c, lane);
  const float i = pad_gate(conv_b, gw, gb, H, H + c, lane);
  const PadConsts k = consts(c, r, i, silu_f(conv_b[c]), lam);
  for (int64_t row = lane; row < n_rows; row += 64) {
    const float P = (float)(pad ? pad[row] : pad_len);
    h0[row * H + c] = k.b * expm1_ratio(P, k.s);
  }
}

// backward, per channel (one wave each): its gate pre-activations again, the
// per-row gradient sums in row order (lane 0), drg [2H] / dxb (the part of d
// xc_p that flows through b_p) for k_pad_prefix_bwd3, dlam, dgate_b, and the
// channel's two rows of dW_g = drg (x) xc_p (lanes along the row: coalesced)
__global__ __launch_bounds__(256) void k_pad_prefix_bwd1(
    const float* __restrict__ conv_b, const float* __restrict__ gw, const float* __restrict__ gb,
    const float* __restrict__ lam, const int64_t* __restrict__ pad, int64_t pad_len,
    int64_t n_rows, int H, const float* __restrict__ dh0, float* __restrict__ drg,
    float* __restrict__ dxb, float* __restrict__ dgb, float* __restrict__ dlam,
    float* __restrict__ dgw, int acc) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= H) return;
  const float xc = silu_f(conv_b[c]);
  const float r = pad_gate(conv_b, gw, gb, H, c, lane);
  const float i = pad_gate(conv_b, gw, gb, H, H + c, lane);
  const PadConsts k = consts(c, r, i, xc, lam);
  float dr = 0.0f, di = 0.0f;
  if (lane == 0) {
    float gb_ = 0.0f, gs = 0.0f;   // dL/db_p, dL/ds, rows in order
    for (int64_t row = 0; row < n_rows; ++row) {
      const float P = (float)(pad ? pad[row] : pad_len);
      const float g = dh0[row * H + c];
      gb_ = fmaf(g, expm1_ratio(P, k.s), gb_);
      gs = fmaf(g * k.b, expm1_ratio_ds(P, k.s), gs);
    }
    if (k.clamped) gs = 0.0f;                        // clamp_min(1e-20) passes no gradient
    // b = beta xc; beta = q sg_i; q = sqrt(1 - alpha^2 + 1e-8); alpha = exp(-s_raw)
    const float dbeta = gb_ * k.xc;
    dxb[c] = gb_ * k.beta;
    const float dq = dbeta * k.sg_i;
    const float dsg_i = dbeta * k.q;
    const float dalpha = dq * (-k.alpha / k.q);
    const float ds = gs + dalpha * (-k.alpha);
    const float dl = ds * k.sg_r * dsoftplus_f(lam[c]);   // s = softplus(lam) sg_r
    dlam[c] = acc ? dlam[c] + dl : dl;
    dr = ds * k.sp * k.sg_r * (1.0f - k.sg_r);
    di = dsg_i * k.sg_i * (1.0f - k.sg_i);
    drg[c] = dr;
    drg[H + c] = di;
    dgb[c] = acc ? dgb[c] + dr : dr;
    dgb[H + c] = acc ? dgb[H + c] + di : di;
  }
  dr = __shfl(dr, 0);
  di = __shfl(di, 0);
  float* wr = dgw + (int64_t)c * H;
  float* wi = dgw + (int64_t)(H + c) * H;
#pragma unroll 4
  for (int kk = lane; kk < H; kk += 64) {
    const float x = silu_f(conv_b[kk]);
    const float vr = dr * x, vi = di * x;
    wr[kk] = acc ? wr[kk] + vr : vr;
    wi[kk] = acc ? wi[kk] + vi : vi;
  }
}

// dconv_b = (W_g^T drg + dxb) silu'(conv_b): 64 columns per workgroup, 16
// row groups (o = g, g+16, ... in order) combined in order g = 0..15
__global__ __launch_bounds__(1024) void k_pad_prefix_bwd3(const float* __restrict__ conv_b,
                                                          const float* __restrict__ gw, int H,
                                                          const float* __restrict__ drg,
                                                          const float* __restrict__ dxb,
                                                          float* __restrict__ dconv_b, int accum) {
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float acc = 0.0f;
  if (c < H) {
    // 8 rows' loads in flight per batch (a dependent chain of 2H / 16 = 32
    // load round trips before), the fma order unchanged
    int o = ty;
    for (; o + 7 * 16 < 2 * H; o += 8 * 16) {
      float w[8], g[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        w[q] = gw[(int64_t)(o + 16 * q) * H + c];
        g[q] = drg[o + 16 * q];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) acc = fmaf(w[q], g[q], acc);
    }
    for (; o < 2 * H; o += 16) acc = fmaf(gw[(int64_t)o * H + c], drg[o], acc);
  }
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && c < H) {
    float t = red[0][tx];
#pragma unroll
    for (int g = 1; g < 16; ++g) t += red[g][tx];
    const float v = (t + dxb[c]) * dsilu_f(conv_b[c]);
    dconv_b[c] = accum ? dconv_b[c] + v : v;
  }
}

}  // namespace

int launch_pad_prefix_fwd(const float* conv_b, const float* gw, const float* gb,
                          const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                          int64_t H, float* h0, float* ws, hipStream_t st) {
  (void)ws;
  hipLaunchKernelGGL(k_pad_prefix_fwd, dim3((unsigned)((H + 3) / 4)), dim3(256), 0, st, conv_b, gw,
                     gb, lam, pad, pad_len, n_rows, (int)H, h0);
  return launch_status("rb_pad_prefix_fwd");
}

int launch_pad_prefix_bwd(const float* conv_b, const float* gw, const float* gb,
                          const float* lam, const int64_t* pad, int64_t pad_len, int64_t n_rows,
                          int64_t H, const float* dh0, float* dconv_b, float* dgw, float* dgb,
                          float* dlam, float* ws, int accumulate, hipStream_t st) {
  float* drg = ws + 2 * H;
  float* dxb = ws + 4 * H;
  hipLaunchKernelGGL(k_pad_prefix_bwd1, dim3((unsigned)((H + 3) / 4)), dim3(256), 0, st, conv_b,
                     gw, gb, lam, pad, pad_len, n_rows, (int)H, dh0, drg, dxb, dgb, dlam, dgw,
                     accumulate);
  hipLaunchKernelGGL(k_pad_prefix_bwd3, dim3((unsigned)((H + 63) / 64)), dim3(1024), 0, st, conv_b,
                     gw, (int)H, drg, dxb, dconv_b, accumulate);
  return launch_status("rb_pad_prefix_bwd");
}

}  // namespace rb
