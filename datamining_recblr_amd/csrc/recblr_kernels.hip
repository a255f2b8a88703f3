// recblr_kernels.hip — hand-written gfx950 (CDNA4) kernels for the RecBLR
// sequence encoder hot path, exported through the C-ABI in
// include/recblr_hip.h.
//
// Design:
//   * activations are channel-last [B, L, H] fp32; one wave lane = one channel,
//     so every per-timestep access of a wave is one contiguous 256-B segment;
//   * the BD-LRU recurrence h_t = a_t h_{t-1} + b_t is a chunked scan: a
//     workgroup owns (batch b, 64 channels) and walks the sequence in tiles of
//     RB_TILE steps; inside a tile each wave scans its own TC-step chunk in
//     registers (upsweep), the chunk summaries (prod a, local h) are combined
//     across waves through LDS (scan of summaries), and each wave re-applies
//     its exact carry-in (downsweep).  The tile's outgoing carry is kept in
//     registers and checkpointed once per tile so the backward pass can
//     recompute h without storing it;
//   * the reference-layout shim (parallel_scan on [B, C, T], T contiguous)
//     is a wave-per-row scan: 4 consecutive steps per lane (float4), a
//     Kogge-Stone scan of the lane summaries with wavefront shuffles, and a
//     serial carry across 256-step blocks.
// The combine operator is the reference's first_order_op
// (parallel_scan.py:35-41): (x_l, f_l) o (x_r, f_r) = (x_l f_r + x_r, f_l f_r),
// evaluated without FMA contraction like the reference (enable_fp_fusion=False,
// parallel_scan.py:92) — the library is built with -ffp-contract=off.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/recblr_hip.h"

namespace {

constexpr int kWave = 64;

thread_local std::string g_last_error;

int fail(const char* msg) {
  g_last_error = msg;
  return RB_EINVAL;
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return static_cast<int>(e);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// scalar math, written to follow torch's definitions
// ---------------------------------------------------------------------------
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

// ---------------------------------------------------------------------------
// Reference-layout scan: rows of T contiguous fp32, one wave per row.
// ---------------------------------------------------------------------------
template <bool VEC4>
__global__ void __launch_bounds__(256)
k_scan_rows_fwd(const float* __restrict__ gates, const float* __restrict__ tokens,
                float* __restrict__ out, int64_t rows, int64_t T) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // wave-uniform
  const float* g = gates + row * T;
  const float* x = tokens + row * T;
  float* o = out + row * T;
  float carry = 0.0f;
  for (int64_t t0 = 0; t0 < T; t0 += 4 * kWave) {
    const int64_t t = t0 + 4 * lane;
    float a[4], v[4];
    if (VEC4 && t + 3 < T) {
      const float4 ga = *reinterpret_cast<const float4*>(g + t);
      const float4 xa = *reinterpret_cast<const float4*>(x + t);
      a[0] = ga.x; a[1] = ga.y; a[2] = ga.z; a[3] = ga.w;
      v[0] = xa.x; v[1] = xa.y; v[2] = xa.z; v[3] = xa.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = t + j < T;
        a[j] = ok ? g[t + j] : 1.0f;  // identity element (x=0, f=1)
        v[j] = ok ? x[t + j] : 0.0f;
      }
    }
    // upsweep inside the lane
    float A = a[0], X = v[0];
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      X = X * a[j] + v[j];
      A = A * a[j];
    }
    // Kogge-Stone inclusive scan of lane summaries across the wave
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const float Ap = __shfl_up(A, off, kWave);
      const float Xp = __shfl_up(X, off, kWave);
      if (lane >= off) {
        X = Xp * A + X;
        A = Ap * A;
      }
    }
    float Ae = __shfl_up(A, 1, kWave);
    float Xe = __shfl_up(X, 1, kWave);
    if (lane == 0) {
      Ae = 1.0f;
      Xe = 0.0f;
    }
    // downsweep: lane carry-in = carry o exclusive-prefix
    float h = carry * Ae + Xe;
    float res[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      h = h * a[j] + v[j];
      res[j] = h;
    }
    if (VEC4 && t + 3 < T) {
      *reinterpret_cast<float4*>(o + t) = make_float4(res[0], res[1], res[2], res[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (t + j < T) o[t + j] = res[j];
    }
    const float A63 = __shfl(A, kWave - 1, kWave);
    const float X63 = __shfl(X, kWave - 1, kWave);
    carry = carry * A63 + X63;
  }
}

// Reverse scan with shifted gates (parallel_scan.py:106-113):
//   d_t = d_{t+1} * a_{t+1} + grad_t, d_gates_t = h_{t-1} d_t, d_tokens = d.
template <bool VEC4>
__global__ void __launch_bounds__(256)
k_scan_rows_bwd(const float* __restrict__ gates, const float* __restrict__ states,
                const float* __restrict__ grad, float* __restrict__ d_gates,
                float* __restrict__ d_tokens, int64_t rows, int64_t T) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* g = gates + row * T;
  const float* s = states + row * T;
  const float* gr = grad + row * T;
  float* dg = d_gates + row * T;
  float* dt = d_tokens + row * T;
  const int64_t nblk = (T + 4 * kWave - 1) / (4 * kWave);
  float carry = 0.0f;     // d at the first step after the block
  float a_next = 1.0f;    // gates at the first step after the block
  for (int64_t blk = nblk - 1; blk >= 0; --blk) {
    const int64_t t0 = blk * 4 * kWave;
    const int64_t t = t0 + 4 * lane;
    float a[4], y[4], hs[4];
    if (VEC4 && t + 3 < T) {
      const float4 ga = *reinterpret_cast<const float4*>(g + t);
      const float4 ya = *reinterpret_cast<const float4*>(gr + t);
      const float4 sa = *reinterpret_cast<const float4*>(s + t);
      a[0] = ga.x; a[1] = ga.y; a[2] = ga.z; a[3] = ga.w;
      y[0] = ya.x; y[1] = ya.y; y[2] = ya.z; y[3] = ya.w;
      hs[0] = sa.x; hs[1] = sa.y; hs[2] = sa.z; hs[3] = sa.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = t + j < T;
        a[j] = ok ? g[t + j] : 1.0f;
        y[j] = ok ? gr[t + j] : 0.0f;
        hs[j] = ok ? s[t + j] : 0.0f;
      }
    }
    // shifted gates: as[j] = a_{t+j+1}
    float as[4];
    const float a_lane_next = __shfl_down(a[0], 1, kWave);
    as[0] = a[1];
    as[1] = a[2];
    as[2] = a[3];
    as[3] = (lane == kWave - 1) ? a_next : a_lane_next;
    // elements past the end of the row are identities
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (t + j >= T) as[j] = 1.0f;
    // upsweep inside the lane, from the right
    float A = as[3], D = y[3];
#pragma unroll
    for (int j = 2; j >= 0; --j) {
      D = D * as[j] + y[j];
      A = A * as[j];
    }
    // reverse Kogge-Stone across the wave
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const float An = __shfl_down(A, off, kWave);
      const float Dn = __shfl_down(D, off, kWave);
      if (lane + off < kWave) {
        D = Dn * A + D;
        A = An * A;
      }
    }
    float Ae = __shfl_down(A, 1, kWave);
    float De = __shfl_down(D, 1, kWave);
    if (lane == kWave - 1) {
      Ae = 1.0f;
      De = 0.0f;
    }
    float d = carry * Ae + De;
    // h_{t-1} for the lane's first element
    float hprev0 = __shfl_up(hs[3], 1, kWave);
    if (lane == 0) hprev0 = (t0 > 0) ? s[t0 - 1] : 0.0f;
    float dres[4], gres[4];
#pragma unroll
    for (int j = 3; j >= 0; --j) {
      d = d * as[j] + y[j];
      const float hp = (j == 0) ? hprev0 : hs[j - 1];
      dres[j] = d;
      gres[j] = hp * d;
    }
    if (VEC4 && t + 3 < T) {
      *reinterpret_cast<float4*>(dt + t) = make_float4(dres[0], dres[1], dres[2], dres[3]);
      *reinterpret_cast<float4*>(dg + t) = make_float4(gres[0], gres[1], gres[2], gres[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (t + j < T) {
          dt[t + j] = dres[j];
          dg[t + j] = gres[j];
        }
    }
    const float A0 = __shfl(A, 0, kWave);
    const float D0 = __shfl(D, 0, kWave);
    carry = carry * A0 + D0;
    a_next = __shfl(a[0], 0, kWave);
  }
}

// ---------------------------------------------------------------------------
// Causal depthwise conv + bias + SiLU, channel-last.  One wave = (b, 64
// channels, TC consecutive steps); waves are independent.
// ---------------------------------------------------------------------------
template <int K, int TC>
__global__ void __launch_bounds__(256)
k_conv_silu_fwd(const float* __restrict__ x, int64_t x_rs, const float* __restrict__ w,
                const float* __restrict__ bias, float* __restrict__ xc, int64_t xc_rs,
                int64_t B, int L, int H, int ncg, int nchunk) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int chunk = (int)(gw % nchunk);
  const int64_t tmp = gw / nchunk;
  const int cgi = (int)(tmp % ncg);
  const int64_t b = tmp / ncg;
  if (b >= B) return;
  const int c = cgi * kWave + lane;
  const bool cv = c < H;
  const int cc = cv ? c : H - 1;
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[(int64_t)cc * K + k];
  const float bi = bias[cc];
  const int t0 = chunk * TC;
  const int64_t rowb = b * L;
  // window holds x[t-K+1 .. t]
  float win[K];
#pragma unroll
  for (int k = 0; k < K - 1; ++k) {
    const int t = t0 - (K - 1) + k;
    const int tc = t < 0 ? 0 : (t >= L ? L - 1 : t);
    const float v = x[(rowb + tc) * x_rs + cc];
    win[k] = (t >= 0 && t < L) ? v : 0.0f;
  }
  float xv[TC];
#pragma unroll
  for (int j = 0; j < TC; ++j) {
    const int t = t0 + j;
    const int tc = t >= L ? L - 1 : t;
    xv[j] = x[(rowb + tc) * x_rs + cc];
  }
#pragma unroll
  for (int j = 0; j < TC; ++j) {
    const int t = t0 + j;
    win[K - 1] = xv[j];
    float acc = bi;
#pragma unroll
    for (int k = 0; k < K; ++k) acc = acc + wk[k] * win[k];
    if (cv && t < L) xc[(rowb + t) * xc_rs + c] = silu_f(acc);
#pragma unroll
    for (int k = 0; k < K - 1; ++k) win[k] = win[k + 1];
  }
}

// Backward: workgroup = (b, 64 channels), W waves walk the sequence in tiles
// of W*TC steps so the dW / dbias partial sums for this batch row can be
// reduced in LDS without atomics.
template <int K, int W, int TC>
__global__ void __launch_bounds__(W * 64)
k_conv_silu_bwd(const float* __restrict__ x, int64_t x_rs, const float* __restrict__ w,
                const float* __restrict__ bias, const float* __restrict__ g1,
                const float* __restrict__ g2, float* __restrict__ dx, int64_t dx_rs,
                float* __restrict__ dw_part, float* __restrict__ db_part,
                int L, int H, int ncg) {
  __shared__ float red[W][K + 1][kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int64_t b = blockIdx.x / ncg;
  const int cgi = blockIdx.x - (int)(b * ncg);
  const int c = cgi * kWave + lane;
  const bool cv = c < H;
  const int cc = cv ? c : H - 1;
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[(int64_t)cc * K + k];
  const float bi = bias[cc];
  const int64_t rowb = b * L;
  float accw[K], accb = 0.0f;
#pragma unroll
  for (int k = 0; k < K; ++k) accw[k] = 0.0f;

  constexpr int NX = TC + 2 * (K - 1);  // x[t0-K+1 .. t0+TC+K-2]
  constexpr int ND = TC + K - 1;        // du[t0 .. t0+TC+K-2]
  for (int tb = 0; tb < L; tb += W * TC) {
    const int t0 = tb + wv * TC;
    if (t0 >= L) break;  // wave-uniform
    float xs[NX];
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      const int t = t0 - (K - 1) + m;
      const int tc = t < 0 ? 0 : (t >= L ? L - 1 : t);
      const float v = x[(rowb + tc) * x_rs + cc];
      xs[m] = (t >= 0 && t < L) ? v : 0.0f;
    }
    float gs[ND];
#pragma unroll
    for (int m = 0; m < ND; ++m) {
      const int t = t0 + m;
      const int tc = t >= L ? L - 1 : t;
      float v = g1[(rowb + tc) * H + cc];
      if (g2 != nullptr) v = v + g2[(rowb + tc) * H + cc];
      gs[m] = (t < L) ? v : 0.0f;
    }
    float du[ND];
#pragma unroll
    for (int m = 0; m < ND; ++m) {
      float acc = bi;
#pragma unroll
      for (int k = 0; k < K; ++k) acc = acc + wk[k] * xs[m + k];
      du[m] = gs[m] * dsilu_f(acc);  // gs is 0 past the end
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int t = t0 + j;
      // dx_t = sum_k w_k du_{t+K-1-k}
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < K; ++k) acc = acc + wk[k] * du[j + K - 1 - k];
      if (cv && t < L) dx[(rowb + t) * dx_rs + c] = acc;
      if (t < L) {
        accb = accb + du[j];
#pragma unroll
        for (int k = 0; k < K; ++k) accw[k] = accw[k] + du[j] * xs[j + k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) red[wv][k][lane] = accw[k];
  red[wv][K][lane] = accb;
  __syncthreads();
  if (wv == 0 && cv) {
#pragma unroll
    for (int k = 0; k <= K; ++k) {
      float s = 0.0f;
#pragma unroll
      for (int q = 0; q < W; ++q) s = s + red[q][k][lane];
      if (k < K)
        dw_part[(b * K + k) * H + c] = s;
      else
        db_part[b * H + c] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// Fused gates + BD-LRU scan + silu(z) merge.
// ---------------------------------------------------------------------------
template <int W, int TC>
__global__ void __launch_bounds__(W * 64)
k_gate_scan_fwd(const float* __restrict__ rg, int64_t rg_rs, const float* __restrict__ xc,
                int64_t xc_rs, const float* __restrict__ z, int64_t z_rs,
                const float* __restrict__ lam, const float* __restrict__ h0,
                float* __restrict__ y, int64_t y_rs, float* __restrict__ carries,
                int L, int H, int ncg) {
  static_assert(W * TC == RB_TILE, "tile");
  __shared__ float sA[2][W][kWave];
  __shared__ float sX[2][W][kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int64_t b = blockIdx.x / ncg;
  const int cgi = blockIdx.x - (int)(b * ncg);
  const int c = cgi * kWave + lane;
  const bool cv = c < H;
  const int cc = cv ? c : H - 1;
  const float nsp = -softplus_f(lam[cc]);
  float carry = (h0 != nullptr) ? h0[cc] : 0.0f;
  const int nT = (L + RB_TILE - 1) / RB_TILE;
  const int64_t rowb = b * L;
  for (int tile = 0; tile < nT; ++tile) {
    const int buf = tile & 1;
    if (wv == 0 && cv) carries[(b * nT + tile) * H + c] = carry;
    const int t0 = tile * RB_TILE + wv * TC;
    float rv[TC], iv[TC], xv[TC], zv[TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int t = t0 + j;
      const int64_t row = rowb + (t >= L ? L - 1 : t);
      rv[j] = rg[row * rg_rs + cc];
      iv[j] = rg[row * rg_rs + H + cc];
      xv[j] = xc[row * xc_rs + cc];
      zv[j] = z[row * z_rs + cc];
    }
    float al[TC], bp[TC];
    float A = 1.0f, X = 0.0f;
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const bool ok = t0 + j < L;
      const float a = expf(nsp * sigm(rv[j]));
      const float beta = sqrtf(1.0f - a * a + 1e-8f) * sigm(iv[j]);
      al[j] = ok ? a : 1.0f;
      bp[j] = ok ? beta * xv[j] : 0.0f;
      X = X * al[j] + bp[j];
      A = A * al[j];
    }
    sA[buf][wv][lane] = A;
    sX[buf][wv][lane] = X;
    __syncthreads();
    float run = carry, cin = carry;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      if (k == wv) cin = run;
      run = run * sA[buf][k][lane] + sX[buf][k][lane];
    }
    float h = cin;
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int t = t0 + j;
      h = h * al[j] + bp[j];
      if (cv && t < L) y[(rowb + t) * y_rs + c] = silu_f(zv[j]) * h;
    }
    carry = run;
  }
}

template <int W, int TC>
__global__ void __launch_bounds__(W * 64)
k_gate_scan_bwd(const float* __restrict__ rg, int64_t rg_rs, const float* __restrict__ xc,
                int64_t xc_rs, const float* __restrict__ z, int64_t z_rs,
                const float* __restrict__ lam, const float* __restrict__ carries,
                const float* __restrict__ dy, float* __restrict__ drg, int64_t drg_rs,
                float* __restrict__ dxc, float* __restrict__ dz, int64_t dz_rs,
                float* __restrict__ part, float* __restrict__ dh0_part,
                int64_t B, int L, int H, int ncg) {
  static_assert(W * TC == RB_TILE, "tile");
  __shared__ float sA[2][W][kWave];
  __shared__ float sX[2][W][kWave];
  __shared__ float sE[2][W][kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int64_t b = blockIdx.x / ncg;
  const int cgi = blockIdx.x - (int)(b * ncg);
  const int c = cgi * kWave + lane;
  const bool cv = c < H;
  const int cc = cv ? c : H - 1;
  const float lamc = lam[cc];
  const float sp = softplus_f(lamc);
  const float nsp = -sp;
  const int nT = (L + RB_TILE - 1) / RB_TILE;
  const int64_t rowb = b * L;
  float ecarry = 0.0f;  // dL/dh at the step just after the tile, times a there
  float acc_v = 0.0f, acc_r = 0.0f, acc_i = 0.0f;
  for (int tile = nT - 1; tile >= 0; --tile) {
    const int buf = tile & 1;
    const float hcar = carries[(b * nT + tile) * H + cc];
    const int t0 = tile * RB_TILE + wv * TC;
    float rv[TC], iv[TC], xv[TC], zv[TC], gv[TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int t = t0 + j;
      const int64_t row = rowb + (t >= L ? L - 1 : t);
      rv[j] = rg[row * rg_rs + cc];
      iv[j] = rg[row * rg_rs + H + cc];
      xv[j] = xc[row * xc_rs + cc];
      zv[j] = z[row * z_rs + cc];
      gv[j] = dy[row * H + cc];
    }
    float al[TC], bp[TC];
    float A = 1.0f, X = 0.0f;
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const bool ok = t0 + j < L;
      const float a = expf(nsp * sigm(rv[j]));
      const float beta = sqrtf(1.0f - a * a + 1e-8f) * sigm(iv[j]);
      al[j] = ok ? a : 1.0f;
      bp[j] = ok ? beta * xv[j] : 0.0f;
      if (!ok) gv[j] = 0.0f;
      X = X * al[j] + bp[j];
      A = A * al[j];
    }
    // local reverse summary: e_first = E + A * e_after
    float E = 0.0f;
#pragma unroll
    for (int j = TC - 1; j >= 0; --j) {
      const float d = E + gv[j] * silu_f(zv[j]);
      E = d * al[j];
    }
    sA[buf][wv][lane] = A;
    sX[buf][wv][lane] = X;
    sE[buf][wv][lane] = E;
    __syncthreads();
    float run = hcar, cin = hcar;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      if (k == wv) cin = run;
      run = run * sA[buf][k][lane] + sX[buf][k][lane];
    }
    float erun = ecarry, ein = ecarry;
#pragma unroll
    for (int k = W - 1; k >= 0; --k) {
      if (k == wv) ein = erun;
      erun = erun * sA[buf][k][lane] + sE[buf][k][lane];
    }
    // recompute h; dz needs h_t, the scan gradient needs h_{t-1}
    float hp[TC];
    float h = cin;
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int t = t0 + j;
      hp[j] = h;
      h = h * al[j] + bp[j];
      if (cv && t < L) dz[(rowb + t) * dz_rs + c] = (gv[j] * h) * dsilu_f(zv[j]);
    }
    float e = ein;
#pragma unroll
    for (int j = TC - 1; j >= 0; --j) {
      const int t = t0 + j;
      const bool ok = cv && t < L;
      const float d = e + gv[j] * silu_f(zv[j]);   // dL/dh_t
      const float a = al[j];
      const float sr = sigm(rv[j]);
      const float si = sigm(iv[j]);
      const float sq = sqrtf(1.0f - a * a + 1e-8f);
      const float beta = sq * si;
      const float dbeta = d * xv[j];
      const float dsq = dbeta * si;
      const float di = (dbeta * sq) * ((1.0f - si) * si);
      const float du = dsq / (2.0f * sq);
      const float da = hp[j] * d + (-du) * (2.0f * a);
      const float dv = da * a;
      const float dr = (dv * nsp) * ((1.0f - sr) * sr);
      if (ok) {
        const int64_t row = rowb + t;
        drg[row * drg_rs + c] = dr;
        drg[row * drg_rs + H + c] = di;
        dxc[row * H + c] = d * beta;
        acc_v = acc_v + dv * sr;
        acc_r = acc_r + dr;
        acc_i = acc_i + di;
      }
      e = d * a;
    }
    if (tile == 0 && wv == 0 && cv) dh0_part[b * H + c] = e;
    ecarry = erun;
  }
  // reduce the per-channel partial sums over the W waves
  __syncthreads();
  sA[0][wv][lane] = acc_v;
  sX[0][wv][lane] = acc_r;
  sE[0][wv][lane] = acc_i;
  __syncthreads();
  if (wv == 0 && cv) {
    float sv = 0.0f, sr = 0.0f, si = 0.0f;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      sv = sv + sA[0][k][lane];
      sr = sr + sX[0][k][lane];
      si = si + sE[0][k][lane];
    }
    // lam enters as -softplus(lam): dlam = -sum(dv * sr) * softplus'(lam)
    part[b * H + c] = -sv * dsoftplus_f(lamc);
    part[(B + b) * H + c] = sr;
    part[(2 * B + b) * H + c] = si;
  }
}

constexpr int kFwdW = 4, kFwdTC = RB_TILE / kFwdW;   // 4 waves x 16 steps
constexpr int kBwdW = 8, kBwdTC = RB_TILE / kBwdW;   // 8 waves x 8 steps
constexpr int kConvTC = 16;
constexpr int kConvBwdW = 4, kConvBwdTC = 16;

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <int K>
int conv_fwd_k(const float* x, int64_t x_rs, const float* w, const float* bias, float* xc,
               int64_t xc_rs, int64_t B, int64_t L, int64_t H, hipStream_t st) {
  const int ncg = (int)((H + kWave - 1) / kWave);
  const int nchunk = (int)((L + kConvTC - 1) / kConvTC);
  const int64_t waves = B * ncg * nchunk;
  const int64_t blocks = (waves + 3) / 4;
  hipLaunchKernelGGL((k_conv_silu_fwd<K, kConvTC>), dim3((unsigned)blocks), dim3(256), 0, st, x,
                     x_rs, w, bias, xc, xc_rs, B, (int)L, (int)H, ncg, nchunk);
  return launch_status("rb_conv_silu_fwd");
}

template <int K>
int conv_bwd_k(const float* x, int64_t x_rs, const float* w, const float* bias, const float* g1,
               const float* g2, float* dx, int64_t dx_rs, float* dw_part, float* db_part,
               int64_t B, int64_t L, int64_t H, hipStream_t st) {
  const int ncg = (int)((H + kWave - 1) / kWave);
  hipLaunchKernelGGL((k_conv_silu_bwd<K, kConvBwdW, kConvBwdTC>), dim3((unsigned)(B * ncg)),
                     dim3(kConvBwdW * 64), 0, st, x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part,
                     db_part, (int)L, (int)H, ncg);
  return launch_status("rb_conv_silu_bwd");
}

int check_dims(int64_t B, int64_t L, int64_t H) {
  if (B <= 0 || L <= 0 || H <= 0) return fail("B, L and H must be positive");
  if (L > (1 << 30) || H > (1 << 24)) return fail("L or H too large");
  if (B * ((H + 63) / 64) > 0x7fffffffLL) return fail("grid too large");
  return 0;
}

}  // namespace

extern "C" {

int rb_version(void) { return 1; }

const char* rb_last_error_string(void) { return g_last_error.c_str(); }

int rb_num_kernels(void) { return 12; }

int rb_scan_fwd(const float* gates, const float* tokens, float* states, int64_t B, int64_t C,
                int64_t T, void* stream) {
  if (!gates || !tokens || !states) return fail("rb_scan_fwd: null pointer");
  if (B <= 0 || C <= 0 || T <= 0) return fail("rb_scan_fwd: B, C, T must be positive");
  const int64_t rows = B * C;
  const int64_t blocks = (rows + 3) / 4;
  if (blocks > 0x7fffffffLL) return fail("rb_scan_fwd: too many rows");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool vec = (T % 4 == 0) && aligned16(gates) && aligned16(tokens) && aligned16(states);
  if (vec)
    hipLaunchKernelGGL(k_scan_rows_fwd<true>, dim3((unsigned)blocks), dim3(256), 0, st, gates,
                       tokens, states, rows, T);
  else
    hipLaunchKernelGGL(k_scan_rows_fwd<false>, dim3((unsigned)blocks), dim3(256), 0, st, gates,
                       tokens, states, rows, T);
  return launch_status("rb_scan_fwd");
}

int rb_scan_bwd(const float* gates, const float* states, const float* grad, float* d_gates,
                float* d_tokens, int64_t B, int64_t C, int64_t T, void* stream) {
  if (!gates || !states || !grad || !d_gates || !d_tokens)
    return fail("rb_scan_bwd: null pointer");
  if (B <= 0 || C <= 0 || T <= 0) return fail("rb_scan_bwd: B, C, T must be positive");
  const int64_t rows = B * C;
  const int64_t blocks = (rows + 3) / 4;
  if (blocks > 0x7fffffffLL) return fail("rb_scan_bwd: too many rows");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool vec = (T % 4 == 0) && aligned16(gates) && aligned16(states) && aligned16(grad) &&
                   aligned16(d_gates) && aligned16(d_tokens);
  if (vec)
    hipLaunchKernelGGL(k_scan_rows_bwd<true>, dim3((unsigned)blocks), dim3(256), 0, st, gates,
                       states, grad, d_gates, d_tokens, rows, T);
  else
    hipLaunchKernelGGL(k_scan_rows_bwd<false>, dim3((unsigned)blocks), dim3(256), 0, st, gates,
                       states, grad, d_gates, d_tokens, rows, T);
  return launch_status("rb_scan_bwd");
}

int rb_conv_silu_fwd(const float* x, int64_t x_rs, const float* w, const float* bias, float* xc,
                     int64_t xc_rs, int64_t B, int64_t L, int64_t H, int64_t K, void* stream) {
  if (!x || !w || !bias || !xc) return fail("rb_conv_silu_fwd: null pointer");
  if (int r = check_dims(B, L, H)) return r;
  if (x_rs < H || xc_rs < H) return fail("rb_conv_silu_fwd: row stride < H");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (K) {
    case 1: return conv_fwd_k<1>(x, x_rs, w, bias, xc, xc_rs, B, L, H, st);
    case 2: return conv_fwd_k<2>(x, x_rs, w, bias, xc, xc_rs, B, L, H, st);
    case 3: return conv_fwd_k<3>(x, x_rs, w, bias, xc, xc_rs, B, L, H, st);
    case 4: return conv_fwd_k<4>(x, x_rs, w, bias, xc, xc_rs, B, L, H, st);
    case 5: return conv_fwd_k<5>(x, x_rs, w, bias, xc, xc_rs, B, L, H, st);
    case 6: return conv_fwd_k<6>(x, x_rs, w, bias, xc, xc_rs, B, L, H, st);
    case 7: return conv_fwd_k<7>(x, x_rs, w, bias, xc, xc_rs, B, L, H, st);
    case 8: return conv_fwd_k<8>(x, x_rs, w, bias, xc, xc_rs, B, L, H, st);
    default: return fail("rb_conv_silu_fwd: kernel size K must be in [1, 8]");
  }
}

int rb_conv_silu_bwd(const float* x, int64_t x_rs, const float* w, const float* bias,
                     const float* g1, const float* g2, float* dx, int64_t dx_rs, float* dw_part,
                     float* db_part, int64_t B, int64_t L, int64_t H, int64_t K, void* stream) {
  if (!x || !w || !bias || !g1 || !dx || !dw_part || !db_part)
    return fail("rb_conv_silu_bwd: null pointer");
  if (int r = check_dims(B, L, H)) return r;
  if (x_rs < H || dx_rs < H) return fail("rb_conv_silu_bwd: row stride < H");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (K) {
    case 1: return conv_bwd_k<1>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, st);
    case 2: return conv_bwd_k<2>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, st);
    case 3: return conv_bwd_k<3>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, st);
    case 4: return conv_bwd_k<4>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, st);
    case 5: return conv_bwd_k<5>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, st);
    case 6: return conv_bwd_k<6>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, st);
    case 7: return conv_bwd_k<7>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, st);
    case 8: return conv_bwd_k<8>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, st);
    default: return fail("rb_conv_silu_bwd: kernel size K must be in [1, 8]");
  }
}

int rb_gate_scan_fwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                     const float* z, int64_t z_rs, const float* lam, const float* h0, float* y,
                     int64_t y_rs, float* carries, int64_t B, int64_t L, int64_t H,
                     void* stream) {
  if (!rg || !xc || !z || !lam || !y || !carries) return fail("rb_gate_scan_fwd: null pointer");
  if (int r = check_dims(B, L, H)) return r;
  if (rg_rs < 2 * H || xc_rs < H || z_rs < H || y_rs < H)
    return fail("rb_gate_scan_fwd: row stride too small");
  const int ncg = (int)((H + kWave - 1) / kWave);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL((k_gate_scan_fwd<kFwdW, kFwdTC>), dim3((unsigned)(B * ncg)),
                     dim3(kFwdW * 64), 0, st, rg, rg_rs, xc, xc_rs, z, z_rs, lam, h0, y, y_rs,
                     carries, (int)L, (int)H, ncg);
  return launch_status("rb_gate_scan_fwd");
}

int rb_gate_scan_bwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                     const float* z, int64_t z_rs, const float* lam, const float* carries,
                     const float* dy, float* drg, int64_t drg_rs, float* dxc, float* dz,
                     int64_t dz_rs, float* part, float* dh0_part, int64_t B, int64_t L,
                     int64_t H, void* stream) {
  if (!rg || !xc || !z || !lam || !carries || !dy || !drg || !dxc || !dz || !part || !dh0_part)
    return fail("rb_gate_scan_bwd: null pointer");
  if (int r = check_dims(B, L, H)) return r;
  if (rg_rs < 2 * H || xc_rs < H || z_rs < H || drg_rs < 2 * H || dz_rs < H)
    return fail("rb_gate_scan_bwd: row stride too small");
  const int ncg = (int)((H + kWave - 1) / kWave);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL((k_gate_scan_bwd<kBwdW, kBwdTC>), dim3((unsigned)(B * ncg)),
                     dim3(kBwdW * 64), 0, st, rg, rg_rs, xc, xc_rs, z, z_rs, lam, carries, dy,
                     drg, drg_rs, dxc, dz, dz_rs, part, dh0_part, B, (int)L, (int)H, ncg);
  return launch_status("rb_gate_scan_bwd");
}

}  // extern "C"
