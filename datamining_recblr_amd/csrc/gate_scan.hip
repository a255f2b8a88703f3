// gate_scan.hip — fused BD-LRU gates + chunked scan + silu(z) merge
// (reference RecBLR.py:196-206 without the GEMMs), forward and backward.
//
// Layout: see common.h.  A wave owns batch row b and G*VEC channels; its 64
// lanes are Q time chunks x G channel groups, so one tile = Q*TC = RB_TILE
// steps.  Per tile:
//   upsweep   each lane loads its TC steps (VEC channels, 16-B loads),
//             computes alpha/b' and its chunk summary (prod alpha, local h);
//   scan      the Q summaries are scanned across lanes (shuffles at stride G)
//             and combined with the carry entering the tile;
//   downsweep each lane re-runs its TC steps from its exact carry-in.
// The state entering every tile is checkpointed (carries[b, tile, c]) so the
// backward recomputes h instead of storing it.  The backward walks the tiles
// in reverse with a second (reverse) scan for the adjoint
//   e_t = alpha_t * d_t,  d_t = dL/dh_t = e_{t+1} + dy_t * silu(z_t).
#include "common.h"

namespace rb {
namespace {

template <int VEC, int Q, int TC>
__global__ void __launch_bounds__(256)
k_gate_scan_fwd(const float* __restrict__ rg, int rg_rs, const float* __restrict__ xc, int xc_rs,
                const float* __restrict__ z, int z_rs, const float* __restrict__ lam,
                const float* __restrict__ h0, float* __restrict__ y, int y_rs,
                float* __restrict__ carries, int64_t B, int L, int H, int ncw) {
  constexpr int G = kWave / Q;
  constexpr int TILE = Q * TC;
  static_assert(TILE == RB_TILE, "tile must match the carries checkpoint stride");
  const int lane = threadIdx.x & (kWave - 1);
  const int q = lane / G;
  const int g = lane - q * G;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = wid / ncw;
  if (b >= B) return;  // wave-uniform
  const int c0 = (int)(wid - b * ncw) * (G * VEC) + g * VEC;
  const bool cv = c0 < H;
  const int cc = cv ? c0 : 0;
  const int64_t row0 = b * L;
  const float* rgb = rg + row0 * rg_rs + cc;
  const float* xcb = xc + row0 * xc_rs + cc;
  const float* zb = z + row0 * z_rs + cc;
  float* yb = y + row0 * y_rs + cc;

  float nsp[VEC], carry[VEC];
  ldv(nsp, lam + cc);
#pragma unroll
  for (int v = 0; v < VEC; ++v) nsp[v] = -softplus_f(nsp[v]);
  if (h0 != nullptr) {
    ldv(carry, h0 + cc);
  } else {
#pragma unroll
    for (int v = 0; v < VEC; ++v) carry[v] = 0.0f;
  }
  const int nT = (L + TILE - 1) / TILE;
  for (int tile = 0; tile < nT; ++tile) {
    if (carries != nullptr && q == 0 && cv) stv(carries + (b * nT + tile) * H + c0, carry);
    const int t0 = tile * TILE + q * TC;
    float al[TC][VEC], bp[TC][VEC], zv[TC][VEC];
    {
      float rv[TC][VEC], iv[TC][VEC];
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        const int t = min(t0 + j, L - 1);
        ldv(rv[j], rgb + t * rg_rs);
        ldv(iv[j], rgb + t * rg_rs + H);
        ldv(bp[j], xcb + t * xc_rs);
        ldv(zv[j], zb + t * z_rs);
      }
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        const bool ok = t0 + j < L;
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const float a = fexp(nsp[v] * fsigm(rv[j][v]));
          const float beta = fsqrt(1.0f - a * a + 1e-8f) * fsigm(iv[j][v]);
          al[j][v] = ok ? a : 1.0f;
          bp[j][v] = ok ? beta * bp[j][v] : 0.0f;
        }
      }
    }
    float cin[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      float A = 1.0f, X = 0.0f;
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        X = X * al[j][v] + bp[j][v];
        A = A * al[j][v];
      }
#pragma unroll
      for (int k = 1; k < Q; k <<= 1) {
        const float Ap = __shfl_up(A, k * G, kWave);
        const float Xp = __shfl_up(X, k * G, kWave);
        if (q >= k) {
          X = Xp * A + X;
          A = Ap * A;
        }
      }
      float Ae = __shfl_up(A, G, kWave);
      float Xe = __shfl_up(X, G, kWave);
      if (q == 0) {
        Ae = 1.0f;
        Xe = 0.0f;
      }
      cin[v] = carry[v] * Ae + Xe;
      const float At = __shfl(A, (Q - 1) * G + g, kWave);
      const float Xt = __shfl(X, (Q - 1) * G + g, kWave);
      carry[v] = carry[v] * At + Xt;
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      float out[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        cin[v] = cin[v] * al[j][v] + bp[j][v];
        out[v] = fsilu(zv[j][v]) * cin[v];
      }
      if (cv && t0 + j < L) stv(yb + (t0 + j) * y_rs, out);
    }
  }
}

template <int VEC, int Q, int TC>
__global__ void __launch_bounds__(256)
k_gate_scan_bwd(const float* __restrict__ rg, int rg_rs, const float* __restrict__ xc, int xc_rs,
                const float* __restrict__ z, int z_rs, const float* __restrict__ lam,
                const float* __restrict__ carries, const float* __restrict__ dy,
                float* __restrict__ drg, int drg_rs, float* __restrict__ dxc,
                float* __restrict__ dz, int dz_rs, float* __restrict__ part,
                float* __restrict__ dh0_part, int64_t B, int L, int H, int ncw) {
  constexpr int G = kWave / Q;
  constexpr int TILE = Q * TC;
  static_assert(TILE == RB_TILE, "tile must match the carries checkpoint stride");
  const int lane = threadIdx.x & (kWave - 1);
  const int q = lane / G;
  const int g = lane - q * G;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = wid / ncw;
  if (b >= B) return;
  const int c0 = (int)(wid - b * ncw) * (G * VEC) + g * VEC;
  const bool cv = c0 < H;
  const int cc = cv ? c0 : 0;
  const int64_t row0 = b * L;
  const float* rgb = rg + row0 * rg_rs + cc;
  const float* xcb = xc + row0 * xc_rs + cc;
  const float* zb = z + row0 * z_rs + cc;
  const float* dyb = dy + row0 * H + cc;
  float* drgb = drg + row0 * drg_rs + cc;
  float* dxcb = dxc + row0 * H + cc;
  float* dzb = dz + row0 * dz_rs + cc;

  float lamv[VEC], nsp[VEC];
  ldv(lamv, lam + cc);
#pragma unroll
  for (int v = 0; v < VEC; ++v) nsp[v] = -softplus_f(lamv[v]);
  float ecarry[VEC], acc_v[VEC], acc_r[VEC], acc_i[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) ecarry[v] = acc_v[v] = acc_r[v] = acc_i[v] = 0.0f;

  const int nT = (L + TILE - 1) / TILE;
  for (int tile = nT - 1; tile >= 0; --tile) {
    const int t0 = tile * TILE + q * TC;
    float hcar[VEC];
    ldv(hcar, carries + (b * nT + tile) * H + cc);
    float rv[TC][VEC], iv[TC][VEC], xv[TC][VEC], zv[TC][VEC], gv[TC][VEC], al[TC][VEC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int t = min(t0 + j, L - 1);
      ldv(rv[j], rgb + t * rg_rs);
      ldv(iv[j], rgb + t * rg_rs + H);
      ldv(xv[j], xcb + t * xc_rs);
      ldv(zv[j], zb + t * z_rs);
      ldv(gv[j], dyb + t * H);
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const bool ok = t0 + j < L;
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const float a = fexp(nsp[v] * fsigm(rv[j][v]));
        al[j][v] = ok ? a : 1.0f;
        if (!ok) gv[j][v] = 0.0f;
      }
    }
    float cin[VEC], ein[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      // chunk summaries: forward (A, X) and reverse (A, E)
      float A = 1.0f, X = 0.0f, E = 0.0f;
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        const float a = al[j][v];
        const float bpj = (t0 + j < L)
            ? fsqrt(1.0f - a * a + 1e-8f) * fsigm(iv[j][v]) * xv[j][v] : 0.0f;
        X = X * a + bpj;
        A = A * a;
      }
#pragma unroll
      for (int j = TC - 1; j >= 0; --j) {
        const float d = E + gv[j][v] * fsilu(zv[j][v]);
        E = d * al[j][v];
      }
      // forward scan over earlier chunks -> carry into this chunk
      float Af = A, Xf = X;
#pragma unroll
      for (int k = 1; k < Q; k <<= 1) {
        const float Ap = __shfl_up(Af, k * G, kWave);
        const float Xp = __shfl_up(Xf, k * G, kWave);
        if (q >= k) {
          Xf = Xp * Af + Xf;
          Af = Ap * Af;
        }
      }
      float Ae = __shfl_up(Af, G, kWave);
      float Xe = __shfl_up(Xf, G, kWave);
      if (q == 0) {
        Ae = 1.0f;
        Xe = 0.0f;
      }
      cin[v] = hcar[v] * Ae + Xe;
      // reverse scan over later chunks -> adjoint flowing into this chunk
      float Ab = A, Eb = E;
#pragma unroll
      for (int k = 1; k < Q; k <<= 1) {
        const float An = __shfl_down(Ab, k * G, kWave);
        const float En = __shfl_down(Eb, k * G, kWave);
        if (q + k < Q) {
          Eb = En * Ab + Eb;
          Ab = An * Ab;
        }
      }
      float Ase = __shfl_down(Ab, G, kWave);
      float Ese = __shfl_down(Eb, G, kWave);
      if (q == Q - 1) {
        Ase = 1.0f;
        Ese = 0.0f;
      }
      ein[v] = ecarry[v] * Ase + Ese;
      const float At = __shfl(Ab, g, kWave);
      const float Et = __shfl(Eb, g, kWave);
      ecarry[v] = ecarry[v] * At + Et;
    }
    // recompute h (h_{t-1} for the scan gradient, h_t for dz)
    float hp[TC][VEC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const bool ok = t0 + j < L;
      float dzo[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const float a = al[j][v];
        const float bpj = ok ? fsqrt(1.0f - a * a + 1e-8f) * fsigm(iv[j][v]) * xv[j][v] : 0.0f;
        hp[j][v] = cin[v];
        cin[v] = cin[v] * a + bpj;
        dzo[v] = (gv[j][v] * cin[v]) * fdsilu(zv[j][v]);
      }
      if (cv && ok) stv(dzb + (t0 + j) * dz_rs, dzo);
    }
#pragma unroll
    for (int j = TC - 1; j >= 0; --j) {
      const bool ok = t0 + j < L;
      float dro[VEC], dio[VEC], dxo[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const float a = al[j][v];
        const float d = ein[v] + gv[j][v] * fsilu(zv[j][v]);   // dL/dh_t
        const float sr = fsigm(rv[j][v]);
        const float si = fsigm(iv[j][v]);
        const float sq = fsqrt(1.0f - a * a + 1e-8f);
        const float dbeta = d * xv[j][v];
        const float du = (dbeta * si) * (0.5f * frcp(sq));
        const float da = hp[j][v] * d + (-du) * (2.0f * a);
        const float dv = da * a;
        dro[v] = (dv * nsp[v]) * ((1.0f - sr) * sr);
        dio[v] = (dbeta * sq) * ((1.0f - si) * si);
        dxo[v] = d * (sq * si);
        if (ok) {
          acc_v[v] = acc_v[v] + dv * sr;
          acc_r[v] = acc_r[v] + dro[v];
          acc_i[v] = acc_i[v] + dio[v];
        }
        ein[v] = d * a;
      }
      if (cv && ok) {
        const int t = t0 + j;
        stv(drgb + t * drg_rs, dro);
        stv(drgb + t * drg_rs + H, dio);
        stv(dxcb + t * H, dxo);
      }
    }
    if (tile == 0 && q == 0 && cv) stv(dh0_part + b * H + c0, ein);
  }
  // per-channel partial sums: butterfly over the Q lanes sharing the channels
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
#pragma unroll
    for (int k = G; k < kWave; k <<= 1) {
      acc_v[v] += __shfl_xor(acc_v[v], k, kWave);
      acc_r[v] += __shfl_xor(acc_r[v], k, kWave);
      acc_i[v] += __shfl_xor(acc_i[v], k, kWave);
    }
    // Lambda enters as -softplus(Lambda): dLambda = -sum(dv * sr) * softplus'(Lambda)
    acc_v[v] = -acc_v[v] * dsoftplus_f(lamv[v]);
  }
  if (q == 0 && cv) {
    stv(part + b * H + c0, acc_v);
    stv(part + (B + b) * H + c0, acc_r);
    stv(part + (2 * B + b) * H + c0, acc_i);
  }
}

// forward: 4 chunks x 4 steps, 16 lanes x 4 channels = 64 channels per wave
constexpr int kFwdQ = 4, kFwdTC = RB_TILE / kFwdQ;
// backward holds ~7 values per (step, channel): 8 chunks x 2 steps, 32 channels/wave
constexpr int kBwdQ = 8, kBwdTC = RB_TILE / kBwdQ;

}  // namespace

int launch_gate_fwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                    const float* z, int64_t z_rs, const float* lam, const float* h0, float* y,
                    int64_t y_rs, float* carries, int64_t B, int64_t L, int64_t H,
                    hipStream_t st) {
  const bool vec = H % 4 == 0 && rg_rs % 4 == 0 && xc_rs % 4 == 0 && z_rs % 4 == 0 &&
                   y_rs % 4 == 0 && aligned16(rg) && aligned16(xc) && aligned16(z) &&
                   aligned16(y) && aligned16(lam) && (h0 == nullptr || aligned16(h0)) &&
                   (carries == nullptr || aligned16(carries));
  const int V = vec ? 4 : 1;
  const int span = (kWave / kFwdQ) * V;
  const int ncw = (int)((H + span - 1) / span);
  const int64_t blocks = (B * ncw + 3) / 4;
  if (vec)
    hipLaunchKernelGGL((k_gate_scan_fwd<4, kFwdQ, kFwdTC>), dim3((unsigned)blocks), dim3(256), 0,
                       st, rg, (int)rg_rs, xc, (int)xc_rs, z, (int)z_rs, lam, h0, y, (int)y_rs,
                       carries, B, (int)L, (int)H, ncw);
  else
    hipLaunchKernelGGL((k_gate_scan_fwd<1, kFwdQ, kFwdTC>), dim3((unsigned)blocks), dim3(256), 0,
                       st, rg, (int)rg_rs, xc, (int)xc_rs, z, (int)z_rs, lam, h0, y, (int)y_rs,
                       carries, B, (int)L, (int)H, ncw);
  return launch_status("rb_gate_scan_fwd");
}

int launch_gate_bwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                    const float* z, int64_t z_rs, const float* lam, const float* carries,
                    const float* dy, float* drg, int64_t drg_rs, float* dxc, float* dz,
                    int64_t dz_rs, float* part, float* dh0_part, int64_t B, int64_t L,
                    int64_t H, hipStream_t st) {
  const bool vec = H % 4 == 0 && rg_rs % 4 == 0 && xc_rs % 4 == 0 && z_rs % 4 == 0 &&
                   drg_rs % 4 == 0 && dz_rs % 4 == 0 && aligned16(rg) && aligned16(xc) &&
                   aligned16(z) && aligned16(lam) && aligned16(carries) && aligned16(dy) &&
                   aligned16(drg) && aligned16(dxc) && aligned16(dz) && aligned16(part) &&
                   aligned16(dh0_part);
  const int V = vec ? 4 : 1;
  const int span = (kWave / kBwdQ) * V;
  const int ncw = (int)((H + span - 1) / span);
  const int64_t blocks = (B * ncw + 3) / 4;
  if (vec)
    hipLaunchKernelGGL((k_gate_scan_bwd<4, kBwdQ, kBwdTC>), dim3((unsigned)blocks), dim3(256), 0,
                       st, rg, (int)rg_rs, xc, (int)xc_rs, z, (int)z_rs, lam, carries, dy, drg,
                       (int)drg_rs, dxc, dz, (int)dz_rs, part, dh0_part, B, (int)L, (int)H, ncw);
  else
    hipLaunchKernelGGL((k_gate_scan_bwd<1, kBwdQ, kBwdTC>), dim3((unsigned)blocks), dim3(256), 0,
                       st, rg, (int)rg_rs, xc, (int)xc_rs, z, (int)z_rs, lam, carries, dy, drg,
                       (int)drg_rs, dxc, dz, (int)dz_rs, part, dh0_part, B, (int)L, (int)H, ncw);
  return launch_status("rb_gate_scan_bwd");
}

}  // namespace rb
