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

#include <initializer_list>

namespace rb {
namespace {

template <typename T, int VEC, int TC>
struct FwdIn {
  RawVec<T, VEC> r[TC], i[TC], x[TC], z[TC];
};

// backward operands as loaded: raw storage words (bf16 stays packed until the
// tile is processed, so a prefetched tile costs half the registers)
template <typename T, int VEC, int TC>
struct BwdIn {
  RawVec<T, VEC> r[TC], i[TC], x[TC], z[TC], g[TC];
};

// PF: software-prefetch the next tile's operands before computing this one
// (two register buffers), so a wave keeps its loads in flight across the
// shuffle/compute/store phase of the previous tile.
template <typename T, int VEC, int Q, int TC, bool PF>
__global__ void __launch_bounds__(256)
k_gate_scan_fwd(const T* __restrict__ rg, int rg_rs, const T* __restrict__ xc, int xc_rs,
                const T* __restrict__ z, int z_rs, const float* __restrict__ lam,
                const float* __restrict__ gbias, const float* __restrict__ h0, int h0_bs,
                T* __restrict__ y, int y_rs,
                float* __restrict__ carries, int64_t B, int Lmax, int H, int ncw,
                const int64_t* __restrict__ offs, T* __restrict__ y_last,
                const int64_t* __restrict__ order) {
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
  // dense rows (b, t) at b * Lmax + t, or packed variable-length sequences:
  // sequence b at rows offs[b] .. offs[b+1] (wave-uniform)
  int64_t row0;
  int L;
  if (offs != nullptr) {
    row0 = offs[b];
    L = (int)(offs[b + 1] - row0);
  } else {
    row0 = b * Lmax;
    L = Lmax;
  }
  const T* rgb = rg + row0 * rg_rs + cc;
  const T* xcb = xc + row0 * xc_rs + cc;
  const T* zb = z + row0 * z_rs + cc;
  T* yb = y + row0 * y_rs + cc;

  float nsp[VEC], carry[VEC], br[VEC], bi[VEC];
  ldc(nsp, lam + cc);
#pragma unroll
  for (int v = 0; v < VEC; ++v) nsp[v] = -softplus_f(nsp[v]);
  if (gbias != nullptr) {   // the gates GEMM's bias, added here instead of in its epilogue
    ldc(br, gbias + cc);
    ldc(bi, gbias + H + cc);
  } else {
#pragma unroll
    for (int v = 0; v < VEC; ++v) br[v] = bi[v] = 0.0f;
  }
  if (h0 != nullptr) {
    ldc(carry, h0 + b * h0_bs + cc);
  } else {
#pragma unroll
    for (int v = 0; v < VEC; ++v) carry[v] = 0.0f;
  }
  const int nT = (L + TILE - 1) / TILE;          // tiles of this row
  const int nTc = (Lmax + TILE - 1) / TILE;      // carries row stride

  auto load = [&](FwdIn<T, VEC, TC>& in, int tile) {
    const int t0 = tile * TILE + q * TC;
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int t = min(t0 + j, L - 1);
      ld_raw(in.r[j], rgb + t * rg_rs);
      ld_raw(in.i[j], rgb + t * rg_rs + H);
      ld_raw(in.x[j], xcb + t * xc_rs);
      ld_raw(in.z[j], zb + t * z_rs);
    }
  };
  auto process = [&](const FwdIn<T, VEC, TC>& raw, int tile) {
    struct {
      float r[TC][VEC], i[TC][VEC], x[TC][VEC], z[TC][VEC];
    } in;
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      unpack_raw(in.r[j], raw.r[j]);
      unpack_raw(in.i[j], raw.i[j]);
      unpack_raw(in.x[j], raw.x[j]);
      unpack_raw(in.z[j], raw.z[j]);
    }
    if (carries != nullptr && q == 0 && cv) stv(carries + (b * nTc + tile) * H + c0, carry);
    const int t0 = tile * TILE + q * TC;
    // in.r <- alpha, in.x <- b' = beta * xc
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const bool ok = t0 + j < L;
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const float a = fexp(nsp[v] * fsigm(in.r[j][v] + br[v]));
        const float beta = fsqrt(1.0f - a * a + 1e-8f) * fsigm(in.i[j][v] + bi[v]);
        in.r[j][v] = ok ? a : 1.0f;
        in.x[j][v] = ok ? beta * in.x[j][v] : 0.0f;
      }
    }
    float cin[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      float A = 1.0f, X = 0.0f;
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        X = X * in.r[j][v] + in.x[j][v];
        A = A * in.r[j][v];
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
        cin[v] = cin[v] * in.r[j][v] + in.x[j][v];
        out[v] = fsilu(in.z[j][v]) * cin[v];
      }
      if (y_last != nullptr) {   // only each sequence's last position is kept: [B, H]
        if (cv && t0 + j == L - 1) stv(y_last + (order ? order[b] : b) * H + c0, out);
      } else if (cv && t0 + j < L) {
        stv(yb + (t0 + j) * y_rs, out);
      }
    }
  };

  FwdIn<T, VEC, TC> bufA, bufB;
  if constexpr (PF) {
    load(bufA, 0);
    for (int tile = 0; tile < nT; tile += 2) {
      if (tile + 1 < nT) load(bufB, tile + 1);
      process(bufA, tile);
      if (tile + 1 < nT) {
        if (tile + 2 < nT) load(bufA, tile + 2);
        process(bufB, tile + 1);
      }
    }
  } else {
    for (int tile = 0; tile < nT; ++tile) {
      load(bufA, tile);
      process(bufA, tile);
    }
  }
}

// Cross-chunk scans of the backward: the Q time chunks of a channel group sit
// on Q consecutive lanes, so "value of chunk q-k / q+k" is a DPP row shift
// (VALU, no LDS round trip as with ds_bpermute) and "chunk 0's value" a
// ds_swizzle broadcast.  Lanes whose source crosses a group edge get a wrong
// value that the callers never use (they mask with q >= k / q + k < Q).
template <int K>
__device__ __forceinline__ float dpp_from_lower(float x) {   // lane i - K, K in 1..8
  static_assert(K >= 1 && K <= 8, "row shift within a 16-lane DPP row");
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x),
                                                    0x110 + K, 0xF, 0xF, false));
}
template <int K>
__device__ __forceinline__ float dpp_from_upper(float x) {   // lane i + K
  static_assert(K >= 1 && K <= 8, "row shift within a 16-lane DPP row");
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x),
                                                    0x100 + K, 0xF, 0xF, false));
}
template <int Q>
__device__ __forceinline__ float group_first(float x) {      // lane i & ~(Q - 1)
  static_assert(Q >= 2 && Q <= 32 && (Q & (Q - 1)) == 0, "power-of-two groups within 32 lanes");
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x1F & ~(Q - 1)));
}
// inclusive scans of (A, X) pairs over the Q chunk lanes: from lower chunks
// (X = X_lower * A + X, A = A_lower * A) and from upper chunks (reverse)
template <int Q, int K = 1>
__device__ __forceinline__ void scan_from_lower(float& A, float& X, int q) {
  if constexpr (K < Q) {
    const float Ap = dpp_from_lower<K>(A);
    const float Xp = dpp_from_lower<K>(X);
    if (q >= K) {
      X = Xp * A + X;
      A = Ap * A;
    }
    scan_from_lower<Q, 2 * K>(A, X, q);
  }
}
template <int Q, int K = 1>
__device__ __forceinline__ void scan_from_upper(float& A, float& E, int q) {
  if constexpr (K < Q) {
    const float An = dpp_from_upper<K>(A);
    const float En = dpp_from_upper<K>(E);
    if (q + K < Q) {
      E = En * A + E;
      A = An * A;
    }
    scan_from_upper<Q, 2 * K>(A, E, q);
  }
}

template <typename T, int VEC, int Q, int TC, bool PF, int VH = VEC>
__global__ void __launch_bounds__(256, VH < VEC ? 2 : 1)   // channel passes: 2 waves per SIMD
k_gate_scan_bwd(const T* __restrict__ rg, int rg_rs, const T* __restrict__ xc, int xc_rs,
                const T* __restrict__ z, int z_rs, const float* __restrict__ lam,
                const float* __restrict__ gbias, const float* __restrict__ carries,
                const T* __restrict__ dy,
                T* __restrict__ drg, int drg_rs, T* __restrict__ dxc, int dxc_rs,
                T* __restrict__ dz, int dz_rs, float* __restrict__ part,
                float* __restrict__ dh0_part, int64_t B, int Lmax, int H, int ncw,
                const int64_t* __restrict__ offs, int pair, const T* __restrict__ dy_last,
                const int64_t* __restrict__ order) {
  constexpr int G = kWave / Q;
  constexpr int TILE = Q * TC;
  static_assert(TILE == RB_TILE, "tile must match the carries checkpoint stride");
  const int lane = threadIdx.x & (kWave - 1);
  const int q = lane & (Q - 1);   // time chunk on the low lane bits (scans: DPP)
  const int g = lane / Q;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  // pair: the wave walks sequence bw and then sequence B-1-bw (packed batches
  // are sorted longest first, so every wave gets about the same number of
  // tiles and pays its per-wave prologue/epilogue once for two sequences)
  const int64_t bw = wid / ncw;
  if (bw >= (pair ? (B + 1) / 2 : B)) return;
  const int c0 = (int)(wid - bw * ncw) * (G * VEC) + g * VEC;
  const bool cv = c0 < H;
  const int cc = cv ? c0 : 0;
  // dense rows (b, t) at b * Lmax + t, or packed variable-length sequences:
  // sequence b at rows offs[b] .. offs[b+1] (wave-uniform)
  int64_t b = bw, row0 = 0, bl = bw;   // bl: the batch row of dy_last
  int L = 0;
  const T *rgb = nullptr, *xcb = nullptr, *zb = nullptr, *dyb = nullptr;
  T *drgb = nullptr, *dxcb = nullptr, *dzb = nullptr;
  auto bind = [&](int64_t bs) {
    b = bs;
    bl = order != nullptr ? order[bs] : bs;
    if (offs != nullptr) {
      row0 = offs[b];
      L = (int)(offs[b + 1] - row0);
    } else {
      row0 = b * Lmax;
      L = Lmax;
    }
    rgb = rg + row0 * rg_rs + cc;
    xcb = xc + row0 * xc_rs + cc;
    zb = z + row0 * z_rs + cc;
    dyb = dy + row0 * H + cc;
    drgb = drg + row0 * drg_rs + cc;
    dxcb = dxc + row0 * dxc_rs + cc;
    dzb = dz + row0 * dz_rs + cc;
  };

  float lamv[VEC], nsp[VEC], br[VEC], bi[VEC];
  ldc(lamv, lam + cc);
#pragma unroll
  for (int v = 0; v < VEC; ++v) nsp[v] = -softplus_f(lamv[v]);
  if (gbias != nullptr) {
    ldc(br, gbias + cc);
    ldc(bi, gbias + H + cc);
  } else {
#pragma unroll
    for (int v = 0; v < VEC; ++v) br[v] = bi[v] = 0.0f;
  }
  float ecarry[VEC], acc_v[VEC], acc_r[VEC], acc_i[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) acc_v[v] = acc_r[v] = acc_i[v] = 0.0f;
  const int nTc = (Lmax + TILE - 1) / TILE;      // carries row stride

  auto load = [&](BwdIn<T, VEC, TC>& in, int tile) {
    const int t0 = tile * TILE + q * TC;
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int t = min(t0 + j, L - 1);
      ld_raw(in.r[j], rgb + t * rg_rs);
      ld_raw(in.i[j], rgb + t * rg_rs + H);
      ld_raw(in.x[j], xcb + t * xc_rs);
      ld_raw(in.z[j], zb + t * z_rs);
      if (dy_last == nullptr) {
        ld_raw(in.g[j], dyb + t * H);
      } else if (t == L - 1) {   // dy is zero except at each sequence's last position
        ld_raw(in.g[j], dy_last + bl * H + cc);
      } else {
        zero_raw(in.g[j]);
      }
    }
  };
  // VH < VEC: the tile's math runs VH channels at a time (the per-channel
  // recurrences are independent; the same operations in the same order, so
  // bit-identical), its results collected in storage format and stored as
  // VEC-wide vectors after the last pass — a third of the live registers.
  constexpr bool SPLIT = VH < VEC;
  static_assert(VEC % VH == 0 && (!SPLIT || VH % 2 == 0), "channel passes");
  auto process = [&](const BwdIn<T, VEC, TC>& raw, int tile) {
    float hcar[VEC];
    ldc(hcar, carries + (b * nTc + tile) * H + cc);
    const int t0 = tile * TILE + q * TC;
    RawVec<T, VEC> odz[SPLIT ? TC : 1], odr[SPLIT ? TC : 1], odi[SPLIT ? TC : 1],
        odx[SPLIT ? TC : 1];
#pragma unroll
    for (int h0 = 0; h0 < VEC; h0 += VH) {
      struct {
        float r[TC][VH], i[TC][VH], x[TC][VH], z[TC][VH], g[TC][VH];
      } in;
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        // (channel passes: this pass's words through an empty volatile asm,
        // ordered after the previous pass's results below, so the compiler
        // cannot interleave the passes and the register saving is real)
        RawVec<T, VEC> wr = raw.r[j], wi = raw.i[j], wx = raw.x[j], wz = raw.z[j], wg = raw.g[j];
        if constexpr (SPLIT) {
          opaque_part<VH>(wr, h0);
          opaque_part<VH>(wi, h0);
          opaque_part<VH>(wx, h0);
          opaque_part<VH>(wz, h0);
          opaque_part<VH>(wg, h0);
        }
        unpack_part(in.r[j], wr, h0);
        unpack_part(in.i[j], wi, h0);
        unpack_part(in.x[j], wx, h0);
        unpack_part(in.z[j], wz, h0);
        unpack_part(in.g[j], wg, h0);
      }
#pragma unroll
      for (int j = 0; j < TC; ++j)
#pragma unroll
        for (int v = 0; v < VH; ++v) {
          in.r[j][v] += br[h0 + v];
          in.i[j][v] += bi[h0 + v];
        }
      // per-step derived values, each transcendental evaluated once
      float al[TC][VH], sr[TC][VH], si[TC][VH], sq[TC][VH], bp[TC][VH], gs[TC][VH],
          dsz[TC][VH];
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        const bool ok = t0 + j < L;
#pragma unroll
        for (int v = 0; v < VH; ++v) {
          sr[j][v] = fsigm(in.r[j][v]);
          const float a = ok ? fexp(nsp[h0 + v] * sr[j][v]) : 1.0f;
          al[j][v] = a;
          si[j][v] = fsigm(in.i[j][v]);
          sq[j][v] = fsqrt(1.0f - a * a + 1e-8f);
          bp[j][v] = ok ? sq[j][v] * si[j][v] * in.x[j][v] : 0.0f;
          const float zz = in.z[j][v];
          const float sz = fsigm(zz);
          const float g = ok ? in.g[j][v] : 0.0f;   // dy past the end contributes nothing
          in.g[j][v] = g;
          gs[j][v] = g * (zz * sz);
          dsz[j][v] = sz * (1.0f + zz * (1.0f - sz));
        }
      }
      float cin[VH], ein[VH];
#pragma unroll
      for (int v = 0; v < VH; ++v) {
        float A = 1.0f, X = 0.0f, E = 0.0f;
#pragma unroll
        for (int j = 0; j < TC; ++j) {
          X = X * al[j][v] + bp[j][v];
          A = A * al[j][v];
        }
#pragma unroll
        for (int j = TC - 1; j >= 0; --j) {
          const float d = E + gs[j][v];
          E = d * al[j][v];
        }
        float Af = A, Xf = X;
        scan_from_lower<Q>(Af, Xf, q);
        float Ae = dpp_from_lower<1>(Af);
        float Xe = dpp_from_lower<1>(Xf);
        if (q == 0) {
          Ae = 1.0f;
          Xe = 0.0f;
        }
        cin[v] = hcar[h0 + v] * Ae + Xe;
        float Ab = A, Eb = E;
        scan_from_upper<Q>(Ab, Eb, q);
        float Ase = dpp_from_upper<1>(Ab);
        float Ese = dpp_from_upper<1>(Eb);
        if (q == Q - 1) {
          Ase = 1.0f;
          Ese = 0.0f;
        }
        ein[v] = ecarry[h0 + v] * Ase + Ese;
        const float At = group_first<Q>(Ab);
        const float Et = group_first<Q>(Eb);
        ecarry[h0 + v] = ecarry[h0 + v] * At + Et;
      }
      float hp[TC][VH];
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        const bool ok = t0 + j < L;
        float dzo[VH];
#pragma unroll
        for (int v = 0; v < VH; ++v) {
          hp[j][v] = cin[v];
          cin[v] = cin[v] * al[j][v] + bp[j][v];
          dzo[v] = (in.g[j][v] * cin[v]) * dsz[j][v];
        }
        if constexpr (SPLIT) pack_part(odz[j], dzo, h0);
        else if (cv && ok) stv(dzb + (t0 + j) * dz_rs, dzo);
      }
#pragma unroll
      for (int j = TC - 1; j >= 0; --j) {
        const bool ok = t0 + j < L;
        float dro[VH], dio[VH], dxo[VH];
#pragma unroll
        for (int v = 0; v < VH; ++v) {
          const float a = al[j][v];
          const float d = ein[v] + gs[j][v];   // dL/dh_t
          const float dbeta = d * in.x[j][v];
          const float du = (dbeta * si[j][v]) * (0.5f * frcp(sq[j][v]));
          const float da = hp[j][v] * d + (-du) * (2.0f * a);
          const float dv = da * a;
          dro[v] = (dv * nsp[h0 + v]) * ((1.0f - sr[j][v]) * sr[j][v]);
          dio[v] = (dbeta * sq[j][v]) * ((1.0f - si[j][v]) * si[j][v]);
          dxo[v] = d * (sq[j][v] * si[j][v]);
          acc_v[h0 + v] = acc_v[h0 + v] + (ok ? dv * sr[j][v] : 0.0f);
          acc_r[h0 + v] = acc_r[h0 + v] + (ok ? dro[v] : 0.0f);
          acc_i[h0 + v] = acc_i[h0 + v] + (ok ? dio[v] : 0.0f);
          ein[v] = d * a;
        }
        if constexpr (SPLIT) {
          pack_part(odr[j], dro, h0);
          pack_part(odi[j], dio, h0);
          pack_part(odx[j], dxo, h0);
        } else if (cv && ok) {
          const int t = t0 + j;
          stv(drgb + t * drg_rs, dro);
          stv(drgb + t * drg_rs + H, dio);
          stv(dxcb + t * dxc_rs, dxo);
        }
      }
      if (tile == 0 && q == 0 && cv) stv(dh0_part + b * H + c0 + h0, ein);
      if constexpr (SPLIT) {   // the pass's results exist before the next pass starts
#pragma unroll
        for (int j = 0; j < TC; ++j) {
          opaque_part<VH>(odz[j], h0);
          opaque_part<VH>(odr[j], h0);
          opaque_part<VH>(odi[j], h0);
          opaque_part<VH>(odx[j], h0);
        }
#pragma unroll
        for (int v = 0; v < VH; ++v)
          asm volatile("" : "+v"(ecarry[h0 + v]), "+v"(acc_v[h0 + v]), "+v"(acc_r[h0 + v]),
                       "+v"(acc_i[h0 + v]));
      }
    }
    if constexpr (SPLIT) {
#pragma unroll
      for (int j = 0; j < TC; ++j)
        if (cv && t0 + j < L) stv_raw(dzb + (t0 + j) * dz_rs, odz[j]);
#pragma unroll
      for (int j = TC - 1; j >= 0; --j) {
        if (cv && t0 + j < L) {
          const int t = t0 + j;
          stv_raw(drgb + t * drg_rs, odr[j]);
          stv_raw(drgb + t * drg_rs + H, odi[j]);
          stv_raw(dxcb + t * dxc_rs, odx[j]);
        }
      }
    }
  };

  BwdIn<T, VEC, TC> bufA, bufB;
  const int nseq = (pair && B - 1 - bw != bw) ? 2 : 1;
  for (int sq_i = 0; sq_i < nseq; ++sq_i) {
    bind(sq_i == 0 ? bw : B - 1 - bw);
    const int nT = (L + TILE - 1) / TILE;          // tiles of this row
#pragma unroll
    for (int v = 0; v < VEC; ++v) ecarry[v] = 0.0f;
    if constexpr (PF) {
      if (nT > 0) load(bufA, nT - 1);
      for (int tile = nT - 1; tile >= 0; tile -= 2) {
        if (tile - 1 >= 0) load(bufB, tile - 1);
        process(bufA, tile);
        if (tile - 1 >= 0) {
          if (tile - 2 >= 0) load(bufA, tile - 2);
          process(bufB, tile - 1);
        }
      }
    } else {
      for (int tile = nT - 1; tile >= 0; --tile) {
        load(bufA, tile);
        process(bufA, tile);
      }
    }
    if (nT == 0 && q == 0 && cv) stv(dh0_part + b * H + c0, ecarry);   // empty row: zeros
  }
  // per-channel partial sums: butterfly over the Q lanes sharing the channels
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
#pragma unroll
    for (int k = 1; k < Q; k <<= 1) {   // the Q chunk lanes of this channel group
      acc_v[v] += __shfl_xor(acc_v[v], k, kWave);
      acc_r[v] += __shfl_xor(acc_r[v], k, kWave);
      acc_i[v] += __shfl_xor(acc_i[v], k, kWave);
    }
    // Lambda enters as -softplus(Lambda): dLambda = -sum(dv * sr) * softplus'(Lambda)
    acc_v[v] = -acc_v[v] * dsoftplus_f(lamv[v]);
  }
  if (q == 0 && cv) {
    stv(part + bw * H + c0, acc_v);
    stv(part + (B + bw) * H + c0, acc_r);
    stv(part + (2 * B + bw) * H + c0, acc_i);
    if (nseq == 2) {   // the partner's rows of the per-row partial sums: zeros
      const int64_t bp = B - 1 - bw;
      float zero[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) zero[v] = 0.0f;
      stv(part + bp * H + c0, zero);
      stv(part + (B + bp) * H + c0, zero);
      stv(part + (2 * B + bp) * H + c0, zero);
    }
  }
}

// Tuned on MI355X at B=2048, L=200, H=256 (tools/kbench.hip): the forward
// runs 4 chunks x 4 steps with 2 channels per lane and a one-tile register
// prefetch; the backward (about 7 live values per step and channel) 8 chunks
// x 2 steps with 4 channels per lane.  Both sit at the data-movement ceiling
// of their read/write mix (a copy kernel with the same 4R+1W pattern and no
// math runs at the same rate).
constexpr int kFwdQ = 4, kFwdTC = RB_TILE / kFwdQ;
constexpr int kBwdQ = 8, kBwdTC = RB_TILE / kBwdQ;
constexpr bool kBwdPair = true;   // packed batches: a long and a short sequence per wave

// alignment/stride check for VEC-wide access: activation pointers (T) need
// sizeof(T)*V-byte alignment, the fp32 per-channel vectors 4*V
template <typename T, int V>
bool vec_ok(int64_t H, std::initializer_list<int64_t> strides,
            std::initializer_list<const void*> act, std::initializer_list<const void*> f32) {
  if (H % V) return false;
  for (int64_t s : strides)
    if (s % V) return false;
  for (const void* p : act)
    if (p != nullptr && (reinterpret_cast<uintptr_t>(p) % (sizeof(T) * V))) return false;
  for (const void* p : f32)
    if (p != nullptr && (reinterpret_cast<uintptr_t>(p) % (4 * V))) return false;
  return true;
}

template <typename T, int V, bool PF = true>
int gate_fwd_v(const T* rg, int64_t rg_rs, const T* xc, int64_t xc_rs, const T* z,
               int64_t z_rs, const float* lam, const float* gb, const float* h0, int64_t h0_bs,
               T* y, int64_t y_rs, float* carries, int64_t B, int64_t L, int64_t H,
               const int64_t* offs, hipStream_t st, T* y_last, const int64_t* order = nullptr) {
  const int span = (kWave / kFwdQ) * V;
  const int ncw = (int)((H + span - 1) / span);
  const int64_t blocks = (B * ncw + 3) / 4;
  hipLaunchKernelGGL((k_gate_scan_fwd<T, V, kFwdQ, kFwdTC, PF>), dim3((unsigned)blocks),
                     dim3(256), 0, st, rg, (int)rg_rs, xc, (int)xc_rs, z, (int)z_rs, lam, gb,
                     h0, (int)h0_bs, y, (int)y_rs, carries, B, (int)L, (int)H, ncw, offs, y_last, order);
  return launch_status("rb_gate_scan_fwd");
}

template <typename T, int V, int Q = kBwdQ, int TC = kBwdTC, bool PF = false, int VH = V>
int gate_bwd_v(const T* rg, int64_t rg_rs, const T* xc, int64_t xc_rs, const T* z,
               int64_t z_rs, const float* lam, const float* gb, const float* carries,
               const T* dy, T* drg, int64_t drg_rs, T* dxc, int64_t dxc_rs, T* dz, int64_t dz_rs,
               float* part, float* dh0_part, int64_t B, int64_t L, int64_t H, const int64_t* offs,
               hipStream_t st, const T* dy_last, const int64_t* order = nullptr) {
  const int span = (kWave / Q) * V;
  const int ncw = (int)((H + span - 1) / span);
  // packed (variable-length, longest-first) batches: one wave per sequence pair
  const int pair = offs != nullptr && kBwdPair;
  const int64_t Bw = pair ? (B + 1) / 2 : B;
  const int64_t blocks = (Bw * ncw + 3) / 4;
  hipLaunchKernelGGL((k_gate_scan_bwd<T, V, Q, TC, PF, VH>), dim3((unsigned)blocks),
                     dim3(256), 0, st, rg, (int)rg_rs, xc, (int)xc_rs, z, (int)z_rs, lam, gb,
                     carries, dy, drg, (int)drg_rs, dxc, (int)dxc_rs, dz, (int)dz_rs, part,
                     dh0_part, B, (int)L, (int)H, ncw, offs, pair, dy_last, order);
  return launch_status("rb_gate_scan_bwd");
}

// widest vector the layout allows: fp32 fwd 2 / bwd 4 channels per lane
// (8 / 16 B); bf16 4 / 4 channels (8 / 8 B)
template <typename T>
int gate_fwd_t(const T* rg, int64_t rg_rs, const T* xc, int64_t xc_rs, const T* z,
               int64_t z_rs, const float* lam, const float* gb, const float* h0, int64_t h0_bs,
               T* y, int64_t y_rs, float* carries, int64_t B, int64_t L, int64_t H,
               const int64_t* offs, hipStream_t st, T* y_last, const int64_t* order) {
  constexpr int VW = sizeof(T) == 2 ? 4 : 2;
  const auto strides = {rg_rs, xc_rs, z_rs, y_rs, h0_bs};
  const auto act = {(const void*)rg, (const void*)xc, (const void*)z, (const void*)y,
                    (const void*)y_last};
  const auto f32 = {(const void*)lam, (const void*)gb, (const void*)h0, (const void*)carries};
  // bf16: no register prefetch (measured 3% faster at config 5, tools/kbench.hip)
  if (vec_ok<T, VW>(H, strides, act, f32))
    return gate_fwd_v<T, VW, sizeof(T) == 4>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, h0, h0_bs,
                                             y, y_rs, carries, B, L, H, offs, st, y_last, order);
  if (vec_ok<T, 2>(H, strides, act, f32))
    return gate_fwd_v<T, 2>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, h0, h0_bs, y, y_rs, carries,
                            B, L, H, offs, st, y_last, order);
  return gate_fwd_v<T, 1>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, h0, h0_bs, y, y_rs, carries, B,
                          L, H, offs, st, y_last, order);
}

template <typename T>
int gate_bwd_t(const T* rg, int64_t rg_rs, const T* xc, int64_t xc_rs, const T* z,
               int64_t z_rs, const float* lam, const float* gb, const float* carries,
               const T* dy, T* drg, int64_t drg_rs, T* dxc, int64_t dxc_rs, T* dz, int64_t dz_rs,
               float* part, float* dh0_part, int64_t B, int64_t L, int64_t H, const int64_t* offs,
               hipStream_t st, const T* dy_last, const int64_t* order) {
  constexpr int VW = 4;
  const auto strides = {rg_rs, xc_rs, z_rs, drg_rs, dxc_rs, dz_rs};
  const auto act = {(const void*)rg, (const void*)xc, (const void*)z, (const void*)dy,
                    (const void*)drg, (const void*)dxc, (const void*)dz, (const void*)dy_last};
  const auto f32 = {(const void*)lam, (const void*)gb, (const void*)carries, (const void*)part,
                    (const void*)dh0_part};
  // bf16 (configs[4], L = 2048): 4 chunks x 4 steps (128-B row pieces per
  // wave), the tile's math in two passes of 2 channels so the kernel fits 256
  // registers: 2 waves per SIMD hide the loads that one wave with a register
  // prefetch of the next tile (417 registers, round 1-4) could not —
  // 3.89 vs 4.37 ms at configs[4], bit-identical (tools/gate_bf16_probe.hip,
  // profiles/r05_gb_probe.txt)
  if constexpr (sizeof(T) == 2) {
    if (vec_ok<T, VW>(H, strides, act, f32))
      return gate_bwd_v<T, VW, 4, 4, false, 2>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, carries,
                                               dy, drg, drg_rs, dxc, dxc_rs, dz, dz_rs, part,
                                               dh0_part, B, L, H, offs, st, dy_last, order);
  }
  if (vec_ok<T, VW>(H, strides, act, f32)) {
    return gate_bwd_v<T, VW>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, carries, dy, drg, drg_rs,
                             dxc, dxc_rs, dz, dz_rs, part, dh0_part, B, L, H, offs, st, dy_last, order);
  }
  if (vec_ok<T, 2>(H, strides, act, f32))
    return gate_bwd_v<T, 2>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, carries, dy, drg, drg_rs,
                            dxc, dxc_rs, dz, dz_rs, part, dh0_part, B, L, H, offs, st, dy_last, order);
  return gate_bwd_v<T, 1>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, carries, dy, drg, drg_rs, dxc,
                          dxc_rs, dz, dz_rs, part, dh0_part, B, L, H, offs, st, dy_last, order);
}

}  // namespace

int launch_gate_fwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                    const float* z, int64_t z_rs, const float* lam, const float* gb,
                    const float* h0, int64_t h0_bs, float* y, int64_t y_rs, float* carries,
                    int64_t B, int64_t L, int64_t H, const int64_t* offs, hipStream_t st,
                    float* y_last, const int64_t* order) {
  return gate_fwd_t<float>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, h0, h0_bs, y, y_rs, carries,
                           B, L, H, offs, st, y_last, order);
}

int launch_gate_fwd_bf16(const bf16_t* rg, int64_t rg_rs, const bf16_t* xc, int64_t xc_rs,
                         const bf16_t* z, int64_t z_rs, const float* lam, const float* gb,
                         const float* h0, int64_t h0_bs, bf16_t* y, int64_t y_rs, float* carries,
                         int64_t B, int64_t L, int64_t H, const int64_t* offs, hipStream_t st) {
  return gate_fwd_t<bf16_t>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, h0, h0_bs, y, y_rs, carries,
                            B, L, H, offs, st, nullptr, nullptr);
}

int launch_gate_bwd(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                    const float* z, int64_t z_rs, const float* lam, const float* gb,
                    const float* carries, const float* dy, float* drg, int64_t drg_rs, float* dxc,
                    int64_t dxc_rs, float* dz, int64_t dz_rs, float* part, float* dh0_part,
                    int64_t B, int64_t L, int64_t H, const int64_t* offs, hipStream_t st,
                    const float* dy_last, const int64_t* order) {
  return gate_bwd_t<float>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, carries, dy, drg, drg_rs, dxc,
                           dxc_rs, dz, dz_rs, part, dh0_part, B, L, H, offs, st, dy_last, order);
}

int launch_gate_bwd_bf16(const bf16_t* rg, int64_t rg_rs, const bf16_t* xc, int64_t xc_rs,
                         const bf16_t* z, int64_t z_rs, const float* lam, const float* gb,
                         const float* carries, const bf16_t* dy, bf16_t* drg, int64_t drg_rs,
                         bf16_t* dxc, int64_t dxc_rs, bf16_t* dz, int64_t dz_rs, float* part,
                         float* dh0_part, int64_t B, int64_t L, int64_t H, const int64_t* offs,
                         hipStream_t st) {
  return gate_bwd_t<bf16_t>(rg, rg_rs, xc, xc_rs, z, z_rs, lam, gb, carries, dy, drg, drg_rs,
                            dxc, dxc_rs, dz, dz_rs, part, dh0_part, B, L, H, offs, st, nullptr, nullptr);
}

}  // namespace rb
