// conv_silu.hip — causal depthwise conv1d (kernel K, zero history) + bias +
// SiLU on channel-last [B, L, H] (reference RecBLR.py:182-193), fwd and bwd.
//
// Same wave layout as the gate scan (common.h): lane = (time chunk q, channel
// group g), VEC = 4 channels per lane so every access is a 16-B load/store
// and one wave-instruction touches Q contiguous 256-B row segments.
#include "common.h"

// the input rows are re-read by the neighbouring time tile (K-1 halo rows):
// default cache policy (ldc)
//
// steps per lane of the row-tiled packed forward at K = 4 (tile = 4 x TC rows;
// each tile re-fetches K-1 halo rows its predecessor loaded).  Round 5 cut
// the halo's measured re-reads two ways, and both ran slower at the bench
// shape (0.61-0.62 of 8 TB/s against 0.69; profiles/r05_conv_ab_*.txt):
// a workgroup's 4 waves on 4 consecutive tiles of one channel group (PMC
// read 1.09x the algorithmic bytes instead of 1.20x, but each workgroup reads
// 256-B pieces of 64 rows instead of whole 1-KB rows) and a wave walking 4
// consecutive tiles (1.12x; a quarter of the waves in flight).  The kernel
// already streams at the 1R + 1W copy rate of these boxes (0.66-0.73).
constexpr int kConvRowsTC = 4;

namespace rb {
namespace {

template <typename T, int K, int VEC, int Q, int TC>
__global__ void __launch_bounds__(256)
k_conv_silu_fwd(const T* __restrict__ x, int x_rs, const float* __restrict__ w,
                const float* __restrict__ bias, T* __restrict__ xc, int xc_rs, int64_t B,
                int Lmax, int H, int ncw, int ntile, const int64_t* __restrict__ offs) {
  constexpr int G = kWave / Q;
  constexpr int NX = TC + K - 1;
  const int lane = threadIdx.x & (kWave - 1);
  const int q = lane / G;
  const int g = lane - q * G;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int tile = (int)(wid % ntile);
  const int64_t tmp = wid / ntile;
  const int cw = (int)(tmp % ncw);
  const int64_t b = tmp / ncw;
  if (b >= B) return;
  const int c0 = cw * (G * VEC) + g * VEC;
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
  if (tile * (Q * TC) >= L) return;   // past this sequence's end (wave-uniform)
  const T* xb = x + row0 * x_rs + cc;
  T* ob = xc + row0 * xc_rs + cc;
  float wk[K][VEC], bi[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
#pragma unroll
    for (int k = 0; k < K; ++k) wk[k][v] = w[(cc + v) * K + k];
  }
  ldc(bi, bias + cc);
  const int t0 = tile * (Q * TC) + q * TC;
  float xs[NX][VEC];   // x[t0-K+1 .. t0+TC-1]
#pragma unroll
  for (int m = 0; m < NX; ++m) {
    const int t = t0 - (K - 1) + m;
    const int tc = t < 0 ? 0 : (t >= L ? L - 1 : t);
    ldc(xs[m], xb + tc * x_rs);
    if (t < 0) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) xs[m][v] = 0.0f;
    }
  }
#pragma unroll
  for (int j = 0; j < TC; ++j) {
    float out[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      float acc = bi[v];
#pragma unroll
      for (int k = 0; k < K; ++k) acc = acc + wk[k][v] * xs[j + k][v];
      out[v] = fsilu(acc);
    }
    if (cv && t0 + j < L) stv(ob + (t0 + j) * xc_rs, out);
  }
}

// Row-tiled forward for packed sequences: waves tile the packed rows
// [0, ntok) themselves (16 rows x G*VEC channels each, channel block fastest),
// ignoring sequence boundaries, so no wave is launched past a sequence's end.
// row_pos[r] = position of packed row r inside its sequence: the tap at lag l
// contributes to row r only if l <= row_pos[r] (zero history before a
// sequence's first row, exactly the per-sequence kernel's masking).
template <typename T, int K, int VEC, int Q, int TC>
__global__ void __launch_bounds__(256)
k_conv_silu_fwd_rows(const T* __restrict__ x, int x_rs, const float* __restrict__ w,
                     const float* __restrict__ bias, T* __restrict__ xc, int xc_rs,
                     int64_t ntok, int H, int ncw, const int64_t* __restrict__ row_pos) {
  constexpr int G = kWave / Q;
  constexpr int NX = TC + K - 1;
  const int lane = threadIdx.x & (kWave - 1);
  const int q = lane / G;
  const int g = lane - q * G;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int cw = (int)(wid % ncw);
  const int64_t tile = wid / ncw;
  if (tile * (Q * TC) >= ntok) return;   // wave-uniform
  const int c0 = cw * (G * VEC) + g * VEC;
  const bool cv = c0 < H;
  const int cc = cv ? c0 : 0;
  float wk[K][VEC], bi[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
#pragma unroll
    for (int k = 0; k < K; ++k) wk[k][v] = w[(cc + v) * K + k];
  }
  ldc(bi, bias + cc);
  const int64_t r0 = tile * (Q * TC) + q * TC;
  float xs[NX][VEC];   // x[r0-K+1 .. r0+TC-1]
#pragma unroll
  for (int m = 0; m < NX; ++m) {
    int64_t r = r0 - (K - 1) + m;
    r = r < 0 ? 0 : (r >= ntok ? ntok - 1 : r);
    ldc(xs[m], x + r * x_rs + cc);
  }
  int64_t pj[TC];
#pragma unroll
  for (int j = 0; j < TC; ++j) pj[j] = row_pos[min(r0 + j, ntok - 1)];
#pragma unroll
  for (int j = 0; j < TC; ++j) {
    float out[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      float acc = bi[v];
#pragma unroll
      for (int k = 0; k < K; ++k)   // lag K-1-k: rows before the sequence start are zero
        acc = acc + (K - 1 - k <= pj[j] ? wk[k][v] * xs[j + k][v] : 0.0f);
      out[v] = fsilu(acc);
    }
    if (cv && r0 + j < ntok) stv(xc + (r0 + j) * xc_rs + cc, out);
  }
}

// Backward.  A wave owns (b, channels) for the whole sequence so its dW/dbias
// partial sums are complete per batch row (written to dw_part/db_part, summed
// over b by the caller: deterministic, no atomics).  Tiles are walked from the
// end; the K-1 "look-ahead" du values a chunk needs come from the next chunk's
// lane by shuffle, or from the previous (later) tile for the last chunk.
// PF: the next (earlier) tile's rows are loaded, in storage format, before the
// current tile is computed, so a wave keeps two tiles of loads in flight —
// what long sequences (configs[4], L = 2048: 128 tiles walked by one wave)
// need to cover HBM latency.
template <typename T, int VEC, int NX, int TC>
struct ConvBwdIn {
  RawVec<T, VEC> xs[NX], g1[TC], g2[TC];
};

template <typename T, int K, int VEC, int Q, int TC, bool PF = false>
__global__ void __launch_bounds__(256)
k_conv_silu_bwd(const T* __restrict__ x, int x_rs, const float* __restrict__ w,
                const float* __restrict__ bias, const T* __restrict__ g1,
                const T* __restrict__ g2, T* __restrict__ dx, int dx_rs,
                float* __restrict__ dw_part, float* __restrict__ db_part, int64_t B, int Lmax,
                int H, int ncw, const int64_t* __restrict__ offs) {
  constexpr int G = kWave / Q;
  constexpr int NX = TC + K - 1;
  constexpr int KH = K > 1 ? K - 1 : 1;
  static_assert(TC >= K - 1, "chunk must cover the look-ahead");
  const int lane = threadIdx.x & (kWave - 1);
  const int q = lane / G;
  const int g = lane - q * G;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = wid / ncw;
  if (b >= B) return;
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
  const T* xb = x + row0 * x_rs + cc;
  const T* g1b = g1 + row0 * H + cc;
  const T* g2b = g2 ? g2 + row0 * H + cc : nullptr;
  T* dxb = dx + row0 * dx_rs + cc;
  float wk[K][VEC], bi[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
#pragma unroll
    for (int k = 0; k < K; ++k) wk[k][v] = w[(cc + v) * K + k];
  }
  ldc(bi, bias + cc);
  float accw[K][VEC], accb[VEC], halo[KH][VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    accb[v] = 0.0f;
#pragma unroll
    for (int k = 0; k < K; ++k) accw[k][v] = 0.0f;
#pragma unroll
    for (int m = 0; m < KH; ++m) halo[m][v] = 0.0f;
  }
  constexpr int TILE = Q * TC;
  const int nT = (L + TILE - 1) / TILE;
  using In = ConvBwdIn<T, VEC, NX, TC>;
  auto load = [&](In& in, int tile) {
    const int t0 = tile * TILE + q * TC;
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      const int t = t0 - (K - 1) + m;
      const int tc = t < 0 ? 0 : (t >= L ? L - 1 : t);
      ld_raw<false>(in.xs[m], xb + tc * x_rs);
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int tc = min(t0 + j, L - 1);
      ld_raw(in.g1[j], g1b + tc * H);
      if (g2b != nullptr) ld_raw(in.g2[j], g2b + tc * H);
    }
  };
  auto process = [&](const In& in, int tile) {
    const int t0 = tile * TILE + q * TC;
    float xs[NX][VEC], du[TC][VEC];
#pragma unroll
    for (int m = 0; m < NX; ++m) {
      unpack_raw(xs[m], in.xs[m]);
      if (t0 - (K - 1) + m < 0) {
#pragma unroll
        for (int v = 0; v < VEC; ++v) xs[m][v] = 0.0f;
      }
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      unpack_raw(du[j], in.g1[j]);
      if (g2b != nullptr) {
        float t2[VEC];
        unpack_raw(t2, in.g2[j]);
#pragma unroll
        for (int v = 0; v < VEC; ++v) du[j][v] = du[j][v] + t2[v];
      }
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const bool ok = t0 + j < L;
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float acc = bi[v];
#pragma unroll
        for (int k = 0; k < K; ++k) acc = acc + wk[k][v] * xs[j + k][v];
        du[j][v] = ok ? du[j][v] * fdsilu(acc) : 0.0f;
        if (ok) {
          accb[v] = accb[v] + du[j][v];
#pragma unroll
          for (int k = 0; k < K; ++k) accw[k][v] = accw[k][v] + du[j][v] * xs[j + k][v];
        }
      }
    }
    // look-ahead du[t0+TC .. t0+TC+K-2]
    float dn[KH][VEC];
#pragma unroll
    for (int m = 0; m < KH; ++m) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const float nb = __shfl_down(du[m][v], G, kWave);
        dn[m][v] = (q == Q - 1) ? halo[m][v] : nb;
        halo[m][v] = __shfl(du[m][v], g, kWave);   // chunk 0 of this tile, for the next one
      }
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      float out[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int m = j + K - 1 - k;   // du index, may run into the look-ahead
          const float dv = m < TC ? du[m < TC ? m : 0][v] : dn[m >= TC ? m - TC : 0][v];
          acc = acc + wk[k][v] * dv;
        }
        out[v] = acc;
      }
      if (cv && t0 + j < L) stv(dxb + (t0 + j) * dx_rs, out);
    }
  };
  In bufA, bufB;
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
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
#pragma unroll
    for (int s = G; s < kWave; s <<= 1) {
      accb[v] += __shfl_xor(accb[v], s, kWave);
#pragma unroll
      for (int k = 0; k < K; ++k) accw[k][v] += __shfl_xor(accw[k][v], s, kWave);
    }
  }
  if (q == 0 && cv) {
    if (db_part == nullptr) {
      // folded: one row of (K + 1) * H partials per sequence, dW in the
      // weight's own [c, k] order, then dbias — one column sum gives both,
      // already in parameter layout
      float* row = dw_part + b * (K + 1) * H;
      if constexpr (K == 4 && VEC == 4) {
        // a lane's 4 channels x 4 taps are 16 consecutive floats: 16-B stores
        // (the vector path checked dw_part's alignment; H % 4 == 0)
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const float o[4] = {accw[0][v], accw[1][v], accw[2][v], accw[3][v]};
          stv(row + (c0 + v) * K, o);
        }
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v)
#pragma unroll
          for (int k = 0; k < K; ++k) row[(c0 + v) * K + k] = accw[k][v];
      }
      stv(row + K * H + c0, accb);
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) stv(dw_part + (b * K + k) * H + c0, accw[k]);
      stv(db_part + b * H + c0, accb);
    }
  }
}

constexpr int kConvQ = 4;

template <typename T, int K, int TC, int VW = 4>
int conv_fwd_t(const T* x, int64_t x_rs, const float* w, const float* bias, T* xc,
               int64_t xc_rs, int64_t B, int64_t L, int64_t H, bool vec, const int64_t* offs,
               hipStream_t st) {
  const int V = vec ? VW : 1;
  const int span = (kWave / kConvQ) * V;
  const int ncw = (int)((H + span - 1) / span);
  const int ntile = (int)((L + kConvQ * TC - 1) / (kConvQ * TC));
  const int64_t waves = B * ncw * ntile;
  const int64_t blocks = (waves + 3) / 4;
  if (blocks > 0x7fffffffLL) return fail("rb_conv_silu_fwd: grid too large");
  if (vec)
    hipLaunchKernelGGL((k_conv_silu_fwd<T, K, VW, kConvQ, TC>), dim3((unsigned)blocks), dim3(256),
                       0, st, x, (int)x_rs, w, bias, xc, (int)xc_rs, B, (int)L, (int)H, ncw, ntile, offs);
  else
    hipLaunchKernelGGL((k_conv_silu_fwd<T, K, 1, kConvQ, TC>), dim3((unsigned)blocks), dim3(256),
                       0, st, x, (int)x_rs, w, bias, xc, (int)xc_rs, B, (int)L, (int)H, ncw, ntile, offs);
  return launch_status("rb_conv_silu_fwd");
}

template <typename T, int K, int TC, int VW = 4>
int conv_fwd_rows_t(const T* x, int64_t x_rs, const float* w, const float* bias, T* xc,
                    int64_t xc_rs, int64_t ntok, int64_t H, bool vec, const int64_t* pos,
                    hipStream_t st) {
  const int V = vec ? VW : 1;
  const int span = (kWave / kConvQ) * V;
  const int ncw = (int)((H + span - 1) / span);
  const int64_t ntile = (ntok + kConvQ * TC - 1) / (kConvQ * TC);
  const int64_t blocks = (ntile * ncw + 3) / 4;
  if (blocks > 0x7fffffffLL) return fail("rb_conv_silu_fwd_rows: grid too large");
  if (blocks == 0) return 0;
  if (vec)
    hipLaunchKernelGGL((k_conv_silu_fwd_rows<T, K, VW, kConvQ, TC>), dim3((unsigned)blocks),
                       dim3(256), 0, st, x, (int)x_rs, w, bias, xc, (int)xc_rs, ntok, (int)H, ncw,
                       pos);
  else
    hipLaunchKernelGGL((k_conv_silu_fwd_rows<T, K, 1, kConvQ, TC>), dim3((unsigned)blocks),
                       dim3(256), 0, st, x, (int)x_rs, w, bias, xc, (int)xc_rs, ntok, (int)H, ncw,
                       pos);
  return launch_status("rb_conv_silu_fwd_rows");
}

// backward chunks per tile: 4 x 4 steps (8 x 4 is 3% faster on dense L = 200
// rows in tools/kbench.hip but 2% slower on the bench's packed sequences; bf16
// at configs[4]: 0.59 of 8 TB/s with 4 chunks, 0.38 with 8)
template <typename T>
constexpr int conv_bwd_q() { return 4; }

template <typename T, int K, int TC>
int conv_bwd_t(const T* x, int64_t x_rs, const float* w, const float* bias, const T* g1,
               const T* g2, T* dx, int64_t dx_rs, float* dw_part, float* db_part,
               int64_t B, int64_t L, int64_t H, bool vec, const int64_t* offs, hipStream_t st) {
  constexpr int kQ = conv_bwd_q<T>();
  const int V = vec ? 4 : 1;
  const int span = (kWave / kQ) * V;
  const int ncw = (int)((H + span - 1) / span);
  const int64_t blocks = (B * ncw + 3) / 4;
  if (vec)
    hipLaunchKernelGGL((k_conv_silu_bwd<T, K, 4, kQ, TC>), dim3((unsigned)blocks), dim3(256),
                       0, st, x, (int)x_rs, w, bias, g1, g2, dx, (int)dx_rs, dw_part, db_part, B,
                       (int)L, (int)H, ncw, offs);
  else
    hipLaunchKernelGGL((k_conv_silu_bwd<T, K, 1, kQ, TC>), dim3((unsigned)blocks), dim3(256),
                       0, st, x, (int)x_rs, w, bias, g1, g2, dx, (int)dx_rs, dw_part, db_part, B,
                       (int)L, (int)H, ncw, offs);
  return launch_status("rb_conv_silu_bwd");
}

// 4 channels per lane: 16-B (fp32) or 8-B (bf16) accesses
template <typename T>
bool al4(const void* p) {
  return p == nullptr || reinterpret_cast<uintptr_t>(p) % (4 * sizeof(T)) == 0;
}

template <typename T>
int conv_fwd_k(const T* x, int64_t x_rs, const float* w, const float* bias, T* xc, int64_t xc_rs,
               int64_t B, int64_t L, int64_t H, int64_t K, const int64_t* offs, hipStream_t st) {
  const bool vec = H % 4 == 0 && x_rs % 4 == 0 && xc_rs % 4 == 0 && al4<T>(x) && al4<T>(xc) &&
                   aligned16(bias);
  // bf16 at K = 4: 8 channels (16 B) per lane, 8-step chunks (tools/kbench.hip: 6% faster
  // at config 5)
  if (sizeof(T) == 2 && K == 4 && vec && H % 8 == 0 && x_rs % 8 == 0 && xc_rs % 8 == 0 &&
      aligned16(x) && aligned16(xc) && aligned16(bias) && aligned16(w))
    return conv_fwd_t<T, 4, 8, 8>(x, x_rs, w, bias, xc, xc_rs, B, L, H, true, offs, st);
  switch (K) {
    case 1: return conv_fwd_t<T, 1, 4>(x, x_rs, w, bias, xc, xc_rs, B, L, H, vec, offs, st);
    case 2: return conv_fwd_t<T, 2, 4>(x, x_rs, w, bias, xc, xc_rs, B, L, H, vec, offs, st);
    case 3: return conv_fwd_t<T, 3, 4>(x, x_rs, w, bias, xc, xc_rs, B, L, H, vec, offs, st);
    case 4: return conv_fwd_t<T, 4, 4>(x, x_rs, w, bias, xc, xc_rs, B, L, H, vec, offs, st);
    case 5: return conv_fwd_t<T, 5, 4>(x, x_rs, w, bias, xc, xc_rs, B, L, H, vec, offs, st);
    case 6: return conv_fwd_t<T, 6, 4>(x, x_rs, w, bias, xc, xc_rs, B, L, H, vec, offs, st);
    case 7: return conv_fwd_t<T, 7, 4>(x, x_rs, w, bias, xc, xc_rs, B, L, H, vec, offs, st);
    case 8: return conv_fwd_t<T, 8, 4>(x, x_rs, w, bias, xc, xc_rs, B, L, H, vec, offs, st);
    default: return fail("rb_conv_silu_fwd: kernel size K must be in [1, 8]");
  }
}

template <typename T>
int conv_fwd_rows_k(const T* x, int64_t x_rs, const float* w, const float* bias, T* xc,
                    int64_t xc_rs, int64_t ntok, int64_t H, int64_t K, const int64_t* pos,
                    hipStream_t st) {
  const bool vec = H % 4 == 0 && x_rs % 4 == 0 && xc_rs % 4 == 0 && al4<T>(x) && al4<T>(xc) &&
                   aligned16(bias);
  if (sizeof(T) == 2 && K == 4 && vec && H % 8 == 0 && x_rs % 8 == 0 && xc_rs % 8 == 0 &&
      aligned16(x) && aligned16(xc) && aligned16(bias) && aligned16(w))
    return conv_fwd_rows_t<T, 4, 8, 8>(x, x_rs, w, bias, xc, xc_rs, ntok, H, true, pos, st);
  switch (K) {
    case 1: return conv_fwd_rows_t<T, 1, 4>(x, x_rs, w, bias, xc, xc_rs, ntok, H, vec, pos, st);
    case 2: return conv_fwd_rows_t<T, 2, 4>(x, x_rs, w, bias, xc, xc_rs, ntok, H, vec, pos, st);
    case 3: return conv_fwd_rows_t<T, 3, 4>(x, x_rs, w, bias, xc, xc_rs, ntok, H, vec, pos, st);
    case 4: return conv_fwd_rows_t<T, 4, kConvRowsTC>(x, x_rs, w, bias, xc, xc_rs, ntok, H, vec, pos, st);
    case 5: return conv_fwd_rows_t<T, 5, 4>(x, x_rs, w, bias, xc, xc_rs, ntok, H, vec, pos, st);
    case 6: return conv_fwd_rows_t<T, 6, 4>(x, x_rs, w, bias, xc, xc_rs, ntok, H, vec, pos, st);
    case 7: return conv_fwd_rows_t<T, 7, 4>(x, x_rs, w, bias, xc, xc_rs, ntok, H, vec, pos, st);
    case 8: return conv_fwd_rows_t<T, 8, 4>(x, x_rs, w, bias, xc, xc_rs, ntok, H, vec, pos, st);
    default: return fail("rb_conv_silu_fwd_rows: kernel size K must be in [1, 8]");
  }
}

template <typename T>
int conv_bwd_k(const T* x, int64_t x_rs, const float* w, const float* bias, const T* g1,
               const T* g2, T* dx, int64_t dx_rs, float* dw_part, float* db_part, int64_t B,
               int64_t L, int64_t H, int64_t K, const int64_t* offs, hipStream_t st) {
  const bool vec = H % 4 == 0 && x_rs % 4 == 0 && dx_rs % 4 == 0 && al4<T>(x) && al4<T>(g1) &&
                   al4<T>(g2) && al4<T>(dx) && aligned16(dw_part) && aligned16(db_part) &&
                   aligned16(bias);
  switch (K) {
    case 1: return conv_bwd_t<T, 1, 4>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, vec, offs, st);
    case 2: return conv_bwd_t<T, 2, 4>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, vec, offs, st);
    case 3: return conv_bwd_t<T, 3, 4>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, vec, offs, st);
    case 4: return conv_bwd_t<T, 4, 4>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, vec, offs, st);
    case 5: return conv_bwd_t<T, 5, 4>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, vec, offs, st);
    case 6: return conv_bwd_t<T, 6, 8>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, vec, offs, st);
    case 7: return conv_bwd_t<T, 7, 8>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, vec, offs, st);
    case 8: return conv_bwd_t<T, 8, 8>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, vec, offs, st);
    default: return fail("rb_conv_silu_bwd: kernel size K must be in [1, 8]");
  }
}

}  // namespace

int launch_conv_fwd(const float* x, int64_t x_rs, const float* w, const float* bias, float* xc,
                    int64_t xc_rs, int64_t B, int64_t L, int64_t H, int64_t K,
                    const int64_t* offs, hipStream_t st) {
  return conv_fwd_k<float>(x, x_rs, w, bias, xc, xc_rs, B, L, H, K, offs, st);
}

int launch_conv_fwd_bf16(const bf16_t* x, int64_t x_rs, const float* w, const float* bias,
                         bf16_t* xc, int64_t xc_rs, int64_t B, int64_t L, int64_t H, int64_t K,
                         const int64_t* offs, hipStream_t st) {
  return conv_fwd_k<bf16_t>(x, x_rs, w, bias, xc, xc_rs, B, L, H, K, offs, st);
}

int launch_conv_fwd_rows(const float* x, int64_t x_rs, const float* w, const float* bias,
                         float* xc, int64_t xc_rs, int64_t ntok, int64_t H, int64_t K,
                         const int64_t* pos, hipStream_t st) {
  return conv_fwd_rows_k<float>(x, x_rs, w, bias, xc, xc_rs, ntok, H, K, pos, st);
}

int launch_conv_fwd_rows_bf16(const bf16_t* x, int64_t x_rs, const float* w, const float* bias,
                              bf16_t* xc, int64_t xc_rs, int64_t ntok, int64_t H, int64_t K,
                              const int64_t* pos, hipStream_t st) {
  return conv_fwd_rows_k<bf16_t>(x, x_rs, w, bias, xc, xc_rs, ntok, H, K, pos, st);
}

int launch_conv_bwd(const float* x, int64_t x_rs, const float* w, const float* bias,
                    const float* g1, const float* g2, float* dx, int64_t dx_rs, float* dw_part,
                    float* db_part, int64_t B, int64_t L, int64_t H, int64_t K,
                    const int64_t* offs, hipStream_t st) {
  return conv_bwd_k<float>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, K,
                           offs, st);
}

int launch_conv_bwd_bf16(const bf16_t* x, int64_t x_rs, const float* w, const float* bias,
                         const bf16_t* g1, const bf16_t* g2, bf16_t* dx, int64_t dx_rs,
                         float* dw_part, float* db_part, int64_t B, int64_t L, int64_t H,
                         int64_t K, const int64_t* offs, hipStream_t st) {
  return conv_bwd_k<bf16_t>(x, x_rs, w, bias, g1, g2, dx, dx_rs, dw_part, db_part, B, L, H, K,
                            offs, st);
}

}  // namespace rb
