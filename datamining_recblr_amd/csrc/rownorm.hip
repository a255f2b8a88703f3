// rownorm.hip — fused row kernels around the BD-LRU: dropout + residual +
// LayerNorm (with an optional embedding gather) and the FFN's SiLU + dropout
// (reference RecBLR.py:76-78 embedding -> dropout -> LayerNorm,
// :142 LayerNorm(dropout(GRL(x)) + x), :219-225 FeedForward).
//
//   s = A[row] * keep * scale + r[row]      (A[row] = table[idx[row]] if idx)
//   y = (s - mean) * rstd * gamma + beta,   rstd = 1 / sqrt(var + eps)
//
// The LayerNorm kernels load with the default cache policy (ldc) and store
// per direction (st_ln below); the SiLU kernels stream (ldv/stv).
//
// Rows of D floats are spread over LPR lanes holding NV float4s each
// (LPR * NV * 4 = D), so one wave covers 64/LPR rows per step; row statistics
// are shuffle reductions inside the lane group.  Dropout keep-flags come from
// an explicit uint8 mask or are regenerated from a counter-based Philox
// stream (common.h), identically in forward and backward.  Column sums that
// torch would compute with separate reduction kernels (dgamma, dbeta, the
// bias gradient of the producing GEMM) are per-block partials, summed in a
// fixed order by the caller.
#include "common.h"

namespace rb {
namespace {

// Store policy of the LayerNorm outputs: nontemporal both ways.  The
// forward's (y, s): its consumers, the in-projection GEMM and through it the
// conv, read faster (conv forward 0.65 -> 0.69,
// profiles/r02_ab_ln_store_policy.log).  The backward's (ds, da): round 2
// measured the kernel alone slower with nt (0.68 -> 0.61), but in the round-6
// step (its consumers the weight-stationary dU / dX GEMMs) the whole step
// runs 5.406-5.419 vs 5.411-5.434 ms (profiles/r06_ab_ln_bwd_store_policy.txt).
constexpr bool kLnFwdNT = true, kLnBwdNT = true;
template <bool NT, int V>
__device__ __forceinline__ void st_ln(float* p, const float (&o)[V]) {
  if constexpr (NT) stv(p, o); else stc(p, o);
}

template <int LPR>
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// 4 waves each; grid-stride over rows.  The backward kernels' grid is also
// their partial count (dgamma/dbeta/dbias rows); the forward kernels take
// 4x the blocks (more rows in flight: add_ln_fwd 0.67 -> 0.69, silu fwd
// 0.67 -> 0.70 of HBM; the same for the backward kernels lost 1-2% to
// the larger partial sums; tools/ab_bench.sh, profiles/r02_ab_row_blocks.log)
constexpr int kRowBlocks = 1024;
constexpr int kRowBlocksFwd = 4 * kRowBlocks;

template <int NV, int LPR>
__global__ void __launch_bounds__(256)
k_add_ln_fwd(const float* __restrict__ a, const int64_t* __restrict__ idx, int64_t nidx,
             DropSpec drop, const float* __restrict__ r, const float* __restrict__ gamma,
             const float* __restrict__ beta, float eps, float* __restrict__ y,
             float* __restrict__ s_out, float* __restrict__ mean_out,
             float* __restrict__ rstd_out, int64_t rows) {
  constexpr int D = LPR * NV * 4;
  constexpr int RPW = kWave / LPR;   // rows per wave step
  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane / LPR;
  const int l = lane - sub * LPR;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  float gm[NV][4], bt[NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    ldc(gm[k], gamma + (l + k * LPR) * 4);
    ldc(bt[k], beta + (l + k * LPR) * 4);
  }
  for (int64_t row0 = wave * RPW; row0 < rows; row0 += nwaves * RPW) {
    const int64_t row = row0 + sub;
    const bool ok = row < rows;
    const int64_t rr = ok ? row : rows - 1;
    // gathered rows are clamped into the table: an out-of-range id reads a
    // valid row instead of faulting the device
    const float* arow = idx ? a + min(max(idx[rr], (int64_t)0), nidx - 1) * D : a + rr * D;
    float s[NV][4];
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (l + k * LPR) * 4;
      ldc(s[k], arow + c);
      float m[4];
      drop.get4(rr * D + c, m);
#pragma unroll
      for (int v = 0; v < 4; ++v) s[k][v] = s[k][v] * m[v];
      if (r) {
        float t[4];
        ldc(t, r + rr * D + c);
#pragma unroll
        for (int v = 0; v < 4; ++v) s[k][v] = s[k][v] + t[v];
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) sum += s[k][v];
    }
    const float mu = row_sum<LPR>(sum) * (1.0f / D);
    float sq = 0.0f;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float dv = s[k][v] - mu;
        sq += dv * dv;
      }
    const float var = row_sum<LPR>(sq) * (1.0f / D);
    const float rs = 1.0f / sqrtf(var + eps);
    if (ok) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (l + k * LPR) * 4;
        float o[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) o[v] = (s[k][v] - mu) * rs * gm[k][v] + bt[k][v];
        st_ln<kLnFwdNT>(y + row * D + c, o);
        if (s_out) st_ln<kLnFwdNT>(s_out + row * D + c, s[k]);
      }
      if (l == 0) {
        if (mean_out) mean_out[row] = mu;
        if (rstd_out) rstd_out[row] = rs;
      }
    }
  }
}

// Backward of k_add_ln_fwd given the saved s, mean, rstd:
//   xh = (s - mean) rstd, g = dy * gamma,
//   ds = rstd (g - mean(g) - xh mean(g xh)),  da = ds * keep * scale,
// partial column sums per block: dgamma += dy xh, dbeta += dy and, if asked,
// dbias += da (the bias gradient of the GEMM that produced a).
template <int NV, int LPR>
__global__ void __launch_bounds__(256)
k_add_ln_bwd(const float* __restrict__ dy, const float* __restrict__ dy2,
             const float* __restrict__ s,
             const float* __restrict__ gamma, const float* __restrict__ mean,
             const float* __restrict__ rstd, DropSpec drop, float* __restrict__ ds_out,
             float* __restrict__ da_out, float* __restrict__ dgamma_part,
             float* __restrict__ dbeta_part, float* __restrict__ dbias_part, int64_t rows) {
  constexpr int D = LPR * NV * 4;
  constexpr int RPW = kWave / LPR;
  __shared__ float red[3][4][D];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int sub = lane / LPR;
  const int l = lane - sub * LPR;
  const int64_t wave = (int64_t)blockIdx.x * 4 + wv;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  float gm[NV][4], accg[NV][4], accb[NV][4], acca[NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    ldc(gm[k], gamma + (l + k * LPR) * 4);
#pragma unroll
    for (int v = 0; v < 4; ++v) accg[k][v] = accb[k][v] = acca[k][v] = 0.0f;
  }
  for (int64_t row0 = wave * RPW; row0 < rows; row0 += nwaves * RPW) {
    const int64_t row = row0 + sub;
    const bool ok = row < rows;
    const int64_t rr = ok ? row : rows - 1;
    const float mu = mean[rr], rs = rstd[rr];
    float xh[NV][4], g[NV][4];
    float sg = 0.0f, sgx = 0.0f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (l + k * LPR) * 4;
      float dyv[4];
      ldc(dyv, dy + rr * D + c);
      if (dy2) {  // a second gradient of the same output (autograd's sum)
        float d2[4];
        ldc(d2, dy2 + rr * D + c);
#pragma unroll
        for (int v = 0; v < 4; ++v) dyv[v] += d2[v];
      }
      ldc(xh[k], s + rr * D + c);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if (!ok) dyv[v] = 0.0f;
        xh[k][v] = (xh[k][v] - mu) * rs;
        g[k][v] = dyv[v] * gm[k][v];
        sg += g[k][v];
        sgx += g[k][v] * xh[k][v];
        accg[k][v] += dyv[v] * xh[k][v];
        accb[k][v] += dyv[v];
      }
    }
    const float mg = row_sum<LPR>(sg) * (1.0f / D);
    const float mgx = row_sum<LPR>(sgx) * (1.0f / D);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (l + k * LPR) * 4;
      float d[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) d[v] = ok ? rs * (g[k][v] - mg - xh[k][v] * mgx) : 0.0f;
      if (ok && ds_out) st_ln<kLnBwdNT>(ds_out + row * D + c, d);
      if (da_out || dbias_part) {
        float m[4];
        drop.get4(rr * D + c, m);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          d[v] = d[v] * m[v];
          acca[k][v] += d[v];
        }
        if (ok && da_out) st_ln<kLnBwdNT>(da_out + row * D + c, d);
      }
    }
  }
  // column partials: reduce the RPW row groups of the wave, then the 4 waves
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int o = LPR; o < kWave; o <<= 1) {
        accg[k][v] += __shfl_xor(accg[k][v], o, kWave);
        accb[k][v] += __shfl_xor(accb[k][v], o, kWave);
        acca[k][v] += __shfl_xor(acca[k][v], o, kWave);
      }
  if (sub == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (l + k * LPR) * 4;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        red[0][wv][c + v] = accg[k][v];
        red[1][wv][c + v] = accb[k][v];
        red[2][wv][c + v] = acca[k][v];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    const int64_t o = (int64_t)blockIdx.x * D + c;
    dgamma_part[o] = ((red[0][0][c] + red[0][1][c]) + red[0][2][c]) + red[0][3][c];
    dbeta_part[o] = ((red[1][0][c] + red[1][1][c]) + red[1][2][c]) + red[1][3][c];
    if (dbias_part) dbias_part[o] = ((red[2][0][c] + red[2][1][c]) + red[2][2][c]) + red[2][3][c];
  }
}

// FFN inner activation on rows of C = LPR * NV * 4: u = silu(a) * keep * scale
template <int NV, int LPR>
__global__ void __launch_bounds__(256)
k_silu_dropout_fwd(const float* __restrict__ a, const float* __restrict__ bias, DropSpec drop,
                   float* __restrict__ u, int64_t rows) {
  constexpr int C = LPR * NV * 4;
  constexpr int RPW = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane / LPR;
  const int l = lane - sub * LPR;
  float bv[NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if (bias) {
      ldc(bv[k], bias + (l + k * LPR) * 4);
    } else {
#pragma unroll
      for (int v = 0; v < 4; ++v) bv[k][v] = 0.0f;
    }
  }
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t row0 = wave * RPW; row0 < rows; row0 += nwaves * RPW) {
    const int64_t row = row0 + sub;
    if (row >= rows) continue;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t e = row * C + (l + k * LPR) * 4;
      float x[4], m[4], o[4];
      ldv(x, a + e);
      drop.get4(e, m);
#pragma unroll
      for (int v = 0; v < 4; ++v) o[v] = fsilu(x[v] + bv[k][v]) * m[v];
      stv(u + e, o);
    }
  }
}

// da = du * keep * scale * silu'(a); column partials of da = the bias
// gradient of the GEMM that produced a.
template <int NV, int LPR>
__global__ void __launch_bounds__(256)
k_silu_dropout_bwd(const float* __restrict__ a, const float* __restrict__ bias, DropSpec drop,
                   const float* __restrict__ du, float* __restrict__ da,
                   float* __restrict__ dbias_part, int64_t rows) {
  constexpr int C = LPR * NV * 4;
  constexpr int RPW = kWave / LPR;
  __shared__ float red[4][C];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int sub = lane / LPR;
  const int l = lane - sub * LPR;
  float bv[NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if (bias) {
      ldc(bv[k], bias + (l + k * LPR) * 4);
    } else {
#pragma unroll
      for (int v = 0; v < 4; ++v) bv[k][v] = 0.0f;
    }
  }
  const int64_t wave = (int64_t)blockIdx.x * 4 + wv;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  float acc[NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[k][v] = 0.0f;
  for (int64_t row0 = wave * RPW; row0 < rows; row0 += nwaves * RPW) {
    const int64_t row = row0 + sub;
    if (row >= rows) continue;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t e = row * C + (l + k * LPR) * 4;
      float x[4], g[4], m[4], o[4];
      ldv(x, a + e);
      ldv(g, du + e);
      drop.get4(e, m);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        o[v] = (g[v] * m[v]) * fdsilu(x[v] + bv[k][v]);
        acc[k][v] += o[v];
      }
      stv(da + e, o);
    }
  }
  if (dbias_part == nullptr) return;   // grid-uniform
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int o = LPR; o < kWave; o <<= 1) acc[k][v] += __shfl_xor(acc[k][v], o, kWave);
  if (sub == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int v = 0; v < 4; ++v) red[wv][(l + k * LPR) * 4 + v] = acc[k][v];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    dbias_part[(int64_t)blockIdx.x * C + c] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

// explicit keep-mask materialisation of a Philox stream (tests, debugging)
__global__ void k_dropout_mask(DropSpec drop, uint8_t* __restrict__ out, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float m[4];
    drop.get4(i * 4, m);
    uchar4 o;
    o.x = m[0] != 0.0f; o.y = m[1] != 0.0f; o.z = m[2] != 0.0f; o.w = m[3] != 0.0f;
    reinterpret_cast<uchar4*>(out)[i] = o;
  }
}

template <int LPR, int MAXB = kRowBlocks>
int64_t row_blocks(int64_t rows) {
  constexpr int RPB = 4 * (kWave / LPR);
  return std::max<int64_t>(1, std::min<int64_t>(MAXB, (rows + RPB - 1) / RPB));
}

template <int NV, int LPR>
int add_ln_fwd_t(const float* a, const int64_t* idx, int64_t nidx, const DropSpec& drop,
                 const float* r, const float* gamma, const float* beta, float eps, float* y,
                 float* s_out, float* mean, float* rstd, int64_t rows, hipStream_t st) {
  hipLaunchKernelGGL((k_add_ln_fwd<NV, LPR>), dim3((unsigned)row_blocks<LPR, kRowBlocksFwd>(rows)),
                     dim3(256), 0,
                     st, a, idx, nidx, drop, r, gamma, beta, eps, y, s_out, mean, rstd, rows);
  return launch_status("rb_add_ln_fwd");
}

template <int NV, int LPR>
int add_ln_bwd_t(const float* dy, const float* dy2, const float* s, const float* gamma,
                 const float* mean, const float* rstd, const DropSpec& drop, float* ds, float* da,
                 float* dgp, float* dbp, float* dbiasp, int64_t nparts, int64_t rows,
                 hipStream_t st) {
  hipLaunchKernelGGL((k_add_ln_bwd<NV, LPR>), dim3((unsigned)nparts), dim3(256), 0, st, dy, dy2, s,
                     gamma, mean, rstd, drop, ds, da, dgp, dbp, dbiasp, rows);
  return launch_status("rb_add_ln_bwd");
}

template <int NV, int LPR>
int silu_fwd_t(const float* a, const float* bias, const DropSpec& drop, float* u, int64_t rows,
               hipStream_t st) {
  hipLaunchKernelGGL((k_silu_dropout_fwd<NV, LPR>),
                     dim3((unsigned)(row_blocks<LPR, 2 * kRowBlocksFwd>(rows))),
                     dim3(256), 0, st, a, bias, drop, u, rows);
  return launch_status("rb_silu_dropout_fwd");
}

template <int NV, int LPR>
int silu_bwd_t(const float* a, const float* bias, const DropSpec& drop, const float* du, float* da,
               float* dbias_part, int64_t nparts, int64_t rows, hipStream_t st) {
  hipLaunchKernelGGL((k_silu_dropout_bwd<NV, LPR>), dim3((unsigned)nparts), dim3(256), 0, st, a,
                     bias, drop, du, da, dbias_part, rows);
  return launch_status("rb_silu_dropout_bwd");
}

}  // namespace

int64_t ln_num_parts(int64_t rows, int64_t d) {
  switch (d) {
    case 16: return row_blocks<4>(rows);
    case 32: return row_blocks<8>(rows);
    case 64: return row_blocks<16>(rows);
    case 128: return row_blocks<32>(rows);
    default: return row_blocks<64>(rows);
  }
}

// width -> (NV, LPR): LPR lanes per row, NV float4 per lane, LPR * NV * 4 == width
#define RB_ROW_DISPATCH(D, FN, ...)                          \
  switch (D) {                                               \
    case 16: return FN<1, 4>(__VA_ARGS__);                   \
    case 32: return FN<1, 8>(__VA_ARGS__);                   \
    case 64: return FN<1, 16>(__VA_ARGS__);                  \
    case 128: return FN<1, 32>(__VA_ARGS__);                 \
    case 256: return FN<1, 64>(__VA_ARGS__);                 \
    case 512: return FN<2, 64>(__VA_ARGS__);                 \
    case 1024: return FN<4, 64>(__VA_ARGS__);                \
    default:                                                 \
      return fail("row kernels: width must be one of 16, 32, 64, 128, 256, 512, 1024"); \
  }

int launch_add_ln_fwd(const float* a, const int64_t* idx, int64_t nidx, const DropSpec& drop,
                      const float* r, const float* gamma, const float* beta, float eps, float* y,
                      float* s_out, float* mean, float* rstd, int64_t rows, int64_t d,
                      hipStream_t st) {
  RB_ROW_DISPATCH(d, add_ln_fwd_t, a, idx, nidx, drop, r, gamma, beta, eps, y, s_out, mean,
                  rstd, rows, st)
}

int launch_add_ln_bwd(const float* dy, const float* dy2, const float* s, const float* gamma,
                      const float* mean, const float* rstd, const DropSpec& drop, float* ds,
                      float* da, float* dgp, float* dbp, float* dbiasp, int64_t nparts,
                      int64_t rows, int64_t d, hipStream_t st) {
  RB_ROW_DISPATCH(d, add_ln_bwd_t, dy, dy2, s, gamma, mean, rstd, drop, ds, da, dgp, dbp, dbiasp,
                  nparts, rows, st)
}

int launch_silu_dropout_fwd(const float* a, const float* bias, const DropSpec& drop, float* u,
                            int64_t rows, int64_t cols, hipStream_t st) {
  RB_ROW_DISPATCH(cols, silu_fwd_t, a, bias, drop, u, rows, st)
}

int launch_silu_dropout_bwd(const float* a, const float* bias, const DropSpec& drop,
                            const float* du, float* da, float* dbias_part, int64_t nparts,
                            int64_t rows, int64_t cols, hipStream_t st) {
  RB_ROW_DISPATCH(cols, silu_bwd_t, a, bias, drop, du, da, dbias_part, nparts, rows, st)
}

int launch_dropout_mask(const DropSpec& drop, uint8_t* out, int64_t n, hipStream_t st) {
  const int64_t n4 = n / 4;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(4096, (n4 + 255) / 256));
  hipLaunchKernelGGL(k_dropout_mask, dim3((unsigned)blocks), dim3(256), 0, st, drop, out, n4);
  return launch_status("rb_dropout_mask");
}

}  // namespace rb
