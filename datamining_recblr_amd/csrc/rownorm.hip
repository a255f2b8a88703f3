// rownorm.hip — fused "dropout + residual + LayerNorm" row kernels and the
// FFN's fused SiLU + dropout, for the blocks around the BD-LRU
// (reference RecBLR.py:76-78 embedding -> dropout -> LayerNorm,
// :142 LayerNorm(dropout(GRL(x)) + x), :219-225 FeedForward).
//
//   s = A[row] * mask * scale + r[row]      (A[row] = table[idx[row]] if idx)
//   y = (s - mean) * rstd * gamma + beta,   rstd = 1 / sqrt(var + eps)
//
// torch runs each of these as 3-5 separate kernels with a [rows, d] HBM round
// trip between each (and its LayerNorm launches one workgroup per 128-float
// row).  Here one wave handles 64/LPR rows at a time, each row spread over LPR
// lanes holding NV float4s (LPR * NV * 4 = d); row statistics are reduced
// with shuffles inside the row's lane group.
#include "common.h"

namespace rb {
namespace {

template <int LPR>
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ void ld_mask4(float (&m)[4], const uint8_t* p) {
  const uchar4 t = *reinterpret_cast<const uchar4*>(p);
  m[0] = t.x; m[1] = t.y; m[2] = t.z; m[3] = t.w;
}

template <int NV, int LPR>
__global__ void __launch_bounds__(256)
k_add_ln_fwd(const float* __restrict__ a, const int64_t* __restrict__ idx, int64_t nidx,
             const uint8_t* __restrict__ mask, float scale, const float* __restrict__ r,
             const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
             float* __restrict__ y, float* __restrict__ s_out, float* __restrict__ mean_out,
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
    ldv(gm[k], gamma + (l + k * LPR) * 4);
    ldv(bt[k], beta + (l + k * LPR) * 4);
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
      ldv(s[k], arow + c);
      if (mask) {
        float m[4];
        ld_mask4(m, mask + rr * D + c);
#pragma unroll
        for (int v = 0; v < 4; ++v) s[k][v] = s[k][v] * m[v] * scale;
      }
      if (r) {
        float t[4];
        ldv(t, r + rr * D + c);
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
        stv(y + row * D + c, o);
        if (s_out) stv(s_out + row * D + c, s[k]);
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
//   ds = rstd (g - mean(g) - xh mean(g xh)),  da = ds * mask * scale,
//   dgamma += dy * xh, dbeta += dy (per-block partial sums, deterministic).
template <int NV, int LPR>
__global__ void __launch_bounds__(256)
k_add_ln_bwd(const float* __restrict__ dy, const float* __restrict__ s,
             const float* __restrict__ gamma, const float* __restrict__ mean,
             const float* __restrict__ rstd, const uint8_t* __restrict__ mask, float scale,
             float* __restrict__ ds_out, float* __restrict__ da_out,
             float* __restrict__ dgamma_part, float* __restrict__ dbeta_part, int64_t rows) {
  constexpr int D = LPR * NV * 4;
  constexpr int RPW = kWave / LPR;
  __shared__ float red[2][4][D];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int sub = lane / LPR;
  const int l = lane - sub * LPR;
  const int64_t wave = (int64_t)blockIdx.x * 4 + wv;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  float gm[NV][4], accg[NV][4], accb[NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    ldv(gm[k], gamma + (l + k * LPR) * 4);
#pragma unroll
    for (int v = 0; v < 4; ++v) accg[k][v] = accb[k][v] = 0.0f;
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
      ldv(dyv, dy + rr * D + c);
      ldv(xh[k], s + rr * D + c);
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
    if (ok) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (l + k * LPR) * 4;
        float d[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) d[v] = rs * (g[k][v] - mg - xh[k][v] * mgx);
        if (ds_out) stv(ds_out + row * D + c, d);
        if (da_out) {
          if (mask) {
            float m[4];
            ld_mask4(m, mask + row * D + c);
#pragma unroll
            for (int v = 0; v < 4; ++v) d[v] = d[v] * m[v] * scale;
          }
          stv(da_out + row * D + c, d);
        }
      }
    }
  }
  // dgamma / dbeta: reduce the RPW row groups of the wave, then the 4 waves
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int o = LPR; o < kWave; o <<= 1) {
        accg[k][v] += __shfl_xor(accg[k][v], o, kWave);
        accb[k][v] += __shfl_xor(accb[k][v], o, kWave);
      }
  if (sub == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (l + k * LPR) * 4;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        red[0][wv][c + v] = accg[k][v];
        red[1][wv][c + v] = accb[k][v];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    dgamma_part[(int64_t)blockIdx.x * D + c] =
        ((red[0][0][c] + red[0][1][c]) + red[0][2][c]) + red[0][3][c];
    dbeta_part[(int64_t)blockIdx.x * D + c] =
        ((red[1][0][c] + red[1][1][c]) + red[1][2][c]) + red[1][3][c];
  }
}

// u = silu(a) * mask * scale (mask optional); the FFN's inner activation.
__global__ void __launch_bounds__(256)
k_silu_dropout_fwd(const float4* __restrict__ a, const uchar4* __restrict__ mask, float scale,
                   float4* __restrict__ u, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 x = a[i];
    float4 o = make_float4(fsilu(x.x), fsilu(x.y), fsilu(x.z), fsilu(x.w));
    if (mask) {
      const uchar4 m = mask[i];
      o.x *= m.x * scale; o.y *= m.y * scale; o.z *= m.z * scale; o.w *= m.w * scale;
    }
    u[i] = o;
  }
}

__global__ void __launch_bounds__(256)
k_silu_dropout_bwd(const float4* __restrict__ a, const uchar4* __restrict__ mask, float scale,
                   const float4* __restrict__ du, float4* __restrict__ da, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 x = a[i];
    float4 g = du[i];
    if (mask) {
      const uchar4 m = mask[i];
      g.x *= m.x * scale; g.y *= m.y * scale; g.z *= m.z * scale; g.w *= m.w * scale;
    }
    da[i] = make_float4(g.x * fdsilu(x.x), g.y * fdsilu(x.y), g.z * fdsilu(x.z),
                        g.w * fdsilu(x.w));
  }
}

constexpr int kRowBlocks = 1024;   // 4 waves each; grid-stride over rows

template <int NV, int LPR>
int ln_fwd_t(const float* a, const int64_t* idx, int64_t nidx, const uint8_t* mask, float scale, const float* r,
             const float* gamma, const float* beta, float eps, float* y, float* s_out,
             float* mean, float* rstd, int64_t rows, hipStream_t st) {
  constexpr int RPB = 4 * (kWave / LPR);
  const int64_t blocks = std::min<int64_t>(kRowBlocks * 2, (rows + RPB - 1) / RPB);
  hipLaunchKernelGGL((k_add_ln_fwd<NV, LPR>), dim3((unsigned)blocks), dim3(256), 0, st, a, idx,
                     nidx, mask, scale, r, gamma, beta, eps, y, s_out, mean, rstd, rows);
  return launch_status("rb_add_ln_fwd");
}

template <int NV, int LPR>
int ln_bwd_t(const float* dy, const float* s, const float* gamma, const float* mean,
             const float* rstd, const uint8_t* mask, float scale, float* ds, float* da,
             float* dgp, float* dbp, int64_t nparts, int64_t rows, hipStream_t st) {
  hipLaunchKernelGGL((k_add_ln_bwd<NV, LPR>), dim3((unsigned)nparts), dim3(256), 0, st, dy, s,
                     gamma, mean, rstd, mask, scale, ds, da, dgp, dbp, rows);
  return launch_status("rb_add_ln_bwd");
}

}  // namespace

int64_t ln_num_parts(int64_t rows) {
  return std::max<int64_t>(1, std::min<int64_t>(kRowBlocks, (rows + 31) / 32));
}

// d -> (NV, LPR): LPR lanes per row, NV float4 per lane, LPR * NV * 4 == d
#define RB_LN_DISPATCH(D, CALL)                 \
  switch (D) {                                  \
    case 16: return CALL(1, 4);                 \
    case 32: return CALL(1, 8);                 \
    case 64: return CALL(1, 16);                \
    case 128: return CALL(1, 32);               \
    case 256: return CALL(1, 64);               \
    case 512: return CALL(2, 64);               \
    case 1024: return CALL(4, 64);              \
    default: return fail("layer norm: d must be one of 16, 32, 64, 128, 256, 512, 1024"); \
  }

int launch_add_ln_fwd(const float* a, const int64_t* idx, int64_t nidx, const uint8_t* mask,
                      float scale,
                      const float* r, const float* gamma, const float* beta, float eps, float* y,
                      float* s_out, float* mean, float* rstd, int64_t rows, int64_t d,
                      hipStream_t st) {
#define RB_CALL(NV, LPR) \
  ln_fwd_t<NV, LPR>(a, idx, nidx, mask, scale, r, gamma, beta, eps, y, s_out, mean, rstd, rows, st)
  RB_LN_DISPATCH(d, RB_CALL)
#undef RB_CALL
}

int launch_add_ln_bwd(const float* dy, const float* s, const float* gamma, const float* mean,
                      const float* rstd, const uint8_t* mask, float scale, float* ds, float* da,
                      float* dgp, float* dbp, int64_t nparts, int64_t rows, int64_t d,
                      hipStream_t st) {
#define RB_CALL(NV, LPR) \
  ln_bwd_t<NV, LPR>(dy, s, gamma, mean, rstd, mask, scale, ds, da, dgp, dbp, nparts, rows, st)
  RB_LN_DISPATCH(d, RB_CALL)
#undef RB_CALL
}

int launch_silu_dropout_fwd(const float* a, const uint8_t* mask, float scale, float* u,
                            int64_t n, hipStream_t st) {
  const int64_t n4 = n / 4;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(8192, (n4 + 255) / 256));
  hipLaunchKernelGGL(k_silu_dropout_fwd, dim3((unsigned)blocks), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(a), reinterpret_cast<const uchar4*>(mask),
                     scale, reinterpret_cast<float4*>(u), n4);
  return launch_status("rb_silu_dropout_fwd");
}

int launch_silu_dropout_bwd(const float* a, const uint8_t* mask, float scale, const float* du,
                            float* da, int64_t n, hipStream_t st) {
  const int64_t n4 = n / 4;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(8192, (n4 + 255) / 256));
  hipLaunchKernelGGL(k_silu_dropout_bwd, dim3((unsigned)blocks), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(a), reinterpret_cast<const uchar4*>(mask),
                     scale, reinterpret_cast<const float4*>(du), reinterpret_cast<float4*>(da),
                     n4);
  return launch_status("rb_silu_dropout_bwd");
}

}  // namespace rb
