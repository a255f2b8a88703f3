// gemm_small.hip — the f16 two-part split GEMMs (gemm_half.hip's scheme) for
// few rows: the last layer's gathered tail (B = 2048 rows: RecBLR.py:167,
// 213, 214 on the gather_indexes rows), the rows past the last whole round of
// the persistent k_gemm_nt_h (which would otherwise run on an eighth of the
// chip), and weight gradients below linear.MIN_ROWS_FOR_SPLIT.
//
// k_gemm_nt_hs: out[M, C] = A[M, R] . Bm[C, R]^T (+ bias).  A 512-thread
//   workgroup per 32 x 32 output block: the 8 waves split R into eighths,
//   each loads its whole slice of both operands into registers at once (one
//   memory round trip: these launches are latency-bound), and the eight
//   partial accumulators meet in LDS (summed in wave order).  A rows are
//   scaled by their EXACT max over R (the slices' maxima combined in LDS),
//   so no value can leave fp16's range and no recompute path is needed; the
//   weights use the image's per-column scales.  A rows are re-read from L2
//   by the C/32 column-block workgroups.  rmax (max |A| per 32-row group) is
//   written by the first column block.
// k_gemm_tn_hs: dW[N, K] = dY[M, N]^T X[M, K] (+ dW when accumulate).  A
//   512-thread workgroup per 32 x 32 block of dW: the 8 waves split the rows
//   M, each scales its slice PER COLUMN of both operands (exact column max
//   over the slice: column magnitudes spread over any range keep 22 bits),
//   and the 8 un-scaled partials are summed in LDS in wave order.
#include "common.h"

namespace rb {
namespace {

typedef _Float16 f16x8s __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2s __attribute__((ext_vector_type(2)));
typedef float f32x16s __attribute__((ext_vector_type(16)));
typedef float f32x4s __attribute__((ext_vector_type(4)));
typedef float f32x2s __attribute__((ext_vector_type(2)));

constexpr int kSW = 14;   // operand scale: max lands in [2^13, 2^14)

__device__ __forceinline__ void split2s(f32x2s x, f16x2s& h0, f16x2s& h1) {
  h0 = __builtin_convertvector(x, f16x2s);
  const f32x2s r = x - __builtin_convertvector(h0, f32x2s);
  h1 = __builtin_convertvector(r, f16x2s);
}

__device__ __forceinline__ void split8(f32x4s p, f32x4s q, float sc, f16x8s& a0, f16x8s& a1) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x2s v = (t < 2 ? f32x2s{p[2 * t], p[2 * t + 1]} : f32x2s{q[2 * t - 4], q[2 * t - 3]}) * sc;
    f16x2s h0, h1;
    split2s(v, h0, h1);
    a0[2 * t] = h0[0]; a0[2 * t + 1] = h0[1];
    a1[2 * t] = h1[0]; a1[2 * t + 1] = h1[1];
  }
}

__device__ __forceinline__ f32x16s mfma3(f16x8s a0, f16x8s a1, f16x8s b0, f16x8s b1, f32x16s c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, c, 0, 0, 0);
}

__device__ __forceinline__ int exp_of(float m) {
  return m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
}

template <bool BIAS>
__global__ void __launch_bounds__(512) k_gemm_nt_hs(const float* __restrict__ A, int64_t lda,
                                                    int64_t M, int R,
                                                    const f16x8s* __restrict__ Wf,
                                                    const int* __restrict__ ew, int C,
                                                    const float* __restrict__ bias,
                                                    float* __restrict__ out, int64_t ldo,
                                                    float* __restrict__ rmax) {
  constexpr int KMAX = 8;   // k16 blocks per wave held in registers (R <= 8 x 8 x 16 = 1024)
  __shared__ float s_max[8][32];
  __shared__ int s_er[32];
  __shared__ f32x16s s_acc[8][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t r0 = (int64_t)blockIdx.x * 32;
  const int cb = blockIdx.y;                    // 32-column block
  const int KB = R / 16;
  // wave w: k16 blocks [kb0, kb1), an eighth of R (loaded once, into registers)
  const int kb0 = KB * wave / 8, kb1 = KB * (wave + 1) / 8;
  int64_t row = r0 + (lane & 31);
  row = row < M ? row : M - 1;
  const float* arow = A + row * lda + 8 * (lane >> 5);
  const f16x8s* wb = Wf + (int64_t)cb * KB * 2 * 64 + lane;
  f32x4s p[KMAX], q[KMAX];
  f16x8s b0[KMAX], b1[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    if (kb0 + j < kb1) {
      const int kb = kb0 + j;
      p[j] = *reinterpret_cast<const f32x4s*>(arow + kb * 16);
      q[j] = *reinterpret_cast<const f32x4s*>(arow + kb * 16 + 4);
      b0[j] = wb[(kb * 2) * 64];
      b1[j] = wb[(kb * 2 + 1) * 64];
    }
  }
  // exact row max over R: each wave's slice, then the 8 slices in LDS
  float m = 0.0f;
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    if (kb0 + j < kb1) {
      m = fmaxf(m, fmaxf(fmaxf(fmaxf(fabsf(p[j][0]), fabsf(p[j][1])), fmaxf(fabsf(p[j][2]), fabsf(p[j][3]))),
                         fmaxf(fmaxf(fabsf(q[j][0]), fabsf(q[j][1])), fmaxf(fabsf(q[j][2]), fabsf(q[j][3])))));
    }
  }
  m = fmaxf(m, __shfl_xor(m, 32));
  if (lane < 32) s_max[wave][lane] = m;
  __syncthreads();
  if (tid < 32) {
    float mm = s_max[0][tid];
#pragma unroll
    for (int w = 1; w < 8; ++w) mm = fmaxf(mm, s_max[w][tid]);
    s_er[tid] = exp_of(mm);
    s_max[0][tid] = mm;
  }
  __syncthreads();
  if (rmax != nullptr && cb == 0 && tid < 64) {
    float g = tid < 32 && r0 + tid < M ? s_max[0][tid] : 0.0f;
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) g = fmaxf(g, __shfl_xor(g, o));
    if (tid == 0) rmax[blockIdx.x] = g;
  }
  const float sc = __builtin_amdgcn_ldexpf(1.0f, kSW - s_er[lane & 31]);
  f32x16s acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    if (kb0 + j < kb1) {
      f16x8s a0, a1;
      split8(p[j], q[j], sc, a0, a1);
      acc = mfma3(a0, a1, b0[j], b1[j], acc);
    }
  }
  s_acc[wave][lane] = acc;
  __syncthreads();
  if (wave >= 2) return;
  // waves 0 and 1 each finish 8 of the 16 accumulator registers: the eight
  // K slices summed in wave order
  const int col = cb * 32 + (lane & 31);
  const int ec = ew[col];
  const float bv = BIAS ? bias[col] : 0.0f;
#pragma unroll
  for (int ee = 0; ee < 8; ++ee) {
    const int e = wave * 8 + ee;
    float v = s_acc[0][lane][e];
#pragma unroll
    for (int w = 1; w < 8; ++w) v += s_acc[w][lane][e];
    const int rr = 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3);
    const int64_t r = r0 + rr;
    if (r < M) {
      const float o = __builtin_amdgcn_ldexpf(v, s_er[rr] + ec - 2 * kSW);
      out[r * ldo + col] = BIAS ? o + bv : o;
    }
  }
}

__global__ void __launch_bounds__(512) k_gemm_tn_hs(const float* __restrict__ Y, int64_t ldy,
                                                    const float* __restrict__ X, int64_t ldx,
                                                    int64_t M, int N, int K,
                                                    float* __restrict__ dw, int accumulate) {
  __shared__ f32x16s s_acc[8][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.y * 32, k0 = blockIdx.x * 32;
  // wave's row slice: 16-row steps, [m_begin, m_end)
  const int64_t steps = (M + 15) / 16;
  const int64_t s_begin = steps * wave / 8, s_end = steps * (wave + 1) / 8;
  const int h = lane >> 5, c = lane & 31;
  const float* yc = Y + n0 + c;
  const float* xc = X + k0 + c;
  // exact column maxima over the slice (lane: column c, rows 8h .. 8h+7 of each step)
  float my = 0.0f, mx = 0.0f;
  for (int64_t s = s_begin; s < s_end; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t m = s * 16 + 8 * h + j;
      if (m < M) {
        my = fmaxf(my, fabsf(yc[m * ldy]));
        mx = fmaxf(mx, fabsf(xc[m * ldx]));
      }
    }
  }
  my = fmaxf(my, __shfl_xor(my, 32));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  const int ey = exp_of(my), ex = exp_of(mx);
  const float sy = __builtin_amdgcn_ldexpf(1.0f, kSW - ey);
  const float sx = __builtin_amdgcn_ldexpf(1.0f, kSW - ex);
  f32x16s acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
  // chunks of 4 steps: 64 loads per lane in flight before the MFMAs
  for (int64_t sc0 = s_begin; sc0 < s_end; sc0 += 4) {
    float yv[4][8], xv[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t m = (sc0 + u) * 16 + 8 * h + j;
        const bool ok = sc0 + u < s_end && m < M;
        yv[u][j] = ok ? yc[m * ldy] : 0.0f;
        xv[u][j] = ok ? xc[m * ldx] : 0.0f;
      }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (sc0 + u < s_end) {
        f16x8s a0, a1, b0, b1;
        split8(f32x4s{yv[u][0], yv[u][1], yv[u][2], yv[u][3]},
               f32x4s{yv[u][4], yv[u][5], yv[u][6], yv[u][7]}, sy, a0, a1);
        split8(f32x4s{xv[u][0], xv[u][1], xv[u][2], xv[u][3]},
               f32x4s{xv[u][4], xv[u][5], xv[u][6], xv[u][7]}, sx, b0, b1);
        acc = mfma3(a0, a1, b0, b1, acc);
      }
    }
  }
  // un-scale: dW row n (C-layout row) carries dY column n's exponent, column
  // k (this lane's column) X column k's
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int rr = 8 * (e >> 2) + 4 * h + (e & 3);
    const int eyr = __shfl(ey, rr);
    acc[e] = __builtin_amdgcn_ldexpf(acc[e], eyr + ex - 2 * kSW);
  }
  s_acc[wave][lane] = acc;
  __syncthreads();
  if (wave != 0) return;
  f32x16s sum = s_acc[0][lane];
#pragma unroll
  for (int w = 1; w < 8; ++w) sum += s_acc[w][lane];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int rr = 8 * (e >> 2) + 4 * h + (e & 3);
    float* o = dw + (int64_t)(n0 + rr) * K + k0 + c;
    *o = accumulate ? *o + sum[e] : sum[e];
  }
}

}  // namespace

int launch_gemm_nt_hs(const float* A, int64_t lda, int64_t M, int R, const void* Wf, int C,
                      const float* bias, float* out, int64_t ldo, float* rmax, hipStream_t st) {
  if (M <= 0) return 0;
  const f16x8s* wf = (const f16x8s*)Wf;
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * R * 4);
  if (R > 8 * 8 * 16) return fail("rb_gemm_nt_h: the few-rows kernel needs R <= 1024");
  const dim3 grid((unsigned)((M + 31) / 32), (unsigned)(C / 32));
  if (bias)
    k_gemm_nt_hs<true><<<grid, 512, 0, st>>>(A, lda, M, R, wf, ew, C, bias, out, ldo, rmax);
  else
    k_gemm_nt_hs<false><<<grid, 512, 0, st>>>(A, lda, M, R, wf, ew, C, bias, out, ldo, rmax);
  return launch_status("rb_gemm_nt_hs");
}

int launch_gemm_tn_hs(const float* Y, int64_t ldy, const float* X, int64_t ldx, int64_t M, int N,
                      int K, float* dw, int accumulate, hipStream_t st) {
  const dim3 grid((unsigned)(K / 32), (unsigned)(N / 32));
  k_gemm_tn_hs<<<grid, 512, 0, st>>>(Y, ldy, X, ldx, M, N, K, dw, accumulate);
  return launch_status("rb_gemm_tn_hs");
}

}  // namespace rb
