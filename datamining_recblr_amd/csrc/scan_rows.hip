// scan_rows.hip — parallel_scan on the reference layout [B, C, T] (T contiguous).
//
// One wave per row.  Each lane owns 4 consecutive steps (one float4), reduces
// them to a summary (prod a, local h), the 64 lane summaries are combined by
// a Kogge-Stone scan with wavefront shuffles, and the row walks its 256-step
// blocks with a serial carry.  The combine operator is the reference's
// first_order_op (parallel_scan.py:35-41): (x_l, f_l) o (x_r, f_r) =
// (x_l f_r + x_r, f_l f_r); the backward is the reverse scan with shifted
// gates of Scan.backward (parallel_scan.py:97-114).
#include "common.h"

namespace rb {
namespace {

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

}  // namespace

int launch_scan_fwd(const float* gates, const float* tokens, float* states, int64_t rows,
                    int64_t T, hipStream_t st) {
  const int64_t blocks = (rows + 3) / 4;
  const bool vec = (T % 4 == 0) && aligned16(gates) && aligned16(tokens) && aligned16(states);
  if (vec)
    hipLaunchKernelGGL(k_scan_rows_fwd<true>, dim3((unsigned)blocks), dim3(256), 0, st, gates,
                       tokens, states, rows, T);
  else
    hipLaunchKernelGGL(k_scan_rows_fwd<false>, dim3((unsigned)blocks), dim3(256), 0, st, gates,
                       tokens, states, rows, T);
  return launch_status("rb_scan_fwd");
}

int launch_scan_bwd(const float* gates, const float* states, const float* grad, float* d_gates,
                    float* d_tokens, int64_t rows, int64_t T, hipStream_t st) {
  const int64_t blocks = (rows + 3) / 4;
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

}  // namespace rb
