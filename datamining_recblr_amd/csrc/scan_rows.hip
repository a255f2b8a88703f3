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

template <typename TS, bool VEC4>
__global__ void __launch_bounds__(256)
k_scan_rows_fwd(const TS* __restrict__ gates, const TS* __restrict__ tokens,
                TS* __restrict__ out, int64_t rows, int64_t T) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // wave-uniform
  const TS* g = gates + row * T;
  const TS* x = tokens + row * T;
  TS* o = out + row * T;
  float carry = 0.0f;
  for (int64_t t0 = 0; t0 < T; t0 += 4 * kWave) {
    const int64_t t = t0 + 4 * lane;
    float a[4], v[4];
    if (VEC4 && t + 3 < T) {
      ldv(a, g + t);
      ldv(v, x + t);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = t + j < T;
        a[j] = ok ? (float)g[t + j] : 1.0f;  // identity element (x=0, f=1)
        v[j] = ok ? (float)x[t + j] : 0.0f;
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
      stv(o + t, res);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (t + j < T) o[t + j] = (TS)res[j];
    }
    const float A63 = __shfl(A, kWave - 1, kWave);
    const float X63 = __shfl(X, kWave - 1, kWave);
    carry = carry * A63 + X63;
  }
}

// Reverse scan with shifted gates (parallel_scan.py:106-113):
//   d_t = d_{t+1} * a_{t+1} + grad_t, d_gates_t = h_{t-1} d_t, d_tokens = d.
template <typename TS, bool VEC4>
__global__ void __launch_bounds__(256)
k_scan_rows_bwd(const TS* __restrict__ gates, const TS* __restrict__ states,
                const TS* __restrict__ grad, TS* __restrict__ d_gates,
                TS* __restrict__ d_tokens, int64_t rows, int64_t T) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TS* g = gates + row * T;
  const TS* s = states + row * T;
  const TS* gr = grad + row * T;
  TS* dg = d_gates + row * T;
  TS* dt = d_tokens + row * T;
  const int64_t nblk = (T + 4 * kWave - 1) / (4 * kWave);
  float carry = 0.0f;     // d at the first step after the block
  float a_next = 1.0f;    // gates at the first step after the block
  for (int64_t blk = nblk - 1; blk >= 0; --blk) {
    const int64_t t0 = blk * 4 * kWave;
    const int64_t t = t0 + 4 * lane;
    float a[4], y[4], hs[4];
    if (VEC4 && t + 3 < T) {
      ldv(a, g + t);
      ldv(y, gr + t);
      ldv(hs, s + t);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = t + j < T;
        a[j] = ok ? (float)g[t + j] : 1.0f;
        y[j] = ok ? (float)gr[t + j] : 0.0f;
        hs[j] = ok ? (float)s[t + j] : 0.0f;
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
    if (lane == 0) hprev0 = (t0 > 0) ? (float)s[t0 - 1] : 0.0f;
    float dres[4], gres[4];
#pragma unroll
    for (int j = 3; j >= 0; --j) {
      d = d * as[j] + y[j];
      const float hp = (j == 0) ? hprev0 : hs[j - 1];
      dres[j] = d;
      gres[j] = hp * d;
    }
    if (VEC4 && t + 3 < T) {
      stv(dt + t, dres);
      stv(dg + t, gres);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (t + j < T) {
          dt[t + j] = (TS)dres[j];
          dg[t + j] = (TS)gres[j];
        }
    }
    const float A0 = __shfl(A, 0, kWave);
    const float D0 = __shfl(D, 0, kWave);
    carry = carry * A0 + D0;
    a_next = __shfl(a[0], 0, kWave);
  }
}

template <typename TS>
bool al4s(const void* p) { return reinterpret_cast<uintptr_t>(p) % (4 * sizeof(TS)) == 0; }

template <typename TS>
int scan_fwd_t(const TS* gates, const TS* tokens, TS* states, int64_t rows, int64_t T,
               hipStream_t st) {
  const int64_t blocks = (rows + 3) / 4;
  const bool vec = (T % 4 == 0) && al4s<TS>(gates) && al4s<TS>(tokens) && al4s<TS>(states);
  if (vec)
    hipLaunchKernelGGL((k_scan_rows_fwd<TS, true>), dim3((unsigned)blocks), dim3(256), 0, st,
                       gates, tokens, states, rows, T);
  else
    hipLaunchKernelGGL((k_scan_rows_fwd<TS, false>), dim3((unsigned)blocks), dim3(256), 0, st,
                       gates, tokens, states, rows, T);
  return launch_status("rb_scan_fwd");
}

template <typename TS>
int scan_bwd_t(const TS* gates, const TS* states, const TS* grad, TS* d_gates, TS* d_tokens,
               int64_t rows, int64_t T, hipStream_t st) {
  const int64_t blocks = (rows + 3) / 4;
  const bool vec = (T % 4 == 0) && al4s<TS>(gates) && al4s<TS>(states) && al4s<TS>(grad) &&
                   al4s<TS>(d_gates) && al4s<TS>(d_tokens);
  if (vec)
    hipLaunchKernelGGL((k_scan_rows_bwd<TS, true>), dim3((unsigned)blocks), dim3(256), 0, st,
                       gates, states, grad, d_gates, d_tokens, rows, T);
  else
    hipLaunchKernelGGL((k_scan_rows_bwd<TS, false>), dim3((unsigned)blocks), dim3(256), 0, st,
                       gates, states, grad, d_gates, d_tokens, rows, T);
  return launch_status("rb_scan_bwd");
}

}  // namespace

int launch_scan_fwd(const float* gates, const float* tokens, float* states, int64_t rows,
                    int64_t T, hipStream_t st) {
  return scan_fwd_t<float>(gates, tokens, states, rows, T, st);
}

int launch_scan_fwd_bf16(const bf16_t* gates, const bf16_t* tokens, bf16_t* states,
                         int64_t rows, int64_t T, hipStream_t st) {
  return scan_fwd_t<bf16_t>(gates, tokens, states, rows, T, st);
}

int launch_scan_bwd(const float* gates, const float* states, const float* grad, float* d_gates,
                    float* d_tokens, int64_t rows, int64_t T, hipStream_t st) {
  return scan_bwd_t<float>(gates, states, grad, d_gates, d_tokens, rows, T, st);
}

int launch_scan_bwd_bf16(const bf16_t* gates, const bf16_t* states, const bf16_t* grad,
                         bf16_t* d_gates, bf16_t* d_tokens, int64_t rows, int64_t T,
                         hipStream_t st) {
  return scan_bwd_t<bf16_t>(gates, states, grad, d_gates, d_tokens, rows, T, st);
}

}  // namespace rb
