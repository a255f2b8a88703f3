// reduce.hip — fixed-order column sums of per-block / per-split partials.
//
// Every backward kernel here writes partial sums (per batch row, per row
// block, per split-K slice) instead of using atomics; this one launch turns
// them into the final gradients.  It replaces torch's sum(0), which for
// these shapes costs a hipMemset of a semaphore buffer plus a reduction
// launch, and fixes the summation order independently of the device:
//   out[m, c] = ((S_0 + S_1) + ...) + S_{RG-1},  S_g = sum_{p = g, g+RG, ...} in[m, p, c]
// with RG = 4 (P <= 256) or 16 row groups, each S_g summed in increasing p
// (16 for the wide weight-gradient partials, read four columns per thread).
#include "common.h"

namespace rb {
namespace {

template <int RG>
__global__ __launch_bounds__(64 * RG) void k_colsum(const float* __restrict__ in, int64_t P,
                                                    int64_t C, int64_t rs, int64_t ms,
                                                    int64_t cblocks, float* __restrict__ out) {
  __shared__ float red[RG][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t m = blockIdx.x / cblocks;
  const int64_t c = (blockIdx.x - m * cblocks) * 64 + tx;
  const float* base = in + m * ms + c;
  float s = 0.0f;
  if (c < C) {
    int64_t p = ty;
    for (; p + 3 * RG < P; p += 4 * RG) {   // 4 independent loads in flight, order kept
      const float a = base[p * rs], b = base[(p + RG) * rs];
      const float d = base[(p + 2 * RG) * rs], e = base[(p + 3 * RG) * rs];
      s = (((s + a) + b) + d) + e;
    }
    for (; p < P; p += RG) s += base[p * rs];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < C) {
    float t = red[0][tx];
#pragma unroll
    for (int g = 1; g < RG; ++g) t += red[g][tx];
    out[m * C + c] = t;
  }
}

// The same sums, four adjacent columns per thread (16-B loads; C, rs, ms
// multiples of 4 and 16-B aligned operands): per column the identical order,
// so the results are bitwise those of k_colsum.
template <int RG>
__global__ __launch_bounds__(64 * RG) void k_colsum4(const float* __restrict__ in, int64_t P,
                                                     int64_t C, int64_t rs, int64_t ms,
                                                     int64_t cblocks, float* __restrict__ out) {
  __shared__ float4 red[RG][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t m = blockIdx.x / cblocks;
  const int64_t c = ((blockIdx.x - m * cblocks) * 64 + tx) * 4;
  const float* base = in + m * ms + c;
  float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  auto add = [](float4& acc, const float4& v) {
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  };
  if (c < C) {
    int64_t p = ty;
    for (; p + 3 * RG < P; p += 4 * RG) {
      const float4 a = *reinterpret_cast<const float4*>(base + p * rs);
      const float4 b = *reinterpret_cast<const float4*>(base + (p + RG) * rs);
      const float4 d = *reinterpret_cast<const float4*>(base + (p + 2 * RG) * rs);
      const float4 e = *reinterpret_cast<const float4*>(base + (p + 3 * RG) * rs);
      add(s, a); add(s, b); add(s, d); add(s, e);
    }
    for (; p < P; p += RG) add(s, *reinterpret_cast<const float4*>(base + p * rs));
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < C) {
    float4 t = red[0][tx];
#pragma unroll
    for (int g = 1; g < RG; ++g) add(t, red[g][tx]);
    *reinterpret_cast<float4*>(out + m * C + c) = t;
  }
}

// The two-level sum of rb_colsum_chunked in ONE launch: workgroup (m, column
// block, chunk) sums the chunk's CH rows in k_colsum<RG>'s order and stores
// the chunk sum to part[m][chunk]; the last of a column block's nch
// workgroups to arrive (an agent-scope ticket) sums the chunk sums in the
// same order, so the result is bitwise that of two k_colsum<RG> launches
// (chunks, then the chunk sums).  Hand-off: plain stores, every storing wave
// drains, the workgroup barrier, one agent-scope release before the ticket;
// the last arriver acquires before reading (cdna_hip_programming.md §6
// Guideline 16, the counter form) and resets its ticket for the next call
// (the tickets are zeroed once when the caller allocates them).
template <int RG, int CH>
__global__ __launch_bounds__(64 * RG) void k_colsum_2l(const float* __restrict__ in, int64_t C,
                                                       int64_t rs, int64_t cblocks, int nch,
                                                       float* __restrict__ part,
                                                       unsigned* __restrict__ cnt,
                                                       float* __restrict__ out) {
  constexpr int NL = CH / RG;   // rows per thread, all loads in flight at once (one
                                // round trip: a runtime chunk size left the compiler
                                // four dependent batches of four, ~8-13 us per call)
  __shared__ float red[RG][64];
  __shared__ int s_last;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t b = blockIdx.x;
  const int ch = (int)(b % nch);
  const int64_t mc = b / nch;
  const int64_t m = mc / cblocks;
  const int64_t c = (mc - m * cblocks) * 64 + tx;
  {
    const float* base = in + ((m * nch + ch) * (int64_t)CH) * rs + c;
    float s = 0.0f;
    if (c < C) {
      float v[NL];
#pragma unroll
      for (int i = 0; i < NL; ++i) v[i] = base[(int64_t)(ty + i * RG) * rs];
#pragma unroll
      for (int i = 0; i < NL; ++i) s += v[i];   // increasing p: k_colsum<RG>'s order
    }
    red[ty][tx] = s;
    __syncthreads();
    if (ty == 0 && c < C) {
      float t = red[0][tx];
#pragma unroll
      for (int g = 1; g < RG; ++g) t += red[g][tx];
      part[(m * nch + ch) * C + c] = t;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // keep: the fence's own wait may be dropped
    // wrapping increment (old >= nch - 1 ? 0 : old + 1): the ticket is back
    // at 0 after the last arrival without a separate reset store, and a
    // ticket outside [0, nch) is pulled back into range by the next launch
    const unsigned old = __builtin_amdgcn_atomic_inc32(&cnt[mc], (unsigned)(nch - 1),
                                                       __ATOMIC_RELAXED, "agent");
    const int last = old == (unsigned)(nch - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;   // workgroup-uniform
  const float* base = part + m * nch * C + c;
  float s = 0.0f;
  if (c < C) {
    int p = ty;
    for (; p + 7 * RG < nch; p += 8 * RG) {   // 8 independent loads in flight, order kept
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = base[(int64_t)(p + i * RG) * C];
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[i];
    }
    for (; p < nch; p += RG) s += base[(int64_t)p * C];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < C) {
    float t = red[0][tx];
#pragma unroll
    for (int g = 1; g < RG; ++g) t += red[g][tx];
    out[m * C + c] = t;
  }
}

// out[g] = max |x[r][c]| over the rows r of 32-row group g (a partial last
// group too) and all c < C: the row-group maxima rb_gemm_tn_h takes as operand
// scales, for tensors no f16 GEMM has read.  One 256-thread workgroup per
// group: the group's rows x 16-B pieces (or single columns) spread over the
// threads, every load independent, then a workgroup max.
__global__ __launch_bounds__(256) void k_group_absmax(const float* __restrict__ x, int64_t n,
                                                      int64_t c, int64_t ld,
                                                      float* __restrict__ out, int vec4) {
  __shared__ float red[4];
  const int64_t g = blockIdx.x;
  const int64_t r0 = g * 32;
  const int nr = (int)((r0 + 32 < n ? r0 + 32 : n) - r0);
  float m = 0.0f;
  if (vec4) {
    const int c4 = (int)(c / 4);
    const int tot = nr * c4;
#pragma unroll 4
    for (int e = threadIdx.x; e < tot; e += 256) {
      const int r = e / c4, k = e - r * c4;
      const float4 v = *reinterpret_cast<const float4*>(x + (r0 + r) * ld + 4 * k);
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  } else {
    const int64_t tot = (int64_t)nr * c;
    for (int64_t e = threadIdx.x; e < tot; e += 256) {
      const int64_t r = e / c, k = e - r * c;
      m = fmaxf(m, fabsf(x[(r0 + r) * ld + k]));
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[g] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

}  // namespace

int launch_group_absmax(const float* x, int64_t n, int64_t c, int64_t ld, float* out,
                        hipStream_t st) {
  const int64_t ng = (n + 31) / 32;
  const int vec4 = c % 4 == 0 && ld % 4 == 0 && aligned16(x) && c <= (int64_t)1 << 24;
  if (ng > 0x7fffffffLL || (!vec4 && c > ((int64_t)1 << 40)))
    return fail("rb_group_absmax: too many groups");
  hipLaunchKernelGGL(k_group_absmax, dim3((unsigned)ng), dim3(256), 0, st, x, n, c, ld, out, vec4);
  return launch_status("rb_group_absmax");
}

int launch_colsum(const float* in, int64_t M, int64_t P, int64_t C, int64_t rs, int64_t ms,
                  float* out, hipStream_t st) {
  // wide partials (the weight gradients' [S, N*K] row-chunk sums): 16-B
  // loads, 16 row groups (64 KB in flight per CU)
  if (C >= 8192 && P >= 64 && C % 4 == 0 && rs % 4 == 0 && ms % 4 == 0 && aligned16(in) &&
      aligned16(out)) {
    const int64_t cb4 = (C / 4 + 63) / 64;
    hipLaunchKernelGGL(k_colsum4<16>, dim3((unsigned)(M * cb4)), dim3(1024), 0, st, in, P, C, rs,
                       ms, cb4, out);
    return launch_status("rb_colsum");
  }
  if (C >= 8192 && P <= 256 && C % 4 == 0 && rs % 4 == 0 && ms % 4 == 0 && aligned16(in) &&
      aligned16(out)) {
    // few wide partials (split-K GEMM slices): the k_colsum<4> order, 16-B loads
    const int64_t cb4 = (C / 4 + 63) / 64;
    hipLaunchKernelGGL(k_colsum4<4>, dim3((unsigned)(M * cb4)), dim3(256), 0, st, in, P, C, rs,
                       ms, cb4, out);
    return launch_status("rb_colsum");
  }
  const int64_t cblocks = (C + 63) / 64;
  const unsigned grid = (unsigned)(M * cblocks);
  if (P <= 256)
    hipLaunchKernelGGL(k_colsum<4>, dim3(grid), dim3(256), 0, st, in, P, C, rs, ms, cblocks, out);
  else
    hipLaunchKernelGGL(k_colsum<16>, dim3(grid), dim3(1024), 0, st, in, P, C, rs, ms, cblocks,
                       out);
  return launch_status("rb_colsum");
}

int launch_colsum_chunked(const float* in, int64_t M, int64_t P, int64_t C, int64_t rs, int CH,
                          float* part, unsigned* cnt, float* out, hipStream_t st) {
  const int64_t cblocks = (C + 63) / 64;
  const int nch = (int)(P / CH);
  const dim3 grid((unsigned)(M * cblocks * nch));
  switch (CH) {
    case 64:
      hipLaunchKernelGGL((k_colsum_2l<4, 64>), grid, dim3(256), 0, st, in, C, rs, cblocks, nch,
                         part, cnt, out);
      break;
    case 128:
      hipLaunchKernelGGL((k_colsum_2l<4, 128>), grid, dim3(256), 0, st, in, C, rs, cblocks, nch,
                         part, cnt, out);
      break;
    case 256:
      hipLaunchKernelGGL((k_colsum_2l<4, 256>), grid, dim3(256), 0, st, in, C, rs, cblocks, nch,
                         part, cnt, out);
      break;
    default:
      return fail("rb_colsum_chunked: chunk_rows must be 64, 128 or 256");
  }
  return launch_status("rb_colsum_chunked");
}

}  // namespace rb
