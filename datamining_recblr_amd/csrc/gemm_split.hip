// gemm_split.hip — fp32 projection GEMMs on the bf16 MFMA pipe.
//
// The encoder's projections (RecBLR.py:162,165,167,213,214 — nn.Linear in
// fp32) are tall-skinny: 409,600 rows at the benchmark shape, K, N in
// {128, 256, 512}.  gfx950's fp32 MFMA (v_mfma_f32_32x32x2_f32) peaks at
// 157 TFLOP/s, 1/16 of the bf16 pipe.  Here every fp32 operand x is split
// EXACTLY into three bf16 parts, x = x0 + x1 + x2 (x0 = bf16(x),
// x1 = bf16(x - x0), x2 = bf16(x - x0 - x1); |x1| <= 2^-9 |x|,
// |x2| <= 2^-18 |x|, remainder <= 2^-27 |x|), and the product is accumulated
// from the six partial products whose weight is >= 2^-18:
//     a.b ~= a0b0 + (a0b1 + a1b0) + (a0b2 + a1b1 + a2b0)
// Each partial product is exact in the fp32 accumulator (8 x 8 significant
// bits); the dropped terms (a1b2, a2b1, a2b2) are <= 2^-26 relative, below
// fp32's own rounding unit 2^-24.  So the result carries fp32 accuracy
// (tests/test_gpu_gemm.py: error vs fp64 on a par with hipBLASLt's fp32
// kernels) at 6/16 of the bf16 MFMA cost: an effective 2.67x of the fp32
// MFMA peak.
//
// k_gemm_nt: out[M, C] (+)= A[M, R] . Bm[C, R]^T (+ bias[C])
//   A   — fp32 activation rows (row stride lda), streamed from HBM once;
//         split on the fly into LDS (3 bf16 planes, MFMA-fragment order).
//   Bm  — the weight (forward: Bm = W [N, K]; input gradient: Bm = W^T),
//         pre-split once per call by k_split_weight into fragment order so a
//         wave loads each 32x16 fragment as one contiguous 1 KB (L2-resident).
// Workgroup: 256 threads = 4 waves (2 x 2), tile 128 rows x 128 columns,
// k-step 32, LDS double buffer for A; each wave owns 64 x 64 = 2 x 2 blocks of
// v_mfma_f32_32x32x16_bf16.  Column tiles of one row tile are dispatched to
// the same XCD back to back, so their A re-reads hit that XCD's L2.
//
// k_gemm_tn (weight gradient, split-K): part[s][C, R] = dY[rows_s]^T . X[rows_s]
//   (RecBLR.py autograd of the same Linears): both operands streamed along
//   the reduction (row) axis, split while being transposed into LDS.
#include "common.h"

namespace rb {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// exact 3-way split of two floats into packed bf16 pairs (v_cvt_pk_bf16_f32,
// round to nearest even; the residuals are exact in fp32)
__device__ __forceinline__ void split2(float a, float b, bf16x2& p0, bf16x2& p1, bf16x2& p2) {
  const f32x2 x = {a, b};
  p0 = __builtin_convertvector(x, bf16x2);
  const f32x2 r1 = x - __builtin_convertvector(p0, f32x2);
  p1 = __builtin_convertvector(r1, bf16x2);
  const f32x2 r2 = r1 - __builtin_convertvector(p1, f32x2);
  p2 = __builtin_convertvector(r2, bf16x2);
}

__device__ __forceinline__ bf16x4 cat4(bf16x2 a, bf16x2 b) {
  return bf16x4{a[0], a[1], b[0], b[1]};
}

// Fragment-ordered split weight: for Bm [C, R] (C % 32 == 0, R % 16 == 0)
//   Wf[((cb * (R/16) + kb) * 3 + plane) * 64 + lane][j]
//     = plane part of Bm[cb*32 + (lane & 31)][kb*16 + 8*(lane >> 5) + j]
// Bm = W (transpose = 0, W [C, R]) or W^T (transpose = 1, W [R, C]).
__global__ void __launch_bounds__(256) k_split_weight(const float* __restrict__ W, int64_t ldw,
                                                      int C, int R, int transpose,
                                                      bf16x8* __restrict__ Wf) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (cb, kb, lane)
  const int KB = R / 16;
  const int64_t total = (int64_t)(C / 32) * KB * 64;
  if (idx >= total) return;
  const int lane = (int)(idx & 63);
  const int64_t frag = idx >> 6;
  const int kb = (int)(frag % KB);
  const int cb = (int)(frag / KB);
  const int c = cb * 32 + (lane & 31);
  const int r0 = kb * 16 + 8 * (lane >> 5);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    v[j] = transpose ? W[(int64_t)(r0 + j) * ldw + c] : W[(int64_t)c * ldw + r0 + j];
  bf16x8 o0, o1, o2;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    bf16x2 p0, p1, p2;
    split2(v[j], v[j + 1], p0, p1, p2);
    o0[j] = p0[0]; o0[j + 1] = p0[1];
    o1[j] = p1[0]; o1[j + 1] = p1[1];
    o2[j] = p2[0]; o2[j + 1] = p2[1];
  }
  bf16x8* dst = Wf + (frag * 3) * 64 + lane;
  dst[0] = o0;
  dst[64] = o1;
  dst[128] = o2;
}

// Several weights in one launch (rb_gemm_split_weights): job j owns the
// 256-thread blocks [bstart[j], bstart[j+1]), each block one job (uniform).
struct SplitJobs {
  const float* W[RB_MAX_SPLIT_JOBS];
  bf16x8* Wf[RB_MAX_SPLIT_JOBS];
  int64_t ldw[RB_MAX_SPLIT_JOBS];
  int C[RB_MAX_SPLIT_JOBS], R[RB_MAX_SPLIT_JOBS], tr[RB_MAX_SPLIT_JOBS];
  int bstart[RB_MAX_SPLIT_JOBS + 1];
  int n;
};

__global__ void __launch_bounds__(256) k_split_weights(const SplitJobs jobs) {
  int j = 0;
  while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.bstart[j + 1]) ++j;
  const int C = jobs.C[j], R = jobs.R[j], transpose = jobs.tr[j];
  const int64_t ldw = jobs.ldw[j];
  const float* __restrict__ W = jobs.W[j];
  const int64_t idx = (int64_t)(blockIdx.x - jobs.bstart[j]) * 256 + threadIdx.x;
  const int KB = R / 16;
  const int64_t total = (int64_t)(C / 32) * KB * 64;
  if (idx >= total) return;
  const int lane = (int)(idx & 63);
  const int64_t frag = idx >> 6;
  const int kb = (int)(frag % KB);
  const int cb = (int)(frag / KB);
  const int c = cb * 32 + (lane & 31);
  const int r0 = kb * 16 + 8 * (lane >> 5);
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    v[k] = transpose ? W[(int64_t)(r0 + k) * ldw + c] : W[(int64_t)c * ldw + r0 + k];
  bf16x8 o0, o1, o2;
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
    bf16x2 p0, p1, p2;
    split2(v[k], v[k + 1], p0, p1, p2);
    o0[k] = p0[0]; o0[k + 1] = p0[1];
    o1[k] = p1[0]; o1[k + 1] = p1[1];
    o2[k] = p2[0]; o2[k + 1] = p2[1];
  }
  bf16x8* dst = jobs.Wf[j] + (frag * 3) * 64 + lane;
  dst[0] = o0;
  dst[64] = o1;
  dst[128] = o2;
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// NT GEMM: out[M, C] (+)= A[M, R] . Bm[C, R]^T (+ bias)
//
// One 512-thread workgroup per CU, persistent over its tiles (tile T =
// blockIdx.x + i * gridDim.x).  Tile 256 rows x 128 columns, k-step 32.
// Every k-step's operands travel global -> LDS by LDS-DMA
// (global_load_lds_dwordx4), waited with counted vmcnt:
//   A  raw fp32 tile (256 x 32: full 128-B row segments — 16-float slices
//      halve the HBM stream rate, tools/streamprobe.hip), 3-stage ring, issued
//      two k-steps ahead;
//   B  the k-step's pre-split weight fragments (4 column blocks x 2 k16 x 3
//      planes, 24 KB, L2-resident), 2-stage ring, one k-step ahead.
// Waves: 4 (rows) x 2 (columns); wave (wm, wn) owns rows 64wm..64wm+63 and
// columns 64wn..64wn+63 (2 x 2 blocks of v_mfma_f32_32x32x16_bf16).  A wave
// reads its A fragments as fp32 and splits them in registers.
// The column tiles of one row tile are neighbouring workgroups of one XCD
// (same blockIdx % 8) working in step, so their A re-reads hit that L2.
constexpr int G_BM = 256, G_BN = 128, G_BK = 32;
constexpr int G_NSA = 3, G_NSB = 2, G_WAVES = 8, G_WG_PER_CU = 1;
constexpr int G_THREADS = 64 * G_WAVES;
constexpr int G_LA = G_NSA - 1;                            // A steps in flight
constexpr int G_BDMA = (G_BN / 32) * 2 * 3 / G_WAVES;      // B DMAs per wave per step
constexpr int G_A_STAGE = G_BM * G_BK * 4;               // 32 KB
constexpr int G_B_STAGE = (G_BN / 32) * 2 * 3 * 1024;    // 24 KB
constexpr int G_LDS = G_NSA * G_A_STAGE + G_NSB * G_B_STAGE;  // 144 KB

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <typename T>
__device__ __forceinline__ T ds_read16(uint32_t addr) {
  T r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 8 fp32 -> three bf16x8 planes
__device__ __forceinline__ void split8(f32x4 x0, f32x4 x1, bf16x8 (&a)[3]) {
  const float xs[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    bf16x2 p0, p1, p2;
    split2(xs[j], xs[j + 1], p0, p1, p2);
    a[0][j] = p0[0]; a[0][j + 1] = p0[1];
    a[1][j] = p1[0]; a[1][j + 1] = p1[1];
    a[2][j] = p2[0]; a[2][j + 1] = p2[1];
  }
}

// the deferred epilogue's prefetched old outputs (accumulate mode only)
template <bool ACC>
struct OldVals {
  f32x2 v[8];
};
template <>
struct OldVals<false> {};

template <bool BIAS, bool ACC>
__global__ void __launch_bounds__(G_THREADS, G_WG_PER_CU) k_gemm_nt(const float* __restrict__ A, int64_t lda,
                                                    int64_t M, int R,
                                                    const bf16x8* __restrict__ Wf, int C,
                                                    const float* __restrict__ bias,
                                                    float* __restrict__ out, int64_t ldo,
                                                    int m_tiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nct = C / G_BN;
  const int KT = R / G_BK;
  const int KB16 = R / 16;
  const int n_tiles = ((m_tiles + 7) >> 3) * 8 * nct;
  const int G = gridDim.x;
  const int my_tiles = (int)blockIdx.x < n_tiles ? (n_tiles - 1 - (int)blockIdx.x) / G + 1 : 0;
  const int U = my_tiles * KT;  // k-steps of this workgroup
  if (U == 0) return;

  auto tile_of = [&](int i, int& mt, int& ct) {
    const int T = blockIdx.x + i * G;
    const int g = T >> 3;
    ct = g % nct;
    mt = (g / nct) * 8 + (T & 7);
  };

  // A stage image: row-major 128-B rows, 16-B chunk c of row r stored at
  // chunk c ^ ((r >> 1) & 7) (conflict-free fragment reads).  Each wave
  // DMAs rows 32w..32w+31 (4 instructions of 8 rows x 128 B).
  const int a_row8 = lane >> 3, a_pc = lane & 7;
  auto issueA = [&](int u) {
    const int i = u / KT, kt = u - i * KT;
    int mt, ct;
    tile_of(i, mt, ct);
    char* st = smem + (u % G_NSA) * G_A_STAGE;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rr = (wave * 4 + q) * 8 + a_row8;
      int64_t row = (int64_t)mt * G_BM + rr;
      if (row >= M) row = M - 1;
      const int lc = a_pc ^ ((rr >> 1) & 7);
      const float* src = A + row * lda + kt * G_BK + lc * 4;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + (wave * 4 + q) * 1024),
                                       16, 0, 0);
    }
  };
  // B stage image: fragment f = (cb * 2 + s) * 3 + plane, 1 KB each; wave w
  // DMAs fragments 3w..3w+2.
  auto issueB = [&](int u) {
    const int i = u / KT, kt = u - i * KT;
    int mt, ct;
    tile_of(i, mt, ct);
    char* st = smem + G_NSA * G_A_STAGE + (u % G_NSB) * G_B_STAGE;
#pragma unroll
    for (int q = 0; q < G_BDMA; ++q) {
      const int f = wave * G_BDMA + q;
      const int cb = f / 6, s = (f / 3) & 1, plane = f % 3;
      const bf16x8* src =
          Wf + ((int64_t)((ct * (G_BN / 32) + cb) * KB16 + kt * 2 + s) * 3 + plane) * 64 + lane;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + f * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[m][n][e] = 0.0f;

  issueB(0);
  for (int a = 0; a < G_LA && a < U; ++a) issueA(a);

  const uint32_t smem_base = (uint32_t)(uintptr_t)(lds_ptr_t)smem;
  // fragment read offsets inside an A stage: row 64wm + 32rb + (lane & 31),
  // logical chunks 4s + 2h and 4s + 2h + 1
  uint32_t a_off[2][2][2];  // [rb][s][half]
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int row = wm * 64 + rb * 32 + (lane & 31);
    const int sw = (row >> 1) & 7;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        a_off[rb][s][c] = row * 128 + (((4 * s + 2 * (lane >> 5) + c) ^ sw) << 4);
  }
  const int ccol = lane & 31;

  // deferred epilogue: quarter q stores block (m, n) = (q & 1, q >> 1) of the
  // previous tile (8 dwordx2 stores: lanes (2p, 2p+1) swap one value so each
  // stores 2 adjacent columns of one row)
  f32x16 pend[2][2];
  int pend_mt = -1, pend_ct = 0, pend_q = 4;
  bool stored_prev = false;  // step u-1 issued 8 stores after its DMAs
  // ACC: the old output values of the next quarter, loaded one phase ahead
  // (before the step's DMAs, so waiting for them never drains those)
  OldVals<ACC> oldb;
  auto load_old = [&]() {
    if constexpr (ACC) {
      f32x2 (&oldv)[8] = oldb.v;
      const int m = pend_q & 1, n = pend_q >> 1;
      const bool full = (int64_t)pend_mt * G_BM + G_BM <= M;
      const bool odd = lane & 1;
      const int col = pend_ct * G_BN + wn * 64 + n * 32 + (ccol & ~1);
      const int64_t rbase = (int64_t)pend_mt * G_BM + wm * 64 + m * 32 + 4 * (lane >> 5);
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        const int64_t r = rbase + (e & 3) + 8 * (e >> 2) + (odd ? 1 : 0);
        oldv[e >> 1] = (full || r < M) ? *reinterpret_cast<const f32x2*>(out + r * ldo + col)
                                       : f32x2{0.0f, 0.0f};
      }
    }
  };
  auto store_block = [&](const f32x16& blk, int m, int n) {
    const bool full = (int64_t)pend_mt * G_BM + G_BM <= M;
    const bool odd = lane & 1;
    const int col = pend_ct * G_BN + wn * 64 + n * 32 + (ccol & ~1);
    float b0 = 0.0f, b1 = 0.0f;
    if (BIAS) { b0 = bias[col]; b1 = bias[col + 1]; }
    const int64_t rbase = (int64_t)pend_mt * G_BM + wm * 64 + m * 32 + 4 * (lane >> 5);
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      const float send = odd ? blk[e] : blk[e + 1];
      const float recv = __builtin_bit_cast(
          float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1, 0xF, 0xF, false));
      float v0 = odd ? recv : blk[e];
      float v1 = odd ? blk[e + 1] : recv;
      const int64_t r = rbase + (e & 3) + 8 * (e >> 2) + (odd ? 1 : 0);
      if (full || r < M) {
        f32x2* o = reinterpret_cast<f32x2*>(out + r * ldo + col);
        if (BIAS) { v0 += b0; v1 += b1; }
        if constexpr (ACC) {
          v0 += oldb.v[e >> 1][0];
          v1 += oldb.v[e >> 1][1];
        }
        __builtin_nontemporal_store(f32x2{v0, v1}, o);
      }
    }
    return full;
  };
  // static register indexing (a runtime pend[q] would live in scratch)
  auto store_quarter = [&]() {
    const int q = pend_q++;
    if (q == 0) return store_block(pend[0][0], 0, 0);
    if (q == 1) return store_block(pend[1][0], 1, 0);
    if (q == 2) return store_block(pend[0][1], 0, 1);
    return store_block(pend[1][1], 1, 1);
  };

  int i = 0, kt = 0;
  for (int u = 0; u < U; ++u) {
    // operands of step u landed (own DMAs): the ops younger than B(u) are
    // A(u+1) (4) and the 8 deferred stores step u-1 issued after it
    if (u + 1 < U) {
      constexpr int NA = G_LA == 2 ? 4 : 0;
      if (stored_prev) wait_vm<NA + 8>(); else wait_vm<NA>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();

    // per k16 sub-step: 4 A + 6 B fragment reads, split, 24 MFMAs; the next
    // steps' DMAs and a quarter of the previous tile's stores go between the
    // two sub-steps
    const uint32_t sa = smem_base + (u % G_NSA) * G_A_STAGE;
    const uint32_t sb = smem_base + G_NSA * G_A_STAGE + (u % G_NSB) * G_B_STAGE + lane * 16;
    auto substep = [&](int s) {
      f32x4 x[2][2];
      bf16x8 b[2][3];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int c = 0; c < 2; ++c) x[rb][c] = ds_read16<f32x4>(sa + a_off[rb][s][c]);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          b[cb][p] = ds_read16<bf16x8>(sb + (((wn * 2 + cb) * 2 + s) * 3 + p) * 1024);
      asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(x[0][0]), "+v"(x[0][1]), "+v"(x[1][0]), "+v"(x[1][1]));
      bf16x8 a[2][3];
      split8(x[0][0], x[0][1], a[0]);
      split8(x[1][0], x[1][1], a[1]);
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[0][2]), "+v"(b[1][0]), "+v"(b[1][1]),
                     "+v"(b[1][2]));
      // small partial products first; 4 independent accumulators interleave
      constexpr int PA[6] = {2, 1, 0, 1, 0, 0};
      constexpr int PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            acc[m][n] = mfma(a[m][PA[q]], b[n][PB[q]], acc[m][n]);
          }
    };
    if (pend_mt >= 0 && pend_q < 4) load_old();
    substep(0);
    if (u + 1 < U) issueB(u + 1);
    if (u + G_LA < U) issueA(u + G_LA);
    stored_prev = false;
    if (pend_mt >= 0 && pend_q < 4) {
      // a partial tile's guarded stores may issue fewer than 8: not counted
      stored_prev = store_quarter();
    }
    substep(1);

    if (kt == KT - 1) {
      // the tile's results move to pend[] and are stored a quarter per step
      // during the next tile's first 4 steps (behind its MFMAs)
      int mt, ct;
      tile_of(i, mt, ct);
      // tiles shorter than 4 steps: finish the previous tile first (extra
      // stores only make the next vmcnt waits stricter)
      while (pend_mt >= 0 && pend_q < 4) {
        load_old();
        store_quarter();
      }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          pend[m][n] = acc[m][n];
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[m][n][e] = 0.0f;
        }
      pend_mt = mt < m_tiles ? mt : -1;
      pend_ct = ct;
      pend_q = 0;
      kt = 0;
      ++i;
    } else {
      ++kt;
    }
  }
  while (pend_mt >= 0 && pend_q < 4) {
    load_old();
    store_quarter();
  }
}

template <bool BIAS, bool ACC>
void set_lds_attr() {
  static bool done = false;  // benign race: idempotent
  if (!done) {
    (void)hipFuncSetAttribute((const void*)k_gemm_nt<BIAS, ACC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, G_LDS);
    done = true;
  }
}

template <bool BIAS, bool ACC>
void run_nt(const float* A, int64_t lda, int64_t M, int R, const bf16x8* wf, int C,
            const float* bias, float* out, int64_t ldo, int m_tiles, unsigned grid,
            hipStream_t st) {
  set_lds_attr<BIAS, ACC>();
  k_gemm_nt<BIAS, ACC><<<grid, G_THREADS, G_LDS, st>>>(A, lda, M, R, wf, C, bias, out, ldo, m_tiles);
}

}  // namespace

int launch_split_weight(const float* W, int64_t ldw, int C, int R, int transpose, void* Wf,
                        hipStream_t st) {
  const int64_t total = (int64_t)(C / 32) * (R / 16) * 64;
  k_split_weight<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(W, ldw, C, R, transpose,
                                                                  (bf16x8*)Wf);
  return launch_status("rb_gemm_split_weight");
}

int launch_split_weights(const rb_split_job* jobs, int n, hipStream_t st) {
  SplitJobs sj{};
  sj.n = n;
  int blocks = 0;
  for (int j = 0; j < n; ++j) {
    sj.W[j] = jobs[j].W;
    sj.Wf[j] = (bf16x8*)jobs[j].Wf;
    sj.ldw[j] = jobs[j].ldw;
    sj.C[j] = (int)jobs[j].C;
    sj.R[j] = (int)jobs[j].R;
    sj.tr[j] = (int)jobs[j].transpose;
    sj.bstart[j] = blocks;
    blocks += (int)(((jobs[j].C / 32) * (jobs[j].R / 16) * 64 + 255) / 256);
  }
  sj.bstart[n] = blocks;
  k_split_weights<<<(unsigned)blocks, 256, 0, st>>>(sj);
  return launch_status("rb_gemm_split_weights");
}

int launch_gemm_nt(const float* A, int64_t lda, int64_t M, int R, const void* Wf, int C,
                   const float* bias, float* out, int64_t ldo, int accumulate, hipStream_t st) {
  const int m_tiles = (int)((M + G_BM - 1) / G_BM);
  const int64_t n_tiles = (int64_t)((m_tiles + 7) / 8) * 8 * (C / G_BN);
  // persistent: one workgroup per CU (a multiple of 8: the XCD pairing above)
  const unsigned grid = (unsigned)std::min<int64_t>(n_tiles, (int64_t)num_cus() / 8 * 8 * G_WG_PER_CU);
  const bf16x8* wf = (const bf16x8*)Wf;
  if (bias && accumulate)
    run_nt<true, true>(A, lda, M, R, wf, C, bias, out, ldo, m_tiles, grid, st);
  else if (bias)
    run_nt<true, false>(A, lda, M, R, wf, C, bias, out, ldo, m_tiles, grid, st);
  else if (accumulate)
    run_nt<false, true>(A, lda, M, R, wf, C, bias, out, ldo, m_tiles, grid, st);
  else
    run_nt<false, false>(A, lda, M, R, wf, C, bias, out, ldo, m_tiles, grid, st);
  return launch_status("rb_gemm_nt");
}

}  // namespace rb
