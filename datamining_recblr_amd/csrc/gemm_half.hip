// gemm_half.hip — fp32 projection GEMMs on the f16 MFMA pipe, 3 products.
//
// The encoder's projections (RecBLR.py:162,165,167,213,214 — nn.Linear in
// fp32) are tall and skinny (ntok ~ 200k-410k rows, K, N in {128, 256, 512}):
// at the HBM roofline they are bound by their row streams (the fp32 output
// write or the fp32 input read), not by arithmetic, as soon as the
// arithmetic runs at >= 1/3 of the bf16 pipe.  The six-product bf16 split
// (round 1's gemm_split.hip, since removed) needs 6x the bf16 flops and is MFMA-bound at the tile
// level; here each operand is split into TWO fp16 parts and three products
// are accumulated:
//     x = 2^-s (x0 + x1),  x0 = f16(x 2^s),  x1 = f16(x 2^s - x0)
//     a.b ~= 2^-(sa+sb) (a0 b0 + a0 b1 + a1 b0)
// fp16 carries 11 significant bits, so x0 + x1 holds 22 (|x - x0 - x1| <=
// 2^-22 |x| for values near the scale, RNE), every product is exact in the
// fp32 accumulator and the dropped a1 b1 is <= 2^-22 relative: the result is
// within a few fp32 units of an fp32 GEMM (tests/test_gpu_gemm.py measures it
// against fp64 beside hipBLASLt's fp32 kernels).  fp16's exponent range is
// handled with power-of-two scales, which are exact:
//   * weights (Bm [C, R]): one scale per output column c (a row of Bm), fixed
//     when the image is built: the column max lands in [2^13, 2^14);
//   * activations / gradients (A [M, R]): one scale per ROW (a row scale
//     factors out of out[m, :]), chosen online: the first 16 k-values of a
//     tile's row set its max to [2^3, 2^4), and 11 bits of headroom keep
//     every later value < 2^15 (finite in fp16).  A later value beyond the
//     headroom (rare: a row whose first 16 entries are all tiny or zero)
//     re-scales that row — its accumulators are multiplied by the exact
//     power-of-two ratio — so no input overflows and no row loses precision.
//     Values far below their row max keep an absolute error <= 2^-29 of it
//     (fp16 subnormal residuals), far below fp32 rounding of the dot product.
// The output is un-scaled in the epilogue with v_ldexp (exact).
//
// k_gemm_nt_h: out[M, C] (+)= A[M, R] . Bm[C, R]^T (+ bias[C])
//   One 512-thread workgroup per CU, persistent over 256 x 128 tiles, k-step
//   32.  A (raw fp32, full 128-B row segments) and the pre-split weight
//   fragments reach LDS by LDS-DMA (global_load_lds_dwordx4) into 3- and
//   2-stage rings waited with counted vmcnt.  8 waves x 32 rows each: a wave
//   DMAs, reads and splits only its own 32 rows (every A element is split
//   once) and multiplies them by all 128 columns (4 blocks of
//   v_mfma_f32_32x32x16_f16 x 3 products per k16).  The epilogue (un-scale,
//   bias) is deferred by one tile and stored a block per k-step behind the
//   next tile's MFMAs, as dwordx4 row pieces after a 4 x 4 transpose inside
//   each lane quad (4 stores per block instead of 16 dword column stores).
//   The next steps' DMAs are issued right after each k-step's barrier.  Per k-step the instruction stream is kept lean:
//   DMA and store addresses are a wave-uniform base plus a constant 32-bit
//   lane offset, tile coordinates advance incrementally (divisions once per
//   tile), and the overflow check is one compare + ballot per k16.
#include "common.h"

#include <type_traits>

namespace rb {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTA = 4;       // row scale target: first-k16 row max in [2^(kTA-1), 2^kTA)
constexpr int kHead = 11;    // later values up to 2^(kTA + kHead) = 2^15 (fp16 max 65504)
constexpr int kTW = 14;      // weight column scale target: column max in [2^13, 2^14)
constexpr int kSent = -4096; // row exponent of a row that has been all zero so far

// 2 fp32 (already scaled) -> hi, lo fp16 pairs (v_cvt_pk_f16_f32, RNE; the
// residual is exact in fp32)
__device__ __forceinline__ void split2h(f32x2 x, f16x2& h0, f16x2& h1) {
  h0 = __builtin_convertvector(x, f16x2);
  const f32x2 r = x - __builtin_convertvector(h0, f32x2);
  h1 = __builtin_convertvector(r, f16x2);
}

__device__ __forceinline__ f32x16 mfma_h(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// max(|a|, |b|, |c|) in one instruction (no NaN canonicalisation: a NaN input
// propagates to the output through the MFMA anyway)
__device__ __forceinline__ float max3abs(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ float max8abs(f32x4 x, f32x4 y) {
  float m = max3abs(x[0], x[1], x[2]);
  m = max3abs(m, x[3], y[0]);
  m = max3abs(m, y[1], y[2]);
  float r;
  asm("v_max_f32 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(y[3]));
  return r;
}

// ---------------------------------------------------------------------------
// Weight image: Bm [C, R] (Bm = W, or W^T with transpose) ->
//   planes: Wf[((cb * (R/16) + kb) * 2 + p) * 64 + lane] (16 B each) = plane p
//     of Bm[cb*32 + (lane & 31)][kb*16 + 8*(lane >> 5) + 0..7] * 2^(kTW - e_c)
//   exps:   int32 e_c at byte offset C*R*4 (frexp exponent of max_r |Bm[c, r]|)
// One workgroup per (job, 32-column block).
struct SplitJobsH {
  const float* W[RB_MAX_SPLIT_JOBS];
  f16x8* Wf[RB_MAX_SPLIT_JOBS];
  int64_t ldw[RB_MAX_SPLIT_JOBS];
  int C[RB_MAX_SPLIT_JOBS], R[RB_MAX_SPLIT_JOBS], tr[RB_MAX_SPLIT_JOBS];
  int bstart[RB_MAX_SPLIT_JOBS + 1];
  int n;
};

__global__ void __launch_bounds__(256) k_split_weights_h(const SplitJobsH jobs) {
  __shared__ float smax[256];
  __shared__ int sexp[32];
  int j = 0;
  while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.bstart[j + 1]) ++j;
  const int C = jobs.C[j], R = jobs.R[j], tr = jobs.tr[j];
  const int64_t ldw = jobs.ldw[j];
  const float* __restrict__ W = jobs.W[j];
  const int cb = blockIdx.x - jobs.bstart[j];
  const int tid = threadIdx.x;
  auto bm = [&](int c, int r) -> float {
    return tr ? W[(int64_t)r * ldw + c] : W[(int64_t)c * ldw + r];
  };
  // column maxima: 8 threads per column, consecutive threads on consecutive
  // addresses (W^T: 32 columns are one 128-B row piece; W: each column is a
  // row of W, read as float4 runs), four independent loads in flight
  const bool vec = (reinterpret_cast<uintptr_t>(W) & 15) == 0 && (ldw & 3) == 0;
  if (tr || !vec) {
    const int c = cb * 32 + (tid & 31);
    float m0 = 0.0f, m1 = 0.0f;
    int r = tid >> 5;
    for (; r + 8 < R; r += 16) {
      m0 = fmaxf(m0, fabsf(bm(c, r)));
      m1 = fmaxf(m1, fabsf(bm(c, r + 8)));
    }
    if (r < R) m0 = fmaxf(m0, fabsf(bm(c, r)));
    smax[(tid & 31) * 8 + (tid >> 5)] = fmaxf(m0, m1);
  } else {
    const int cl = tid >> 3, c = cb * 32 + cl;
    const float* row = W + (int64_t)c * ldw;
    float m0 = 0.0f, m1 = 0.0f;
    for (int r = (tid & 7) * 4; r < R; r += 64) {   // R % 16 == 0: whole float4 runs
      const f32x4 a = *reinterpret_cast<const f32x4*>(row + r);
      m0 = fmaxf(m0, fmaxf(fabsf(a[0]), fabsf(a[1])));
      m1 = fmaxf(m1, fmaxf(fabsf(a[2]), fabsf(a[3])));
      if (r + 32 < R) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(row + r + 32);
        m0 = fmaxf(m0, fmaxf(fabsf(b[0]), fabsf(b[1])));
        m1 = fmaxf(m1, fmaxf(fabsf(b[2]), fabsf(b[3])));
      }
    }
    smax[cl * 8 + (tid & 7)] = fmaxf(m0, m1);
  }
  __syncthreads();
  if (tid < 32) {
    float m = smax[tid * 8];
#pragma unroll
    for (int q = 1; q < 8; ++q) m = fmaxf(m, smax[tid * 8 + q]);
    const int e = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
    sexp[tid] = e;
    int* ew = reinterpret_cast<int*>(reinterpret_cast<char*>(jobs.Wf[j]) + (int64_t)C * R * 4);
    ew[cb * 32 + tid] = e;
  }
  __syncthreads();
  const int KB = R / 16;
  for (int it = tid; it < KB * 64; it += 256) {
    const int kb = it >> 6, lane = it & 63;
    const int c = cb * 32 + (lane & 31);
    const int r0 = kb * 16 + 8 * (lane >> 5);
    const int sh = kTW - sexp[lane & 31];
    f16x8 o0, o1;
#pragma unroll
    for (int q = 0; q < 8; q += 2) {
      const f32x2 x = {__builtin_amdgcn_ldexpf(bm(c, r0 + q), sh),
                       __builtin_amdgcn_ldexpf(bm(c, r0 + q + 1), sh)};
      f16x2 h0, h1;
      split2h(x, h0, h1);
      o0[q] = h0[0]; o0[q + 1] = h0[1];
      o1[q] = h1[0]; o1[q + 1] = h1[1];
    }
    f16x8* dst = jobs.Wf[j] + ((int64_t)(cb * KB + kb) * 2) * 64 + lane;
    dst[0] = o0;
    dst[64] = o1;
  }
  // the weight-stationary kernel's image of the same 32 columns (gemm_ws.hip,
  // v_mfma_f32_16x16x32_f16 operand order, same column exponents) at
  // ws_image_offset(C, R): Wi[((c16 * KS + s) * 2 + p) * 64 + lane] = plane p
  // of Bm[16 c16 + (lane & 15)][32 s + 8 (lane >> 4) + 0..7]
  if (R % 32 == 0) {
    f16x8* wi = reinterpret_cast<f16x8*>(reinterpret_cast<char*>(jobs.Wf[j]) + ws_image_offset(C, R));
    const int KS = R / 32;
    for (int it = tid; it < 2 * KS * 64; it += 256) {
      const int h = it / (KS * 64), s = (it >> 6) % KS, lane = it & 63;
      const int cl = 16 * h + (lane & 15);
      const int c = cb * 32 + cl;
      const int r0 = 32 * s + 8 * (lane >> 4);
      const int sh = kTW - sexp[cl];
      f16x8 o0, o1;
#pragma unroll
      for (int q = 0; q < 8; q += 2) {
        const f32x2 x = {__builtin_amdgcn_ldexpf(bm(c, r0 + q), sh),
                         __builtin_amdgcn_ldexpf(bm(c, r0 + q + 1), sh)};
        f16x2 h0, h1;
        split2h(x, h0, h1);
        o0[q] = h0[0]; o0[q + 1] = h0[1];
        o1[q] = h1[0]; o1[q + 1] = h1[1];
      }
      f16x8* dst = wi + ((int64_t)((2 * cb + h) * KS + s) * 2) * 64 + lane;
      dst[0] = o0;
      dst[64] = o1;
    }
  }
}

// ---------------------------------------------------------------------------
constexpr int N_WAVES = 8;
constexpr int N_BM = 32 * N_WAVES, N_BN = 128, N_BK = 32;
constexpr int N_NSA = 3, N_NSB = 2;
constexpr int N_THREADS = 64 * N_WAVES;
constexpr int N_LA = N_NSA - 1;                       // A steps in flight
constexpr int N_NB = N_BN / 32;                       // column blocks per wave (4)
constexpr int N_BFRAG = N_NB * 2 * 2;                 // B fragments per step (16)
constexpr int N_BDMA = N_BFRAG / N_WAVES;             // B DMAs per wave per step (2)
constexpr int N_A_STAGE = N_BM * N_BK * 4;            // 32 KB
constexpr int N_B_STAGE = N_BFRAG * 1024;             // 16 KB
constexpr int N_RING = N_NSA * N_A_STAGE + N_NSB * N_B_STAGE;  // 128 KB
// + the column exponents and the bias of all C columns (C <= 1024)
constexpr int N_MAXC = 1024;
constexpr int N_MAXFLAG = 32;  // flagged tiles listed per wave (beyond: redo all)
constexpr int N_LDS = N_RING + N_MAXC * 8 + N_WAVES * N_MAXFLAG * 4;

// NB column blocks of 32 per wave: NB = 4 (256 x 128 tiles, the tile's
// results stored a block per k-step during the next tile) or NB = 8 (256 x
// 256 tiles for C % 256 == 0: a quarter fewer bytes through each CU's load
// path per output — every A row is re-read C/256 instead of C/128 times and
// each weight fragment DMA serves twice the outputs — with the results
// stored at the tile's end, 2 A stages)
template <int NB>
struct NtCfg {
  static constexpr int BN = 32 * NB;
  static constexpr int BFRAG = NB * 4;                  // B fragments per k-step
  static constexpr int BDMA = BFRAG / N_WAVES;          // B DMAs per wave per k-step
  static constexpr int B_STAGE = BFRAG * 1024;
  static constexpr int NSA = NB == 4 ? N_NSA : 2;
  static constexpr int RING = NSA * N_A_STAGE + N_NSB * B_STAGE;
  static constexpr int LDS = RING + N_MAXC * 8 + N_WAVES * N_MAXFLAG * 4;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <typename T>
__device__ __forceinline__ T hds_read16(uint32_t addr) {
  T r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
__device__ __forceinline__ int hds_read_i32(uint32_t addr) {
  int r;
  asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

template <int N>
__device__ __forceinline__ void hwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// quad_perm DPP moves (lane k of each quad reads lane k ^ 1 / k ^ 2)
__device__ __forceinline__ float dpp_xor1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_xor2(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
}

// 4 x 4 transpose inside each lane quad: on entry lane k of a quad holds
// column k (v[r] = row r), on exit row k (v[c] = column c).  Two butterfly
// stages (lane distance 2, then 1), each a select + DPP move + select.
__device__ __forceinline__ void quad_transpose(float (&v)[4], int lane) {
  const bool b1 = (lane & 2) != 0, b0 = (lane & 1) != 0;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const float y = dpp_xor2(b1 ? v[r] : v[r + 2]);
    if (b1) v[r] = y; else v[r + 2] = y;
  }
#pragma unroll
  for (int r = 0; r < 4; r += 2) {
    const float y = dpp_xor1(b0 ? v[r] : v[r + 1]);
    if (b0) v[r] = y; else v[r + 1] = y;
  }
}

// ACT (the FeedForward's first projection, RecBLR.py:219-221): a second
// output act = dropout(silu(out)) — out with the bias, i.e. the activation's
// input — written beside out by the same epilogue (same row stride ldo);
// the dropout keep-flags are DropSpec's Philox stream at element index
// e_base + row * C + col, exactly the flags k_silu_dropout_fwd draws for
// that element, so act equals the separate kernel's output bit for bit.
//
// DACT (the same activation's backward, fused into the input-gradient GEMM
// dU = dA2 W_2 of the FeedForward's second projection): the tile's dU values
// never reach HBM; the epilogue loads the activation's input `pre` at the
// same positions and stores dA1 = dU * keep * scale * silu'(pre) — what
// k_silu_dropout_bwd computes from dU, bit for bit — and sums dA1 over the
// tile's rows into per-wave LDS column sums (fixed order, deterministic),
// written at the end as the workgroup's row of dpart [gridDim.x, C] (the
// w_1 bias gradient's partials).  Rows of a tile flagged for the cold
// recompute tail are summed there instead, from their recomputed values.
constexpr int N_DACT_MAXC = 512;   // LDS column sums: 8 waves x C floats
// The NT GEMM over the tiles of one launch phase: workgroup `bid` of `G`
// takes tiles bid, bid + G, ...  (k_gemm_nt_h: one phase; k_gemm_nt_h2: the
// whole rounds of 256 x 128 / 256 x 256 tiles, then the rows past them as
// 256 x 64 tiles, in one launch).
template <bool BIAS, bool WIDE, int NB, bool ACT = false, bool DACT = false>
__device__ __forceinline__ void nt_h_body(char* smem, const int bid, const int G,
                                          const float* __restrict__ A, int64_t lda, int64_t M,
                                          int R, const f16x8* __restrict__ Wf,
                                          const int* __restrict__ ew, int C,
                                          const float* __restrict__ bias, float* __restrict__ out,
                                          int64_t ldo, float* __restrict__ rmax, int m_tiles,
                                          float* __restrict__ act, DropSpec drop, int64_t e_base,
                                          const float* __restrict__ pre,
                                          float* __restrict__ dpart) {
  using CF = NtCfg<NB>;
  constexpr int N_BN = CF::BN, N_NB = NB, N_BDMA = CF::BDMA, N_NSA = CF::NSA, N_LA = N_NSA - 1;
  constexpr int N_B_STAGE = CF::B_STAGE, N_RING = CF::RING;
  // deferred epilogue for NB = 4 (NB = 8 and DACT: stored at the tile's end)
  constexpr bool DEFER = NB == 4 && !DACT;   // DACT: stored at the tile's end
  static_assert(!(NB == 8) || WIDE, "256-column tiles store through the wide epilogue");
  static_assert(!ACT || WIDE, "the activation output rides the wide epilogue");
  static_assert(!DACT || (WIDE && !ACT && !BIAS), "DACT: wide epilogue, no bias");
  const int64_t act_delta = ACT ? (reinterpret_cast<char*>(act) - reinterpret_cast<char*>(out)) : 0;
  const int64_t pre_delta =
      DACT ? (reinterpret_cast<const char*>(pre) - reinterpret_cast<const char*>(out)) : 0;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nct = C / N_BN;
  const int KT = R / N_BK;
  const int KB16 = R / 16;
  const int n_tiles = ((m_tiles + 7) >> 3) * 8 * nct;
  const int my_tiles = bid < n_tiles ? (n_tiles - 1 - bid) / G + 1 : 0;
  const int U = my_tiles * KT;  // k-steps of this workgroup
  if (U == 0) {
    if (DACT)
      for (int c = tid; c < C; c += N_THREADS) dpart[(int64_t)bid * C + c] = 0.0f;
    return;
  }

  // column exponents and bias into LDS (before any DMA: ordinary loads)
  int* s_ew = reinterpret_cast<int*>(smem + N_RING);
  float* s_bias = reinterpret_cast<float*>(smem + N_RING + N_MAXC * 4);
  for (int c = tid; c < C; c += N_THREADS) {
    s_ew[c] = ew[c];
    if (BIAS) s_bias[c] = bias[c];
  }
  // DACT: per-wave column sums of dA1 (wave-private: no atomics)
  float* s_col = reinterpret_cast<float*>(smem + CF::LDS) + wave * N_DACT_MAXC;
  if (DACT)
    for (int c = lane; c < C; c += 64) s_col[c] = 0.0f;
  __syncthreads();

  // tile T = bid + i*G: the column tiles of one row tile are
  // neighbouring workgroups of one XCD (same blockIdx % 8), so their A
  // re-reads hit that XCD's L2.  (Divisions: once per tile and stream.)
  auto tile_of = [&](int i, int& mt, int& ct) {
    const int T = bid + i * G;
    const int g = T >> 3;
    ct = g % nct;
    mt = (g / nct) * 8 + (T & 7);
  };

  // ---- A stream (own rows; issued N_LA steps ahead).  Stage image:
  // row-major 128-B rows, 16-B chunk c of stage row r at chunk
  // c ^ ((r >> 1) & 7) (conflict-free fragment reads); wave w owns stage
  // rows 32w..32w+31 = 4 DMAs of 8 rows x 128 B.  Addresses: a uniform base
  // (the wave's first row, the k-step) + a 32-bit per-lane offset.
  int a_i = 0, a_kt = 0, a_slot = 0;
  const char* a_base = nullptr;
  int a_off[4];
  auto a_tile = [&]() {
    int mt, ct;
    tile_of(a_i, mt, ct);
    const int64_t r0 = (int64_t)mt * N_BM + wave * 32;
    a_base = reinterpret_cast<const char*>(A + r0 * lda);
    const int64_t lim = M - 1 - r0;  // rows past M repeat row M-1
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rr = q * 8 + (lane >> 3);
      const int64_t r = rr < lim ? rr : lim;
      const int srow = wave * 32 + rr;
      const int lc = (lane & 7) ^ ((srow >> 1) & 7);
      a_off[q] = (int)(r * lda * 4) + lc * 16;
    }
  };
  // (default cache policy: the nontemporal hint where each A row is read
  // once measured 1% slower)
  auto issueA = [&]() {
    char* st = smem + a_slot * N_A_STAGE + wave * 4096;
    const char* b = a_base + a_kt * (N_BK * 4);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((const void*)(b + a_off[q]), (lds_ptr_t)(st + q * 1024),
                                       16, 0, 0);
    a_slot = a_slot + 1 == N_NSA ? 0 : a_slot + 1;
    if (++a_kt == KT) {
      a_kt = 0;
      if (++a_i < my_tiles) a_tile();
    }
  };
  // ---- B stream (the k-step's 16 weight fragments, 1 KB each, shared by
  // the 8 waves; issued one step ahead): fragment f = (n * 2 + s) * 2 + p,
  // wave w DMAs fragments N_BDMA*w ...
  int b_i = 0, b_kt = 0, b_slot = 0;
  const f16x8* b_base = nullptr;
  auto b_tile = [&]() {
    int mt, ct;
    tile_of(b_i, mt, ct);
    b_base = Wf + (int64_t)ct * N_NB * KB16 * 2 * 64 + lane;
  };
  auto issueB = [&]() {
    char* st = smem + N_NSA * N_A_STAGE + b_slot * N_B_STAGE;
#pragma unroll
    for (int q = 0; q < N_BDMA; ++q) {
      const int f = wave * N_BDMA + q;
      const int n = f >> 2, s = (f >> 1) & 1, p = f & 1;
      const f16x8* src = b_base + ((n * KB16 + b_kt * 2 + s) * 2 + p) * 64;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + f * 1024), 16, 0, 0);
    }
    b_slot ^= 1;
    if (++b_kt == KT) {
      b_kt = 0;
      if (++b_i < my_tiles) b_tile();
    }
  };

  f32x16 acc[N_NB];
#pragma unroll
  for (int n = 0; n < N_NB; ++n)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[n][e] = 0.0f;

  a_tile();
  b_tile();
  issueB();
  for (int a = 0; a < N_LA && a < U; ++a) issueA();

  const uint32_t smem_base = (uint32_t)(uintptr_t)(lds_ptr_t)smem;
  const uint32_t s_ew_addr = smem_base + N_RING;
  const uint32_t s_bias_addr = smem_base + N_RING + N_MAXC * 4;
  // fragment read offsets inside an A stage: row 32*wave + (lane & 31),
  // logical chunks 4s + 2h and 4s + 2h + 1
  uint32_t a_rd[2][2];
  {
    const int row = wave * 32 + (lane & 31);
    const int sw = (row >> 1) & 7;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        a_rd[s][c] = row * 128 + (((4 * s + 2 * (lane >> 5) + c) ^ sw) << 4);
  }
  const int ccol = lane & 31;
  // C-layout row of accumulator register j: 8*(j>>2) + 4*(lane>>5) + (j&3)
  auto crow = [&](int j) { return 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3); };

  // per-row scale state of this lane's row (lanes l and l+32 hold the same row)
  int er = kSent;
  float scl = 1.0f, thr = 0.0f;
  float tmax = 0.0f;         // max |A| over the lane's values of the current tile (rmax)
  bool flag_tile = false;    // a row of this wave overflowed its headroom in this tile
  int nflag = 0;             // flagged tiles (their iteration index i, in LDS)
  int* s_flag = reinterpret_cast<int*>(smem + N_RING + N_MAXC * 8) + wave * N_MAXFLAG;

  // deferred epilogue: pend[n] (un-scaled) stored one block per k-step during
  // the next tile; 16 dword stores per block (lane: one column, 16 rows)
  f32x16 pend[DEFER ? N_NB : 1];
  float pbias[N_NB];
  int pend_q = N_NB;
  bool pend_on = false, pend_full = true;
  const char* pend_base = nullptr;  // the wave's first row of the pending tile
  int64_t pend_r0 = 0;
  int pend_c0 = 0;                  // its first column (ACT's dropout element index)
  // narrow stores: lane = one column, 16 dword stores per block (2 rows of
  // 128 B each); wide stores (WIDE: out 16-B aligned, ldo % 4 == 0): each
  // group of 4 registers transposed inside the lane quads, so a lane holds 4
  // columns of one row: 4 dwordx4 stores per block (8 rows of 128 B each)
  const int st_lane = WIDE ? (int)(((4 * (lane >> 5) + (lane & 3)) * ldo + (lane & 28)) * 4)
                           : (int)((4 * (lane >> 5)) * ldo * 4) + ccol * 4;
  auto store_block = [&](const f32x16& blk, int n) {
    if constexpr (WIDE) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = BIAS ? blk[4 * g + r] + pbias[n] : blk[4 * g + r];
        quad_transpose(v, lane);
        f32x4* o = (f32x4*)(pend_base + (int64_t)(8 * g) * ldo * 4 + n * 128 + st_lane);
        const int64_t row = pend_r0 + 8 * g + 4 * (lane >> 5) + (lane & 3);
        if (pend_full || row < M)
          __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, o);
        if constexpr (ACT) {
          float m[4];
          drop.get4(e_base + row * C + pend_c0 + n * 32 + (lane & 28), m);
          f32x4 a;
#pragma unroll
          for (int r = 0; r < 4; ++r) a[r] = fsilu(v[r]) * m[r];
          if (pend_full || row < M)
            __builtin_nontemporal_store(a, (f32x4*)(reinterpret_cast<char*>(o) + act_delta));
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int rj = 8 * (j >> 2) + (j & 3);
        float* o = (float*)(pend_base + (int64_t)rj * ldo * 4 + n * 128 + st_lane);
        const float v = BIAS ? blk[j] + pbias[n] : blk[j];
        if (pend_full || pend_r0 + crow(j) < M) __builtin_nontemporal_store(v, o);
      }
    }
  };
  // DACT: the activation's backward on one un-scaled dU block of the pending
  // tile (pend_*): dA1 = dU * keep * scale * silu'(pre) stored, and summed
  // over the block's rows into the wave's LDS column sums unless the cold
  // tail will redo the tile (skip_sums).  ld_pre loads a block's `pre`
  // values (ordinary loads: the compiler places their waits); rows past M
  // load row M - 1 and store nothing.
  const int rq = 4 * (lane >> 5) + (lane & 3);   // a lane's row in an 8-row group (wide layout)
  auto ld_pre = [&](int n, f32x4 (&q)[4]) {
    if constexpr (DACT) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t row = pend_r0 + 8 * g + rq;
        int64_t off = (int64_t)(8 * g) * ldo * 4 + n * 128 + st_lane + pre_delta;
        if (!pend_full && row >= M) off -= (row - (M - 1)) * ldo * 4;
        q[g] = *reinterpret_cast<const f32x4*>(pend_base + off);
      }
    }
  };
  auto dact_block = [&](const f32x16& blk, int n, const f32x4 (&pq)[4], bool skip_sums) {
    if constexpr (DACT) {
      float cs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = blk[4 * g + r];
        quad_transpose(v, lane);
        const int64_t row = pend_r0 + 8 * g + rq;
        const bool ok = pend_full || row < M;
        float mk[4];
        drop.get4(e_base + row * C + pend_c0 + n * 32 + (lane & 28), mk);
        const f32x4 pv = pq[g];
        f32x4 d;
#pragma unroll
        for (int r = 0; r < 4; ++r) d[r] = (v[r] * mk[r]) * fdsilu(pv[r] + 0.0f);
        if (ok) {
          __builtin_nontemporal_store(
              d, (f32x4*)(pend_base + (int64_t)(8 * g) * ldo * 4 + n * 128 + st_lane));
#pragma unroll
          for (int r = 0; r < 4; ++r) cs[r] += d[r];
        }
      }
      if (!skip_sums) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          cs[r] += dpp_xor1(cs[r]);
          cs[r] += dpp_xor2(cs[r]);
          cs[r] += __shfl_xor(cs[r], 32);
        }
        if ((lane & 3) == 0 && lane < 32) {
#pragma unroll
          for (int r = 0; r < 4; ++r) s_col[pend_c0 + n * 32 + (lane & 28) + r] += cs[r];
        }
      }
    }
  };
  // DEFER + DACT: the pending block's `pre` values, loaded one k-step ahead
  f32x4 pq1[4];
  bool pend_skip = false;
  auto store_quarter = [&]() {
    const int q = pend_q++;
    if constexpr (DEFER && DACT) {
      if (q == 0) dact_block(pend[0], 0, pq1, pend_skip);
      else if (q == 1) dact_block(pend[1], 1, pq1, pend_skip);
      else if (q == 2) dact_block(pend[2], 2, pq1, pend_skip);
      else dact_block(pend[3], 3, pq1, pend_skip);
      if (q + 1 < N_NB) ld_pre(q + 1, pq1);
    } else if constexpr (DEFER) {
      if (q == 0) store_block(pend[0], 0);
      else if (q == 1) store_block(pend[1], 1);
      else if (q == 2) store_block(pend[2], 2);
      else store_block(pend[3], 3);
    }
    return pend_full;
  };
  // DACT tile end (no DEFER): acc[n] holds the tile's un-scaled dU blocks;
  // the next block's `pre` values load behind the current block's math
  auto dact_epilogue = [&](bool skip_sums) {
    if constexpr (DACT && !DEFER) {
      f32x4 pq[2][4];
      ld_pre(0, pq[0]);
#pragma unroll
      for (int n = 0; n < N_NB; ++n) {
        if (n + 1 < N_NB) ld_pre(n + 1, pq[(n + 1) & 1]);
        dact_block(acc[n], n, pq[n & 1], skip_sums);
      }
    }
  };
  bool stored_prev = false;

  int i = 0, kt = 0, c_slot_a = 0, c_slot_b = 0;
  int cur_mt, cur_ct;
  tile_of(0, cur_mt, cur_ct);
  for (int u = 0; u < U; ++u) {
    // operands of step u landed (own DMAs): the ops younger than B(u) are
    // A(u-1+N_LA) (4, issued by step u-1 if it exists) and the 16 deferred
    // stores step u-1 issued after it (at u = 0 the prologue's extra A
    // batches make this wait conservative, never short)
    {
      const bool ya = u > 0 && u - 1 + N_LA < U;
      // stores after the DMAs: one block per step (DEFER), or the whole
      // tile at its end (NB = 8; ACT: twice as many).  vmcnt counts to 63: a
      // larger allowance is clamped, which only waits for more
      // (DEFER + DACT: each step's 4 stores are followed by the next block's
      // 4 `pre` loads)
      constexpr int NST_ = DEFER ? (WIDE ? (DACT || ACT ? 8 : 4) : 16) : (ACT ? 8 : 4) * NB;
      constexpr int NST = NST_ > 59 ? 59 : NST_;
      if constexpr (N_LA == 1) {
        // A(u) itself was issued in step u-1 (after B(u)): only the stores
        // issued after it may stay in flight
        if (stored_prev) hwait_vm<NST>(); else hwait_vm<0>();
      } else if (ya) {
        if (stored_prev) hwait_vm<4 + NST>(); else hwait_vm<4>();
      } else if (u == 0 && U > 1) {
        hwait_vm<4 * (N_LA - 1)>();
      } else {
        if (stored_prev) hwait_vm<NST>(); else hwait_vm<0>();
      }
    }
    __builtin_amdgcn_s_barrier();
    // the next steps' DMAs right after the barrier: their slots were last
    // read in step u-1, which every wave has finished (2-4% faster than after
    // substep 0; staggering the issue of the two waves of a SIMD: null).  B
    // before A, the stores after: the counted waits above rely on that order
    if (u + 1 < U) issueB();
    if (u + N_LA < U) issueA();

    const uint32_t sa = smem_base + c_slot_a * N_A_STAGE;
    const uint32_t sb = smem_base + N_NSA * N_A_STAGE + c_slot_b * N_B_STAGE + lane * 16;
    auto substep = [&](int s) {
      const f32x4 x0 = hds_read16<f32x4>(sa + a_rd[s][0]);
      const f32x4 x1 = hds_read16<f32x4>(sa + a_rd[s][1]);
      // B fragments two column blocks ahead of the MFMAs that use them
      auto rb = [&](int n, int p) { return hds_read16<f16x8>(sb + ((n * 2 + s) * 2 + p) * 1024); };
      f16x8 bq[N_NB][2];
      bq[0][0] = rb(0, 0); bq[0][1] = rb(0, 1); bq[1][0] = rb(1, 0); bq[1][1] = rb(1, 1);
      f32x4 xa = x0, xb = x1;
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(xa), "+v"(xb));
      const float mx = max8abs(xa, xb);
      tmax = fmaxf(tmax, mx);
      if (kt == 0 && s == 0) {
        // tile start: the row scale from the first 16 k-values of the row
        const float mm = fmaxf(mx, __shfl_xor(mx, 32));
        const bool z = !(mm > 0.0f);
        const int e = __builtin_amdgcn_frexp_expf(mm);
        er = z ? kSent : e;
        scl = z ? 1.0f : __builtin_amdgcn_ldexpf(1.0f, kTA - e);
        thr = z ? 0.0f : __builtin_amdgcn_ldexpf(1.0f, e + kHead);
      } else {
        // rare: a value beyond its row's headroom (its fp16 image may
        // overflow): the wave's rows of this tile are recomputed exactly
        // after the main loop
        flag_tile = flag_tile || __builtin_amdgcn_ballot_w64(mx > thr) != 0;
      }
      f16x8 a0, a1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x2 v = (q < 2 ? f32x2{xa[2 * q], xa[2 * q + 1]}
                               : f32x2{xb[2 * q - 4], xb[2 * q - 3]}) * scl;
        f16x2 h0, h1;
        split2h(v, h0, h1);
        a0[2 * q] = h0[0]; a0[2 * q + 1] = h0[1];
        a1[2 * q] = h1[0]; a1[2 * q + 1] = h1[1];
      }
      // per column block: the small partial products first; block n + 2's
      // fragments are read behind block n's MFMAs
#pragma unroll
      for (int n = 0; n < N_NB; ++n) {
        if (n + 1 < N_NB)
          asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(bq[n][0]), "+v"(bq[n][1]));
        else
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(bq[n][0]), "+v"(bq[n][1]));
        acc[n] = mfma_h(a1, bq[n][0], acc[n]);
        acc[n] = mfma_h(a0, bq[n][1], acc[n]);
        acc[n] = mfma_h(a0, bq[n][0], acc[n]);
        if (n + 2 < N_NB) {
          bq[n + 2][0] = rb(n + 2, 0);
          bq[n + 2][1] = rb(n + 2, 1);
        }
      }
    };
    substep(0);
    stored_prev = false;
    if (DEFER && pend_on && pend_q < N_NB) {
      // a partial tile's guarded stores may issue fewer than 16: not counted
      stored_prev = store_quarter();
    }
    substep(1);
    c_slot_a = c_slot_a + 1 == N_NSA ? 0 : c_slot_a + 1;
    c_slot_b ^= 1;

    if (kt == KT - 1) {
      // DEFER: the tile's results (un-scaled) move to pend[] and are stored a
      // block per step during the next tile's first steps (behind its MFMAs);
      // NB = 8: un-scaled and stored now
      if constexpr (DEFER) {
        while (pend_on && pend_q < N_NB) store_quarter();
      }
      int ecol[N_NB];
#pragma unroll
      for (int n = 0; n < N_NB; ++n) ecol[n] = hds_read_i32(s_ew_addr + (cur_ct * N_BN + n * 32 + ccol) * 4);
      if (BIAS) {
#pragma unroll
        for (int n = 0; n < N_NB; ++n)
          pbias[n] = __builtin_bit_cast(float, hds_read_i32(s_bias_addr + (cur_ct * N_BN + n * 32 + ccol) * 4));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int n = 0; n < N_NB; ++n) {
        asm volatile("" : "+v"(ecol[n]));
        if (BIAS) asm volatile("" : "+v"(pbias[n]));
      }
      if constexpr (DEFER) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int erj = __shfl(er, crow(j)) - kTA - kTW;
#pragma unroll
          for (int n = 0; n < N_NB; ++n) {
            pend[n][j] = __builtin_amdgcn_ldexpf(acc[n][j], erj + ecol[n]);
            acc[n][j] = 0.0f;
          }
        }
      } else {
        const int64_t r0 = (int64_t)cur_mt * N_BM + wave * 32;
        const bool full = r0 + 32 <= M;
        if (cur_mt < m_tiles) {
          pend_base = reinterpret_cast<const char*>(out + r0 * ldo + cur_ct * N_BN);
          pend_r0 = r0;
          pend_c0 = cur_ct * N_BN;
          pend_full = full;
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int erj = __shfl(er, crow(j)) - kTA - kTW;
#pragma unroll
            for (int n = 0; n < N_NB; ++n) acc[n][j] = __builtin_amdgcn_ldexpf(acc[n][j], erj + ecol[n]);
          }
          if constexpr (DACT) {
            dact_epilogue(flag_tile);
          } else {
#pragma unroll
            for (int n = 0; n < N_NB; ++n) store_block(acc[n], n);
          }
          stored_prev = full;
        }
#pragma unroll
        for (int n = 0; n < N_NB; ++n)
#pragma unroll
          for (int j = 0; j < 16; ++j) acc[n][j] = 0.0f;
      }
      if (rmax && cur_ct == 0 && cur_mt < m_tiles) {
        // max |A| of the wave's 32 rows (all R columns): the weight-gradient
        // kernel's operand scale (rows past M repeat row M-1: harmless)
        float w = tmax;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) w = fmaxf(w, __shfl_xor(w, o));
        const int64_t grp = (int64_t)cur_mt * (N_BM / 32) + wave;
        if (lane == 0 && grp * 32 < M) rmax[grp] = w;
      }
      tmax = 0.0f;
      const bool tile_flagged = flag_tile;
      if (flag_tile) {
        if (nflag < N_MAXFLAG) s_flag[nflag] = i;
        ++nflag;
        flag_tile = false;
      }
      if constexpr (DEFER) {
        pend_on = cur_mt < m_tiles;
        pend_r0 = (int64_t)cur_mt * N_BM + wave * 32;
        pend_c0 = cur_ct * N_BN;
        pend_full = pend_r0 + 32 <= M;
        pend_base = reinterpret_cast<const char*>(out + pend_r0 * ldo + cur_ct * N_BN);
        pend_q = 0;
        if (DACT && pend_on) {   // the first block's `pre`, stored during the next step
          pend_skip = tile_flagged;
          ld_pre(0, pq1);
        }
      }
      kt = 0;
      ++i;
      if (i < my_tiles) tile_of(i, cur_mt, cur_ct);
    } else {
      ++kt;
    }
  }
  while (pend_on && pend_q < N_NB) store_quarter();

  // cold tail: the wave's rows of every flagged tile again, with each row's
  // exact max known first (no overflow possible), operands straight from
  // global memory, stored directly (after this wave's earlier stores)
  if (nflag > 0) {
    hwait_vm<0>();
    const int ntodo = nflag > N_MAXFLAG ? my_tiles : nflag;
    // DACT, every tile redone: the wave's column sums start over
    if (DACT && nflag > N_MAXFLAG)
      for (int c = lane; c < C; c += 64) s_col[c] = 0.0f;
    for (int f = 0; f < ntodo; ++f) {
      const int ii = nflag > N_MAXFLAG ? f : s_flag[f];
      int mt, ct;
      tile_of(ii, mt, ct);
      if (mt >= m_tiles) continue;
      int64_t row = (int64_t)mt * N_BM + wave * 32 + (lane & 31);
      if (row >= M) row = M - 1;
      const float* arow = A + row * lda + 8 * (lane >> 5);
      float m = 0.0f;
      for (int kb = 0; kb < KB16; ++kb) {
        const f32x4 p = *reinterpret_cast<const f32x4*>(arow + kb * 16);
        const f32x4 q = *reinterpret_cast<const f32x4*>(arow + kb * 16 + 4);
        m = fmaxf(m, max8abs(p, q));
      }
      m = fmaxf(m, __shfl_xor(m, 32));
      const int e = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
      const float sc = __builtin_amdgcn_ldexpf(1.0f, kTW - e);  // row max < 2^14
      int erow[16];  // the exact exponent of each C-layout row
#pragma unroll
      for (int j = 0; j < 16; ++j) erow[j] = __shfl(e, crow(j)) - 2 * kTW;
      // one column block at a time (the A row is re-read per block from L2:
      // a cold path, kept to one accumulator block of registers)
      for (int n = 0; n < N_NB; ++n) {
        f32x16 c;
#pragma unroll
        for (int j = 0; j < 16; ++j) c[j] = 0.0f;
        for (int kb = 0; kb < KB16; ++kb) {
          const f32x4 p = *reinterpret_cast<const f32x4*>(arow + kb * 16);
          const f32x4 q = *reinterpret_cast<const f32x4*>(arow + kb * 16 + 4);
          f16x8 a0, a1;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const f32x2 v = (t < 2 ? f32x2{p[2 * t], p[2 * t + 1]} : f32x2{q[2 * t - 4], q[2 * t - 3]}) * sc;
            f16x2 h0, h1;
            split2h(v, h0, h1);
            a0[2 * t] = h0[0]; a0[2 * t + 1] = h0[1];
            a1[2 * t] = h1[0]; a1[2 * t + 1] = h1[1];
          }
          const f16x8* bp = Wf + ((int64_t)((ct * N_NB + n) * KB16 + kb) * 2) * 64 + lane;
          const f16x8 b0 = bp[0], b1 = bp[64];
          c = mfma_h(a1, b0, c);
          c = mfma_h(a0, b1, c);
          c = mfma_h(a0, b0, c);
        }
        const int col = ct * N_BN + n * 32 + ccol;
        const int ecol = s_ew[col];
        const float bv = BIAS ? s_bias[col] : 0.0f;
        float csum = 0.0f;   // DACT: this lane's rows of the column
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int64_t r = (int64_t)mt * N_BM + wave * 32 + crow(j);
          if (r < M) {
            float v = __builtin_amdgcn_ldexpf(c[j], erow[j] + ecol) + bv;
            if constexpr (DACT) {
              float mk[4];
              const int64_t ei = e_base + r * C + col;
              drop.get4(ei & ~(int64_t)3, mk);
              const int q = (int)(ei & 3);
              v = (v * (q == 0 ? mk[0] : q == 1 ? mk[1] : q == 2 ? mk[2] : mk[3])) *
                  fdsilu(pre[r * ldo + col] + 0.0f);
              csum += v;
            }
            out[r * ldo + col] = v;
            if constexpr (ACT) {
              float mk[4];
              const int64_t ei = e_base + r * C + col;
              drop.get4(ei & ~(int64_t)3, mk);
              const int q = (int)(ei & 3);   // (no dynamic register indexing)
              act[r * ldo + col] = fsilu(v) * (q == 0 ? mk[0] : q == 1 ? mk[1] : q == 2 ? mk[2] : mk[3]);
            }
          }
        }
        if constexpr (DACT) {
          csum += __shfl_xor(csum, 32);
          if (lane < 32) s_col[col] += csum;
        }
      }
    }
  }
  if constexpr (DACT) {
    // the workgroup's column sums, waves in a fixed order
    __syncthreads();
    const float* s_all = reinterpret_cast<const float*>(smem + CF::LDS);
    for (int c = tid; c < C; c += N_THREADS) {
      float t = s_all[c];
#pragma unroll
      for (int w = 1; w < N_WAVES; ++w) t += s_all[w * N_DACT_MAXC + c];
      dpart[(int64_t)bid * C + c] = t;
    }
  }
}

template <bool BIAS, bool WIDE, int NB, bool ACT = false, bool DACT = false>
__global__ void __launch_bounds__(N_THREADS, 1) k_gemm_nt_h(const float* __restrict__ A, int64_t lda,
                                                          int64_t M, int R,
                                                          const f16x8* __restrict__ Wf,
                                                          const int* __restrict__ ew, int C,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ out, int64_t ldo,
                                                          float* __restrict__ rmax, int m_tiles,
                                                          float* __restrict__ act, DropSpec drop,
                                                          int64_t e_base,
                                                          const float* __restrict__ pre,
                                                          float* __restrict__ dpart) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  nt_h_body<BIAS, WIDE, NB, ACT, DACT>(smem, (int)blockIdx.x, (int)gridDim.x, A, lda, M, R, Wf, ew,
                                       C, bias, out, ldo, rmax, m_tiles, act, drop, e_base, pre,
                                       dpart);
}

// One phase's operands (the rows [r0, r0 + M) of a call).
struct NtPhase {
  const float* A;
  int64_t M;
  float* out;
  float* rmax;
  float* act;
  const float* pre;
  float* dpart;
  int64_t e_base;
  int m_tiles;
  int grid;
};

// Both phases of a call in one launch: the whole rounds on NB-column tiles,
// then the rows past them on 256 x 64 tiles (2-4x as many tiles, so the
// partial round fills the chip).  A workgroup starts its tail tiles as soon
// as its own main tiles are done; the LDS is reused after a barrier (every
// DMA of the main phase has landed: each step waits for its own operands).
template <bool BIAS, int NB, bool ACT = false, bool DACT = false>
__global__ void __launch_bounds__(N_THREADS, 1)
k_gemm_nt_h2(int64_t lda, int R, const f16x8* __restrict__ Wf, const int* __restrict__ ew, int C,
             const float* __restrict__ bias, int64_t ldo, DropSpec drop, NtPhase main_ph,
             NtPhase tail_ph) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bid = (int)blockIdx.x;
  if (bid < main_ph.grid)
    nt_h_body<BIAS, true, NB, ACT, DACT>(smem, bid, main_ph.grid, main_ph.A, lda, main_ph.M, R, Wf,
                                         ew, C, bias, main_ph.out, ldo, main_ph.rmax,
                                         main_ph.m_tiles, main_ph.act, drop, main_ph.e_base,
                                         main_ph.pre, main_ph.dpart);
  __syncthreads();
  if (bid < tail_ph.grid)
    nt_h_body<BIAS, true, 2, ACT, DACT>(smem, bid, tail_ph.grid, tail_ph.A, lda, tail_ph.M, R, Wf,
                                        ew, C, bias, tail_ph.out, ldo, tail_ph.rmax,
                                        tail_ph.m_tiles, tail_ph.act, drop, tail_ph.e_base,
                                        tail_ph.pre, tail_ph.dpart);
}

// ---------------------------------------------------------------------------
// k_gemm_tn_h (weight gradient, split over rows):
//   part[s][n, k] = sum over rows m of chunk s of dY[m, n] X[m, k]
// (RecBLR.py:162,165,167,213,214: F.linear's dW = dY^T X).  The reduction
// axis m is each operand's row axis, so the MFMA fragments (8 consecutive m
// of one column per lane) are gathered by a transpose in LDS: every m-step of
// 32 rows, each thread loads 8 rows x 4 columns of raw fp32 (16-B loads, two
// steps ahead, in registers), scales, splits into the two fp16 planes and
// writes each column's 8 values as one 16-B chunk of a column-major image
// (80-B column pitch, chunk XOR (col >> 4) & 3: conflict-free writes and
// fragment reads).  Scales: one power of two per operand and row chunk, from
// the max over the chunk's 32-row groups that the forward / input-gradient
// GEMMs wrote (rmax): values within 2^17 of the chunk max keep 22 bits.
// Workgroup: 256 threads (2 x 2 waves of 64 x 64), a 128 x 128 tile of dW;
// the tiles of one row chunk run on one XCD (their row re-reads hit its L2).
constexpr int T_BT = 128;
constexpr int T_PITCH = 80;                   // bytes per column of an image plane
constexpr int kTT = 14;                       // chunk max lands in [2^13, 2^14)

// Tile of dW: (128 NBN) x (128 NBK), NBN * NBK <= 2, 4 NBN NBK waves of
// 64 x 64.  A 256-wide side (N % 256 == 0, else K % 256 == 0) halves the
// re-reads of the other operand's rows: each row of dY is read K / (128 NBK)
// times and each row of X N / (128 NBN) times, and these kernels are bound by
// those row streams through each CU's load path (a quarter fewer bytes for
// every projection shape).
template <int NBN, int NBK>
struct TnCfg {
  static constexpr int THREADS = 256 * NBN * NBK;
  static constexpr int YC = T_BT * NBN, XC = T_BT * NBK;       // dY / X columns of the tile
  static constexpr int YPLANE = YC * T_PITCH, XPLANE = XC * T_PITCH;
  static constexpr int STAGE = 2 * YPLANE + 2 * XPLANE;        // dY planes 0, 1, X planes 0, 1
  static constexpr int LDS = 2 * STAGE;                        // double buffered
  static constexpr int LOADERS = (YC + XC) / 4 * 4;            // 4 columns x 8 rows per thread
};

__device__ __forceinline__ uint32_t tn_off(int col, int chunk) {
  return col * T_PITCH + ((chunk ^ ((col >> 4) & 3)) << 4);
}

__device__ __forceinline__ void hds_write16(uint32_t addr, f16x8 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

template <int NBN, int NBK>
__device__ __attribute__((noinline)) void tn_percol(char* smem, const float* __restrict__ Y, int64_t ldy, const float* __restrict__ X,
                                        int64_t ldx, int64_t M, int N, int K,
                                        const float* __restrict__ ymax,
                                        const float* __restrict__ xmax, float* __restrict__ parts,
                                        int S, int64_t mk, int nt_k);

// The body of k_gemm_tn_h.  PERCOL = false: the chunk scales, then (a column
// spread past 2^16) tn_percol; PERCOL = true: the tile's chunk again with the
// column scales the first pass left in stage 0's padding bytes.
template <int NBN, int NBK, bool PERCOL>
__device__ __forceinline__ void tn_body(char* smem, const float* __restrict__ Y, int64_t ldy, const float* __restrict__ X,
                                        int64_t ldx, int64_t M, int N, int K,
                                        const float* __restrict__ ymax,
                                        const float* __restrict__ xmax, float* __restrict__ parts,
                                        int S, int64_t mk, int nt_k) {
  using CF = TnCfg<NBN, NBK>;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / (2 * NBK), wk = wave % (2 * NBK);
  // block -> (tile, split): the tiles of one split share an XCD
  const int G = gridDim.x;
  const int idx = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int nt = (N / CF::YC) * nt_k;
  const int tile = idx % nt, s = idx / nt;
  if (s >= S) return;   // the grid's padding to a multiple of 8 (workgroup-uniform)
  const int n0 = (tile / nt_k) * CF::YC, k0 = (tile % nt_k) * CF::XC;
  const int64_t r_begin = (int64_t)s * mk;
  const int64_t r_end = r_begin + mk < M ? r_begin + mk : M;
  const int64_t nrows = r_end > r_begin ? r_end - r_begin : 0;
  const int T = (int)((nrows + 31) / 32);

  // chunk scales from the 32-row group maxima
  float my = 0.0f, mx = 0.0f;
  for (int64_t g = r_begin / 32 + tid; g * 32 < r_end; g += CF::THREADS) {
    my = fmaxf(my, ymax[g]);
    mx = fmaxf(mx, xmax[g]);
  }
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    my = fmaxf(my, __shfl_xor(my, o));
    mx = fmaxf(mx, __shfl_xor(mx, o));
  }
  constexpr int NW = CF::THREADS / 64;
  if (lane == 0) { red[wave] = my; red[NW + wave] = mx; }
  __syncthreads();
  my = 0.0f;
  mx = 0.0f;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    my = fmaxf(my, red[w]);
    mx = fmaxf(mx, red[NW + w]);
  }
  const int ey = my > 0.0f ? __builtin_amdgcn_frexp_expf(my) : 0;
  const int ex = mx > 0.0f ? __builtin_amdgcn_frexp_expf(mx) : 0;
  __syncthreads();

  // conversion role: threads [0, YC) load dY, [YC, YC + XC) load X (YC / 4
  // column groups x 4 row groups, resp. XC / 4 x 4); columns 4cc..4cc+3,
  // rows 8rg..8rg+7 of each m-step; the remaining threads only multiply
  const bool loader = tid < CF::LOADERS;
  const int op = tid < CF::YC ? 0 : 1;
  const int lt = op == 0 ? tid : tid - CF::YC;
  const int ncg = (op == 0 ? CF::YC : CF::XC) / 4;   // column groups of the operand
  const int cc = loader ? lt % ncg : 0;
  const int rg = loader ? lt / ncg : 0;
  const int64_t ld = op == 0 ? ldy : ldx;
  // the operand scale of each of the thread's 4 columns: the chunk's (the
  // first pass) or the column's own (the redo pass, below)
  float scv[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    int e = op == 0 ? ey : ex;
    if constexpr (PERCOL) {
      const int col = 4 * cc + c;
      e = *reinterpret_cast<const int*>(smem + (op == 0 ? col * T_PITCH
                                                        : 2 * CF::YPLANE + col * T_PITCH) + 64);
    }
    scv[c] = __builtin_amdgcn_ldexpf(1.0f, kTT - e);
  }
  float cm[4] = {0.0f, 0.0f, 0.0f, 0.0f};   // max |value| of the thread's columns
  const uint32_t smem_base = (uint32_t)(uintptr_t)(lds_ptr_t)smem;

  f32x4 raw0[8], raw1[8];
  // The operand rows of the chunk through a buffer descriptor (wave-uniform
  // base: the chunk's first row of this wave's operand; records: the chunk's
  // bytes): 32-bit lane offsets, and rows past the chunk read as zeros by the
  // descriptor's range check — which covers the lane offset only, so the row
  // is in the lane offset, never in the scalar one.  Plain (default-policy)
  // loads: the other tiles of this split re-read these rows from L2.
  const float* cbase = (op == 0 ? Y + n0 : X + k0) + r_begin * ld;
  const uint64_t cb = reinterpret_cast<uint64_t>(cbase);
  // (readfirstlane returns int: through uint32_t, or the low word's sign
  // would extend into the high one)
  const uint64_t cbu =
      (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)cb) |
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(cb >> 32)) << 32);
  const uint32_t ld4 = __builtin_amdgcn_readfirstlane((uint32_t)(ld * 4));
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(cbu), 0, (int)(nrows * ld4), 0x00020000);
  const uint32_t voff = (uint32_t)(rg * 8) * ld4 + (uint32_t)(16 * cc);
  // (scheduling barriers on both sides keep each batch in program order
  // between the conversions: loads the scheduler moved into a conversion made
  // the compiler's counted waits drain the other register set)
  auto load = [&](int t, f32x4 (&r)[8]) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      r[q] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + (uint32_t)(t * 32 + q) * ld4, 0, 0));
    __builtin_amdgcn_sched_barrier(0);
  };
  // columns 2p, 2p + 1 of the thread's 8 x 4 block of step t into image
  // `buf` (rows past the chunk are zeros from the loads: no branch, so the
  // conversion sits in one basic block with the MFMAs it overlaps).  The
  // packed scale / residual operate on the two columns of one row — a register
  // pair as the 16-B load left it; pairing two rows of one column instead made
  // hipcc regroup every loaded register at the loop's back edge, which waits
  // for the loads just issued — and the fp16 results are regrouped into each
  // column's 8 rows by the packs that build the LDS chunk.
  auto convert_pair = [&](const f32x4 (&r)[8], int buf, int p) {
    const uint32_t img = smem_base + buf * CF::STAGE + (op == 0 ? 0 : 2 * CF::YPLANE);
    const uint32_t plane = op == 0 ? CF::YPLANE : CF::XPLANE;
    const f32x2 sc{scv[2 * p], scv[2 * p + 1]};
    f16x8 h0[2], h1[2];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const f32x2 v{r[q][2 * p], r[q][2 * p + 1]};
      f16x2 p0, p1;
      split2h(v * sc, p0, p1);
      h0[0][q] = p0[0]; h0[1][q] = p0[1];
      h1[0][q] = p1[0]; h1[1][q] = p1[1];
    }
    if constexpr (!PERCOL) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int q = 0; q < 8; q += 4) {
          cm[2 * p + c] = max3abs(cm[2 * p + c], r[q][2 * p + c], r[q + 1][2 * p + c]);
          cm[2 * p + c] = max3abs(cm[2 * p + c], r[q + 2][2 * p + c], r[q + 3][2 * p + c]);
        }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint32_t off = tn_off(4 * cc + 2 * p + c, rg);
      hds_write16(img + off, h0[c]);
      hds_write16(img + plane + off, h1[c]);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;

  const int h = lane >> 5;
  // The products of image `buf` (one m-step of 32 rows: two substeps of 16);
  // with CONV, step t's columns converted into image nbuf in front of each
  // substep's fragment reads — substep 1's splits and LDS writes issue while
  // substep 0's MFMAs execute (each substep: two columns, fragment reads,
  // their wait, 12 MFMAs).
  // LATE (loader waves 4-7 of a 512-thread workgroup): each substep's MFMAs
  // first, then its columns' conversion, so the two waves of a SIMD alternate
  // between the split and the matrix pipe instead of converting in lock step
  auto mma = [&](int buf, auto conv_c, const f32x4 (&r)[8], int t, int nbuf, auto late_c) {
    (void)t;
    constexpr bool CONV = decltype(conv_c)::value;
    constexpr bool LATE = decltype(late_c)::value;
    const uint32_t iy = smem_base + buf * CF::STAGE;
    const uint32_t ix = iy + 2 * CF::YPLANE;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      if constexpr (CONV && !LATE) convert_pair(r, nbuf, st);
      // B fragments of both column blocks, then the A fragments one row
      // block at a time (24 fragment registers live, not 32)
      f16x8 b[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t ob = tn_off(64 * wk + 32 * j + (lane & 31), 2 * st + h);
        b[j][0] = hds_read16<f16x8>(ix + ob);
        b[j][1] = hds_read16<f16x8>(ix + CF::XPLANE + ob);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t oa = tn_off(64 * wm + 32 * i + (lane & 31), 2 * st + h);
        f16x8 a0 = hds_read16<f16x8>(iy + oa);
        f16x8 a1 = hds_read16<f16x8>(iy + CF::YPLANE + oa);
        if (i == 0)
          asm volatile("s_waitcnt lgkmcnt(0)"
                       : "+v"(a0), "+v"(a1), "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[1][0]),
                         "+v"(b[1][1]));
        else
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a0), "+v"(a1));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = mfma_h(a1, b[j][0], acc[i][j]);
          acc[i][j] = mfma_h(a0, b[j][1], acc[i][j]);
          acc[i][j] = mfma_h(a0, b[j][0], acc[i][j]);
        }
      }
      if constexpr (CONV && LATE) convert_pair(r, nbuf, st);
    }
  };
  using conv_t = std::true_type;
  using noconv_t = std::false_type;

  // Pipeline: raw0 / raw1 hold the register copies of steps loaded two steps
  // ahead; image t & 1 holds step t.  Step t's products run with step t+1's
  // conversion into the other image (last read by step t-1's products, which
  // every wave finished before the previous barrier); one barrier per step.
  // The loop is branch-free (T rounded up to even; steps past the chunk load
  // and multiply zeros) and loader and non-loader waves run their own copy:
  // with no VMEM under a branch the compiler's vmcnt waits for step t+1's
  // registers count step t+2's loads as still in flight instead of draining
  // them (a load under a branch made it wait for all of them, which left one
  // step of lead instead of two).
  const int Tp = (T + 1) & ~1;
  auto loader_loop = [&](auto late_c) {
    load(0, raw0);
    load(1, raw1);
    convert_pair(raw0, 0, 0);
    convert_pair(raw0, 0, 1);
    load(2, raw0);
    __syncthreads();
    for (int t = 0; t < Tp; t += 2) {
      mma(0, conv_t{}, raw1, t + 1, 1, late_c);
      load(t + 3, raw1);
      __syncthreads();
      mma(1, conv_t{}, raw0, t + 2, 0, late_c);
      load(t + 4, raw0);
      __syncthreads();
    }
  };
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (wv < CF::LOADERS / 64) {
    if (CF::THREADS == 512 && wv >= 4) loader_loop(std::true_type{});
    else loader_loop(std::false_type{});
  } else {
    __syncthreads();
    for (int t = 0; t < Tp; t += 2) {
      mma(0, noconv_t{}, raw1, 0, 0, std::false_type{});
      __syncthreads();
      mma(1, noconv_t{}, raw0, 0, 0, std::false_type{});
      __syncthreads();
    }
  }

  // Column spread.  The chunk scale keeps 22 bits for values within 2^17 of
  // the chunk max; a whole column far below it (dY / X columns spread over
  // more than 2^16 inside one chunk) would lose bits at its own scale.  Such
  // a tile's chunk is done again (tn_percol, a cold path) with one scale per
  // column — exact powers of two that factor out of dW[n, k] = sum_m dY[m, n]
  // X[m, k] — from the column maxima of the values this pass loaded, left in
  // the 16 padding bytes of each column's slot of stage 0 (the images use
  // bytes 0-63 of the 80-B pitch).
  constexpr int NCOL = CF::YC + CF::XC;
  constexpr int pass = PERCOL ? 1 : 0;
  if constexpr (!PERCOL) {
    __syncthreads();   // every wave's last stage reads are done: the LDS is free
    float* s_cm = reinterpret_cast<float*>(smem + CF::STAGE);   // [4 row groups][NCOL]
    int* s_redo = reinterpret_cast<int*>(smem + CF::STAGE) + 4 * NCOL;
    if (tid == 0) *s_redo = 0;
    if (loader) {
#pragma unroll
      for (int c = 0; c < 4; ++c) s_cm[rg * NCOL + (op == 0 ? 0 : CF::YC) + 4 * cc + c] = cm[c];
    }
    __syncthreads();
    for (int col = tid; col < NCOL; col += CF::THREADS) {
      const float m = fmaxf(fmaxf(s_cm[col], s_cm[NCOL + col]),
                            fmaxf(s_cm[2 * NCOL + col], s_cm[3 * NCOL + col]));
      const int ec = col < CF::YC ? ey : ex;   // the chunk exponent
      if (m > 0.0f && m < __builtin_amdgcn_ldexpf(1.0f, ec - 16)) *s_redo = 1;   // all store 1
      const int e = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
      const int slot = col < CF::YC ? col * T_PITCH : 2 * CF::YPLANE + (col - CF::YC) * T_PITCH;
      *reinterpret_cast<int*>(smem + slot + 64) = e;
    }
    __syncthreads();
    if (*s_redo != 0) {   // workgroup-uniform
      tn_percol<NBN, NBK>(smem, Y, ldy, X, ldx, M, N, K, ymax, xmax, parts, S, mk, nt_k);
      return;
    }
  }

  // un-scale and store the partial tile (every split writes its slot, empty
  // chunks zeros; nontemporal: no dirty L2 lines for the kernel boundary to
  // write back before the column sum, 5.546-5.551 vs 5.553-5.565 ms per step,
  // profiles/r06_ab_tnnt.txt): the chunk exponents, or (pass 1) each column's
  float* out = parts + (int64_t)s * N * K;
  if constexpr (pass == 0) {
    const int sh = ey + ex - 2 * kTT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = k0 + 64 * wk + 32 * j + (lane & 31);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = n0 + 64 * wm + 32 * i + 8 * (e >> 2) + 4 * h + (e & 3);
          __builtin_nontemporal_store(__builtin_amdgcn_ldexpf(acc[i][j][e], sh), out + (int64_t)row * K + col);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int nl = 64 * wm + 32 * i + 8 * (e >> 2) + 4 * h + (e & 3);
        const int en = *reinterpret_cast<const int*>(smem + nl * T_PITCH + 64) - 2 * kTT;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int kl = 64 * wk + 32 * j + (lane & 31);
          const int ek = *reinterpret_cast<const int*>(smem + 2 * CF::YPLANE + kl * T_PITCH + 64);
          __builtin_nontemporal_store(__builtin_amdgcn_ldexpf(acc[i][j][e], en + ek), out + (int64_t)(n0 + nl) * K + k0 + kl);
        }
      }
  }
}

template <int NBN, int NBK>
__device__ __attribute__((noinline)) void tn_percol(char* smem, const float* __restrict__ Y, int64_t ldy, const float* __restrict__ X,
                                        int64_t ldx, int64_t M, int N, int K,
                                        const float* __restrict__ ymax,
                                        const float* __restrict__ xmax, float* __restrict__ parts,
                                        int S, int64_t mk, int nt_k) {
  tn_body<NBN, NBK, true>(smem, Y, ldy, X, ldx, M, N, K, ymax, xmax, parts, S, mk, nt_k);
}

template <int NBN, int NBK>
__global__ void __launch_bounds__(256 * NBN * NBK, 2 / (NBN * NBK))
k_gemm_tn_h(const float* __restrict__ Y, int64_t ldy, const float* __restrict__ X, int64_t ldx,
            int64_t M, int N, int K, const float* __restrict__ ymax,
            const float* __restrict__ xmax, float* __restrict__ parts, int S, int64_t mk,
            int nt_k) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  tn_body<NBN, NBK, false>(smem, Y, ldy, X, ldx, M, N, K, ymax, xmax, parts, S, mk, nt_k);
}


template <bool BIAS, bool WIDE, int NB, bool ACT = false, bool DACT = false>
void run_nt_h(const float* A, int64_t lda, int64_t M, int R, const f16x8* wf, const int* ew, int C,
              const float* bias, float* out, int64_t ldo, float* rmax, int m_tiles, unsigned grid,
              hipStream_t st, float* act = nullptr, DropSpec drop = DropSpec{}, int64_t e_base = 0,
              const float* pre = nullptr, float* dpart = nullptr) {
  constexpr int lds = NtCfg<NB>::LDS + (DACT ? N_WAVES * N_DACT_MAXC * 4 : 0);
  static_assert(lds <= 160 * 1024, "LDS");
  static bool done = false;  // benign race: idempotent
  if (!done) {
    (void)hipFuncSetAttribute((const void*)k_gemm_nt_h<BIAS, WIDE, NB, ACT, DACT>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    done = true;
  }
  k_gemm_nt_h<BIAS, WIDE, NB, ACT, DACT><<<grid, N_THREADS, lds, st>>>(
      A, lda, M, R, wf, ew, C, bias, out, ldo, rmax, m_tiles, act, drop, e_base, pre, dpart);
}


// One phase of a call: the rows [r0, r0 + M) on tiles nbcols columns wide.
NtPhase nt_phase(const float* A, int64_t lda, int64_t r0, int64_t M, float* out, int64_t ldo,
                 float* rmax, int C, int nbcols, int G0, float* act = nullptr,
                 const float* pre = nullptr, float* dpart = nullptr) {
  NtPhase p{};
  p.A = A + r0 * lda;
  p.M = M;
  p.out = out + r0 * ldo;
  p.rmax = rmax ? rmax + r0 / 32 : nullptr;
  p.act = act ? act + r0 * ldo : nullptr;
  p.pre = pre ? pre + r0 * ldo : nullptr;
  p.dpart = dpart;
  p.e_base = r0 * C;
  p.m_tiles = (int)((M + N_BM - 1) / N_BM);
  const int64_t nt = (int64_t)((p.m_tiles + 7) / 8) * 8 * (C / nbcols);
  p.grid = M > 0 ? (int)std::min<int64_t>(nt, (int64_t)G0) : 0;
  return p;
}

template <bool BIAS, int NB, bool ACT = false, bool DACT = false>
void run_nt_h2(int64_t lda, int R, const f16x8* wf, const int* ew, int C, const float* bias,
               int64_t ldo, DropSpec drop, const NtPhase& mp, const NtPhase& tp, hipStream_t st) {
  constexpr int base = NtCfg<NB>::LDS > NtCfg<2>::LDS ? NtCfg<NB>::LDS : NtCfg<2>::LDS;
  constexpr int lds = base + (DACT ? N_WAVES * N_DACT_MAXC * 4 : 0);
  static_assert(lds <= 160 * 1024, "LDS");
  static bool done = false;  // benign race: idempotent
  if (!done) {
    (void)hipFuncSetAttribute((const void*)k_gemm_nt_h2<BIAS, NB, ACT, DACT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    done = true;
  }
  const unsigned grid = (unsigned)std::max(mp.grid, tp.grid);
  k_gemm_nt_h2<BIAS, NB, ACT, DACT><<<grid, N_THREADS, lds, st>>>(lda, R, wf, ew, C, bias, ldo,
                                                                  drop, mp, tp);
}

}  // namespace

int launch_split_weights_h(const rb_split_job* jobs, int n, hipStream_t st) {
  SplitJobsH sj{};
  sj.n = n;
  int blocks = 0;
  for (int j = 0; j < n; ++j) {
    sj.W[j] = jobs[j].W;
    sj.Wf[j] = (f16x8*)jobs[j].Wf;
    sj.ldw[j] = jobs[j].ldw;
    sj.C[j] = (int)jobs[j].C;
    sj.R[j] = (int)jobs[j].R;
    sj.tr[j] = (int)jobs[j].transpose;
    sj.bstart[j] = blocks;
    blocks += (int)(jobs[j].C / 32);
  }
  sj.bstart[n] = blocks;
  k_split_weights_h<<<(unsigned)blocks, 256, 0, st>>>(sj);
  return launch_status("rb_gemm_h_split_weights");
}

// Which kernel takes rb_gemm_nt_h's large-M calls (rb_gemm_nt_h_mode): 1 the
// weight-stationary kernel (gemm_ws.hip, default since round 6), 0 the
// persistent tiles below (A/B).  Below NT_WS_MIN_ROWS rows the launches here
// (tail tiles, the few-rows kernel) keep every call: a weight-stationary
// workgroup loads its 32 KB weight slice per wave before its first block.
static int g_nt_mode = 1;
constexpr int64_t NT_WS_MIN_ROWS = 16384;
int gemm_nt_h_mode(int mode) {
  const int prev = g_nt_mode;
  if (mode == 0 || mode == 1) g_nt_mode = mode;
  return prev;
}

int launch_gemm_nt_h(const float* A, int64_t lda, int64_t M, int R, const void* Wf, int C,
                     const float* bias, float* out, int64_t ldo, int accumulate, float* rmax,
                     hipStream_t st) {
  (void)accumulate;  // rejected by rb_gemm_nt_h
  if (g_nt_mode == 1 && M >= NT_WS_MIN_ROWS && nt_ws_ok(M, R, C, A, lda, out, ldo))
    return launch_gemm_nt_ws(A, lda, M, R, Wf, C, bias, out, ldo, rmax, st);
  const bool wide = (reinterpret_cast<uintptr_t>(out) & 15) == 0 && ldo % 4 == 0;
  const bool nb8 = wide && C % 256 == 0;
  // The persistent grid runs whole rounds of G tiles; the rows past the last
  // whole round would run on a fraction of the chip (800 row tiles on 256
  // CUs: a fourth round on 32 of them, +18% time for +4% rows), so they run
  // as a second launch of 256 x 64 tiles (2-4x as many, each a fraction of
  // the time).  Below one round, or for C % 128 != 0, every row goes to that
  // launch, or to the few-rows kernel (gemm_small.hip) for the few-thousand-
  // row shapes it wins, or for C % 64 != 0.
  const int G0 = num_cus() / 8 * 8 * (8 / N_WAVES);
  // (the few-rows kernel holds R <= 1024; beyond, the persistent kernel takes
  // every row, a partial round included)
  const int nct0 = C % 128 ? 0 : C / (nb8 ? 256 : 128);
  if (R > 1024 && nct0 == 0) return fail("rb_gemm_nt_h: C % 128 != 0 needs R <= 1024");
  const int64_t rows_round = nct0 ? (int64_t)(G0 / nct0) * N_BM : 0;
  int64_t M_main = R > 1024 ? M
                 : (nct0 && G0 % nct0 == 0 && rows_round > 0) ? M / rows_round * rows_round
                                                              : (nct0 ? M : 0);
  const f16x8* wf = (const f16x8*)Wf;
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * R * 4);
  if (M_main < M) {
    // a partial round of 256 x 64 tiles: 4x (2x) the 256 x 256 (256 x 128)
    // tiles of the main launch, each a quarter (half) of their time
    // below one round: the few-rows kernel only where it measured faster
    // (a few thousand rows with K = 512, or C = 128; tools/gemmbench_h.hip,
    // profiles/r03_gemmbench_small_m.log) — at 8,192 rows it is 2.7x slower
    const bool few = M_main == 0 && M <= 4096 && (R > 256 || C < 256);
    if (!few && wide && C % 64 == 0 && M_main > 0) {
      // both phases in one launch (k_gemm_nt_h2)
      const int G0w = num_cus() / 8 * 8 * (8 / N_WAVES);
      const NtPhase mp = nt_phase(A, lda, 0, M_main, out, ldo, rmax, C, nb8 ? 256 : 128, G0w);
      const NtPhase tp = nt_phase(A, lda, M_main, M - M_main, out, ldo, rmax, C, 64, G0w);
      if (bias) {
        if (nb8) run_nt_h2<true, 8>(lda, R, wf, ew, C, bias, ldo, DropSpec{}, mp, tp, st);
        else run_nt_h2<true, 4>(lda, R, wf, ew, C, bias, ldo, DropSpec{}, mp, tp, st);
      } else {
        if (nb8) run_nt_h2<false, 8>(lda, R, wf, ew, C, bias, ldo, DropSpec{}, mp, tp, st);
        else run_nt_h2<false, 4>(lda, R, wf, ew, C, bias, ldo, DropSpec{}, mp, tp, st);
      }
      return launch_status("rb_gemm_nt_h");
    }
    if (!few && wide && C % 64 == 0) {
      const int64_t Mt = M - M_main;
      const int mt_t = (int)((Mt + N_BM - 1) / N_BM);
      const int64_t nt_t = (int64_t)((mt_t + 7) / 8) * 8 * (C / 64);
      const unsigned grid_t = (unsigned)std::min<int64_t>(nt_t, (int64_t)num_cus() / 8 * 8 * (8 / N_WAVES));
      const float* At = A + M_main * lda;
      float* ot = out + M_main * ldo;
      float* rt = rmax ? rmax + M_main / 32 : nullptr;
      if (bias) run_nt_h<true, true, 2>(At, lda, Mt, R, wf, ew, C, bias, ot, ldo, rt, mt_t, grid_t, st);
      else run_nt_h<false, true, 2>(At, lda, Mt, R, wf, ew, C, bias, ot, ldo, rt, mt_t, grid_t, st);
      const int rc = launch_status("rb_gemm_nt_h");
      if (rc || M_main == 0) return rc;
    } else
    {
      const int rc = launch_gemm_nt_hs(A + M_main * lda, lda, M - M_main, R, Wf, C, bias,
                                       out + M_main * ldo, ldo,
                                       rmax ? rmax + M_main / 32 : nullptr, st);
      if (rc || M_main == 0) return rc;
    }
  }
  M = M_main;
  const int m_tiles = (int)((M + N_BM - 1) / N_BM);
  const int64_t n_tiles = (int64_t)((m_tiles + 7) / 8) * 8 * (C / (nb8 ? 256 : 128));
  // persistent: one workgroup per CU (a multiple of 8: the XCD pairing above)
  const unsigned grid = (unsigned)std::min<int64_t>(n_tiles, (int64_t)num_cus() / 8 * 8 * (8 / N_WAVES));
  if (bias) {
    if (nb8) run_nt_h<true, true, 8>(A, lda, M, R, wf, ew, C, bias, out, ldo, rmax, m_tiles, grid, st);
    else if (wide) run_nt_h<true, true, 4>(A, lda, M, R, wf, ew, C, bias, out, ldo, rmax, m_tiles, grid, st);
    else run_nt_h<true, false, 4>(A, lda, M, R, wf, ew, C, bias, out, ldo, rmax, m_tiles, grid, st);
  } else {
    if (nb8) run_nt_h<false, true, 8>(A, lda, M, R, wf, ew, C, bias, out, ldo, rmax, m_tiles, grid, st);
    else if (wide) run_nt_h<false, true, 4>(A, lda, M, R, wf, ew, C, bias, out, ldo, rmax, m_tiles, grid, st);
    else run_nt_h<false, false, 4>(A, lda, M, R, wf, ew, C, bias, out, ldo, rmax, m_tiles, grid, st);
  }
  return launch_status("rb_gemm_nt_h");
}

// out = A Bm^T + bias and act = dropout(silu(out)) in one pass (the
// FeedForward's first projection + its activation, RecBLR.py:219-221).  The
// same row split as launch_gemm_nt_h; only the shapes whose every row runs on
// a wide-epilogue launch are taken (16-B aligned out / act, ldo % 4 == 0,
// C % 256 == 0, not the few-rows kernel's shapes): nt_h_act_ok says which.
bool nt_h_act_ok(int64_t M, int R, int C, const float* out, const float* act, int64_t ldo) {
  const bool wide = (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(act) & 15) == 0 && ldo % 4 == 0;
  const bool few = M <= 4096 && (R > 256 || C < 256);
  return wide && C % 256 == 0 && C <= N_MAXC && R <= 1024 && !few;
}

// ACT's main launch: 256 x 256 tiles stored at the tile's end (264 us at
// 204,632 rows against 140 + 135-142 us for the GEMM and the activation
// kernel; 256 x 128 tiles with the deferred epilogue took 995 us,
// profiles/r03_ffn_probe2.txt)
constexpr int ACT_NB = 8;
int launch_gemm_nt_h_act(const float* A, int64_t lda, int64_t M, int R, const void* Wf, int C,
                         const float* bias, float* out, int64_t ldo, float* rmax, float* act,
                         DropSpec drop, hipStream_t st) {
  if (g_nt_mode == 1 && M >= NT_WS_MIN_ROWS && nt_ws_act_ok(M, R, C, A, lda, out, act, ldo))
    return launch_gemm_nt_ws_act(A, lda, M, R, Wf, C, bias, out, ldo, rmax, act, drop, st);
  if (!nt_h_act_ok(M, R, C, out, act, ldo))
    return fail("rb_gemm_nt_h_act: shape or alignment without a wide-epilogue launch");
  const int G0 = num_cus() / 8 * 8 * (8 / N_WAVES);
  const int nct0 = C / (32 * ACT_NB);
  const int64_t rows_round = (int64_t)(G0 / nct0) * N_BM;
  const int64_t M_main = (G0 % nct0 == 0 && rows_round > 0) ? M / rows_round * rows_round : M;
  const f16x8* wf = (const f16x8*)Wf;
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * R * 4);
  if (M_main > 0 && M_main < M) {   // both phases in one launch (k_gemm_nt_h2)
    const NtPhase mp = nt_phase(A, lda, 0, M_main, out, ldo, rmax, C, 32 * ACT_NB, G0, act);
    const NtPhase tp = nt_phase(A, lda, M_main, M - M_main, out, ldo, rmax, C, 64, G0, act);
    if (bias) run_nt_h2<true, ACT_NB, true>(lda, R, wf, ew, C, bias, ldo, drop, mp, tp, st);
    else run_nt_h2<false, ACT_NB, true>(lda, R, wf, ew, C, bias, ldo, drop, mp, tp, st);
    return launch_status("rb_gemm_nt_h_act");
  }
  if (M_main < M) {   // the rows past the last whole round: 256 x 64 tiles
    const int64_t Mt = M - M_main;
    const int mt_t = (int)((Mt + N_BM - 1) / N_BM);
    const int64_t nt_t = (int64_t)((mt_t + 7) / 8) * 8 * (C / 64);
    const unsigned grid_t = (unsigned)std::min<int64_t>(nt_t, (int64_t)G0);
    const float* At = A + M_main * lda;
    float* ot = out + M_main * ldo;
    float* at = act + M_main * ldo;
    float* rt = rmax ? rmax + M_main / 32 : nullptr;
    if (bias) run_nt_h<true, true, 2, true>(At, lda, Mt, R, wf, ew, C, bias, ot, ldo, rt, mt_t, grid_t, st, at, drop, M_main * C);
    else run_nt_h<false, true, 2, true>(At, lda, Mt, R, wf, ew, C, bias, ot, ldo, rt, mt_t, grid_t, st, at, drop, M_main * C);
    const int rc = launch_status("rb_gemm_nt_h_act");
    if (rc || M_main == 0) return rc;
  }
  const int m_tiles = (int)((M_main + N_BM - 1) / N_BM);
  const int64_t n_tiles = (int64_t)((m_tiles + 7) / 8) * 8 * nct0;
  const unsigned grid = (unsigned)std::min<int64_t>(n_tiles, (int64_t)G0);
  if (bias) run_nt_h<true, true, ACT_NB, true>(A, lda, M_main, R, wf, ew, C, bias, out, ldo, rmax, m_tiles, grid, st, act, drop, 0);
  else run_nt_h<false, true, ACT_NB, true>(A, lda, M_main, R, wf, ew, C, bias, out, ldo, rmax, m_tiles, grid, st, act, drop, 0);
  return launch_status("rb_gemm_nt_h_act");
}

// The backward of launch_gemm_nt_h_act's activation fused into the
// input-gradient GEMM that produces its output gradient: dU = A Bm^T is
// never stored; out = dU * keep * scale * silu'(pre) (pre: the activation's
// input, [M, C] with row stride ldo) and dpart [n_parts, C] receives the
// workgroups' column sums of out (rows past the launches' grids zeroed).
// The same row split and shape contract as the forward (nt_h_act_ok), C <=
// 512.
// DACT's main launch: 256 x 128 tiles stored at the tile's end (the 256 x 256
// tile's 128 accumulators leave no registers for the epilogue's operands)
constexpr int DACT_NB = 4;
int64_t nt_h_dact_parts() { return 2 * (int64_t)(num_cus() / 8 * 8 * (8 / N_WAVES)); }

int launch_gemm_nt_h_dact(const float* A, int64_t lda, int64_t M, int R, const void* Wf, int C,
                          float* out, int64_t ldo, float* rmax, const float* pre, DropSpec drop,
                          float* dpart, int64_t n_parts, hipStream_t st) {
  if (g_nt_mode == 1 && M >= NT_WS_MIN_ROWS && nt_ws_act_ok(M, R, C, A, lda, out, pre, ldo))
    return launch_gemm_nt_ws_dact(A, lda, M, R, Wf, C, out, ldo, rmax, pre, drop, dpart, n_parts, st);
  if (!nt_h_act_ok(M, R, C, out, pre, ldo) || C > N_DACT_MAXC)
    return fail("rb_gemm_nt_h_dact: shape or alignment without a wide-epilogue launch");
  const int G0 = num_cus() / 8 * 8 * (8 / N_WAVES);
  const int nct0 = C / (32 * DACT_NB);
  const int64_t rows_round = (int64_t)(G0 / nct0) * N_BM;
  const int64_t M_main = (G0 % nct0 == 0 && rows_round > 0) ? M / rows_round * rows_round : M;
  const f16x8* wf = (const f16x8*)Wf;
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * R * 4);
  const int m_tiles = (int)((M_main + N_BM - 1) / N_BM);
  const int64_t n_tiles = (int64_t)((m_tiles + 7) / 8) * 8 * nct0;
  const unsigned grid = M_main > 0 ? (unsigned)std::min<int64_t>(n_tiles, (int64_t)G0) : 0u;
  const int64_t Mt = M - M_main;
  const int mt_t = (int)((Mt + N_BM - 1) / N_BM);
  const int64_t nt_t = (int64_t)((mt_t + 7) / 8) * 8 * (C / 64);
  const unsigned grid_t = Mt > 0 ? (unsigned)std::min<int64_t>(nt_t, (int64_t)G0) : 0u;
  if ((int64_t)grid + grid_t > n_parts) return fail("rb_gemm_nt_h_dact: dpart has too few rows");
  if (Mt > 0 && M_main > 0) {   // both phases in one launch (k_gemm_nt_h2)
    const NtPhase mp = nt_phase(A, lda, 0, M_main, out, ldo, rmax, C, 32 * DACT_NB, G0, nullptr,
                                pre, dpart);
    const NtPhase tp = nt_phase(A, lda, M_main, Mt, out, ldo, rmax, C, 64, G0, nullptr, pre,
                                dpart + (int64_t)grid * C);
    run_nt_h2<false, DACT_NB, false, true>(lda, R, wf, ew, C, nullptr, ldo, drop, mp, tp, st);
    const int rc = launch_status("rb_gemm_nt_h_dact");
    if (rc) return rc;
  } else if (Mt > 0) {   // the rows past the last whole round: 256 x 64 tiles
    run_nt_h<false, true, 2, false, true>(A + M_main * lda, lda, Mt, R, wf, ew, C, nullptr,
                                          out + M_main * ldo, ldo, rmax ? rmax + M_main / 32 : nullptr,
                                          mt_t, grid_t, st, nullptr, drop, M_main * C,
                                          pre + M_main * ldo, dpart + (int64_t)grid * C);
    const int rc = launch_status("rb_gemm_nt_h_dact");
    if (rc) return rc;
  }
  if (M_main > 0 && Mt == 0) {
    run_nt_h<false, true, DACT_NB, false, true>(A, lda, M_main, R, wf, ew, C, nullptr, out, ldo, rmax,
                                          m_tiles, grid, st, nullptr, drop, 0, pre, dpart);
    const int rc = launch_status("rb_gemm_nt_h_dact");
    if (rc) return rc;
  }
  const int64_t used = (int64_t)grid + grid_t;
  if (used < n_parts &&
      hipMemsetAsync(dpart + used * C, 0, (size_t)(n_parts - used) * C * 4, st) != hipSuccess)
    return fail("rb_gemm_nt_h_dact: hipMemsetAsync failed");
  return 0;
}

// dW tile: 256 x 128 when N % 256 == 0 (2), else 128 x 256 when K % 256 == 0
// (1), else 128 x 128 (0).  The big tiles are 512-thread workgroups, one per
// CU, so the same split count S (~2 x CUs / (N/128 x K/128)) fills the chip.
inline int tn_tile_shape(int N, int K) {
  return N % 256 == 0 ? 2 : (K % 256 == 0 ? 1 : 0);
}

int launch_gemm_tn_h(const float* Y, int64_t ldy, const float* X, int64_t ldx, int64_t M, int N,
                     int K, const float* ymax, const float* xmax, float* parts, int S,
                     hipStream_t st) {
  // rows per split: a multiple of 32 (the rmax groups)
  const int64_t mk = ((M + S - 1) / S + 31) / 32 * 32;
  auto run = [&](auto nbn_c, auto nbk_c) {
    constexpr int NBN = decltype(nbn_c)::value, NBK = decltype(nbk_c)::value;
    using CF = TnCfg<NBN, NBK>;
    static bool done = false;  // benign race: idempotent
    if (!done) {
      (void)hipFuncSetAttribute((const void*)k_gemm_tn_h<NBN, NBK>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, CF::LDS);
      done = true;
    }
    const int nt_k = K / CF::XC;
    const int nt = (N / CF::YC) * nt_k;
    // (the block -> (tile, split) map needs a multiple of 8 workgroups: any
    // split count, the padding workgroups return at once)
    k_gemm_tn_h<NBN, NBK><<<(unsigned)((nt * S + 7) / 8 * 8), CF::THREADS, CF::LDS, st>>>(
        Y, ldy, X, ldx, M, N, K, ymax, xmax, parts, S, mk, nt_k);
  };
  switch (tn_tile_shape(N, K)) {
    case 2: run(std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{}); break;
    case 1: run(std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{}); break;
    default: run(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{}); break;
  }
  return launch_status("rb_gemm_tn_h");
}

}  // namespace rb
