// gemm_ws.hip — weight-stationary f16x3 NT GEMM: out[M, C] = A[M, K] . Bm[C, K]^T
// (+ bias), fp32 in and out, the two-part fp16 split and three products of
// gemm_half.hip (RecBLR.py:162,165,167,213,214: the encoder's nn.Linear
// forward / input-gradient GEMMs at ntok ~ 200k-410k rows, K in {128, 256,
// 512}).  rb_gemm_nt_h runs it for M >= NT_WS_MIN_ROWS (gemm_half.hip).
//
// Why not gemm_half.hip's persistent tiles (round 6):
// those stream 256 x 256 output tiles with BOTH operands through each CU's
// load path every k-step — the weight fragments are as many bytes as the A
// rows — and their eight waves run each k-step in lock step, so MFMAs, LDS
// reads, the split and the memory issue add up (1.9x the streaming floor,
// MFMA busy <= 0.29).  Here:
//   * each wave keeps its slice of the weight image in REGISTERS for the
//     whole launch (NCB 16-column blocks x K: <= 8,192 values = 128 VGPRs);
//     a workgroup owns a fixed column tile of 8 x 16 NCB columns (K = 128:
//     512, 256: 256, 512: 128) and streams 32-row blocks of A;
//   * the A block comes in ONCE per CU (LDS-DMA for K <= 256, each wave its
//     own 4 rows, read back by the lanes that loaded them — no barrier, hand-
//     counted vmcnt; K = 512: into registers, the compiler's waits), each
//     row's EXACT max over K is reduced across its 16 lanes (DPP), scaled to
//     [2^13, 2^14), split and written into a double-buffered LDS image in the
//     v_mfma_f32_16x16x32_f16 operand layout (XOR-swizzled: conflict-free
//     8-B writes and 16-B reads).  The exact row max replaces the persistent
//     kernel's online scale and its cold recompute tail (rows whose first
//     16 values are small: in the training step the gates input gradient
//     hit it);
//   * every wave multiplies the 32-row block by its columns with the weight
//     slice as the FIRST operand, so a lane holds one row and 4 consecutive
//     columns of each 16 x 16 result; un-scaled (v_ldexp) + bias, paired
//     blocks exchanged by a bank-masked DPP row_ror:8 into whole 128-B row
//     pieces, and stored (nontemporal, through a buffer descriptor whose
//     range drops rows past M) between the NEXT block's MFMA units, so the
//     store stream keeps flowing while the matrix pipe works;
//   * one barrier per block; waves 4-7 split block b + 1 before multiplying
//     block b and waves 0-3 after, so the two waves of a SIMD alternate
//     between the matrix pipe and the split;
//   * the loop has no branch around a vector-memory instruction (blocks past
//     the end run as dummies on zero-record descriptors), so every vmcnt
//     wait is exact.
// The only per-block traffic through a CU's load path is A; A is re-read
// only by the C / (128 NCB) column tiles (gates fwd / dX: 2, the other
// encoder shapes: 1), on the same XCD at the same time.
// Measured (tools/gemm_ws_probe.hip, M = 204,632, profiles/r06_ws_probe.txt):
// the eight encoder shapes 0.66-0.97x the persistent kernel's time.
#include "common.h"

#include <type_traits>
#include <utility>

namespace rb {
namespace ws {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kTR = 14;   // row scale: the row max lands in [2^13, 2^14)
constexpr int kTC = 14;   // column scale (weights), as gemm_half.hip's kTW
constexpr int WAVES = 8, THREADS = 64 * WAVES, RB = 32;

// K inputs, NCB 16-column blocks per wave (B slice: 8 NCB KS VGPRs, <= 128),
// D blocks of A in flight (D raw register sets of NLD 16-B loads)
template <int K, int NCB_, int D_>
struct Cfg {
  static constexpr int KS = K / 32;            // k32 steps
  static constexpr int NCB = NCB_;             // 16-column blocks per wave
  static constexpr int D = D_;                 // prefetch depth (blocks)
  static constexpr int WC = 16 * NCB;          // columns per wave
  static constexpr int NT = WC * WAVES;        // columns per workgroup (column tile)
  static constexpr int NLD = K / 64;           // raw 16-B loads per lane per block
  static constexpr int IMG = RB * K * 4;       // image bytes per block (two f16 planes)
  static constexpr int NST = 2 * NCB;          // dwordx4 stores per lane per block
  // two images, (exp, max) per row and buffer, column exponents + bias
  static constexpr int INFO = 2 * IMG;
  static constexpr int COLS = INFO + 2 * RB * 8;
  // LN epilogue (EPI 3): per buffer, row and wave the (mean, M2) of the wave's
  // 16 columns of the row
  static constexpr int STATS = COLS + NT * 8;
  // STG (K <= 256): the raw A rows land in LDS by LDS-DMA (each wave its own
  // rows, read back by the same lanes: no barrier, hand-counted vmcnt waits,
  // no registers held by loads in flight); K = 512: in registers (D = 1)
  static constexpr bool STG = K <= 256;
  static constexpr int STAGE = STATS + 2 * 2 * RB * WAVES * 4;
  static constexpr int LDS = STAGE + (STG ? D * WAVES * NLD * 1024 : 0);
  static_assert(KS * NCB <= 16 && NCB >= 1, "B slice <= 128 VGPRs");
  static_assert(LDS <= 160 * 1024, "LDS");
};

__device__ __forceinline__ void split2h(f32x2 x, f16x2& h0, f16x2& h1) {
  h0 = __builtin_convertvector(x, f16x2);
  const f32x2 r = x - __builtin_convertvector(h0, f32x2);
  h1 = __builtin_convertvector(r, f16x2);
}

__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float max4abs(f32x4 x) {
  float m, r;
  asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(m) : "v"(x[0]), "v"(x[1]), "v"(x[2]));
  asm("v_max_f32 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(x[3]));
  return r;
}

__device__ __forceinline__ float dpp_x1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_x2(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
}
// lane k of each quad: column k (v[r] = row r) -> row k (v[c] = column c)
__device__ __forceinline__ void quad_transpose(float (&v)[4], int lane) {
  const bool b1 = (lane & 2) != 0, b0 = (lane & 1) != 0;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const float y = dpp_x2(b1 ? v[r] : v[r + 2]);
    if (b1) v[r] = y; else v[r + 2] = y;
  }
#pragma unroll
  for (int r = 0; r < 4; r += 2) {
    const float y = dpp_x1(b0 ? v[r] : v[r + 1]);
    if (b0) v[r] = y; else v[r + 1] = y;
  }
}

template <typename T>
__device__ __forceinline__ T lds_read16(uint32_t addr) {
  T r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
template <int OFF, typename T>
__device__ __forceinline__ T lds_read16o(uint32_t addr) {
  T r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ void lds_write8(uint32_t addr, f16x4 v) {
  asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(addr), "v"(v), "n"(OFF) : "memory");
}
// 16-B global load into registers: an ordinary load, so the compiler places
// (and counts) the vmcnt wait before the first use.  (An inline-asm load that
// the compiler cannot see lets it copy or reuse the destination registers
// while the load is in flight: round 6's first version faulted that way.)
__device__ __forceinline__ f32x4 gload16(const char* base, uint32_t off) {
  return *reinterpret_cast<const f32x4*>(base + off);
}
// 16-B LDS-DMA piece: lane l's bytes at LDS address lds + 16 l
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(uintptr_t)lds, 16,
                                           voff, 0, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Weight image (written by gemm_half.hip's k_split_weights_h beside its own,
// at byte offset ws_image_offset(C, K) of the same buffer):
//   Wi[((cb * KS + s) * 2 + p) * 64 + lane] (16 B) = plane p of
//     Bm[16 cb + (lane & 15)][32 s + 8 (lane >> 4) + 0..7] * 2^(kTC - e_c)
//   exps: int32 e_c at byte offset C * K * 4 (shared with the persistent
//   kernel's image: the same column exponents)
// ABL (timing-only ablations, results not meaningful): 1 no MFMAs, 2 no
// split (loads still waited), 4 no stores, 8 no A loads, 16 no fragment reads;
// 32 (results exact): depth 1 with every wave in the late role.
// EPI: 0 out (+ bias); 1 (ACT, the FeedForward's w_1, RecBLR.py:219-221)
// out = A Bm^T + bias and act = dropout(silu(out)) — the keep-flags drop's
// Philox stream at element index row * C + col, as rb_silu_dropout_fwd draws
// them; 2 (DACT, its backward fused into dU = dA2 W_2) out = dU * keep *
// scale * silu'(pre), dU never stored, and the columns' sums of out per
// workgroup into dpart (the w_1 bias gradient's partials, a fixed order);
// 3 (LN, C = 128: the residual + dropout + LayerNorm after the FeedForward's
// w_2 / the out-projection, RecBLR.py:142, 225-227) s = dropout(out) + pre
// (the residual, [M, 128] at ldo) into `out`, y = LayerNorm(s) into `act`,
// the rows' mean and rstd into ln — rb_add_ln_fwd's outputs, its s bit for
// bit (the same keep-flags per element).  The row statistics need all 8
// waves' columns: each wave leaves its 16 columns' (mean, M2) per row in LDS,
// and after the block's barrier the next iteration combines them (Chan's
// pairwise formula, a fixed order) and normalises the block, whose y is then
// stored between the next block's MFMA units like every deferred result.
struct LnSpec {
  const float* gamma = nullptr;
  const float* beta = nullptr;
  float eps = 0.0f;
  float* mean = nullptr;
  float* rstd = nullptr;
};

template <int K, int NCB, int D, bool BIAS, bool DEFER, int ABL, int EPI = 0>
__global__ void __launch_bounds__(THREADS, 1)
k_gemm_nt_ws(const float* __restrict__ A, int64_t lda, int64_t M, const f16x8* __restrict__ Wi,
             const int* __restrict__ ew, int C, const float* __restrict__ bias,
             float* __restrict__ out, int64_t ldo, float* __restrict__ rmax,
             float* __restrict__ act, DropSpec drop, const float* __restrict__ pre,
             float* __restrict__ dpart, LnSpec ln) {
  using CF = Cfg<K, NCB, D>;
  constexpr int KS = CF::KS, WC = CF::WC, NT = CF::NT, NLD = CF::NLD, NST = CF::NST;
  constexpr bool TWO = EPI == 1 || EPI == 3;        // a second output (act / y)
  constexpr bool PRE = EPI == 2 || EPI == 3;        // a second [M, C] operand (pre / residual)
  constexpr int NSTT = TWO ? 2 * NST : NST;         // result stores per block
  constexpr int NPRE = PRE ? 2 * NCB : 0;           // `pre` loads per block
  constexpr int NSO = NSTT + 1 + (EPI == 3 ? 2 : 0);   // stores per block: + rmax (+ mean, rstd)
  static_assert(EPI != 3 || (NCB == 1 && DEFER), "LN epilogue: whole 128-column rows, deferred stores");
  // depth 1 (K = 512, registers): waves 4-7 take the early role too — they
  // split block b + 1 (loaded during block b - 1) and then issue block b + 2's
  // loads into the freed registers before multiplying block b (2-4% on the
  // K = 512 shapes against all waves late, profiles/r06_early1_probe.txt;
  // ABL bit 32 restores all-late for that A/B)
  constexpr bool EARLY1 = D == 1 && (ABL & 32) == 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x, G = gridDim.x;
  const int nct = C / NT;
  // work item it = bid + i G -> column tile (it / 8) % nct, row block
  // (it / (8 nct)) * 8 + it % 8; G % (8 nct) == 0 (host), so a workgroup's
  // column tile is fixed and the column tiles of one row block are
  // workgroups b, b + 8, ... of one XCD
  const int ct = (bid >> 3) % nct;
  const int64_t nrb = (M + RB - 1) / RB;
  const int64_t rb0 = (int64_t)(bid / (8 * nct)) * 8 + (bid & 7);
  const int64_t rbs = (int64_t)(G / (8 * nct)) * 8;
  const int nb = rb0 < nrb ? (int)((nrb - 1 - rb0) / rbs + 1) : 0;
  // DACT: this workgroup's row of dpart among its column tile's G / nct
  const int64_t prow = (int64_t)(bid / (8 * nct)) * 8 + (bid & 7);
  if (nb == 0) {
    if constexpr (EPI == 2)
      for (int c = tid; c < NT; c += THREADS) dpart[prow * C + ct * NT + c] = 0.0f;
    return;
  }

  const uint32_t sbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)smem;
  const uint32_t s_info = sbase + CF::INFO;   // [2][RB] exps, then [2][RB] maxima
  const uint32_t s_cols = sbase + CF::COLS;   // [NT] column exps - kTR - kTC, [NT] bias
  for (int c = tid; c < NT; c += THREADS) {
    const int e = ew[ct * NT + c] - kTR - kTC;
    const float bv = BIAS ? bias[ct * NT + c] : 0.0f;
    asm volatile("ds_write_b32 %0, %1" ::"v"(s_cols + c * 4), "v"(e) : "memory");
    asm volatile("ds_write_b32 %0, %1" ::"v"(s_cols + (NT + c) * 4), "v"(bv) : "memory");
  }

  const int col0 = ct * NT + wave * WC;   // the wave's first output column
  // ---- the wave's weight slice, resident for the launch (the MFMA's first
  // operand: lane l holds column l % 16, k = 8 (l / 16) + 0..7 of each step)
  f16x8 bw[NCB][KS][2];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        bw[cb][s][p] = Wi[((int64_t)((col0 / 16 + cb) * KS + s) * 2 + p) * 64 + lane];

  // ---- raw A: lane l loads row 4 wave + l / 16 of the block, 16-B chunks
  // 16 j + l % 16 (a wave-instruction: four 256-B row pieces)
  const int my_row = 4 * wave + (lane >> 4);
  uint32_t woff[NLD];   // image write offset (plane 0) of chunk j
#pragma unroll
  for (int j = 0; j < NLD; ++j) {
    const int c = 16 * j + (lane & 15);
    const int r16 = my_row & 15, rb16 = my_row >> 4;
    const int s = c >> 3, g = (c >> 1) & 3, half = c & 1;
    const int pos = (r16 ^ ((4 * s + g) & 15)) + 16 * g;
    woff[j] = (uint32_t)(((rb16 * KS + s) * 2) * 1024 + pos * 16 + half * 8);
  }
  f32x4 ra[CF::STG ? 1 : D][NLD];
  auto blk_r0 = [&](int b) __attribute__((always_inline)) -> int64_t { return (rb0 + (int64_t)b * rbs) * RB; };
  // wave-uniform buffer descriptor over rows [r0, r0 + n) of a row-major
  // matrix (readfirstlane returns int: through uint32_t, or the low word's
  // sign would extend into the high one); lane offsets past the range read
  // zeros / drop the store, so rows past M need no clamp or branch
  auto rsrc_of = [&](const float* p, int64_t r0, int64_t ld) __attribute__((always_inline)) {
    const uint64_t u = reinterpret_cast<uint64_t>(p + r0 * ld);
    const uint64_t ub = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)u) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(u >> 32)) << 32);
    const int64_t n = M - r0 < RB ? (M - r0 > 0 ? M - r0 : 0) : RB;   // 0: a dummy block
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ub), 0, (int)(n * ld * 4), 0x00020000);
  };
  const uint32_t a_voff = (uint32_t)(my_row * lda * 4) + (uint32_t)(lane & 15) * 16;
  const uint32_t s_stage = sbase + CF::STAGE;   // [D][WAVES][NLD] 1-KB DMA pieces (STG)
  auto stage_of = [&](int set) __attribute__((always_inline)) -> uint32_t { return s_stage + (uint32_t)((set * WAVES + wave) * NLD) * 1024; };
  auto issue = [&](int b, f32x4 (&dst)[NLD], int set) __attribute__((always_inline)) {
    if constexpr ((ABL & 8) != 0) return;
    const auto rs = rsrc_of(A, blk_r0(b), lda);
    // (a compiler barrier after the batch, below: no later vector-memory op
    // may be hoisted above these, or the hand-counted waits would be short)
    if constexpr (CF::STG) {
      // lane l's 16 B of piece j land at stage + j KB + 16 l (M0 = the wave's
      // piece base): the lane that loaded them reads them back
      const uint32_t st = __builtin_amdgcn_readfirstlane(stage_of(set));
#pragma unroll
      for (int j = 0; j < NLD; ++j)
        dma16(rs, st + j * 1024, a_voff + j * 256);
    } else {
#pragma unroll
      for (int j = 0; j < NLD; ++j)
        dst[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, a_voff + j * 256, 0, 0));
    }
    asm volatile("" ::: "memory");
  };

  // split of the block whose raw data is in src into image buffer ib: the
  // lane's row max over its chunks, then over the row's 16 lanes (DPP)
  auto split = [&](f32x4 (&src)[NLD], int ib, int set) __attribute__((always_inline)) {
    if constexpr (CF::STG) {
#pragma unroll
      for (int j = 0; j < NLD; ++j) src[j] = lds_read16<f32x4>(stage_of(set) + j * 1024 + lane * 16);
      if constexpr (NLD == 2) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(src[0]), "+v"(src[1]));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(src[0]), "+v"(src[1]), "+v"(src[2]), "+v"(src[3]));
    }
    if constexpr ((ABL & 2) != 0) {
#pragma unroll
      for (int j = 0; j < NLD; ++j) asm volatile("" ::"v"(src[j]));   // (loads still waited)
      return;
    }
    float mx = max4abs(src[0]);
#pragma unroll
    for (int j = 1; j < NLD; ++j) mx = fmaxf(mx, max4abs(src[j]));
    mx = fmaxf(mx, dpp_x1(mx));
    mx = fmaxf(mx, dpp_x2(mx));
    mx = fmaxf(mx, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, mx), 0x124, 0xF, 0xF, false)));  // row_ror:4
    mx = fmaxf(mx, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, mx), 0x128, 0xF, 0xF, false)));  // row_ror:8
    const int e = mx > 0.0f ? __builtin_amdgcn_frexp_expf(mx) : 0;
    const float sc = __builtin_amdgcn_ldexpf(1.0f, kTR - e);
    const uint32_t img = sbase + ib * CF::IMG;
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const f32x4 v = src[j] * sc;
      f16x2 h0a, h1a, h0b, h1b;
      split2h(f32x2{v[0], v[1]}, h0a, h1a);
      split2h(f32x2{v[2], v[3]}, h0b, h1b);
      lds_write8<0>(img + woff[j], f16x4{h0a[0], h0a[1], h0b[0], h0b[1]});
      lds_write8<1024>(img + woff[j], f16x4{h1a[0], h1a[1], h1b[0], h1b[1]});
    }
    if ((lane & 15) == 0) {
      asm volatile("ds_write_b32 %0, %1" ::"v"(s_info + (ib * RB + my_row) * 4), "v"(e) : "memory");
      asm volatile("ds_write_b32 %0, %1" ::"v"(s_info + (2 * RB + ib * RB + my_row) * 4), "v"(mx) : "memory");
    }
  };

  // MFMA read positions: fragment slot lane of step s at ((lane & 15) ^ (4 (s & 3)
  // + (lane >> 4))) + (lane & 48), 16 B each
  uint32_t rpos[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) rpos[t] = (uint32_t)((((lane & 15) ^ ((4 * t + (lane >> 4)) & 15)) + (lane & 48)) * 16);

  // accumulators: acc[r][cb] = the block's rows 16 r + l % 16 (one per lane),
  // columns 16 cb + 4 (l / 16) + 0..3 (the weight slice is the first operand)
  f32x4 acc[2][NCB];
  auto multiply = [&](int ib, auto&& hook) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) acc[r][cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if constexpr ((ABL & 1) != 0) return;
    const uint32_t img = sbase + ib * CF::IMG;
    f16x8 fa[2][2];   // (plane 0, plane 1) of one (step, rb16) unit, two slots
    auto rd = [&](auto uc, int t) __attribute__((always_inline)) {   // unit u = 2 s + r
      constexpr int u = decltype(uc)::value, s = u >> 1, r = u & 1;
      const uint32_t a = img + rpos[s & 3];
      fa[t][0] = lds_read16o<((r * KS + s) * 2 + 0) * 1024, f16x8>(a);
      fa[t][1] = lds_read16o<((r * KS + s) * 2 + 1) * 1024, f16x8>(a);
    };
    rd(std::integral_constant<int, 0>{}, 0);
    auto unit = [&](auto uc) __attribute__((always_inline)) {
      constexpr int u = decltype(uc)::value, t = u & 1, s = u >> 1, r = u & 1;
      if constexpr ((ABL & 16) != 0) {
        // timing ablation: no fragment reads past the first unit
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[0][0]), "+v"(fa[0][1]));
        fa[1][0] = fa[0][0]; fa[1][1] = fa[0][1];
      } else if constexpr (u + 1 < 2 * KS) {
        rd(std::integral_constant<int, u + 1>{}, t ^ 1);
        asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(fa[t][0]), "+v"(fa[t][1]));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[t][0]), "+v"(fa[t][1]));
      }
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        acc[r][cb] = mfma16(bw[cb][s][0], fa[t][1], acc[r][cb]);
        acc[r][cb] = mfma16(bw[cb][s][1], fa[t][0], acc[r][cb]);
        acc[r][cb] = mfma16(bw[cb][s][0], fa[t][0], acc[r][cb]);
      }
      hook(uc);
    };
    [&]<int... U>(std::integer_sequence<int, U...>) __attribute__((always_inline)) {
      (unit(std::integral_constant<int, U>{}), ...);
    }(std::make_integer_sequence<int, 2 * KS>{});
  };

  const uint32_t ldo4 = (uint32_t)ldo * 4;
  // The epilogue of block b: un-scaled (+ bias) results into pend[] in their
  // store layout, stored by flush(i) — at once (!DEFER) or one at a time
  // between block b + 1's MFMA units (DEFER), so the store stream keeps
  // flowing while the matrix pipe works.  NST stores per block; their lane
  // offsets inside the block are constants (soff), the block's descriptor is
  // pending_rs.
  f32x4 pend[NST];
  uint32_t soff[NST];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if constexpr (NCB == 1) {
      soff[r] = (uint32_t)((16 * r + (lane & 15)) * ldo4) + (uint32_t)(col0 + 4 * (lane >> 4)) * 4;
    } else {
#pragma unroll
      for (int q = 0; q < NCB / 2; ++q) {
        const uint32_t off = (uint32_t)((16 * r + (lane & 7)) * ldo4) +
                             (uint32_t)(col0 + 32 * q + 16 * ((lane >> 3) & 1) + 4 * (lane >> 4)) * 4;
        soff[(q * 2 + r) * 2] = off;
        soff[(q * 2 + r) * 2 + 1] = off + 8 * ldo4;
      }
    }
  }
  __amdgpu_buffer_rsrc_t pending_rs = rsrc_of(out, M, ldo);   // no records: dummy stores
  f32x4 pend2[TWO ? NST : 1];                                 // act / y in store layout
  __amdgpu_buffer_rsrc_t pending_act = rsrc_of(TWO ? act : out, M, ldo);
  auto flush = [&](int i) __attribute__((always_inline)) {
    if constexpr ((ABL & 4) == 0) {
      if (i < NST)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pend[i]), pending_rs, soff[i], 0, 2);
      else if constexpr (TWO)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pend2[i - NST]), pending_act,
                                               soff[i - NST], 0, 2);
    }
  };
  // DACT: the block's `pre` values at the lane's accumulator positions (row
  // 16 r + l % 16, columns 16 cb + 4 (l / 16) ..), loaded when the block's
  // MFMAs start; the lane's running column sums of out
  f32x4 prv[PRE ? 2 : 1][PRE ? NCB : 1];
  f32x4 csum[EPI == 2 ? NCB : 1];
  if constexpr (EPI == 2)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) csum[cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  auto load_pre = [&](int b) __attribute__((always_inline)) {
    if constexpr (PRE) {
      const auto rs = rsrc_of(pre, blk_r0(b), ldo);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          prv[r][cb] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
              rs, (uint32_t)((16 * r + (lane & 15)) * ldo4) + (uint32_t)(col0 + 16 * cb + 4 * (lane >> 4)) * 4,
              0, 0));
      asm volatile("" ::: "memory");
    }
  };
  // LN (EPI 3).  The wave's (mean, M2) of its 16 columns of row 16 r + l % 16:
  // over the lane's 4 values, then the lanes l ^ 16 and l ^ 32 holding the
  // row's other column groups (equal counts: M2 = M2a + M2b + (ma - mb)^2 n / 2;
  // both lanes of a pair compute the same sums), into LDS by lanes 0-15
  const uint32_t s_stats = sbase + CF::STATS;   // [2][RB][WAVES] means, then M2s
  constexpr uint32_t kQ = 2 * RB * WAVES * 4;
  f32x4 gm{}, bt{};                              // the lane's 4 columns' gamma, beta
  float lmu[2] = {0.0f, 0.0f}, lrs[2] = {0.0f, 0.0f};   // the previous block's rows' stats
  if constexpr (EPI == 3) {
    gm = *reinterpret_cast<const f32x4*>(ln.gamma + col0 + 4 * (lane >> 4));
    bt = *reinterpret_cast<const f32x4*>(ln.beta + col0 + 4 * (lane >> 4));
  }
  auto ln_part = [&](f32x4 sv, int ib, int r) __attribute__((always_inline)) {
    float m = ((sv[0] + sv[1]) + (sv[2] + sv[3])) * 0.25f;
    float q = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = sv[i] - m;
      q += d * d;
    }
#pragma unroll
    for (int o = 16, n2 = 2; o <= 32; o <<= 1, n2 <<= 1) {
      const float mo = __shfl_xor(m, o), qo = __shfl_xor(q, o);
      const float d = mo - m;
      m = (m + mo) * 0.5f;
      q = (q + qo) + (d * d) * (float)n2;
    }
    if (lane < 16) {
      const uint32_t a = s_stats + ((ib * RB + 16 * r + lane) * WAVES + wave) * 4;
      asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(m) : "memory");
      asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(a), "v"(q), "n"(kQ) : "memory");
    }
  };
  // the previous block (image buffer ibp): its rows' statistics from the 8
  // waves' parts, then y = (s - mean) rstd gamma + beta from pend into pend2
  auto normalize = [&](int ibp) __attribute__((always_inline)) {
    f32x4 pm[2][2], pq[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const uint32_t a = s_stats + ((ibp * RB + 16 * r + (lane & 15)) * WAVES) * 4;
      pm[r][0] = lds_read16<f32x4>(a);
      pm[r][1] = lds_read16o<16, f32x4>(a);
      pq[r][0] = lds_read16o<kQ, f32x4>(a);
      pq[r][1] = lds_read16o<kQ + 16, f32x4>(a);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pm[0][0]), "+v"(pm[0][1]), "+v"(pm[1][0]), "+v"(pm[1][1]),
                 "+v"(pq[0][0]), "+v"(pq[0][1]), "+v"(pq[1][0]), "+v"(pq[1][1]));
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const f32x4 m0 = pm[r][0], m1 = pm[r][1], q0 = pq[r][0], q1 = pq[r][1];
      const float mu = (((m0[0] + m0[1]) + (m0[2] + m0[3])) + ((m1[0] + m1[1]) + (m1[2] + m1[3]))) * 0.125f;
      float dev = 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d0 = m0[i] - mu, d1 = m1[i] - mu;
        dev += d0 * d0;
        dev += d1 * d1;
      }
      const float m2 = (((q0[0] + q0[1]) + (q0[2] + q0[3])) + ((q1[0] + q1[1]) + (q1[2] + q1[3]))) + dev * 16.0f;
      const float rs = 1.0f / sqrtf(m2 * (1.0f / (float)(8 * WC)) + ln.eps);
#pragma unroll
      for (int i = 0; i < 4; ++i) pend2[r][i] = (pend[r][i] - mu) * rs * gm[i] + bt[i];
      lmu[r] = mu;
      lrs[r] = rs;
    }
  };
  // the previous block's mean / rstd: lanes 0-31 hold rows 0-31 (lane l < 16:
  // r = 0, else r = 1); wave 0 stores, every other wave (and lanes 32-63)
  // issues the same store into no records
  auto ln_store = [&](int bprev) __attribute__((always_inline)) {
    const int64_t r0 = bprev >= 0 ? blk_r0(bprev) : M;
    const bool mine = wave == 0 && r0 < M;
    const int64_t n = mine ? (M - r0 < RB ? M - r0 : RB) : 0;
    const uint32_t off = lane < RB ? (uint32_t)lane * 4 : 0x40000000u;
    const float* bases[2] = {ln.mean, ln.rstd};
    const float vals[2] = {lane < 16 ? lmu[0] : lmu[1], lane < 16 ? lrs[0] : lrs[1]};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint64_t u = reinterpret_cast<uint64_t>(bases[k] + (mine ? r0 : 0));
      const uint64_t ub = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)u) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(u >> 32)) << 32);
      const auto rr = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ub), 0, (int)(n * 4), 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(vals[k]), rr, off, 0, 0);
    }
  };
  auto finish = [&](int b, int ib) __attribute__((always_inline)) {
    const int64_t r0 = blk_r0(b);
    // the lane's two rows' exponents; its columns' exponents and bias read
    // per pair of column blocks (fewer live registers)
    int er[2];
    asm volatile("ds_read_b32 %0, %1" : "=v"(er[0]) : "v"(s_info + (ib * RB + (lane & 15)) * 4));
    asm volatile("ds_read_b32 %0, %1" : "=v"(er[1]) : "v"(s_info + (ib * RB + 16 + (lane & 15)) * 4));
    constexpr int NG = NCB == 1 ? 1 : 2;   // column blocks per group
#pragma unroll
    for (int q = 0; q < NCB / NG; ++q) {
      i32x4 ec[NG];
      f32x4 bc[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int cb = NG * q + g;
        ec[g] = lds_read16<i32x4>(s_cols + (wave * WC + cb * 16 + 4 * (lane >> 4)) * 4);
        if (BIAS) bc[g] = lds_read16<f32x4>(s_cols + (NT + wave * WC + cb * 16 + 4 * (lane >> 4)) * 4);
        else bc[g] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      // one wait tied to every register the reads above define
      if constexpr (NG == 1)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(er[0]), "+v"(er[1]), "+v"(ec[0]), "+v"(bc[0]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(er[0]), "+v"(er[1]), "+v"(ec[0]), "+v"(bc[0]),
                     "+v"(ec[1]), "+v"(bc[1]));
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        f32x4 v[NG];
        f32x4 av[NG];   // ACT: dropout(silu(v))
        const int64_t row = r0 + 16 * r + (lane & 15);
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[g][i] = __builtin_amdgcn_ldexpf(acc[r][NG * q + g][i], er[r] + ec[g][i]);
            if (BIAS) v[g][i] += bc[g][i];
          }
          if constexpr (EPI != 0) {
            // keep-flags of the lane's 4 consecutive columns (element index a
            // multiple of 4: C % 4 == 0)
            float mk[4];
            drop.get4(row * C + col0 + 16 * (NG * q + g) + 4 * (lane >> 4), mk);
            if constexpr (EPI == 1) {
#pragma unroll
              for (int i = 0; i < 4; ++i) av[g][i] = fsilu(v[g][i]) * mk[i];
            } else if constexpr (EPI == 2) {
              const f32x4 pv = prv[r][NG * q + g];
#pragma unroll
              for (int i = 0; i < 4; ++i) v[g][i] = (v[g][i] * mk[i]) * fdsilu(pv[i] + 0.0f);
              csum[NG * q + g] += v[g];   // rows past M: du = 0, pre = 0 -> 0
            } else {
              // s = out * keep * scale + residual (rb_add_ln_fwd's order)
              const f32x4 pv = prv[r][NG * q + g];
#pragma unroll
              for (int i = 0; i < 4; ++i) v[g][i] = v[g][i] * mk[i] + pv[i];
            }
          }
        }
        if constexpr (NG == 1) {
          // lane: row 16 r + l % 16, columns 4 (l / 16) .. + 3: 64-B row pieces
          pend[r] = v[0];
          if constexpr (EPI == 1) pend2[r] = av[0];
          if constexpr (EPI == 3) ln_part(v[0], ib, r);
        } else {
          // blocks 2q, 2q + 1 = 32 columns: lanes with (l & 8) take the other
          // block's value from 8 lanes away (DPP row_ror:8, bank-masked), so
          // store X1 holds rows 0..7 and X2 rows 8..15 of the pair as whole
          // 128-B row pieces: lane l -> row l % 8 (+ 8), columns
          // 16 ((l >> 3) & 1) + 4 (l >> 4) .. + 3
          f32x4 x1, x2;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            // (scalar copies first: __builtin_bit_cast of a vector element
            // lvalue read element 0 for every i in this compiler)
            const float f0 = v[0][i], f1 = v[1][i];
            const int a0 = __float_as_int(f0), a1 = __float_as_int(f1);
            x1[i] = __int_as_float(__builtin_amdgcn_update_dpp(a0, a1, 0x128, 0xF, 0xC, false));
            x2[i] = __int_as_float(__builtin_amdgcn_update_dpp(a1, a0, 0x128, 0xF, 0x3, false));
          }
          pend[(q * 2 + r) * 2] = x1;
          pend[(q * 2 + r) * 2 + 1] = x2;
          if constexpr (EPI == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float f0 = av[0][i], f1 = av[1][i];
              const int a0 = __float_as_int(f0), a1 = __float_as_int(f1);
              x1[i] = __int_as_float(__builtin_amdgcn_update_dpp(a0, a1, 0x128, 0xF, 0xC, false));
              x2[i] = __int_as_float(__builtin_amdgcn_update_dpp(a1, a0, 0x128, 0xF, 0x3, false));
            }
            pend2[(q * 2 + r) * 2] = x1;
            pend2[(q * 2 + r) * 2 + 1] = x2;
          }
        }
      }
    }
    pending_rs = rsrc_of(out, r0, ldo);   // nt stores (aux 2), rows past M dropped
    if constexpr (TWO) pending_act = rsrc_of(act, r0, ldo);
  };
  // rmax: the block's max |A| (its rows' maxima from the split), stored by
  // wave 0 of column tile 0.  Every wave runs this and issues the store (a
  // zero-record descriptor drops it): no branch around a store
  auto rmax_store = [&](int b, int ib) __attribute__((always_inline)) {
    const int64_t r0 = blk_r0(b);
    float x = 0.0f;
    if (lane < RB)
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(s_info + (2 * RB + ib * RB + lane) * 4));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
    const bool mine = rmax != nullptr && ct == 0 && wave == 0 && r0 < M;
    const uint64_t u = reinterpret_cast<uint64_t>(rmax) + (mine ? (uint64_t)(r0 / RB) * 4 : 0);
    const uint64_t ub = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)u) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(u >> 32)) << 32);
    const auto rr = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ub), 0, mine ? 4 : 0, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), rr, 0, 0, 0);
  };

  // ---- prologue: blocks 0 .. D - 1 in flight, block 0 split
  // (STG: the raw sets are LDS pieces, ra[0] is only the split's scratch)
  [&]<int... P>(std::integer_sequence<int, P...>) __attribute__((always_inline)) {
    (issue(P, ra[CF::STG ? 0 : P], P), ...);
  }(std::make_integer_sequence<int, D>{});
  if constexpr (CF::STG) wait_vm<(D - 1) * NLD>();   // block 0's pieces landed
  split(ra[0], 0, 0);
  if constexpr (EARLY1) {
    if (wave >= 4) issue(1, ra[0], 0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // The loop has no branch around a memory instruction: blocks past nb (to a
  // multiple of D) run as dummies whose descriptors have no records (loads
  // read zeros, stores are dropped), and the two wave roles run separate
  // copies of the loop.  So every iteration issues the same vector-memory
  // ops in the same order: NLD loads of block b + D, NST + 1 stores (block b
  // and its rmax word).  STG: the wait before block b + 1's split is counted
  // by hand from that order (block b + 1's pieces were issued D - 1
  // iterations earlier):
  //   LATE (split after this block's stores):  D (NST + 1) + (D - 1) NLD
  //   early (split before them):          (D - 1) (NST + 1) + (D - 1) NLD
  // and in the first D - 1 iterations, whose predecessors were the prologue,
  // b (NST + 1) fewer stores — counted as none (a stricter wait).
  // K = 512 (registers): the compiler waits for its own loads.
  // One block: P = b % D (compile time: the raw register sets are never
  // indexed at run time); LATE: split block b + 1 after the MFMAs.
  auto loop = [&](auto late_c) __attribute__((always_inline)) {
    constexpr bool LATE = decltype(late_c)::value;
    constexpr int YS = (LATE ? D : D - 1) * NSO + D * NPRE + (D - 1) * NLD;
    constexpr int Y0 = (D - 1) * NLD + NPRE + (LATE ? NSO : 0);
    auto body = [&](int b, auto par) __attribute__((always_inline)) {
      constexpr int P = decltype(par)::value;
      const int ib = b & 1;
      auto do_split = [&]() __attribute__((always_inline)) {
        if constexpr (CF::STG) {
          if (b >= D - 1) wait_vm<(YS > 63 ? 63 : YS)>();
          else wait_vm<(Y0 > 63 ? 63 : Y0)>();
        }
        split(ra[CF::STG ? 0 : (P + 1) % D], ib ^ 1, (P + 1) % D);
      };
      if constexpr (EARLY1 && !LATE) {
        do_split();
        issue(b + 2, ra[0], 0);
        load_pre(b);
      } else {
        issue(b + D, ra[CF::STG ? 0 : P], P);   // into the set block b held (split in iteration b - 1)
        load_pre(b);
        if constexpr (!LATE) do_split();
      }
      if constexpr (DEFER) {
        // block b - 1's stores (dummies before block 0) between this block's
        // MFMA units, then its rmax word (LN: block b - 1 normalised first,
        // its statistics stored after the rmax word)
        constexpr int U = 2 * KS, STEP = U / NSTT;
        static_assert(STEP >= 1, "more stores than MFMA units");
        if constexpr (EPI == 3) normalize(ib ^ 1);
        multiply(ib, [&](auto uc) __attribute__((always_inline)) {
          constexpr int u = decltype(uc)::value;
          if constexpr (u % STEP == 0 && u / STEP < NSTT) flush(u / STEP);
        });
        rmax_store(b, ib);
        if constexpr (EPI == 3) ln_store(b - 1);
        finish(b, ib);
      } else {
        multiply(ib, [](auto) __attribute__((always_inline)) {});
        finish(b, ib);
#pragma unroll
        for (int i = 0; i < NSTT; ++i) flush(i);
        rmax_store(b, ib);
      }
      if constexpr (LATE) do_split();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    };
    for (int b = 0; b < nb; b += D) {
      [&]<int... P>(std::integer_sequence<int, P...>) __attribute__((always_inline)) {
        (body(b + P, std::integral_constant<int, P>{}), ...);
      }(std::make_integer_sequence<int, D>{});
    }
  };
  if ((D == 1 && !EARLY1) || wave < 4) loop(std::true_type{});
  else loop(std::false_type{});
  if constexpr (DEFER) {
    const int blast = (nb + D - 1) / D * D - 1;   // the last block the loop ran (maybe a dummy)
    if constexpr (EPI == 3) normalize(blast & 1);
#pragma unroll
    for (int i = 0; i < NSTT; ++i) flush(i);   // the last block's results
    if constexpr (EPI == 3) ln_store(blast);
  }
  if constexpr (EPI == 2) {
    // the wave's column sums: the lane's rows, then the 16 lanes of each
    // 4-column group (DPP, a fixed tree); lanes 0, 16, 32, 48 write them
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float x = csum[cb][i];
        x += dpp_x1(x);
        x += dpp_x2(x);
        x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x124, 0xF, 0xF, false));
        x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x128, 0xF, 0xF, false));
        csum[cb][i] = x;
      }
      if ((lane & 15) == 0)
        *reinterpret_cast<f32x4*>(dpart + prow * C + col0 + 16 * cb + 4 * (lane >> 4)) = csum[cb];
    }
  }
}

template <int K, int NCB, int D, bool BIAS, bool DEFER, int ABL, int EPI = 0>
void run(const float* A, int64_t lda, int64_t M, const void* Wi, const int* ew, int C,
         const float* bias, float* out, int64_t ldo, float* rmax, int grid, hipStream_t st,
         float* act = nullptr, DropSpec drop = DropSpec{}, const float* pre = nullptr,
         float* dpart = nullptr, LnSpec ln = LnSpec{}) {
  using CF = Cfg<K, NCB, D>;
  static bool done = false;   // benign race: idempotent
  if (!done) {
    (void)hipFuncSetAttribute((const void*)k_gemm_nt_ws<K, NCB, D, BIAS, DEFER, ABL, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, CF::LDS);
    done = true;
  }
  k_gemm_nt_ws<K, NCB, D, BIAS, DEFER, ABL, EPI><<<grid, THREADS, CF::LDS, st>>>(
      A, lda, M, (const f16x8*)Wi, ew, C, bias, out, ldo, rmax, act, drop, pre, dpart, ln);
}

// prefetch depth per K (blocks of A in flight): the LDS-DMA sets that fit
// beside the two images (K = 128: 3, 256: 2), one register set for K = 512
template <int K>
constexpr int depth() { return K == 512 ? 1 : K == 256 ? 2 : 3; }

// 16-column blocks per wave: as many as the 128-VGPR weight slice holds
// (16 / (K / 32)) and C's column tiles of 128 NCB divide
inline int ncb_for(int K, int C) {
  int ncb = 16 / (K / 32);
  while (ncb > 1 && C % (128 * ncb)) ncb >>= 1;
  return C % (128 * ncb) ? 0 : ncb;
}

// persistent grid: one workgroup per CU, a multiple of 8 x (column tiles)
inline int grid_for(int64_t M, int C, int ncb) {
  const int nct = C / (128 * ncb);
  const int unit = 8 * nct;
  int grid = num_cus() / unit * unit;
  const int64_t items = (M + RB - 1) / RB * nct;
  if (items < grid) grid = (int)((items + unit - 1) / unit * unit);
  return grid;
}

}  // namespace ws

bool nt_ws_ok(int64_t M, int K, int C, const float* A, int64_t lda, const float* out, int64_t ldo) {
  return (K == 128 || K == 256 || K == 512) && ws::ncb_for(K, C) > 0 && aligned16(A) &&
         lda % 4 == 0 && aligned16(out) && ldo % 4 == 0 && M > 0 &&
         (M + ws::RB - 1) / ws::RB <= 0x3fffffffLL;
}

// Wf: the combined image of gemm_half.hip (persistent-kernel planes, the
// column exponents, then this kernel's planes at ws_image_offset)
int launch_gemm_nt_ws(const float* A, int64_t lda, int64_t M, int K, const void* Wf, int C,
                      const float* bias, float* out, int64_t ldo, float* rmax, hipStream_t st) {
  if (!nt_ws_ok(M, K, C, A, lda, out, ldo)) return fail("rb_gemm_nt_h: no weight-stationary launch for this shape");
  const void* Wi = reinterpret_cast<const char*>(Wf) + ws_image_offset(C, K);
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * K * 4);
  const int ncb = ws::ncb_for(K, C);
  const int grid = ws::grid_for(M, C, ncb);
  auto go = [&](auto kc, auto nc) {
    constexpr int KK = decltype(kc)::value, NC = decltype(nc)::value;
    if (bias) ws::run<KK, NC, ws::depth<KK>(), true, true, 0>(A, lda, M, Wi, ew, C, bias, out, ldo, rmax, grid, st);
    else ws::run<KK, NC, ws::depth<KK>(), false, true, 0>(A, lda, M, Wi, ew, C, bias, out, ldo, rmax, grid, st);
  };
  using std::integral_constant;
  if (K == 128 && ncb == 4) go(integral_constant<int, 128>{}, integral_constant<int, 4>{});
  else if (K == 128 && ncb == 2) go(integral_constant<int, 128>{}, integral_constant<int, 2>{});
  else if (K == 128 && ncb == 1) go(integral_constant<int, 128>{}, integral_constant<int, 1>{});
  else if (K == 256 && ncb == 2) go(integral_constant<int, 256>{}, integral_constant<int, 2>{});
  else if (K == 256 && ncb == 1) go(integral_constant<int, 256>{}, integral_constant<int, 1>{});
  else go(integral_constant<int, 512>{}, integral_constant<int, 1>{});
  return launch_status("rb_gemm_nt_h");
}

// The FeedForward's fused activation on this kernel (EPI 1 / 2): K = 128 only
// (w_1 forward, 128 -> 4d; the dU GEMM, 128 -> 4d), two 16-column blocks per
// wave (the second output or the `pre` operand needs the registers of the
// other two)
bool nt_ws_act_ok(int64_t M, int K, int C, const float* A, int64_t lda, const float* out,
                  const float* other, int64_t ldo) {
  return K == 128 && C % 256 == 0 && nt_ws_ok(M, K, C, A, lda, out, ldo) && aligned16(other);
}

int launch_gemm_nt_ws_act(const float* A, int64_t lda, int64_t M, int K, const void* Wf, int C,
                          const float* bias, float* out, int64_t ldo, float* rmax, float* act,
                          DropSpec drop, hipStream_t st) {
  if (!nt_ws_act_ok(M, K, C, A, lda, out, act, ldo)) return fail("rb_gemm_nt_h_act: shape");
  const void* Wi = reinterpret_cast<const char*>(Wf) + ws_image_offset(C, K);
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * K * 4);
  const int grid = ws::grid_for(M, C, 2);
  if (bias) ws::run<128, 2, ws::depth<128>(), true, true, 0, 1>(A, lda, M, Wi, ew, C, bias, out, ldo, rmax, grid, st, act, drop);
  else ws::run<128, 2, ws::depth<128>(), false, true, 0, 1>(A, lda, M, Wi, ew, C, bias, out, ldo, rmax, grid, st, act, drop);
  return launch_status("rb_gemm_nt_h_act");
}

// dpart [n_parts, C]: the workgroups of each column tile write rows
// [0, grid / column tiles); the rest are zeroed here
int launch_gemm_nt_ws_dact(const float* A, int64_t lda, int64_t M, int K, const void* Wf, int C,
                           float* out, int64_t ldo, float* rmax, const float* pre, DropSpec drop,
                           float* dpart, int64_t n_parts, hipStream_t st) {
  if (!nt_ws_act_ok(M, K, C, A, lda, out, pre, ldo)) return fail("rb_gemm_nt_h_dact: shape");
  const void* Wi = reinterpret_cast<const char*>(Wf) + ws_image_offset(C, K);
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * K * 4);
  const int grid = ws::grid_for(M, C, 2);
  const int64_t used = grid / (C / 256);
  if (used > n_parts) return fail("rb_gemm_nt_h_dact: dpart has too few rows");
  ws::run<128, 2, ws::depth<128>(), false, true, 0, 2>(A, lda, M, Wi, ew, C, nullptr, out, ldo, rmax, grid,
                                                      st, nullptr, drop, pre, dpart);
  const int rc = launch_status("rb_gemm_nt_h_dact");
  if (rc) return rc;
  if (used < n_parts &&
      hipMemsetAsync(dpart + used * C, 0, (size_t)(n_parts - used) * C * 4, st) != hipSuccess)
    return fail("rb_gemm_nt_h_dact: hipMemsetAsync failed");
  return 0;
}

// The residual + dropout + LayerNorm after a C = 128 projection (EPI 3):
// y = LN(dropout(A Bm^T + bias) + resid) into y, s (the LN input) into s_out,
// the rows' mean / rstd; resid, y and s_out [M, 128] at row stride ldo
bool nt_ws_ln_ok(int64_t M, int K, int C, const float* A, int64_t lda, const float* y,
                 const float* s_out, const float* resid, int64_t ldo) {
  return C == 128 && nt_ws_ok(M, K, C, A, lda, y, ldo) && ws::ncb_for(K, C) == 1 &&
         aligned16(s_out) && aligned16(resid);
}

int launch_gemm_nt_ws_ln(const float* A, int64_t lda, int64_t M, int K, const void* Wf, int C,
                         const float* bias, const float* resid, DropSpec drop, const float* gamma,
                         const float* beta, float eps, float* y, float* s_out, float* mean,
                         float* rstd, int64_t ldo, float* rmax, hipStream_t st) {
  if (!nt_ws_ln_ok(M, K, C, A, lda, y, s_out, resid, ldo) || !gamma || !beta || !mean || !rstd ||
      !aligned16(gamma) || !aligned16(beta))
    return fail("rb_gemm_nt_h_ln: shape, alignment or null pointer");
  const void* Wi = reinterpret_cast<const char*>(Wf) + ws_image_offset(C, K);
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * K * 4);
  const int grid = ws::grid_for(M, C, 1);
  ws::LnSpec ln;
  ln.gamma = gamma;
  ln.beta = beta;
  ln.eps = eps;
  ln.mean = mean;
  ln.rstd = rstd;
  auto go = [&](auto kc) {
    constexpr int KK = decltype(kc)::value;
    if (bias) ws::run<KK, 1, ws::depth<KK>(), true, true, 0, 3>(A, lda, M, Wi, ew, C, bias, s_out, ldo, rmax, grid, st, y, drop, resid, nullptr, ln);
    else ws::run<KK, 1, ws::depth<KK>(), false, true, 0, 3>(A, lda, M, Wi, ew, C, bias, s_out, ldo, rmax, grid, st, y, drop, resid, nullptr, ln);
  };
  if (K == 128) go(std::integral_constant<int, 128>{});
  else if (K == 256) go(std::integral_constant<int, 256>{});
  else go(std::integral_constant<int, 512>{});
  return launch_status("rb_gemm_nt_h_ln");
}

}  // namespace rb
