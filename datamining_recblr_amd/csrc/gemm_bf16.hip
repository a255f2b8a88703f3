// gemm_bf16.hip — the projections of bf16 activations (BASELINE configs[4]:
// L = 2,048, d = 256, H = 512, 2M rows per step) on the bf16 MFMA pipe
// (v_mfma_f32_16x16x32_bf16), fp32 accumulation.
//
// rb_gemm_nt_bf16: out[M, C] = A[M, R] . Bm[C, R]^T (+ bias[C]), bf16 out
//   nn.Linear's forward (Bm = W) and input gradient (Bm = W^T) on bf16
//   activations (RecBLR.py:162,165,167 and their autograd).  Bm is the fp32
//   weight rounded to bf16 once per call, in MFMA fragment order
//   (rb_gemm_bf16_weight_image: fragment (16-column block cb, k32 block kb)
//   = 64 lanes x 16 B, lane l: column 16 cb + l % 16, k 32 kb + 8 (l / 16)
//   .. + 7), so a k-step's weight slice is a run of contiguous 1 KB DMAs
//   from L2.
//   The bias is added in fp32 before the one rounding to bf16.
// The weight gradients of these Linears run on hipBLASLt's batched split-K
// (linear.wgrad): round 5's bf16 TN kernel here measured 4-24% behind it
// (profiles/r05_tn48_shapes.txt) and was removed in round 6 (git history).
//
// One 512-thread workgroup per CU, 256 x 256 output tiles, waves 4 x 2
// owning 64 x 128 each (4 x 8 blocks of 16 x 16), every operand global -> LDS
// by LDS-DMA, the next k-step issued right after the barrier that frees its
// slot.  LDS: 160 KB, all of a gfx950 CU (3 A stages, A two k-steps ahead,
// + 2 weight stages).  The launcher checks that the device grants it.
#include "common.h"

#include <type_traits>

namespace rb {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ f32x4 mfma_bf16x16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ T bds_read16(uint32_t addr) {
  T r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
template <int OFF, typename T>
__device__ __forceinline__ T bds_read16o(uint32_t addr) {
  T r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}

template <int N>
__device__ __forceinline__ void bwait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// workgroup barrier that no LDS access is moved across
__device__ __forceinline__ void bbarrier() { asm volatile("s_barrier" ::: "memory"); }

// ---------------------------------------------------------------------------
// weight image: Bm[c][k] = W[c * ldw + k] (transpose = 0) or W[k * ldw + c]
// (transpose = 1: Bm = W^T), rounded to bf16, in 16x16x32 fragment order:
// fragment (16-column block cb, k32 block kb) = 64 lanes x 16 B, lane l:
// column 16 cb + l % 16, k 32 kb + 8 (l / 16) .. + 7
__global__ void __launch_bounds__(256) k_bf16_weight_image(const float* __restrict__ W, int64_t ldw,
                                                           int C, int R, int transpose,
                                                           bf16x8* __restrict__ img) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int KB = R / 32;
  if (t >= (int64_t)(C / 16) * KB * 64) return;
  const int lane = (int)(t & 63);
  const int64_t fi = t >> 6;
  const int cb = (int)(fi / KB), kb = (int)(fi % KB);
  const int c = cb * 16 + (lane & 15), k0 = kb * 32 + 8 * (lane >> 4);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    o[j] = (__bf16)(transpose ? W[(int64_t)(k0 + j) * ldw + c] : W[(int64_t)c * ldw + k0 + j]);
  img[t] = o;
}

// ---------------------------------------------------------------------------
constexpr int BF_BM = 256, BF_BN = 256, BF_BK = 64;
constexpr int BF_WAVES = 8, BF_THREADS = 64 * BF_WAVES;
constexpr int BF_A_STAGE = BF_BM * BF_BK * 2;                   // 32 KB: 256 rows x 128 B
constexpr int BF_B_STAGE = (BF_BN / 32) * (BF_BK / 16) * 1024;  // 32 KB: 8 x 4 fragments
constexpr int BF_NSA = 3;                                       // A stages: 2 k-steps ahead
constexpr int BF_LDS = BF_NSA * BF_A_STAGE + 2 * BF_B_STAGE;    // 160 KB

// Persistent over tiles T = blockIdx.x + i * gridDim.x; the column tiles of
// one row tile are neighbouring workgroups of one XCD (same blockIdx % 8), so
// their A re-reads hit that XCD's L2.  A tile's results are rounded and
// stored at its end; the next k-step's wait counts them (they drain during
// that k-step, behind its MFMAs).  v_mfma_f32_16x16x32_bf16 blocks (round 5:
// the chip holds a higher clock under them than under 32x32x16 at equal
// cycles per FLOP, MI355X_MICROARCH.md DVFS item 7), the weight fragment as
// the first operand, so each accumulator block holds the tile transposed:
// lane l owns one row (l % 16) and 4 consecutive columns 4 (l / 16) ..;
// after packing to bf16, v_permlane16_swap of block pairs gives each lane 8
// consecutive columns, one 16-B store (cdna_hip_programming.md T21).
template <bool BIAS>
__global__ void __launch_bounds__(BF_THREADS, 1)
k_gemm_nt_bf(const __bf16* __restrict__ A, int64_t lda, int64_t M, int R,
             const bf16x8* __restrict__ Wf, int C, const float* __restrict__ bias,
             __bf16* __restrict__ out, int64_t ldo, int m_tiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nct = C / BF_BN, KT = R / BF_BK, KB32 = R / 32;
  const int n_tiles = ((m_tiles + 7) >> 3) * 8 * nct;
  const int G = gridDim.x, bid = blockIdx.x;
  const int my_tiles = bid < n_tiles ? (n_tiles - 1 - bid) / G + 1 : 0;
  const int U = my_tiles * KT;
  if (U == 0) return;
  auto tile_of = [&](int i, int& mt, int& ct) {
    const int T = bid + i * G;
    const int g = T >> 3;
    ct = g % nct;
    mt = (g / nct) * 8 + (T & 7);
  };

  // ---- DMA of one k-step into stage `slot`.  A image: 128-B rows, 16-B
  // chunk c of row r at chunk c ^ ((r >> 1) & 7) (conflict-free fragment
  // reads); wave w moves rows 32w .. 32w + 31 (4 x 8 rows).  B image:
  // fragment (16-column block j, k32 half s) at (2 j + s) KB; wave w moves
  // blocks 2w, 2w + 1.
  int d_i = 0, d_kt = 0, d_mt, d_ct, a_slot = 0;
  const char* d_base = nullptr;   // the wave's first row of the tile (uniform)
  uint32_t d_off[4];              // + 32-bit lane offsets (rows past M repeat row M - 1)
  auto d_tile = [&]() {
    tile_of(d_i, d_mt, d_ct);
    // base row clamped to M - 1 (padding tiles past m_tiles start there), so
    // every lane offset is a non-negative row distance of at most 31
    const int64_t r0 = (int64_t)d_mt * BF_BM + wave * 32;
    const int64_t rb0 = r0 < M ? r0 : M - 1;
    d_base = reinterpret_cast<const char*>(A + rb0 * lda);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rr = q * 8 + (lane >> 3);
      const int64_t r = (r0 + rr < M ? r0 + rr : M - 1) - rb0;
      d_off[q] = (uint32_t)(r * lda * 2) + (((lane & 7) ^ ((rr >> 1) & 7)) << 4);
    }
  };
  d_tile();
  // A (HBM) runs two k-steps ahead through 3 stages, B (L2) one ahead
  // through 2: per wave and k-step 4 DMAs each
  auto issueA = [&]() {
    char* sa = smem + a_slot * BF_A_STAGE + wave * 4096;
    const char* b = d_base + d_kt * (BF_BK * 2);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((const void*)(b + d_off[q]), (lds_ptr_t)(sa + q * 1024), 16, 0, 0);
    a_slot = a_slot == BF_NSA - 1 ? 0 : a_slot + 1;
    if (++d_kt == KT) {
      d_kt = 0;
      if (++d_i < my_tiles) d_tile();
    }
  };
  int b_i = 0, b_kt = 0, b_mt, b_ct;
  tile_of(0, b_mt, b_ct);
  auto issueB = [&](int slot) {
    char* sb = smem + BF_NSA * BF_A_STAGE + slot * BF_B_STAGE + wave * 4096;
    const bf16x8* ws = Wf + ((int64_t)(b_ct * 16 + 2 * wave) * KB32 + b_kt * 2) * 64 + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((const void*)(ws + ((q >> 1) * KB32 + (q & 1)) * 64),
                                       (lds_ptr_t)(sb + q * 1024), 16, 0, 0);
    if (++b_kt == KT) {
      b_kt = 0;
      if (++b_i < my_tiles) tile_of(b_i, b_mt, b_ct);
    }
  };

  // wave tile 64 rows x 128 columns = 4 x 8 blocks of 16 x 16
  f32x4 acc[4][8];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  const uint32_t smem_base = (uint32_t)(uintptr_t)(lds_ptr_t)smem;
  // A fragment (rows 64 wm + 16 rb + lane % 16, k 32 s + 8 (lane / 16) ..):
  // logical chunk 4s + lane / 16 of its row;
  // ((4s + h) ^ sw) << 4 = ((h ^ sw) << 4) ^ (s << 6): one register per rb
  uint32_t a_off[4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int row = wm * 64 + rb * 16 + (lane & 15);
    a_off[rb] = row * 128 + (((lane >> 4) ^ ((row >> 1) & 7)) << 4);
  }

  // issue order: A(0), B(0), A(1); then in step u: B(u + 1), A(u + 2); a
  // tile's 16 result stores (per wave) follow its last step's MFMAs
  issueA();
  issueB(0);
  if (U > 1) issueA();
  int i = 0, kt = 0, sa_slot = 0;
  bool stored_prev = false;
  for (int u = 0; u < U; ++u) {
    // own DMAs A(u), B(u) landed; younger than B(u): A(u + 1) (4, when it
    // exists) and the 16 stores at the end of step u - 1 (a whole tile's)
    if (u + 1 < U) {
      if (stored_prev) bwait_vm<20>(); else bwait_vm<4>();
    } else {
      if (stored_prev) bwait_vm<16>(); else bwait_vm<0>();
    }
    bbarrier();
    if (u + 1 < U) issueB((u + 1) & 1);
    if (u + 2 < U) issueA();
    const uint32_t sa = smem_base + sa_slot * BF_A_STAGE;
    sa_slot = sa_slot == BF_NSA - 1 ? 0 : sa_slot + 1;
    const uint32_t sb =
        smem_base + BF_NSA * BF_A_STAGE + (u & 1) * BF_B_STAGE + wn * 16384 + lane * 16;
    stored_prev = false;
    // two k32 halves; the second half's 12 reads are in flight during the
    // first half's 32 MFMAs
    bf16x8 fa[2][4], fb[2][8];
    auto load = [&](auto S_) {
      constexpr int s = decltype(S_)::value;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) fa[s][rb] = bds_read16<bf16x8>(sa + (a_off[rb] ^ (s << 6)));
      fb[s][0] = bds_read16o<(0 + s) * 1024, bf16x8>(sb);
      fb[s][1] = bds_read16o<(2 + s) * 1024, bf16x8>(sb);
      fb[s][2] = bds_read16o<(4 + s) * 1024, bf16x8>(sb);
      fb[s][3] = bds_read16o<(6 + s) * 1024, bf16x8>(sb);
      fb[s][4] = bds_read16o<(8 + s) * 1024, bf16x8>(sb);
      fb[s][5] = bds_read16o<(10 + s) * 1024, bf16x8>(sb);
      fb[s][6] = bds_read16o<(12 + s) * 1024, bf16x8>(sb);
      fb[s][7] = bds_read16o<(14 + s) * 1024, bf16x8>(sb);
    };
    auto mma = [&](auto S_) {
      constexpr int s = decltype(S_)::value;
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[rb][j] = mfma_bf16x16(fb[s][j], fa[s][rb], acc[rb][j]);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    load(I0{});
    load(I1{});
    asm volatile("s_waitcnt lgkmcnt(12)" : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[0][2]),
                 "+v"(fa[0][3]), "+v"(fb[0][0]), "+v"(fb[0][1]), "+v"(fb[0][2]), "+v"(fb[0][3]),
                 "+v"(fb[0][4]), "+v"(fb[0][5]), "+v"(fb[0][6]), "+v"(fb[0][7]));
    mma(I0{});
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fa[1][2]),
                 "+v"(fa[1][3]), "+v"(fb[1][0]), "+v"(fb[1][1]), "+v"(fb[1][2]), "+v"(fb[1][3]),
                 "+v"(fb[1][4]), "+v"(fb[1][5]), "+v"(fb[1][6]), "+v"(fb[1][7]));
    mma(I1{});

    if (kt == KT - 1) {
      // the tile's results: + bias in fp32, one rounding to bf16, 16-B stores
      int mt, ct;
      tile_of(i, mt, ct);
      const bool full = (int64_t)mt * BF_BM + BF_BM <= M;
      if (mt < m_tiles) {
        // lane l holds row 64 wm + 16 rb + l % 16 of the tile, columns
        // 4g .. 4g + 3 (g = l / 16) of each 16-column block; bf16 pairs
        // packed, then v_permlane16_swap of blocks (j, j + 1): 16-lane rows
        // g = 0, 2 hold columns 8 (g / 2) .. + 7 of block j, rows g = 1, 3
        // those of block j + 1 -> one 16-B store per block pair
        const int g = lane >> 4;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int64_t row = (int64_t)mt * BF_BM + wm * 64 + rb * 16 + (lane & 15);
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const int colj = ct * BF_BN + wn * 128 + 16 * j;
            uint32_t pk[2][2];
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              const int c0 = colj + 16 * jj + 4 * g;
              const f32x4 b4 = BIAS ? *reinterpret_cast<const f32x4*>(bias + c0) : f32x4{0, 0, 0, 0};
              const f32x4 x = acc[rb][j + jj] + b4;
              const u32x2 w = __builtin_bit_cast(u32x2, __builtin_convertvector(x, bf16x4));
              pk[jj][0] = w[0];
              pk[jj][1] = w[1];
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const auto r = __builtin_amdgcn_permlane16_swap(pk[0][q], pk[1][q], false, false);
              pk[0][q] = r[0];
              pk[1][q] = r[1];
            }
            if (full || row < M)
              *reinterpret_cast<uint4*>(out + row * ldo + colj + 16 * (g & 1) + 8 * (g >> 1)) =
                  make_uint4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]);
          }
        }
        stored_prev = full;   // 16 stores issued (partial tiles: fewer, not counted)
      }
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[rb][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      kt = 0;
      ++i;
    } else {
      ++kt;
    }
  }
}

template <typename F>
bool set_lds(F* f, int bytes) {
  return hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) ==
         hipSuccess;
}

}  // namespace

int launch_bf16_weight_image(const float* W, int64_t ldw, int C, int R, int transpose, void* img,
                             hipStream_t st) {
  const int64_t total = (int64_t)(C / 16) * (R / 32) * 64;
  k_bf16_weight_image<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(W, ldw, C, R, transpose,
                                                                       (bf16x8*)img);
  return launch_status("rb_gemm_bf16_weight_image");
}

int launch_gemm_nt_bf16(const void* A, int64_t lda, int64_t M, int R, const void* img, int C,
                        const float* bias, void* out, int64_t ldo, hipStream_t st) {
  static bool attr = false;   // benign race: idempotent
  if (!attr) {
    if (!set_lds(k_gemm_nt_bf<true>, BF_LDS) || !set_lds(k_gemm_nt_bf<false>, BF_LDS))
      return fail("rb_gemm_nt_bf16: the device refused 160 KB of LDS per workgroup (gfx950 only)");
    attr = true;
  }
  const int m_tiles = (int)((M + BF_BM - 1) / BF_BM);
  const int64_t n_tiles = (int64_t)((m_tiles + 7) / 8) * 8 * (C / BF_BN);
  const unsigned grid = (unsigned)std::min<int64_t>(n_tiles, (int64_t)num_cus() / 8 * 8);
  const __bf16* a = (const __bf16*)A;
  const bf16x8* w = (const bf16x8*)img;
  __bf16* o = (__bf16*)out;
  if (bias)
    k_gemm_nt_bf<true><<<grid, BF_THREADS, BF_LDS, st>>>(a, lda, M, R, w, C, bias, o, ldo, m_tiles);
  else
    k_gemm_nt_bf<false><<<grid, BF_THREADS, BF_LDS, st>>>(a, lda, M, R, w, C, bias, o, ldo, m_tiles);
  return launch_status("rb_gemm_nt_bf16");
}

}  // namespace rb
