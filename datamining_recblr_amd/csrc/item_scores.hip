// item_scores.hip — sequence representations scored against the item table on
// fp32 MFMA, without materialising the [B, V] logits:
//   * softmax cross-entropy over all items, forward and backward
//     (RecBLR.py:100-102: logits = seq_output @ item_embedding.weight^T,
//     nn.CrossEntropyLoss, mean over the batch);
//   * the rank of each row's target item among all items (the quantity the
//     full-sort Hit/NDCG/MRR@k evaluation reduces to, RecBLR.py:114-122 and
//     run_with_unseen.py:229-265);
//   * the plain score matrix (full_sort_predict itself).
//
// One wave computes 32 x 32 score tiles with v_mfma_f32_32x32x2_f32 over the
// full feature depth D; the 32-row operand that stays fixed over a wave's
// loop lives in registers, the other is streamed (L1/L2-resident: the item
// table is re-read by every row block).  Each lane owns the half
// k in [h*D/2, h*D/2 + D/2) of every row (h = lane / 32), so step s of the
// MFMA chain sums k = s (lanes 0-31) then k = D/2 + s (lanes 32-63).
// k_target_dot replays that exact fma chain, so a target's score is
// bit-identical to the score the tile kernels compute for it.
//
// An accumulator tile X has its column on the lane and its rows in the 16
// registers (row = (r&3) + 8(r>>2) + 4h), so X feeds the next MFMA as the
// operand summed over X's rows with no data movement: the CE backward uses
// P = softmax - onehot straight from the accumulators for dE = P W and
// dW = P^T E.  Every partial sum is written per split and reduced in a fixed
// order: results are deterministic.
#include <cfloat>
#include <cmath>
#include <type_traits>

#include "common.h"

namespace rb {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWaves = 4;            // waves per workgroup
constexpr int kTile = 32;            // rows (items or sequences) per wave tile
constexpr int64_t kTargetWgs = 512;  // ~2 workgroups per CU over 256 CUs

__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// o[s] = row[h * KH + s] (global or LDS)
template <int KH>
__device__ __forceinline__ void ld_half(float (&o)[KH], const float* row, int h) {
  const float4* p = reinterpret_cast<const float4*>(row + h * KH);
#pragma unroll
  for (int q = 0; q < KH / 4; ++q) {
    const float4 t = p[q];
    o[4 * q] = t.x; o[4 * q + 1] = t.y; o[4 * q + 2] = t.z; o[4 * q + 3] = t.w;
  }
}

// ---- the streamed operand: 32-row tiles through double-buffered LDS ---------------
// The workgroup's 4 waves own 128 fixed rows (one 32-row register operand
// each) and walk the same streamed tiles, so a tile is fetched from L2 once
// per workgroup.  Tiles move global -> LDS by LDS-DMA (global_load_lds,
// 16 B per lane), issued for tile t+1 before tile t is consumed.  The DMA
// image is lane-linear (rows of D floats back to back), so the bank spread
// comes from an XOR swizzle applied on the global side: physical 16-B slot
// `p` of row r holds logical slot p ^ (r mod D/4).  A lane reading 16 B of
// row j at logical slot c reads physical slot c ^ (j mod D/4): the 16 rows
// of a read phase land in 16 distinct bank groups.
template <int D>
struct Stream {
  static constexpr int NS = D / 4;                // 16-B slots per row
  static constexpr int NI = kTile * D * 4 / 1024; // 1-KB wave DMA instructions per tile
  static constexpr int FLOATS = kTile * D;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int D>
__device__ __forceinline__ void tile_dma(float* buf, const float* M, int64_t r0, int64_t n) {
  using S = Stream<D>;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i0 = 0; i0 < S::NI; i0 += kWaves) {
    const int i = i0 + wave;
    if (S::NI % kWaves == 0 || i < S::NI) {
      const int p = i * 64 + lane;
      const int row = p / S::NS, slot = p % S::NS;
      const float* g = M + min(r0 + row, n - 1) * D + (slot ^ (row % S::NS)) * 4;
      __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)(buf + i * 256), 16, 0, 0);
    }
  }
}

// per-row lse (f32) and target (i64) of rows [r0, r0 + 32) -> LDS (wave 0)
__device__ __forceinline__ void rowdata_dma(float* lbuf, int64_t* tbuf, const float* lse,
                                            const int64_t* tgt, int64_t r0, int64_t n) {
  const int lane = threadIdx.x & 63;
  if ((threadIdx.x >> 6) != 0) return;
  __builtin_amdgcn_global_load_lds(lse + min(r0 + (lane & 31), n - 1), (lds_ptr_t)lbuf, 4, 0, 0);
  const char* tp = reinterpret_cast<const char*>(tgt + min(r0 + (lane >> 1), n - 1)) + (lane & 1) * 4;
  __builtin_amdgcn_global_load_lds(tp, (lds_ptr_t)tbuf, 4, 0, 0);
}

// per-row int32 exponents of rows [r0, r0 + 32) -> LDS (wave 0; lanes 32-63
// repeat them into the buffer's upper half)
__device__ __forceinline__ void rowexp_dma(float* ebuf, const float* ex, int64_t r0, int64_t n) {
  const int lane = threadIdx.x & 63;
  if ((threadIdx.x >> 6) != 0) return;
  __builtin_amdgcn_global_load_lds(ex + min(r0 + (lane & 31), n - 1), (lds_ptr_t)ebuf, 4, 0, 0);
}

template <int D>
__device__ __forceinline__ float lds_at(const float* tile, int row, int col) {
  using S = Stream<D>;
  return tile[row * D + (((col >> 2) ^ (row % S::NS)) << 2) + (col & 3)];
}

// Operand reads of the second GEMM: element [crow(s, h)][n*32 + j] of a
// swizzled tile.  With row = R_s + 4h (R_s = (s&3) + 8(s>>2), bit 2 clear)
// the swizzle splits into a lane part that depends only on s&3 and a
// compile-time part, so each read is one ds_read_b32 with an immediate
// offset from one of four per-lane bases.  D >= 32.
template <int D>
struct ColReader {
  int base[4];
  __device__ __forceinline__ ColReader(int j, int h) {
    constexpr int NS = Stream<D>::NS;
    const int H = NS > 4 ? 4 * h : 0;
    const int Lh = (j >> 2) ^ H;
#pragma unroll
    for (int q = 0; q < 4; ++q) base[q] = 4 * h * D + (j & 3) + ((Lh ^ q) << 2);
  }
  template <int S_, int N_>
  __device__ __forceinline__ float at(const float* tile) const {
    constexpr int NS = Stream<D>::NS;
    constexpr int R = (S_ & 3) + 8 * (S_ >> 2);
    constexpr int Xc = R % NS;
    constexpr int off = R * D + (((N_ * 8) ^ (Xc & ~7)) << 2);
    return tile[base[S_ & 3] + off];
  }
};

// X = A B over the full depth with one operand's row j read from a swizzled
// LDS tile (kTileIsA: the tile supplies A) and the other held in registers.
// The tile reads run two 16-B loads ahead of the MFMAs consuming them.
template <int D, int KH, bool kTileIsA>
__device__ __forceinline__ f32x16 lds_dot(const float* tile, int j, int h, const float (&r)[KH]) {
  constexpr int NQ = KH / 4;
  constexpr int AHEAD = NQ < 2 ? NQ : 2;
  const float* row = tile + j * D;
  int sw = j % Stream<D>::NS;
  // opaque per call: keeps the 16 swizzled addresses out of loop-invariant
  // code motion (hoisted, they would pin 16-32 VGPRs for the whole loop)
  asm volatile("" : "+v"(sw));
  auto rd = [&](int q) {
    return *reinterpret_cast<const float4*>(row + (((h * KH / 4) + q) ^ sw) * 4);
  };
  float4 w[NQ];
#pragma unroll
  for (int q = 0; q < AHEAD; ++q) w[q] = rd(q);
  f32x16 acc = {};
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q + AHEAD < NQ) w[q + AHEAD] = rd(q + AHEAD);
    __builtin_amdgcn_sched_barrier(0);
    const float t[4] = {w[q].x, w[q].y, w[q].z, w[q].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = kTileIsA ? t[e] : r[4 * q + e];
      const float b = kTileIsA ? r[4 * q + e] : t[e];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// acc[n] += P^T-operand (registers p, the accumulator tile of the first
// GEMM) x tile rows crow(s, h), columns n*32 + j: the second GEMM of the CE
// backward.  The NT accumulator chains are interleaved.
template <int D, int NT>
__device__ __forceinline__ void gemm2(f32x16 (&acc)[NT], const float (&p)[16], const float* tile,
                                      const ColReader<D>& cr, int j, int h) {
  if constexpr (D >= 32) {
    static_for<0, 16>([&](auto s) {
      static_for<0, NT>([&](auto n) {
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(p[s], cr.template at<s, n>(tile), acc[n], 0,
                                                      0, 0);
      });
    });
  } else {
    const int col = min(j, D - 1);
#pragma unroll
    for (int s = 0; s < 16; ++s)
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(p[s], lds_at<D>(tile, crow(s, h), col), acc[0],
                                                    0, 0, 0);
  }
}

// Tile-relative bounds for the epilogues: item/row index v0 + c is valid when
// lo <= c < hi, and is the target when c == tt (all int32, branch-free).
__device__ __forceinline__ int rel32(int64_t x, int64_t v0) {
  return (int)max<int64_t>(-1, min<int64_t>(x - v0, kTile + 1));
}

// log-sum-exp state (m, s): sum_i exp(x_i) = s * exp(m)
__device__ __forceinline__ void lse_push(float& m, float& s, float x) {
  const float d = x - m;
  const float e = fexp(-fabsf(d));
  s = d > 0.0f ? fmaf(s, e, 1.0f) : s + e;
  m = fmaxf(m, x);
}
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  if (M == -INFINITY) return;
  s = s * fexp(m - M) + s2 * fexp(m2 - M);
  m = M;
}

// ---- target scores: the MFMA chain order, one thread per row ------------------
template <int D>
__global__ __launch_bounds__(256) void k_target_dot(const float* __restrict__ E,
                                                    const float* __restrict__ W,
                                                    const int64_t* __restrict__ tgt, int64_t B,
                                                    int64_t V, float* __restrict__ ts) {
  constexpr int KH = D / 2;
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const int64_t t = tgt[b];
  if (t < 0 || t >= V) {
    ts[b] = NAN;
    return;
  }
  float e0[KH], e1[KH], w0[KH], w1[KH];
  ld_half<KH>(e0, E + b * D, 0);
  ld_half<KH>(e1, E + b * D, 1);
  ld_half<KH>(w0, W + t * D, 0);
  ld_half<KH>(w1, W + t * D, 1);
  float acc = 0.0f;
#pragma unroll
  for (int s = 0; s < KH; ++s) {
    acc = fmaf(w0[s], e0[s], acc);
    acc = fmaf(w1[s], e1[s], acc);
  }
  ts[b] = acc;
}


// Workgroup placement.  The grid is 1-D over RB fixed-row blocks x S splits
// of the streamed operand (S padded to a multiple of 8).  Workgroups are
// dealt to the 8 XCDs round-robin by linear id, so giving split s only ids
// with id % 8 == s % 8 keeps every slice of the streamed operand in one
// XCD's L2 (each XCD streams 1/8 of it) instead of all eight.
struct Place {
  int64_t rb, split;
};

__device__ __forceinline__ bool place(int64_t RB, int64_t S, Place& p) {
  const int64_t L = blockIdx.x, xcd = L & 7, k = L >> 3;
  p.rb = k % RB;
  p.split = (k / RB) * 8 + xcd;
  return p.split < S;
}

// Shared frame of the row-stationary kernels: the workgroup's 4 waves own
// 128 fixed rows (32 per wave) and walk tiles [split*per, ...) of `strm`
// [n_strm, D].  body(tile_index, lds_tile, lds_lse, lds_tgt) runs once per
// streamed tile with the tile resident in LDS; with kRowData 1 the tile's
// per-row lse / target values ride along, with 2 the per-row int32 scale
// exponents of a split image (passed as lse_g, landing in lds_lse), with 3
// all three (the exponents from ex_g into a fifth body argument).
template <int D, int kRowData, class Body>
__device__ __forceinline__ void stream_tiles(const float* strm, int64_t n_strm, int64_t per,
                                             int64_t split, const float* lse_g,
                                             const int64_t* tgt_g, Body&& body,
                                             const float* ex_g = nullptr) {
  using S = Stream<D>;
  // two distinct LDS objects (not one indexed array): the compiler then sees
  // that reads of one buffer cannot alias the DMA in flight into the other
  // and does not drain the DMA (vmcnt(0)) before them
  __shared__ __attribute__((aligned(16))) float buf0[S::FLOATS];
  __shared__ __attribute__((aligned(16))) float buf1[S::FLOATS];
  __shared__ __attribute__((aligned(16))) float lbuf0[64];
  __shared__ __attribute__((aligned(16))) float lbuf1[64];
  __shared__ __attribute__((aligned(16))) int64_t tbuf0[32];
  __shared__ __attribute__((aligned(16))) int64_t tbuf1[32];
  __shared__ __attribute__((aligned(16))) float xbuf0[kRowData == 3 ? 64 : 1];
  __shared__ __attribute__((aligned(16))) float xbuf1[kRowData == 3 ? 64 : 1];
  const int64_t nt = (n_strm + kTile - 1) / kTile;
  const int64_t t0 = split * per, t1 = min(t0 + per, nt);
  if (t0 >= t1) return;
  auto issue = [&](int64_t t, float* b, float* lb, int64_t* tb, float* xb) {
    tile_dma<D>(b, strm, t * kTile, n_strm);
    if constexpr (kRowData == 1 || kRowData == 3) rowdata_dma(lb, tb, lse_g, tgt_g, t * kTile, n_strm);
    if constexpr (kRowData == 2) rowexp_dma(lb, lse_g, t * kTile, n_strm);
    if constexpr (kRowData == 3) rowexp_dma(xb, ex_g, t * kTile, n_strm);
  };
  auto run = [&](int64_t t, const float* b, const float* lb, const int64_t* tb, const float* xb) {
    if constexpr (kRowData == 3) body(t, b, lb, tb, xb);
    else body(t, b, lb, tb);
  };
  issue(t0, buf0, lbuf0, tbuf0, xbuf0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int64_t t = t0; t < t1; t += 2) {
    if (t + 1 < t1) issue(t + 1, buf1, lbuf1, tbuf1, xbuf1);
    run(t, buf0, lbuf0, tbuf0, xbuf0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t + 1 >= t1) break;
    if (t + 2 < t1) issue(t + 2, buf0, lbuf0, tbuf0, xbuf0);
    run(t + 1, buf1, lbuf1, tbuf1, xbuf1);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
}

// ---- CE forward: per (row, vocab split) log-sum-exp partials --------------------
// Tile orientation X^T[v][b] (A = item rows from LDS, B = sequence rows in
// registers): each lane holds one sequence row b and 16 items per tile, so
// its running (m, s) is one pair; the two lane halves merge at the end.  The
// lane whose tile holds b's target stores that score (bit-identical to the
// value inside the log-sum-exp).
template <int D>
__global__ __launch_bounds__(256) void k_ce_fwd(const float* __restrict__ E,
                                                const float* __restrict__ W,
                                                const int64_t* __restrict__ tgt, int64_t B,
                                                int64_t V, int64_t per, int64_t RB, int64_t NS, float* __restrict__ m_part,
                                                float* __restrict__ s_part,
                                                float* __restrict__ ts,
                                                unsigned* __restrict__ ticket) {
  constexpr int KH = D / 2;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0u;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
  Place pl;
  if (!place(RB, NS, pl)) return;
  const int64_t b = (pl.rb * kWaves + wave) * kTile + j;
  const int64_t bc = min(b, B - 1);
  float eb[KH];
  ld_half<KH>(eb, E + bc * D, h);
  const int64_t tb = tgt[bc];
  float m = -INFINITY, s = 0.0f, tsv = 0.0f;
  bool has_ts = false;
  stream_tiles<D, false>(W, V, per, pl.split, nullptr, nullptr,
                         [&](int64_t t, const float* tile, const float*, const int64_t*) {
    const int64_t v0 = t * kTile;
    const f32x16 x = lds_dot<D, KH, true>(tile, j, h, eb);
    const int hi = rel32(V, v0), tt = rel32(tb, v0);
    if (hi >= kTile) {
#pragma unroll
      for (int r = 0; r < 16; ++r) lse_push(m, s, x[r]);
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (crow(r, h) < hi) lse_push(m, s, x[r]);
    }
    if (tt >= 0 && tt < kTile) {   // this tile holds the row's target
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (crow(r, h) == tt) {
          tsv = x[r];
          has_ts = true;
        }
    }
  });
  if (has_ts && b < B) ts[b] = tsv;
  lse_merge(m, s, __shfl_xor(m, 32), __shfl_xor(s, 32));
  if (h == 0 && b < B) {
    m_part[pl.split * B + b] = m;
    s_part[pl.split * B + b] = s;
  }
}

// lse[b] over the S splits (a lane per row, four waves over the splits), the
// per-row loss lse - score(target) (NaN for an out-of-range target, which
// k_ce_fwd never matches), and - in the workgroup that finishes last - the
// batch mean in a fixed order.  `ticket` is zeroed by k_ce_fwd.
__global__ __launch_bounds__(256) void k_ce_rows(const float* __restrict__ m_part,
                                                 const float* __restrict__ s_part, int64_t S,
                                                 const float* __restrict__ ts,
                                                 const int64_t* __restrict__ tgt, int64_t B,
                                                 int64_t V, float* __restrict__ lse,
                                                 float* __restrict__ loss_rows,
                                                 unsigned* __restrict__ ticket,
                                                 float* __restrict__ loss) {
  // 64 rows per workgroup, one per lane; wave w merges splits w, w + 4, ...
  // in order (coalesced: a wave reads 64 consecutive rows of a split), then
  // the four waves' states merge in wave order
  __shared__ float red[256];
  __shared__ float sm[4][64], ss[4][64];
  __shared__ bool last;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * 64 + lane;
  const int64_t bc = b < B ? b : B - 1;
  float m = -INFINITY, s = 0.0f;
  for (int64_t i = w; i < S; i += 4) lse_merge(m, s, m_part[i * B + bc], s_part[i * B + bc]);
  sm[w][lane] = m;
  ss[w][lane] = s;
  __syncthreads();
  if (w == 0 && b < B) {
#pragma unroll
    for (int k = 1; k < 4; ++k) lse_merge(m, s, sm[k][lane], ss[k][lane]);
    const float l = m + logf(s);
    const int64_t t = tgt[b];
    lse[b] = l;
    loss_rows[b] = (t < 0 || t >= V) ? NAN : l - ts[b];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  float acc = 0.0f;
  for (int64_t i = threadIdx.x; i < B; i += 256) acc += loss_rows[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss[0] = red[0] / (float)B;
    *ticket = 0u;
  }
}

// ---- CE backward, dE = P W (per vocab split partials) ----------------------------
// P[b][v] = (exp(x - lse[b]) - [v == target[b]]) * dloss / B
template <int D>
__global__ __launch_bounds__(256) void k_ce_bwd_seq(const float* __restrict__ E,
                                                    const float* __restrict__ W,
                                                    const float* __restrict__ lse,
                                                    const int64_t* __restrict__ tgt,
                                                    const float* __restrict__ dloss, float inv_n,
                                                    int64_t B, int64_t V, int64_t per, int64_t RB, int64_t NS,
                                                    float* __restrict__ de_part) {
  constexpr int KH = D / 2, NT = (D + 31) / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
  Place pl;
  if (!place(RB, NS, pl)) return;
  const int64_t b0 = (pl.rb * kWaves + wave) * kTile;
  const int64_t b = min(b0 + j, B - 1);
  float eb[KH];
  ld_half<KH>(eb, E + b * D, h);
  const float lb = lse[b];
  const int64_t tb = tgt[b];
  const float g = dloss[0] * inv_n;
  f32x16 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) acc[n] = f32x16{};
  const ColReader<D> cr(j, h);
  stream_tiles<D, false>(W, V, per, pl.split, nullptr, nullptr,
                         [&](int64_t t, const float* tile, const float*, const int64_t*) {
    const int64_t v0 = t * kTile;
    const f32x16 x = lds_dot<D, KH, true>(tile, j, h, eb);
    const int hi = rel32(V, v0), tt = rel32(tb, v0);
    float p[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = crow(r, h);
      const float sm = fexp(x[r] - lb) - (c == tt ? 1.0f : 0.0f);
      p[r] = c < hi ? sm * g : 0.0f;
    }
    gemm2<D, NT>(acc, p, tile, cr, j, h);
  });
  if (b0 >= B) return;
  float* out = de_part + pl.split * B * D;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int col = n * 32 + j;
    if (col >= D) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t row = b0 + crow(r, h);
      if (row < B) out[row * D + col] = acc[n][r];
    }
  }
}

// ---- CE backward, dW = P^T E (per row split partials) ----------------------------
// Tile orientation X[b][v] (A = sequence rows from LDS, B = item rows in
// registers): lane holds item column v, so X is the A operand of P^T E.
template <int D>
__global__ __launch_bounds__(256) void k_ce_bwd_item(const float* __restrict__ E,
                                                     const float* __restrict__ W,
                                                     const float* __restrict__ lse,
                                                     const int64_t* __restrict__ tgt,
                                                     const float* __restrict__ dloss, float inv_n,
                                                     int64_t B, int64_t V, int64_t per, int64_t RB, int64_t NS,
                                                     float* __restrict__ dw_part) {
  constexpr int KH = D / 2, NT = (D + 31) / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
  Place pl;
  if (!place(RB, NS, pl)) return;
  const int64_t v0 = (pl.rb * kWaves + wave) * kTile;
  const int64_t v = v0 + j;
  float wb[KH];
  ld_half<KH>(wb, W + min(v, V - 1) * D, h);
  const float g = dloss[0] * inv_n;
  f32x16 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) acc[n] = f32x16{};
  const ColReader<D> cr(j, h);
  stream_tiles<D, true>(E, B, per, pl.split, lse, tgt,
                        [&](int64_t t, const float* tile, const float* lt, const int64_t* tt) {
    const int64_t b0 = t * kTile;
    const f32x16 x = lds_dot<D, KH, true>(tile, j, h, wb);
    const int hi = rel32(B, b0);
    float p[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = crow(r, h);
      const float sm = fexp(x[r] - lt[c]) - (v == tt[c] ? 1.0f : 0.0f);
      p[r] = c < hi ? sm * g : 0.0f;
    }
    gemm2<D, NT>(acc, p, tile, cr, j, h);
  });
  if (v0 >= V) return;
  float* out = dw_part + pl.split * V * D;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int col = n * 32 + j;
    if (col >= D) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t row = v0 + crow(r, h);
      if (row < V) out[row * D + col] = acc[n][r];
    }
  }
}

// out[i] = sum_p parts[p * n + i], p in order
__global__ __launch_bounds__(256) void k_sum_parts(const float* __restrict__ parts, int64_t P,
                                                   int64_t n, float* __restrict__ out) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= n) return;
  if (i4 + 4 <= n && (n & 3) == 0) {
    float4 acc = *reinterpret_cast<const float4*>(parts + i4);
    for (int64_t p = 1; p < P; ++p) {
      const float4 t = *reinterpret_cast<const float4*>(parts + p * n + i4);
      acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
    }
    *reinterpret_cast<float4*>(out + i4) = acc;
  } else {
    for (int64_t i = i4; i < min(i4 + 4, n); ++i) {
      float acc = parts[i];
      for (int64_t p = 1; p < P; ++p) acc += parts[p * n + i];
      out[i] = acc;
    }
  }
}

// ---- ranks: #items scoring above / equal to the target -----------------------------
template <int D>
__global__ __launch_bounds__(256) void k_item_rank(const float* __restrict__ E,
                                                   const float* __restrict__ W,
                                                   const float* __restrict__ ts,
                                                   const int64_t* __restrict__ tgt, int64_t B,
                                                   int64_t V, int64_t first, int64_t per, int64_t RB, int64_t NS,
                                                   int* __restrict__ gt_part,
                                                   int* __restrict__ eq_part) {
  constexpr int KH = D / 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
  Place pl;
  if (!place(RB, NS, pl)) return;
  const int64_t b = (pl.rb * kWaves + wave) * kTile + j;
  const int64_t bc = min(b, B - 1);
  float eb[KH];
  ld_half<KH>(eb, E + bc * D, h);
  const float tsb = ts[bc];
  const int64_t tb = tgt[bc];
  int gt = 0, eq = 0;
  stream_tiles<D, false>(W, V, per, pl.split, nullptr, nullptr,
                         [&](int64_t t, const float* tile, const float*, const int64_t*) {
    const int64_t v0 = t * kTile;
    const f32x16 x = lds_dot<D, KH, true>(tile, j, h, eb);
    const int lo = rel32(first, v0), hi = rel32(V, v0), tt = rel32(tb, v0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = crow(r, h);
      const bool ok = (c >= lo) & (c < hi) & (c != tt);
      gt += (ok & (x[r] > tsb)) ? 1 : 0;
      eq += (ok & (x[r] == tsb)) ? 1 : 0;
    }
  });
  gt += __shfl_xor(gt, 32);
  eq += __shfl_xor(eq, 32);
  if (h == 0 && b < B) {
    gt_part[pl.split * B + b] = gt;
    eq_part[pl.split * B + b] = eq;
  }
}

__global__ __launch_bounds__(256) void k_rank_rows(const int* __restrict__ gt_part,
                                                   const int* __restrict__ eq_part, int64_t S,
                                                   const float* __restrict__ ts, int64_t B,
                                                   int64_t* __restrict__ n_gt,
                                                   int64_t* __restrict__ n_eq) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  int64_t g = 0, e = 0;
  for (int64_t i = 0; i < S; ++i) {
    g += gt_part[i * B + b];
    e += eq_part[i * B + b];
  }
  const bool bad = ts[b] != ts[b];  // NaN: target id out of range
  n_gt[b] = bad ? -1 : g;
  if (n_eq) n_eq[b] = bad ? -1 : e;
}

// ---- score matrix (full_sort_predict) and CE gradient of the logits -------------
// X[b][v], lane = item column v, rows b in registers, stored as 128-B row
// segments.  kProbs: stores P[b][v] = (exp(x - lse[b]) - [v + v_off ==
// target[b]]) * dloss / B instead (the logits' gradient, consumed by two
// library GEMMs: dseq = P W, ditems = P^T seq).  out has row stride ld.
template <int D, bool kProbs>
__global__ __launch_bounds__(256) void k_item_scores(const float* __restrict__ E,
                                                     const float* __restrict__ W, int64_t B,
                                                     int64_t V, int64_t per, int64_t RB, int64_t NS,
                                                     float* __restrict__ out, int64_t ld,
                                                     const float* __restrict__ lse,
                                                     const int64_t* __restrict__ tgt,
                                                     const float* __restrict__ dloss, float inv_n,
                                                     int64_t v_off) {
  constexpr int KH = D / 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
  Place pl;
  if (!place(RB, NS, pl)) return;
  const int64_t b0 = (pl.rb * kWaves + wave) * kTile;
  float ea[KH];
  ld_half<KH>(ea, E + min(b0 + j, B - 1) * D, h);
  float lr[kProbs ? 16 : 1];
  int64_t tr[kProbs ? 16 : 1];
  float g = 0.0f;
  if constexpr (kProbs) {
    g = dloss[0] * inv_n;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t row = min(b0 + crow(r, h), B - 1);
      lr[r] = lse[row];
      tr[r] = tgt[row] - v_off;
    }
  }
  stream_tiles<D, false>(W, V, per, pl.split, nullptr, nullptr,
                         [&](int64_t t, const float* tile, const float*, const int64_t*) {
    const int64_t v = t * kTile + j;
    const f32x16 x = lds_dot<D, KH, false>(tile, j, h, ea);
    if (v < V) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = b0 + crow(r, h);
        float val = x[r];
        if constexpr (kProbs) val = (fexp(x[r] - lr[r]) - (v == tr[r] ? 1.0f : 0.0f)) * g;
        if (row < B) out[row * ld + v] = val;
      }
    }
  });
}

// ---- the f16 pipe: two-part split operands -------------------------------------
// The CE forward and the logits' gradient (the training step's two scoring
// kernels) run on v_mfma_f32_32x32x16_f16, 16x the fp32 MFMA rate, with
// fp32-level accuracy (the GEMMs' scheme, csrc/gemm_half.hip): each row x of
// seq and of the item table is scaled by an exact power of two and split,
//   x = 2^(e - kTS) (x0 + x1), x0 = f16(x 2^(kTS - e)), x1 = f16(x 2^(kTS - e) - x0),
// e the frexp exponent of max|x| (the row max lands in [2^13, 2^14)): 22
// significant bits.  A score is x0.y0 + x0.y1 + x1.y0 accumulated in fp32
// (each product exact; the dropped x1.y1 <= 2^-22 relative), un-scaled by
// v_ldexp (exact).  Image row = [x0 (D halfs) | x1 (D halfs)] = the fp32
// row's D*4 bytes, so the tile DMA and its swizzle are unchanged; the
// exponents are one int32 per row beside it.  Both kernels run the three
// products in the same order with the item parts first, so the forward's
// log-sum-exp and the gradient kernel see bit-identical logits.
// The rank / score kernels (evaluation) stay on the fp32 pipe: their target
// score replays the exact fma chain (k_target_dot).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int kTS = 14;

// one wave per row: max|x| over the row, then the two planes (4 values per
// lane and pass)
__global__ __launch_bounds__(256) void k_split_rows_h(const float* __restrict__ X, int64_t N, int D,
                                                      _Float16* __restrict__ img,
                                                      int* __restrict__ ex) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= N) return;
  const float4* x = reinterpret_cast<const float4*>(X + r * D);
  const int nq = D / 4;
  float m = 0.0f;
  for (int q = lane; q < nq; q += 64) {
    const float4 v = x[q];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  const int e = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
  _Float16* h0 = img + r * 2 * D;
  _Float16* h1 = h0 + D;
  for (int q = lane; q < nq; q += 64) {
    const float4 v = x[q];
    const float t[4] = {v.x, v.y, v.z, v.w};
    _Float16 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float sv = __builtin_amdgcn_ldexpf(t[i], kTS - e);   // exact (power of two)
      a[i] = (_Float16)sv;
      b[i] = (_Float16)(sv - (float)a[i]);
    }
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<f16x4*>(h0 + 4 * q) = f16x4{a[0], a[1], a[2], a[3]};
    *reinterpret_cast<f16x4*>(h1 + 4 * q) = f16x4{b[0], b[1], b[2], b[3]};
  }
  if (lane == 0) ex[r] = e;
}

// The same split with the 32-row group maxima of x as a side output (the
// weight-gradient GEMM's operand scales: rb_group_absmax's values, bit for
// bit): 32 rows per workgroup, a wave's 8 rows loaded together (d <= 256:
// one float4 per lane and row), the group's max over the four waves in LDS.
__global__ __launch_bounds__(256) void k_split_rows_hg(const float* __restrict__ X, int64_t N,
                                                       int D, _Float16* __restrict__ img,
                                                       int* __restrict__ ex,
                                                       float* __restrict__ gmax) {
  __shared__ float sm[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 32 + w * 8;
  const int nq = D / 4;
  const float4* x = reinterpret_cast<const float4*>(X);
  float4 v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    v[j] = (r0 + j < N && lane < nq) ? x[(r0 + j) * nq + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  float wm = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float m = fmaxf(fmaxf(fabsf(v[j].x), fabsf(v[j].y)), fmaxf(fabsf(v[j].z), fabsf(v[j].w)));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    wm = fmaxf(wm, m);
    const int64_t r = r0 + j;
    if (r < N) {
      const int e = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
      if (lane < nq) {
        const float t[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
        _Float16 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float sv = __builtin_amdgcn_ldexpf(t[i], kTS - e);
          a[i] = (_Float16)sv;
          b[i] = (_Float16)(sv - (float)a[i]);
        }
        typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
        _Float16* h0 = img + r * 2 * D;
        *reinterpret_cast<f16x4*>(h0 + 4 * lane) = f16x4{a[0], a[1], a[2], a[3]};
        *reinterpret_cast<f16x4*>(h0 + D + 4 * lane) = f16x4{b[0], b[1], b[2], b[3]};
      }
      if (lane == 0) ex[r] = e;
    }
  }
  if (lane == 0) sm[w] = wm;
  __syncthreads();
  if (threadIdx.x == 0) gmax[blockIdx.x] = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
}

// this lane's register operand: row `row` of an image, k-blocks 16s + 8h ..
// 16s + 8h + 7 of both planes (the MFMA fragment of step s)
template <int D>
__device__ __forceinline__ void ld_frag_h(f16x8 (&p0)[D / 16], f16x8 (&p1)[D / 16],
                                          const _Float16* img, int64_t row, int h) {
  const _Float16* r = img + row * 2 * D + 8 * h;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    p0[s] = *reinterpret_cast<const f16x8*>(r + 16 * s);
    p1[s] = *reinterpret_cast<const f16x8*>(r + D + 16 * s);
  }
}

// X = items . seq over the full depth, item row j's fragments from the
// swizzled LDS image tile, the other operand's from registers (kTileIsA:
// the tile supplies A — rows of X are items — else B).  Per k16 step the
// three products item1.seq0, item0.seq1, item0.seq0, in that order in both
// orientations.  The tile reads run one step ahead of the MFMAs.
template <int D, bool kTileIsA>
__device__ __forceinline__ f32x16 lds_dot_h(const float* tile, int j, int h, const f16x8 (&r0)[D / 16],
                                            const f16x8 (&r1)[D / 16]) {
  constexpr int KS = D / 16;
  const float* row = tile + j * D;
  int sw = j % Stream<D>::NS;
  asm volatile("" : "+v"(sw));
  auto rd = [&](int slot) {
    return __builtin_bit_cast(f16x8, *reinterpret_cast<const float4*>(row + ((slot ^ sw) << 2)));
  };
  f16x8 w0[KS], w1[KS];
  w0[0] = rd(h);
  w1[0] = rd(D / 8 + h);
  f32x16 acc = {};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (s + 1 < KS) {
      w0[s + 1] = rd(2 * (s + 1) + h);
      w1[s + 1] = rd(D / 8 + 2 * (s + 1) + h);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (kTileIsA) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w1[s], r0[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w0[s], r1[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w0[s], r0[s], acc, 0, 0, 0);
    } else {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(r0[s], w1[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(r1[s], w0[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(r0[s], w0[s], acc, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

// k_ce_fwd on the f16 pipe: the same tiles, partials and target capture;
// the item exponents of each tile ride along in LDS (rows crow(r, h): four
// 16-B reads)
template <int D>
__global__ __launch_bounds__(256) void k_ce_fwd_h(const _Float16* __restrict__ Ei,
                                                  const int* __restrict__ Ee,
                                                  const _Float16* __restrict__ Wi,
                                                  const int* __restrict__ We,
                                                  const int64_t* __restrict__ tgt, int64_t B,
                                                  int64_t V, int64_t per, int64_t RB, int64_t NS,
                                                  float* __restrict__ m_part,
                                                  float* __restrict__ s_part,
                                                  float* __restrict__ ts,
                                                  unsigned* __restrict__ ticket) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0u;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
  Place pl;
  if (!place(RB, NS, pl)) return;
  const int64_t b = (pl.rb * kWaves + wave) * kTile + j;
  const int64_t bc = min(b, B - 1);
  f16x8 e0[D / 16], e1[D / 16];
  ld_frag_h<D>(e0, e1, Ei, bc, h);
  const int eb = Ee[bc] - 2 * kTS;
  const int64_t tb = tgt[bc];
  float m = -INFINITY, s = 0.0f, tsv = 0.0f;
  bool has_ts = false;
  stream_tiles<D, 2>(reinterpret_cast<const float*>(Wi), V, per, pl.split,
                     reinterpret_cast<const float*>(We), nullptr,
                     [&](int64_t t, const float* tile, const float* ebuf, const int64_t*) {
    const int64_t v0 = t * kTile;
    f32x16 x = lds_dot_h<D, true>(tile, j, h, e0, e1);
    const int4* ev = reinterpret_cast<const int4*>(ebuf);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int4 q = ev[2 * g + h];   // items 8g + 4h .. 8g + 4h + 3 = rows crow(4g .. 4g + 3, h)
      x[4 * g] = __builtin_amdgcn_ldexpf(x[4 * g], q.x + eb);
      x[4 * g + 1] = __builtin_amdgcn_ldexpf(x[4 * g + 1], q.y + eb);
      x[4 * g + 2] = __builtin_amdgcn_ldexpf(x[4 * g + 2], q.z + eb);
      x[4 * g + 3] = __builtin_amdgcn_ldexpf(x[4 * g + 3], q.w + eb);
    }
    const int hi = rel32(V, v0), tt = rel32(tb, v0);
    if (hi >= kTile) {
#pragma unroll
      for (int r = 0; r < 16; ++r) lse_push(m, s, x[r]);
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (crow(r, h) < hi) lse_push(m, s, x[r]);
    }
    if (tt >= 0 && tt < kTile) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (crow(r, h) == tt) {
          tsv = x[r];
          has_ts = true;
        }
    }
  });
  if (has_ts && b < B) ts[b] = tsv;
  lse_merge(m, s, __shfl_xor(m, 32), __shfl_xor(s, 32));
  if (h == 0 && b < B) {
    m_part[pl.split * B + b] = m;
    s_part[pl.split * B + b] = s;
  }
}

// k_item_scores<D, true> on the f16 pipe (the logits' gradient P): seq rows
// in registers (A), item tiles streamed (B) with their exponents.  TR: P^T
// [V, ld] instead (each lane's 16 rows as four 16-B pieces of its item's
// row) and every 32-item group's max |P| (atomicMax into gmax, zeroed by the
// caller): the operands of the input gradients as f16x3 GEMMs
// (scoring._bwd_slices).  MODE 0: P; 1: P^T + gmax; 2: both layouts (P into
// out2 [B, ld2]), gmax and every 32-row group's max |P| (bmax, atomicMax) —
// the operands of both input gradients as rb_gemm_tn_h products
// (scoring._bwd_f16).
template <int D, int MODE>
__global__ __launch_bounds__(256) void k_ce_probs_h(const _Float16* __restrict__ Ei,
                                                    const int* __restrict__ Ee,
                                                    const _Float16* __restrict__ Wi,
                                                    const int* __restrict__ We, int64_t B,
                                                    int64_t V, int64_t per, int64_t RB, int64_t NS,
                                                    float* __restrict__ out, int64_t ld,
                                                    const float* __restrict__ lse,
                                                    const int64_t* __restrict__ tgt,
                                                    const float* __restrict__ dloss, float inv_n,
                                                    int64_t v_off, float* __restrict__ gmax,
                                                    float* __restrict__ out2, int64_t ld2,
                                                    float* __restrict__ bmax) {
  constexpr bool TR = MODE != 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
  Place pl;
  if (!place(RB, NS, pl)) return;
  const int64_t b0 = (pl.rb * kWaves + wave) * kTile;
  f16x8 e0[D / 16], e1[D / 16];
  ld_frag_h<D>(e0, e1, Ei, min(b0 + j, B - 1), h);
  // per output row (registers r): lse, the target's column in this slice
  // (-1 outside it; V < 2^31) and the row's exponent — 48 registers, int32
  // where possible so two waves fit per SIMD
  float lr[16];
  int tr[16], er[16];
  const float g = dloss[0] * inv_n;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t row = min(b0 + crow(r, h), B - 1);
    lr[r] = lse[row];
    const int64_t tv = tgt[row] - v_off;
    tr[r] = (tv >= 0 && tv < V) ? (int)tv : -1;
    er[r] = Ee[row] - 2 * kTS;
  }
  const bool full = b0 + kTile <= B;
  float mb = 0.0f;   // MODE 2: max |P| over the wave's rows and tiles
  stream_tiles<D, 2>(reinterpret_cast<const float*>(Wi), V, per, pl.split,
                     reinterpret_cast<const float*>(We), nullptr,
                     [&](int64_t t, const float* tile, const float* ebuf, const int64_t*) {
    const int v = (int)(t * kTile) + j;
    const f32x16 x = lds_dot_h<D, false>(tile, j, h, e0, e1);
    const int ev = reinterpret_cast<const int*>(ebuf)[j];
    if constexpr (!TR) {
      if (v < V) {
        float* o = out + (b0 + 4 * h) * ld + v;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = crow(r, 0);   // row - b0 - 4h
          const float xs = __builtin_amdgcn_ldexpf(x[r], ev + er[r]);
          const float val = (fexp(xs - lr[r]) - (v == tr[r] ? 1.0f : 0.0f)) * g;
          if (full || b0 + 4 * h + rr < B) o[rr * ld] = val;
        }
      }
    } else {
      float m = 0.0f;
      if (v < V) {
        float* o = out + (int64_t)v * ld + b0 + 4 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // rows b0 + 8q + 4h + 0..3
          rb_f32x4 val4;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = 4 * q + u;
            const float xs = __builtin_amdgcn_ldexpf(x[r], ev + er[r]);
            const bool in = full || b0 + 8 * q + 4 * h + u < B;
            val4[u] = in ? (fexp(xs - lr[r]) - (v == tr[r] ? 1.0f : 0.0f)) * g : 0.0f;
            m = fmaxf(m, fabsf(val4[u]));
          }
          if (full) {
            *reinterpret_cast<rb_f32x4*>(o + 8 * q) = val4;
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (b0 + 8 * q + 4 * h + u < B) o[8 * q + u] = val4[u];
          }
          if constexpr (MODE == 2) {   // the same values row-major: out2[b][v]
            float* o2 = out2 + (b0 + 8 * q + 4 * h) * ld2 + v;
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (full || b0 + 8 * q + 4 * h + u < B) o2[u * ld2] = val4[u];
          }
        }
      }
      if constexpr (MODE == 2) mb = fmaxf(mb, m);
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) m = fmaxf(m, __shfl_xor(m, sh));
      if (lane == 0)   // non-negative floats order as their bit patterns
        atomicMax(reinterpret_cast<int*>(gmax) + t, __float_as_int(m));
    }
  });
  if constexpr (MODE == 2) {
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) mb = fmaxf(mb, __shfl_xor(mb, sh));
    if (lane == 0 && b0 < B) atomicMax(reinterpret_cast<int*>(bmax) + b0 / kTile, __float_as_int(mb));
    // out2's padding columns [V, ld2) of the wave's rows: zeros (the first
    // item split's workgroups; no separate fill launch)
    if (pl.split == 0 && ld2 > V) {
      for (int r = 0; r < kTile && b0 + r < B; ++r)
        for (int64_t v = V + lane; v < ld2; v += 64) out2[(b0 + r) * ld2 + v] = 0.0f;
    }
  }
}

// ---- host side ---------------------------------------------------------------------
size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

struct Grid2 {
  int64_t blocks, splits, per;  // blocks over the fixed axis, splits of the streamed axis
  unsigned wgs() const { return (unsigned)(blocks * ((splits + 7) / 8 * 8)); }  // see place()
};

// fixed axis: n_fixed rows (kWaves*kTile per workgroup); streamed axis: n_stream tiles
Grid2 plan(int64_t n_fixed, int64_t n_stream_tiles) {
  const int64_t blocks = (n_fixed + kWaves * kTile - 1) / (kWaves * kTile);
  int64_t s = (kTargetWgs + blocks - 1) / blocks;
  s = std::max<int64_t>(1, std::min<int64_t>(s, n_stream_tiles));
  const int64_t per = (n_stream_tiles + s - 1) / s;
  return {blocks, (n_stream_tiles + per - 1) / per, per};
}

int64_t ntiles(int64_t n) { return (n + kTile - 1) / kTile; }

struct CeWs {
  size_t ts, m, s, rows, ticket, de, dw, total;
};

CeWs ce_layout(int64_t B, int64_t V, int64_t D) {
  const Grid2 f = plan(B, ntiles(V)), w = plan(V, ntiles(B));
  CeWs o{};
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t r = off; off = al256(off + bytes); return r; };
  o.ts = take(B * 4);
  o.m = take(f.splits * B * 4);
  o.s = take(f.splits * B * 4);
  o.rows = take(B * 4);
  o.ticket = take(4);
  o.de = take(f.splits * B * D * 4);
  o.dw = take(w.splits * V * D * 4);
  o.total = off;
  return o;
}

struct RankWs {
  size_t ts, gt, eq, total;
};

RankWs rank_layout(int64_t B, int64_t V) {
  const Grid2 f = plan(B, ntiles(V));
  RankWs o{};
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t r = off; off = al256(off + bytes); return r; };
  o.ts = take(B * 4);
  o.gt = take(f.splits * B * 4);
  o.eq = take(f.splits * B * 4);
  o.total = off;
  return o;
}

#define RB_ITEM_DISPATCH(D, FN, ...)              \
  switch (D) {                                    \
    case 16: FN<16>(__VA_ARGS__); break;          \
    case 32: FN<32>(__VA_ARGS__); break;          \
    case 64: FN<64>(__VA_ARGS__); break;          \
    case 128: FN<128>(__VA_ARGS__); break;        \
    case 256: FN<256>(__VA_ARGS__); break;        \
    default: return fail("item scores: d must be 16, 32, 64, 128 or 256"); \
  }

template <int D>
void target_dot_t(const float* E, const float* W, const int64_t* tgt, int64_t B, int64_t V,
                  float* ts, hipStream_t st) {
  hipLaunchKernelGGL(k_target_dot<D>, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, E, W,
                     tgt, B, V, ts);
}

template <int D>
void ce_fwd_t(const float* E, const float* W, const int64_t* tgt, int64_t B, int64_t V,
              const Grid2& g, float* m, float* s, float* ts, unsigned* ticket, hipStream_t st) {
  hipLaunchKernelGGL(k_ce_fwd<D>, dim3(g.wgs()), dim3(256), 0, st,
                     E, W, tgt, B, V, g.per, g.blocks, g.splits, m, s, ts, ticket);
}

template <int D>
void ce_bwd_seq_t(const float* E, const float* W, const float* lse, const int64_t* tgt,
                  const float* dloss, float inv_n, int64_t B, int64_t V, const Grid2& g,
                  float* part, hipStream_t st) {
  hipLaunchKernelGGL(k_ce_bwd_seq<D>, dim3(g.wgs()), dim3(256), 0,
                     st, E, W, lse, tgt, dloss, inv_n, B, V, g.per, g.blocks, g.splits, part);
}

template <int D>
void ce_bwd_item_t(const float* E, const float* W, const float* lse, const int64_t* tgt,
                   const float* dloss, float inv_n, int64_t B, int64_t V, const Grid2& g,
                   float* part, hipStream_t st) {
  hipLaunchKernelGGL(k_ce_bwd_item<D>, dim3(g.wgs()), dim3(256), 0,
                     st, E, W, lse, tgt, dloss, inv_n, B, V, g.per, g.blocks, g.splits, part);
}

template <int D>
void rank_t(const float* E, const float* W, const float* ts, const int64_t* tgt, int64_t B,
            int64_t V, int64_t first, const Grid2& g, int* gt, int* eq, hipStream_t st) {
  hipLaunchKernelGGL(k_item_rank<D>, dim3(g.wgs()), dim3(256), 0,
                     st, E, W, ts, tgt, B, V, first, g.per, g.blocks, g.splits, gt, eq);
}

template <int D>
void scores_t(const float* E, const float* W, int64_t B, int64_t V, const Grid2& g, float* out,
              hipStream_t st) {
  hipLaunchKernelGGL((k_item_scores<D, false>), dim3(g.wgs()), dim3(256), 0, st, E, W, B, V, g.per,
                     g.blocks, g.splits, out, V, nullptr, nullptr, nullptr, 0.0f, (int64_t)0);
}

template <int D>
void probs_t(const float* E, const float* W, int64_t B, int64_t V, const Grid2& g, float* out,
             int64_t ld, const float* lse, const int64_t* tgt, const float* dloss, float inv_n,
             int64_t v_off, hipStream_t st) {
  hipLaunchKernelGGL((k_item_scores<D, true>), dim3(g.wgs()), dim3(256), 0, st, E, W, B, V, g.per,
                     g.blocks, g.splits, out, ld, lse, tgt, dloss, inv_n, v_off);
}

template <int D>
void ce_fwd_h_t(const void* Ei, const int* Ee, const void* Wi, const int* We, const int64_t* tgt,
                int64_t B, int64_t V, const Grid2& g, float* m, float* s, float* ts,
                unsigned* ticket, hipStream_t st) {
  hipLaunchKernelGGL(k_ce_fwd_h<D>, dim3(g.wgs()), dim3(256), 0, st, (const _Float16*)Ei, Ee,
                     (const _Float16*)Wi, We, tgt, B, V, g.per, g.blocks, g.splits, m, s, ts,
                     ticket);
}

template <int D>
void probs_h_t(const void* Ei, const int* Ee, const void* Wi, const int* We, int64_t B, int64_t V,
               const Grid2& g, float* out, int64_t ld, const float* lse, const int64_t* tgt,
               const float* dloss, float inv_n, int64_t v_off, float* gmax, float* out2,
               int64_t ld2, float* bmax, hipStream_t st) {
  if (out2)
    hipLaunchKernelGGL((k_ce_probs_h<D, 2>), dim3(g.wgs()), dim3(256), 0, st,
                       (const _Float16*)Ei, Ee, (const _Float16*)Wi, We, B, V, g.per, g.blocks,
                       g.splits, out, ld, lse, tgt, dloss, inv_n, v_off, gmax, out2, ld2, bmax);
  else if (gmax)
    hipLaunchKernelGGL((k_ce_probs_h<D, 1>), dim3(g.wgs()), dim3(256), 0, st,
                       (const _Float16*)Ei, Ee, (const _Float16*)Wi, We, B, V, g.per, g.blocks,
                       g.splits, out, ld, lse, tgt, dloss, inv_n, v_off, gmax, nullptr,
                       (int64_t)0, nullptr);
  else
    hipLaunchKernelGGL((k_ce_probs_h<D, 0>), dim3(g.wgs()), dim3(256), 0, st,
                       (const _Float16*)Ei, Ee, (const _Float16*)Wi, We, B, V, g.per, g.blocks,
                       g.splits, out, ld, lse, tgt, dloss, inv_n, v_off, gmax, nullptr,
                       (int64_t)0, nullptr);
}

void sum_parts(const float* parts, int64_t P, int64_t n, float* out, hipStream_t st) {
  const int64_t threads = (n + 3) / 4;
  hipLaunchKernelGGL(k_sum_parts, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, parts,
                     P, n, out);
}

}  // namespace

int64_t item_ce_workspace_bytes(int64_t B, int64_t V, int64_t D) {
  return (int64_t)ce_layout(B, V, D).total;
}

int64_t item_rank_workspace_bytes(int64_t B, int64_t V) {
  return (int64_t)rank_layout(B, V).total;
}

int launch_item_ce_fwd(const float* E, const float* W, const int64_t* tgt, int64_t B, int64_t V,
                       int64_t D, float* lse, float* loss, void* ws, int64_t ws_bytes,
                       hipStream_t st) {
  const CeWs L = ce_layout(B, V, D);
  if (ws_bytes < (int64_t)L.total) return fail("rb_item_ce_fwd: workspace too small");
  char* w = static_cast<char*>(ws);
  float* ts = reinterpret_cast<float*>(w + L.ts);
  float* m = reinterpret_cast<float*>(w + L.m);
  float* s = reinterpret_cast<float*>(w + L.s);
  float* rows = reinterpret_cast<float*>(w + L.rows);
  const Grid2 g = plan(B, ntiles(V));
  unsigned* ticket = reinterpret_cast<unsigned*>(w + L.ticket);
  RB_ITEM_DISPATCH(D, ce_fwd_t, E, W, tgt, B, V, g, m, s, ts, ticket, st);
  hipLaunchKernelGGL(k_ce_rows, dim3((unsigned)((B + 63) / 64)), dim3(256), 0, st, m,
                     s, g.splits, ts, tgt, B, V, lse, rows, ticket, loss);
  return launch_status("rb_item_ce_fwd");
}

int launch_item_ce_bwd(const float* E, const float* W, const int64_t* tgt, const float* lse,
                       const float* dloss, int64_t B, int64_t V, int64_t D, float* dE, float* dW,
                       void* ws, int64_t ws_bytes, hipStream_t st) {
  const CeWs L = ce_layout(B, V, D);
  if (ws_bytes < (int64_t)L.total) return fail("rb_item_ce_bwd: workspace too small");
  char* w = static_cast<char*>(ws);
  const float inv_n = 1.0f / (float)B;
  if (dE) {
    float* part = reinterpret_cast<float*>(w + L.de);
    const Grid2 g = plan(B, ntiles(V));
    RB_ITEM_DISPATCH(D, ce_bwd_seq_t, E, W, lse, tgt, dloss, inv_n, B, V, g, part, st);
    sum_parts(part, g.splits, B * D, dE, st);
  }
  if (dW) {
    float* part = reinterpret_cast<float*>(w + L.dw);
    const Grid2 g = plan(V, ntiles(B));
    RB_ITEM_DISPATCH(D, ce_bwd_item_t, E, W, lse, tgt, dloss, inv_n, B, V, g, part, st);
    sum_parts(part, g.splits, V * D, dW, st);
  }
  return launch_status("rb_item_ce_bwd");
}

int launch_item_rank(const float* E, const float* W, const int64_t* tgt, int64_t B, int64_t V,
                     int64_t D, int64_t first, int64_t* n_gt, int64_t* n_eq, void* ws,
                     int64_t ws_bytes, hipStream_t st) {
  const RankWs L = rank_layout(B, V);
  if (ws_bytes < (int64_t)L.total) return fail("rb_item_rank: workspace too small");
  char* w = static_cast<char*>(ws);
  float* ts = reinterpret_cast<float*>(w + L.ts);
  int* gt = reinterpret_cast<int*>(w + L.gt);
  int* eq = reinterpret_cast<int*>(w + L.eq);
  const Grid2 g = plan(B, ntiles(V));
  RB_ITEM_DISPATCH(D, target_dot_t, E, W, tgt, B, V, ts, st);
  RB_ITEM_DISPATCH(D, rank_t, E, W, ts, tgt, B, V, first, g, gt, eq, st);
  hipLaunchKernelGGL(k_rank_rows, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, gt, eq,
                     g.splits, ts, B, n_gt, n_eq);
  return launch_status("rb_item_rank");
}

int launch_item_ce_probs(const float* E, const float* W, const int64_t* tgt, const float* lse,
                         const float* dloss, int64_t B, int64_t V, int64_t D, int64_t v_off,
                         int64_t n_total, float* out, int64_t ld, hipStream_t st) {
  const Grid2 g = plan(B, ntiles(V));
  const float inv_n = 1.0f / (float)B;
  (void)n_total;
  RB_ITEM_DISPATCH(D, probs_t, E, W, B, V, g, out, ld, lse, tgt, dloss, inv_n, v_off, st);
  return launch_status("rb_item_ce_probs");
}

int launch_item_split_h(const float* X, int64_t N, int64_t D, void* img, int* ex, float* gmax,
                        hipStream_t st) {
  if (gmax != nullptr) {
    hipLaunchKernelGGL(k_split_rows_hg, dim3((unsigned)((N + 31) / 32)), dim3(256), 0, st, X, N,
                       (int)D, (_Float16*)img, ex, gmax);
    return launch_status("rb_item_split_h");
  }
  hipLaunchKernelGGL(k_split_rows_h, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, X, N, (int)D,
                     (_Float16*)img, ex);
  return launch_status("rb_item_split_h");
}

int launch_item_ce_fwd_h(const void* Ei, const int* Ee, const void* Wi, const int* We,
                         const int64_t* tgt, int64_t B, int64_t V, int64_t D, float* lse,
                         float* loss, void* ws, int64_t ws_bytes, hipStream_t st) {
  const CeWs L = ce_layout(B, V, D);
  if (ws_bytes < (int64_t)L.total) return fail("rb_item_ce_fwd_h: workspace too small");
  char* w = static_cast<char*>(ws);
  float* ts = reinterpret_cast<float*>(w + L.ts);
  float* m = reinterpret_cast<float*>(w + L.m);
  float* s = reinterpret_cast<float*>(w + L.s);
  float* rows = reinterpret_cast<float*>(w + L.rows);
  const Grid2 g = plan(B, ntiles(V));
  unsigned* ticket = reinterpret_cast<unsigned*>(w + L.ticket);
  RB_ITEM_DISPATCH(D, ce_fwd_h_t, Ei, Ee, Wi, We, tgt, B, V, g, m, s, ts, ticket, st);
  hipLaunchKernelGGL(k_ce_rows, dim3((unsigned)((B + 63) / 64)), dim3(256), 0, st, m,
                     s, g.splits, ts, tgt, B, V, lse, rows, ticket, loss);
  return launch_status("rb_item_ce_fwd_h");
}

int launch_item_ce_probs_h(const void* Ei, const int* Ee, const void* Wi, const int* We,
                           const int64_t* tgt, const float* lse, const float* dloss, int64_t B,
                           int64_t V, int64_t D, int64_t v_off, float* out, int64_t ld,
                           float* gmax, float* out2, int64_t ld2, float* bmax, hipStream_t st) {
  const Grid2 g = plan(B, ntiles(V));
  const float inv_n = 1.0f / (float)B;
  RB_ITEM_DISPATCH(D, probs_h_t, Ei, Ee, Wi, We, B, V, g, out, ld, lse, tgt, dloss, inv_n, v_off,
                   gmax, out2, ld2, bmax, st);
  return launch_status(out2 ? "rb_item_ce_probs_h_both"
                            : gmax ? "rb_item_ce_probs_h_t" : "rb_item_ce_probs_h");
}

int launch_item_scores(const float* E, const float* W, int64_t B, int64_t V, int64_t D,
                       float* out, hipStream_t st) {
  const Grid2 g = plan(B, ntiles(V));
  RB_ITEM_DISPATCH(D, scores_t, E, W, B, V, g, out, st);
  return launch_status("rb_item_scores");
}

}  // namespace rb
