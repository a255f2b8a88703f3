// embedding.hip — deterministic scatter-add backward of the item embedding
// gather (reference RecBLR.py:76, nn.Embedding(n_items, d, padding_idx=0)).
//
//   dW[v] = sum over positions p with idx[p] == v of grad[p]   (dW[pad] = 0)
//
// torch sorts the indices and runs a segmented reduction whose sum_and_scatter
// kernel took ~4.8 ms per training step at B=2048 L=200 d=128.  Here:
//   1. vals = the positions grouped by key, in position order inside every
//      key (a stable counting sort, three launches, for V <= kPlanMaxKeys:
//      256 row blocks count their keys in LDS; one thread per key scans
//      its counts over the blocks, and the last workgroup to finish turns
//      the key totals into the key segments seg[v], the chunk offsets and
//      descriptors; each block places its positions, ranks inside a wave
//      from ballots over the key bits; larger V: rocPRIM's stable radix
//      sort, a binary search for seg and a scan for the chunks — 15
//      launches);
//   2. seg[v] = first slot of key v, v in [0, V];
//   3. every key's run is cut into chunks of kChunk rows (long runs of very
//      popular items are spread over many waves); chunk offsets by a scan;
//   4. one wave per chunk sums its rows in a fixed order (its key and rows
//      from a chunk descriptor planned with the sort); single-chunk keys
//      write dW directly, the rest write a partial;
//   5. one wave per multi-chunk key adds its partials in chunk order.
// Every sum has a fixed order, so the result is bitwise reproducible, and no
// float atomics are used.
#include "common.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

namespace rb {
namespace {

constexpr int kChunk = 64;
constexpr unsigned kEmbMergeLimit = 0;   // rocPRIM's default: 1 << 20

__global__ void k_emb_prep(const int64_t* __restrict__ idx, int* __restrict__ keys,
                           int* __restrict__ vals, int64_t M) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M;
       i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = (int)idx[i];
    vals[i] = (int)i;
  }
}

// seg[v] = first sorted position with key >= v, v in [0, V]; keys outside
// [0, V) fall outside every segment and are ignored (never dereferenced)
__global__ void k_emb_segments(const int* __restrict__ keys, int64_t M, int V,
                               int* __restrict__ seg) {
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v <= V; v += gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = M;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < v) lo = mid + 1; else hi = mid;
    }
    seg[v] = (int)lo;
  }
}

// nch[v] = chunks of key v for v < V, nch[V] = 0 (so the scan's last entry is the total)
__global__ void k_emb_chunks(const int* __restrict__ seg, int V, int* __restrict__ nch) {
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v <= V; v += gridDim.x * blockDim.x) {
    const int n = v < V ? seg[v + 1] - seg[v] : 0;
    nch[v] = (n + kChunk - 1) / kChunk;
  }
}

// One wave per chunk.  choff = exclusive scan of nch (choff[V] = total).
template <int NV>
__global__ void __launch_bounds__(256)
k_emb_chunk_sum(const int* __restrict__ vals, const int* __restrict__ seg,
                const int* __restrict__ nch, const int* __restrict__ choff,
                const float* __restrict__ grad, int d, int V, int padding_idx,
                float* __restrict__ dw, float* __restrict__ partial) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int total = choff[V];
  if (c >= total) return;
  // key owning chunk c: last v with choff[v] <= c
  int lo = 0, hi = V;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (choff[mid] <= c) lo = mid; else hi = mid;
  }
  const int v = lo;
  if (v == padding_idx) return;   // its row is zeroed by k_emb_finish
  const int ci = (int)(c - choff[v]);
  const int beg = seg[v] + ci * kChunk;
  const int end = min(seg[v + 1], beg + kChunk);
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.0f;
  int j = beg;
  for (; j + 4 <= end; j += 4) {   // 4 rows in flight
    int p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) p[u] = vals[j + u];
    float x[4][NV];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int col = lane + k * kWave;
        x[u][k] = col < d ? grad[(int64_t)p[u] * d + col] : 0.0f;
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < NV; ++k) acc[k] += x[u][k];
  }
  for (; j < end; ++j) {
    const int p = vals[j];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int col = lane + k * kWave;
      acc[k] += col < d ? grad[(int64_t)p * d + col] : 0.0f;
    }
  }
  float* out = nch[v] == 1 ? dw + (int64_t)v * d : partial + c * d;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int col = lane + k * kWave;
    if (col < d) out[col] = acc[k];
  }
}

// desc[c] = {key, first row, end row, single-chunk key} of chunk c, planned
// on the side stream with the sort: the apply kernel needs one 16-B load to
// place its chunk (instead of a 14-step dependent binary search over choff)
__global__ void k_emb_chunk_desc(const int* __restrict__ seg, const int* __restrict__ nch,
                                 const int* __restrict__ choff, int V, int4* __restrict__ desc) {
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x) {
    const int n = nch[v], o = choff[v], s0 = seg[v], s1 = seg[v + 1];
    for (int i = 0; i < n; ++i)
      desc[o + i] = make_int4(v, s0 + i * kChunk, min(s1, s0 + (i + 1) * kChunk), n == 1);
  }
}

// The apply kernel for 16-B aligned rows (d % 4 == 0): one wave per chunk of
// <= 64 rows.  Three dependent steps only: the chunk descriptor, the chunk's
// row ids (one per lane, one load), then every row of the chunk at once — the
// two half-waves take alternate rows (512 B of a row per instruction, 16 B
// per lane), 16 rows per half-wave in flight.  Each half sums its rows in
// position order and the halves are added (even rows + odd rows): a fixed
// order, bitwise reproducible.
template <int NV4>
__global__ void __launch_bounds__(256)
k_emb_chunk_sum4(const int* __restrict__ vals, const int* __restrict__ choff,
                 const int4* __restrict__ desc, const float* __restrict__ grad, int d, int V,
                 int padding_idx, float* __restrict__ dw, float* __restrict__ partial) {
  const int lane = threadIdx.x & (kWave - 1);
  const int hw = lane >> 5, l32 = lane & 31;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int total = choff[V];
  const int4 dc = desc[c < total ? c : 0];
  if (c >= total || dc.x == padding_idx) return;   // the padding row: zeroed by k_emb_finish
  const int beg = dc.y, n = dc.z - dc.y;
  const int pv = lane < n ? vals[beg + lane] : 0;
  const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  float4 acc[NV4];
#pragma unroll
  for (int k = 0; k < NV4; ++k) acc[k] = zero;
  for (int r0 = 0; r0 < n; r0 += 32) {
    float4 x[16][NV4];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int r = r0 + 2 * u + hw;
      const int p = __shfl(pv, r & 63);
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        const int col = 4 * (l32 + 32 * k);
        x[u][k] = (r < n && col < d) ? *reinterpret_cast<const float4*>(grad + (int64_t)p * d + col)
                                     : zero;
      }
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        acc[k].x += x[u][k].x; acc[k].y += x[u][k].y;
        acc[k].z += x[u][k].z; acc[k].w += x[u][k].w;
      }
  }
  float* out = dc.w ? dw + (int64_t)dc.x * d : partial + c * d;
#pragma unroll
  for (int k = 0; k < NV4; ++k) {
    float4 t = acc[k];
    t.x += __shfl_xor(t.x, 32); t.y += __shfl_xor(t.y, 32);
    t.z += __shfl_xor(t.z, 32); t.w += __shfl_xor(t.w, 32);
    const int col = 4 * (l32 + 32 * k);
    if (hw == 0 && col < d) *reinterpret_cast<float4*>(out + col) = t;
  }
}

// One 4-wave block per key: keys with no rows (and the padding id) get zeros;
// multi-chunk keys sum their partials, wave w taking chunks w, w+4, ... and
// the four wave sums combined in a fixed order (bitwise reproducible).
template <int NV>
__global__ void __launch_bounds__(256)
k_emb_finish(const int* __restrict__ nch, const int* __restrict__ choff,
             const float* __restrict__ partial, int d, int V, int padding_idx,
             float* __restrict__ dw) {
  __shared__ float red[4][NV * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  const int v = blockIdx.x;
  const int n = v == padding_idx ? 0 : nch[v];
  if (n == 1) return;   // written by k_emb_chunk_sum
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.0f;
  const int c0 = choff[v];
  for (int c = c0 + wv; c < c0 + n; c += 4)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int col = lane + k * kWave;
      acc[k] += col < d ? partial[(int64_t)c * d + col] : 0.0f;
    }
#pragma unroll
  for (int k = 0; k < NV; ++k) red[wv][lane + k * kWave] = acc[k];
  __syncthreads();
  for (int col = threadIdx.x; col < d; col += blockDim.x)
    dw[(int64_t)v * d + col] = ((red[0][col] + red[1][col]) + red[2][col]) + red[3][col];
}

// ---- the counting-sort plan (V <= kPlanMaxKeys) -----------------------------------
constexpr int kPlanBlocks = 256;       // T: row blocks of the counting sort
constexpr int kPlanMaxKeys = 16384;    // LDS key counters (64 KB)

// cnt[t * V + v] = positions of block t (rows [t*per, (t+1)*per)) with key v
// (block-major: each block writes its V counts contiguously)
__global__ void __launch_bounds__(1024) k_emb_hist(const int64_t* __restrict__ idx, int64_t M,
                                                   int V, int64_t per, int* __restrict__ cnt,
                                                   unsigned* __restrict__ ticket) {
  __shared__ int h[kPlanMaxKeys];
  if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0u;   // k_emb_keys' arrival count
  for (int v = threadIdx.x; v < V; v += blockDim.x) h[v] = 0;
  __syncthreads();
  const int64_t beg = (int64_t)blockIdx.x * per, end = min(M, beg + per);
  for (int64_t i = beg + threadIdx.x; i < end; i += blockDim.x) {
    const int64_t k = idx[i];
    if (k >= 0 && k < V) atomicAdd(&h[k], 1);   // integer counts: order-independent
  }
  __syncthreads();
  int* row = cnt + (int64_t)blockIdx.x * V;
  for (int v = threadIdx.x; v < V; v += blockDim.x) row[v] = h[v];
}

// exclusive workgroup-wide scan (1024 threads, one value each); *total = sum
__device__ int block_scan_excl(int x, int* sh, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  if (w == 0) {
    int s = lane < 16 ? sh[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(s, o);
      if (lane >= o) s += y;
    }
    if (lane < 16) sh[16 + lane] = s;
  }
  __syncthreads();
  const int before = w ? sh[16 + w - 1] : 0;
  *total = sh[16 + 15];
  __syncthreads();
  return before + incl - x;
}

// The last workgroup (1024 threads): seg, nch, choff (exclusive scans over the keys, in key
// order) and the chunk descriptors; thread j owns keys [j*kpt, (j+1)*kpt)
__device__ void emb_offsets(const int* __restrict__ tot, int V, int* __restrict__ seg,
                            int* __restrict__ nch, int* __restrict__ choff,
                            int4* __restrict__ desc, int* ts, int* sh) {
  for (int v = threadIdx.x; v < V; v += 1024) ts[v] = tot[v];
  __syncthreads();
  const int kpt = (V + 1023) / 1024;
  const int v0 = threadIdx.x * kpt, v1 = min(V, v0 + kpt);
  int sum = 0, chs = 0;
  for (int v = v0; v < v1; ++v) {
    const int s = ts[v];
    sum += s;
    chs += (s + kChunk - 1) / kChunk;
  }
  int all, all_ch;
  int pos = block_scan_excl(sum, sh, &all);
  int cpos = block_scan_excl(chs, sh, &all_ch);
  for (int v = v0; v < v1; ++v) {
    const int s = ts[v];
    const int n = (s + kChunk - 1) / kChunk;
    seg[v] = pos;
    nch[v] = n;
    choff[v] = cpos;
    for (int i = 0; i < n; ++i)
      desc[cpos + i] = make_int4(v, pos + i * kChunk, min(pos + s, pos + (i + 1) * kChunk), n == 1);
    pos += s;
    cpos += n;
  }
  if (threadIdx.x == 0) {
    seg[V] = all;
    nch[V] = 0;
    choff[V] = all_ch;
  }
}

// cnt[t][v] becomes the exclusive prefix over the blocks (in block order),
// tot[v] the key's count.  64 keys per 1024-thread workgroup: thread (key j =
// tid & 63, block group q = tid >> 6) loads its key's counts of blocks
// 16q .. 16q + 15 (a wave reads 64 consecutive keys of one block per load,
// all 16 loads in flight), the 16 group totals of each key are combined
// through LDS in block order, then every thread writes its prefixes.  (Round
// 4's form, one thread per key walking all 256 blocks, ran on V / 1024 = 11
// workgroups: 63 us at the bench's V = 10,544.)  The last workgroup to finish
// (arrival ticket, zeroed by k_emb_hist) then runs emb_offsets over all keys.
constexpr int kKeysPerWg = 64;
constexpr int kKeyGroups = 1024 / kKeysPerWg;            // 16
constexpr int kBlocksPerGroup = kPlanBlocks / kKeyGroups; // 16
static_assert(kKeyGroups * kBlocksPerGroup == kPlanBlocks, "block groups cover the blocks");
__global__ void __launch_bounds__(1024) k_emb_keys(int* __restrict__ cnt, int V,
                                                   int* __restrict__ tot, int* __restrict__ seg,
                                                   int* __restrict__ nch, int* __restrict__ choff,
                                                   int4* __restrict__ desc,
                                                   unsigned* __restrict__ ticket) {
  __shared__ int ts[kPlanMaxKeys];
  __shared__ int gsum[kKeyGroups][kKeysPerWg];
  __shared__ int sh[32];
  __shared__ int s_last;
  const int j = threadIdx.x & (kKeysPerWg - 1), q = threadIdx.x / kKeysPerWg;
  const int v = blockIdx.x * kKeysPerWg + j;
  const int t0 = q * kBlocksPerGroup;
  int c[kBlocksPerGroup];
  int s = 0;
#pragma unroll
  for (int t = 0; t < kBlocksPerGroup; ++t) c[t] = v < V ? cnt[(int64_t)(t0 + t) * V + v] : 0;
#pragma unroll
  for (int t = 0; t < kBlocksPerGroup; ++t) s += c[t];
  gsum[q][j] = s;
  __syncthreads();
  int carry = 0;
  for (int g = 0; g < q; ++g) carry += gsum[g][j];
  if (v < V) {
#pragma unroll
    for (int t = 0; t < kBlocksPerGroup; ++t) {
      cnt[(int64_t)(t0 + t) * V + v] = carry;
      carry += c[t];
    }
    if (q == kKeyGroups - 1) tot[v] = carry;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;   // workgroup-uniform
  emb_offsets(tot, V, seg, nch, choff, desc, ts, sh);
}

// Block t (one wave) places its positions in position order: slot = seg[k]
// + the key's positions in earlier blocks + its earlier positions in this
// block; inside a 64-row step the lanes with equal keys are found from
// ballots over the key bits, and each key's running count stays in LDS
// across the block's steps.  The global loads are batched kPlaceSteps steps
// at a time (the ids, then seg[k] and cnt[t][k] of all of them in flight) so
// only the LDS ranking runs step by step: round 4's form waited for two
// dependent global loads per 64-row step (119 us for the bench's 800-row
// blocks, latency-bound at one wave per block).
constexpr int kPlaceSteps = 8;
__global__ void __launch_bounds__(64) k_emb_place(const int64_t* __restrict__ idx, int64_t M,
                                                  int V, int bits, int64_t per,
                                                  const int* __restrict__ seg,
                                                  const int* __restrict__ cnt,
                                                  int* __restrict__ vals) {
  __shared__ int run[kPlanMaxKeys];
  const int lane = threadIdx.x;
  for (int v = lane; v < V; v += 64) run[v] = 0;
  __syncthreads();
  const int64_t beg = (int64_t)blockIdx.x * per, end = min(M, beg + per);
  const uint64_t lt = (uint64_t(1) << lane) - 1;
  const int* crow = cnt + (int64_t)blockIdx.x * V;
  for (int64_t r0 = beg; r0 < end; r0 += 64 * kPlaceSteps) {
    int k[kPlaceSteps], base[kPlaceSteps];
    bool ok[kPlaceSteps];
#pragma unroll
    for (int st = 0; st < kPlaceSteps; ++st) {
      const int64_t i = r0 + st * 64 + lane;
      const int64_t kk = i < end ? idx[i] : -1;
      ok[st] = kk >= 0 && kk < V;
      k[st] = ok[st] ? (int)kk : 0;
    }
#pragma unroll
    for (int st = 0; st < kPlaceSteps; ++st) base[st] = seg[k[st]] + crow[k[st]];
#pragma unroll
    for (int st = 0; st < kPlaceSteps; ++st) {
      if (r0 + st * 64 >= end) break;   // wave-uniform
      uint64_t same = __builtin_amdgcn_ballot_w64(ok[st]);
      for (int b = 0; b < bits; ++b) {
        const bool bit = (k[st] >> b) & 1;
        const uint64_t m = __builtin_amdgcn_ballot_w64(ok[st] && bit);
        same &= bit ? m : ~m;
      }
      if (ok[st]) {
        const int before = run[k[st]];
        const int64_t slot = (int64_t)base[st] + before + __popcll(same & lt);
        if (slot < M) vals[slot] = (int)(r0 + st * 64 + lane);   // always (a permutation)
        // the group's lowest lane advances the key's count (groups: distinct keys)
        if ((same & lt) == 0) run[k[st]] = before + __popcll(same);
      }
    }
  }
}

// rocPRIM picks its block-sort + merge-sort path below 2^20 items (~100 us
// for the bench's ~205k packed positions: block sort plus 14 merge passes);
// a merge-sort limit of 0 selects Onesweep, the LSD radix sort (stable: the
// positions of one key stay in order), two 8-bit passes over the 14 key bits
using EmbSortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, kEmbMergeLimit>;

int key_bits(int64_t V) {
  int b = 1;
  while ((int64_t(1) << b) < V) ++b;
  return b;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct EmbWs {
  size_t keys_in, keys_out, vals_in, vals_out, seg, nch, choff, desc, partial, sort_tmp, scan_tmp,
      cnt, tot, ticket;
  size_t sort_bytes, scan_bytes, total;
};

EmbWs emb_layout(int64_t M, int64_t V, int64_t d) {
  EmbWs w{};
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = align256(off + bytes); return o; };
  w.keys_in = take(M * 4);
  w.keys_out = take(M * 4);
  w.vals_in = take(M * 4);
  w.vals_out = take(M * 4);
  w.seg = take((V + 1) * 4);
  w.nch = take((V + 1) * 4);
  w.choff = take((V + 1) * 4);
  const int64_t max_chunks = M / kChunk + V + 1;
  w.desc = take((size_t)max_chunks * 16);
  w.partial = take((size_t)max_chunks * d * 4);
  w.sort_bytes = 0;
  (void)rocprim::radix_sort_pairs<EmbSortCfg>(nullptr, w.sort_bytes, (const int*)nullptr, (int*)nullptr,
                            (const int*)nullptr, (int*)nullptr, (size_t)M, 0, key_bits(V));
  w.sort_tmp = take(w.sort_bytes);
  w.scan_bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, w.scan_bytes, (const int*)nullptr, (int*)nullptr, 0,
                          (size_t)(V + 1), rocprim::plus<int>());
  w.scan_tmp = take(w.scan_bytes);
  w.cnt = V <= kPlanMaxKeys ? take((size_t)V * kPlanBlocks * 4) : 0;
  w.tot = V <= kPlanMaxKeys ? take((size_t)V * 4) : 0;
  w.ticket = V <= kPlanMaxKeys ? take(4) : 0;
  w.total = off;
  return w;
}

template <int NV>
int emb_sums(const EmbWs& w, char* ws, const float* grad, int64_t M, int64_t d, int64_t V,
             int64_t padding_idx, float* dw, hipStream_t st) {
  const int* vals = reinterpret_cast<const int*>(ws + w.vals_out);
  const int* seg = reinterpret_cast<const int*>(ws + w.seg);
  const int* nch = reinterpret_cast<const int*>(ws + w.nch);
  const int* choff = reinterpret_cast<const int*>(ws + w.choff);
  float* partial = reinterpret_cast<float*>(ws + w.partial);
  const int4* desc = reinterpret_cast<const int4*>(ws + w.desc);
  const int64_t max_chunks = M / kChunk + V + 1;
  const unsigned cblocks = (unsigned)((max_chunks + 3) / 4);
  if (d % 4 == 0 && aligned16(grad) && aligned16(dw)) {
    if (d <= 128)
      hipLaunchKernelGGL((k_emb_chunk_sum4<1>), dim3(cblocks), dim3(256), 0, st, vals, choff, desc,
                         grad, (int)d, (int)V, (int)padding_idx, dw, partial);
    else if (d <= 256)
      hipLaunchKernelGGL((k_emb_chunk_sum4<2>), dim3(cblocks), dim3(256), 0, st, vals, choff, desc,
                         grad, (int)d, (int)V, (int)padding_idx, dw, partial);
    else
      hipLaunchKernelGGL((k_emb_chunk_sum4<4>), dim3(cblocks), dim3(256), 0, st, vals, choff, desc,
                         grad, (int)d, (int)V, (int)padding_idx, dw, partial);
  } else {
    hipLaunchKernelGGL((k_emb_chunk_sum<NV>), dim3(cblocks), dim3(256), 0, st, vals, seg, nch,
                       choff, grad, (int)d, (int)V, (int)padding_idx, dw, partial);
  }
  hipLaunchKernelGGL((k_emb_finish<NV>), dim3((unsigned)V), dim3(256), 0, st, nch,
                     choff, partial, (int)d, (int)V, (int)padding_idx, dw);
  return launch_status("rb_embedding_bwd");
}

}  // namespace

int64_t emb_workspace_bytes(int64_t M, int64_t V, int64_t d) {
  return (int64_t)emb_layout(M, V, d).total;
}

int launch_embedding_plan(const int64_t* idx, int64_t M, int64_t d, int64_t V, void* workspace,
                          int64_t ws_bytes, hipStream_t st) {
  const EmbWs w = emb_layout(M, V, d);
  if (ws_bytes < (int64_t)w.total) return fail("rb_embedding_bwd: workspace too small");
  char* ws = static_cast<char*>(workspace);
  int* keys_in = reinterpret_cast<int*>(ws + w.keys_in);
  int* keys_out = reinterpret_cast<int*>(ws + w.keys_out);
  int* vals_in = reinterpret_cast<int*>(ws + w.vals_in);
  int* vals_out = reinterpret_cast<int*>(ws + w.vals_out);
  int* seg = reinterpret_cast<int*>(ws + w.seg);
  int* nch = reinterpret_cast<int*>(ws + w.nch);
  int* choff = reinterpret_cast<int*>(ws + w.choff);
  if (V <= kPlanMaxKeys && M < ((int64_t)1 << 31)) {   // the counting sort: three launches
    int* cnt = reinterpret_cast<int*>(ws + w.cnt);
    int* tot = reinterpret_cast<int*>(ws + w.tot);
    unsigned* ticket = reinterpret_cast<unsigned*>(ws + w.ticket);
    const int64_t per = (M + kPlanBlocks - 1) / kPlanBlocks;
    hipLaunchKernelGGL(k_emb_hist, dim3(kPlanBlocks), dim3(1024), 0, st, idx, M, (int)V, per, cnt,
                       ticket);
    hipLaunchKernelGGL(k_emb_keys, dim3((unsigned)((V + kKeysPerWg - 1) / kKeysPerWg)), dim3(1024), 0, st, cnt,
                       (int)V, tot, seg, nch, choff, reinterpret_cast<int4*>(ws + w.desc), ticket);
    hipLaunchKernelGGL(k_emb_place, dim3(kPlanBlocks), dim3(64), 0, st, idx, M, (int)V,
                       key_bits(V), per, seg, cnt, vals_out);
    return launch_status("rb_embedding_plan");
  }
  const int64_t pblocks = std::min<int64_t>(4096, (M + 255) / 256);
  hipLaunchKernelGGL(k_emb_prep, dim3((unsigned)pblocks), dim3(256), 0, st, idx, keys_in, vals_in,
                     M);
  size_t sb = w.sort_bytes;
  if (rocprim::radix_sort_pairs<EmbSortCfg>(ws + w.sort_tmp, sb, keys_in, keys_out, vals_in, vals_out,
                                (size_t)M, 0, key_bits(V), st) != hipSuccess)
    return fail("rb_embedding_bwd: radix sort failed");
  const unsigned vb = (unsigned)((V + 256) / 256);
  hipLaunchKernelGGL(k_emb_segments, dim3(vb), dim3(256), 0, st, keys_out, M, (int)V, seg);
  hipLaunchKernelGGL(k_emb_chunks, dim3(vb), dim3(256), 0, st, seg, (int)V, nch);
  size_t scb = w.scan_bytes;
  if (rocprim::exclusive_scan(ws + w.scan_tmp, scb, nch, choff, 0, (size_t)(V + 1),
                              rocprim::plus<int>(), st) != hipSuccess)
    return fail("rb_embedding_bwd: scan failed");
  hipLaunchKernelGGL(k_emb_chunk_desc, dim3(vb), dim3(256), 0, st, seg, nch, choff, (int)V,
                     reinterpret_cast<int4*>(ws + w.desc));
  return launch_status("rb_embedding_plan");
}

int launch_embedding_apply(const float* grad, int64_t M, int64_t d, int64_t V,
                           int64_t padding_idx, float* dw, void* workspace, int64_t ws_bytes,
                           hipStream_t st) {
  const EmbWs w = emb_layout(M, V, d);
  if (ws_bytes < (int64_t)w.total) return fail("rb_embedding_bwd: workspace too small");
  char* ws = static_cast<char*>(workspace);
  if (d <= 64) return emb_sums<1>(w, ws, grad, M, d, V, padding_idx, dw, st);
  if (d <= 128) return emb_sums<2>(w, ws, grad, M, d, V, padding_idx, dw, st);
  if (d <= 256) return emb_sums<4>(w, ws, grad, M, d, V, padding_idx, dw, st);
  if (d <= 512) return emb_sums<8>(w, ws, grad, M, d, V, padding_idx, dw, st);
  return fail("rb_embedding_bwd: d must be <= 512");
}

int launch_embedding_bwd(const int64_t* idx, const float* grad, int64_t M, int64_t d, int64_t V,
                         int64_t padding_idx, float* dw, void* workspace, int64_t ws_bytes,
                         hipStream_t st) {
  if (int rc = launch_embedding_plan(idx, M, d, V, workspace, ws_bytes, st)) return rc;
  return launch_embedding_apply(grad, M, d, V, padding_idx, dw, workspace, ws_bytes, st);
}

}  // namespace rb
