// embedding.hip — deterministic scatter-add backward of the item embedding
// gather (reference RecBLR.py:76, nn.Embedding(n_items, d, padding_idx=0)).
//
//   dW[v] = sum over positions p with idx[p] == v of grad[p]   (dW[pad] = 0)
//
// torch sorts the indices and runs a segmented reduction whose sum_and_scatter
// kernel took ~4.8 ms per training step at B=2048 L=200 d=128.  Here:
//   1. keys = int32(idx), vals = position; rocPRIM stable radix sort on the
//      log2(V) key bits (positions stay in order inside every key);
//   2. seg[v] = lower_bound(sorted keys, v) for v in [0, V];
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
  size_t keys_in, keys_out, vals_in, vals_out, seg, nch, choff, desc, partial, sort_tmp, scan_tmp;
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
