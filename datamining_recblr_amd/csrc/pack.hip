// pack.hip — the packed-sequence plan of RecBLR._forward_packed in one launch.
//
// RecBole right-pads every sequence of a batch to L (RecBLR.py:75 reads
// item_seq [B, L] and item_seq_len [B]); the encoder runs only each
// sequence's first len_b positions, packed back to back longest first
// (DESIGN.md §3).  Given the packed order and the row offsets, one wave per
// packed sequence writes
//   ids[r]  = item_seq[order[s], t]   (the packed item ids the embedding reads)
//   pos[r]  = t                       (row r's position inside its sequence)
//   inv[order[s]]  = s,  last[order[s]] = offs[s+1] - 1
// for r = offs[s] + t — what a dozen torch index/arange/scatter launches did.
#include "common.h"

namespace rb {
namespace {

__global__ void __launch_bounds__(256)
k_pack_plan(const int64_t* __restrict__ seq, int64_t seq_rs, const int64_t* __restrict__ offs,
            const int64_t* __restrict__ order, int64_t B, int64_t* __restrict__ ids,
            int64_t* __restrict__ pos, int64_t* __restrict__ inv, int64_t* __restrict__ last) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= B) return;   // wave-uniform
  const int lane = threadIdx.x & 63;
  const int64_t b = order[s];
  const int64_t r0 = offs[s];
  const int64_t len = offs[s + 1] - r0;
  const int64_t* src = seq + b * seq_rs;
  for (int64_t t = lane; t < len; t += 64) {
    ids[r0 + t] = src[t];
    pos[r0 + t] = t;
  }
  if (lane == 0) {
    inv[b] = s;
    last[b] = r0 + len - 1;
  }
}

}  // namespace

int launch_pack_plan(const int64_t* seq, int64_t seq_rs, const int64_t* offs,
                     const int64_t* order, int64_t B, int64_t* ids, int64_t* pos, int64_t* inv,
                     int64_t* last, hipStream_t st) {
  const int64_t blocks = (B + 3) / 4;
  hipLaunchKernelGGL(k_pack_plan, dim3((unsigned)blocks), dim3(256), 0, st, seq, seq_rs, offs,
                     order, B, ids, pos, inv, last);
  return launch_status("rb_pack_plan");
}

}  // namespace rb
