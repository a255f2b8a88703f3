// ce_h_probe.hip — the f16-pipe CE kernels at the bench's shape (B=2048,
// V=10544, d=128): rb_item_ce_fwd_h and rb_item_ce_probs_h_both, median of
// repeated launches.  Built against a csrc tree given by -I (the product's,
// or a copy with another workgroup target: tools/gpu_r05_ce.sh).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       -I datamining_recblr_amd/csrc tools/ce_h_probe.hip -o tools/bin/ce_h_probe
#include "capi.hip"
#include "conv_silu.hip"
#include "gate_scan.hip"
#include "scan_rows.hip"
#include "rownorm.hip"
#include "embedding.hip"
#include "item_scores.hip"
#include "pad_prefix.hip"
#include "reduce.hip"
#include "gemm_half.hip"
#include "gemm_bf16.hip"
#include "pack.hip"
#include "gemm_small.hip"
#include "adam.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)
#define RC(x)                                                  \
  do {                                                         \
    if ((x) != 0) {                                            \
      fprintf(stderr, "%s:%d native call failed\n", __FILE__, __LINE__); \
      exit(1);                                                 \
    }                                                          \
  } while (0)

__global__ void fillr(float* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = scale * ((h & 0xffffff) / 16777216.0f - 0.5f);
  }
}
__global__ void fill_idx(int64_t* p, int64_t n, int64_t V) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (i * 7919 + 13) % V;
}

int main(int argc, char** argv) {
  const int64_t B = argc > 1 ? atoll(argv[1]) : 2048, V = argc > 2 ? atoll(argv[2]) : 10544,
                d = argc > 3 ? atoll(argv[3]) : 128;
  const int reps = argc > 4 ? atoi(argv[4]) : 30;
  float *E, *W, *lse, *loss, *dl, *probs, *probs_t, *gm_r, *gm_i;
  int64_t* tgt;
  void *eimg, *wimg;
  int *eexp, *wexp;
  const int64_t ld = (V + 3) / 4 * 4, ldt = (B + 3) / 4 * 4;
  CK(hipMalloc(&E, B * d * 4)); CK(hipMalloc(&W, V * d * 4));
  CK(hipMalloc(&lse, B * 4)); CK(hipMalloc(&loss, 4)); CK(hipMalloc(&dl, 4));
  CK(hipMalloc(&tgt, B * 8));
  CK(hipMalloc(&eimg, B * d * 4)); CK(hipMalloc(&wimg, V * d * 4));
  CK(hipMalloc(&eexp, B * 4)); CK(hipMalloc(&wexp, V * 4));
  CK(hipMalloc(&probs, B * ld * 4)); CK(hipMalloc(&probs_t, V * ldt * 4));
  CK(hipMalloc(&gm_r, (B + 31) / 32 * 4)); CK(hipMalloc(&gm_i, (V + 31) / 32 * 4));
  fillr<<<1024, 256>>>(E, B * d, 1u, 1.0f);
  fillr<<<1024, 256>>>(W, V * d, 2u, 1.0f);
  fillr<<<1, 1>>>(dl, 1, 3u, 0.0f);
  fill_idx<<<(B + 255) / 256, 256>>>(tgt, B, V);
  RC(rb_item_split_h(E, B, d, eimg, eexp, nullptr, 0));
  RC(rb_item_split_h(W, V, d, wimg, wexp, nullptr, 0));
  const int64_t ws_b = rb_item_ce_workspace(B, V, d);
  void* ws; CK(hipMalloc(&ws, ws_b));
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto time_us = [&](auto&& f) {
    std::vector<float> v;
    for (int r = 0; r < reps + 3; ++r) {
      CK(hipEventRecord(a, 0));
      f();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (r >= 3) v.push_back(ms * 1000.f);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const float tf = time_us([&] {
    RC(rb_item_ce_fwd_h(eimg, eexp, wimg, wexp, tgt, B, V, d, lse, loss, ws, ws_b, 0));
  });
  const float tp = time_us([&] {
    RC(rb_item_ce_probs_h_both(eimg, eexp, wimg, wexp, tgt, lse, dl, B, V, d, 0, probs, ld,
                               probs_t, ldt, gm_r, gm_i, 0));
  });
  float lh;
  CK(hipMemcpy(&lh, loss, 4, hipMemcpyDeviceToHost));
  printf("ce_fwd_h %8.2f us  ce_probs_h_both %8.2f us  (loss %.6f)\n", tf, tp, lh);
  return 0;
}
