// itembench.hip — timing of the item-scoring kernels (csrc/item_scores.hip)
// at the benchmark's CE shape (B=2048, V=10544, d=128 by default), plus a
// pure-MFMA issue-rate probe; -DRB_ITEM_PROF adds per-wave cycle counts.
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       tools/itembench.hip -o tools/itembench && tools/itembench [B V d]
#include "../datamining_recblr_amd/csrc/capi.hip"
#include "../datamining_recblr_amd/csrc/conv_silu.hip"
#include "../datamining_recblr_amd/csrc/gate_scan.hip"
#include "../datamining_recblr_amd/csrc/scan_rows.hip"
#include "../datamining_recblr_amd/csrc/rownorm.hip"
#include "../datamining_recblr_amd/csrc/embedding.hip"
#include "../datamining_recblr_amd/csrc/item_scores.hip"
#include "../datamining_recblr_amd/csrc/pad_prefix.hip"
#include "../datamining_recblr_amd/csrc/reduce.hip"

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

__global__ void fill(float* p, int64_t n, uint32_t seed, float scale) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = scale * ((h & 0xffffff) / 16777216.0f - 0.5f);
  }
}
__global__ void fill_idx(int64_t* p, int64_t n, int64_t V) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (i * 7919 + 13) % V;
}

// pure MFMA issue-rate probe: NCH independent 32x32x2 f32 accumulator chains per wave
template <int NCH>
__global__ __launch_bounds__(256) void k_mfma_probe(int iters, float* out) {
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  f32x16 acc[NCH];
  for (int c = 0; c < NCH; ++c) acc[c] = f32x16{};
  float a = threadIdx.x * 1e-3f, b = 1.0f + blockIdx.x * 1e-6f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16 / NCH; ++u)
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
  }
  float s = 0.f;
  for (int c = 0; c < NCH; ++c) s += acc[c][threadIdx.x & 15];
  if (s == 12345.f) out[0] = s;
}

template <class F>
static float time_us(F&& f, int reps = 20) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
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
}

int main(int argc, char** argv) {
  const int64_t B = argc > 1 ? atoll(argv[1]) : 2048, V = argc > 2 ? atoll(argv[2]) : 10544,
                d = argc > 3 ? atoll(argv[3]) : 128;
  float *E, *W, *lse, *loss, *dE, *dW, *dl;
  int64_t *tgt, *gt, *eq;
  CK(hipMalloc(&E, B * d * 4)); CK(hipMalloc(&W, V * d * 4));
  CK(hipMalloc(&lse, B * 4)); CK(hipMalloc(&loss, 4)); CK(hipMalloc(&dl, 4));
  CK(hipMalloc(&dE, B * d * 4)); CK(hipMalloc(&dW, V * d * 4));
  CK(hipMalloc(&tgt, B * 8)); CK(hipMalloc(&gt, B * 8)); CK(hipMalloc(&eq, B * 8));
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, E, B * d, 1u, 1.0f);
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, W, V * d, 2u, 1.0f);
  hipLaunchKernelGGL(fill, dim3(1), dim3(1), 0, 0, dl, 1, 3u, 0.0f);
  hipLaunchKernelGGL(fill_idx, dim3((B + 255) / 256), dim3(256), 0, 0, tgt, B, V);
  const int64_t ws_b = std::max(rb_item_ce_workspace(B, V, d), rb_item_rank_workspace(B, V, d));
  void* ws; CK(hipMalloc(&ws, ws_b));
  float* scores; CK(hipMalloc(&scores, B * V * 4));
  const double gf = 2.0 * B * V * d / 1e9;
  auto rep = [&](const char* n, float us, double gflop) {
    printf("%-10s %9.2f us  %7.1f TF/s (algorithmic)\n", n, us, gflop / us * 1e3);
  };
  printf("B=%ld V=%ld d=%ld\n", (long)B, (long)V, (long)d);
  rep("ce_fwd", time_us([&] { rb_item_ce_fwd(E, W, tgt, B, V, d, lse, loss, ws, ws_b, 0); }), gf);
  rep("ce_bwd", time_us([&] { rb_item_ce_bwd(E, W, tgt, lse, dl, B, V, d, dE, dW, ws, ws_b, 0); }),
      2 * gf);
  rep("ce_bwd_dE",
      time_us([&] { rb_item_ce_bwd(E, W, tgt, lse, dl, B, V, d, dE, nullptr, ws, ws_b, 0); }), gf);
  rep("ce_bwd_dW",
      time_us([&] { rb_item_ce_bwd(E, W, tgt, lse, dl, B, V, d, nullptr, dW, ws, ws_b, 0); }), gf);
  rep("rank", time_us([&] { rb_item_rank(E, W, tgt, B, V, d, 1, gt, eq, ws, ws_b, 0); }), gf);
  rep("scores", time_us([&] { rb_item_scores(E, W, B, V, d, scores, 0); }), gf);
#ifdef RB_ITEM_PROF
  {
    auto dump = [&](const char* nm) {
      std::vector<uint64_t> h(65536 * 4);
      CK(hipDeviceSynchronize());
      CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(rb::g_item_prof), h.size() * 8));
      double pro = 0, body = 0, wait = 0, tiles = 0; int n = 0; double mx = 0;
      for (int i = 0; i < 65536; ++i) {
        if (h[4 * i + 3] == 0) continue;
        pro += h[4 * i]; body += h[4 * i + 1]; wait += h[4 * i + 2]; tiles += h[4 * i + 3]; ++n;
        mx = std::max(mx, (double)(h[4 * i] + h[4 * i + 1] + h[4 * i + 2]));
      }
      printf("PROF %-8s waves %d  per-wave: prologue %.0f cyc, body %.0f cyc/tile, wait %.0f cyc/tile, tiles %.1f, max total %.0f cyc\n",
             nm, n, pro / n, body / tiles, wait / tiles, tiles / n, mx);
      CK(hipMemset((void*)0, 0, 0));
    };
    uint64_t* sym; CK(hipGetSymbolAddress((void**)&sym, HIP_SYMBOL(rb::g_item_prof)));
    CK(hipMemset(sym, 0, 65536 * 32));
    rb_item_scores(E, W, B, V, d, scores, 0); dump("scores");
    CK(hipMemset(sym, 0, 65536 * 32));
    rb_item_ce_fwd(E, W, tgt, B, V, d, lse, loss, ws, ws_b, 0); dump("ce_fwd");
    CK(hipMemset(sym, 0, 65536 * 32));
    rb_item_ce_bwd(E, W, tgt, lse, dl, B, V, d, dE, nullptr, ws, ws_b, 0); dump("bwd_dE");
    CK(hipMemset(sym, 0, 65536 * 32));
    rb_item_ce_bwd(E, W, tgt, lse, dl, B, V, d, nullptr, dW, ws, ws_b, 0); dump("bwd_dW");
  }
#endif
  for (int wps : {1, 2, 4}) {           // waves per SIMD (workgroups of 4 waves per CU)
    const int wgs = 256 * wps, iters = 256;
    const double gfl = 2.0 * 32 * 32 * 2 * 16 * iters * wgs * 4 / 1e9;
    char nm[64];
    snprintf(nm, sizeof nm, "mfma1_w%d", wps);
    rep(nm, time_us([&] { hipLaunchKernelGGL(k_mfma_probe<1>, dim3(wgs), dim3(256), 0, 0, iters, dl); }), gfl);
    snprintf(nm, sizeof nm, "mfma2_w%d", wps);
    rep(nm, time_us([&] { hipLaunchKernelGGL(k_mfma_probe<2>, dim3(wgs), dim3(256), 0, 0, iters, dl); }), gfl);
    snprintf(nm, sizeof nm, "mfma4_w%d", wps);
    rep(nm, time_us([&] { hipLaunchKernelGGL(k_mfma_probe<4>, dim3(wgs), dim3(256), 0, 0, iters, dl); }), gfl);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
