// conv_bwd_probe.hip — the conv backward (k_conv_silu_bwd, K = 4) in chunk /
// step-count variants, dense rows: bf16 at configs[4] (B=1024, L=2048,
// H=512) and fp32 at the bench's shape (B=2048, L=200, H=256), alternated,
// with a checksum of every output (same arithmetic per element; the dW / dbias
// partial sums re-associate with the chunk count).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       tools/conv_bwd_probe.hip -o tools/bin/conv_bwd_probe
#include "../datamining_recblr_amd/csrc/capi.hip"
#include "../datamining_recblr_amd/csrc/conv_silu.hip"
#include "../datamining_recblr_amd/csrc/gate_scan.hip"
#include "../datamining_recblr_amd/csrc/scan_rows.hip"
#include "../datamining_recblr_amd/csrc/rownorm.hip"
#include "../datamining_recblr_amd/csrc/embedding.hip"
#include "../datamining_recblr_amd/csrc/item_scores.hip"
#include "../datamining_recblr_amd/csrc/pad_prefix.hip"
#include "../datamining_recblr_amd/csrc/reduce.hip"
#include "../datamining_recblr_amd/csrc/gemm_half.hip"
#include "../datamining_recblr_amd/csrc/gemm_bf16.hip"
#include "../datamining_recblr_amd/csrc/pack.hip"
#include "../datamining_recblr_amd/csrc/gemm_small.hip"
#include "../datamining_recblr_amd/csrc/adam.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

using namespace rb;

__global__ void fill_bf16(bf16_t* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = (bf16_t)(scale * ((float)(h & 0xffffff) / 8388608.0f - 1.0f));
  }
}
__global__ void fill_f32(float* p, int64_t n, uint32_t seed, float scale, float off) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = off + scale * ((float)(h & 0xffffff) / 8388608.0f - 1.0f);
  }
}
// order-independent checksum of 32-bit words: sum of mixed words (wraps)
__global__ void cksum(const uint32_t* p, int64_t n, unsigned long long* out) {
  unsigned long long s = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t w = p[i] * 0x9E3779B97F4A7C15ull ^ (uint64_t)i;
    s += w ^ (w >> 29);
  }
  atomicAdd(out, s);
}


template <typename T>
void fill(T* p, int64_t n, uint32_t seed, float scale) {
  if constexpr (sizeof(T) == 2) fill_bf16<<<4096, 256>>>((bf16_t*)p, n, seed, scale);
  else fill_f32<<<4096, 256>>>((float*)p, n, seed, scale, 0.0f);
}

template <typename T>
void run(int64_t B, int L, int H, int rounds) {
  const int64_t N = B * L * H;
  constexpr int K = 4;
  T *xz, *g1, *g2, *dxz;
  float *w, *bias, *dwp;
  CK(hipMalloc(&xz, 2 * N * sizeof(T))); CK(hipMalloc(&g1, N * sizeof(T)));
  CK(hipMalloc(&g2, N * sizeof(T))); CK(hipMalloc(&dxz, 2 * N * sizeof(T)));
  CK(hipMalloc(&w, H * K * 4)); CK(hipMalloc(&bias, H * 4));
  CK(hipMalloc(&dwp, B * (K + 1) * H * 4));
  fill(xz, 2 * N, 1, 1.5f); fill(g1, N, 2, 0.1f); fill(g2, N, 3, 0.1f);
  fill_f32<<<64, 256>>>(w, H * K, 4, 0.5f, 0.0f);
  fill_f32<<<64, 256>>>(bias, H, 5, 0.1f, 0.0f);
  CK(hipDeviceSynchronize());
  unsigned long long* cs;
  CK(hipMalloc(&cs, 8));
  struct V { const char* name; std::function<void()> f; std::vector<float> ms; unsigned long long s1 = 0, s2 = 0; };
  std::vector<V> vs;
#define CV(NAME, VEC, Q, TC, PF)                                                              \
  vs.push_back({NAME, [=] {                                                                   \
    const int span = (kWave / Q) * VEC;                                                       \
    const int ncw = (H + span - 1) / span;                                                    \
    const int64_t blocks = (B * ncw + 3) / 4;                                                 \
    hipLaunchKernelGGL((k_conv_silu_bwd<T, K, VEC, Q, TC, PF>), dim3((unsigned)blocks),       \
                       dim3(256), 0, 0, (const T*)xz, 2 * H, w, bias, (const T*)g1,           \
                       (const T*)g2, dxz, 2 * H, dwp, (float*)nullptr, B, L, H, ncw,          \
                       (const int64_t*)nullptr);                                              \
  }})
  CV("v4 q4 tc4 (shipped)", 4, 4, 4, false);
  CV("v4 q4 tc8", 4, 4, 8, false);
  CV("v4 q2 tc8", 4, 2, 8, false);
  CV("v4 q4 tc6", 4, 4, 6, false);
  CV("v4 q8 tc4", 4, 8, 4, false);
  CV("v4 q4 tc4 pf", 4, 4, 4, true);
  CV("v4 q4 tc8 pf", 4, 4, 8, true);
  const double bytes = 4.0 * N * sizeof(T);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& v : vs) { v.f(); CK(hipDeviceSynchronize()); }
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      CK(hipEventRecord(e0));
      v.f();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  for (auto& v : vs) {
    CK(hipMemset(dxz, 0, 2 * N * sizeof(T))); CK(hipMemset(dwp, 0, B * (K + 1) * H * 4));
    v.f();
    CK(hipMemset(cs, 0, 8));
    cksum<<<4096, 256>>>((const uint32_t*)dxz, 2 * N * sizeof(T) / 4, cs);
    CK(hipMemcpy(&v.s1, cs, 8, hipMemcpyDeviceToHost));
    CK(hipMemset(cs, 0, 8));
    cksum<<<1024, 256>>>((const uint32_t*)dwp, B * (K + 1) * H, cs);
    CK(hipMemcpy(&v.s2, cs, 8, hipMemcpyDeviceToHost));
  }
  printf("%s B=%lld L=%d H=%d  (median of %d, alternated; 3R + 1W bytes)\n",
         sizeof(T) == 2 ? "bf16" : "fp32", (long long)B, L, H, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("  %-22s %9.1f us  %.3f of 8 TB/s  dx %s  dw %s\n", v.name, med * 1e3,
           bytes / (med * 1e-3) / 8e12, v.s1 == vs[0].s1 ? "= shipped" : "DIFFERS",
           v.s2 == vs[0].s2 ? "= shipped" : "differs");
  }
  CK(hipFree(xz)); CK(hipFree(g1)); CK(hipFree(g2)); CK(hipFree(dxz));
  CK(hipFree(w)); CK(hipFree(bias)); CK(hipFree(dwp)); CK(hipFree(cs));
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  run<bf16_t>(1024, 2048, 512, rounds);
  run<float>(2048, 200, 256, rounds);
  return 0;
}
