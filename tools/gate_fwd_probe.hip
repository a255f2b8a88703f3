// gate_fwd_probe.hip — the bf16 gate forward at configs[4] (B=1024, L=2048,
// H=512, dense) in chunk / width variants, alternated, with a checksum of y
// and the carries against the shipped variant.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       tools/gate_fwd_probe.hip -o tools/bin/gate_fwd_probe
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

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const int64_t B = 1024;
  const int L = 2048, H = 512;
  const int64_t N = B * L * H;
  const int nT = (L + RB_TILE - 1) / RB_TILE;
  bf16_t *rg, *xz, *xc, *y;
  float *lam, *car;
  CK(hipMalloc(&rg, 2 * N * 2)); CK(hipMalloc(&xz, 2 * N * 2)); CK(hipMalloc(&xc, N * 2));
  CK(hipMalloc(&y, N * 2)); CK(hipMalloc(&lam, H * 4)); CK(hipMalloc(&car, B * nT * H * 4));
  fill_bf16<<<4096, 256>>>(rg, 2 * N, 1, 2.0f);
  fill_bf16<<<4096, 256>>>(xz, 2 * N, 2, 1.5f);
  fill_bf16<<<4096, 256>>>(xc, N, 3, 1.0f);
  fill_f32<<<64, 256>>>(lam, H, 5, 1.0f, 0.5f);
  CK(hipDeviceSynchronize());
  unsigned long long* cs;
  CK(hipMalloc(&cs, 8));
  struct V { const char* name; std::function<void()> f; std::vector<float> ms; unsigned long long sum = 0; };
  std::vector<V> vs;
#define FV(NAME, VEC, PF)                                                                      \
  vs.push_back({NAME, [=] {                                                                    \
    gate_fwd_v<bf16_t, VEC, PF>(rg, 2 * H, xc, H, xz + H, 2 * H, lam, nullptr, nullptr, 0, y, H, \
                                car, B, L, H, nullptr, 0, nullptr, nullptr);                   \
  }})
  FV("v4 q4 tc4 (shipped)", 4, false);
  FV("v4 q4 tc4 pf", 4, true);
  FV("v8 q4 tc4", 8, false);
  FV("v2 q4 tc4", 2, false);
  const double bytes = 5.0 * N * 2;
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
    CK(hipMemset(y, 0, N * 2)); CK(hipMemset(car, 0, B * nT * H * 4));
    v.f();
    CK(hipMemset(cs, 0, 8));
    cksum<<<4096, 256>>>((const uint32_t*)y, N / 2, cs);
    cksum<<<4096, 256>>>((const uint32_t*)car, B * nT * H, cs);
    CK(hipMemcpy(&v.sum, cs, 8, hipMemcpyDeviceToHost));
  }
  printf("bf16 gate forward B=%lld L=%d H=%d  (median of %d, alternated; 5 streams)\n",
         (long long)B, L, H, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("  %-22s %9.1f us  %.3f of 8 TB/s  cksum %016llx %s\n", v.name, med * 1e3,
           bytes / (med * 1e-3) / 8e12, v.sum, v.sum == vs[0].sum ? "= shipped" : "differs");
  }
  return 0;
}
