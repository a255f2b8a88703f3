// gate_bf16_probe.hip — the gate backward in channel-pass variants, dense
// rows: bf16 at configs[4] (B=1024, L=2048, H=512) and fp32 at the bench's
// shape (B=2048, L=200, H=256), alternated, with a checksum of every output
// against the first variant of each.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       tools/gate_bf16_probe.hip -o tools/bin/gate_bf16_probe
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
void run(int64_t B, int L, int H, int rounds) {
  const int64_t N = B * L * H;
  const int nT = (L + RB_TILE - 1) / RB_TILE;
  T *rg, *xz, *xc, *dy, *drg, *dxc, *dxz;
  float *lam, *car, *part, *dh0;
  CK(hipMalloc(&rg, 2 * N * sizeof(T))); CK(hipMalloc(&xz, 2 * N * sizeof(T)));
  CK(hipMalloc(&xc, N * sizeof(T))); CK(hipMalloc(&dy, N * sizeof(T)));
  CK(hipMalloc(&drg, 2 * N * sizeof(T))); CK(hipMalloc(&dxc, N * sizeof(T)));
  CK(hipMalloc(&dxz, 2 * N * sizeof(T)));
  CK(hipMalloc(&lam, H * 4)); CK(hipMalloc(&car, B * nT * H * 4));
  CK(hipMalloc(&part, 4 * B * H * 4)); CK(hipMalloc(&dh0, B * H * 4));
  auto fillT = [](T* p, int64_t n, uint32_t seed, float scale) {
    if constexpr (sizeof(T) == 2) fill_bf16<<<4096, 256>>>((bf16_t*)p, n, seed, scale);
    else fill_f32<<<4096, 256>>>((float*)p, n, seed, scale, 0.0f);
  };
  fillT(rg, 2 * N, 1, 2.0f);
  fillT(xz, 2 * N, 2, 1.5f);
  fillT(xc, N, 3, 1.0f);
  fillT(dy, N, 4, 0.1f);
  fill_f32<<<64, 256>>>(lam, H, 5, 1.0f, 0.5f);
  fill_f32<<<4096, 256>>>(car, B * nT * H, 6, 0.5f, 0.0f);
  CK(hipDeviceSynchronize());
  unsigned long long* cs;
  CK(hipMalloc(&cs, 8));
  struct V { const char* name; std::function<void()> f; std::vector<float> ms; unsigned long long sum = 0; };
  std::vector<V> vs;
  auto args = [=](auto fn) {
    return [=] {
      fn(rg, 2 * H, xc, H, xz + H, 2 * H, lam, nullptr, car, dy, drg, 2 * H, dxc, H, dxz + H,
         2 * H, part, dh0, B, L, H);
    };
  };
#define VARIANT(NAME, ...)                                                                     \
  vs.push_back({NAME, args([](auto... a) {                                                     \
                  gate_bwd_v<T, __VA_ARGS__>(a..., nullptr, (hipStream_t)0, nullptr, nullptr); \
                })})
  if constexpr (sizeof(T) == 2) {
    VARIANT("v4 q4 tc4 vh2 (shipped)", 4, 4, 4, false, 2);
    VARIANT("v4 q4 tc4 pf", 4, 4, 4, true);
  } else {
    VARIANT("v4 q8 tc2 (shipped)", 4, 8, 2, false);
    VARIANT("v4 q8 tc2 vh2", 4, 8, 2, false, 2);
    VARIANT("v4 q4 tc4 vh2", 4, 4, 4, false, 2);
    VARIANT("v4 q8 tc2 pf vh2", 4, 8, 2, true, 2);
  }
#undef VARIANT
  const double bytes = 9.0 * N * sizeof(T);
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
    CK(hipMemset(drg, 0, 2 * N * sizeof(T))); CK(hipMemset(dxc, 0, N * sizeof(T)));
    CK(hipMemset(dxz, 0, 2 * N * sizeof(T)));
    CK(hipMemset(part, 0, 4 * B * H * 4)); CK(hipMemset(dh0, 0, B * H * 4));
    v.f();
    CK(hipMemset(cs, 0, 8));
    cksum<<<4096, 256>>>((const uint32_t*)drg, 2 * N * sizeof(T) / 4, cs);
    cksum<<<4096, 256>>>((const uint32_t*)dxc, N * sizeof(T) / 4, cs);
    cksum<<<4096, 256>>>((const uint32_t*)dxz, 2 * N * sizeof(T) / 4, cs);
    cksum<<<1024, 256>>>((const uint32_t*)part, 3 * B * H, cs);
    cksum<<<1024, 256>>>((const uint32_t*)dh0, B * H, cs);
    CK(hipMemcpy(&v.sum, cs, 8, hipMemcpyDeviceToHost));
  }
  printf("%s B=%lld L=%d H=%d  (median of %d, alternated)\n", sizeof(T) == 2 ? "bf16" : "fp32",
         (long long)B, L, H, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("  %-26s %9.1f us  %.3f of 8 TB/s  cksum %016llx %s\n", v.name, med * 1e3,
           bytes / (med * 1e-3) / 8e12, v.sum, v.sum == vs[0].sum ? "= first" : "differs");
  }
  CK(hipFree(rg)); CK(hipFree(xz)); CK(hipFree(xc)); CK(hipFree(dy)); CK(hipFree(drg));
  CK(hipFree(dxc)); CK(hipFree(dxz)); CK(hipFree(lam)); CK(hipFree(car)); CK(hipFree(part));
  CK(hipFree(dh0)); CK(hipFree(cs));
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  run<bf16_t>(1024, 2048, 512, rounds);
  run<float>(2048, 200, 256, rounds);
  return 0;
}
