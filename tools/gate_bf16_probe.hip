// gate_bf16_probe.hip — the configs[4] bf16 gate backward (B=1024, L=2048,
// H=512, dense) in channel-pass variants, alternated, with a checksum of
// every output against the shipped variant (bit-identical expected).
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

int main(int argc, char** argv) {
  const int64_t B = argc > 1 ? atoll(argv[1]) : 1024;
  const int L = argc > 2 ? atoi(argv[2]) : 2048;
  const int H = argc > 3 ? atoi(argv[3]) : 512;
  const int rounds = argc > 4 ? atoi(argv[4]) : 7;
  const int64_t N = B * L * H;
  const int nT = (L + RB_TILE - 1) / RB_TILE;
  bf16_t *rg, *xz, *xc, *dy, *drg, *dxc, *dxz;
  float *lam, *car, *part, *dh0;
  CK(hipMalloc(&rg, 2 * N * 2)); CK(hipMalloc(&xz, 2 * N * 2)); CK(hipMalloc(&xc, N * 2));
  CK(hipMalloc(&dy, N * 2)); CK(hipMalloc(&drg, 2 * N * 2)); CK(hipMalloc(&dxc, N * 2));
  CK(hipMalloc(&dxz, 2 * N * 2));
  CK(hipMalloc(&lam, H * 4)); CK(hipMalloc(&car, B * nT * H * 4));
  CK(hipMalloc(&part, 4 * B * H * 4)); CK(hipMalloc(&dh0, B * H * 4));
  fill_bf16<<<4096, 256>>>(rg, 2 * N, 1, 2.0f);
  fill_bf16<<<4096, 256>>>(xz, 2 * N, 2, 1.5f);
  fill_bf16<<<4096, 256>>>(xc, N, 3, 1.0f);
  fill_bf16<<<4096, 256>>>(dy, N, 4, 0.1f);
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
                  gate_bwd_v<bf16_t, __VA_ARGS__>(a..., nullptr, (hipStream_t)0, nullptr, nullptr); \
                })})
  VARIANT("v4 q4 tc4 pf (shipped)", 4, 4, 4, true);
  VARIANT("v4 q4 tc4 pf vh2", 4, 4, 4, true, 2);
  VARIANT("v8 q8 tc2 pf vh2", 8, 8, 2, true, 2);
  VARIANT("v8 q8 tc2 pf vh4", 8, 8, 2, true, 4);
  VARIANT("v4 q4 tc4 vh2", 4, 4, 4, false, 2);
  VARIANT("v8 q8 tc2 vh2", 8, 8, 2, false, 2);
  VARIANT("v8 q8 tc2 vh4", 8, 8, 2, false, 4);
  const double bytes = 9.0 * N * 2;
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
  // checksums of every output, per variant (outputs cleared before each run)
  for (auto& v : vs) {
    CK(hipMemset(drg, 0, 2 * N * 2)); CK(hipMemset(dxc, 0, N * 2)); CK(hipMemset(dxz, 0, 2 * N * 2));
    CK(hipMemset(part, 0, 4 * B * H * 4)); CK(hipMemset(dh0, 0, B * H * 4));
    v.f();
    CK(hipMemset(cs, 0, 8));
    cksum<<<4096, 256>>>((const uint32_t*)drg, N, cs);
    cksum<<<4096, 256>>>((const uint32_t*)dxc, N / 2, cs);
    cksum<<<4096, 256>>>((const uint32_t*)dxz, N, cs);
    cksum<<<1024, 256>>>((const uint32_t*)part, 3 * B * H, cs);
    cksum<<<1024, 256>>>((const uint32_t*)dh0, B * H, cs);
    CK(hipMemcpy(&v.sum, cs, 8, hipMemcpyDeviceToHost));
  }
  printf("B=%lld L=%d H=%d  (median of %d, alternated)\n", (long long)B, L, H, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%-26s %9.1f us  %.3f of 8 TB/s  cksum %016llx %s\n", v.name, med * 1e3,
           bytes / (med * 1e-3) / 8e12, v.sum, v.sum == vs[0].sum ? "= shipped" : "DIFFERS");
  }
  return 0;
}
