// copyprobe.hip — what streaming rate does this MI355X reach for plain copies?
// (1R+1W float4 with U independent 16-B loads per thread in flight, grid
// sizes, nontemporal hints), as the ceiling for the channel-last kernels.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copyU(const v4f* __restrict__ a, v4f* __restrict__ o, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride * U) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = i + u * stride;
      if (k < n4) v[u] = NT ? __builtin_nontemporal_load(a + k) : a[k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = i + u * stride;
      if (k < n4) { if (NT) __builtin_nontemporal_store(v[u], o + k); else o[k] = v[u]; }
    }
  }
}

// contiguous chunk per block (each block streams its own 256*U*16-B pieces)
template <int U>
__global__ __launch_bounds__(256) void copyChunk(const float4* __restrict__ a, float4* __restrict__ o, int64_t n4, int64_t per) {
  const int64_t b0 = (int64_t)blockIdx.x * per, b1 = std::min(b0 + per, n4);
  for (int64_t i = b0 + threadIdx.x; i < b1; i += 256 * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { const int64_t k = i + u * 256; if (k < b1) v[u] = a[k]; }
#pragma unroll
    for (int u = 0; u < U; ++u) { const int64_t k = i + u * 256; if (k < b1) o[k] = v[u]; }
  }
}

int main() {
  const int64_t n = 2048LL * 200 * 256;   // floats, 420 MB
  float *a, *o;
  CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&o, n * 4));
  CK(hipMemset(a, 1, n * 4)); CK(hipMemset(o, 0, n * 4));
  const int64_t n4 = n / 4;
  struct C { const char* nm; std::function<void()> f; };
  std::vector<C> cs;
  for (int g : {2048, 8192, 32768}) {
    char* s1 = new char[64]; snprintf(s1, 64, "U1 g%d", g);
    cs.push_back({s1, [=] { hipLaunchKernelGGL((copyU<1, false>), dim3(g), dim3(256), 0, 0, (const v4f*)a, (v4f*)o, n4); }});
    char* s2 = new char[64]; snprintf(s2, 64, "U4 g%d", g);
    cs.push_back({s2, [=] { hipLaunchKernelGGL((copyU<4, false>), dim3(g), dim3(256), 0, 0, (const v4f*)a, (v4f*)o, n4); }});
    char* s3 = new char[64]; snprintf(s3, 64, "U4 NT g%d", g);
    cs.push_back({s3, [=] { hipLaunchKernelGGL((copyU<4, true>), dim3(g), dim3(256), 0, 0, (const v4f*)a, (v4f*)o, n4); }});
    char* s4 = new char[64]; snprintf(s4, 64, "U8 g%d", g);
    cs.push_back({s4, [=] { hipLaunchKernelGGL((copyU<8, false>), dim3(g), dim3(256), 0, 0, (const v4f*)a, (v4f*)o, n4); }});
  }
  for (int g : {1024, 4096, 16384}) {
    char* s = new char[64]; snprintf(s, 64, "chunk U4 g%d", g);
    const int64_t per = (n4 + g - 1) / g;
    cs.push_back({s, [=] { hipLaunchKernelGGL((copyChunk<4>), dim3(g), dim3(256), 0, 0, (const float4*)a, (float4*)o, n4, per); }});
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& c : cs) c.f();
  CK(hipDeviceSynchronize());
  for (auto& c : cs) {
    std::vector<float> ms;
    for (int r = 0; r < 15; ++r) {
      CK(hipEventRecord(e0, 0)); c.f(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float t; CK(hipEventElapsedTime(&t, e0, e1)); ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double t = ms[7];
    printf("%-18s %8.1f us  %7.1f GB/s  %.3f of 8 TB/s\n", c.nm, t * 1e3, 2.0 * n * 4 / (t * 1e-3) / 1e9, 2.0 * n * 4 / (t * 1e-3) / 8e12);
  }
  return 0;
}
