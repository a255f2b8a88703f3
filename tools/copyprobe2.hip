// copyprobe2.hip — second pass at this MI355X's streaming ceiling: one-shot
// grids (one float4 per thread, no loop) and large grid-stride grids, block
// size, buffer size, read-only / write-only / copy / 4R+1W, nontemporal hints.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/copyprobe2.hip -o tools/bin/copyprobe2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ v4f ld(const v4f* p) { return NT & 1 ? __builtin_nontemporal_load(p) : *p; }
template <int NT>
__device__ __forceinline__ void st(v4f v, v4f* p) { if (NT & 2) __builtin_nontemporal_store(v, p); else *p = v; }

// one float4 per thread per input, V float4s per thread along a contiguous run
template <int NT, int V>
__global__ void copy1(const v4f* __restrict__ a, v4f* __restrict__ o, int64_t n4) {
  const int64_t base = ((int64_t)blockIdx.x * blockDim.x) * V + threadIdx.x;
  v4f v[V];
#pragma unroll
  for (int u = 0; u < V; ++u) { const int64_t k = base + u * blockDim.x; if (k < n4) v[u] = ld<NT>(a + k); }
#pragma unroll
  for (int u = 0; u < V; ++u) { const int64_t k = base + u * blockDim.x; if (k < n4) st<NT>(v[u], o + k); }
}

template <int NT, int V>
__global__ void read1(const v4f* __restrict__ a, float* sink, int64_t n4) {
  const int64_t base = ((int64_t)blockIdx.x * blockDim.x) * V + threadIdx.x;
  v4f acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < V; ++u) { const int64_t k = base + u * blockDim.x; if (k < n4) acc += ld<NT>(a + k); }
  if (acc[0] == 1234.5f) sink[threadIdx.x] = acc[1];
}

template <int NT, int V>
__global__ void write1(v4f* __restrict__ o, int64_t n4) {
  const int64_t base = ((int64_t)blockIdx.x * blockDim.x) * V + threadIdx.x;
  const v4f z = {1, 2, 3, 4};
#pragma unroll
  for (int u = 0; u < V; ++u) { const int64_t k = base + u * blockDim.x; if (k < n4) st<NT>(z, o + k); }
}

// 4 inputs -> 1 output (gate-forward-like mix), one float4 each per thread
template <int NT>
__global__ void mix41(const v4f* __restrict__ a, const v4f* __restrict__ b, const v4f* __restrict__ c,
                      const v4f* __restrict__ d, v4f* __restrict__ o, int64_t n4) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n4) st<NT>(ld<NT>(a + k) + ld<NT>(b + k) * ld<NT>(c + k) + ld<NT>(d + k), o + k);
}

// 5 inputs -> 4 outputs (gate-backward-like mix)
template <int NT>
__global__ void mix54(const v4f* __restrict__ a, const v4f* __restrict__ b, const v4f* __restrict__ c,
                      const v4f* __restrict__ d, const v4f* __restrict__ e, v4f* __restrict__ o0,
                      v4f* __restrict__ o1, v4f* __restrict__ o2, v4f* __restrict__ o3, int64_t n4) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n4) {
    const v4f x = ld<NT>(a + k), y = ld<NT>(b + k), z = ld<NT>(c + k), w = ld<NT>(d + k), q = ld<NT>(e + k);
    st<NT>(x * y, o0 + k); st<NT>(z + w, o1 + k); st<NT>(q * x, o2 + k); st<NT>(y - q, o3 + k);
  }
}

// grid-stride copy, fixed grid
template <int NT>
__global__ void copyGS(const v4f* __restrict__ a, v4f* __restrict__ o, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) st<NT>(ld<NT>(a + i), o + i);
}

int main(int argc, char** argv) {
  const int64_t mb = argc > 1 ? atoll(argv[1]) : 420;  // MB per buffer
  const int64_t n = mb * 1000000 / 4 / 1024 * 1024;
  const int64_t n4 = n / 4;
  float* buf[10];
  for (int i = 0; i < 10; ++i) { CK(hipMalloc(&buf[i], n * 4)); CK(hipMemset(buf[i], 0, n * 4)); }
  float* sink; CK(hipMalloc(&sink, 1 << 16));
  const v4f* a = (const v4f*)buf[0];
  v4f* o = (v4f*)buf[1];
  struct C { std::string nm; double bytes; std::function<void()> f; };
  std::vector<C> cs;
  auto gridfor = [&](int bs, int V) { return (unsigned)((n4 + (int64_t)bs * V - 1) / ((int64_t)bs * V)); };
#define ADD(NM, BYTES, ...) cs.push_back({NM, BYTES, [=] { __VA_ARGS__; }})
  for (int bs : {256, 512, 1024}) {
    ADD("copy1 V1 bs" + std::to_string(bs), 2.0 * n * 4, copy1<0, 1><<<gridfor(bs, 1), bs>>>(a, o, n4));
    ADD("copy1 V1 nt3 bs" + std::to_string(bs), 2.0 * n * 4, copy1<3, 1><<<gridfor(bs, 1), bs>>>(a, o, n4));
    ADD("copy1 V1 ntst bs" + std::to_string(bs), 2.0 * n * 4, copy1<2, 1><<<gridfor(bs, 1), bs>>>(a, o, n4));
    ADD("copy1 V2 bs" + std::to_string(bs), 2.0 * n * 4, copy1<0, 2><<<gridfor(bs, 2), bs>>>(a, o, n4));
    ADD("copy1 V4 bs" + std::to_string(bs), 2.0 * n * 4, copy1<0, 4><<<gridfor(bs, 4), bs>>>(a, o, n4));
  }
  for (int g : {4096, 16384, 65536})
    ADD("copyGS g" + std::to_string(g), 2.0 * n * 4, copyGS<0><<<g, 256>>>(a, o, n4));
  ADD("read1 V1 bs256", 1.0 * n * 4, read1<0, 1><<<gridfor(256, 1), 256>>>(a, sink, n4));
  ADD("read1 V4 bs256", 1.0 * n * 4, read1<0, 4><<<gridfor(256, 4), 256>>>(a, sink, n4));
  ADD("read1 V4 nt bs256", 1.0 * n * 4, read1<1, 4><<<gridfor(256, 4), 256>>>(a, sink, n4));
  ADD("write1 V1 bs256", 1.0 * n * 4, write1<0, 1><<<gridfor(256, 1), 256>>>(o, n4));
  ADD("write1 V4 bs256", 1.0 * n * 4, write1<0, 4><<<gridfor(256, 4), 256>>>(o, n4));
  ADD("write1 V4 nt bs256", 1.0 * n * 4, write1<2, 4><<<gridfor(256, 4), 256>>>(o, n4));
  const v4f* b4[5] = {(const v4f*)buf[2], (const v4f*)buf[3], (const v4f*)buf[4], (const v4f*)buf[5], (const v4f*)buf[0]};
  v4f* o4[4] = {(v4f*)buf[6], (v4f*)buf[7], (v4f*)buf[8], (v4f*)buf[9]};
  for (int bs : {256, 512}) {
    ADD("mix41 bs" + std::to_string(bs), 5.0 * n * 4, mix41<0><<<gridfor(bs, 1), bs>>>(b4[0], b4[1], b4[2], b4[3], o4[0], n4));
    ADD("mix41 nt bs" + std::to_string(bs), 5.0 * n * 4, mix41<3><<<gridfor(bs, 1), bs>>>(b4[0], b4[1], b4[2], b4[3], o4[0], n4));
    ADD("mix54 bs" + std::to_string(bs), 9.0 * n * 4,
        mix54<0><<<gridfor(bs, 1), bs>>>(b4[0], b4[1], b4[2], b4[3], b4[4], o4[0], o4[1], o4[2], o4[3], n4));
    ADD("mix54 nt bs" + std::to_string(bs), 9.0 * n * 4,
        mix54<3><<<gridfor(bs, 1), bs>>>(b4[0], b4[1], b4[2], b4[3], b4[4], o4[0], o4[1], o4[2], o4[3], n4));
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& c : cs) c.f();
  CK(hipDeviceSynchronize());
  printf("buffers %lld MB each\n", (long long)(n * 4 / 1000000));
  for (auto& c : cs) {
    std::vector<float> ms;
    for (int r = 0; r < 15; ++r) {
      CK(hipEventRecord(e0, 0)); c.f(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float t; CK(hipEventElapsedTime(&t, e0, e1)); ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double t = ms[7];
    printf("%-22s %8.1f us  %7.1f GB/s  %.3f of 8 TB/s  (best %.3f)\n", c.nm.c_str(), t * 1e3, c.bytes / (t * 1e-3) / 1e9,
           c.bytes / (t * 1e-3) / 8e12, c.bytes / (ms[0] * 1e-3) / 8e12);
  }
  return 0;
}
