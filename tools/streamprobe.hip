// streamprobe.hip — read-stream rate into LDS on this MI355X: LDS-DMA
// (global_load_lds_dwordx4) rings of NS stages vs register staging, for
// contiguous pieces and for the GEMM's k-sliced row pieces (16 rows x 64 B
// per wave-instruction).  Sizing input for csrc/gemm_split.hip.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/streamprobe.hip -o tools/bin/streamprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// PAT 0: each WG streams a contiguous chunk, stage = WAVES KB contiguous
// PAT 1: k-sliced: stage = 256 rows x 16 floats of a [rows, R] matrix (R = 256)
template <int NS, int PAT, int PER>
__global__ __launch_bounds__(512, 1) void glds_ring(const float* __restrict__ a, int64_t n_floats,
                                                    float* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int STAGE = 8 * PER * 1024;  // 8 waves x PER KB
  const int64_t stage_floats = STAGE / 4;
  const int64_t n_stages_total = n_floats / stage_floats;
  const int G = gridDim.x;
  const int64_t my = (n_stages_total - blockIdx.x + G - 1) / G;
  auto issue = [&](int64_t u) {
    const int64_t sidx = blockIdx.x + u * G;  // global stage index
    char* st = smem + (u % NS) * STAGE;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const float* src;
      if (PAT == 0) {
        src = a + sidx * stage_floats + (wave * PER + q) * 256 + lane * 4;
      } else {
        // k-sliced [rows, 256] matrix: a stage = (8 * PER * 1024) / (4 * BKF) rows x BKF floats
        constexpr int BKF = PAT == 1 ? 16 : PAT == 2 ? 32 : 64;
        constexpr int ROWS = STAGE / (4 * BKF);
        constexpr int KS = 256 / BKF;                 // stages per row tile
        constexpr int LPR = BKF / 4;                  // lanes per row
        const int64_t tile = sidx / KS, kb = sidx % KS;
        const int rr = ((wave * PER + q) * 64 + lane) / LPR;
        const int c = ((wave * PER + q) * 64 + lane) % LPR;
        src = a + (tile * ROWS + rr) * 256 + kb * BKF + c * 4;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + (wave * PER + q) * 1024),
                                       16, 0, 0);
    }
  };
  for (int64_t u = 0; u < NS - 1 && u < my; ++u) issue(u);
  float accum = 0.0f;
  for (int64_t u = 0; u < my; ++u) {
    if (u + NS - 2 < my) wait_vm<(NS - 2) * PER>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (u + NS - 1 < my) issue(u + NS - 1);
    const uint32_t addr = (uint32_t)(uintptr_t)(lds_ptr_t)(smem + (u % NS) * STAGE) + threadIdx.x * 16;
    f32x4 v;
    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr));
    accum += v[0];
  }
  if (accum == 1234.5f) sink[threadIdx.x] = accum;
}

// register staging: U float4 loads in flight per thread, summed
template <int U>
__global__ __launch_bounds__(512) void reg_stream(const f32x4* __restrict__ a, int64_t n4, float* sink) {
  const int64_t stride = (int64_t)gridDim.x * 512;
  f32x4 acc = {0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * 512 + threadIdx.x; i < n4; i += stride * U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = i + u * stride;
      v[u] = k < n4 ? a[k] : f32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc[0] == 1234.5f) sink[threadIdx.x] = acc[1];
}

int main() {
  const int64_t n = 409600LL * 256;  // 420 MB
  float *a, *sink;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(a, 0, n * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    std::vector<float> ts;
    for (int r = 0; r < 8; ++r) {
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2] * 1e3;
    printf("%-34s %8.1f us  %7.1f GB/s\n", name, us, n * 4.0 / us / 1e3);
  };
#define GL(NS, PAT, PER, GRID)                                                                  \
  {                                                                                             \
    auto k = glds_ring<NS, PAT, PER>;                                                           \
    const int lds = NS * 8 * PER * 1024;                                                        \
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);      \
    char nm[64];                                                                                \
    snprintf(nm, 64, "glds NS=%d pat=%d per=%d grid=%d", NS, PAT, PER, GRID);                   \
    run(nm, [&] { k<<<GRID, 512, lds>>>(a, n, sink); });                                        \
  }
  GL(5, 0, 2, 256)
  GL(5, 1, 2, 256) GL(3, 1, 4, 256)
  GL(5, 2, 2, 256) GL(3, 2, 4, 256) GL(8, 2, 1, 512) GL(5, 2, 1, 512)
  GL(5, 3, 2, 256) GL(3, 3, 4, 256) GL(8, 3, 1, 512)
  run("reg U4 grid 1024", [&] { reg_stream<4><<<1024, 512>>>((const f32x4*)a, n / 4, sink); });
  run("reg U8 grid 1024", [&] { reg_stream<8><<<1024, 512>>>((const f32x4*)a, n / 4, sink); });
  run("reg U4 grid 4096", [&] { reg_stream<4><<<4096, 512>>>((const f32x4*)a, n / 4, sink); });
  run("reg U8 grid 256", [&] { reg_stream<8><<<256, 512>>>((const f32x4*)a, n / 4, sink); });
  run("reg U16 grid 256", [&] { reg_stream<16><<<256, 512>>>((const f32x4*)a, n / 4, sink); });
  return 0;
}
