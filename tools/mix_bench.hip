// mix_bench.hip — the HBM ceiling of the gate-scan backward's access mix.
//
// rb_gate_scan_bwd streams 5 fp32 operands in (rg's r and i halves, xc, z,
// dy) and 4 out (drg's halves, dxc, dz) per packed row and channel, at the
// encoder's layout: rg / drg [M, 2H] and z / dz inside [M, 2H] buffers
// (stride 2H), xc / dy / dxc [M, H].  This measures a kernel with exactly that
// access pattern and no math (16-B per lane, one row x 4 channels per lane),
// so the scan kernel's rate can be read against what the memory system gives
// the mix, rather than against the 8 TB/s datasheet peak.  Also: the
// forward's 4R+1W mix, read-only and write-only streams, and the same 5R+4W
// launch right after a kernel that dirtied 840 MB (the predecessor effect).
// Before every timed launch a 1 GiB buffer is written and then read, so no
// operand starts in the Infinity Cache.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mix_bench.hip -o tools/bin/mix_bench
#include <hip/hip_runtime.h>

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

typedef float f4 __attribute__((ext_vector_type(4)));

struct Ops {
  const float *rg, *xc, *xz, *dy;   // reads: rg r/i [M, 2H], xc [M, H], z = xz + H [M, 2H], dy
  float *drg, *dxc, *dxz;           // writes: drg r/i, dxc, dz = dxz + H
};

// NR reads / NW writes out of the 5 / 4 streams above; one lane = one row x 4 channels
template <int NR, int NW>
__global__ void __launch_bounds__(256) k_mix(Ops o, int64_t M, int H) {
  const int cg = H / 4;
  const int64_t n = M * cg;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / cg;
    const int c = (int)(i - m * cg) * 4;
    f4 s = {0.f, 0.f, 0.f, 0.f};
    if (NR > 0) s += *(const f4*)(o.rg + m * 2 * H + c);
    if (NR > 1) s += *(const f4*)(o.rg + m * 2 * H + H + c);
    if (NR > 2) s += *(const f4*)(o.xc + m * H + c);
    if (NR > 3) s += *(const f4*)(o.xz + m * 2 * H + H + c);
    if (NR > 4) s += *(const f4*)(o.dy + m * H + c);
    if (NR == 0) s = f4{(float)m, 1.f, 2.f, (float)c};
    if (NW > 0) *(f4*)(o.drg + m * 2 * H + c) = s;
    if (NW > 1) *(f4*)(o.drg + m * 2 * H + H + c) = s * 2.f;
    if (NW > 2) *(f4*)(o.dxc + m * H + c) = s * 3.f;
    if (NW > 3) *(f4*)(o.dxz + m * 2 * H + H + c) = s * 4.f;
    if (NW == 0 && s.x == 12345.678f) o.drg[0] = s.y;   // keeps the reads
  }
}

__global__ void k_flush(float* p, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    p[i] = p[i] * 0.5f + v;
}

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atoll(argv[1]) : 204632;
  const int H = 256;
  const int reps = argc > 2 ? atoi(argv[2]) : 7;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *rg, *xc, *xz, *dy, *drg, *dxc, *dxz, *fl;
  const int64_t n1 = M * H, flush_n = (int64_t)1 << 28;   // 1 GiB
  CK(hipMalloc(&rg, n1 * 8));
  CK(hipMalloc(&xc, n1 * 4));
  CK(hipMalloc(&xz, n1 * 8));
  CK(hipMalloc(&dy, n1 * 4));
  CK(hipMalloc(&drg, n1 * 8));
  CK(hipMalloc(&dxc, n1 * 4));
  CK(hipMalloc(&dxz, n1 * 8));
  CK(hipMalloc(&fl, flush_n * 4));
  CK(hipMemset(rg, 0, n1 * 8));
  CK(hipMemset(xc, 0, n1 * 4));
  CK(hipMemset(xz, 0, n1 * 8));
  CK(hipMemset(dy, 0, n1 * 4));
  CK(hipMemset(fl, 0, flush_n * 4));
  Ops o{rg, xc, xz, dy, drg, dxc, dxz};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned grid = (unsigned)(cus * 8);
  auto flush = [&]() {
    k_flush<<<grid, 256>>>(fl, flush_n, 1.0f);
  };
  struct V {
    const char* name;
    int nr, nw;
    bool dirty;
    void (*launch)(Ops, int64_t, int, unsigned);
  };
  auto timed = [&](void (*launch)(Ops, int64_t, int, unsigned), bool dirty) {
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
      flush();
      if (dirty) k_mix<0, 4><<<grid, 256>>>(o, M, H);   // 840 MB just written
      CK(hipEventRecord(e0, 0));
      launch(o, M, H, grid);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
  };
  const V vs[] = {
      {"5R+4W (gate-scan backward)", 5, 4, false,
       [](Ops o, int64_t M, int H, unsigned g) { k_mix<5, 4><<<g, 256>>>(o, M, H); }},
      {"5R+4W after 840 MB of writes", 5, 4, true,
       [](Ops o, int64_t M, int H, unsigned g) { k_mix<5, 4><<<g, 256>>>(o, M, H); }},
      {"4R+1W (gate-scan forward)", 4, 1, false,
       [](Ops o, int64_t M, int H, unsigned g) { k_mix<4, 1><<<g, 256>>>(o, M, H); }},
      {"5R", 5, 0, false,
       [](Ops o, int64_t M, int H, unsigned g) { k_mix<5, 0><<<g, 256>>>(o, M, H); }},
      {"4W", 0, 4, false,
       [](Ops o, int64_t M, int H, unsigned g) { k_mix<0, 4><<<g, 256>>>(o, M, H); }},
      {"1R+1W (copy)", 1, 1, false,
       [](Ops o, int64_t M, int H, unsigned g) { k_mix<1, 1><<<g, 256>>>(o, M, H); }},
  };
  printf("M=%lld H=%d grid=%u (fp32, 16 B per lane; bytes = streams x M x H x 4)\n",
         (long long)M, H, grid);
  for (const V& v : vs) {
    const double us = timed(v.launch, v.dirty);
    const double bytes = (double)(v.nr + v.nw) * M * H * 4;
    printf("%-30s %8.1f us  %6.0f MB  %5.2f TB/s  (%.3f of 8 TB/s)\n", v.name, us, bytes / 1e6,
           bytes / us / 1e6, bytes / us / 1e6 / 8.0);
  }
  return 0;
}
