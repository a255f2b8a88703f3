// patprobe.hip — the gate backward's data movement with trivial math: 5 reads
// (r, i from a [N, 2H] tensor, x [N, H], z = the second half of a [N, 2H]
// tensor, g [N, H]) and 4 writes (dr, di into [N, 2H], dx [N, H], dz into the
// second half of [N, 2H]) over B sequences of L rows, H = 256, fp32.
// Which access pattern sets the rate: a wave walking its sequence (Q time
// chunks x TC rows per tile, 128-B .. 1-KB row segments) or one-shot threads.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/patprobe.hip -o tools/bin/patprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4f ld(const float* p) {
  return NT ? __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p)) : *reinterpret_cast<const v4f*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(float* p, v4f v) {
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p)); else *reinterpret_cast<v4f*>(p) = v;
}

struct Bufs {
  const float *rg, *x, *z, *g;
  float *drg, *dx, *dz;
};

// walking wave: wave = (sequence b, channel window); lanes = Q row chunks x G groups
// TM: time-major rows (row of (b, t) = t * B + b) instead of b * L + t
template <int Q, int TC, bool NT, bool TM = false>
__global__ void __launch_bounds__(256) walk(Bufs p, int B, int L, int H, int ncw) {
  constexpr int G = 64 / Q;
  const int lane = threadIdx.x & 63;
  const int q = lane / G, g = lane % G;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = wid / ncw;
  if (b >= B) return;
  const int c = (int)(wid % ncw) * G * 4 + g * 4;
  const int64_t row0 = b * L;
  const int nT = (L + Q * TC - 1) / (Q * TC);
  for (int tile = nT - 1; tile >= 0; --tile) {
    v4f r[TC], i[TC], x[TC], z[TC], gg[TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int tt = std::min(tile * Q * TC + q * TC + j, L - 1);
      const int64_t t = TM ? (int64_t)tt * B + b : row0 + tt;
      r[j] = ld<NT>(p.rg + t * 2 * H + c);
      i[j] = ld<NT>(p.rg + t * 2 * H + H + c);
      x[j] = ld<NT>(p.x + t * H + c);
      z[j] = ld<NT>(p.z + t * 2 * H + H + c);
      gg[j] = ld<NT>(p.g + t * H + c);
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int tt = tile * Q * TC + q * TC + j;
      if (tt < L) {
        const int64_t t = TM ? (int64_t)tt * B + b : row0 + tt;
        st<NT>(p.drg + t * 2 * H + c, r[j] * x[j]);
        st<NT>(p.drg + t * 2 * H + H + c, i[j] + gg[j]);
        st<NT>(p.dx + t * H + c, z[j] * gg[j]);
        st<NT>(p.dz + t * 2 * H + H + c, x[j] - r[j]);
      }
    }
  }
}

// one-shot: one thread = one (row, 4 channels); consecutive threads along channels
template <bool NT>
__global__ void __launch_bounds__(256) oneshot(Bufs p, int64_t rows, int H) {
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t t = e / H;
  const int c = (int)(e % H);
  if (t >= rows) return;
  const v4f r = ld<NT>(p.rg + t * 2 * H + c), i = ld<NT>(p.rg + t * 2 * H + H + c);
  const v4f x = ld<NT>(p.x + t * H + c), z = ld<NT>(p.z + t * 2 * H + H + c), gg = ld<NT>(p.g + t * H + c);
  st<NT>(p.drg + t * 2 * H + c, r * x);
  st<NT>(p.drg + t * 2 * H + H + c, i + gg);
  st<NT>(p.dx + t * H + c, z * gg);
  st<NT>(p.dz + t * 2 * H + H + c, x - r);
}

// one-shot with the walking kernel's lane shape: one wave = Q rows x 4G channels
template <int Q, bool NT>
__global__ void __launch_bounds__(256) oneshot_q(Bufs p, int64_t rows, int H, int ncw) {
  constexpr int G = 64 / Q;
  const int lane = threadIdx.x & 63;
  const int q = lane / G, g = lane % G;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t t = (wid / ncw) * Q + q;
  const int c = (int)(wid % ncw) * G * 4 + g * 4;
  if (t >= rows) return;
  const v4f r = ld<NT>(p.rg + t * 2 * H + c), i = ld<NT>(p.rg + t * 2 * H + H + c);
  const v4f x = ld<NT>(p.x + t * H + c), z = ld<NT>(p.z + t * 2 * H + H + c), gg = ld<NT>(p.g + t * H + c);
  st<NT>(p.drg + t * 2 * H + c, r * x);
  st<NT>(p.drg + t * 2 * H + H + c, i + gg);
  st<NT>(p.dx + t * H + c, z * gg);
  st<NT>(p.dz + t * 2 * H + H + c, x - r);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 2048, L = argc > 2 ? atoi(argv[2]) : 200, H = 256;
  const int64_t N = (int64_t)B * L * H;
  auto alloc = [&](int64_t n) { float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemset(d, 0, n * 4)); return d; };
  Bufs p{alloc(2 * N), alloc(N), alloc(2 * N), alloc(N), alloc(2 * N), alloc(N), alloc(2 * N)};
  const double bytes = 9.0 * N * 4;
  struct C { std::string nm; std::function<void()> f; std::vector<float> ms; };
  std::vector<C> cs;
#define WALK(Q, TC, NT)                                                                     \
  {                                                                                         \
    const int ncw = H / ((64 / Q) * 4);                                                     \
    const int blocks = (int)(((int64_t)B * ncw + 3) / 4);                                   \
    cs.push_back({"walk Q" #Q " TC" #TC " nt" #NT, [=] { walk<Q, TC, NT><<<blocks, 256>>>(p, B, L, H, ncw); }, {}}); \
  }
#define WALKTM(Q, TC)                                                                       \
  {                                                                                         \
    const int ncw = H / ((64 / Q) * 4);                                                     \
    const int blocks = (int)(((int64_t)B * ncw + 3) / 4);                                   \
    cs.push_back({"walk time-major Q" #Q " TC" #TC, [=] { walk<Q, TC, true, true><<<blocks, 256>>>(p, B, L, H, ncw); }, {}}); \
  }
  WALKTM(8, 2) WALKTM(4, 4) WALKTM(1, 16)
  WALK(8, 2, true) WALK(8, 2, false) WALK(4, 4, true) WALK(2, 8, true) WALK(1, 16, true) WALK(8, 1, true) WALK(16, 1, true)
  cs.push_back({"oneshot nt", [=] { oneshot<true><<<(unsigned)(N / 4 / 256), 256>>>(p, (int64_t)B * L, H); }, {}});
  cs.push_back({"oneshot", [=] { oneshot<false><<<(unsigned)(N / 4 / 256), 256>>>(p, (int64_t)B * L, H); }, {}});
#define OSQ(Q)                                                                               \
  {                                                                                          \
    const int ncw = H / ((64 / Q) * 4);                                                      \
    const int64_t waves = ((int64_t)B * L / Q) * ncw;                                        \
    cs.push_back({"oneshot Q" #Q " nt", [=] { oneshot_q<Q, true><<<(unsigned)((waves + 3) / 4), 256>>>(p, (int64_t)B * L, H, ncw); }, {}}); \
  }
  OSQ(8) OSQ(4) OSQ(1)
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& c : cs) c.f();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < 9; ++r)
    for (auto& c : cs) {
      CK(hipEventRecord(e0, 0)); c.f(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float t; CK(hipEventElapsedTime(&t, e0, e1)); c.ms.push_back(t);
    }
  printf("B=%d L=%d H=%d (5R+4W, %.0f MB)\n", B, L, H, bytes / 1e6);
  for (auto& c : cs) {
    std::sort(c.ms.begin(), c.ms.end());
    const double t = c.ms[c.ms.size() / 2];
    printf("%-22s %8.1f us  %.3f of 8 TB/s\n", c.nm.c_str(), t * 1e3, bytes / (t * 1e-3) / 8e12);
  }
  return 0;
}
