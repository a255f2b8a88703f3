// flat5to4.hip — is the gate backward's 5-read / 4-write rate (0.60-0.66 of
// 8 TB/s for rb_gate_scan_bwd and its own access pattern) a
// property of the kernel's layout or of moving nine streams with four of them
// written?  Times the same bytes ([N, H] fp32 streams, B = 2048, L = 200,
// H = 256 dense) in layouts from the most streaming-friendly to the kernel's:
//   copy      1R + 1W float4, grid-stride (the guide's ceiling, 0.79)
//   sep9      5 + 4 separate contiguous arrays, float4 grid-stride
//   strided   the kernel's buffers and row strides (rg [N, 2H] = r | i,
//             z at +H of xz [N, 2H], drg [N, 2H], dz at +H of dxz), a wave per
//             1-KB row, grid-stride over rows in order
//   rowsrev   as strided, each wave walking its own 200-row sequence backwards
//             (the kernel's time order), one row per step
//   seqQ8     the kernel's lane layout (8 time chunks x 8 channel groups of 4,
//             tiles of 16 steps walked backwards: tools/kbench.hip pattern5to4)
//   5R1W / 1R4W  read-heavy and write-heavy halves of sep9
// each with default-policy, nontemporal and mixed (nt loads / plain stores and
// the reverse) accesses.  Timing only.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/flat5to4.hip -o tools/bin/flat5to4
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
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

template <bool NT>
__device__ __forceinline__ f4 ld_(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st_(f4 v, f4* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

#define ld ld_<(NT == 1 || NT == 2)>
#define st st_<(NT == 1 || NT == 3)>

template <int NT>
__global__ void __launch_bounds__(256) k_copy(const f4* a, f4* o, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x)
    st(ld(a + i), o + i);
}

struct Sep {
  const f4* in[5];
  f4* out[4];
};

template <int NT, int NR, int NW>
__global__ void __launch_bounds__(256) k_sep(Sep s, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    f4 acc = ld(s.in[0] + i);
#pragma unroll
    for (int k = 1; k < NR; ++k) acc += ld(s.in[k] + i);
#pragma unroll
    for (int k = 0; k < NW; ++k) st(acc * (float)(k + 1), s.out[k] + i);
  }
}

// the kernel's buffers: rows of H channels, 64 lanes x 4 channels = one row
struct Bufs {
  const float *rg, *xz, *xc, *dy;
  float *drg, *dxc, *dxz;
};

template <int NT>
__device__ __forceinline__ void row_step(const Bufs& b, int64_t t, int c, int H) {
  const f4 r = ld((const f4*)(b.rg + t * 2 * H + c));
  const f4 i = ld((const f4*)(b.rg + t * 2 * H + H + c));
  const f4 x = ld((const f4*)(b.xc + t * H + c));
  const f4 z = ld((const f4*)(b.xz + t * 2 * H + H + c));
  const f4 d = ld((const f4*)(b.dy + t * H + c));
  st(r * d, (f4*)(b.drg + t * 2 * H + c));
  st(i * d, (f4*)(b.drg + t * 2 * H + H + c));
  st(x * d, (f4*)(b.dxc + t * H + c));
  st(z * d, (f4*)(b.dxz + t * 2 * H + H + c));
}

// grid-stride over rows in order, a wave per row (H = 256)
template <int NT>
__global__ void __launch_bounds__(256) k_strided(Bufs b, int64_t rows, int H) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t t = w0; t < rows; t += nw) row_step<NT>(b, t, lane * 4, H);
}

// a wave per sequence of L rows, walked backwards one row per step
template <int NT>
__global__ void __launch_bounds__(256) k_rowsrev(Bufs b, int64_t B, int L, int H) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= B) return;
  for (int j = L - 1; j >= 0; --j) row_step<NT>(b, s * L + j, lane * 4, H);
}

// a wave per sequence, 4 rows per step (all loads of the 4 rows, then the
// stores), backwards
template <int NT>
__global__ void __launch_bounds__(256) k_rowsrev4(Bufs b, int64_t B, int L, int H) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= B) return;
  const int c = lane * 4;
  for (int j0 = L - 4; j0 > -4; j0 -= 4) {
    f4 r[4], i[4], x[4], z[4], d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t t = s * L + max(j0 + u, 0);
      r[u] = ld((const f4*)(b.rg + t * 2 * H + c));
      i[u] = ld((const f4*)(b.rg + t * 2 * H + H + c));
      x[u] = ld((const f4*)(b.xc + t * H + c));
      z[u] = ld((const f4*)(b.xz + t * 2 * H + H + c));
      d[u] = ld((const f4*)(b.dy + t * H + c));
    }
#pragma unroll
    for (int u = 3; u >= 0; --u) {
      if (j0 + u < 0) continue;
      const int64_t t = s * L + j0 + u;
      st(r[u] * d[u], (f4*)(b.drg + t * 2 * H + c));
      st(i[u] * d[u], (f4*)(b.drg + t * 2 * H + H + c));
      st(x[u] * d[u], (f4*)(b.dxc + t * H + c));
      st(z[u] * d[u], (f4*)(b.dxz + t * 2 * H + H + c));
    }
  }
}

// the kernel's lane layout: lane = g * Q + q, q one of Q time chunks of TC
// steps, g one of 64 / Q groups of 4 channels; tiles of Q * TC steps walked
// backwards (tools/kbench.hip pattern5to4)
template <int NT, int Q, int TC>
__global__ void __launch_bounds__(256) k_seq(Bufs b, int64_t B, int L, int H, int ncw) {
  constexpr int G = 64 / Q, TILE = Q * TC;
  const int lane = threadIdx.x & 63, q = lane & (Q - 1), g = lane / Q;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t s = wid / ncw;
  if (s >= B) return;
  const int c = (int)(wid - s * ncw) * (G * 4) + g * 4;
  const int nT = (L + TILE - 1) / TILE;
  for (int tile = nT - 1; tile >= 0; --tile) {
    const int t0 = tile * TILE + q * TC;
    f4 r[TC], i[TC], x[TC], z[TC], d[TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int64_t t = s * L + min(t0 + j, L - 1);
      r[j] = ld((const f4*)(b.rg + t * 2 * H + c));
      i[j] = ld((const f4*)(b.rg + t * 2 * H + H + c));
      x[j] = ld((const f4*)(b.xc + t * H + c));
      z[j] = ld((const f4*)(b.xz + t * 2 * H + H + c));
      d[j] = ld((const f4*)(b.dy + t * H + c));
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      if (t0 + j >= L) continue;
      const int64_t t = s * L + t0 + j;
      st(r[j] * d[j], (f4*)(b.drg + t * 2 * H + c));
      st(i[j] * d[j], (f4*)(b.drg + t * 2 * H + H + c));
      st(x[j] * d[j], (f4*)(b.dxc + t * H + c));
      st(z[j] * d[j], (f4*)(b.dxz + t * 2 * H + H + c));
    }
  }
}

// the kernel layout with W waves per workgroup (W = 8: the workgroup spans
// whole 1-KB rows of one sequence) and optionally a barrier after each tile
// (the workgroup's stores of a tile issued together)
template <int NT, int Q, int TC, int W, bool BAR>
__global__ void __launch_bounds__(64 * W) k_seqw(Bufs b, int64_t B, int L, int H, int ncw) {
  constexpr int G = 64 / Q, TILE = Q * TC;
  const int lane = threadIdx.x & 63, q = lane & (Q - 1), g = lane / Q;
  const int64_t wid = (int64_t)blockIdx.x * W + (threadIdx.x >> 6);
  const int64_t s = wid / ncw;
  if (s >= B) return;   // whole workgroups (B * ncw % W == 0 here)
  const int c = (int)(wid - s * ncw) * (G * 4) + g * 4;
  const int nT = (L + TILE - 1) / TILE;
  for (int tile = nT - 1; tile >= 0; --tile) {
    const int t0 = tile * TILE + q * TC;
    f4 r[TC], i[TC], x[TC], z[TC], d[TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int64_t t = s * L + min(t0 + j, L - 1);
      r[j] = ld((const f4*)(b.rg + t * 2 * H + c));
      i[j] = ld((const f4*)(b.rg + t * 2 * H + H + c));
      x[j] = ld((const f4*)(b.xc + t * H + c));
      z[j] = ld((const f4*)(b.xz + t * 2 * H + H + c));
      d[j] = ld((const f4*)(b.dy + t * H + c));
    }
    if (BAR) __syncthreads();
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      if (t0 + j >= L) continue;
      const int64_t t = s * L + t0 + j;
      st(r[j] * d[j], (f4*)(b.drg + t * 2 * H + c));
      st(i[j] * d[j], (f4*)(b.drg + t * 2 * H + H + c));
      st(x[j] * d[j], (f4*)(b.dxc + t * H + c));
      st(z[j] * d[j], (f4*)(b.dxz + t * 2 * H + H + c));
    }
  }
}

__global__ void fill(float* p, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    p[i] = (h & 0xffff) / 65536.0f - 0.5f;
  }
}

struct Case {
  std::string name;
  double bytes;
  std::function<void()> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 2048, L = argc > 2 ? atoi(argv[2]) : 200;
  const int rounds = argc > 3 ? atoi(argv[3]) : 11;
  constexpr int H = 256;
  const int64_t rows = (int64_t)B * L, n = rows * H, n4 = n / 4;
  auto alloc = [&](int64_t cnt, uint32_t seed) {
    float* p;
    CK(hipMalloc(&p, cnt * 4));
    hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, p, cnt, seed);
    return p;
  };
  // separate arrays for sep9
  Sep s{};
  for (int k = 0; k < 5; ++k) s.in[k] = (const f4*)alloc(n, 10 + k);
  for (int k = 0; k < 4; ++k) s.out[k] = (f4*)alloc(n, 20 + k);
  Bufs b{alloc(2 * n, 1), alloc(2 * n, 2), alloc(n, 3), alloc(n, 4),
         alloc(2 * n, 5), alloc(n, 6), alloc(2 * n, 7)};
  CK(hipDeviceSynchronize());
  const double S = (double)n * 4;
  const int grid = 256 * 8;
  std::vector<Case> cs;
  // policies: 0 plain, 1 nt, 2 nt loads + plain stores, 3 plain loads + nt stores
  static const char* pol[4] = {" plain", " nt", " ntL plainS", " plainL ntS"};
  auto all4 = [&](const char* nm, double bytes, std::function<void(int)> f) {
    for (int k = 0; k < 4; ++k) cs.push_back({std::string(nm) + pol[k], bytes, [=] { f(k); }, {}});
  };
#define DISPATCH(KER, GRID, ...)                                                            \
  [=](int k) {                                                                              \
    if (k == 0) hipLaunchKernelGGL(KER(0), dim3(GRID), dim3(256), 0, 0, __VA_ARGS__);       \
    else if (k == 1) hipLaunchKernelGGL(KER(1), dim3(GRID), dim3(256), 0, 0, __VA_ARGS__);  \
    else if (k == 2) hipLaunchKernelGGL(KER(2), dim3(GRID), dim3(256), 0, 0, __VA_ARGS__);  \
    else hipLaunchKernelGGL(KER(3), dim3(GRID), dim3(256), 0, 0, __VA_ARGS__);              \
  }
#define K_COPY(p) k_copy<p>
#define K_SEP54(p) k_sep<p, 5, 4>
#define K_SEP51(p) k_sep<p, 5, 1>
#define K_SEP14(p) k_sep<p, 1, 4>
#define K_STR(p) k_strided<p>
#define K_REV(p) k_rowsrev<p>
#define K_REV4(p) k_rowsrev4<p>
#define K_SEQ8(p) k_seq<p, 8, 2>
#define K_SEQ1(p) k_seq<p, 1, 4>
  all4("copy 1R1W", 2 * S, DISPATCH(K_COPY, grid, s.in[0], s.out[0], n4));
  all4("sep9 5R4W", 9 * S, DISPATCH(K_SEP54, grid, s, n4));
  all4("sep 5R1W", 6 * S, DISPATCH(K_SEP51, grid, s, n4));
  all4("sep 1R4W", 5 * S, DISPATCH(K_SEP14, grid, s, n4));
  all4("strided rows", 9 * S, DISPATCH(K_STR, grid, b, rows, H));
  const unsigned gB = (unsigned)((B + 3) / 4);
  all4("rowsrev x1", 9 * S, DISPATCH(K_REV, gB, b, (int64_t)B, L, H));
  all4("rowsrev x4", 9 * S, DISPATCH(K_REV4, gB, b, (int64_t)B, L, H));
  const int ncw8 = H / 32;
  const unsigned g8 = (unsigned)(((int64_t)B * ncw8 + 3) / 4);
  all4("seq q8 tc2 (kernel layout)", 9 * S, DISPATCH(K_SEQ8, g8, b, (int64_t)B, L, H, ncw8));
  // workgroup width and per-tile barriers (policy: nt, the kernel's)
#define SEQW(W, BAR)                                                                         \
  cs.push_back({"seq q8 tc2 wg" #W " bar" #BAR " nt", 9 * S, [=] {                          \
    hipLaunchKernelGGL((k_seqw<1, 8, 2, W, BAR>), dim3((unsigned)(((int64_t)B * ncw8 + W - 1) / W)), \
                       dim3(64 * W), 0, 0, b, (int64_t)B, L, H, ncw8);                       \
  }, {}})
  SEQW(4, false);
  SEQW(4, true);
  SEQW(8, false);
  SEQW(8, true);
  SEQW(2, false);
  SEQW(16, true);
  const int ncw1 = H / 256;
  const unsigned g1 = (unsigned)(((int64_t)B * ncw1 + 3) / 4);
  all4("seq q1 tc4 (row-wide)", 9 * S, DISPATCH(K_SEQ1, g1, b, (int64_t)B, L, H, ncw1));
  if (getenv("F54_WG_ONLY")) {   // the workgroup-width sweep only (+ references)
    std::vector<Case> keep;
    for (auto& c : cs)
      if (c.name.find("wg") != std::string::npos || c.name.find("copy 1R1W nt") != std::string::npos ||
          c.name == "seq q8 tc2 (kernel layout) nt")
        keep.push_back(c);
    cs.swap(keep);
  }

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& c : cs) c.run();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (auto& c : cs) {
      CK(hipEventRecord(e0, 0));
      c.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      c.ms.push_back(ms);
    }
  CK(hipGetLastError());
  printf("B=%d L=%d H=%d dense, [N, H] fp32 streams of %.0f MB (median of %d)\n", B, L, H, S / 1e6,
         rounds);
  for (auto& c : cs) {
    std::sort(c.ms.begin(), c.ms.end());
    const double med = c.ms[c.ms.size() / 2];
    printf("%-34s %8.1f us  %.3f of 8 TB/s\n", c.name.c_str(), med * 1e3,
           c.bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
