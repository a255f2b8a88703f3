// streambench.hip — the gate backward's 5-read / 4-write access pattern
// (r, i, xc, z, dy -> dr, di, dxc, dz at the encoder's row strides) under
// different wave/lane mappings, trivial arithmetic, beside plain copies.
// Which mapping the memory system rewards decides the layout of
// k_gate_scan_bwd.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/streambench.hip -o tools/bin/streambench
//   tools/bin/streambench [ntok=204800] [H=256] [reps=15]
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
__device__ __forceinline__ void st4(float* p, f4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p));
  else *reinterpret_cast<f4*>(p) = v;
}
__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

struct Bufs {
  const float *rg, *xc, *xz, *dy;
  float *drg, *dxc, *dxz;
  int64_t ntok;
  int H;
};

// (1) the kernel's mapping: a wave = one sequence x 32 channels; lane = (time
// chunk q of 8, channel group g of 8), 4 channels per lane; a load
// instruction covers 8 rows x 128 B.  Sequences of L rows, walked in reverse
// 16-row tiles.
template <bool NT>
__global__ void __launch_bounds__(256) p_seq(Bufs b, int L) {
  const int H = b.H;
  const int lane = threadIdx.x & 63, q = lane & 7, g = lane >> 3;
  const int ncw = H / 32;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t s = wid / ncw;
  if (s * L >= b.ntok) return;
  const int c0 = (int)(wid - s * ncw) * 32 + g * 4;
  const int64_t row0 = s * L;
  for (int tile = (L + 15) / 16 - 1; tile >= 0; --tile) {
    f4 r[2], i[2], x[2], z[2], d[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t t = row0 + min(tile * 16 + q * 2 + j, L - 1);
      r[j] = ld4(b.rg + t * 2 * H + c0);
      i[j] = ld4(b.rg + t * 2 * H + H + c0);
      x[j] = ld4(b.xc + t * H + c0);
      z[j] = ld4(b.xz + t * 2 * H + H + c0);
      d[j] = ld4(b.dy + t * H + c0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tt = tile * 16 + q * 2 + j;
      if (tt >= L) continue;
      const int64_t t = row0 + tt;
      st4<NT>(b.dxz + t * 2 * H + H + c0, z[j] * d[j]);
      st4<NT>(b.drg + t * 2 * H + c0, r[j] * d[j]);
      st4<NT>(b.drg + t * 2 * H + H + c0, i[j] * d[j]);
      st4<NT>(b.dxc + t * H + c0, x[j] * d[j]);
    }
  }
}

// (1b) the kernel's mapping generalised: lane = (time chunk q of Q, channel
// group g of G = 64/Q), 4 channels per lane, a wave = one sequence x 4G
// channels walking reverse tiles of Q*TC rows; a load instruction covers Q
// rows x 16G bytes.  Q = 1: whole 1 KB rows, one wave per sequence (x H/256).
template <int Q, int TC, bool NT>
__global__ void __launch_bounds__(256) p_seqq(Bufs b, int L) {
  constexpr int G = 64 / Q;
  const int H = b.H;
  const int lane = threadIdx.x & 63, q = lane % Q, g = lane / Q;
  const int ncw = H / (4 * G);
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t s = wid / ncw;
  if (s * L >= b.ntok) return;
  const int c0 = (int)(wid - s * ncw) * 4 * G + g * 4;
  const int64_t row0 = s * L;
  constexpr int TILE = Q * TC;
  for (int tile = (L + TILE - 1) / TILE - 1; tile >= 0; --tile) {
    f4 r[TC], i[TC], x[TC], z[TC], d[TC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int64_t t = row0 + min(tile * TILE + q * TC + j, L - 1);
      r[j] = ld4(b.rg + t * 2 * H + c0);
      i[j] = ld4(b.rg + t * 2 * H + H + c0);
      x[j] = ld4(b.xc + t * H + c0);
      z[j] = ld4(b.xz + t * 2 * H + H + c0);
      d[j] = ld4(b.dy + t * H + c0);
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int tt = tile * TILE + q * TC + j;
      if (tt >= L) continue;
      const int64_t t = row0 + tt;
      st4<NT>(b.dxz + t * 2 * H + H + c0, z[j] * d[j]);
      st4<NT>(b.drg + t * 2 * H + c0, r[j] * d[j]);
      st4<NT>(b.drg + t * 2 * H + H + c0, i[j] * d[j]);
      st4<NT>(b.dxc + t * H + c0, x[j] * d[j]);
    }
  }
}

// (2) row-wide waves: lane = 4 channels of 256 (one wave instruction = one
// whole 1 KB row segment of a stream); a wave owns RW consecutive rows and
// walks them TS at a time (TS rows x 5 loads in flight per lane).
template <int TS, bool NT, bool REV>
__global__ void __launch_bounds__(256) p_row(Bufs b, int RW) {
  const int H = b.H;
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t r0 = wid * RW;
  if (r0 >= b.ntok) return;
  const int64_t r1 = min<int64_t>(r0 + RW, b.ntok);
  for (int cb = 0; cb < H; cb += 256) {
    const int c0 = cb + lane * 4;
    for (int64_t k = 0; k < r1 - r0; k += TS) {
      f4 r[TS], i[TS], x[TS], z[TS], d[TS];
#pragma unroll
      for (int j = 0; j < TS; ++j) {
        int64_t t = REV ? r1 - 1 - (k + j) : r0 + k + j;
        t = REV ? max(t, r0) : min(t, r1 - 1);
        r[j] = ld4(b.rg + t * 2 * H + c0);
        i[j] = ld4(b.rg + t * 2 * H + H + c0);
        x[j] = ld4(b.xc + t * H + c0);
        z[j] = ld4(b.xz + t * 2 * H + H + c0);
        d[j] = ld4(b.dy + t * H + c0);
      }
#pragma unroll
      for (int j = 0; j < TS; ++j) {
        if (k + j >= r1 - r0) continue;
        const int64_t t = REV ? r1 - 1 - (k + j) : r0 + k + j;
        st4<NT>(b.dxz + t * 2 * H + H + c0, z[j] * d[j]);
        st4<NT>(b.drg + t * 2 * H + c0, r[j] * d[j]);
        st4<NT>(b.drg + t * 2 * H + H + c0, i[j] * d[j]);
        st4<NT>(b.dxc + t * H + c0, x[j] * d[j]);
      }
    }
  }
}

// (3) row-wide waves with loads of the next TS rows issued before the stores
// of the current ones (two register buffers)
template <int TS, bool NT>
__global__ void __launch_bounds__(256) p_row_pf(Bufs b, int RW) {
  const int H = b.H;
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t r0 = wid * RW;
  if (r0 >= b.ntok) return;
  const int64_t r1 = min<int64_t>(r0 + RW, b.ntok);
  const int c0 = lane * 4;
  f4 r[2][TS], i[2][TS], x[2][TS], z[2][TS], d[2][TS];
  auto load = [&](int buf, int64_t k) {
#pragma unroll
    for (int j = 0; j < TS; ++j) {
      const int64_t t = min(r0 + k + j, r1 - 1);
      r[buf][j] = ld4(b.rg + t * 2 * H + c0);
      i[buf][j] = ld4(b.rg + t * 2 * H + H + c0);
      x[buf][j] = ld4(b.xc + t * H + c0);
      z[buf][j] = ld4(b.xz + t * 2 * H + H + c0);
      d[buf][j] = ld4(b.dy + t * H + c0);
    }
  };
  auto store = [&](int buf, int64_t k) {
#pragma unroll
    for (int j = 0; j < TS; ++j) {
      if (r0 + k + j >= r1) continue;
      const int64_t t = r0 + k + j;
      st4<NT>(b.dxz + t * 2 * H + H + c0, z[buf][j] * d[buf][j]);
      st4<NT>(b.drg + t * 2 * H + c0, r[buf][j] * d[buf][j]);
      st4<NT>(b.drg + t * 2 * H + H + c0, i[buf][j] * d[buf][j]);
      st4<NT>(b.dxc + t * H + c0, x[buf][j] * d[buf][j]);
    }
  };
  const int64_t n = r1 - r0;
  load(0, 0);
  for (int64_t k = 0; k < n; k += 2 * TS) {
    if (k + TS < n) load(1, k + TS);
    store(0, k);
    if (k + TS < n) {
      if (k + 2 * TS < n) load(0, k + 2 * TS);
      store(1, k + TS);
    }
  }
}

// references: float4 copy (1R 1W) and the forward's 4R 1W at the same strides
template <bool NT>
__global__ void __launch_bounds__(256) p_copy(const float* a, float* o, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    st4<NT>(o + 4 * i, ld4(a + 4 * i));
}
template <bool NT>
__global__ void __launch_bounds__(256) p_4r1w(Bufs b, int RW) {
  const int H = b.H;
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t r0 = wid * RW;
  if (r0 >= b.ntok) return;
  const int64_t r1 = min<int64_t>(r0 + RW, b.ntok);
  const int c0 = lane * 4;
  for (int64_t k = 0; k < r1 - r0; k += 4) {
    f4 r[4], i[4], x[4], z[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t t = min(r0 + k + j, r1 - 1);
      r[j] = ld4(b.rg + t * 2 * H + c0);
      i[j] = ld4(b.rg + t * 2 * H + H + c0);
      x[j] = ld4(b.xc + t * H + c0);
      z[j] = ld4(b.xz + t * 2 * H + H + c0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (k + j < r1 - r0) st4<NT>(b.dxc + (r0 + k + j) * H + c0, r[j] * i[j] + x[j] * z[j]);
  }
}

__global__ void fill(float* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    p[i] = (float)(i % 97) * 0.01f;
}

int main(int argc, char** argv) {
  const int64_t ntok = argc > 1 ? atoll(argv[1]) : 204800;
  const int H = argc > 2 ? atoi(argv[2]) : 256;
  const int reps = argc > 3 ? atoi(argv[3]) : 15;
  float *rg, *xc, *xz, *dy, *drg, *dxc, *dxz;
  CK(hipMalloc(&rg, ntok * 2 * H * 4));
  CK(hipMalloc(&xc, ntok * H * 4));
  CK(hipMalloc(&xz, ntok * 2 * H * 4));
  CK(hipMalloc(&dy, ntok * H * 4));
  CK(hipMalloc(&drg, ntok * 2 * H * 4));
  CK(hipMalloc(&dxc, ntok * H * 4));
  CK(hipMalloc(&dxz, ntok * 2 * H * 4));
  for (auto [p, n] : {std::pair<float*, int64_t>{rg, ntok * 2 * H}, {xc, ntok * H},
                      {xz, ntok * 2 * H}, {dy, ntok * H}})
    fill<<<4096, 256>>>(p, n);
  CK(hipDeviceSynchronize());
  Bufs b{rg, xc, xz, dy, drg, dxc, dxz, ntok, H};
  const double n9 = 9.0 * ntok * H * 4, n5 = 5.0 * ntok * H * 4;
  struct Case {
    std::string name;
    double bytes;
    std::function<void()> f;
  };
  std::vector<Case> cs;
  auto grid = [](int64_t waves) { return dim3((unsigned)((waves + 3) / 4)); };
  for (int L : {100, 200}) {
    const int64_t waves = (ntok / L) * (H / 32);
    cs.push_back({"seq L=" + std::to_string(L) + " (kernel layout)", n9,
                  [=] { p_seq<true><<<grid(waves), 256>>>(b, L); }});
    cs.push_back({"seq L=" + std::to_string(L) + " plain stores", n9,
                  [=] { p_seq<false><<<grid(waves), 256>>>(b, L); }});
  }
  {
    const int L = 100;
    auto add = [&](const char* nm, auto kern, int Q) {
      const int64_t waves = (ntok / L) * (H / (4 * (64 / Q)));
      cs.push_back({std::string(nm), n9, [=] { kern<<<grid(waves), 256>>>(b, L); }});
    };
    add("seqq Q=8 TC=2", p_seqq<8, 2, true>, 8);
    add("seqq Q=8 TC=4", p_seqq<8, 4, true>, 8);
    add("seqq Q=4 TC=4", p_seqq<4, 4, true>, 4);
    add("seqq Q=4 TC=2", p_seqq<4, 2, true>, 4);
    add("seqq Q=2 TC=4", p_seqq<2, 4, true>, 2);
    add("seqq Q=2 TC=8", p_seqq<2, 8, true>, 2);
    add("seqq Q=1 TC=4", p_seqq<1, 4, true>, 1);
    add("seqq Q=1 TC=8", p_seqq<1, 8, true>, 1);
    add("seqq Q=16 TC=1", p_seqq<16, 1, true>, 16);
    add("seqq Q=16 TC=2", p_seqq<16, 2, true>, 16);
  }
  for (int RW : {8, 16, 32}) {
    const int64_t waves = (ntok + RW - 1) / RW;
    cs.push_back({"row RW=" + std::to_string(RW) + " TS=2 nt", n9,
                  [=] { p_row<2, true, false><<<grid(waves), 256>>>(b, RW); }});
    cs.push_back({"row RW=" + std::to_string(RW) + " TS=4 nt", n9,
                  [=] { p_row<4, true, false><<<grid(waves), 256>>>(b, RW); }});
    cs.push_back({"row RW=" + std::to_string(RW) + " TS=4 plain", n9,
                  [=] { p_row<4, false, false><<<grid(waves), 256>>>(b, RW); }});
    cs.push_back({"row RW=" + std::to_string(RW) + " TS=4 nt rev", n9,
                  [=] { p_row<4, true, true><<<grid(waves), 256>>>(b, RW); }});
    cs.push_back({"row_pf RW=" + std::to_string(RW) + " TS=2 nt", n9,
                  [=] { p_row_pf<2, true><<<grid(waves), 256>>>(b, RW); }});
    cs.push_back({"row_pf RW=" + std::to_string(RW) + " TS=4 nt", n9,
                  [=] { p_row_pf<4, true><<<grid(waves), 256>>>(b, RW); }});
  }
  cs.push_back({"copy 1R1W nt", 2.0 * ntok * 2 * H * 4,
                [=] { p_copy<true><<<8192, 256>>>(rg, drg, ntok * 2 * H / 4); }});
  cs.push_back({"copy 1R1W plain", 2.0 * ntok * 2 * H * 4,
                [=] { p_copy<false><<<8192, 256>>>(rg, drg, ntok * 2 * H / 4); }});
  cs.push_back({"4R1W row RW=16 nt", n5,
                [=] { p_4r1w<true><<<grid((ntok + 15) / 16), 256>>>(b, 16); }});
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < 2; ++round) {
    for (auto& c : cs) {
      c.f();
      CK(hipDeviceSynchronize());
      std::vector<float> ts;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        c.f();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const float ms = ts[ts.size() / 2];
      printf("round %d  %-34s %8.1f us  %7.1f GB/s  frac %.3f\n", round, c.name.c_str(), ms * 1e3,
             c.bytes / (ms * 1e-3) / 1e9, c.bytes / (ms * 1e-3) / 1e9 / 8000.0);
      fflush(stdout);
    }
  }
  return 0;
}
