// kbench.hip — standalone variant sweep of the channel-last kernels at the
// benchmark shape (B=2048, L=200, H=256 by default).  Includes the kernel
// sources directly so every template variant can be instantiated and timed
// with hipEvents in one process (interleaved rounds, median).
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 \
//       -I include tools/kbench.hip -o tools/kbench && tools/kbench [B L H]
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
#include "../datamining_recblr_amd/csrc/pack.hip"
#include "../datamining_recblr_amd/csrc/probe.hip"
#include "../datamining_recblr_amd/csrc/gemm_small.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

using namespace rb;

struct Case {
  const char* name;
  double bytes;
  std::function<void()> run;
  std::vector<float> ms;
};

__global__ void fill(float* p, int64_t n, uint32_t seed, float lo, float hi) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = lo + (hi - lo) * (h & 0xffffff) / 16777216.0f;
  }
}

static float* dalloc(int64_t n, uint32_t seed, float lo = -1.f, float hi = 1.f) {
  float* p;
  CK(hipMalloc(&p, n * sizeof(float)));
  hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, p, n, seed, lo, hi);
  return p;
}

struct GateBufs {
  float *rg, *xc, *z, *y, *car, *dy, *drg, *dxc, *dz, *part, *dh0, *lam;
  int rg_rs, xc_rs, z_rs, drg_rs, dxc_rs, dz_rs;
};

// T: activation storage (float, or bf16_t reading the same buffers as bf16
// for timing); which = 1 fwd, 2 bwd, 3 both
template <typename T, int VEC, int Q, int TC, bool PF = false>
void add_gate(std::vector<Case>& cs, const char* nm, int B, int L, int H, GateBufs g, double N,
              int which = 3) {
  constexpr int G = 64 / Q;
  const int ncw = (H + G * VEC - 1) / (G * VEC);
  const int64_t blocks = ((int64_t)B * ncw + 3) / 4;
  const double es = sizeof(T);
  auto A = [](float* p) { return reinterpret_cast<T*>(p); };
  if (which & 1) {
    char* f = (char*)malloc(64);
    snprintf(f, 64, "gate_fwd %s", nm);
    cs.push_back({f, 5 * N * es, [=] {
      hipLaunchKernelGGL((k_gate_scan_fwd<T, VEC, Q, TC, PF>), dim3(blocks), dim3(256), 0, 0,
                         A(g.rg), g.rg_rs, A(g.xc), g.xc_rs, A(g.z), g.z_rs, g.lam, nullptr,
                         nullptr, 0, A(g.y), H, g.car, (int64_t)B, L, H, ncw, nullptr, (T*)nullptr);
    }, {}});
  }
  if (which & 2) {
    char* f2 = (char*)malloc(64);
    snprintf(f2, 64, "gate_bwd %s", nm);
    cs.push_back({f2, 9 * N * es, [=] {
      hipLaunchKernelGGL((k_gate_scan_bwd<T, VEC, Q, TC, PF>), dim3(blocks), dim3(256), 0, 0,
                         A(g.rg), g.rg_rs, A(g.xc), g.xc_rs, A(g.z), g.z_rs, g.lam, nullptr, g.car,
                         A(g.dy), A(g.drg), g.drg_rs, A(g.dxc), g.dxc_rs, A(g.dz), g.dz_rs, g.part,
                         g.dh0, (int64_t)B, L, H, ncw, nullptr, 0, (const T*)nullptr);
    }, {}});
  }
}

template <typename T, int K, int VEC, int Q, int TC, bool PF = false>
void add_conv(std::vector<Case>& cs, const char* nm, int B, int L, int H, float* x, float* w,
              float* bias, float* xc, float* g1, float* dx, float* dwp, float* dbp, double N,
              int which = 3) {
  constexpr int G = 64 / Q;
  const int ncw = (H + G * VEC - 1) / (G * VEC);
  const int ntile = (L + Q * TC - 1) / (Q * TC);
  const double es = sizeof(T);
  auto A = [](float* p) { return reinterpret_cast<T*>(p); };
  if (which & 1) {
    char* f = (char*)malloc(64);
    snprintf(f, 64, "conv_fwd %s", nm);
    cs.push_back({f, 2 * N * es, [=] {
      const int64_t blocks = ((int64_t)B * ncw * ntile + 3) / 4;
      hipLaunchKernelGGL((k_conv_silu_fwd<T, K, VEC, Q, TC>), dim3(blocks), dim3(256), 0, 0,
                         A(x), 2 * H, w, bias, A(xc), H, (int64_t)B, L, H, ncw, ntile, nullptr);
    }, {}});
  }
  if (which & 2) {
    char* f2 = (char*)malloc(64);
    snprintf(f2, 64, "conv_bwd %s", nm);
    cs.push_back({f2, 3 * N * es, [=] {
      const int64_t blocks = ((int64_t)B * ncw + 3) / 4;
      hipLaunchKernelGGL((k_conv_silu_bwd<T, K, VEC, Q, TC, PF>), dim3(blocks), dim3(256), 0, 0,
                         A(x), 2 * H, w, bias, A(g1), (const T*)nullptr, A(dx), 2 * H, dwp, dbp,
                         (int64_t)B, L, H, ncw, nullptr);
    }, {}});
  }
}

// pure 1R+1W float4 copy (the guide's copy ceiling)
__global__ void copy4(const float4* a, float4* o, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x)
    o[i] = a[i];
}

// pure data movement: 4 reads + 1 write per element, flat float4 grid-stride
__global__ void flat4to1(const float4* a, const float4* b, const float4* c, const float4* d,
                         float4* o, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 x = a[i], y = b[i], z = c[i], w = d[i];
    o[i] = make_float4(x.x + y.x + z.x + w.x, x.y + y.y + z.y + w.y, x.z + y.z + z.z + w.z,
                       x.w + y.w + z.w + w.w);
  }
}

// same wave/lane layout and row strides as k_gate_scan_fwd, trivial math
template <int Q, int TC>
__global__ void __launch_bounds__(256)
pattern4to1(const float* rg, int rg_rs, const float* xc, int xc_rs, const float* z, int z_rs,
            float* y, int y_rs, int64_t B, int L, int H, int ncw) {
  constexpr int G = 64 / Q, VEC = 4, TILE = Q * TC;
  const int lane = threadIdx.x & 63, q = lane / G, g = lane - q * G;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = wid / ncw;
  if (b >= B) return;
  const int c0 = (int)(wid - b * ncw) * (G * VEC) + g * VEC;
  const int64_t row0 = b * L;
  const float* rgb = rg + row0 * rg_rs + c0;
  const float* xcb = xc + row0 * xc_rs + c0;
  const float* zb = z + row0 * z_rs + c0;
  float* yb = y + row0 * y_rs + c0;
  const int nT = (L + TILE - 1) / TILE;
  for (int tile = 0; tile < nT; ++tile) {
    const int t0 = tile * TILE + q * TC;
    float r[TC][4], i[TC][4], x[TC][4], zz[TC][4];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int t = min(t0 + j, L - 1);
      ldv(r[j], rgb + t * rg_rs);
      ldv(i[j], rgb + t * rg_rs + H);
      ldv(x[j], xcb + t * xc_rs);
      ldv(zz[j], zb + t * z_rs);
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      float o[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) o[v] = r[j][v] + i[j][v] + x[j][v] + zz[j][v];
      if (t0 + j < L) stv(yb + (t0 + j) * y_rs, o);
    }
  }
}

// the gate backward's access pattern (5 reads, 4 writes per step and
// channel, same strides and wave/lane layout, reverse tile order), trivial math
template <int Q, int TC, typename T = float, int VEC = 4>
__global__ void __launch_bounds__(256)
pattern5to4(const T* rg, int rg_rs, const T* xc, int xc_rs, const T* z, int z_rs,
            const T* dy, T* drg, int drg_rs, T* dxc, int dxc_rs, T* dz, int dz_rs,
            int64_t B, int L, int H, int ncw) {
  constexpr int G = 64 / Q, TILE = Q * TC;
  const int lane = threadIdx.x & 63, q = lane & (Q - 1), g = lane / Q;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = wid / ncw;
  if (b >= B) return;
  const int c0 = (int)(wid - b * ncw) * (G * VEC) + g * VEC;
  const int64_t row0 = b * L;
  const int nT = (L + TILE - 1) / TILE;
  for (int tile = nT - 1; tile >= 0; --tile) {
    const int t0 = tile * TILE + q * TC;
    float r[TC][VEC], i[TC][VEC], x[TC][VEC], zz[TC][VEC], d[TC][VEC];
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const int64_t t = row0 + min(t0 + j, L - 1);
      ldv(r[j], rg + t * rg_rs + c0);
      ldv(i[j], rg + t * rg_rs + H + c0);
      ldv(x[j], xc + t * xc_rs + c0);
      ldv(zz[j], z + t * z_rs + c0);
      ldv(d[j], dy + t * H + c0);
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      if (t0 + j >= L) continue;
      const int64_t t = row0 + t0 + j;
      float o1[VEC], o2[VEC], o3[VEC], o4[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        o1[v] = r[j][v] * d[j][v];
        o2[v] = i[j][v] * d[j][v];
        o3[v] = x[j][v] * d[j][v];
        o4[v] = zz[j][v] * d[j][v];
      }
      stv(dz + t * dz_rs + c0, o4);
      stv(drg + t * drg_rs + c0, o1);
      stv(drg + t * drg_rs + H + c0, o2);
      stv(dxc + t * dxc_rs + c0, o3);
    }
  }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 2048;
  const int L = argc > 2 ? atoi(argv[2]) : 200;
  const int H = argc > 3 ? atoi(argv[3]) : 256;
  const int rounds = argc > 4 ? atoi(argv[4]) : 15;
  const bool bf16_only = argc > 5 && atoi(argv[5]) == 1;   // the config-5 bf16 sweep only
  const bool packed_only = argc > 5 && atoi(argv[5]) == 2; // gate bwd: dense vs packed lengths
  const bool predecessor = argc > 5 && atoi(argv[5]) == 3;  // gate bwd after different kernels
  const double N = (double)B * L * H;
  const int64_t n = (int64_t)B * L * H;
  const int nT = (L + RB_TILE - 1) / RB_TILE;
  float* rg = dalloc(2 * n, 1, -2, 2);
  float* xz = dalloc(2 * n, 2);
  float* xc = dalloc(n, 3);
  float* lam = dalloc(H, 4, -7, -2);
  float* y = dalloc(n, 5);
  float* car = dalloc((int64_t)B * nT * H, 6);
  float* dy = dalloc(n, 7);
  float* drg = dalloc(2 * n, 8);
  float* dxc = dalloc(n, 9);
  float* dz = dalloc(2 * n, 10);
  float* part = dalloc(3 * (int64_t)B * H, 11);
  float* dh0 = dalloc((int64_t)B * H, 12);
  float* w = dalloc(H * 8, 13);
  float* bias = dalloc(H, 14);
  float* dwp = dalloc((int64_t)B * 9 * H, 15);
  float* dbp = dalloc((int64_t)B * H, 16);
  float* g1 = dalloc(n, 17);
  float* dxo = dalloc(2 * n, 18);
  float* sg = dalloc(n, 19, 0.9f, 1.0f);   // [B, H, T] scan operands (T = L here)
  float* sx = dalloc(n, 20);
  float* so = dalloc(n, 21);
  float* sd = dalloc(n, 22);
  CK(hipDeviceSynchronize());

  if (predecessor) {
    // the dense gate backward timed alone, with HIP events around it only,
    // right after (no sync) a preceding launch: nothing (GPU idle), a float4
    // copy, the f16x3 gates GEMM (MFMA-heavy), or another gate backward
    float* A = dalloc((int64_t)B * L * H, 50);
    float* O = dalloc((int64_t)B * L * 2 * H, 51);
    float* W = dalloc((int64_t)2 * H * H, 52, -0.05f, 0.05f);
    void* Wf;
    CK(hipMalloc(&Wf, (size_t)2 * H * H * 4 + 8192));
    rb_split_job job{W, H, 2 * H, H, 0, Wf};
    CK((hipError_t)launch_split_weights_h(&job, 1, 0));
    auto gate = [=] {
      gate_bwd_v<float, 4>(rg, 2 * H, xc, H, xz + H, 2 * H, lam, nullptr, car, dy, drg, 2 * H, dxc,
                           H, dz + H, 2 * H, part, dh0, B, L, H, nullptr, 0, nullptr);
    };
    struct Pre { const char* name; std::function<void()> run; };
    std::vector<Pre> pres = {
        {"idle", [] {}},
        {"copy4 x3", [=] { for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, (const float4*)xc, (float4*)dxc, n / 4); }},
        {"gemm_nt_h x3", [=] { for (int k = 0; k < 3; ++k) launch_gemm_nt_h(A, H, (int64_t)B * L, H, Wf, 2 * H, nullptr, O, 2 * H, 0, nullptr, 0); }},
        {"gate_bwd x3", [=] { for (int k = 0; k < 3; ++k) gate(); }},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ms(pres.size());
    for (int r = 0; r < rounds; ++r)
      for (size_t i = 0; i < pres.size(); ++i) {
        CK(hipDeviceSynchronize());
        pres[i].run();
        CK(hipEventRecord(e0, 0));
        gate();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms[i].push_back(t);
      }
    printf("B=%d L=%d H=%d dense gate backward after a predecessor (median of %d)\n", B, L, H, rounds);
    for (size_t i = 0; i < pres.size(); ++i) {
      std::sort(ms[i].begin(), ms[i].end());
      const double med = ms[i][ms[i].size() / 2];
      printf("after %-14s %8.1f us  %.3f of 8 TB/s\n", pres[i].name, med * 1e3, 9 * N * 4 / (med * 1e-3) / 8e12);
    }
    return 0;
  }

  std::vector<Case> cs;
  GateBufs sep{rg, xc, xz + H, y, car, dy, drg, dxc, dz + H, part, dh0, lam,
               2 * H, H, 2 * H, 2 * H, H, 2 * H};
  float* P = dalloc(3 * n, 31, -1, 1);   // [r | i | xc] rows
  float* Qb = dalloc(3 * n, 32);          // [dr | di | dxc] rows
  GateBufs comb{P, P + 2 * H, xz + H, y, car, dy, Qb, Qb + 2 * H, dz + H, part, dh0, lam,
                3 * H, 3 * H, 2 * H, 3 * H, 3 * H, 2 * H};
  if (packed_only) {
    // the bench's packed batch: lengths uniform in 1..L, sequences longest
    // first, rows concatenated (ntok ~ B * L / 2); bytes = 9 streams x ntok x H
    std::vector<int64_t> lens(B), offs_h(B + 1, 0);
    uint64_t st = 12345;
    for (int i = 0; i < B; ++i) {
      st = st * 6364136223846793005ULL + 1442695040888963407ULL;
      lens[i] = 1 + (int64_t)((st >> 33) % L);
    }
    std::vector<int64_t> unsorted = lens;
    std::sort(lens.begin(), lens.end(), [](int64_t a, int64_t b) { return a > b; });
    auto mk_offs = [&](const std::vector<int64_t>& ls) {
      std::vector<int64_t> o(B + 1, 0);
      for (int i = 0; i < B; ++i) o[i + 1] = o[i] + ls[i];
      int64_t* d;
      CK(hipMalloc(&d, (B + 1) * 8));
      CK(hipMemcpy(d, o.data(), (B + 1) * 8, hipMemcpyHostToDevice));
      return std::make_pair(d, o[B]);
    };
    auto [offs_sorted, ntok] = mk_offs(lens);
    auto [offs_unsorted, ntok2] = mk_offs(unsorted);
    (void)ntok2;
    const double NP = (double)ntok * H;
    auto bwd = [=](const char* nm, const int64_t* offs, bool dma, double bytes) {
      return Case{nm, bytes, [=] {
        if (dma)
          launch_gate_bwd(rg, 2 * H, xc, H, xz + H, 2 * H, lam, nullptr, car, dy, drg, 2 * H, dxc,
                          H, dz + H, 2 * H, part, dh0, B, L, H, offs, 0);
        else
          gate_bwd_v<float, 4>(rg, 2 * H, xc, H, xz + H, 2 * H, lam, nullptr, car, dy, drg, 2 * H,
                               dxc, H, dz + H, 2 * H, part, dh0, B, L, H, offs, 0, nullptr);
      }, {}};
    };
    cs.push_back({"pattern5to4 q8 tc2 dense", 9 * N * 4, [=] {
      const int ncw = H / 32;
      hipLaunchKernelGGL((pattern5to4<8, 2>), dim3(((int64_t)B * ncw + 3) / 4), dim3(256), 0, 0,
                         rg, 2 * H, xc, H, xz + H, 2 * H, dy, drg, 2 * H, dxc, H, dz + H, 2 * H,
                         (int64_t)B, L, H, ncw);
    }, {}});
    cs.push_back({"pattern5to4 q4 tc4 dense", 9 * N * 4, [=] {
      const int ncw = H / 64;
      hipLaunchKernelGGL((pattern5to4<4, 4>), dim3(((int64_t)B * ncw + 3) / 4), dim3(256), 0, 0,
                         rg, 2 * H, xc, H, xz + H, 2 * H, dy, drg, 2 * H, dxc, H, dz + H, 2 * H,
                         (int64_t)B, L, H, ncw);
    }, {}});
    cs.push_back({"pattern5to4 q2 tc8 dense", 9 * N * 4, [=] {
      const int ncw = H / 128;
      hipLaunchKernelGGL((pattern5to4<2, 8>), dim3(((int64_t)B * ncw + 3) / 4), dim3(256), 0, 0,
                         rg, 2 * H, xc, H, xz + H, 2 * H, dy, drg, 2 * H, dxc, H, dz + H, 2 * H,
                         (int64_t)B, L, H, ncw);
    }, {}});
    cs.push_back(bwd("bwd dense regs", nullptr, false, 9 * N * 4));
    cs.push_back(bwd("bwd dense dma", nullptr, true, 9 * N * 4));
    cs.push_back(bwd("bwd packed regs", offs_sorted, false, 9 * NP * 4));
    cs.push_back(bwd("bwd packed dma", offs_sorted, true, 9 * NP * 4));
    cs.push_back(bwd("bwd packed-unsorted dma", offs_unsorted, true, 9 * NP * 4));
    // conv backward on the packed batch: 3 reads (x, the two dxc terms) + 1
    // write (dx) per element; chunk layouts, prefetch
    auto cbp = [&](const char* nm, auto kern, int Q, int VEC) {
      const int span = (64 / Q) * VEC;
      const int ncw = (H + span - 1) / span;
      const int64_t blocks = ((int64_t)B * ncw + 3) / 4;
      cs.push_back({nm, 4 * NP * 4, [=] {
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, 0, (const float*)xz, 2 * H,
                           w, bias, (const float*)g1, (const float*)dy, dxo, 2 * H, dwp,
                           (float*)nullptr, (int64_t)B, L, H, ncw, offs_sorted);
      }, {}});
    };
    cbp("conv_bwd packed q4 tc4 (shipped)", k_conv_silu_bwd<float, 4, 4, 4, 4, false>, 4, 4);
    cbp("conv_bwd packed q4 tc4 pf", k_conv_silu_bwd<float, 4, 4, 4, 4, true>, 4, 4);
    cbp("conv_bwd packed q8 tc4", k_conv_silu_bwd<float, 4, 4, 8, 4, false>, 8, 4);
    cbp("conv_bwd packed q4 tc8", k_conv_silu_bwd<float, 4, 4, 4, 8, false>, 4, 4);
    cbp("conv_bwd packed q2 tc8", k_conv_silu_bwd<float, 4, 4, 2, 8, false>, 2, 4);
    cbp("conv_bwd packed v2 q4 tc4", k_conv_silu_bwd<float, 4, 2, 4, 4, false>, 4, 2);
    cbp("conv_bwd packed q4 tc4 (shipped, again)", k_conv_silu_bwd<float, 4, 4, 4, 4, false>, 4, 4);
    cbp("conv_bwd packed q8 tc4 (again)", k_conv_silu_bwd<float, 4, 4, 8, 4, false>, 8, 4);
    cs.push_back({"copy4 (1R+1W float4)", 2 * NP * 4, [=] {
      hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, (const float4*)xc, (float4*)dxc,
                         (int64_t)(NP / 4));
    }, {}});
    if (getenv("KB_CONV_ONLY")) goto timed;
    cs.push_back({"gate_fwd packed", 5 * NP * 4, [=] {
      launch_gate_fwd(rg, 2 * H, xc, H, xz + H, 2 * H, lam, nullptr, nullptr, 0, y, H, car, B, L,
                      H, offs_sorted, 0);
    }, {}});
    cs.push_back({"gate_fwd dense", 5 * N * 4, [=] {
      launch_gate_fwd(rg, 2 * H, xc, H, xz + H, 2 * H, lam, nullptr, nullptr, 0, y, H, car, B, L,
                      H, nullptr, 0);
    }, {}});
  } else if (bf16_only) {
    {
      auto bp = [](float* p) { return reinterpret_cast<bf16_t*>(p); };
      cs.push_back({"pattern5to4 bf16 v4 q4 tc4", 9 * N * 2, [=] {
        const int ncw = H / 64;
        hipLaunchKernelGGL((pattern5to4<4, 4, bf16_t, 4>), dim3(((int64_t)B * ncw + 3) / 4),
                           dim3(256), 0, 0, bp(rg), 2 * H, bp(xc), H, bp(xz + H), 2 * H, bp(dy),
                           bp(drg), 2 * H, bp(dxc), H, bp(dz + H), 2 * H, (int64_t)B, L, H, ncw);
      }, {}});
      cs.push_back({"pattern5to4 bf16 v8 q8 tc2", 9 * N * 2, [=] {
        const int ncw = H / 64;
        hipLaunchKernelGGL((pattern5to4<8, 2, bf16_t, 8>), dim3(((int64_t)B * ncw + 3) / 4),
                           dim3(256), 0, 0, bp(rg), 2 * H, bp(xc), H, bp(xz + H), 2 * H, bp(dy),
                           bp(drg), 2 * H, bp(dxc), H, bp(dz + H), 2 * H, (int64_t)B, L, H, ncw);
      }, {}});
      cs.push_back({"pattern5to4 f32 v4 q8 tc2", 9 * N * 4, [=] {
        const int ncw = H / 32;
        hipLaunchKernelGGL((pattern5to4<8, 2>), dim3(((int64_t)B * ncw + 3) / 4), dim3(256), 0, 0,
                           rg, 2 * H, xc, H, xz + H, 2 * H, dy, drg, 2 * H, dxc, H, dz + H, 2 * H,
                           (int64_t)B, L, H, ncw);
      }, {}});
    }
    {
      auto bp = [](float* p) { return reinterpret_cast<bf16_t*>(p); };
      cs.push_back({"gate_bwd bf16 v4 q4 tc4 dma", 9 * N * 2, [=] {
        gate_bwd_v<bf16_t, 4, 4, 4, false, true>(bp(rg), 2 * H, bp(xc), H, bp(xz + H), 2 * H, lam,
                                                 nullptr, car, bp(dy), bp(drg), 2 * H, bp(dxc), H,
                                                 bp(dz + H), 2 * H, part, dh0, B, L, H, nullptr, 0,
                                                 nullptr);
      }, {}});
      cs.push_back({"gate_bwd bf16 v4 q4 tc4 pf (shipped)", 9 * N * 2, [=] {
        gate_bwd_v<bf16_t, 4, 4, 4, true>(bp(rg), 2 * H, bp(xc), H, bp(xz + H), 2 * H, lam,
                                          nullptr, car, bp(dy), bp(drg), 2 * H, bp(dxc), H,
                                          bp(dz + H), 2 * H, part, dh0, B, L, H, nullptr, 0,
                                          nullptr);
      }, {}});
    }
    if (getenv("KB_DMA_ONLY")) goto timed;
    add_gate<bf16_t, 4, 4, 4, true>(cs, "bf16 v4 q4 tc4 pf", B, L, H, sep, N, 1);
    add_gate<bf16_t, 4, 4, 4, false>(cs, "bf16 v4 q4 tc4", B, L, H, sep, N, 1);
    add_gate<bf16_t, 8, 8, 2, true>(cs, "bf16 v8 q8 tc2 pf", B, L, H, sep, N, 1);
    add_gate<bf16_t, 4, 8, 2, true>(cs, "bf16 v4 q8 tc2 pf", B, L, H, sep, N, 1);
    add_gate<bf16_t, 8, 8, 2, false>(cs, "bf16 v8 q8 tc2", B, L, H, sep, N, 1);
    add_gate<bf16_t, 8, 4, 4, false>(cs, "bf16 v8 q4 tc4", B, L, H, sep, N, 1);
    add_gate<bf16_t, 2, 4, 4, true>(cs, "bf16 v2 q4 tc4 pf", B, L, H, sep, N, 1);
    add_gate<bf16_t, 4, 8, 2, false>(cs, "bf16 v4 q8 tc2", B, L, H, sep, N, 2);
    add_gate<bf16_t, 4, 8, 2, true>(cs, "bf16 v4 q8 tc2 pf", B, L, H, sep, N, 2);
    add_gate<bf16_t, 8, 8, 2, true>(cs, "bf16 v8 q8 tc2 pf", B, L, H, sep, N, 2);
    add_gate<bf16_t, 4, 4, 4, true>(cs, "bf16 v4 q4 tc4 pf", B, L, H, sep, N, 2);
    add_gate<float, 4, 8, 2, true>(cs, "f32 v4 q8 tc2 pf", B, L, H, sep, N, 2);
    add_conv<bf16_t, 4, 4, 4, 4, true>(cs, "bf16 v4 q4 tc4 pf", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N, 2);
    add_conv<bf16_t, 4, 8, 4, 4, true>(cs, "bf16 v8 q4 tc4 pf", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N, 2);
    add_conv<bf16_t, 4, 4, 8, 4, true>(cs, "bf16 v4 q8 tc4 pf", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N, 2);
    add_conv<float, 4, 4, 4, 4, true>(cs, "f32 v4 q4 tc4 pf", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N, 2);
    add_gate<bf16_t, 8, 8, 2, false>(cs, "bf16 v8 q8 tc2", B, L, H, sep, N, 2);
    add_gate<bf16_t, 4, 4, 4, false>(cs, "bf16 v4 q4 tc4", B, L, H, sep, N, 2);
    add_gate<bf16_t, 8, 16, 1, false>(cs, "bf16 v8 q16 tc1", B, L, H, sep, N, 2);
    add_gate<bf16_t, 4, 16, 1, false>(cs, "bf16 v4 q16 tc1", B, L, H, sep, N, 2);
    add_gate<float, 4, 8, 2, false>(cs, "f32 v4 q8 tc2", B, L, H, sep, N, 2);
    add_gate<float, 2, 4, 4, true>(cs, "f32 v2 q4 tc4 pf", B, L, H, sep, N, 1);
    add_conv<bf16_t, 4, 4, 4, 4>(cs, "bf16 v4 q4 tc4", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
    add_conv<bf16_t, 4, 8, 4, 4>(cs, "bf16 v8 q4 tc4", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
    add_conv<bf16_t, 4, 8, 4, 8>(cs, "bf16 v8 q4 tc8", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
    add_conv<bf16_t, 4, 8, 8, 4>(cs, "bf16 v8 q8 tc4", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
    add_conv<bf16_t, 4, 4, 8, 4>(cs, "bf16 v4 q8 tc4", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
    add_conv<float, 4, 4, 4, 4>(cs, "f32 v4 q4 tc4", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
    cs.push_back({"copy4 (1R+1W float4)", 2 * N * 4, [=] {
      hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, (const float4*)xc, (float4*)dxc, n / 4);
    }, {}});
  } else {
  add_gate<float, 2, 4, 4, true>(cs, "v2 q4 tc4 pf  sep", B, L, H, sep, N);
  add_gate<float, 4, 8, 2, false>(cs, "v4 q8 tc2     sep", B, L, H, sep, N);
  add_gate<float, 4, 8, 2, true>(cs, "v4 q8 tc2 pf  sep", B, L, H, sep, N, 2);
  add_conv<float, 4, 4, 4, 4, true>(cs, "v4 q4 tc4 pf", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N, 2);
  add_gate<float, 2, 4, 4, true>(cs, "v2 q4 tc4 pf  comb", B, L, H, comb, N);
  add_gate<float, 4, 8, 2, false>(cs, "v4 q8 tc2     comb", B, L, H, comb, N);
  add_gate<float, 4, 4, 4, true>(cs, "v4 q4 tc4 pf  comb", B, L, H, comb, N);
  add_gate<float, 2, 8, 2, false>(cs, "v2 q8 tc2     comb", B, L, H, comb, N);
  add_conv<float, 4, 4, 4, 8>(cs, "v4 q4 tc8", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
  add_conv<float, 4, 4, 4, 4>(cs, "v4 q4 tc4", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
  add_conv<float, 4, 2, 4, 4>(cs, "v2 q4 tc4", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
  add_conv<float, 4, 4, 2, 8>(cs, "v4 q2 tc8", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
  add_conv<float, 4, 2, 2, 8>(cs, "v2 q2 tc8", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
  add_conv<float, 4, 4, 8, 4>(cs, "v4 q8 tc4", B, L, H, xz, w, bias, xc, g1, dxo, dwp, dbp, N);
  cs.push_back({"scan_rows_fwd [B,H,L]", 3 * N * 4, [=] {
    launch_scan_fwd(sg, sx, so, (int64_t)B * H, L, 0);
  }, {}});
  cs.push_back({"scan_rows_bwd [B,H,L]", 5 * N * 4, [=] {
    launch_scan_bwd(sg, so, sx, sd, y, (int64_t)B * H, L, 0);
  }, {}});
  cs.push_back({"flat4to1 (4R+1W float4)", 5 * N * 4, [=] {
    hipLaunchKernelGGL(flat4to1, dim3(4096), dim3(256), 0, 0, (const float4*)rg, (const float4*)(rg + n),
                       (const float4*)xc, (const float4*)g1, (float4*)y, n / 4);
  }, {}});
  cs.push_back({"pattern4to1 q4 tc4", 5 * N * 4, [=] {
    const int ncw = H / 64;
    hipLaunchKernelGGL((pattern4to1<4, 4>), dim3(((int64_t)B * ncw + 3) / 4), dim3(256), 0, 0, rg,
                       2 * H, xc, H, xz + H, 2 * H, y, H, (int64_t)B, L, H, ncw);
  }, {}});
  cs.push_back({"pattern4to1 q1 tc16", 5 * N * 4, [=] {
    const int ncw = H / 256;
    hipLaunchKernelGGL((pattern4to1<1, 16>), dim3(((int64_t)B * ncw + 3) / 4), dim3(256), 0, 0, rg,
                       2 * H, xc, H, xz + H, 2 * H, y, H, (int64_t)B, L, H, ncw);
  }, {}});
  cs.push_back({"copy4 (1R+1W float4)", 2 * N * 4, [=] {
    hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, (const float4*)xc, (float4*)dxc, n / 4);
  }, {}});
  // the same gate kernels with the operand arrays staggered inside one pool
  // (tests whether equal 2 MB alignment of the streams costs channel balance)
  {
    const int64_t pool_f = 8 * n + (1 << 22);
    float* pool = dalloc(pool_f, 40);
    const int64_t offs[3][6] = {{0, 2304, 4608, 6912, 9216, 11520},            // 9 KB steps
                                {0, 16448, 32896, 49344, 65792, 82240},        // 64 KB + 64 B
                                {0, 262208, 524416, 786624, 1048832, 1311040}}; // 1 MB + 256 B
    for (int k = 0; k < 3; ++k) {
      const int64_t* o = offs[k];
      float* rg2 = pool + o[0];
      float* xz2 = rg2 + 2 * n + o[1];
      float* xc2 = xz2 + 2 * n + o[2];
      float* y2 = xc2 + n + o[3];
      GateBufs st{rg2, xc2, xz2 + H, y2, car, dy, drg, dxc, dz + H, part, dh0, lam,
                  2 * H, H, 2 * H, 2 * H, H, 2 * H};
      char* nm = (char*)malloc(64);
      snprintf(nm, 64, "v2 q4 tc4 pf stag%d", k);
      add_gate<float, 2, 4, 4, true>(cs, nm, B, L, H, st, N);
    }
  }
  cs.push_back({"hipMemcpy d2d (R+W)", 2 * N * 4, [=] {
    CK(hipMemcpyAsync(dxc, xc, n * sizeof(float), hipMemcpyDeviceToDevice, 0));
  }, {}});
  }

timed:
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& c : cs) c.run();  // warm-up
  CK(hipDeviceSynchronize());
  // KB_REPS=k: k back-to-back launches per timed sample (per-launch time shown)
  const int reps = getenv("KB_REPS") ? std::max(1, atoi(getenv("KB_REPS"))) : 1;
  for (int r = 0; r < rounds; ++r) {
    for (auto& c : cs) {
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < reps; ++k) c.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      c.ms.push_back(ms / reps);
    }
  }
  CK(hipGetLastError());
  printf("B=%d L=%d H=%d  N=%.0f  (median of %d)\n", B, L, H, N, rounds);
  for (auto& c : cs) {
    std::sort(c.ms.begin(), c.ms.end());
    const double med = c.ms[c.ms.size() / 2];
    printf("%-26s %9.1f us  %7.1f GB/s  %.3f of 8 TB/s\n", c.name, med * 1e3,
           c.bytes / (med * 1e-3) / 1e9, c.bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
