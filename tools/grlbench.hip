// grlbench.hip — timing of the fused GatedRecurrentLayer kernels
// (csrc/grl_fused.hip: rb_grl_fwd / rb_grl_bwd) at the benchmark's packed
// shape (B = 2048, L = 200, lengths ~U{1..L}, H = 256, kc = 4), random
// operands (timing only; parity lives in tests/test_gpu_fused.py).
// Ablation builds: -DGRL_PROBE=<mask> (see grl_fused.hip).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       tools/grlbench.hip -o tools/bin/grlbench
#include <cstdio>

#include "../datamining_recblr_amd/csrc/grl_fused.hip"

namespace rb {
int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
  return (int)e;
}
int fail(const char* m) {
  fprintf(stderr, "%s\n", m);
  return -1;
}
}  // namespace rb
using namespace rb;

#include <algorithm>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void fill(float* p, int64_t n, uint32_t seed, float scale) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = scale * ((h & 0xffffff) / 16777216.0f - 0.5f);
  }
}

// a plausible f16 weight image: small values, exponents 0
__global__ void fill_img(_Float16* p, int64_t n, int* e, int ne) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t j = i; j < n; j += (int64_t)gridDim.x * blockDim.x)
    p[j] = (_Float16)(((j * 2654435761u) & 1023) / 1024.0f - 0.5f);
  for (int64_t j = i; j < ne; j += (int64_t)gridDim.x * blockDim.x) e[j] = 0;
}

static float* dalloc(int64_t n, uint32_t seed, float scale) {
  float* p;
  CK(hipMalloc(&p, n * 4));
  fill<<<1024, 256>>>(p, n, seed, scale);
  return p;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 2048, L = argc > 2 ? atoi(argv[2]) : 200;
  const int iters = argc > 3 ? atoi(argv[3]) : 20;
  const bool fixed = getenv("GRL_FIXED") != nullptr;
  constexpr int H = 256, KC = 4;
  int G = 0;
  CK(hipDeviceGetAttribute(&G, hipDeviceAttributeMultiprocessorCount, 0));
  std::mt19937 rng(1234);
  std::vector<int64_t> lens(B);
  for (auto& l : lens) l = fixed ? L : 1 + (int64_t)(rng() % L);
  std::sort(lens.begin(), lens.end(), std::greater<int64_t>());
  std::vector<int64_t> offs(B + 1, 0);
  for (int b = 0; b < B; ++b) offs[b + 1] = offs[b] + lens[b];
  const int64_t ntok = offs[B];
  // serpentine work lists (kernels.grl_pieces)
  std::vector<int> span_of(B), order(B);
  for (int k = 0; k < B; ++k) {
    const int r = k / G, j = k % G;
    span_of[k] = r % 2 == 0 ? j : G - 1 - j;
    order[k] = k;
  }
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return span_of[a] < span_of[b]; });
  std::vector<int> pieces(3 * B + G + 1, 0);
  std::vector<int64_t> rows(G, 0);
  for (int i = 0; i < B; ++i) {
    const int k = order[i];
    pieces[i] = (int)offs[k];
    pieces[B + i] = (int)lens[k];
    pieces[2 * B + i] = k;
    pieces[3 * B + span_of[k] + 1] += 1;
    rows[span_of[k]] += lens[k];
  }
  for (int g = 0; g < G; ++g) pieces[3 * B + g + 1] += pieces[3 * B + g];
  const int64_t max_rows = *std::max_element(rows.begin(), rows.end());
  const int64_t max_tiles = (max_rows + 63) / 64;
  printf("B=%d L=%d ntok=%lld G=%d max span rows=%lld (mean %.1f) max_tiles=%lld probe=%d\n", B, L,
         (long long)ntok, G, (long long)max_rows, (double)ntok / G, (long long)max_tiles,
         GRL_PROBE);

  int* d_pieces;
  CK(hipMalloc(&d_pieces, pieces.size() * 4));
  CK(hipMemcpy(d_pieces, pieces.data(), pieces.size() * 4, hipMemcpyHostToDevice));
  float* xz = dalloc(ntok * 2 * H, 1, 4.0f);
  float* conv_w = dalloc(H * KC, 2, 1.0f);
  float* conv_b = dalloc(H, 3, 0.2f);
  float* gate_b = dalloc(2 * H, 4, 0.2f);
  float* lam = dalloc(H, 5, 1.0f);
  float* h0 = dalloc(H, 6, 0.5f);
  const int64_t img_half = (int64_t)2 * H * H * 2;   // f16 elements of a [2H, H] image (2 planes)
  _Float16 *wf, *wft;
  CK(hipMalloc(&wf, img_half * 2 + 2 * H * 4));
  CK(hipMalloc(&wft, img_half * 2 + 2 * H * 4));
  fill_img<<<512, 256>>>(wf, img_half, reinterpret_cast<int*>(wf + img_half), 2 * H);
  fill_img<<<512, 256>>>(wft, img_half, reinterpret_cast<int*>(wft + img_half), 2 * H);
  float* y = dalloc(ntok * H, 7, 0.0f);
  float* tc = dalloc(G * max_tiles * H, 8, 0.0f);
  float* dy = dalloc(ntok * H, 9, 1.0f);
  float* dxz = dalloc(ntok * 2 * H, 10, 0.0f);
  float* drg = dalloc(ntok * 2 * H, 11, 0.0f);
  float* xc = dalloc(ntok * H, 12, 0.0f);
  const int64_t nr = (ntok + 31) / 32;
  float* rmax = dalloc(2 * nr, 13, 0.0f);
  float* part = dalloc((int64_t)G * 4 * H, 14, 0.0f);
  float* cpart = dalloc((int64_t)G * 8 * (H * KC + H), 15, 0.0f);
  CK(hipDeviceSynchronize());

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto fwd = [&]() {
    return launch_grl_fwd(xz, 2 * H, conv_w, KC, conv_b, wf, gate_b, lam, h0, d_pieces, B, G, ntok,
                          y, H, nullptr, nullptr, nullptr, nullptr, 0, nullptr, tc, max_tiles, 0);
  };
  const int nTc = (L + 15) / 16;
  float* car = dalloc((int64_t)B * nTc * H, 16, 0.0f);
  float* rgo = dalloc(ntok * 2 * H, 17, 0.0f);
  auto fwd_legacy = [&]() {   // the three-launch backward's operands as side outputs
    return launch_grl_fwd(xz, 2 * H, conv_w, KC, conv_b, wf, gate_b, lam, h0, d_pieces, B, G, ntok,
                          y, H, nullptr, xc, rgo, car, nTc, rmax, nullptr, 0, 0);
  };
  auto bwd = [&]() {
    return launch_grl_bwd(xz, 2 * H, conv_w, KC, conv_b, wf, wft, gate_b, lam, h0, d_pieces, B, G,
                          ntok, tc, max_tiles, dy, nullptr, dxz, 2 * H, drg, xc, rmax, rmax + nr,
                          part, cpart, 0);
  };
#ifdef GRL_STAMPS
  auto stamps = [&](int w, const char* const* names, int n) {
    unsigned long long st[2][20];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(grl_stamps), sizeof(st)));
    double tot = 0;
    for (int k = 0; k < n; ++k) tot += (double)st[w][k];
    for (int k = 0; k < n; ++k) printf("    %-14s %5.1f%%\n", names[k], 100.0 * st[w][k] / tot);
  };
  auto zero = [&]() {
    unsigned long long z[2][20] = {};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(grl_stamps), z, sizeof(z)));
  };
  zero();
#endif
  const double fwd_bytes = 3.0 * ntok * H * 4, bwd_bytes = 8.0 * ntok * H * 4;
  for (int w = 0; w < 3; ++w) { fwd(); bwd(); }
  CK(hipDeviceSynchronize());
  float ms;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) fwd();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("fwd  %8.1f us  %6.0f GB/s (x, z, y)\n", 1e3 * ms / iters, fwd_bytes / (1e6 * ms / iters));
#ifdef GRL_STAMPS
  CK(hipDeviceSynchronize());
  {
    const char* names[] = {"rowmap", "A", "A.sync", "C.gemm", "D", "D.sync"};
    stamps(0, names, 6);
  }
#endif
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) fwd_legacy();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("fwd+ %8.1f us  (y + xc, rg, 16-step carries: the three-launch backward's operands)\n",
         1e3 * ms / iters);
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) bwd();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("bwd  %8.1f us  %6.0f GB/s (x, z, dy, dx, dz, dr, di, xc)\n", 1e3 * ms / iters,
         bwd_bytes / (1e6 * ms / iters));
  CK(hipDeviceSynchronize());
#ifdef GRL_STAMPS
  {
    const char* names[] = {"rowmap", "A", "A.sync", "C.gemm1", "C.sync", "D.fwd", "D.rev",
                           "D.sync", "E", "E.sync", "F.gemm2", "F.sync", "G", "G.sync", "H1",
                           "H1.sync", "H2", "H2.sync+halo"};
    stamps(1, names, 18);
  }
#endif
  return 0;
}
