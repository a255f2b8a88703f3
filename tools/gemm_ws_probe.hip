// gemm_ws_probe.hip — the weight-stationary f16x3 NT GEMM (csrc/gemm_ws.hip)
// against the persistent k_gemm_nt_h (csrc/gemm_half.hip) on the encoder's eight
// projection shapes at the bench's packed row count: time (alternated, median
// and min of reps), the error of both against fp64 on sampled rows (relative
// to sum |a||b| of each output), the row-group maxima (rmax) equal.
// Columns: the persistent kernel (rb_gemm_nt_h_mode 0), the weight-stationary
// kernel with stores at each block's end, and with stores deferred between
// the next block's MFMA units (the shipped form); with argv[4] = 1 also three
// timing-only ablations of the shipped form (no MFMAs, no fragment reads, no
// stores; results not meaningful).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++20 -I include \
//       tools/gemm_ws_probe.hip -o tools/bin/gemm_ws_probe
#include <cstdio>

#include "../datamining_recblr_amd/csrc/gemm_half.hip"
#include "../datamining_recblr_amd/csrc/gemm_small.hip"
#include "../datamining_recblr_amd/csrc/gemm_ws.hip"

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
int num_cus() {
  int n = 0;
  (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, 0);
  return n;
}
}  // namespace rb
using namespace rb;

// variant: bit 0 deferred stores, bits 4.. ablation mask (gemm_ws.hip's ABL)
static int run_ws(const float* A, int64_t lda, int64_t M, int K, const void* Wf, int C,
                  const float* bias, float* out, int64_t ldo, float* rmax, int variant) {
  const void* Wi = reinterpret_cast<const char*>(Wf) + ws_image_offset(C, K);
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * K * 4);
  const int ncb = ws::ncb_for(K, C);
  const int grid = ws::grid_for(M, C, ncb);
  const bool defer = variant & 1;
  const int abl = variant >> 4;
  int rc = 0;
  const bool early1 = variant & 2;   // K = 512: every wave late at depth 1 (ABL bit 32; round 6's first form)
  auto go = [&](auto kc, auto nc) {
    constexpr int KK = decltype(kc)::value, NC = decltype(nc)::value;
    auto g3 = [&](auto ac, auto dc) {
      constexpr int AB = decltype(ac)::value, DD = decltype(dc)::value;
      if (bias) {
        if (defer) ws::run<KK, NC, DD, true, true, AB>(A, lda, M, Wi, ew, C, bias, out, ldo, rmax, grid, 0);
        else ws::run<KK, NC, DD, true, false, AB>(A, lda, M, Wi, ew, C, bias, out, ldo, rmax, grid, 0);
      } else {
        if (defer) ws::run<KK, NC, DD, false, true, AB>(A, lda, M, Wi, ew, C, bias, out, ldo, rmax, grid, 0);
        else ws::run<KK, NC, DD, false, false, AB>(A, lda, M, Wi, ew, C, bias, out, ldo, rmax, grid, 0);
      }
    };
    auto g2 = [&](auto ac) { g3(ac, std::integral_constant<int, ws::depth<KK>()>{}); };
    switch (abl | (early1 ? 32 : 0)) {
      case 0: g2(std::integral_constant<int, 0>{}); break;
      case 32: g2(std::integral_constant<int, 32>{}); break;
      case 1: g2(std::integral_constant<int, 1>{}); break;
      case 4: g2(std::integral_constant<int, 4>{}); break;
      case 16: g2(std::integral_constant<int, 16>{}); break;
      default: rc = fail("ablation");
    }
  };
  using std::integral_constant;
  if (K == 128 && ncb == 4) go(integral_constant<int, 128>{}, integral_constant<int, 4>{});
  else if (K == 128 && ncb == 2) go(integral_constant<int, 128>{}, integral_constant<int, 2>{});
  else if (K == 256 && ncb == 2) go(integral_constant<int, 256>{}, integral_constant<int, 2>{});
  else if (K == 256 && ncb == 1) go(integral_constant<int, 256>{}, integral_constant<int, 1>{});
  else if (K == 512 && ncb == 1) go(integral_constant<int, 512>{}, integral_constant<int, 1>{});
  else return fail("shape");
  return rc ? rc : launch_status("ws");
}

#include <algorithm>
#include <cmath>
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

__global__ void fill(float* p, int64_t n, uint32_t seed, float scale) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = scale * ((h & 0xffffff) / 16777216.0f - 0.5f);
  }
}

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atoll(argv[1]) : 204632;
  const int reps = argc > 2 ? atoi(argv[2]) : 7;
  const int only = argc > 3 ? atoi(argv[3]) : -1;
  const bool ablate = argc > 4 ? atoi(argv[4]) != 0 : false;
  struct Shape { const char* name; int R, C; };
  const Shape shapes[] = {{"in.fwd", 128, 512}, {"in.dX", 512, 128}, {"gates.fwd", 256, 512},
                          {"gates.dX", 512, 256}, {"out.fwd", 256, 128}, {"out.dX", 128, 256},
                          {"w2.fwd", 512, 128}, {"w2.dX", 128, 512}};
  float *A, *W, *O0, *O1, *bias, *rm0, *rm1;
  void* Wf;
  CK(hipMalloc(&A, M * 512 * 4));
  CK(hipMalloc(&O0, M * 512 * 4));
  CK(hipMalloc(&O1, M * 512 * 4));
  CK(hipMalloc(&W, 512 * 512 * 4));
  CK(hipMalloc(&bias, 512 * 4));
  CK(hipMalloc(&rm0, (M / 32 + 1) * 4));
  CK(hipMalloc(&rm1, (M / 32 + 1) * 4));
  CK(hipMalloc(&Wf, 2 * 512 * 512 * 4 + 4096));
  fill<<<4096, 256>>>(A, M * 512, 1, 2.0f);
  fill<<<256, 256>>>(W, 512 * 512, 2, 0.1f);
  fill<<<2, 256>>>(bias, 512, 3, 1.0f);
  // a few rows far from 1 (scales), one zero row
  {
    std::vector<float> row(512);
    for (int k = 0; k < 512; ++k) row[k] = ldexpf((float)((k * 37) % 11) - 5.0f, 40);
    CK(hipMemcpy(A + 7 * 512, row.data(), 512 * 4, hipMemcpyHostToDevice));
    for (int k = 0; k < 512; ++k) row[k] = ldexpf((float)((k * 13) % 7) - 3.0f, -50);
    CK(hipMemcpy(A + 1000 * 512, row.data(), 512 * 4, hipMemcpyHostToDevice));
    CK(hipMemset(A + 2001 * 512, 0, 512 * 4));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto&& f) {
    CK(hipEventRecord(e0, 0));
    if (f()) exit(1);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f;
  };
  double tot[3] = {0, 0, 0};
  int si = -1;
  for (const Shape& s : shapes) {
    ++si;
    if (only >= 0 && si != only) continue;
    const int R = s.R, C = s.C;
    const bool use_bias = (si % 2) == 0;
    rb_split_job job{W, R, C, R, 0, Wf};
    CK((hipError_t)launch_split_weights_h(&job, 1, 0));
    const float* bp = use_bias ? bias : nullptr;
    std::vector<float> t[3];
    const int abl[] = {1 | 16, 1 | 256, 1 | 64};
    std::vector<float> ta[3];
    for (int rep = 0; rep < reps; ++rep) {
      if (ablate)
        for (int a = 0; a < 3; ++a)
          ta[a].push_back(timeit([&] { return run_ws(A, R, M, R, Wf, C, bp, O1, C, rm1, abl[a]); }));
      t[0].push_back(timeit([&] { gemm_nt_h_mode(0); return launch_gemm_nt_h(A, R, M, R, Wf, C, bp, O0, C, 0, rm0, 0); }));
      t[2].push_back(timeit([&] { return run_ws(A, R, M, R, Wf, C, bp, O1, C, rm1, 1); }));
      // last: the checks below read this variant's output
      t[1].push_back(timeit([&] { return run_ws(A, R, M, R, Wf, C, bp, O1, C, rm1, 1 | 2); }));
    }
    if (ablate) {
      for (int a = 0; a < 3; ++a) std::sort(ta[a].begin(), ta[a].end());
      printf("  ablations (defer): no MFMA %.1f  no fragment reads %.1f  no stores %.1f us\n", ta[0][reps / 2],
             ta[1][reps / 2], ta[2][reps / 2]);
    }
    CK(hipDeviceSynchronize());
    // errors vs fp64 on sampled rows
    const int64_t rows[] = {0, 1, 7, 31, 32, 1000, 2001, 4095, 4096, 77777, M / 2, M - 33, M - 2, M - 1};
    std::vector<float> hw((size_t)C * R), ha(R), h0(C), h1(C);
    CK(hipMemcpy(hw.data(), W, hw.size() * 4, hipMemcpyDeviceToHost));
    std::vector<float> hb(C, 0.0f);
    if (use_bias) CK(hipMemcpy(hb.data(), bias, C * 4, hipMemcpyDeviceToHost));
    double err0 = 0, err1 = 0;
    for (int64_t r : rows) {
      CK(hipMemcpy(ha.data(), A + r * R, R * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h0.data(), O0 + r * C, C * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h1.data(), O1 + r * C, C * 4, hipMemcpyDeviceToHost));
      for (int c = 0; c < C; ++c) {
        double ref = hb[c], mag = fabs(hb[c]);
        for (int k = 0; k < R; ++k) {
          ref += (double)ha[k] * hw[(size_t)c * R + k];
          mag += fabs((double)ha[k] * hw[(size_t)c * R + k]);
        }
        const double d = mag > 0 ? 1.0 / mag : 1.0;
        err0 = std::max(err0, fabs(h0[c] - ref) * d);
        err1 = std::max(err1, fabs(h1[c] - ref) * d);
        if (!std::isfinite(h1[c]) || fabs(h1[c] - ref) * d > 1e-5) {
          if (err1 > 1e-5) {
            printf("  BAD %s row %lld col %d: ws %.9g ref %.9g shipped %.9g\n", s.name, (long long)r, c,
                   h1[c], ref, h0[c]);
          }
        }
      }
    }
    // rmax equal
    const int64_t ng = (M + 31) / 32;
    std::vector<float> g0(ng), g1(ng);
    CK(hipMemcpy(g0.data(), rm0, ng * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g1.data(), rm1, ng * 4, hipMemcpyDeviceToHost));
    int64_t rbad = 0;
    for (int64_t g = 0; g < ng; ++g) rbad += g0[g] != g1[g];
    double us[3], mn[3];
    for (int v = 0; v < 3; ++v) {
      std::sort(t[v].begin(), t[v].end());
      us[v] = t[v][t[v].size() / 2];
      mn[v] = t[v][0];
      tot[v] += us[v];
    }
    const double bytes = (double)M * (R + C) * 4;
    printf("%-10s R=%3d C=%3d bias=%d  shipped %7.1f (min %7.1f)  ws-d1late %7.1f (min %7.1f)  ws-defer %7.1f (min %7.1f)  ws/shipped %.3f  [%.2f TB/s]  err shipped %.2e ws %.2e  rmax mismatches %lld\n",
           s.name, R, C, (int)use_bias, us[0], mn[0], us[1], mn[1], us[2], mn[2],
           std::min(us[1], us[2]) / us[0], bytes / std::min(us[1], us[2]) / 1e6, err0, err1, (long long)rbad);
    fflush(stdout);
  }
  printf("total shipped %.1f  ws %.1f  ws-defer %.1f us\n", tot[0], tot[1], tot[2]);
  return 0;
}
