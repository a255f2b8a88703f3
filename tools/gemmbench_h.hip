// gemmbench_h.hip — timing of the f16 two-part split GEMM (csrc/gemm_half.hip)
// on the encoder's projection shapes.  Ablation builds:
//   -DHN_NO_SPLIT / -DHN_NO_MFMA / -DHN_NO_BARRIER / -DHN_HALF_B (wrong results: run with
//   GB_NOCHECK=1) / -DHN_NO_ADMA / -DHN_NSA=n / -DHN_LATE_DMA / -DHN_NARROW_STORE / -DHN_WAVES=n;
//   -DHN_STAMPS prints each
//   k-step segment's share of the waves' cycles
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       tools/gemmbench_h.hip -o tools/bin/gemmbench_h
#include <cstdio>

#include "../datamining_recblr_amd/csrc/gemm_half.hip"
#include "../datamining_recblr_amd/csrc/gemm_small.hip"

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
  struct Shape { const char* name; int R, C; };
  const Shape shapes[] = {{"in.fwd", 128, 512}, {"in.dX", 512, 128}, {"gates.fwd", 256, 512},
                          {"gates.dX", 512, 256}, {"out.fwd", 256, 128}, {"out.dX", 128, 256},
                          {"w2.fwd", 512, 128}, {"w2.dX", 128, 512}};
  float *A, *W, *O;
  void* Wf;
  CK(hipMalloc(&A, M * 512 * 4));
  CK(hipMalloc(&O, M * 512 * 4));
  CK(hipMalloc(&W, 512 * 512 * 4));
  CK(hipMalloc(&Wf, 512 * 512 * 4 + 4096));
  fill<<<4096, 256>>>(A, M * 512, 1, 2.0f);
  fill<<<256, 256>>>(W, 512 * 512, 2, 0.1f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  double tot = 0, totb = 0;
  for (const Shape& s : shapes) {
    rb_split_job job{W, s.R, s.C, s.R, 0, Wf};
    CK((hipError_t)launch_split_weights_h(&job, 1, 0));
    std::vector<float> ts;
    for (int rep = 0; rep < 12; ++rep) {
      CK(hipEventRecord(e0, 0));
      int rc = launch_gemm_nt_h(A, s.R, M, s.R, Wf, s.C, nullptr, O, s.C, 0, nullptr, 0);
      if (rc) { fprintf(stderr, "launch failed %d\n", rc); return 1; }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    {
      // sampled check against fp64 on the host: rows at both ends and a stride
      std::vector<float> hw((size_t)s.C * s.R), ha(s.R), ho(s.C);
      CK(hipMemcpy(hw.data(), W, hw.size() * 4, hipMemcpyDeviceToHost));
      double worst = 0;
      for (int64_t r = 0; r < M; r += (r < 300 || r > M - 300) ? 1 : 997) {
        CK(hipMemcpy(ha.data(), A + r * s.R, s.R * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ho.data(), O + r * s.C, s.C * 4, hipMemcpyDeviceToHost));
        for (int c = 0; c < s.C; ++c) {
          double ref = 0, mag = 0;
          for (int k = 0; k < s.R; ++k) {
            ref += (double)ha[k] * hw[(size_t)c * s.R + k];
            mag += fabs((double)ha[k] * hw[(size_t)c * s.R + k]);
          }
          worst = std::max(worst, fabs(ho[c] - ref) / (mag + 1e-30));
        }
      }
      if (!(worst < 1e-6)) {
        fprintf(stderr, "%s: WRONG RESULT (max err %.3e)\n", s.name, worst);
        if (!getenv("GB_NOCHECK")) return 2;   // ablation builds: time anyway
      }
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    const double fl = 2.0 * M * s.R * s.C;
    const double by = 4.0 * M * (s.R + s.C);
    tot += us;
    totb += by;
    printf("%-10s R=%3d C=%3d  %7.1f us  %6.1f TF  %6.2f TB/s\n", s.name, s.R, s.C, us,
           fl / us / 1e6, by / us / 1e6);
#ifdef HN_STAMPS
    {
      // segment shares summed over every wave of the last run
      std::vector<unsigned long long> st(2048 * 8 * HN_NSEG);
      CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(hn_stamps), st.size() * 8));
      double seg[HN_NSEG] = {0}, all = 0;
      for (size_t w = 0; w < st.size() / HN_NSEG; ++w)
        for (int k = 0; k < HN_NSEG; ++k) seg[k] += (double)st[w * HN_NSEG + k];
      for (int k = 0; k < HN_NSEG; ++k) all += seg[k];
      const char* nm[HN_NSEG] = {"wait", "barrier", "sub0", "dma+st", "sub1", "tile"};
      printf("    stamps (share of wave time):");
      for (int k = 0; k < HN_NSEG; ++k) printf(" %s %.3f", nm[k], seg[k] / all);
      printf("  | mean per-wave cycles %.0f\n", all / (256.0 * 8));
    }
#endif
  }
  printf("total %.1f us  (%.2f TB/s)\n", tot, totb / tot / 1e6);

  // weight gradients (rb_gemm_tn_h): dW[N, K] = dY^T X over M rows, row-chunk
  // partials [S, N, K] (S as linear._tn_splits picks for 256 CUs); the
  // operands' 32-row-group maxima: the fill's bound (|x| <= 1)
  struct TShape { const char* name; int N, K; };
  const TShape tsh[] = {{"gates.dW", 512, 256}, {"in.dW", 512, 128}, {"w2.dW", 128, 512},
                        {"out.dW", 128, 256}};
  float *X, *rm, *parts;
  CK(hipMalloc(&X, M * 512 * 4));
  CK(hipMalloc(&rm, ((M + 31) / 32) * 4));
  CK(hipMalloc(&parts, (size_t)256 * 512 * 256 * 4));
  fill<<<4096, 256>>>(X, M * 512, 3, 2.0f);
  {
    std::vector<float> ones((M + 31) / 32, 1.0f);
    CK(hipMemcpy(rm, ones.data(), ones.size() * 4, hipMemcpyHostToDevice));
  }
  double ttot = 0;
  for (const TShape& t : tsh) {
    const int nt = (t.N / 128) * (t.K / 128);
    const int S = getenv("GB_TN_S") ? atoi(getenv("GB_TN_S"))
                                     : std::max(8, (2 * num_cus() / nt) / 8 * 8);
    std::vector<float> ts;
    for (int rep = 0; rep < 12; ++rep) {
      CK(hipEventRecord(e0, 0));
      int rc = launch_gemm_tn_h(A, t.N, X, t.K, M, t.N, t.K, rm, rm, parts, S, 0);
      if (rc) { fprintf(stderr, "tn launch failed %d\n", rc); return 1; }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    {
      // a few dW entries against fp64 (all M rows)
      std::vector<float> hp((size_t)S * t.N * t.K);
      CK(hipMemcpy(hp.data(), parts, hp.size() * 4, hipMemcpyDeviceToHost));
      std::vector<float> ca(M), cb(M);
      double worst = 0;
      for (int e = 0; e < 6; ++e) {
        const int n = (e * 97) % t.N, k = (e * 61 + 5) % t.K;
        CK(hipMemcpy2D(ca.data(), 4, A + n, (size_t)t.N * 4, 4, M, hipMemcpyDeviceToHost));
        CK(hipMemcpy2D(cb.data(), 4, X + k, (size_t)t.K * 4, 4, M, hipMemcpyDeviceToHost));
        double ref = 0, mag = 0, got = 0;
        for (int64_t m = 0; m < M; ++m) {
          ref += (double)ca[m] * cb[m];
          mag += fabs((double)ca[m] * cb[m]);
        }
        for (int sp = 0; sp < S; ++sp) got += hp[((size_t)sp * t.N + n) * t.K + k];
        worst = std::max(worst, fabs(got - ref) / mag);
      }
      if (!(worst < 1e-6)) {
        fprintf(stderr, "%s: WRONG RESULT (max err %.3e)\n", t.name, worst);
        if (!getenv("GB_NOCHECK")) return 2;
      }
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    const double by = 4.0 * M * (t.N + t.K);
    ttot += us;
    printf("%-10s N=%3d K=%3d S=%3d %7.1f us  %6.1f TF  %6.2f TB/s\n", t.name, t.N, t.K, S, us,
           2.0 * M * t.N * t.K / us / 1e6, by / us / 1e6);
  }
  printf("tn total %.1f us\n", ttot);
  return 0;
}
