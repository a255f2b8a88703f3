// gate_ab.hip — the gates projection with the BD-LRU epilogue
// (launch_gate_gemm_h, csrc/gemm_half.hip GATE) against the two launches it
// replaces (launch_gemm_nt_h + launch_gate_fwd) at the bench's packed shape
// (lengths ~U{1..200} longest first, H = 256), built against a source tree
// given by -DGEMM_DIR (tools/gate_ab_variants.py builds ablated copies).
#include <cstdio>

#define STR2(x) #x
#define STR(x) STR2(x)
#include STR(GEMM_DIR/gemm_half.hip)
#include STR(GEMM_DIR/gemm_small.hip)
#include STR(GEMM_DIR/gate_scan.hip)

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

__global__ void fill(float* p, int64_t n, uint32_t seed, float scale, float off) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = off + scale * ((h & 0xffffff) / 16777216.0f - 0.5f);
  }
}

static double median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 2048;
  const int reps = argc > 2 ? atoi(argv[2]) : 9;
  const int H = 256, L = 200;
  std::mt19937 rng(7);
  std::vector<int> lens(B);
  for (int& l : lens) l = 1 + (int)(rng() % L);
  std::sort(lens.begin(), lens.end(), std::greater<int>());
  std::vector<int64_t> offs(B + 1, 0);
  for (int b = 0; b < B; ++b) offs[b + 1] = offs[b] + lens[b];
  const int64_t M = offs[B];
  std::vector<int> rinfo(M);
  for (int b = 0; b < B; ++b)
    for (int t = 0; t < lens[b]; ++t)
      rinfo[offs[b] + t] = (b << 9) | (t == lens[b] - 1 ? 256 : 0) | t;
  const int nTc = (L + 15) / 16;
  float *xc, *xz, *W, *gb, *lam, *h0, *rg, *y, *carries, *rmax;
  void *Wf, *tails;
  int *d_rinfo, *err;
  int64_t* d_offs;
  CK(hipMalloc(&xc, M * H * 4));
  CK(hipMalloc(&xz, M * 2 * H * 4));
  CK(hipMalloc(&W, 2 * H * H * 4));
  CK(hipMalloc(&Wf, 2 * H * H * 4 + 4096));
  CK(hipMalloc(&gb, 2 * H * 4));
  CK(hipMalloc(&lam, H * 4));
  CK(hipMalloc(&h0, H * 4));
  CK(hipMalloc(&rg, M * 2 * H * 4));
  CK(hipMalloc(&y, M * H * 4));
  CK(hipMalloc(&carries, (int64_t)B * nTc * H * 4));
  CK(hipMalloc(&rmax, (M / 32 + 1) * 4));
  CK(hipMalloc(&tails, (M / 256 + 1) * H * 8));
  CK(hipMalloc(&d_rinfo, M * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&d_offs, (B + 1) * 8));
  CK(hipMemset(tails, 0, (M / 256 + 1) * H * 8));
  CK(hipMemset(err, 0, 4));
  CK(hipMemcpy(d_rinfo, rinfo.data(), M * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_offs, offs.data(), (B + 1) * 8, hipMemcpyHostToDevice));
  fill<<<4096, 256>>>(xc, M * H, 1, 1.0f, 0.2f);
  fill<<<4096, 256>>>(xz, M * 2 * H, 2, 2.0f, 0.0f);
  fill<<<256, 256>>>(W, 2 * H * H, 3, 0.1f, 0.0f);
  fill<<<4, 256>>>(gb, 2 * H, 4, 0.2f, 0.0f);
  fill<<<4, 256>>>(lam, H, 5, 2.0f, -4.0f);
  fill<<<4, 256>>>(h0, H, 6, 1.0f, 0.0f);
  rb_split_job job{W, H, 2 * H, H, 0, Wf};
  CK((hipError_t)launch_split_weights_h(&job, 1, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t epoch = 0;
  auto time_it = [&](auto&& fn) {
    std::vector<float> ts;
    for (int rep = 0; rep < reps; ++rep) {
      CK(hipEventRecord(e0, 0));
      fn();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    return median(ts);
  };
  const double t_gemm = time_it([&] {
    launch_gemm_nt_h(xc, H, M, H, Wf, 2 * H, nullptr, rg, 2 * H, 0, rmax, 0);
  });
  const double t_scan = time_it([&] {
    launch_gate_fwd(rg, 2 * H, xc, H, xz + H, 2 * H, lam, gb, h0, 0, y, H, carries, B, L, H,
                    d_offs, 0);
  });
  const double t_gate = time_it([&] {
    ++epoch;
    launch_gate_gemm_h(xc, H, M, H, Wf, xz + H, 2 * H, gb, lam, h0, rg, 2 * H, y, H, nullptr,
                       nullptr, carries, nTc, d_rinfo, rmax, tails, epoch, err, 0);
  });
  int herr = 0;
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  printf("%s M=%lld  gemm %.1f us  gate_scan_fwd %.1f us  (sum %.1f)  gate_gemm %.1f us  err %d\n",
         STR(VARIANT), (long long)M, t_gemm, t_scan, t_gemm + t_scan, t_gate, herr);
  return 0;
}
