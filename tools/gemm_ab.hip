// gemm_ab.hip — the f16x3 NT GEMM (csrc/gemm_half.hip) timed at the
// encoder's packed row count on its eight projection shapes, built against a
// given source tree (-DGEMM_DIR=...), so two trees can be A/B-timed and their
// outputs compared by checksum (FNV-1a over the output bytes).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       -DGEMM_DIR=../datamining_recblr_amd/csrc tools/gemm_ab.hip -o tools/bin/gemm_ab
#include <cstdio>

#define STR2(x) #x
#define STR(x) STR2(x)
#include STR(GEMM_DIR/gemm_half.hip)
#include STR(GEMM_DIR/gemm_small.hip)

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
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// max |x| of every 32-row group of a [n, c] row-major matrix
__global__ void gmax32(const float* x, int64_t n, int c, float* out) {
  const int64_t g = blockIdx.x;
  float m = 0.0f;
  for (int64_t i = threadIdx.x; i < 32LL * c; i += blockDim.x) {
    const int64_t r = g * 32 + i / c;
    if (r < n) m = fmaxf(m, fabsf(x[r * c + i % c]));
  }
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float sm[4];
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[g] = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
}

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
  const int reps = argc > 2 ? atoi(argv[2]) : 9;
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
  double tot = 0;
  std::vector<uint32_t> h;
  for (const Shape& s : shapes) {
    rb_split_job job{W, s.R, s.C, s.R, 0, Wf};
    CK((hipError_t)launch_split_weights_h(&job, 1, 0));
    std::vector<float> ts;
    for (int rep = 0; rep < reps; ++rep) {
      CK(hipEventRecord(e0, 0));
      if (launch_gemm_nt_h(A, s.R, M, s.R, Wf, s.C, nullptr, O, s.C, 0, nullptr, 0)) return 1;
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    h.resize((size_t)M * s.C);
    CK(hipMemcpy(h.data(), O, h.size() * 4, hipMemcpyDeviceToHost));
    uint64_t f = 1469598103934665603ull;
    for (uint32_t w : h) { f ^= w; f *= 1099511628211ull; }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    tot += us;
    const double bytes = (double)M * (s.R + s.C) * 4;
    printf("%-10s R=%3d C=%3d  %7.1f us  %5.2f TB/s  min %7.1f  fnv %016llx\n", s.name, s.R, s.C,
           us, bytes / us / 1e6, ts[0], (unsigned long long)f);
  }
  printf("total %.1f us\n", tot);
  // weight gradients dW = dY^T X (split partials, no column sum)
  struct TShape { const char* name; int N, K, S; };
  const TShape tshapes[] = {{"gates.dW", 512, 256, 64}, {"in.dW", 512, 128, 128},
                            {"w2.dW", 128, 512, 128}, {"out.dW", 128, 256, 256},
                            // the CE backward's products (B = 2048 rows of P, V = 10544
                            // rows of P^T): M below, N, K, S
                            {"ce.ditems", 10752, 128, 8}, {"ce.dseq", 2048, 128, 32}};
  const int64_t tM[] = {M, M, M, M, 2048, 10544};
  float *Y, *ymax, *xmax, *parts;
  CK(hipMalloc(&Y, M * 512 * 4));
  CK(hipMalloc(&ymax, (M / 32 + 1) * 4));
  CK(hipMalloc(&xmax, (M / 32 + 1) * 4));
  CK(hipMalloc(&parts, (size_t)16 << 20 << 2));
  fill<<<4096, 256>>>(Y, M * 512, 3, 1.0f);
  double ttot = 0;
  for (int si = 0; si < 6; ++si) {
    const TShape& s = tshapes[si];
    const int64_t Mt = tM[si];
    if ((int64_t)Mt * s.N > M * 512 || (int64_t)s.S * s.N * s.K > (16 << 20)) return 2;
    gmax32<<<(unsigned)((Mt + 31) / 32), 256>>>(Y, Mt, s.N, ymax);
    gmax32<<<(unsigned)((Mt + 31) / 32), 256>>>(A, Mt, s.K, xmax);
    std::vector<float> ts;
    for (int rep = 0; rep < reps; ++rep) {
      CK(hipEventRecord(e0, 0));
      if (launch_gemm_tn_h(Y, s.N, A, s.K, Mt, s.N, s.K, ymax, xmax, parts, s.S, 0)) return 1;
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1e3f);
    }
    h.resize((size_t)s.S * s.N * s.K);
    CK(hipMemcpy(h.data(), parts, h.size() * 4, hipMemcpyDeviceToHost));
    uint64_t f = 1469598103934665603ull;
    for (uint32_t w : h) { f ^= w; f *= 1099511628211ull; }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    ttot += us;
    const double bytes = (double)Mt * (s.N + s.K) * 4;
    printf("%-10s N=%3d K=%3d S=%3d  %7.1f us  %5.2f TB/s  min %7.1f  fnv %016llx\n", s.name, s.N,
           s.K, s.S, us, bytes / us / 1e6, ts[0], (unsigned long long)f);
  }
  printf("tn total %.1f us\n", ttot);
  return 0;
}
