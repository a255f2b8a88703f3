// ce_tn_probe.hip — the CE backward's two products on the weight-gradient
// kernel (rb_gemm_tn_h; scoring._bwd_f16) at the bench shape (B = 2048,
// V = 10,544 padded to 10,752, d = 128) in three cache states: warm (the same
// P re-read), cold (1 GiB written between reps) and right after P is
// rewritten (as in the step, where rb_item_ce_probs_h_both writes both
// layouts just before), over row-split counts S.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       -DGEMM_DIR=../datamining_recblr_amd/csrc tools/ce_tn_probe.hip -o tools/bin/ce_tn_probe
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

__global__ void fill(float* p, int64_t n, uint32_t seed, float scale) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = scale * ((h & 0xffffff) / 16777216.0f);
  }
}

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

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 7;
  const int64_t B = 2048, V = 10544, Vp = 10752, d = 128;
  float *P, *Pt, *seq, *tab, *pmax, *ptmax, *smax, *tmax, *parts, *junk;
  CK(hipMalloc(&P, B * Vp * 4));
  CK(hipMalloc(&Pt, V * B * 4));
  CK(hipMalloc(&seq, B * d * 4));
  CK(hipMalloc(&tab, V * d * 4));
  CK(hipMalloc(&pmax, (B / 32) * 4));
  CK(hipMalloc(&ptmax, (V / 32 + 1) * 4));
  CK(hipMalloc(&smax, (B / 32) * 4));
  CK(hipMalloc(&tmax, (V / 32 + 1) * 4));
  const size_t PARTS = (size_t)64 * Vp * d * 4;   // the largest S x N x K here
  CK(hipMalloc(&parts, PARTS));
  const int64_t JUNK = (int64_t)1 << 28;   // 1 GiB of floats
  CK(hipMalloc(&junk, JUNK * 4));
  fill<<<4096, 256>>>(P, B * Vp, 1, 1e-3f);
  fill<<<4096, 256>>>(Pt, V * B, 2, 1e-3f);
  fill<<<256, 256>>>(seq, B * d, 3, 1.0f);
  fill<<<256, 256>>>(tab, V * d, 4, 0.1f);
  gmax32<<<(unsigned)(B / 32), 256>>>(P, B, (int)Vp, pmax);
  gmax32<<<(unsigned)((V + 31) / 32), 256>>>(Pt, V, (int)B, ptmax);
  gmax32<<<(unsigned)(B / 32), 256>>>(seq, B, (int)d, smax);
  gmax32<<<(unsigned)((V + 31) / 32), 256>>>(tab, V, (int)d, tmax);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* modes[] = {"warm", "cold", "afterwrite"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int which = 0; which < 2; ++which) {
      const int Ss[] = {8, 16, 32, 64};
      for (int S : Ss) {
        if (which == 0 && (int64_t)S * 32 > B) continue;
        std::vector<float> ts;
        for (int rep = 0; rep < reps; ++rep) {
          if (mode == 1) fill<<<4096, 256>>>(junk, JUNK, 9 + rep, 1.0f);
          if (mode == 2) {
            fill<<<4096, 256>>>(junk, JUNK, 9 + rep, 1.0f);
            fill<<<4096, 256>>>(P, B * Vp, 1, 1e-3f);    // both layouts rewritten, as the
            fill<<<4096, 256>>>(Pt, V * B, 2, 1e-3f);    // probs kernel does before them
          }
          CK(hipEventRecord(e0, 0));
          const size_t need = (size_t)S * (which == 0 ? Vp : B) * d * 4;
          if (need > PARTS) return 3;
          int rc = which == 0
                       ? launch_gemm_tn_h(P, Vp, seq, d, B, (int)Vp, (int)d, pmax, smax, parts, S, 0)
                       : launch_gemm_tn_h(Pt, B, tab, d, V, (int)B, (int)d, ptmax, tmax, parts, S, 0);
          if (rc) return 1;
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ts.push_back(ms * 1e3f);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-10s %-7s S=%3d  median %7.1f us  min %7.1f\n", modes[mode],
               which == 0 ? "ditems" : "dseq", S, ts[ts.size() / 2], ts[0]);
      }
    }
  }
  return 0;
}
