// gemm_epi.hip — epilogue-schedule experiments on the f16x3 NT GEMM
// (csrc/gemm_half.hip) at the encoder's packed row count.
//
// The 256 x 256 tiles (C % 256 == 0) store their 256 KB of results at the
// tile's end; every workgroup runs the same tile lengths, so all CUs store at
// once and then all load at once.  Variants, alternated per shape:
//   prod     launch_gemm_nt_h as shipped
//   stagger  the same two-phase kernel, odd workgroups run their tail tiles
//            (256 x 64) first, so half the chip is offset by a tail tile
//   nb4      256 x 128 main tiles with the deferred epilogue (a block stored
//            per k-step during the next tile) even where C % 256 == 0
// Every variant's output is compared bitwise with prod's.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       tools/gemm_epi.hip -o tools/bin/gemm_epi
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

namespace {
template <int NB>
__global__ void __launch_bounds__(N_THREADS, 1)
k_stagger(int64_t lda, int R, const f16x8* __restrict__ Wf, const int* __restrict__ ew, int C,
          int64_t ldo, NtPhase mp, NtPhase tp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bid = (int)blockIdx.x;
  const bool tail_first = (bid & 1) != 0;
  for (int ph = 0; ph < 2; ++ph) {
    const bool main_now = (ph == 0) != tail_first;
    if (main_now) {
      if (bid < mp.grid)
        nt_h_body<false, true, NB>(smem, bid, mp.grid, mp.A, lda, mp.M, R, Wf, ew, C, nullptr,
                                   mp.out, ldo, nullptr, mp.m_tiles, nullptr, DropSpec{}, 0,
                                   nullptr, nullptr);
    } else {
      if (bid < tp.grid)
        nt_h_body<false, true, 2>(smem, bid, tp.grid, tp.A, lda, tp.M, R, Wf, ew, C, nullptr,
                                  tp.out, ldo, nullptr, tp.m_tiles, nullptr, DropSpec{}, 0,
                                  nullptr, nullptr);
    }
    __syncthreads();
  }
}
}  // namespace

// variant 1: stagger; variant 2: NB = 4 main tiles
int launch_variant(int v, const float* A, int64_t M, int R, const void* Wf, int C, float* out,
                   hipStream_t st) {
  const int G0 = num_cus() / 8 * 8;
  const bool nb8 = C % 256 == 0 && v != 2;
  const int nct0 = C / (nb8 ? 256 : 128);
  const int64_t rows_round = (int64_t)(G0 / nct0) * N_BM;
  const int64_t M_main = M / rows_round * rows_round;
  const f16x8* wf = (const f16x8*)Wf;
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * R * 4);
  const NtPhase mp = nt_phase(A, R, 0, M_main, out, C, nullptr, C, nb8 ? 256 : 128, G0);
  const NtPhase tp = nt_phase(A, R, M_main, M - M_main, out, C, nullptr, C, 64, G0);
  if (v == 2) {
    run_nt_h2<false, 4>(R, R, wf, ew, C, nullptr, C, DropSpec{}, mp, tp, st);
    return launch_status("nb4");
  }
  constexpr int lds8 = NtCfg<8>::LDS, lds4 = NtCfg<4>::LDS;
  const unsigned grid = (unsigned)std::max(mp.grid, tp.grid);
  if (nb8) {
    (void)hipFuncSetAttribute((const void*)k_stagger<8>, hipFuncAttributeMaxDynamicSharedMemorySize, lds8);
    k_stagger<8><<<grid, N_THREADS, lds8, st>>>(R, R, wf, ew, C, C, mp, tp);
  } else {
    (void)hipFuncSetAttribute((const void*)k_stagger<4>, hipFuncAttributeMaxDynamicSharedMemorySize, lds4);
    k_stagger<4><<<grid, N_THREADS, lds4, st>>>(R, R, wf, ew, C, C, mp, tp);
  }
  return launch_status("stagger");
}
}  // namespace rb
using namespace rb;

#include <algorithm>
#include <cstdlib>
#include <cstring>
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
  const int reps = argc > 2 ? atoi(argv[2]) : 9;
  struct Shape { const char* name; int R, C; };
  const Shape shapes[] = {{"in.fwd", 128, 512}, {"in.dX", 512, 128}, {"gates.fwd", 256, 512},
                          {"gates.dX", 512, 256}, {"out.fwd", 256, 128}, {"out.dX", 128, 256},
                          {"w2.fwd", 512, 128}, {"w2.dX", 128, 512}};
  float *A, *W, *O0, *O1;
  void* Wf;
  CK(hipMalloc(&A, M * 512 * 4));
  CK(hipMalloc(&O0, M * 512 * 4));
  CK(hipMalloc(&O1, M * 512 * 4));
  CK(hipMalloc(&W, 512 * 512 * 4));
  CK(hipMalloc(&Wf, 512 * 512 * 4 + 4096));
  fill<<<4096, 256>>>(A, M * 512, 1, 2.0f);
  fill<<<256, 256>>>(W, 512 * 512, 2, 0.1f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* vn[3] = {"prod", "stagger", "nb4"};
  double tot[3] = {0, 0, 0};
  std::vector<float> h0, h1;
  for (const Shape& s : shapes) {
    rb_split_job job{W, s.R, s.C, s.R, 0, Wf};
    CK((hipError_t)launch_split_weights_h(&job, 1, 0));
    std::vector<float> ts[3];
    for (int rep = 0; rep < reps; ++rep) {
      for (int v = 0; v < 3; ++v) {
        float* O = v == 0 ? O0 : O1;
        CK(hipEventRecord(e0, 0));
        const int rc = v == 0 ? launch_gemm_nt_h(A, s.R, M, s.R, Wf, s.C, nullptr, O, s.C, 0,
                                                 nullptr, 0)
                              : launch_variant(v, A, M, s.R, Wf, s.C, O, 0);
        if (rc) { fprintf(stderr, "launch failed %d\n", rc); return 1; }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts[v].push_back(ms * 1e3f);
        if (rep == 0 && v > 0) {
          h0.resize((size_t)M * s.C);
          h1.resize((size_t)M * s.C);
          CK(hipMemcpy(h0.data(), O0, h0.size() * 4, hipMemcpyDeviceToHost));
          CK(hipMemcpy(h1.data(), O1, h1.size() * 4, hipMemcpyDeviceToHost));
          if (memcmp(h0.data(), h1.data(), h0.size() * 4) != 0)
            printf("  %s %s: output differs from prod\n", s.name, vn[v]);
        }
      }
    }
    printf("%-10s R=%3d C=%3d", s.name, s.R, s.C);
    for (int v = 0; v < 3; ++v) {
      std::sort(ts[v].begin(), ts[v].end());
      const double us = ts[v][ts[v].size() / 2];
      tot[v] += us;
      printf("  %s %7.1f", vn[v], us);
    }
    printf("\n");
  }
  printf("total");
  for (int v = 0; v < 3; ++v) printf("  %s %.1f", vn[v], tot[v]);
  printf("\n");
  return 0;
}
