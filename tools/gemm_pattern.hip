// gemm_pattern.hip — the NT GEMM's HBM byte pattern without the GEMM: each
// row of A [M, R] fp32 is read once and a row of C fp32 outputs is written
// (out[m, c] = rowsum(A[m, :]) + c), float4 loads and nontemporal float4
// stores, 4 waves x 8 rows per 256-thread block.  The time of this kernel is
// the streaming floor of an out = A W^T with the weights on chip, to set
// beside tools/gemmbench_h's no-MFMA ablation (-DHN_NO_MFMA).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_pattern.hip -o tools/bin/gemm_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// one wave per 8 rows; lane l: row 8 * wave_row + (l >> 3), float4 column
// group (l & 7) + 8 j (reads: R/4 float4 per row over 8 lanes)
template <int R, int C>
__global__ void __launch_bounds__(256) pattern(const float* __restrict__ A, float* __restrict__ out,
                                               int64_t M) {
  const int lane = threadIdx.x & 63;
  const int64_t wrow = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8;
  const int64_t row = wrow + (lane >> 3);
  if (wrow >= M) return;
  const int64_t r = row < M ? row : M - 1;
  const f32x4* a = reinterpret_cast<const f32x4*>(A + r * R);
  f32x4 s = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < R / 32; ++j) s += __builtin_nontemporal_load(a + (lane & 7) + 8 * j);
  float t = s[0] + s[1] + s[2] + s[3];
  t += __shfl_xor(t, 1);
  t += __shfl_xor(t, 2);
  t += __shfl_xor(t, 4);
  if (row >= M) return;
  f32x4* o = reinterpret_cast<f32x4*>(out + row * C);
#pragma unroll
  for (int j = 0; j < C / 32; ++j) {
    const float c0 = (float)(4 * ((lane & 7) + 8 * j));
    __builtin_nontemporal_store(f32x4{t + c0, t + c0 + 1, t + c0 + 2, t + c0 + 3}, o + (lane & 7) + 8 * j);
  }
}

template <int R, int C>
void run(const char* name, const float* A, float* out, int64_t M) {
  const unsigned blocks = (unsigned)((M + 31) / 32);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 5; ++w) pattern<R, C><<<blocks, 256>>>(A, out, M);
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int it = 0; it < iters; ++it) pattern<R, C><<<blocks, 256>>>(A, out, M);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1e3 * ms / iters;
  const double bytes = (double)M * (R + C) * 4;
  printf("%-10s R=%-4d C=%-4d %8.1f us  %6.2f TB/s  (%.3f of 8 TB/s)\n", name, R, C, us,
         bytes / us * 1e-6, bytes / us * 1e-6 / 8.0);
}

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atoll(argv[1]) : 204632;
  float *A, *out;
  CK(hipMalloc(&A, (size_t)M * 512 * 4));
  CK(hipMalloc(&out, (size_t)M * 512 * 4));
  CK(hipMemset(A, 0, (size_t)M * 512 * 4));
  for (int rep = 0; rep < 2; ++rep) {
    run<128, 512>("in.fwd", A, out, M);
    run<512, 128>("in.dX", A, out, M);
    run<256, 512>("gates.fwd", A, out, M);
    run<512, 256>("gates.dX", A, out, M);
    run<256, 128>("out.fwd", A, out, M);
    run<128, 256>("out.dX", A, out, M);
    run<512, 128>("w2.fwd", A, out, M);
    run<128, 512>("w2.dX", A, out, M);
  }
  CK(hipFree(A));
  CK(hipFree(out));
  return 0;
}
