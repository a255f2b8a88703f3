// tr16_probe.hip — what ds_read_b64_tr_b16 delivers: a 32 x 64 f16 LDS
// matrix with element (row, col) = row * 64 + col (exact in f16), each lane
// of a 16-lane group addressing row q = (lane >> 2) & 3, columns 4p .. 4p+3
// (p = lane & 3) of a 4-row block; prints every lane's 4 elements.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __fp16 fp16x4_t __attribute__((__vector_size__(8)));
typedef __attribute__((address_space(3))) fp16x4_t* lds_h4_ptr;
__global__ void k(float* out) {
  __shared__ __attribute__((aligned(16))) _Float16 t[32 * 64];
  for (int i = threadIdx.x; i < 32 * 64; i += 64) t[i] = (_Float16)(float)i;
  __syncthreads();
  const int lane = threadIdx.x, q = (lane >> 2) & 3, p = lane & 3;
  const int row = 4 * (lane >> 5) + q;               // lane half h: rows 4h .. 4h + 3
  const int col = 16 * ((lane >> 4) & 1) + 4 * p;    // group: 16 columns
  const fp16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_h4_ptr)(t + row * 64 + col));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = (float)v[e];
}
int main() {
  float* d;
  hipMalloc(&d, 64 * 4 * 4);
  k<<<1, 64>>>(d);
  float h[256];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int e = 0; e < 4; ++e) {
      const int v = (int)h[l * 4 + e];
      printf("  (r%2d,c%2d)", v / 64, v % 64);
    }
    printf("\n");
  }
  return 0;
}
