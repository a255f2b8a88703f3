// tr16_gather_probe.hip — item_scores.hip's tile_gather_h (the CE backward's
// transposed fragment gather) on a swizzled image tile whose element (row,
// half-column) holds row * 256 + col, against the expected rows crow(8 kb +
// k, h) of column ch0 + (lane & 31): prints mismatches per (D, kb, plane).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __fp16 fp16x4_t __attribute__((__vector_size__(8)));
typedef __attribute__((address_space(3))) fp16x4_t* lds_h4_ptr;

template <int D>
__device__ __forceinline__ f16x8 tile_gather_h(const _Float16* tile, int ch0, int kb, int lane) {
  constexpr int NS = D / 4;
  const int h = lane >> 5, q = (lane >> 2) & 3;
  const int c = ch0 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  f16x8 r;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * kb + 8 * i + 4 * h + q;
    const _Float16* a = tile + row * 2 * D + (((c >> 3) ^ (row % NS)) << 3) + (c & 7);
    const fp16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_h4_ptr)(a));
#pragma unroll
    for (int e = 0; e < 4; ++e) r[4 * i + e] = __builtin_bit_cast(_Float16, v[e]);
  }
  return r;
}

template <int D>
__global__ void k(int* bad, int enc) {
  constexpr int NS = D / 4;
  __shared__ __attribute__((aligned(16))) _Float16 t[32 * 2 * D];
  // image: logical half-column lc of row r stored at physical slot (lc>>3) ^ (r % NS);
  // enc 0: the element holds its row, enc 1: its logical column (exact in f16)
  for (int i = threadIdx.x; i < 32 * 2 * D; i += 64) {
    const int r = i / (2 * D), pc = i % (2 * D);
    const int lc = ((((pc >> 3) ^ (r % NS))) << 3) + (pc & 7);   // XOR is an involution
    t[i] = (_Float16)(float)(enc == 0 ? r : lc);
  }
  __syncthreads();
  const int lane = threadIdx.x, h = lane >> 5;
  int nbad = 0;
  for (int kb = 0; kb < 2; ++kb)
    for (int p = 0; p < 2; ++p)
      for (int n = 0; n < D / 32; ++n) {
        const int ch0 = p * D + 32 * n;
        const f16x8 g = tile_gather_h<D>(t, ch0, kb, lane);
        for (int kk = 0; kk < 8; ++kk) {
          const int row = 16 * kb + 8 * (kk >> 2) + 4 * h + (kk & 3);
          const int want = enc == 0 ? row : ch0 + (lane & 31);
          if ((int)(float)g[kk] != want) ++nbad;
        }
      }
  atomicAdd(bad, nbad);
}

int main() {
  int* d;
  (void)hipMalloc(&d, 16);
  int h;
  for (int enc = 0; enc < 2; ++enc) {
    (void)hipMemset(d, 0, 4);
    k<32><<<1, 64>>>(d, enc);
    (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("D=32 enc %d mismatches %d\n", enc, h);
    (void)hipMemset(d, 0, 4);
    k<128><<<1, 64>>>(d, enc);
    (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("D=128 enc %d mismatches %d\n", enc, h);
  }
  return 0;
}
