// tr16_gather_probe.hip — item_scores.hip's tile_gather_h (the CE backward's
// transposed fragment gather) on a swizzled image tile whose element (row,
// half-column) holds row * 256 + col, against the expected rows crow(8 kb +
// k, h) of column ch0 + (lane & 31): prints mismatches per (D, kb, plane).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __fp16 fp16x4_t __attribute__((__vector_size__(8)));
typedef __attribute__((address_space(3))) fp16x4_t* lds_h4_ptr;

// EV: the even swizzle (2 r mod NS) item_scores.hip's fused CE kernels use;
// otherwise r mod NS, the other streamed tiles' swizzle
template <int D, bool EV>
__device__ __forceinline__ int swz(int r) {
  constexpr int NS = D / 4;
  return EV ? (2 * r) & (NS - 1) : r % NS;
}

template <int D, bool EV>
__device__ __forceinline__ f16x8 tile_gather_h(const _Float16* tile, int ch0, int kb, int lane) {
  const int h = lane >> 5, q = (lane >> 2) & 3;
  const int c = ch0 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  f16x8 r;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * kb + 8 * i + 4 * h + q;
    const _Float16* a = tile + row * 2 * D + (((c >> 3) ^ swz<D, EV>(row)) << 3) + (c & 7);
    const fp16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_h4_ptr)(a));
#pragma unroll
    for (int e = 0; e < 4; ++e) r[4 * i + e] = __builtin_bit_cast(_Float16, v[e]);
  }
  return r;
}

template <int D, bool EV>
__global__ void k(int* bad, int enc) {
  __shared__ __attribute__((aligned(16))) _Float16 t[32 * 2 * D];
  // image: logical half-column lc of row r stored at physical slot (lc>>3) ^ swz(r);
  // enc 0: the element holds its row, enc 1: its logical column (exact in f16)
  for (int i = threadIdx.x; i < 32 * 2 * D; i += 64) {
    const int r = i / (2 * D), pc = i % (2 * D);
    const int lc = ((((pc >> 3) ^ swz<D, EV>(r))) << 3) + (pc & 7);   // XOR is an involution
    t[i] = (_Float16)(float)(enc == 0 ? r : lc);
  }
  __syncthreads();
  const int lane = threadIdx.x, h = lane >> 5;
  int nbad = 0;
  for (int kb = 0; kb < 2; ++kb)
    for (int p = 0; p < 2; ++p)
      for (int n = 0; n < D / 32; ++n) {
        const int ch0 = p * D + 32 * n;
        const f16x8 g = tile_gather_h<D, EV>(t, ch0, kb, lane);
        for (int kk = 0; kk < 8; ++kk) {
          const int row = 16 * kb + 8 * (kk >> 2) + 4 * h + (kk & 3);
          const int want = enc == 0 ? row : ch0 + (lane & 31);
          if ((int)(float)g[kk] != want) ++nbad;
        }
      }
  atomicAdd(bad, nbad);
}

// rows each lane receives (D = 32, r mod NS swizzle, kb = 0), for the record
__global__ void dump(float* o) {
  constexpr int D = 32;
  __shared__ __attribute__((aligned(16))) _Float16 t[32 * 2 * D];
  for (int i = threadIdx.x; i < 32 * 2 * D; i += 64) t[i] = (_Float16)(float)(i / (2 * D));
  __syncthreads();
  const f16x8 g = tile_gather_h<D, false>(t, 0, 0, threadIdx.x);
  for (int k = 0; k < 8; ++k) o[threadIdx.x * 8 + k] = (float)g[k];
}

int main() {
  int* d;
  (void)hipMalloc(&d, 16);
  int h;
  for (int ev = 0; ev < 2; ++ev)
    for (int enc = 0; enc < 2; ++enc) {
      const char* sw = ev ? "2r mod NS" : "r mod NS";
      (void)hipMemset(d, 0, 4);
      if (ev) k<32, true><<<1, 64>>>(d, enc); else k<32, false><<<1, 64>>>(d, enc);
      (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
      printf("swizzle %-9s D=32  enc %d mismatches %d\n", sw, enc, h);
      (void)hipMemset(d, 0, 4);
      if (ev) k<64, true><<<1, 64>>>(d, enc); else k<64, false><<<1, 64>>>(d, enc);
      (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
      printf("swizzle %-9s D=64  enc %d mismatches %d\n", sw, enc, h);
      (void)hipMemset(d, 0, 4);
      if (ev) k<128, true><<<1, 64>>>(d, enc); else k<128, false><<<1, 64>>>(d, enc);
      (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
      printf("swizzle %-9s D=128 enc %d mismatches %d\n", sw, enc, h);
    }
  float* o;
  (void)hipMalloc(&o, 64 * 8 * 4);
  dump<<<1, 64>>>(o);
  float ho[64 * 8];
  (void)hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
  printf("rows received (D=32, kb=0; expected 8i + 4h + e for element 4i + e):\n");
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int k = 0; k < 8; ++k) printf(" %2d", (int)ho[l * 8 + k]);
    printf("\n");
  }
  return 0;
}
