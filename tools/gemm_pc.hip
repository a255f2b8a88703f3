// gemm_pc.hip — producer/consumer experiment for the f16x3 NT GEMM
// (csrc/gemm_half.hip, k_gemm_nt_h): the same operands, split and products,
// with the work divided by role inside each 512-thread workgroup:
//   waves 0-3 (consumers, one per SIMD): a 64-row slice of a 256 x 128 tile
//     each (2 row blocks x 4 column blocks, 128 accumulators): LDS fragment
//     reads, the A split, the MFMAs, the tile-end epilogue — no DMA;
//   waves 4-7 (producers): every LDS-DMA of the A rows and weight fragments,
//     NSA / NSB-slot rings, two k-steps ahead; each waits (counted vmcnt) for
//     the next step's pieces before the k-step barrier.
// The B fragments of a substep are read once and used by both row blocks
// (half the B LDS reads per output of k_gemm_nt_h's 256 x 128 tiles).
// Timed against launch_gemm_nt_h on the encoder's eight projection shapes at
// whole rounds of rows (no tail), outputs compared with fp64 samples.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -I include \
//       tools/gemm_pc.hip -o tools/bin/gemm_pc
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
#ifndef PC_NSA
#define PC_NSA 3
#endif
constexpr int P_NSA = PC_NSA, P_NSB = 3;
constexpr int P_BM = 256, P_BN = 128, P_BK = 32;
constexpr int P_A_STAGE = P_BM * P_BK * 4;      // 32 KB
constexpr int P_BFRAG = 16;                     // 4 column blocks x 2 substeps x 2 planes
constexpr int P_B_STAGE = P_BFRAG * 1024;       // 16 KB
constexpr int P_RING = P_NSA * P_A_STAGE + P_NSB * P_B_STAGE;
constexpr int P_LDS = P_RING + 1024 * 4;        // + column exponents (C <= 1024)

__device__ unsigned g_pc_flags;

__global__ void __launch_bounds__(512, 1)
k_gemm_nt_pc(const float* __restrict__ A, int64_t lda, int64_t M, int R,
             const f16x8* __restrict__ Wf, const int* __restrict__ ew, int C,
             float* __restrict__ out, int64_t ldo, int m_tiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool consumer = wave < 4;
  const int nct = C / P_BN;
  const int KT = R / P_BK;
  const int KB16 = R / 16;
  const int n_tiles = ((m_tiles + 7) >> 3) * 8 * nct;
  const int G = gridDim.x;
  const int bid = blockIdx.x;
  const int my_tiles = bid < n_tiles ? (n_tiles - 1 - bid) / G + 1 : 0;
  const int U = my_tiles * KT;
  if (U == 0) return;
  int* s_ew = reinterpret_cast<int*>(smem + P_RING);
  for (int c = tid; c < C; c += 512) s_ew[c] = ew[c];
  __syncthreads();
  auto tile_of = [&](int i, int& mt, int& ct) {
    const int T = bid + i * G;
    const int g = T >> 3;
    ct = g % nct;
    mt = (g / nct) * 8 + (T & 7);
  };
  const uint32_t smem_base = (uint32_t)(uintptr_t)(lds_ptr_t)smem;

  if (!consumer) {
    // ---------------- producers: waves 4-7, p = wave - 4 -------------------
    const int p = wave - 4;
    int a_i = 0, a_kt = 0, a_slot = 0;
    const char* a_base = nullptr;
    int a_off[8];
    auto a_tile = [&]() {
      int mt, ct;
      tile_of(a_i, mt, ct);
      const int64_t r0 = (int64_t)mt * P_BM + p * 64;
      a_base = reinterpret_cast<const char*>(A + r0 * lda);
      const int64_t lim = M - 1 - r0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int rr = q * 8 + (lane >> 3);
        const int64_t r = rr < lim ? rr : lim;
        const int srow = p * 64 + rr;
        const int lc = (lane & 7) ^ ((srow >> 1) & 7);
        a_off[q] = (int)(r * lda * 4) + lc * 16;
      }
    };
    int b_i = 0, b_kt = 0, b_slot = 0;
    const f16x8* b_base = nullptr;
    auto b_tile = [&]() {
      int mt, ct;
      tile_of(b_i, mt, ct);
      b_base = Wf + (int64_t)ct * 4 * KB16 * 2 * 64 + lane;
    };
    auto issue = [&]() {
      char* st = smem + a_slot * P_A_STAGE + p * 8192;
      const char* b = a_base + a_kt * (P_BK * 4);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        __builtin_amdgcn_global_load_lds((const void*)(b + a_off[q]), (lds_ptr_t)(st + q * 1024),
                                         16, 0, 0);
      char* sbs = smem + P_NSA * P_A_STAGE + b_slot * P_B_STAGE;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = p * 4 + q;
        const int n = f >> 2, s = (f >> 1) & 1, pl = f & 1;
        const f16x8* src = b_base + ((n * KB16 + b_kt * 2 + s) * 2 + pl) * 64;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(sbs + f * 1024), 16, 0, 0);
      }
      a_slot = a_slot + 1 == P_NSA ? 0 : a_slot + 1;
      b_slot = b_slot + 1 == P_NSB ? 0 : b_slot + 1;
      if (++a_kt == KT) {
        a_kt = 0;
        if (++a_i < my_tiles) a_tile();
      }
      if (++b_kt == KT) {
        b_kt = 0;
        if (++b_i < my_tiles) b_tile();
      }
    };
    a_tile();
    b_tile();
    constexpr int LA = P_NSA - 1;   // steps in flight (NSB >= NSA assumed)
    int issued = 0;
    for (; issued < LA && issued < U; ++issued) issue();
    // step 0 landed: its 12 pieces are the oldest
    if (issued >= 2) hwait_vm<12 * (LA - 1)>(); else hwait_vm<0>();
    __builtin_amdgcn_s_barrier();
    for (int u = 0; u < U; ++u) {
      // slot of step u + LA was read at step u - 1 (finished: the barrier)
      if (issued < U) { issue(); ++issued; }
      // step u + 1 landed: the pieces of the steps after it may stay in flight
      const int after = issued - (u + 2);   // steps issued beyond u + 1
      if (after >= 2) hwait_vm<24>();
      else if (after == 1) hwait_vm<12>();
      else hwait_vm<0>();
      __builtin_amdgcn_s_barrier();
    }
    return;
  }

  // ---------------- consumers: waves 0-3, c = wave --------------------------
  const int c = wave;
  f32x16 acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][n][e] = 0.0f;
  uint32_t a_rd[2][2][2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int row = c * 64 + rb * 32 + (lane & 31);
    const int sw = (row >> 1) & 7;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        a_rd[rb][s][q] = row * 128 + (((4 * s + 2 * (lane >> 5) + q) ^ sw) << 4);
  }
  auto crow = [&](int j) { return 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3); };
  int er[2] = {kSent, kSent};
  float scl[2] = {1.0f, 1.0f}, thr[2] = {0.0f, 0.0f};
  bool flag_tile = false;
  unsigned nflag = 0;
  const int st_lane = (int)(((4 * (lane >> 5) + (lane & 3)) * ldo + (lane & 28)) * 4);
  int kt = 0, i = 0, slot_a = 0, slot_b = 0;
  int cur_mt, cur_ct;
  tile_of(0, cur_mt, cur_ct);
  __builtin_amdgcn_s_barrier();   // the producers' prologue: step 0 landed
  for (int u = 0; u < U; ++u) {
    const uint32_t sa = smem_base + slot_a * P_A_STAGE;
    const uint32_t sb = smem_base + P_NSA * P_A_STAGE + slot_b * P_B_STAGE + lane * 16;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      f16x8 bq[4][2];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        bq[n][0] = hds_read16<f16x8>(sb + ((n * 2 + s) * 2 + 0) * 1024);
        bq[n][1] = hds_read16<f16x8>(sb + ((n * 2 + s) * 2 + 1) * 1024);
      }
      f32x4 x[2][2];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        x[rb][0] = hds_read16<f32x4>(sa + a_rd[rb][s][0]);
        x[rb][1] = hds_read16<f32x4>(sa + a_rd[rb][s][1]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(bq[0][0]), "+v"(bq[0][1]), "+v"(bq[1][0]), "+v"(bq[1][1]),
                     "+v"(bq[2][0]), "+v"(bq[2][1]), "+v"(bq[3][0]), "+v"(bq[3][1]),
                     "+v"(x[0][0]), "+v"(x[0][1]), "+v"(x[1][0]), "+v"(x[1][1]));
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const f32x4 xa = x[rb][0], xb = x[rb][1];
        const float mx = max8abs(xa, xb);
        if (kt == 0 && s == 0) {
          const float mm = fmaxf(mx, __shfl_xor(mx, 32));
          const bool z = !(mm > 0.0f);
          const int e = __builtin_amdgcn_frexp_expf(mm);
          er[rb] = z ? kSent : e;
          scl[rb] = z ? 1.0f : __builtin_amdgcn_ldexpf(1.0f, kTA - e);
          thr[rb] = z ? 0.0f : __builtin_amdgcn_ldexpf(1.0f, e + kHead);
        } else {
          flag_tile = flag_tile || __builtin_amdgcn_ballot_w64(mx > thr[rb]) != 0;
        }
        f16x8 a0, a1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2 v = (q < 2 ? f32x2{xa[2 * q], xa[2 * q + 1]}
                                 : f32x2{xb[2 * q - 4], xb[2 * q - 3]}) * scl[rb];
          f16x2 h0, h1;
          split2h(v, h0, h1);
          a0[2 * q] = h0[0]; a0[2 * q + 1] = h0[1];
          a1[2 * q] = h1[0]; a1[2 * q + 1] = h1[1];
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          acc[rb][n] = mfma_h(a1, bq[n][0], acc[rb][n]);
          acc[rb][n] = mfma_h(a0, bq[n][1], acc[rb][n]);
          acc[rb][n] = mfma_h(a0, bq[n][0], acc[rb][n]);
        }
      }
    }
    slot_a = slot_a + 1 == P_NSA ? 0 : slot_a + 1;
    slot_b = slot_b + 1 == P_NSB ? 0 : slot_b + 1;
    if (kt == KT - 1) {
      // tile end: un-scale and store (wide: 4 x 4 quad transposes, dwordx4)
      int ecol[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) ecol[n] = s_ew[cur_ct * P_BN + n * 32 + (lane & 31)];
      if (cur_mt < m_tiles) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const int64_t r0 = (int64_t)cur_mt * P_BM + c * 64 + rb * 32;
          const bool full = r0 + 32 <= M;
          const char* base = reinterpret_cast<const char*>(out + r0 * ldo + cur_ct * P_BN);
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int erj = __shfl(er[rb], crow(j)) - kTA - kTW;
#pragma unroll
            for (int n = 0; n < 4; ++n)
              acc[rb][n][j] = __builtin_amdgcn_ldexpf(acc[rb][n][j], erj + ecol[n]);
          }
#pragma unroll
          for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              float v[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = acc[rb][n][4 * g + r];
              quad_transpose(v, lane);
              f32x4* o = (f32x4*)(base + (int64_t)(8 * g) * ldo * 4 + n * 128 + st_lane);
              const int64_t row = r0 + 8 * g + 4 * (lane >> 5) + (lane & 3);
              if (full || row < M) __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, o);
            }
        }
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[a][n][e] = 0.0f;
      if (flag_tile) ++nflag;
      flag_tile = false;
      kt = 0;
      ++i;
      if (i < my_tiles) tile_of(i, cur_mt, cur_ct);
    } else {
      ++kt;
    }
    __builtin_amdgcn_s_barrier();
  }
  if (lane == 0 && nflag) atomicAdd(&g_pc_flags, nflag);
}
}  // namespace

int launch_gemm_nt_pc(const float* A, int64_t M, int R, const void* Wf, int C, float* out,
                      hipStream_t st) {
  const f16x8* wf = (const f16x8*)Wf;
  const int* ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(Wf) + (int64_t)C * R * 4);
  const int m_tiles = (int)((M + P_BM - 1) / P_BM);
  const int64_t n_tiles = (int64_t)((m_tiles + 7) / 8) * 8 * (C / P_BN);
  const unsigned grid = (unsigned)std::min<int64_t>(n_tiles, (int64_t)num_cus() / 8 * 8);
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)k_gemm_nt_pc, hipFuncAttributeMaxDynamicSharedMemorySize,
                              P_LDS);
    done = true;
  }
  k_gemm_nt_pc<<<grid, 512, P_LDS, st>>>(A, R, M, R, wf, ew, C, out, C, m_tiles);
  return launch_status("gemm_nt_pc");
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
  const int64_t M = argc > 1 ? atoll(argv[1]) : 196608;
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
  double tot[2] = {0, 0};
  for (const Shape& s : shapes) {
    rb_split_job job{W, s.R, s.C, s.R, 0, Wf};
    CK((hipError_t)launch_split_weights_h(&job, 1, 0));
    std::vector<float> ts[2];
    for (int rep = 0; rep < reps; ++rep) {
      for (int v = 0; v < 2; ++v) {
        CK(hipEventRecord(e0, 0));
        const int rc = v == 0 ? launch_gemm_nt_h(A, s.R, M, s.R, Wf, s.C, nullptr, O0, s.C, 0,
                                                 nullptr, 0)
                              : launch_gemm_nt_pc(A, M, s.R, Wf, s.C, O1, 0);
        if (rc) { fprintf(stderr, "launch failed %d\n", rc); return 1; }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts[v].push_back(ms * 1e3f);
      }
    }
    // sampled check of the P/C output against fp64, and its max difference to prod
    std::vector<float> hw((size_t)s.C * s.R), ha(s.R), h0(s.C), h1(s.C);
    CK(hipMemcpy(hw.data(), W, hw.size() * 4, hipMemcpyDeviceToHost));
    double worst = 0, dprod = 0;
    for (int64_t r = 0; r < M; r += (r < 300 || r > M - 300) ? 1 : 997) {
      CK(hipMemcpy(ha.data(), A + r * s.R, s.R * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h0.data(), O0 + r * s.C, s.C * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h1.data(), O1 + r * s.C, s.C * 4, hipMemcpyDeviceToHost));
      for (int c = 0; c < s.C; ++c) {
        double ref = 0, mag = 0;
        for (int k = 0; k < s.R; ++k) {
          ref += (double)ha[k] * hw[(size_t)c * s.R + k];
          mag += fabs((double)ha[k] * hw[(size_t)c * s.R + k]);
        }
        worst = std::max(worst, fabs(h1[c] - ref) / (mag + 1e-30));
        dprod = std::max(dprod, (double)fabs(h1[c] - h0[c]));
      }
    }
    printf("%-10s R=%3d C=%3d", s.name, s.R, s.C);
    for (int v = 0; v < 2; ++v) {
      std::sort(ts[v].begin(), ts[v].end());
      const double us = ts[v][ts[v].size() / 2];
      tot[v] += us;
      printf("  %s %7.1f", v == 0 ? "prod" : "pc", us);
    }
    printf("  pc err %.2e (vs prod %.2e)%s\n", worst, dprod, worst < 1e-6 ? "" : "  WRONG");
  }
  unsigned fl = 0;
  CK(hipMemcpyFromSymbol(&fl, HIP_SYMBOL(g_pc_flags), 4));
  printf("total  prod %.1f  pc %.1f   (flagged tiles %u)\n", tot[0], tot[1], fl);
  return 0;
}
