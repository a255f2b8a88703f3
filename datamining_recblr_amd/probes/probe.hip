// probe.hip — measurement aids for bench.py, built into their own library
// (lib/libdmrecblr_probe.so, probes/recblr_probe.h), not the product's: the
// gate-scan backward's memory access pattern with trivial arithmetic, and the
// projection GEMMs' row streams without the product.
//
// k_probe_gate_bwd_pattern reads r, i (rg), xc, z, dy and writes dr, di
// (drg), dxc, dz exactly as k_gate_scan_bwd<float, 4, 8, 2> does — the same
// row strides, wave -> (sequence pair, 32-channel span) mapping (packed
// batches: sequence b and B-1-b on one wave), lane layout (8 time chunks x 8
// channel groups, 16-B accesses), reverse tile order and write guards — but
// computes each output as one product.  Its rate is the ceiling the memory
// system grants that pattern on the box and moment it runs, which bench.py
// reports beside the kernel's own rate (roofline.pattern).
#include "../csrc/common.h"

namespace rb {
namespace {

constexpr int kPQ = 8, kPTC = 2, kPV = 4, kPG = kWave / kPQ;

__global__ void __launch_bounds__(256)
k_probe_gate_bwd_pattern(const float* __restrict__ rg, int rg_rs, const float* __restrict__ xc,
                         int xc_rs, const float* __restrict__ z, int z_rs,
                         const float* __restrict__ dy, float* __restrict__ drg, int drg_rs,
                         float* __restrict__ dxc, int dxc_rs, float* __restrict__ dz, int dz_rs,
                         int64_t B, int Lmax, int H, int ncw, const int64_t* __restrict__ offs,
                         int pair) {
  constexpr int TILE = kPQ * kPTC;
  const int lane = threadIdx.x & (kWave - 1);
  const int q = lane & (kPQ - 1);
  const int g = lane / kPQ;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t bw = wid / ncw;
  if (bw >= (pair ? (B + 1) / 2 : B)) return;
  const int c0 = (int)(wid - bw * ncw) * (kPG * kPV) + g * kPV;
  if (c0 >= H) return;
  const int nseq = (pair && B - 1 - bw != bw) ? 2 : 1;
  for (int sq = 0; sq < nseq; ++sq) {
    const int64_t b = sq == 0 ? bw : B - 1 - bw;
    int64_t row0;
    int L;
    if (offs != nullptr) {
      row0 = offs[b];
      L = (int)(offs[b + 1] - row0);
    } else {
      row0 = b * Lmax;
      L = Lmax;
    }
    const int nT = (L + TILE - 1) / TILE;
    for (int tile = nT - 1; tile >= 0; --tile) {
      const int t0 = tile * TILE + q * kPTC;
      float r[kPTC][kPV], i[kPTC][kPV], x[kPTC][kPV], zz[kPTC][kPV], d[kPTC][kPV];
#pragma unroll
      for (int j = 0; j < kPTC; ++j) {
        const int64_t t = row0 + min(t0 + j, L - 1);
        ldv(r[j], rg + t * rg_rs + c0);
        ldv(i[j], rg + t * rg_rs + H + c0);
        ldv(x[j], xc + t * xc_rs + c0);
        ldv(zz[j], z + t * z_rs + c0);
        ldv(d[j], dy + t * H + c0);
      }
#pragma unroll
      for (int j = 0; j < kPTC; ++j) {
        if (t0 + j >= L) continue;
        const int64_t t = row0 + t0 + j;
        float o1[kPV], o2[kPV], o3[kPV], o4[kPV];
#pragma unroll
        for (int v = 0; v < kPV; ++v) {
          o1[v] = r[j][v] * d[j][v];
          o2[v] = i[j][v] * d[j][v];
          o3[v] = x[j][v] * d[j][v];
          o4[v] = zz[j][v] * d[j][v];
        }
        stv(dz + t * dz_rs + c0, o4);
        stv(drg + t * drg_rs + c0, o1);
        stv(drg + t * drg_rs + H + c0, o2);
        stv(dxc + t * dxc_rs + c0, o3);
      }
    }
  }
}

}  // namespace

int launch_probe_gate_bwd_pattern(const float* rg, int64_t rg_rs, const float* xc, int64_t xc_rs,
                                  const float* z, int64_t z_rs, const float* dy, float* drg,
                                  int64_t drg_rs, float* dxc, int64_t dxc_rs, float* dz,
                                  int64_t dz_rs, int64_t B, int64_t L, int64_t H,
                                  const int64_t* offs, hipStream_t st) {
  const int span = kPG * kPV;
  const int ncw = (int)((H + span - 1) / span);
  const int pair = offs != nullptr;
  const int64_t Bw = pair ? (B + 1) / 2 : B;
  const int64_t blocks = (Bw * ncw + 3) / 4;
  hipLaunchKernelGGL(k_probe_gate_bwd_pattern, dim3((unsigned)blocks), dim3(256), 0, st, rg,
                     (int)rg_rs, xc, (int)xc_rs, z, (int)z_rs, dy, drg, (int)drg_rs, dxc,
                     (int)dxc_rs, dz, (int)dz_rs, B, (int)L, (int)H, ncw, offs, pair);
  return launch_status("rb_probe_gate_bwd_pattern");
}

// k_probe_gemm_pattern: the f16x3 NT GEMM's HBM bytes without the GEMM —
// each row of A [M, R] read once (16-B loads), C outputs of that row written
// (16-B nontemporal stores, the GEMM epilogue's policy); 8 lanes per row, a
// wave 8 rows.  Its time is the streaming floor bench.py sets beside each
// projection GEMM (gemm.pattern; tools/gemm_pattern.hip is the standalone
// sweep).
__global__ void __launch_bounds__(256)
k_probe_gemm_pattern(const float* __restrict__ A, int64_t M, int R, float* __restrict__ out,
                     int C) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wrow = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8;
  if (wrow >= M) return;
  const int64_t row = wrow + (lane >> 3);
  const int64_t r = row < M ? row : M - 1;
  const rb_f32x4* a = reinterpret_cast<const rb_f32x4*>(A + r * R);
  rb_f32x4 s = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int j = lane & 7; j < R / 4; j += 8) s += __builtin_nontemporal_load(a + j);
  float t = s[0] + s[1] + s[2] + s[3];
  t += __shfl_xor(t, 1);
  t += __shfl_xor(t, 2);
  t += __shfl_xor(t, 4);
  if (row >= M) return;
  rb_f32x4* o = reinterpret_cast<rb_f32x4*>(out + row * C);
  for (int j = lane & 7; j < C / 4; j += 8)
    __builtin_nontemporal_store(rb_f32x4{t, t + 1.0f, t + 2.0f, t + 3.0f}, o + j);
}

}  // namespace rb

namespace rb {
int launch_probe_gemm_pattern(const float* A, int64_t M, int64_t R, float* out, int64_t C,
                              hipStream_t st) {
  const int64_t blocks = (M + 31) / 32;
  hipLaunchKernelGGL(k_probe_gemm_pattern, dim3((unsigned)blocks), dim3(256), 0, st, A, M, (int)R,
                     out, (int)C);
  return launch_status("rb_probe_gemm_pattern");
}
}  // namespace rb
