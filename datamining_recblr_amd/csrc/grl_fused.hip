// grl_fused.hip — GatedRecurrentLayer's core as ONE kernel (forward):
//   causal depthwise conv + SiLU  (RecBLR.py:182-193)
//   -> behaviour-gate projection   rg = xc W_g^T (+ b_g)      (RecBLR.py:196)
//   -> alpha / beta gates, BD-LRU scan from the pad-prefix state, silu(z) h
//                                                           (RecBLR.py:197-206)
// on packed sequences, fp32, H = 256 channels (d = 128): x and z are read,
// y (or each sequence's last row) is written; xc, rg (without bias) and the
// scan's 16-step carry checkpoints are optional side outputs for the
// backward.  Compared with the three-launch path (conv, gates GEMM, gate
// scan: 10 [ntok, H] streams) the xc / rg round trips through HBM are gone.
//
// Work division.  A 512-thread workgroup (8 waves, one per CU: 133 KB of
// LDS) owns a list of whole sequences ("pieces" — the host pairs the
// longest with the shortest so every list holds ~ntok / G rows) and walks
// their rows as one virtual row stream in 64-row tiles, carrying the scan
// state across tiles (a sequence start resets it to the pad-prefix state
// h0).  Per tile:
//   A  wave w: rows 8w..8w+7, lane = 4 channels (whole 1 KB rows): conv +
//      SiLU exactly as k_conv_silu_fwd_rows; xc (fp32) to LDS and to HBM;
//      each row scaled by its exact max (a power of two) and split into two
//      fp16 planes (x = 2^-s (x0 + x1), 22 bits), written to LDS as the MFMA
//      A fragments.
//   C  wave w: gate columns r_c and i_c of channels 32w..32w+31 for the 64
//      rows: 2 x 2 blocks of v_mfma_f32_32x32x16_f16, three products per
//      k16 (a0 b0 + a0 b1 + a1 b0, the gemm_half.hip scheme), weight
//      fragments streamed from L2 (the image of rb_gemm_h_split_weights).
//   D  in the MFMA accumulator layout (lane: one channel, 16 rows per
//      block): bias, alpha, beta, b' = beta xc, the scan (each lane chains its
//      eight 4-row groups with its partner lane's), y = silu(z) h.
#include "common.h"

namespace rb {
namespace {

typedef _Float16 f16x8g __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4g __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2g __attribute__((ext_vector_type(2)));
typedef float f32x16g __attribute__((ext_vector_type(16)));
typedef float f32x4g __attribute__((ext_vector_type(4)));
typedef float f32x2g __attribute__((ext_vector_type(2)));

constexpr int GH = 256;                       // channels
constexpr int GT = 64;                        // rows per tile
constexpr int KBG = GH / 16;                  // k16 blocks of the gates GEMM
constexpr int kSWg = 14;                      // operand scale target (max in [2^13, 2^14))
constexpr int XC_PITCH = GH * 4 + 16;         // fp32 xc row in LDS (+16 B: bank spread)
constexpr int FRAG_PITCH = 64 * 16 + 16;      // one (row block, k16) fragment (+16 B)
constexpr int PLANE_BYTES = 2 * KBG * FRAG_PITCH;
constexpr int LDS_XC = 0;
constexpr int LDS_PLANE0 = GT * XC_PITCH;
constexpr int LDS_PLANE1 = LDS_PLANE0 + PLANE_BYTES;
constexpr int LDS_ER = LDS_PLANE1 + PLANE_BYTES;
constexpr int LDS_ROW = LDS_ER + GT * 4;       // per row: global row
constexpr int LDS_POS = LDS_ROW + GT * 4;       //          position in its sequence (-1: none)
constexpr int LDS_SEQ = LDS_POS + GT * 4;       //          packed sequence index
constexpr int LDS_LAST = LDS_SEQ + GT * 4;      //          last row of its sequence
constexpr int LDS_BYTES = LDS_LAST + GT * 4;

typedef int i32x4g __attribute__((ext_vector_type(4)));

// Ablation switches of tools/grlbench.hip (wrong results; never set in the
// library build): 1 weight fragments not loaded, 2 no gates GEMM at all,
// 4 no x / xz row loads, 8 no per-channel z / dy loads and y / dz / drg stores
#ifndef GRL_PROBE
#define GRL_PROBE 0
#endif

__device__ __forceinline__ f32x16g mfma_g(f16x8g a, f16x8g b, f32x16g c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// A lane-dependent value the compiler may not hoist out of the tile loop:
// LDS addresses are built as (this per-lane base) + compile-time offsets, so
// they fold into the ds_read/ds_write immediate instead of 100+ hoisted
// address registers (which spilled).
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

struct GrlFwdArgs {
  const float* xz;            // [ntok, 2H] (x | z), row stride xz_rs
  int64_t xz_rs;
  const float* conv_w;        // [H, KC]
  const float* conv_b;        // [H]
  const f16x8g* wf;           // f16 image of W_g [2H, H] (rb_gemm_h_split_weights)
  const int* ew;              // its 2H column exponents
  const float* gate_b;        // [2H]
  const float* lam;           // [H]
  const float* h0;            // [H]: the pad-prefix state every sequence starts from
  const int* pieces;          // [3B + G + 1]: row start, length, sequence of each piece; span starts
  int B, G;
  int64_t ntok;
  float* y;                   // [ntok, H] (y_rs) or null
  int64_t y_rs;
  float* y_last;              // [B, H] or null: each sequence's last row only
  float* xc_out;              // [ntok, H] or null
  float* rg_out;              // [ntok, 2H] or null (the GEMM without its bias)
  float* carries;             // [B, nTc, H] or null: state entering every 16-step tile
  int nTc;
  float* xc_rmax;             // [ceil(ntok/32)] or null, zeroed by the caller: max |xc| per
                              // 32-row group (the gates weight gradient's operand scale)
  float* tile_carries;        // [G, max_tiles, H] or null: the state entering each of this
  int max_tiles;              // workgroup's 64-row tiles (the fused backward's checkpoints)
};

template <int KC>
__global__ void __launch_bounds__(512, 1) k_grl_fwd(const GrlFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;                 // lane half (C layout: rows 4h..4h+3 of each 8)
  const int g = blockIdx.x;
  const int* p_row = a.pieces;
  const int* p_len = a.pieces + a.B;
  const int* p_seq = a.pieces + 2 * a.B;
  const int* span = a.pieces + 3 * a.B;
  const int pb = span[g], pe = span[g + 1];
  if (pb >= pe) return;                    // workgroup-uniform
  int span_rows = 0;
  for (int p = pb; p < pe; ++p) span_rows += p_len[p];

  const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)smem;
  float* s_xc = reinterpret_cast<float*>(smem + LDS_XC);
  int* s_er = reinterpret_cast<int*>(smem + LDS_ER);
  int* s_row = reinterpret_cast<int*>(smem + LDS_ROW);
  int* s_pos = reinterpret_cast<int*>(smem + LDS_POS);
  int* s_seq = reinterpret_cast<int*>(smem + LDS_SEQ);
  int* s_last = reinterpret_cast<int*>(smem + LDS_LAST);

  // ---- per-lane constants (phase A's conv weights are re-read per tile: L1)
  // Phases C/D: channel c of this wave's 32 (r column c, i column H + c)
  const int c = 32 * wave + (lane & 31);
  const float nsp = -softplus_f(a.lam[c]);
  const float br = a.gate_b[c], bi = a.gate_b[GH + c];
  const int ec_r = a.ew[c], ec_i = a.ew[GH + c];
  const float hz = a.h0 ? a.h0[c] : 0.0f;
  // element offsets are 32-bit (rb_grl_fwd checks ntok * row stride < 2^31)
  const int xzr = (int)a.xz_rs, yr = (int)a.y_rs;
  // the wave's r and i column blocks of the weight image (wave-uniform bases)
  const char* wr = reinterpret_cast<const char*>(a.wf) + (int64_t)wave * KBG * 2048;
  const char* wi = reinterpret_cast<const char*>(a.wf) + (int64_t)(8 + wave) * KBG * 2048;

  float carry = 0.0f;                      // state entering the tile (channel c)
  // virtual-row cursor over the pieces (wave-uniform)
  int cur_p = pb, cur_off = 0;

  for (int v0 = 0; v0 < span_rows; v0 += GT) {
    if (a.tile_carries && h == 0)
      a.tile_carries[((int64_t)g * a.max_tiles + v0 / GT) * GH + c] = carry;
    // ---- row map of the tile: lane r describes virtual row v0 + r
    int rp = cur_p, roff = cur_off + lane;
    while (rp < pe && roff >= p_len[rp]) {
      roff -= p_len[rp];
      ++rp;
    }
    const bool rvalid = rp < pe;
    const int rrow = rvalid ? p_row[rp] + roff : 0;          // global row
    const int rpos = rvalid ? roff : -1;                     // position in its sequence
    const int rseq = rvalid ? p_seq[rp] : 0;
    const bool rlast = rvalid && roff == p_len[rp] - 1;
    {  // advance the cursor past this tile (lane 63's row + 1)
      int np = __builtin_amdgcn_readlane(rp, 63), noff = __builtin_amdgcn_readlane(roff, 63) + 1;
      if (np < pe && noff >= p_len[np]) { ++np; noff = 0; }
      cur_p = np;
      cur_off = noff;
    }

    // per-lane LDS bases of this tile (see opaque())
    // (region offsets inside opaque(): the per-row constants fold into the
    // 16-bit ds_* immediates)
    char* const ab_xc = smem + opaque(LDS_XC + 16 * lane);
    char* const ab_fr = smem + opaque(LDS_PLANE0 + (lane >> 2) * FRAG_PITCH +
                                      32 * ((lane >> 1) & 1) * 16 + 8 * (lane & 1));
    char* const db = smem + opaque(LDS_ER + 16 * h);               // per-row int arrays
    char* const xb = smem + opaque(LDS_XC + 4 * h * XC_PITCH + 4 * c);   // s_xc[4h][c]
    char* const gb = smem + opaque(LDS_PLANE0 + lane * 16);         // GEMM A fragments
    // ---- phase A: conv + SiLU, LDS images (channels 4*lane .. 4*lane+3)
    float cw[KC][4], cb[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
#pragma unroll
      for (int k = 0; k < KC; ++k) cw[k][v] = a.conv_w[(4 * lane + v) * KC + k];
      cb[v] = a.conv_b[4 * lane + v];
    }
#pragma unroll 2
    for (int j = 0; j < 8; ++j) {
      const int vr = 8 * wave + j;
      const int grow = __builtin_amdgcn_readlane(rrow, vr);
      const int pos = __builtin_amdgcn_readlane(rpos, vr);   // -1: past the span
      f32x4g xcv = {0.0f, 0.0f, 0.0f, 0.0f};
      if (pos >= 0) {
        f32x4g xs[KC];
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          if (KC - 1 - k <= pos && !(GRL_PROBE & 4))
            xs[k] = *reinterpret_cast<const f32x4g*>(a.xz + (uint32_t)((grow - (KC - 1 - k)) * xzr + 4 * lane));
          else
            xs[k] = f32x4g{0.0f, 0.0f, 0.0f, 0.0f};
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          float acc = cb[v];
#pragma unroll
          for (int k = 0; k < KC; ++k)   // lag KC-1-k: rows before the sequence start are zero
            acc = acc + (KC - 1 - k <= pos ? cw[k][v] * xs[k][v] : 0.0f);
          xcv[v] = fsilu(acc);
        }
        if (a.xc_out) __builtin_nontemporal_store(xcv, reinterpret_cast<f32x4g*>(a.xc_out + (uint32_t)(grow * GH + 4 * lane)));
      }
      *reinterpret_cast<f32x4g*>(ab_xc + vr * XC_PITCH) = xcv;
      const float m = wave_max(fmaxf(fmaxf(fabsf(xcv[0]), fabsf(xcv[1])), fmaxf(fabsf(xcv[2]), fabsf(xcv[3]))));
      const int e = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
      if (lane == 0) {
        if (a.xc_rmax && pos >= 0)   // non-negative floats order as their bit patterns
          atomicMax(reinterpret_cast<int*>(a.xc_rmax) + (grow >> 5), __float_as_int(m));
        s_er[vr] = e;
        s_row[vr] = grow;
        s_pos[vr] = pos;
        s_seq[vr] = __builtin_amdgcn_readlane(rseq, vr);
        s_last[vr] = __builtin_amdgcn_readlane((int)rlast, vr);
      }
      const float sc = __builtin_amdgcn_ldexpf(1.0f, kSWg - e);
      f16x4g h0v, h1v;
#pragma unroll
      for (int v = 0; v < 4; v += 2) {
        const f32x2g xv = f32x2g{xcv[v], xcv[v + 1]} * sc;
        const f16x2g p0 = __builtin_convertvector(xv, f16x2g);
        const f16x2g p1 = __builtin_convertvector(xv - __builtin_convertvector(p0, f32x2g), f16x2g);
        h0v[v] = p0[0]; h0v[v + 1] = p0[1];
        h1v[v] = p1[0]; h1v[v + 1] = p1[1];
      }
      // A fragment (row block vr / 32, k16 block lane / 4): fragment lane
      // (vr % 32) + 32 * ((lane >> 1) & 1), halfs 4 * (lane & 1) .. + 3
      const int fo = (vr >> 5) * KBG * FRAG_PITCH + (vr & 31) * 16;
      *reinterpret_cast<f16x4g*>(ab_fr + fo) = h0v;
      *reinterpret_cast<f16x4g*>(ab_fr + PLANE_BYTES + fo) = h1v;
    }
    __syncthreads();

    // ---- phase C: r / i columns of channels 32w.. for the 64 rows
    f32x16g ar[2], ai[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int e = 0; e < 16; ++e) { ar[rb][e] = 0.0f; ai[rb][e] = 0.0f; }
    // weight fragments: a wave-uniform base (kb advances it) + the lane's 16 B
    const int wl = opaque(lane * 16);
    auto wfrag = [&](const char* base, int kb, int p) {
#if GRL_PROBE & 1
      return f16x8g{} + (_Float16)(kb + p);
#else
      return *reinterpret_cast<const f16x8g*>(base + kb * 2048 + p * 1024 + wl);
#endif
    };
    f16x8g br0 = wfrag(wr, 0, 0), br1 = wfrag(wr, 0, 1), bi0 = wfrag(wi, 0, 0), bi1 = wfrag(wi, 0, 1);
#pragma unroll 1
    for (int kb = 0; kb < ((GRL_PROBE & 2) ? 0 : KBG); ++kb) {
      f16x8g nr0, nr1, ni0, ni1;
      if (kb + 1 < KBG) {
        nr0 = wfrag(wr, kb + 1, 0); nr1 = wfrag(wr, kb + 1, 1);
        ni0 = wfrag(wi, kb + 1, 0); ni1 = wfrag(wi, kb + 1, 1);
      }
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int fo = (rb * KBG + kb) * FRAG_PITCH;
        const f16x8g a0 = *reinterpret_cast<const f16x8g*>(gb + fo);
        const f16x8g a1 = *reinterpret_cast<const f16x8g*>(gb + PLANE_BYTES + fo);
        ar[rb] = mfma_g(a1, br0, ar[rb]);
        ar[rb] = mfma_g(a0, br1, ar[rb]);
        ar[rb] = mfma_g(a0, br0, ar[rb]);
        ai[rb] = mfma_g(a1, bi0, ai[rb]);
        ai[rb] = mfma_g(a0, bi1, ai[rb]);
        ai[rb] = mfma_g(a0, bi0, ai[rb]);
      }
      if (kb + 1 < KBG) { br0 = nr0; br1 = nr1; bi0 = ni0; bi1 = ni1; }
    }

#define DROW(rc) (*reinterpret_cast<const int*>(db + (LDS_ROW - LDS_ER) + 4 * (rc)))
#define DPOS(rc) (*reinterpret_cast<const int*>(db + (LDS_POS - LDS_ER) + 4 * (rc)))
#define DSEQ(rc) (*reinterpret_cast<const int*>(db + (LDS_SEQ - LDS_ER) + 4 * (rc)))
#define DLAST(rc) (*reinterpret_cast<const int*>(db + (LDS_LAST - LDS_ER) + 4 * (rc)))
#define DER(rc) (*reinterpret_cast<const int*>(db + 4 * (rc)))
    // ---- phase D: gates, scan, merge (lane: channel c, rows of its C layout),
    // one 32-row block at a time; alpha -> ar, b' -> ai in place
    float run = carry;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      float zr[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);   // row = rc + 4h
        zr[e] = DPOS(rc) >= 0 && !(GRL_PROBE & 8) ? a.xz[(uint32_t)(DROW(rc) * xzr + GH + c)] : 0.0f;
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);   // row = rc + 4h
        const int er = DER(rc);
        const float r = __builtin_amdgcn_ldexpf(ar[rb][e], er + ec_r - 2 * kSWg);
        const float i = __builtin_amdgcn_ldexpf(ai[rb][e], er + ec_i - 2 * kSWg);
        const int pos = DPOS(rc);
        if (a.rg_out && pos >= 0) {
          float* o = a.rg_out + (uint32_t)(DROW(rc) * (2 * GH) + c);
          o[0] = r;
          o[GH] = i;
        }
        const float xcv = *reinterpret_cast<const float*>(xb + rc * XC_PITCH);
        const float al = fexp(nsp * fsigm(r + br));
        const float be = fsqrt(1.0f - al * al + 1e-8f) * fsigm(i + bi);
        ar[rb][e] = pos >= 0 ? al : 1.0f;
        ai[rb][e] = pos >= 0 ? be * xcv : 0.0f;
      }
      // aggregates (A, X) of this lane's 4 groups of 4 rows; a sequence start
      // replaces the incoming state by h0
      float cin[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float A = 1.0f, X = 0.0f;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = 4 * q + u;
          const int rc = 32 * rb + 8 * q + u;
          const float al = ar[rb][e], bp = ai[rb][e];
          if (DPOS(rc) == 0) {
            X = al * hz + bp;
            A = 0.0f;
          } else {
            X = X * al + bp;
            A = A * al;
          }
        }
        // the block's 8 groups in row order: (q, half 0), (q, half 1)
        const float pA = __shfl_xor(A, 32), pX = __shfl_xor(X, 32);
        const float A0 = h == 0 ? A : pA, X0 = h == 0 ? X : pX;
        const float A1 = h == 0 ? pA : A, X1 = h == 0 ? pX : X;
        const float c0 = run;
        run = A0 * run + X0;
        const float c1 = run;
        run = A1 * run + X1;
        cin[q] = h == 0 ? c0 : c1;
      }
      // rows: state, output, checkpoints
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float hp = cin[q];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = 4 * q + u;
          const int rc = 32 * rb + 8 * q + u;
          const int pos = DPOS(rc);
          if (pos == 0) hp = hz;
          if (a.carries && pos >= 0 && (pos & 15) == 0)
            a.carries[(uint32_t)((DSEQ(rc) * a.nTc + (pos >> 4)) * GH + c)] = hp;
          const float hn = hp * ar[rb][e] + ai[rb][e];
          hp = hn;
          const float yv = fsilu(zr[e]) * hn;
          if (pos >= 0 && !(GRL_PROBE & 8)) {
            if (a.y) a.y[(uint32_t)(DROW(rc) * yr + c)] = yv;
            else if (a.y_last && DLAST(rc)) a.y_last[(uint32_t)(DSEQ(rc) * GH + c)] = yv;
          }
        }
      }
    }
    carry = run;
#undef DROW
#undef DPOS
#undef DSEQ
#undef DLAST
#undef DER
    __syncthreads();   // LDS is rewritten by the next tile
  }
}

// ---------------------------------------------------------------------------
// Backward of k_grl_fwd, one launch per layer (RecBLR.py:182-206 reversed):
// the same work lists, each workgroup walking its virtual rows in REVERSE
// 64-row tiles, the adjoint state carried across tiles.  Per tile:
//   A  row-wide: conv pre-activations recomputed from x (-> LDS R0, fp32),
//      xc = silu(pre) to HBM (the gates weight gradient's operand) and as
//      the f16 A planes of GEMM 1 (-> LDS R1)
//   C  GEMM 1: r / i of channels 32w.. (as the forward)
//   D  C layout: gates; the forward scan from the tile's checkpoint (the
//      forward's tile_carries) gives h_{t-1} (-> LDS R1, the planes are
//      spent) and dz; the reverse adjoint scan (e_t = a_t (gy_t + e_{t+1}),
//      reset at each sequence's last row) gives d = dL/dh, then dr, di (to
//      HBM), dxc's direct term, the partial sums of dLambda, d gate_b, dh0
//   E  each row of drg scaled by its exact max over all 512 columns (a
//      reduce-scatter inside the wave, then across waves in LDS)
//   F  GEMM 2: dxc_g = drg W_g for channels 32w.. (W_g^T's image), in two
//      K halves: dr's fp16 planes (row-major, LDS R0), then di's
//   G  dpre = dxc_direct silu'(pre) (LDS R1, written in D) + dxc_g silu'(pre)
//      (-> LDS R0)
//   H  row-wide: the conv backward, dx (dpre of the next 3 rows: this tile
//      or the later tile's first rows, kept in LDS), dW / dbias partials
constexpr int DRG_PITCH = GH * 2 + 16;         // a row-major fp16 plane row of one drg half (dr or di)
constexpr int B_R0_BYTES = 2 * GT * DRG_PITCH > GT * XC_PITCH ? 2 * GT * DRG_PITCH : GT * XC_PITCH;
constexpr int B_R0 = 0;                        // pre / the drg half's planes / dpre
constexpr int B_R1 = B_R0_BYTES;               // xc planes / h_{t-1} / dpre's direct term
constexpr int B_HALO = B_R1 + GT * XC_PITCH;   // 3 rows of dpre (the later tile's first rows)
constexpr int B_ER = B_HALO + 3 * XC_PITCH;    // xc row exponents
constexpr int B_ER2 = B_ER + GT * 4;           // drg row exponents
constexpr int B_RMX = B_ER2 + GT * 4;          // drg row maxima
constexpr int B_ROW = B_RMX + GT * 4;
constexpr int B_POS = B_ROW + GT * 4;
constexpr int B_SEQ = B_POS + GT * 4;
constexpr int B_LAST = B_SEQ + GT * 4;         // rows left to the sequence's end (0: last)
constexpr int B_PMAX = B_LAST + GT * 4;        // [8 waves][64 rows] partial drg row maxima
constexpr int B_LDS_BYTES = B_PMAX + 8 * GT * 4;

struct GrlBwdArgs {
  const float* xz;
  int64_t xz_rs;
  const float* conv_w;
  const float* conv_b;
  const f16x8g* wf;           // W_g [2H, H] image (rg = xc W_g^T)
  const int* ew;
  const f16x8g* wft;          // W_g^T [H, 2H] image (dxc_g = drg W_g)
  const int* ewt;
  const float* gate_b;
  const float* lam;
  const float* h0;            // [H] or null
  const int* pieces;
  int B, G;
  int64_t ntok;
  const float* tile_carries;  // [G, max_tiles, H] (k_grl_fwd)
  int max_tiles;
  const float* dy;            // [ntok, H] or null
  const float* dy_last;       // [B, H] or null: dy only at each sequence's last row
  float* dxz;                 // [ntok, 2H]: dx | dz
  int64_t dxz_rs;
  float* drg;                 // [ntok, 2H]
  float* xc_out;              // [ntok, H]
  float* drg_rmax;            // [ceil(ntok/32)], zeroed
  float* xc_rmax;             // [ceil(ntok/32)], zeroed
  float* part;                // [G, 4, H]: dLambda, d gate_b (r, i), dh0
  float* cpart;               // [G * 8, H * KC + H]: d conv_w (weight order), d conv_b
};

template <int KC, bool LASTDY>
__global__ void __launch_bounds__(512, 1) k_grl_bwd(const GrlBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  const int g = blockIdx.x;
  const int* p_row = a.pieces;
  const int* p_len = a.pieces + a.B;
  const int* p_seq = a.pieces + 2 * a.B;
  const int* span = a.pieces + 3 * a.B;
  const int pb = span[g], pe = span[g + 1];
  float* cp = a.cpart + ((int64_t)g * 8 + wave) * (GH * KC + GH);
  if (pb >= pe) {   // empty span: its partial rows are zeros
    for (int i = lane; i < GH * KC + GH; i += 64) cp[i] = 0.0f;
    if (wave == 0)
      for (int i = lane; i < 4 * GH; i += 64) a.part[(int64_t)g * 4 * GH + i] = 0.0f;
    return;
  }
  int span_rows = 0;
  for (int p = pb; p < pe; ++p) span_rows += p_len[p];
  const int n_tiles = (span_rows + GT - 1) / GT;

  const int c = 32 * wave + (lane & 31);
  const float lamc = a.lam[c];
  const float nsp = -softplus_f(lamc);
  const float br = a.gate_b[c], bi = a.gate_b[GH + c];
  const int ec_r = a.ew[c], ec_i = a.ew[GH + c], ec_t = a.ewt[c];
  const float hz = a.h0 ? a.h0[c] : 0.0f;
  // element offsets are 32-bit (rb_grl_bwd checks ntok * row stride < 2^31)
  const int xzr = (int)a.xz_rs, dxr = (int)a.dxz_rs;
  const char* wr = reinterpret_cast<const char*>(a.wf) + (int64_t)wave * KBG * 2048;
  const char* wi = reinterpret_cast<const char*>(a.wf) + (int64_t)(8 + wave) * KBG * 2048;
  const char* wt = reinterpret_cast<const char*>(a.wft) + (int64_t)wave * (2 * KBG) * 2048;

  float acc_v = 0.0f, acc_r = 0.0f, acc_i = 0.0f, acc_h = 0.0f;   // channel c
  float cw_acc[KC][4], cb_acc[4];                                  // channels 4*lane..
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    cb_acc[v] = 0.0f;
#pragma unroll
    for (int k = 0; k < KC; ++k) cw_acc[k][v] = 0.0f;
  }
  float eadj = 0.0f;                       // adjoint entering the tile from later rows

  // cursor at the last tile's first virtual row
  int cur_p = pb, cur_off = (n_tiles - 1) * GT;
  while (cur_off >= p_len[cur_p]) { cur_off -= p_len[cur_p]; ++cur_p; }

  for (int t = n_tiles - 1; t >= 0; --t) {
    if (t != n_tiles - 1) {   // move the cursor back by one tile
      cur_off -= GT;
      while (cur_off < 0) { --cur_p; cur_off += p_len[cur_p]; }
    }
    int rp = cur_p, roff = cur_off + lane;
    while (rp < pe && roff >= p_len[rp]) { roff -= p_len[rp]; ++rp; }
    const bool rvalid = rp < pe;
    const int rrow = rvalid ? p_row[rp] + roff : 0;
    const int rpos = rvalid ? roff : -1;
    const int rseq = rvalid ? p_seq[rp] : 0;
    const int rrem = rvalid ? p_len[rp] - 1 - roff : -1;     // rows to the sequence's end

    // per-lane LDS bases; every region's offset is inside opaque() so the
    // per-row constants stay below 64 KiB and fold into ds_* immediates
    char* const ab_pre = smem + opaque(B_R0 + 16 * lane);
    char* const ab_fr = smem + opaque(B_R1 + (lane >> 2) * FRAG_PITCH + 32 * ((lane >> 1) & 1) * 16 +
                                      8 * (lane & 1));
    char* const db = smem + opaque(B_ER + 16 * h);                 // per-row int arrays
    char* const r0c = smem + opaque(B_R0 + 4 * h * XC_PITCH + 4 * c);   // R0 [4h][c]
    char* const r1c = smem + opaque(B_R1 + 4 * h * XC_PITCH + 4 * c);   // R1 [4h][c]
    char* const gb = smem + opaque(B_R1 + lane * 16);
    // GEMM 2's A fragment of lane l: row l % 32, halfs 8 (l / 32) .. + 7 of a k16 block
    char* const g2 = smem + B_R0 + opaque((lane & 31) * DRG_PITCH + 16 * (lane >> 5));

    // ---- A: pre-activations, xc, its f16 planes
    {
      float cw[KC][4], cbv[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
#pragma unroll
        for (int k = 0; k < KC; ++k) cw[k][v] = a.conv_w[(4 * lane + v) * KC + k];
        cbv[v] = a.conv_b[4 * lane + v];
      }
#pragma unroll 2
      for (int j = 0; j < 8; ++j) {
        const int vr = 8 * wave + j;
        const int grow = __builtin_amdgcn_readlane(rrow, vr);
        const int pos = __builtin_amdgcn_readlane(rpos, vr);
        f32x4g pre = {0.0f, 0.0f, 0.0f, 0.0f}, xcv = {0.0f, 0.0f, 0.0f, 0.0f};
        if (pos >= 0) {
          f32x4g xs[KC];
#pragma unroll
          for (int k = 0; k < KC; ++k)
            xs[k] = KC - 1 - k <= pos && !(GRL_PROBE & 4)
                        ? *reinterpret_cast<const f32x4g*>(a.xz + (uint32_t)((grow - (KC - 1 - k)) * xzr + 4 * lane))
                        : f32x4g{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            float acc = cbv[v];
#pragma unroll
            for (int k = 0; k < KC; ++k)
              acc = acc + (KC - 1 - k <= pos ? cw[k][v] * xs[k][v] : 0.0f);
            pre[v] = acc;
            xcv[v] = fsilu(acc);
          }
          __builtin_nontemporal_store(xcv, reinterpret_cast<f32x4g*>(a.xc_out + (uint32_t)(grow * GH + 4 * lane)));
        }
        *reinterpret_cast<f32x4g*>(ab_pre + vr * XC_PITCH) = pre;
        const float m = wave_max(fmaxf(fmaxf(fabsf(xcv[0]), fabsf(xcv[1])), fmaxf(fabsf(xcv[2]), fabsf(xcv[3]))));
        const int e = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
        if (lane == 0) {
          if (a.xc_rmax && pos >= 0)
            atomicMax(reinterpret_cast<int*>(a.xc_rmax) + (grow >> 5), __float_as_int(m));
          *reinterpret_cast<int*>(smem + B_ER + 4 * vr) = e;
          *reinterpret_cast<int*>(smem + B_ROW + 4 * vr) = grow;
          *reinterpret_cast<int*>(smem + B_POS + 4 * vr) = pos;
          *reinterpret_cast<int*>(smem + B_SEQ + 4 * vr) = __builtin_amdgcn_readlane(rseq, vr);
          *reinterpret_cast<int*>(smem + B_LAST + 4 * vr) = __builtin_amdgcn_readlane(rrem, vr);
        }
        const float sc = __builtin_amdgcn_ldexpf(1.0f, kSWg - e);
        f16x4g h0v, h1v;
#pragma unroll
        for (int v = 0; v < 4; v += 2) {
          const f32x2g xv = f32x2g{xcv[v], xcv[v + 1]} * sc;
          const f16x2g p0 = __builtin_convertvector(xv, f16x2g);
          const f16x2g p1 = __builtin_convertvector(xv - __builtin_convertvector(p0, f32x2g), f16x2g);
          h0v[v] = p0[0]; h0v[v + 1] = p0[1];
          h1v[v] = p1[0]; h1v[v + 1] = p1[1];
        }
        const int fo = (vr >> 5) * KBG * FRAG_PITCH + (vr & 31) * 16;
        *reinterpret_cast<f16x4g*>(ab_fr + fo) = h0v;
        *reinterpret_cast<f16x4g*>(ab_fr + PLANE_BYTES + fo) = h1v;
      }
    }
    __syncthreads();

    // ---- C: GEMM 1 (r, i)
    f32x16g ar[2], ai[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int e = 0; e < 16; ++e) { ar[rb][e] = 0.0f; ai[rb][e] = 0.0f; }
    {
      const int wl = opaque(lane * 16);
      auto wfrag = [&](const char* base, int kb, int p) {
#if GRL_PROBE & 1
        return f16x8g{} + (_Float16)(kb + p);
#else
        return *reinterpret_cast<const f16x8g*>(base + kb * 2048 + p * 1024 + wl);
#endif
      };
      f16x8g br0 = wfrag(wr, 0, 0), br1 = wfrag(wr, 0, 1), bi0 = wfrag(wi, 0, 0), bi1 = wfrag(wi, 0, 1);
#pragma unroll 1
      for (int kb = 0; kb < ((GRL_PROBE & 2) ? 0 : KBG); ++kb) {
        f16x8g nr0, nr1, ni0, ni1;
        if (kb + 1 < KBG) {
          nr0 = wfrag(wr, kb + 1, 0); nr1 = wfrag(wr, kb + 1, 1);
          ni0 = wfrag(wi, kb + 1, 0); ni1 = wfrag(wi, kb + 1, 1);
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const int fo = (rb * KBG + kb) * FRAG_PITCH;
          const f16x8g a0 = *reinterpret_cast<const f16x8g*>(gb + fo);
          const f16x8g a1 = *reinterpret_cast<const f16x8g*>(gb + PLANE_BYTES + fo);
          ar[rb] = mfma_g(a1, br0, ar[rb]);
          ar[rb] = mfma_g(a0, br1, ar[rb]);
          ar[rb] = mfma_g(a0, br0, ar[rb]);
          ai[rb] = mfma_g(a1, bi0, ai[rb]);
          ai[rb] = mfma_g(a0, bi1, ai[rb]);
          ai[rb] = mfma_g(a0, bi0, ai[rb]);
        }
        if (kb + 1 < KBG) { br0 = nr0; br1 = nr1; bi0 = ni0; bi1 = ni1; }
      }
    }
    __syncthreads();   // R1's planes are spent: h_{t-1} goes there

#define BPOS(rc) (*reinterpret_cast<const int*>(db + (B_POS - B_ER) + 4 * (rc)))
#define BROW(rc) (*reinterpret_cast<const int*>(db + (B_ROW - B_ER) + 4 * (rc)))
#define BSEQ(rc) (*reinterpret_cast<const int*>(db + (B_SEQ - B_ER) + 4 * (rc)))
#define BREM(rc) (*reinterpret_cast<const int*>(db + (B_LAST - B_ER) + 4 * (rc)))
#define BER(rc) (*reinterpret_cast<const int*>(db + 4 * (rc)))
#define BER2(rc) (*reinterpret_cast<const int*>(db + (B_ER2 - B_ER) + 4 * (rc)))
#define PRE(rc) (*reinterpret_cast<const float*>(r0c + (rc) * XC_PITCH))
#define HPV(rc) (*reinterpret_cast<float*>(r1c + (rc) * XC_PITCH))
    // ---- D (forward part): gates (ar <- sigmoid(r), ai <- sigmoid(i); alpha,
    // beta, b' recomputed from them where needed), the forward scan from the
    // tile's checkpoint: the state entering each 4-row group (cin), dz, and
    // gy = dy silu(z) -> LDS R1
    float cin[2][4];
    {
      float run = a.tile_carries[((int64_t)g * a.max_tiles + t) * GH + c];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        float bp[16], al[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);
          const int er = BER(rc);
          const float r = __builtin_amdgcn_ldexpf(ar[rb][e], er + ec_r - 2 * kSWg) + br;
          const float i = __builtin_amdgcn_ldexpf(ai[rb][e], er + ec_i - 2 * kSWg) + bi;
          const bool ok = BPOS(rc) >= 0;
          const float sr = fsigm(r);
          const float aa = ok ? fexp(nsp * sr) : 1.0f;
          const float si = fsigm(i);
          const float sq = fsqrt(1.0f - aa * aa + 1e-8f);
          bp[e] = ok ? sq * si * fsilu(PRE(rc)) : 0.0f;
          ar[rb][e] = sr;
          ai[rb][e] = si;
          al[e] = aa;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float A = 1.0f, X = 0.0f;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int e = 4 * q + u;
            if (BPOS(32 * rb + 8 * q + u) == 0) {
              X = al[e] * hz + bp[e];
              A = 0.0f;
            } else {
              X = X * al[e] + bp[e];
              A = A * al[e];
            }
          }
          const float pA = __shfl_xor(A, 32), pX = __shfl_xor(X, 32);
          const float A0 = h == 0 ? A : pA, X0 = h == 0 ? X : pX;
          const float A1 = h == 0 ? pA : A, X1 = h == 0 ? pX : X;
          const float c0 = run;
          run = A0 * run + X0;
          const float c1 = run;
          run = A1 * run + X1;
          cin[rb][q] = h == 0 ? c0 : c1;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float hp = cin[rb][q];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int e = 4 * q + u;
            const int rc = 32 * rb + 8 * q + u;
            const int pos = BPOS(rc);
            if (pos == 0) hp = hz;
            const float hn = hp * al[e] + bp[e];
            hp = hn;
            float gsv = 0.0f;
            if (pos >= 0 && !(GRL_PROBE & 8)) {
              const int grow = BROW(rc);
              const float zz = a.xz[(uint32_t)(grow * xzr + GH + c)];
              const float gv = !LASTDY ? a.dy[(uint32_t)(grow * GH + c)]
                                       : (BREM(rc) == 0 ? a.dy_last[(uint32_t)(BSEQ(rc) * GH + c)] : 0.0f);
              const float sz = fsigm(zz);
              a.dxz[(uint32_t)(grow * dxr + GH + c)] = (gv * hn) * (sz * (1.0f + zz * (1.0f - sz)));
              gsv = gv * (zz * sz);
            }
            HPV(rc) = gsv;
          }
        }
      }
    }

    // ---- D (reverse part): adjoint, gate gradients; dr, di -> ar, ai;
    // silu'(pre) stays in dsl, dxc_direct silu'(pre) goes to R1 (over gy)
    float dsl[2][16];
    {
      float run = eadj;
#pragma unroll
      for (int rbr = 0; rbr < 2; ++rbr) {
        const int rb = 1 - rbr;
        // groups of this block in reverse row order: (q, half 1), (q, half 0), q = 3..0
        float ein[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int q = 3 - qq;
          float A = 1.0f, X = 0.0f;
#pragma unroll
          for (int uu = 0; uu < 4; ++uu) {
            const int u = 3 - uu;
            const int e = 4 * q + u;
            const int rc = 32 * rb + 8 * q + u;
            const float aa = BPOS(rc) >= 0 ? fexp(nsp * ar[rb][e]) : 1.0f;
            const float gsv = HPV(rc);
            if (BREM(rc) == 0) {   // a sequence's last row: nothing enters it
              X = aa * gsv;
              A = 0.0f;
            } else {
              X = aa * (gsv + X);
              A = aa * A;
            }
          }
          const float pA = __shfl_xor(A, 32), pX = __shfl_xor(X, 32);
          const float A1 = h == 1 ? A : pA, X1 = h == 1 ? X : pX;   // half 1 comes first
          const float A0 = h == 1 ? pA : A, X0 = h == 1 ? pX : X;
          const float c1 = run;
          run = A1 * run + X1;
          const float c0 = run;
          run = A0 * run + X0;
          ein[q] = h == 1 ? c1 : c0;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // the group's 4 rows: gate values and the forward state again
          float ga[4], gq[4], gx[4], hpv[4];
          {
            float hp = cin[rb][q];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int e = 4 * q + u;
              const int rc = 32 * rb + 8 * q + u;
              const int pos = BPOS(rc);
              const bool ok = pos >= 0;
              const float aa = ok ? fexp(nsp * ar[rb][e]) : 1.0f;
              const float sq = fsqrt(1.0f - aa * aa + 1e-8f);
              const float xcv = fsilu(PRE(rc));
              if (pos == 0) hp = hz;
              hpv[u] = hp;
              hp = hp * aa + (ok ? sq * ai[rb][e] * xcv : 0.0f);
              ga[u] = aa;
              gq[u] = sq;
              gx[u] = xcv;
            }
          }
          float E = ein[q];
#pragma unroll
          for (int uu = 0; uu < 4; ++uu) {
            const int u = 3 - uu;
            const int e = 4 * q + u;
            const int rc = 32 * rb + 8 * q + u;
            const int pos = BPOS(rc);
            const bool ok = pos >= 0;
            const float sr = ar[rb][e], si = ai[rb][e];
            const float aa = ga[u], sq = gq[u];
            const float d = (BREM(rc) == 0 ? 0.0f : E) + HPV(rc);
            const float dbeta = d * gx[u];
            const float du = (dbeta * si) * (0.5f * frcp(sq));
            const float da = hpv[u] * d + (-du) * (2.0f * aa);
            const float dv = da * aa;
            const float dr = ok ? (dv * nsp) * ((1.0f - sr) * sr) : 0.0f;
            const float di = ok ? (dbeta * sq) * ((1.0f - si) * si) : 0.0f;
            const float sl = fdsilu(PRE(rc));
            dsl[rb][e] = sl;
            HPV(rc) = ok ? (d * (sq * si)) * sl : 0.0f;
            if (ok) {
              acc_v += dv * sr;
              acc_r += dr;
              acc_i += di;
            }
            if (ok && !(GRL_PROBE & 8)) {
              const int grow = BROW(rc);
              a.drg[(uint32_t)(grow * (2 * GH) + c)] = dr;
              a.drg[(uint32_t)(grow * (2 * GH) + GH + c)] = di;
            }
            E = d * aa;
            if (pos == 0) acc_h += E;
            ar[rb][e] = dr;
            ai[rb][e] = di;
          }
        }
      }
      eadj = run;
    }

    // ---- E: drg row maxima (reduce-scatter over the 32 lanes of a half:
    // slot s = (rb, e) ends on lane (s & 31) of each half), across waves in LDS
    {
      float v[32];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int e = 0; e < 16; ++e) v[16 * rb + e] = fmaxf(fabsf(ar[rb][e]), fabsf(ai[rb][e]));
#pragma unroll
      for (int m = 16, n = 32; m >= 1; m >>= 1, n >>= 1) {
        const bool up = (lane & m) != 0;
#pragma unroll
        for (int j = 0; j < n / 2; ++j) {
          const float send = up ? v[j] : v[j + n / 2];
          const float keep = up ? v[j + n / 2] : v[j];
          v[j] = fmaxf(keep, __shfl_xor(send, m));
        }
      }
      // lane l of half h now holds slot s = l & 31: rb = s >> 4, e = s & 15
      const int s = lane & 31;
      const int row = 32 * (s >> 4) + 8 * ((s & 15) >> 2) + 4 * h + (s & 3);
      *reinterpret_cast<float*>(smem + B_PMAX + 4 * (wave * GT + row)) = v[0];
    }
    __syncthreads();   // every wave is past its reads of R0 (pre)
    if (wave == 0) {
      float m = 0.0f;
#pragma unroll
      for (int w = 0; w < 8; ++w) m = fmaxf(m, *reinterpret_cast<const float*>(smem + B_PMAX + 4 * (w * GT + lane)));
      *reinterpret_cast<int*>(smem + B_ER2 + 4 * lane) = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
      const int pos = *reinterpret_cast<const int*>(smem + B_POS + 4 * lane);
      if (a.drg_rmax && pos >= 0)
        atomicMax(reinterpret_cast<int*>(a.drg_rmax) + (*reinterpret_cast<const int*>(smem + B_ROW + 4 * lane) >> 5),
                  __float_as_int(m));
    }
    __syncthreads();

    // ---- F: GEMM 2, dxc_g for channels 32w.. (K = 512 in two halves)
    f32x16g ax[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int e = 0; e < 16; ++e) ax[rb][e] = 0.0f;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      // this half's values (dr, then di) -> row-major fp16 planes in R0
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);
          const float sc = __builtin_amdgcn_ldexpf(1.0f, kSWg - BER2(rc));
          const float xv = (half == 0 ? ar[rb][e] : ai[rb][e]) * sc;
          const _Float16 v0 = (_Float16)xv;
          const _Float16 v1 = (_Float16)(xv - (float)v0);
          char* rowp = smem + B_R0 + opaque((rc + 4 * h) * DRG_PITCH + 2 * c);
          *reinterpret_cast<_Float16*>(rowp) = v0;
          *reinterpret_cast<_Float16*>(rowp + GT * DRG_PITCH) = v1;
        }
      __syncthreads();
      {
        const int wl = opaque(lane * 16);
        const char* wth = wt + half * KBG * 2048;
        auto tfrag = [&](int kb, int p) {
#if GRL_PROBE & 1
          return f16x8g{} + (_Float16)(kb + p);
#else
          return *reinterpret_cast<const f16x8g*>(wth + kb * 2048 + p * 1024 + wl);
#endif
        };
        f16x8g b0 = tfrag(0, 0), b1 = tfrag(0, 1);
#pragma unroll 1
        for (int kb = 0; kb < ((GRL_PROBE & 2) ? 0 : KBG); ++kb) {
          f16x8g n0, n1;
          if (kb + 1 < KBG) { n0 = tfrag(kb + 1, 0); n1 = tfrag(kb + 1, 1); }
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            const int fo = rb * 32 * DRG_PITCH + kb * 32;
            const f16x8g a0 = *reinterpret_cast<const f16x8g*>(g2 + fo);
            const f16x8g a1 = *reinterpret_cast<const f16x8g*>(g2 + GT * DRG_PITCH + fo);
            ax[rb] = mfma_g(a1, b0, ax[rb]);
            ax[rb] = mfma_g(a0, b1, ax[rb]);
            ax[rb] = mfma_g(a0, b0, ax[rb]);
          }
          if (kb + 1 < KBG) { b0 = n0; b1 = n1; }
        }
      }
      __syncthreads();   // the planes are spent (the next half, or dpre, reuses R0)
    }

    // ---- G: dpre = dxc_direct silu'(pre) (R1) + dxc_g silu'(pre) -> R0
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);
        const float dg = __builtin_amdgcn_ldexpf(ax[rb][e], BER2(rc) + ec_t - 2 * kSWg);
        *reinterpret_cast<float*>(r0c + rc * XC_PITCH) =
            BPOS(rc) >= 0 ? HPV(rc) + dg * dsl[rb][e] : 0.0f;
      }
    __syncthreads();

    // ---- H: conv backward, row-wide (channels 4*lane..)
    {
      float cw[KC][4];
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int k = 0; k < KC; ++k) cw[k][v] = a.conv_w[(4 * lane + v) * KC + k];
      const char* dp = smem + B_R0 + opaque(16 * lane);
      const char* dh = smem + B_HALO + opaque(16 * lane);
#pragma unroll 2
      for (int j = 0; j < 8; ++j) {
        const int vr = 8 * wave + j;
        const int pos = *reinterpret_cast<const int*>(smem + B_POS + 4 * vr);
        if (pos < 0) continue;
        const int grow = *reinterpret_cast<const int*>(smem + B_ROW + 4 * vr);
        const int rem = *reinterpret_cast<const int*>(smem + B_LAST + 4 * vr);
        const f32x4g dpv = *reinterpret_cast<const f32x4g*>(dp + vr * XC_PITCH);
        f32x4g dxv = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const int lag = KC - 1 - k;   // dpre of row vr + lag reads x_vr through tap k
          if (lag <= rem) {
            const int vn = vr + lag;
            const f32x4g dn = vn < GT ? *reinterpret_cast<const f32x4g*>(dp + vn * XC_PITCH)
                                      : *reinterpret_cast<const f32x4g*>(dh + (vn - GT) * XC_PITCH);
#pragma unroll
            for (int v = 0; v < 4; ++v) dxv[v] = dxv[v] + cw[k][v] * dn[v];
          }
          if (lag <= pos && !(GRL_PROBE & 4)) {   // dW[k] += dpre_vr x_{vr - lag}
            const f32x4g xv = *reinterpret_cast<const f32x4g*>(a.xz + (uint32_t)((grow - lag) * xzr + 4 * lane));
#pragma unroll
            for (int v = 0; v < 4; ++v) cw_acc[k][v] = cw_acc[k][v] + dpv[v] * xv[v];
          }
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) cb_acc[v] = cb_acc[v] + dpv[v];
        __builtin_nontemporal_store(dxv, reinterpret_cast<f32x4g*>(a.dxz + (uint32_t)(grow * dxr + 4 * lane)));
      }
    }
    __syncthreads();
    if (wave == 0) {   // this tile's first 3 rows of dpre: the halo of the next (earlier) tile
#pragma unroll
      for (int j = 0; j < 3; ++j)
        *reinterpret_cast<f32x4g*>(smem + B_HALO + j * XC_PITCH + 16 * lane) =
            *reinterpret_cast<const f32x4g*>(smem + B_R0 + j * XC_PITCH + 16 * lane);
    }
#undef BPOS
#undef BROW
#undef BSEQ
#undef BREM
#undef BER
#undef BER2
#undef PRE
#undef HPV
  }
  // ---- partial sums of this workgroup
  acc_v += __shfl_xor(acc_v, 32);
  acc_r += __shfl_xor(acc_r, 32);
  acc_i += __shfl_xor(acc_i, 32);
  acc_h += __shfl_xor(acc_h, 32);
  if (h == 0) {
    float* pp = a.part + (int64_t)g * 4 * GH;
    pp[c] = -acc_v * dsoftplus_f(lamc);   // Lambda enters as -softplus(Lambda)
    pp[GH + c] = acc_r;
    pp[2 * GH + c] = acc_i;
    pp[3 * GH + c] = acc_h;
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) {
#pragma unroll
    for (int k = 0; k < KC; ++k) cp[(4 * lane + v) * KC + k] = cw_acc[k][v];
    cp[GH * KC + 4 * lane + v] = cb_acc[v];
  }
}

}  // namespace

int grl_fwd_lds_bytes() { return LDS_BYTES; }

int launch_grl_fwd(const float* xz, int64_t xz_rs, const float* conv_w, int KC,
                   const float* conv_b, const void* wf, const float* gate_b, const float* lam,
                   const float* h0, const int* pieces, int64_t B, int64_t G,
                   int64_t ntok, float* y, int64_t y_rs, float* y_last, float* xc_out,
                   float* rg_out, float* carries, int64_t nTc, float* xc_rmax,
                   float* tile_carries, int64_t max_tiles, hipStream_t st) {
  GrlFwdArgs a;
  a.xz = xz; a.xz_rs = xz_rs; a.conv_w = conv_w; a.conv_b = conv_b;
  a.wf = (const f16x8g*)wf;
  a.ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(wf) + (int64_t)2 * GH * GH * 4);
  a.gate_b = gate_b; a.lam = lam; a.h0 = h0;
  a.pieces = pieces; a.B = (int)B; a.G = (int)G; a.ntok = ntok;
  a.y = y; a.y_rs = y_rs; a.y_last = y_last; a.xc_out = xc_out; a.rg_out = rg_out;
  a.carries = carries; a.nTc = (int)nTc; a.xc_rmax = xc_rmax;
  a.tile_carries = tile_carries; a.max_tiles = (int)max_tiles;
  auto run = [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    static bool done = false;  // benign race: idempotent
    if (!done) {
      (void)hipFuncSetAttribute((const void*)k_grl_fwd<K>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
      done = true;
    }
    k_grl_fwd<K><<<(unsigned)G, 512, LDS_BYTES, st>>>(a);
  };
  switch (KC) {
    case 4: run(std::integral_constant<int, 4>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    case 3: run(std::integral_constant<int, 3>{}); break;
    default: return fail("rb_grl_fwd: conv kernel size must be 2, 3 or 4");
  }
  return launch_status("rb_grl_fwd");
}

}  // namespace rb

namespace rb {

int launch_grl_bwd(const float* xz, int64_t xz_rs, const float* conv_w, int KC,
                   const float* conv_b, const void* wf, const void* wft, const float* gate_b,
                   const float* lam, const float* h0, const int* pieces, int64_t B, int64_t G,
                   int64_t ntok, const float* tile_carries, int64_t max_tiles, const float* dy,
                   const float* dy_last, float* dxz, int64_t dxz_rs, float* drg, float* xc_out,
                   float* drg_rmax, float* xc_rmax, float* part, float* cpart, hipStream_t st) {
  GrlBwdArgs a;
  a.xz = xz; a.xz_rs = xz_rs; a.conv_w = conv_w; a.conv_b = conv_b;
  a.wf = (const f16x8g*)wf;
  a.ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(wf) + (int64_t)2 * GH * GH * 4);
  a.wft = (const f16x8g*)wft;
  a.ewt = reinterpret_cast<const int*>(reinterpret_cast<const char*>(wft) + (int64_t)2 * GH * GH * 4);
  a.gate_b = gate_b; a.lam = lam; a.h0 = h0; a.pieces = pieces; a.B = (int)B; a.G = (int)G;
  a.ntok = ntok; a.tile_carries = tile_carries; a.max_tiles = (int)max_tiles; a.dy = dy;
  a.dy_last = dy_last; a.dxz = dxz; a.dxz_rs = dxz_rs; a.drg = drg; a.xc_out = xc_out;
  a.drg_rmax = drg_rmax; a.xc_rmax = xc_rmax; a.part = part; a.cpart = cpart;
  auto run = [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    static bool done = false;  // benign race: idempotent
    if (!done) {
      (void)hipFuncSetAttribute((const void*)k_grl_bwd<K, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, B_LDS_BYTES);
      (void)hipFuncSetAttribute((const void*)k_grl_bwd<K, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, B_LDS_BYTES);
      done = true;
    }
    if (dy_last)
      k_grl_bwd<K, true><<<(unsigned)G, 512, B_LDS_BYTES, st>>>(a);
    else
      k_grl_bwd<K, false><<<(unsigned)G, 512, B_LDS_BYTES, st>>>(a);
  };
  switch (KC) {
    case 4: run(std::integral_constant<int, 4>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    case 3: run(std::integral_constant<int, 3>{}); break;
    default: return fail("rb_grl_bwd: conv kernel size must be 2, 3 or 4");
  }
  return launch_status("rb_grl_bwd");
}

}  // namespace rb
