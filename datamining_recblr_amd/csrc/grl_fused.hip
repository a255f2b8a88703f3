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
  // the wave's r and i column blocks of the weight image (wave-uniform bases)
  const char* wr = reinterpret_cast<const char*>(a.wf) + (int64_t)wave * KBG * 2048;
  const char* wi = reinterpret_cast<const char*>(a.wf) + (int64_t)(8 + wave) * KBG * 2048;

  float carry = 0.0f;                      // state entering the tile (channel c)
  // virtual-row cursor over the pieces (wave-uniform)
  int cur_p = pb, cur_off = 0;

  for (int v0 = 0; v0 < span_rows; v0 += GT) {
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
    char* const ab_xc = smem + LDS_XC + opaque(16 * lane);
    char* const ab_fr = smem + opaque((lane >> 2) * FRAG_PITCH + 32 * ((lane >> 1) & 1) * 16 +
                                      8 * (lane & 1));
    char* const db = smem + opaque(16 * h);                       // per-row int arrays
    char* const xb = smem + LDS_XC + opaque(4 * h * XC_PITCH + 4 * c);   // s_xc[4h][c]
    char* const gb = smem + opaque(lane * 16);                      // GEMM A fragments
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
          if (KC - 1 - k <= pos)
            xs[k] = *reinterpret_cast<const f32x4g*>(a.xz + (int64_t)(grow - (KC - 1 - k)) * a.xz_rs + 4 * lane);
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
        if (a.xc_out) __builtin_nontemporal_store(xcv, reinterpret_cast<f32x4g*>(a.xc_out + (int64_t)grow * GH + 4 * lane));
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
      *reinterpret_cast<f16x4g*>(ab_fr + LDS_PLANE0 + fo) = h0v;
      *reinterpret_cast<f16x4g*>(ab_fr + LDS_PLANE1 + fo) = h1v;
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
      return *reinterpret_cast<const f16x8g*>(base + kb * 2048 + p * 1024 + wl);
    };
    f16x8g br0 = wfrag(wr, 0, 0), br1 = wfrag(wr, 0, 1), bi0 = wfrag(wi, 0, 0), bi1 = wfrag(wi, 0, 1);
#pragma unroll 1
    for (int kb = 0; kb < KBG; ++kb) {
      f16x8g nr0, nr1, ni0, ni1;
      if (kb + 1 < KBG) {
        nr0 = wfrag(wr, kb + 1, 0); nr1 = wfrag(wr, kb + 1, 1);
        ni0 = wfrag(wi, kb + 1, 0); ni1 = wfrag(wi, kb + 1, 1);
      }
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int fo = (rb * KBG + kb) * FRAG_PITCH;
        const f16x8g a0 = *reinterpret_cast<const f16x8g*>(gb + LDS_PLANE0 + fo);
        const f16x8g a1 = *reinterpret_cast<const f16x8g*>(gb + LDS_PLANE1 + fo);
        ar[rb] = mfma_g(a1, br0, ar[rb]);
        ar[rb] = mfma_g(a0, br1, ar[rb]);
        ar[rb] = mfma_g(a0, br0, ar[rb]);
        ai[rb] = mfma_g(a1, bi0, ai[rb]);
        ai[rb] = mfma_g(a0, bi1, ai[rb]);
        ai[rb] = mfma_g(a0, bi0, ai[rb]);
      }
      if (kb + 1 < KBG) { br0 = nr0; br1 = nr1; bi0 = ni0; bi1 = ni1; }
    }

#define DROW(rc) (*reinterpret_cast<const int*>(db + LDS_ROW + 4 * (rc)))
#define DPOS(rc) (*reinterpret_cast<const int*>(db + LDS_POS + 4 * (rc)))
#define DSEQ(rc) (*reinterpret_cast<const int*>(db + LDS_SEQ + 4 * (rc)))
#define DLAST(rc) (*reinterpret_cast<const int*>(db + LDS_LAST + 4 * (rc)))
#define DER(rc) (*reinterpret_cast<const int*>(db + LDS_ER + 4 * (rc)))
    // ---- phase D: gates, scan, merge (lane: channel c, rows of its C layout),
    // one 32-row block at a time; alpha -> ar, b' -> ai in place
    float run = carry;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      float zr[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);   // row = rc + 4h
        zr[e] = DPOS(rc) >= 0 ? a.xz[(int64_t)DROW(rc) * a.xz_rs + GH + c] : 0.0f;
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);   // row = rc + 4h
        const int er = DER(rc);
        const float r = __builtin_amdgcn_ldexpf(ar[rb][e], er + ec_r - 2 * kSWg);
        const float i = __builtin_amdgcn_ldexpf(ai[rb][e], er + ec_i - 2 * kSWg);
        const int pos = DPOS(rc);
        if (a.rg_out && pos >= 0) {
          float* o = a.rg_out + (int64_t)DROW(rc) * (2 * GH) + c;
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
            a.carries[((int64_t)DSEQ(rc) * a.nTc + (pos >> 4)) * GH + c] = hp;
          const float hn = hp * ar[rb][e] + ai[rb][e];
          hp = hn;
          const float yv = fsilu(zr[e]) * hn;
          if (pos >= 0) {
            if (a.y) a.y[(int64_t)DROW(rc) * a.y_rs + c] = yv;
            else if (a.y_last && DLAST(rc)) a.y_last[(int64_t)DSEQ(rc) * GH + c] = yv;
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

}  // namespace

int grl_fwd_lds_bytes() { return LDS_BYTES; }

int launch_grl_fwd(const float* xz, int64_t xz_rs, const float* conv_w, int KC,
                   const float* conv_b, const void* wf, const float* gate_b, const float* lam,
                   const float* h0, const int* pieces, int64_t B, int64_t G,
                   int64_t ntok, float* y, int64_t y_rs, float* y_last, float* xc_out,
                   float* rg_out, float* carries, int64_t nTc, float* xc_rmax,
                   hipStream_t st) {
  GrlFwdArgs a;
  a.xz = xz; a.xz_rs = xz_rs; a.conv_w = conv_w; a.conv_b = conv_b;
  a.wf = (const f16x8g*)wf;
  a.ew = reinterpret_cast<const int*>(reinterpret_cast<const char*>(wf) + (int64_t)2 * GH * GH * 4);
  a.gate_b = gate_b; a.lam = lam; a.h0 = h0;
  a.pieces = pieces; a.B = (int)B; a.G = (int)G; a.ntok = ntok;
  a.y = y; a.y_rs = y_rs; a.y_last = y_last; a.xc_out = xc_out; a.rg_out = rg_out;
  a.carries = carries; a.nTc = (int)nTc; a.xc_rmax = xc_rmax;
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
