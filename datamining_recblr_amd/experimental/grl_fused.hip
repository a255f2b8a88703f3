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
#include "../csrc/common.h"
#include "recblr_exp.h"

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
constexpr int LDS_CW = LDS_LAST + GT * 4;       // conv weights [H][KC] and bias [H] (once)
constexpr int LDS_BYTES = LDS_CW + GH * 4 * 4 + GH * 4;

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

// The lane id again, from an instruction the compiler may neither hoist nor
// reuse: per-phase lane-dependent bases are rebuilt (two VALU ops) instead of
// being kept live across the whole tile loop, where they spilled
__device__ __forceinline__ int fresh_lane() {
  int x;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(x));
  return x;
}

__device__ __forceinline__ float opaque_f(float x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Workgroup barrier ordering LDS only: the kernels never read global memory
// another wave wrote, so the row stores (y, dxz, drg, xc) stay in flight
// across it (__syncthreads would drain them at every phase: vmcnt(0))
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
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
  // row map of the tile at the cursor (lane r: virtual row r; row -1 past
  // the span) and the cursor past it
  int mrow, mpos, mseq, mlast;
  auto row_map = [&]() {
    int rp = cur_p, roff = cur_off + lane;
    while (rp < pe && roff >= p_len[rp]) {
      roff -= p_len[rp];
      ++rp;
    }
    const bool rvalid = rp < pe;
    mrow = rvalid ? p_row[rp] + roff : 0;
    mpos = rvalid ? roff : -1;
    mseq = rvalid ? p_seq[rp] : 0;
    mlast = rvalid && roff == p_len[rp] - 1;
    int np = __builtin_amdgcn_readlane(rp, 63), noff = __builtin_amdgcn_readlane(roff, 63) + 1;
    if (np < pe && noff >= p_len[np]) { ++np; noff = 0; }
    cur_p = np;
    cur_off = noff;
  };
  // Register prefetch, one tile ahead: phase A's x rows (this wave's 8 rows
  // and the KC-1 rows before its first) are issued right after phase A has
  // used the current ones, phase D's z values right after phase D; both
  // land while the GEMM and the scan of the current tile run.
  f32x4g xo[8], xh[KC - 1];
  float zp[2][16];
  auto load_x = [&]() {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int vr = 8 * wave + j;
      const int grow = __builtin_amdgcn_readlane(mrow, vr);
      const int pos = __builtin_amdgcn_readlane(mpos, vr);
      xo[j] = pos >= 0
                  ? *reinterpret_cast<const f32x4g*>(a.xz + (uint32_t)(grow * xzr + 4 * lane))
                  : f32x4g{0.0f, 0.0f, 0.0f, 0.0f};
    }
    const int g0 = __builtin_amdgcn_readlane(mrow, 8 * wave);
    const int p0 = __builtin_amdgcn_readlane(mpos, 8 * wave);
#pragma unroll
    for (int i = 0; i < KC - 1; ++i) {   // row g0 - (KC - 1 - i)
      const int l = KC - 1 - i;
      xh[i] = p0 >= l
                  ? *reinterpret_cast<const f32x4g*>(a.xz + (uint32_t)((g0 - l) * xzr + 4 * lane))
                  : f32x4g{0.0f, 0.0f, 0.0f, 0.0f};
    }
  };
  auto load_z = [&](int rb) {   // C layout: row 32 rb + 8 (e / 4) + 4 h + e % 4
    const int rv = mpos >= 0 ? mrow : -1;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);
        const int r0 = __builtin_amdgcn_readlane(rv, rc), r1 = __builtin_amdgcn_readlane(rv, rc + 4);
        const int grow = h ? r1 : r0;
        zp[rb][e] = grow >= 0 ? a.xz[(uint32_t)(grow * xzr + GH + c)] : 0.0f;
      }
  };
  // conv weights and bias -> LDS once (phase A then issues no global loads
  // of its own: a vector-memory wait there would also wait for the prefetch)
  for (int i = tid; i < GH * KC; i += 512)
    reinterpret_cast<float*>(smem + LDS_CW)[(i / KC) * 4 + i % KC] = a.conv_w[i];
  for (int i = tid; i < GH; i += 512) reinterpret_cast<float*>(smem + LDS_CW + GH * 16)[i] = a.conv_b[i];
  row_map();
  load_x();
  load_z(0);
  load_z(1);
  lds_sync();
  auto store_y = [&]() {
    const char* yb = smem + opaque(LDS_XC + 16 * lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int vr = 8 * wave + j;
      if (s_pos[vr] >= 0)
        __builtin_nontemporal_store(*reinterpret_cast<const f32x4g*>(yb + vr * XC_PITCH),
                                    reinterpret_cast<f32x4g*>(a.y + (uint32_t)(s_row[vr] * yr + 4 * lane)));
    }
  };

  for (int v0 = 0; v0 < span_rows; v0 += GT) {
    if (a.tile_carries && h == 0)
      a.tile_carries[((int64_t)g * a.max_tiles + v0 / GT) * GH + c] = carry;
    const bool more = v0 + GT < span_rows;

    // per-lane LDS bases of this tile (see opaque())
    // (region offsets inside opaque(): the per-row constants fold into the
    // 16-bit ds_* immediates)
    char* const ab_xc = smem + opaque(LDS_XC + 16 * lane);
    char* const ab_fr = smem + opaque(LDS_PLANE0 + (lane >> 2) * FRAG_PITCH +
                                      32 * ((lane >> 1) & 1) * 16 + 8 * (lane & 1));
    char* const db = smem + opaque(LDS_ER + 16 * h);               // per-row int arrays
    char* const xb = smem + opaque(LDS_XC + 4 * h * XC_PITCH + 4 * c);   // s_xc[4h][c]
    char* const gb = smem + opaque(LDS_PLANE0 + lane * 16);         // GEMM A fragments
    // the previous tile's y rows, whole 1 KB rows from LDS (phase D left
    // them in the xc slots: per-lane 4-byte stores there cost 20 % more)
    if (a.y && v0 > 0) store_y();
    // ---- phase A: conv + SiLU, LDS images (channels 4*lane .. 4*lane+3)
    float cw[KC][4], cb[4];
    {
      const char* cwp = smem + opaque(LDS_CW + 64 * lane);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const f32x4g w4 = *reinterpret_cast<const f32x4g*>(cwp + 16 * v);
#pragma unroll
        for (int k = 0; k < KC; ++k) cw[k][v] = w4[k];
      }
      const f32x4g b4 = *reinterpret_cast<const f32x4g*>(smem + opaque(LDS_CW + GH * 16 + 16 * lane));
#pragma unroll
      for (int v = 0; v < 4; ++v) cb[v] = b4[v];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int vr = 8 * wave + j;
      const int grow = __builtin_amdgcn_readlane(mrow, vr);
      const int pos = __builtin_amdgcn_readlane(mpos, vr);   // -1: past the span
      f32x4g xcv = {0.0f, 0.0f, 0.0f, 0.0f};
      if (pos >= 0) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          float acc = cb[v];
#pragma unroll
          for (int k = 0; k < KC; ++k) {   // lag l: rows before the sequence start are zero
            const int l = KC - 1 - k;
            const float xv = j - l >= 0 ? xo[j - l >= 0 ? j - l : 0][v] : xh[j - l >= 0 ? 0 : KC - 1 + j - l][v];
            acc = acc + (l <= pos ? cw[k][v] * xv : 0.0f);
          }
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
        s_seq[vr] = __builtin_amdgcn_readlane(mseq, vr);
        s_last[vr] = __builtin_amdgcn_readlane(mlast, vr);
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
    lds_sync();

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
    // weight fragments two k16 steps ahead (L2 latency over one step's MFMAs)
    f16x8g br0 = wfrag(wr, 0, 0), br1 = wfrag(wr, 0, 1), bi0 = wfrag(wi, 0, 0), bi1 = wfrag(wi, 0, 1);
    f16x8g nr0 = wfrag(wr, 1, 0), nr1 = wfrag(wr, 1, 1), ni0 = wfrag(wi, 1, 0), ni1 = wfrag(wi, 1, 1);
#pragma unroll 1
    for (int kb = 0; kb < KBG; ++kb) {
      f16x8g mr0, mr1, mi0, mi1;
      if (kb + 2 < KBG) {
        mr0 = wfrag(wr, kb + 2, 0); mr1 = wfrag(wr, kb + 2, 1);
        mi0 = wfrag(wi, kb + 2, 0); mi1 = wfrag(wi, kb + 2, 1);
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
      br0 = nr0; br1 = nr1; bi0 = ni0; bi1 = ni1;
      if (kb + 2 < KBG) { nr0 = mr0; nr1 = mr1; ni0 = mi0; ni1 = mi1; }
    }
    // the next tile's row map and x rows, issued behind the last weight loads
    // (vector-memory waits are in order: a later weight wait would wait for
    // them too) and landing under phase D and the next phase A
    if (more) {
      row_map();
      load_x();
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
          const float yv = fsilu(zp[rb][e]) * hn;
          if (a.y)   // over this (row, channel)'s xc, read above
            *reinterpret_cast<float*>(xb + rc * XC_PITCH) = yv;
          else if (pos >= 0 && a.y_last && DLAST(rc))
            a.y_last[(uint32_t)(DSEQ(rc) * GH + c)] = yv;
        }
      }
      if (more) load_z(rb);   // this block's z of the next tile (its row map is current)
    }
    carry = run;
#undef DROW
#undef DPOS
#undef DSEQ
#undef DLAST
#undef DER
    lds_sync();   // LDS is rewritten by the next tile
  }
  if (a.y) store_y();
}

// ---------------------------------------------------------------------------
// Backward of k_grl_fwd, one launch per layer (RecBLR.py:182-206 reversed):
// the same work lists, each workgroup walking its virtual rows in REVERSE
// 64-row tiles, the adjoint state carried across tiles.  Per tile:
//   A  row-wide: xc = silu(conv(x)) recomputed (-> LDS R0, fp32; and to HBM,
//      the gates weight gradient's operand), as the f16 A planes of GEMM 1
//      (-> LDS R1)
//   C  GEMM 1: r / i of channels 32w.. (as the forward)
//   D  C layout: gates; the forward scan from the tile's checkpoint (the
//      forward's tile_carries): dz (to HBM) and gy = dy silu(z) (-> R1, the
//      planes are spent); the reverse adjoint scan (e_t = a_t (gy_t +
//      e_{t+1}), reset at each sequence's last row) gives d = dL/dh, then
//      dr, di, dxc's direct term (kept in registers) and the partial sums of
//      dLambda, d gate_b, dh0
//   E  dr -> R0, di -> R1 (fp32, row-major); then row-wide: each drg row to
//      HBM in 1 KB pieces, its exact max over 512 columns, and in place its
//      f16 planes (x = 2^-s (x0 + x1)) as GEMM 2's A operand
//   F  GEMM 2: dxc_g = drg W_g for channels 32w.. (W_g^T's image), K = 512
//   G  dxc = dxc_g + the direct term (-> R0, C layout)
//   H  row-wide: H1 pre-activations again from x (the rows dW needs anyway),
//      dpre = dxc silu'(pre) in place, dW / dbias partials; H2 dx from dpre of
//      the row and the next KC-1 (later rows: R0 or the halo of the later tile)
// Only the per-lane dz stores are 4-byte scattered; every other row stream is
// written in 16-B lane pieces of whole rows.
constexpr int B_R0 = 0;                        // xc / dr (fp32, then planes) / dxc, dpre
constexpr int B_R1 = GT * XC_PITCH;            // xc planes / gy / di (fp32, then planes)
constexpr int B_HALO = B_R1 + GT * XC_PITCH;   // 3 rows of dpre (the later tile's first rows)
constexpr int B_ER = B_HALO + 3 * XC_PITCH;    // xc row exponents
constexpr int B_ER2 = B_ER + GT * 4;           // drg row exponents
constexpr int B_ROW = B_ER2 + GT * 4;
constexpr int B_POS = B_ROW + GT * 4;
constexpr int B_SEQ = B_POS + GT * 4;
constexpr int B_LAST = B_SEQ + GT * 4;         // rows left to the sequence's end (0: last)
constexpr int B_CW = B_LAST + GT * 4;          // conv weights [H][4] and bias [H] (once)
constexpr int B_LDS_BYTES = B_CW + GH * 16 + GH * 4;
constexpr int PL_LO = GH * 2;                  // a drg half's lo plane, bytes into its row

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
  const float nsp = -softplus_f(lamc), nsp_k = nsp;
  const float br = a.gate_b[c], bi = a.gate_b[GH + c];
  const int ec_r = a.ew[c], ec_i = a.ew[GH + c], ec_t = a.ewt[c];
  const float hz = a.h0 ? a.h0[c] : 0.0f;
  // element offsets are 32-bit (rb_grl_bwd checks ntok * row stride < 2^31)
  const int xzr = (int)a.xz_rs, dxr = (int)a.dxz_rs;
  const char* wr = reinterpret_cast<const char*>(a.wf) + (int64_t)wave * KBG * 2048;
  const char* wi = reinterpret_cast<const char*>(a.wf) + (int64_t)(8 + wave) * KBG * 2048;
  const char* wt = reinterpret_cast<const char*>(a.wft) + (int64_t)wave * (2 * KBG) * 2048;

  // conv weights and bias -> LDS once
  for (int i = tid; i < GH * KC; i += 512)
    reinterpret_cast<float*>(smem + B_CW)[(i / KC) * 4 + i % KC] = a.conv_w[i];
  for (int i = tid; i < GH; i += 512) reinterpret_cast<float*>(smem + B_CW + GH * 16)[i] = a.conv_b[i];

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
  lds_sync();

  // conv weights of channels 4*lane.. from LDS (fresh bases: not kept live)
  auto conv_weights = [&](float (&cw)[KC][4], float (&cbv)[4]) {
    const int lf = fresh_lane();
    const char* cwp = smem + (B_CW + 64 * lf);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const f32x4g w4 = *reinterpret_cast<const f32x4g*>(cwp + 16 * v);
#pragma unroll
      for (int k = 0; k < KC; ++k) cw[k][v] = w4[k];
    }
    const f32x4g b4 = *reinterpret_cast<const f32x4g*>(smem + (B_CW + GH * 16 + 16 * lf));
#pragma unroll
    for (int v = 0; v < 4; ++v) cbv[v] = b4[v];
  };

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

    // ---- A: xc (fp32 -> R0, HBM), its f16 planes (-> R1)
    {
      float cw[KC][4], cbv[4];
      conv_weights(cw, cbv);
      char* const ab_xc = smem + opaque(B_R0 + 16 * lane);
      char* const ab_fr = smem + opaque(B_R1 + (lane >> 2) * FRAG_PITCH + 32 * ((lane >> 1) & 1) * 16 +
                                        8 * (lane & 1));
#pragma unroll 2
      for (int j = 0; j < 8; ++j) {
        const int vr = 8 * wave + j;
        const int grow = __builtin_amdgcn_readlane(rrow, vr);
        const int pos = __builtin_amdgcn_readlane(rpos, vr);
        f32x4g xcv = {0.0f, 0.0f, 0.0f, 0.0f};
        if (pos >= 0) {
          f32x4g xs[KC];
#pragma unroll
          for (int k = 0; k < KC; ++k)
            xs[k] = KC - 1 - k <= pos
                        ? *reinterpret_cast<const f32x4g*>(a.xz + (uint32_t)((grow - (KC - 1 - k)) * xzr + 4 * lane))
                        : f32x4g{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            float acc = cbv[v];
#pragma unroll
            for (int k = 0; k < KC; ++k)
              acc = acc + (KC - 1 - k <= pos ? cw[k][v] * xs[k][v] : 0.0f);
            xcv[v] = fsilu(acc);
          }
          __builtin_nontemporal_store(xcv, reinterpret_cast<f32x4g*>(a.xc_out + (uint32_t)(grow * GH + 4 * lane)));
        }
        *reinterpret_cast<f32x4g*>(ab_xc + vr * XC_PITCH) = xcv;
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
    lds_sync();

    // ---- C: GEMM 1 (r, i)
    f32x16g ar[2], ai[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int e = 0; e < 16; ++e) { ar[rb][e] = 0.0f; ai[rb][e] = 0.0f; }
    {
      const int wl = opaque(lane * 16);
      const char* const gb = smem + opaque(B_R1 + lane * 16);
      auto wfrag = [&](const char* base, int kb, int p) {
        return *reinterpret_cast<const f16x8g*>(base + kb * 2048 + p * 1024 + wl);
      };
      f16x8g br0 = wfrag(wr, 0, 0), br1 = wfrag(wr, 0, 1), bi0 = wfrag(wi, 0, 0), bi1 = wfrag(wi, 0, 1);
      f16x8g nr0 = wfrag(wr, 1, 0), nr1 = wfrag(wr, 1, 1), ni0 = wfrag(wi, 1, 0), ni1 = wfrag(wi, 1, 1);
#pragma unroll 1
      for (int kb = 0; kb < KBG; ++kb) {
        f16x8g mr0, mr1, mi0, mi1;
        if (kb + 2 < KBG) {
          mr0 = wfrag(wr, kb + 2, 0); mr1 = wfrag(wr, kb + 2, 1);
          mi0 = wfrag(wi, kb + 2, 0); mi1 = wfrag(wi, kb + 2, 1);
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
        br0 = nr0; br1 = nr1; bi0 = ni0; bi1 = ni1;
        if (kb + 2 < KBG) { nr0 = mr0; nr1 = mr1; ni0 = mi0; ni1 = mi1; }
      }
    }
    lds_sync();   // R1's planes are spent: gy goes there

// each phase takes fresh (opaque) bases: per-row values are re-read from
// LDS, never kept in registers from one phase to the next
#define GRL_BASES                                                                   \
  const int lane_f = fresh_lane();                                                  \
  const int h = lane_f >> 5;                                                        \
  const int c = 32 * wave + (lane_f & 31);                                          \
  const char* const db = smem + (B_ER + 16 * h);               /* per-row ints */   \
  char* const r0c = smem + (B_R0 + 4 * h * XC_PITCH + 4 * c);  /* R0 [4h][c] */     \
  char* const r1c = smem + (B_R1 + 4 * h * XC_PITCH + 4 * c)   /* R1 [4h][c] */
#define BPOS(rc) (*reinterpret_cast<const int*>(db + (B_POS - B_ER) + 4 * (rc)))
#define BROW(rc) (*reinterpret_cast<const int*>(db + (B_ROW - B_ER) + 4 * (rc)))
#define BSEQ(rc) (*reinterpret_cast<const int*>(db + (B_SEQ - B_ER) + 4 * (rc)))
#define BREM(rc) (*reinterpret_cast<const int*>(db + (B_LAST - B_ER) + 4 * (rc)))
#define BER(rc) (*reinterpret_cast<const int*>(db + 4 * (rc)))
#define BER2(rc) (*reinterpret_cast<const int*>(db + (B_ER2 - B_ER) + 4 * (rc)))
#define XCV(rc) (*reinterpret_cast<const float*>(r0c + (rc) * XC_PITCH))
#define HPV(rc) (*reinterpret_cast<float*>(r1c + (rc) * XC_PITCH))
    // ---- D (forward part): gates (ar <- sigmoid(r), ai <- sigmoid(i); alpha,
    // beta, b' recomputed from them where needed), the forward scan from the
    // tile's checkpoint: the state entering each 4-row group (cin), dz, and
    // gy = dy silu(z) -> LDS R1
    float cin[2][4];
    {
      GRL_BASES;
      float run = a.tile_carries[((int64_t)g * a.max_tiles + t) * GH + c];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        float bp[16], al[16], zv[16], gv[16];
        // this block's z and dy first: their latency hides under the gate math
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if ((e & 3) == 0) __builtin_amdgcn_sched_barrier(0);
          const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);
          zv[e] = gv[e] = 0.0f;
          if (BPOS(rc) >= 0) {
            const int grow = BROW(rc);
            zv[e] = a.xz[(uint32_t)(grow * xzr + GH + c)];
            gv[e] = !LASTDY ? a.dy[(uint32_t)(grow * GH + c)]
                            : (BREM(rc) == 0 ? a.dy_last[(uint32_t)(BSEQ(rc) * GH + c)] : 0.0f);
          }
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if ((e & 3) == 0) __builtin_amdgcn_sched_barrier(0);
          const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);
          const int er = BER(rc);
          const float r = __builtin_amdgcn_ldexpf(ar[rb][e], er + ec_r - 2 * kSWg) + br;
          const float i = __builtin_amdgcn_ldexpf(ai[rb][e], er + ec_i - 2 * kSWg) + bi;
          const bool ok = BPOS(rc) >= 0;
          const float sr = fsigm(r);
          const float aa = ok ? fexp(nsp * sr) : 1.0f;
          const float si = fsigm(i);
          const float sq = fsqrt(1.0f - aa * aa + 1e-8f);
          bp[e] = ok ? sq * si * XCV(rc) : 0.0f;
          ar[rb][e] = sr;
          ai[rb][e] = si;
          al[e] = aa;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          __builtin_amdgcn_sched_barrier(0);   // scheduling region: one 4-row group
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
          __builtin_amdgcn_sched_barrier(0);   // scheduling region: one 4-row group
          float hp = cin[rb][q];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int e = 4 * q + u;
            const int rc = 32 * rb + 8 * q + u;
            const int pos = BPOS(rc);
            if (pos == 0) hp = hz;
            const float hn = hp * al[e] + bp[e];
            hp = hn;
            const float zz = zv[e];
            const float sz = fsigm(zz);
            if (pos >= 0)
              a.dxz[(uint32_t)(BROW(rc) * dxr + GH + c)] = (gv[e] * hn) * (sz * (1.0f + zz * (1.0f - sz)));
            HPV(rc) = gv[e] * (zz * sz);   // 0 past the span (gv = 0)
          }
        }
      }
    }

    // ---- D (reverse part): adjoint, gate gradients; dr, di -> ar, ai; dxc's
    // direct term -> dxd
    float dxd[2][16];
    {
      GRL_BASES;
      float run = eadj;
#pragma unroll
      for (int rbr = 0; rbr < 2; ++rbr) {
        const int rb = 1 - rbr;
        // groups of this block in reverse row order: (q, half 1), (q, half 0), q = 3..0
        float ein[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          __builtin_amdgcn_sched_barrier(0);
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
          __builtin_amdgcn_sched_barrier(0);   // scheduling region: one 4-row group
          // the group's 4 rows: gate values and the forward state again (a
          // fresh copy of nsp: the exps are recomputed, not kept from the
          // aggregate pass)
          float ga[4], gq[4], gx[4], hpv[4];
          const float nspq = opaque_f(nsp_k);
          {
            float hp = cin[rb][q];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int e = 4 * q + u;
              const int rc = 32 * rb + 8 * q + u;
              const int pos = BPOS(rc);
              const bool ok = pos >= 0;
              const float aa = ok ? fexp(nspq * ar[rb][e]) : 1.0f;
              const float sq = fsqrt(1.0f - aa * aa + 1e-8f);
              const float xcv = XCV(rc);
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
            const float dr = ok ? (dv * nspq) * ((1.0f - sr) * sr) : 0.0f;
            const float di = ok ? (dbeta * sq) * ((1.0f - si) * si) : 0.0f;
            dxd[rb][e] = ok ? d * (sq * si) : 0.0f;
            if (ok) {
              acc_v += dv * sr;
              acc_r += dr;
              acc_i += di;
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
    lds_sync();   // every wave is past its reads of xc (R0) and gy (R1)

    // ---- E: dr -> R0, di -> R1 (fp32, row-major), then row-wide
    {
      GRL_BASES;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if ((e & 3) == 0) __builtin_amdgcn_sched_barrier(0);
          const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);
          *reinterpret_cast<float*>(r0c + rc * XC_PITCH) = ar[rb][e];
          *reinterpret_cast<float*>(r1c + rc * XC_PITCH) = ai[rb][e];
        }
    }
    lds_sync();
    {
      char* const e0 = smem + opaque(B_R0 + 16 * lane);
      char* const e1 = smem + opaque(B_R1 + 16 * lane);
#pragma unroll 2
      for (int j = 0; j < 8; ++j) {
        const int vr = 8 * wave + j;
        const int pos = *reinterpret_cast<const int*>(smem + B_POS + 4 * vr);
        const f32x4g dr4 = *reinterpret_cast<const f32x4g*>(e0 + vr * XC_PITCH);
        const f32x4g di4 = *reinterpret_cast<const f32x4g*>(e1 + vr * XC_PITCH);
        const int grow = *reinterpret_cast<const int*>(smem + B_ROW + 4 * vr);
        if (pos >= 0) {
          __builtin_nontemporal_store(dr4, reinterpret_cast<f32x4g*>(a.drg + (uint32_t)(grow * (2 * GH) + 4 * lane)));
          __builtin_nontemporal_store(di4, reinterpret_cast<f32x4g*>(a.drg + (uint32_t)(grow * (2 * GH) + GH + 4 * lane)));
        }
        float m = 0.0f;
#pragma unroll
        for (int v = 0; v < 4; ++v) m = fmaxf(m, fmaxf(fabsf(dr4[v]), fabsf(di4[v])));
        m = wave_max(m);
        const int e = m > 0.0f ? __builtin_amdgcn_frexp_expf(m) : 0;
        if (lane == 0) {
          *reinterpret_cast<int*>(smem + B_ER2 + 4 * vr) = e;
          if (a.drg_rmax && pos >= 0)
            atomicMax(reinterpret_cast<int*>(a.drg_rmax) + (grow >> 5), __float_as_int(m));
        }
        const float sc = __builtin_amdgcn_ldexpf(1.0f, kSWg - e);
        // in place: the row's hi plane at +0, lo plane at +PL_LO (halfs)
        f16x4g rh, rl, ih, il;
#pragma unroll
        for (int v = 0; v < 4; v += 2) {
          const f32x2g xr = f32x2g{dr4[v], dr4[v + 1]} * sc;
          const f16x2g r0 = __builtin_convertvector(xr, f16x2g);
          const f16x2g r1 = __builtin_convertvector(xr - __builtin_convertvector(r0, f32x2g), f16x2g);
          const f32x2g xi = f32x2g{di4[v], di4[v + 1]} * sc;
          const f16x2g i0 = __builtin_convertvector(xi, f16x2g);
          const f16x2g i1 = __builtin_convertvector(xi - __builtin_convertvector(i0, f32x2g), f16x2g);
          rh[v] = r0[0]; rh[v + 1] = r0[1]; rl[v] = r1[0]; rl[v + 1] = r1[1];
          ih[v] = i0[0]; ih[v + 1] = i0[1]; il[v] = i1[0]; il[v + 1] = i1[1];
        }
        // the wave's own row: its 16-B reads above are done before these writes
        *reinterpret_cast<f16x4g*>(e0 - 8 * lane + vr * XC_PITCH) = rh;
        *reinterpret_cast<f16x4g*>(e0 - 8 * lane + vr * XC_PITCH + PL_LO) = rl;
        *reinterpret_cast<f16x4g*>(e1 - 8 * lane + vr * XC_PITCH) = ih;
        *reinterpret_cast<f16x4g*>(e1 - 8 * lane + vr * XC_PITCH + PL_LO) = il;
      }
    }
    lds_sync();

    // ---- F: GEMM 2, dxc_g for channels 32w.. (K = 512: dr's planes in R0,
    // di's in R1)
    f32x16g ax[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int e = 0; e < 16; ++e) ax[rb][e] = 0.0f;
    {
      const int wl = opaque(lane * 16);
      // A fragment of lane l: row l % 32, halfs 8 (l / 32) .. + 7 of a k16 block
      const char* const g2 = smem + opaque((lane & 31) * XC_PITCH + 16 * (lane >> 5));
      auto tfrag = [&](int kk, int p) {
        return *reinterpret_cast<const f16x8g*>(wt + kk * 2048 + p * 1024 + wl);
      };
      f16x8g b0 = tfrag(0, 0), b1 = tfrag(0, 1), n0 = tfrag(1, 0), n1 = tfrag(1, 1);
#pragma unroll 1
      for (int kk = 0; kk < 2 * KBG; ++kk) {
        f16x8g m0, m1;
        if (kk + 2 < 2 * KBG) { m0 = tfrag(kk + 2, 0); m1 = tfrag(kk + 2, 1); }
        const char* const ga = g2 + (kk < KBG ? B_R0 + kk * 32 : B_R1 + (kk - KBG) * 32);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const f16x8g a0 = *reinterpret_cast<const f16x8g*>(ga + rb * 32 * XC_PITCH);
          const f16x8g a1 = *reinterpret_cast<const f16x8g*>(ga + rb * 32 * XC_PITCH + PL_LO);
          ax[rb] = mfma_g(a1, b0, ax[rb]);
          ax[rb] = mfma_g(a0, b1, ax[rb]);
          ax[rb] = mfma_g(a0, b0, ax[rb]);
        }
        b0 = n0; b1 = n1;
        if (kk + 2 < 2 * KBG) { n0 = m0; n1 = m1; }
      }
    }
    lds_sync();   // the planes are spent: dxc goes to R0

    // ---- G: dxc = dxc_g + the direct term -> R0 (C layout)
    {
      GRL_BASES;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if ((e & 3) == 0) __builtin_amdgcn_sched_barrier(0);
          const int rc = 32 * rb + 8 * (e >> 2) + (e & 3);
          *reinterpret_cast<float*>(r0c + rc * XC_PITCH) =
              __builtin_amdgcn_ldexpf(ax[rb][e], BER2(rc) + ec_t - 2 * kSWg) + dxd[rb][e];
        }
    }
    lds_sync();

    // ---- H: conv backward, row-wide (channels 4*lane..).  H1: the
    // pre-activation again from x (the rows dW needs anyway), dpre = dxc
    // silu'(pre) -> R0 in place, dW / dbias partials; H2: dx from dpre of
    // this row and the next KC-1 (later rows: R0 or the halo)
    {
      float cw[KC][4], cbv[4];
      conv_weights(cw, cbv);
      char* const dp = smem + opaque(B_R0 + 16 * lane);
      const char* const dh = smem + opaque(B_HALO + 16 * lane);
#pragma unroll 2
      for (int j = 0; j < 8; ++j) {
        const int vr = 8 * wave + j;
        const int pos = *reinterpret_cast<const int*>(smem + B_POS + 4 * vr);
        f32x4g dpv = {0.0f, 0.0f, 0.0f, 0.0f};
        if (pos >= 0) {
          const int grow = *reinterpret_cast<const int*>(smem + B_ROW + 4 * vr);
          f32x4g xs[KC];
#pragma unroll
          for (int k = 0; k < KC; ++k)
            xs[k] = KC - 1 - k <= pos
                        ? *reinterpret_cast<const f32x4g*>(a.xz + (uint32_t)((grow - (KC - 1 - k)) * xzr + 4 * lane))
                        : f32x4g{0.0f, 0.0f, 0.0f, 0.0f};
          const f32x4g g1 = *reinterpret_cast<const f32x4g*>(dp + vr * XC_PITCH);
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            float acc = cbv[v];
#pragma unroll
            for (int k = 0; k < KC; ++k) acc = acc + (KC - 1 - k <= pos ? cw[k][v] * xs[k][v] : 0.0f);
            dpv[v] = g1[v] * fdsilu(acc);
#pragma unroll
            for (int k = 0; k < KC; ++k) cw_acc[k][v] = cw_acc[k][v] + dpv[v] * xs[k][v];
            cb_acc[v] = cb_acc[v] + dpv[v];
          }
        }
        *reinterpret_cast<f32x4g*>(dp + vr * XC_PITCH) = dpv;
      }
      lds_sync();
#pragma unroll 2
      for (int j = 0; j < 8; ++j) {
        const int vr = 8 * wave + j;
        const int pos = *reinterpret_cast<const int*>(smem + B_POS + 4 * vr);
        if (pos < 0) continue;
        const int grow = *reinterpret_cast<const int*>(smem + B_ROW + 4 * vr);
        const int rem = *reinterpret_cast<const int*>(smem + B_LAST + 4 * vr);
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
        }
        __builtin_nontemporal_store(dxv, reinterpret_cast<f32x4g*>(a.dxz + (uint32_t)(grow * dxr + 4 * lane)));
      }
    }
    lds_sync();
    if (wave == 0) {   // this tile's first 3 rows of dpre: the halo of the next (earlier) tile
#pragma unroll
      for (int j = 0; j < 3; ++j)
        *reinterpret_cast<f32x4g*>(smem + B_HALO + j * XC_PITCH + 16 * lane) =
            *reinterpret_cast<const f32x4g*>(smem + B_R0 + j * XC_PITCH + 16 * lane);
    }
#undef GRL_BASES
#undef BPOS
#undef BROW
#undef BSEQ
#undef BREM
#undef BER
#undef BER2
#undef XCV
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
