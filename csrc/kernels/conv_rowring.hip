// conv_rowring.hip — weight-stationary, row-streaming 3x3 convolution for 64 -> <=64 channels
// at width 56 (ResNet50 stage 2: conv2_block{1,2,3}_2_conv; gfx950).
//
// Why: those three convs are ~9 % of a ResNet50 forward and run at ~20 % of the MFMA peak on
// every implicit-GEMM tile (v2 / ws / pt): with 64 output channels a tile's weights are only
// 64 rows, so each (tap, chunk) K tile moves BM activation rows + 64 weight rows from L2 to LDS
// for 2 x BM x 64 x 64 MACs, and the 3x3 taps re-read every input row 9 times.
//
// What: a workgroup owns a STRIP of one image — consecutive 4-row output tiles (224 pixels,
// the width is 56). It loads the whole 3x3 x 64 x 64 weight block into LDS once (72 KiB, it
// stays there) and streams the input through a ring of 10 image rows (each row: 56 pixels + a
// zero column on both sides, 64 LDS rows of 128 B): tile i reads input rows R_i - 1 .. R_i + 4,
// and while it runs the 2 loader waves fetch the 4 rows tile i + 1 adds (the ring then holds
// exactly both tiles' rows). Every input pixel is loaded ONCE per strip instead of 9 x per tap,
// the weights once per workgroup, and one barrier per tile covers 9 taps x 2 k-steps of MFMAs.
//
// 4 MFMA waves (2 x 2: 112 pixels x 32 channels each) read the next tap's fragments behind the
// current tap's MFMAs (the interleave pinned by sched_group_barrier: with one MFMA wave per SIMD
// nothing else hides a read's latency) and store straight from the accumulators. Cold, ResNet50
// b128: 45 us vs 66 us for the best v2 tile (DESIGN §2 "Row-ring 3x3"). Phase stamps
// (dml_conv_rr_stamped, tools/rr_stamps.py) put the per-CU memory-instruction issue — row DMA
// and output stores, ~60 KiB per CU per tile — beside the MFMAs on a tile's critical path;
// moving the stores to the loader waves or into the MFMA stream (both measured, both slower:
// 53 / 52 us) did not take it off.
//
// K order: tap-major then channel, as v2 (Cin = 64 is one chunk). The launcher refuses anything
// but 3x3 / pad 1 / stride 1, Cin 64, Cout <= 64, W = Wo = 56, no split-K / segments.
//
// Reference compute: the Keras convolutions of models.py:48-69 (ResNet50).
#include "conv_shared.h"

namespace dml {
namespace rr {

using convk::lds_void;
using convk::wait_vmcnt;

constexpr int W56 = 56;                 // image width (= output width)
constexpr int TH = 4;                   // output rows per tile
constexpr int RING = 2 * TH + 2;        // image rows resident: a tile's 6 + the next tile's 4
constexpr int SLOT = 64;                // LDS rows per image row: zero column, 56 pixels, zero column, pad
constexpr int ROWB = 128;               // 64 channels of bf16
constexpr int WROWS = 9 * 64;           // weight LDS rows: [tap][cout]
constexpr int W_BYTES = WROWS * ROWB;   // 72 KiB
constexpr int RING_BYTES = RING * SLOT * ROWB;  // 80 KiB
constexpr int NC = 4, NL = 2, NT = (NC + NL) * 64;  // 4 MFMA waves (2 x 2) + 2 loader waves
constexpr int WTP = 112, WTC = 32, FJ = WTP / 16, FI = WTC / 16;
constexpr int LDS = W_BYTES + RING_BYTES;
static_assert(LDS <= 163840, "LDS");
constexpr int WPL = WROWS / 8 / NL;     // weight pieces (8 LDS rows) per loader lane
constexpr unsigned OOB = 0x80000000u;   // buffer offset past the range: the DMA writes zeros

__device__ __forceinline__ int swz(int row, int ch) { return row * ROWB + ((ch ^ (row & 7)) << 4); }

// phase timestamps (tools/rr_stamps.py; stamps == nullptr in every real launch): lane 0 of MFMA
// wave 0 writes s_memtime into its workgroup's 64-entry row of a debug buffer (vector stores)
#define RR_STAMP(who, k)                                                                                        \
  do {                                                                                                          \
    if (stamps && lane == 0) stamps[((long)blockIdx.x * 2 + (who)) * 64 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

template <bool RES>
__global__ __launch_bounds__(NT) void conv_rr_kernel(DmlConvArgs a, int strips, unsigned long long* stamps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const wl = smem;
  char* const ring = smem + W_BYTES;
  const int ntile = (a.Ho + TH - 1) / TH;
  const int b = blockIdx.x;
  const int n = b / strips, s = b - n * strips;
  const int t0 = s * ntile / strips, t1 = (s + 1) * ntile / strips;
  const int gbase = t0 * TH - 1;  // image row held by ring slot 0 at the strip's start
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int HW = a.H * a.W;

  if (wid >= NC) {
    // ================================ loader wave ================================
    const int lw = wid - NC;
    const int lrow = lane >> 3;                   // row within a 1-KiB piece
    const int lchunk = (lane & 7) ^ (lrow & 7);   // source-side swizzle (pieces start at rows % 8 == 0)
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
    // weights: LDS row t*64 + c <- packed row c, K offset t*64 (Cin = 64: one chunk per tap)
#pragma unroll 4
    for (int i = 0; i < WPL; ++i) {
      const int row = (lw + i * NL) * 8 + lrow;
      const int t = row >> 6, c = row & 63;
      const char* src = (const char*)a.w + ((long)c * a.Kpad + t * 64 + lchunk * 8) * 2;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(wl + (lw + i * NL) * 1024), 16, 0, 0);
    }
    // image rows [g0, g0 + cnt) of image n into their ring slots
    auto rows = [&](int g0, int cnt) __attribute__((always_inline)) {
      const int npiece = cnt * SLOT / 8;
      for (int p = lw; p < npiece; p += NL) {  // p, g, slot, col0: wave-uniform (the DMA's LDS base)
        const int g = g0 + p * 8 / SLOT, col0 = p * 8 % SLOT;
        const int slot = (g - gbase) % RING;
        const int iw = col0 + lrow - 1;            // LDS column c holds input column c - 1
        const bool ok = (unsigned)g < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const unsigned off = ok ? (unsigned)(((n * a.H + g) * a.W + iw) * a.ldx + lchunk * 8) * 2u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void*)(ring + (slot * SLOT + col0) * ROWB), 16, off, 0, 0,
                                                 0);
      }
    };
    if (t0 < t1) rows(t0 * TH - 1, TH + 2);
    for (int t = t0; t < t1; ++t) {
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // tile t's rows (and the weights) published; tile t-1 read
      if (t + 1 < t1) rows((t + 1) * TH + 1, TH);  // tile t+1's new rows: the slots tile t-1 alone used
    }
    return;
  }

  // ================================== MFMA wave ==================================
  const int wc = wid & 1, wp = wid >> 1;
  const int frow = lane & 15, fq = lane >> 4;
  if (wid == 0) RR_STAMP(0, 0);
  int ohl[FJ], col[FJ];
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int p = wp * WTP + j * 16 + frow;
    ohl[j] = p / W56;
    col[j] = p - ohl[j] * W56;  // LDS column of input pixel (ow - 1) = ow: the left zero column is 0
  }
  const int c0 = wc * WTC;
  float4 bv[FI];
  bool cok[FI];
#pragma unroll
  for (int i = 0; i < FI; ++i) {
    const int cc = c0 + i * 16 + fq * 4;
    cok[i] = cc < a.Cout;
    bv[i] = cok[i] ? *(const float4*)(a.bias + cc) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int t = t0; t < t1; ++t) {
    const int r0 = t * TH;
    const int m0 = n * HW + r0 * a.W;
    const int cnt = min(TH, a.Ho - r0) * a.W;
    f32x4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = (f32x4)(0.f);
    const int k = 1 + (t - t0) * 4;
    if (wid == 0) RR_STAMP(0, k);
    __builtin_amdgcn_s_barrier();
    if (wid == 0) RR_STAMP(0, k + 1);
    const int s0 = (r0 - 1 - gbase) % RING;
    int rb[3][FJ];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        int sl = s0 + ohl[j] + r;
        sl = sl >= RING ? sl - RING : sl;
        rb[r][j] = sl * SLOT + col[j];
      }
    bf16x8 fa[2][2][FI], fb[2][2][FJ];
    auto load = [&](int tap, int buf) __attribute__((always_inline)) {
      const int r = tap / 3, sx = tap - r * 3;
      const char* wt = wl + tap * 64 * ROWB;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + fq;
#pragma unroll
        for (int i = 0; i < FI; ++i) fa[buf][ks][i] = *(const bf16x8*)(wt + swz(c0 + i * 16 + frow, c));
#pragma unroll
        for (int j = 0; j < FJ; ++j) fb[buf][ks][j] = *(const bf16x8*)(ring + swz(rb[r][j] + sx, c));
      }
    };
    load(0, 0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap < 8) load(tap + 1, (tap + 1) & 1);
      const int cb = tap & 1;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
          for (int j = 0; j < FJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cb][ks][i], fb[cb][ks][j], acc[i][j], 0, 0, 0);
    }
    // the compiler otherwise reads each fragment just before its MFMA and waits on it (one MFMA
    // wave per SIMD: nothing hides that latency): pin the interleave — tap 0's reads, then per
    // tap one next-tap read after each of the first NR MFMAs
    constexpr int NR = 2 * (FI + FJ), NM = 2 * FI * FJ;
    __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap < 8) {
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
      }
    }
    if (wid == 0) RR_STAMP(0, k + 2);
    uint2 rv[RES ? FI : 1][RES ? FJ : 1];
    if constexpr (RES) {  // residual (no ResNet50 3x3 has one): loaded after the MFMAs, whose
      // fragment double buffers leave no registers to hold it across the taps
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int lp = wp * WTP + j * 16 + frow;
#pragma unroll
        for (int i = 0; i < FI; ++i)
          rv[i][j] = (lp < cnt && cok[i])
                         ? *(const uint2*)((const unsigned short*)a.res + (long)(m0 + lp) * a.ldr + c0 + i * 16 + fq * 4)
                         : make_uint2(0, 0);
      }
    }
    // ---- epilogue straight from the accumulators (lane: 4 channels of one pixel)
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int lp = wp * WTP + j * 16 + frow;
      if (lp >= cnt) continue;
      const long m = m0 + lp;
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        if (!cok[i]) continue;
        const int cc = c0 + i * 16 + fq * 4;
        float v[4] = {acc[i][j][0] + bv[i].x, acc[i][j][1] + bv[i].y, acc[i][j][2] + bv[i].z,
                      acc[i][j][3] + bv[i].w};
        if constexpr (RES) {
          v[0] += bf2f(rv[i][j].x & 0xffff); v[1] += bf2f(rv[i][j].x >> 16);
          v[2] += bf2f(rv[i][j].y & 0xffff); v[3] += bf2f(rv[i][j].y >> 16);
        }
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (a.out_f32)
          *(float4*)((float*)a.y + m * a.ldy + cc) = make_float4(v[0], v[1], v[2], v[3]);
        else
          *(uint2*)((unsigned short*)a.y + m * a.ldy + cc) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
    if (wid == 0) RR_STAMP(0, k + 3);
  }
}

}  // namespace rr

// ============================================================================================
// Generic row-ring family (cfg 160..): the stage-2 kernel's structure for any kh x kw, stride 1,
// 'same' or 'valid' padding, any width, any Cin (multiple of 8), Cout in chunks of COUT_WG.
//
// LDS: the workgroup's weight block [tap][channel group g][cout] and a ring of RING = 2 TH + kh - 1
// image rows, both in 64-B rows (32 channels of bf16): the ring is stored as CG channel-group
// PLANES of RING x SLOTP pixels (SLOTP = W + 2 pw rounded up to 16), so any Cin costs
// ceil(Cin / 32) planes instead of a power-of-two row (Cin 80: 3 planes, the last half zero; the
// DMA's range check writes the zeros). 64-B rows are XOR-swizzled by key(row) = (row >> 1) & 2
// on the chunk: a brute-force search over the ds_read_b128 lane groups (MI355X_MICROARCH LDS
// table) found this key conflict-free for 16 consecutive rows at ANY start offset - needed
// because a tap's 16-pixel fragment starts at an arbitrary column (the 128-B stage-2 kernel's
// row & 7 key has the same property; the {0,2,3,1} key of the BK32 tiles does not).
//
// Block b -> (strip, cout chunk) with the cout chunks of one strip consecutive on one XCD (they
// stream the same input rows: the second..last fetch them from that XCD's L2). A strip is a run of
// TH-row tiles of one image; the host picks TH (as large as the registers and the 160 KiB allow)
// and the strip count (grid >= the CU count). K order = tap-major then channel, as the packed
// weights. MFMA waves: WC x WP, each FI cout fragments x FJ pixel fragments (pixel fragment f of
// a tile goes to wave f % WP), fragments of the next (tap, g) step read behind the current
// step's MFMAs; stores straight from the accumulators (bias, ReLU, channel offset).
namespace rrg {

using convk::lds_void;
using convk::wait_vmcnt;
constexpr unsigned OOB = 0x80000000u;

__device__ __forceinline__ int key(int row) { return (row >> 1) & 2; }

struct Geo {
  int CG, SLOTP, RING, TH, strips, ncc, wbytes, plane, ntile, taps;
};

template <int WC, int WP, int FI, int FJ, int NL>
__global__ __launch_bounds__((WC * WP + NL) * 64) void conv_rrg_kernel(DmlConvArgs a, Geo g) {
  constexpr int NC = WC * WP;
  constexpr int COUT_WG = WC * FI * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const wl = smem;
  char* const ring = smem + g.wbytes;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int cc = L % g.ncc, sidx = L / g.ncc;
  const int n = sidx / g.strips, sp = sidx - n * g.strips;
  const int t0 = sp * g.ntile / g.strips, t1 = (sp + 1) * g.ntile / g.strips;
  const int TH = g.TH, RING = g.RING, SLOTP = g.SLOTP;
  const int gbase = t0 * TH - a.ph;  // image row held by ring slot 0 at the strip's start
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = cc * COUT_WG;

  if (wid >= NC) {
    // ================================ loader wave ================================
    const int lw = wid - NC;
    const int lrow = lane >> 2, lq = lane & 3;
    const int lchunk = lq ^ key(lrow);  // pieces start at rows % 16 == 0
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7ffffff0, 0x00020000);
    // weights: LDS row ((tap * CG + gg) * COUT_WG + cl) <- cout c0 + cl, K tap * Cin + gg * 32 + chunk * 8
    const int wpieces = g.taps * g.CG * COUT_WG / 16;
    for (int p = lw; p < wpieces; p += NL) {
      const int row = p * 16 + lrow;
      const int tg = row / COUT_WG, cl = row - tg * COUT_WG;
      const int tap = tg / g.CG, gg = tg - tap * g.CG;
      const int ch = gg * 32 + lchunk * 8, co = c0 + cl;
      const bool ok = ch < a.Cin && co < a.Cout;
      const unsigned off = ok ? (unsigned)(((long)co * a.Kpad + tap * a.Cin + ch) * 2) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_void*)(wl + p * 1024), 16, off, 0, 0, 0);
    }
    // image rows [r0, r0 + cnt) of image n into their ring slots, every channel-group plane
    const int ppr = SLOTP / 16;  // 1-KiB pieces per ring row and plane
    auto rows = [&](int r0, int cnt) __attribute__((always_inline)) {
      const int npiece = cnt * g.CG * ppr;
      for (int p = lw; p < npiece; p += NL) {  // wave-uniform decomposition
        const int rr = p / (g.CG * ppr), rem = p - rr * (g.CG * ppr);
        const int gg = rem / ppr, pc = rem - gg * ppr;
        const int gr = r0 + rr;
        const int slot = (gr - gbase) % RING;
        const int col = pc * 16 + lrow;  // LDS column c holds input column c - pw
        const int iw = col - a.pw, ch = gg * 32 + lchunk * 8;
        const bool ok = (unsigned)gr < (unsigned)a.H && (unsigned)iw < (unsigned)a.W && ch < a.Cin;
        const unsigned off = ok ? (unsigned)((((long)n * a.H + gr) * a.W + iw) * a.ldx + ch) * 2u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xrs, (lds_void*)(ring + gg * g.plane + (slot * SLOTP + pc * 16) * 64), 16, off, 0, 0, 0);
      }
    };
    if (t0 < t1) rows(gbase, TH + a.kh - 1);
    for (int t = t0; t < t1; ++t) {
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // tile t's rows (and the weights) published; tile t-1 read
      if (t + 1 < t1) rows((t + 1) * TH - a.ph + a.kh - 1, TH);  // the slots only tile t-1 used
    }
    return;
  }

  // ================================== MFMA wave ==================================
  const int wc = wid % WC, wp = wid / WC;
  const int frow = lane & 15, fq = lane >> 4;
  const int tpx = TH * a.Wo;  // pixels of a full tile
  int ohl[FJ], ow[FJ];
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    int p = (j * WP + wp) * 16 + frow;
    p = p < tpx ? p : 0;  // fragment rows past the tile: computed on pixel 0, never stored
    ohl[j] = p / a.Wo;
    ow[j] = p - ohl[j] * a.Wo;
  }
  const int cw = c0 + wc * FI * 16;  // this wave's first cout
  float4 bv[FI];
  bool cok[FI];
#pragma unroll
  for (int i = 0; i < FI; ++i) {
    const int ccx = cw + i * 16 + fq * 4;
    cok[i] = ccx < a.Cout;
    bv[i] = cok[i] ? *(const float4*)(a.bias + ccx) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // A fragment offsets: row base multiple of 16 -> the key is the lane's own
  const int aoff = (wc * FI * 16 + frow) * 64 + ((fq ^ key(frow)) << 4);
  const int nfrag_all = (tpx + 15) >> 4;
  const int nsteps = g.taps * g.CG;
  for (int t = t0; t < t1; ++t) {
    const int r0 = t * TH;
    const int rows_here = min(TH, a.Ho - r0);
    const int cnt = rows_here * a.Wo;
    f32x4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = (f32x4)(0.f);
    __builtin_amdgcn_s_barrier();
    const int s0 = ((t - t0) * TH) % RING;  // slot of input row r0 - ph
    int sl[FJ];                             // ring slot of tap row 0 per fragment
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      int v = s0 + ohl[j];
      sl[j] = v >= RING ? v - RING : v;
    }
    bf16x8 fa[2][FI], fb[2][FJ];
    // B fragment address of (r, s, gg) for fragment j
    auto boff = [&](int j, int r, int sx, int gg) __attribute__((always_inline)) {
      int v = sl[j] + r;
      v = v >= RING ? v - RING : v;
      const int P = v * SLOTP + ow[j] + sx;
      return gg * g.plane + P * 64 + ((fq ^ key(P)) << 4);
    };
    auto load = [&](int st, int buf) __attribute__((always_inline)) {
      const int tap = st / g.CG, gg = st - tap * g.CG;
      const int r = tap / a.kw, sx = tap - r * a.kw;
      const char* wt = wl + st * COUT_WG * 64 + aoff;
#pragma unroll
      for (int i = 0; i < FI; ++i) fa[buf][i] = *(const bf16x8*)(wt + i * 16 * 64);
#pragma unroll
      for (int j = 0; j < FJ; ++j) fb[buf][j] = *(const bf16x8*)(ring + boff(j, r, sx, gg));
    };
    auto mfma = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        if (j * WP + wp >= nfrag_all) continue;  // wave-uniform
#pragma unroll
        for (int i = 0; i < FI; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[buf][i], fb[buf][j], acc[i][j], 0, 0, 0);
      }
    };
    load(0, 0);
    int st = 0;
    for (; st + 2 <= nsteps; st += 2) {
      load(st + 1, 1);
      mfma(0);
      if (st + 2 < nsteps) load(st + 2, 0);
      mfma(1);
    }
    if (st < nsteps) mfma(0);
    // ---- epilogue straight from the accumulators (lane: 4 channels of one pixel)
    const long m0 = ((long)n * a.Ho + r0) * a.Wo;
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int lp = (j * WP + wp) * 16 + frow;
      if (lp >= cnt) continue;
      const long m = m0 + lp;
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        if (!cok[i]) continue;
        const int ccx = cw + i * 16 + fq * 4;
        float v[4] = {acc[i][j][0] + bv[i].x, acc[i][j][1] + bv[i].y, acc[i][j][2] + bv[i].z,
                      acc[i][j][3] + bv[i].w};
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        *(uint2*)((unsigned short*)a.y + m * a.ldy + ccx) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
  }
}

}  // namespace rrg
}  // namespace dml

static bool rr_fits(const DmlConvArgs* a) {
  const int dh = a->dh > 0 ? a->dh : 1, dw = a->dw > 0 ? a->dw : 1;
  return a->kh == 3 && a->kw == 3 && a->ph == 1 && a->pw == 1 && a->sh == 1 && a->sw == 1 && dh == 1 && dw == 1 &&
         a->Cin == 64 && a->Cout <= 64 && a->W == dml::rr::W56 && a->Wo == dml::rr::W56 && a->Ho == a->H &&
         a->ksplit <= 1 && a->nseg == 0 && a->rsub <= 1 && a->ldx % 8 == 0 && a->Kpad >= 9 * 64;
}

extern "C" int dml_conv_rr_init(void) {
  using namespace dml::rr;
  const int rc =
      (int)hipFuncSetAttribute((const void*)conv_rr_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS) |
      (int)hipFuncSetAttribute((const void*)conv_rr_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
  if (rc) dml_set_error("dml_conv_rr_init: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  return rc ? -1 : 0;
}

extern "C" int dml_conv_rr_fits(const DmlConvArgs* a) { return rr_fits(a) ? 1 : 0; }

// cfg 150 / 151 / 152: 2 / 1 / 4 strips per image (ResNet50 b128 at 2: 256 workgroups).
// dml_conv_rr_stamped: the same launch writing phase timestamps (grid x 128 uint64) to `stamps`
extern "C" int dml_conv_rr_stamped(const DmlConvArgs* a, int cfg, void* stamps, hipStream_t s) {
  using namespace dml::rr;
  if (!rr_fits(a) || cfg < 150 || cfg > 152) {
    dml_set_error("dml_conv_rr: needs 3x3 pad 1 stride 1, Cin 64, Cout <= 64, width 56, no split-K / segments");
    return -1;
  }
  const int ntile = (a->Ho + TH - 1) / TH;
  const int strips = cfg == 151 ? 1 : (cfg == 150 ? 2 : 4);
  const int sp = strips < ntile ? strips : ntile;
  const unsigned grid = (unsigned)(a->N * sp);
  unsigned long long* st = (unsigned long long*)stamps;
  if (a->res)
    hipLaunchKernelGGL(conv_rr_kernel<true>, dim3(grid), dim3(NT), LDS, s, *a, sp, st);
  else
    hipLaunchKernelGGL(conv_rr_kernel<false>, dim3(grid), dim3(NT), LDS, s, *a, sp, st);
  DML_CHECK_LAUNCH();
  return 0;
}

extern "C" int dml_conv_rr(const DmlConvArgs* a, int cfg, hipStream_t s) { return dml_conv_rr_stamped(a, cfg, nullptr, s); }

// ------------------------------------------------------------------ generic row-ring family --
// id, WC, WP, FI, FJ, NL: cout chunk WC x FI x 16, at most WP x FJ x 16 pixels per tile.
// cfg = 160 + 2 * instance + strip mode (0: grid ~ one workgroup per CU, 1: twice that).
#define DML_RRG_CFGS(X)                                                  \
  X(0, 2, 2, 2, 7, 2)   /* 64 couts, <= 224 px (the stage-2 layout) */   \
  X(1, 1, 4, 2, 3, 2)   /* 32 couts, <= 192 px */                        \
  X(2, 1, 4, 3, 2, 2)   /* 48 couts, <= 128 px */                        \
  X(3, 1, 4, 4, 2, 2)   /* 64 couts, <= 128 px */                        \
  X(4, 2, 2, 1, 5, 2)   /* 32 couts, <= 160 px */                        \
  X(5, 1, 4, 2, 4, 2)   /* 32 couts, <= 256 px */                        \
  X(6, 2, 4, 2, 2, 2)   /* 64 couts, <= 128 px, 8 MFMA waves */          \
  X(7, 1, 8, 2, 2, 2)   /* 32 couts, <= 256 px, 8 MFMA waves */          \
  X(8, 1, 4, 3, 3, 2)   /* 48 couts, <= 192 px */
#define DML_RRG_N 9

static const int kRrgLds = 163840;

struct RrgShape {
  int WC, WP, FI, FJ, NL;
};
static RrgShape rrg_shape(int inst) {
  switch (inst) {
#define DML_SH(i, WC, WP, FI, FJ, NL) \
  case i: return RrgShape{WC, WP, FI, FJ, NL};
    DML_RRG_CFGS(DML_SH)
#undef DML_SH
    default: return RrgShape{0, 0, 0, 0, 0};
  }
}

// geometry of a launch (false: this config cannot run the conv)
static bool rrg_geo(const DmlConvArgs* a, int cfg, dml::rrg::Geo* g, int* lds, int* nthreads) {
  if (cfg < 160 || cfg >= 160 + 2 * DML_RRG_N) return false;
  const RrgShape sh = rrg_shape((cfg - 160) / 2);
  const int smode = (cfg - 160) % 2;
  const int dh = a->dh > 0 ? a->dh : 1, dw = a->dw > 0 ? a->dw : 1;
  if (a->sh != 1 || a->sw != 1 || dh != 1 || dw != 1 || a->res || a->out_f32 || a->nseg || a->ksplit > 1 ||
      a->rsub > 1 || a->Cin % 8 || a->ldx % 8 || a->Cout % 4 || a->ldy % 4 || a->kh < 1 || a->kw < 1)
    return false;
  const bool same = a->ph == (a->kh - 1) / 2 && a->pw == (a->kw - 1) / 2 && (a->kh & 1) && (a->kw & 1);
  const bool valid = a->ph == 0 && a->pw == 0;
  if (!same && !valid) return false;
  if (a->Ho != a->H + 2 * a->ph - a->kh + 1 || a->Wo != a->W + 2 * a->pw - a->kw + 1 || a->Ho < 1 || a->Wo < 1)
    return false;
  const int taps = a->kh * a->kw;
  if (a->Kpad < taps * a->Cin) return false;
  if ((long)a->N * a->H * a->W * a->ldx * 2 >= 0x7ffffff0L || (long)a->Kpad * ((a->Cout + 255) / 256 * 256) * 2 >= 0x7ffffff0L)
    return false;  // 32-bit buffer offsets
  const int cout_wg = sh.WC * sh.FI * 16;
  g->CG = (a->Cin + 31) / 32;
  g->SLOTP = (a->W + 2 * a->pw + 15) / 16 * 16;
  g->taps = taps;
  g->wbytes = taps * g->CG * cout_wg * 64;
  const int rowb = g->SLOTP * g->CG * 64;  // one ring row, every plane
  const int th_reg = sh.WP * sh.FJ * 16 / a->Wo;
  const int room = kRrgLds - g->wbytes;
  if (room <= 0) return false;
  const int th_lds = (room / rowb - (a->kh - 1)) / 2;
  int th = th_reg < th_lds ? th_reg : th_lds;
  th = th < a->Ho ? th : a->Ho;
  if (th < 1) return false;
  g->TH = th;
  g->RING = 2 * th + a->kh - 1;
  g->plane = g->RING * g->SLOTP * 64;
  g->ncc = (a->Cout + cout_wg - 1) / cout_wg;
  g->ntile = (a->Ho + th - 1) / th;
  const int target = 256 * (smode + 1);
  int strips = (target + a->N * g->ncc - 1) / (a->N * g->ncc);
  strips = strips < 1 ? 1 : (strips > g->ntile ? g->ntile : strips);
  g->strips = strips;
  *lds = g->wbytes + g->CG * g->plane;
  *nthreads = (sh.WC * sh.WP + sh.NL) * 64;
  return *lds <= kRrgLds;
}

extern "C" int dml_conv_rrg_fits(const DmlConvArgs* a, int cfg) {
  dml::rrg::Geo g;
  int lds, nt;
  return rrg_geo(a, cfg, &g, &lds, &nt) ? 1 : 0;
}

// cout chunk of a generic row-ring config (0: not one)
extern "C" int dml_conv_rrg_bn(int cfg) {
  if (cfg < 160 || cfg >= 160 + 2 * DML_RRG_N) return 0;
  const RrgShape sh = rrg_shape((cfg - 160) / 2);
  return sh.WC * sh.FI * 16;
}

// the launch's geometry for tests / tools: {CG, SLOTP, RING, TH, strips, ncc, wbytes, plane, ntile, taps, lds, grid}
extern "C" int dml_conv_rrg_geometry(const DmlConvArgs* a, int cfg, int* out12) {
  dml::rrg::Geo g;
  int lds, nt;
  if (!rrg_geo(a, cfg, &g, &lds, &nt)) return -1;
  const int v[12] = {g.CG, g.SLOTP, g.RING, g.TH, g.strips, g.ncc, g.wbytes, g.plane, g.ntile, g.taps, lds,
                     a->N * g.strips * g.ncc};
  for (int i = 0; i < 12; ++i) out12[i] = v[i];
  return 0;
}

extern "C" int dml_conv_rrg_init(void) {
  using namespace dml::rrg;
  int rc = 0;
#define DML_SET(i, WC, WP, FI, FJ, NL)                                                                          \
  rc |= (int)hipFuncSetAttribute((const void*)conv_rrg_kernel<WC, WP, FI, FJ, NL>,                              \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, kRrgLds);
  DML_RRG_CFGS(DML_SET)
#undef DML_SET
  if (rc) dml_set_error("dml_conv_rrg_init: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  return rc ? -1 : 0;
}

extern "C" int dml_conv_rrg(const DmlConvArgs* a, int cfg, hipStream_t s) {
  using namespace dml::rrg;
  Geo g;
  int lds, nt;
  if (!rrg_geo(a, cfg, &g, &lds, &nt)) {
    dml_set_error("dml_conv_rrg: needs stride 1, 'same' (odd kernel) or 'valid' padding, Cin % 8 == 0, no residual / "
                  "fp32 output / split-K / segments, and a weight block + 2-tile row ring within 160 KiB");
    return -1;
  }
  const unsigned grid = (unsigned)(a->N * g.strips * g.ncc);
  switch ((cfg - 160) / 2) {
#define DML_CASE(i, WC, WP, FI, FJ, NL)                                                     \
  case i:                                                                                  \
    hipLaunchKernelGGL((conv_rrg_kernel<WC, WP, FI, FJ, NL>), dim3(grid), dim3(nt), lds, s, *a, g); \
    break;
    DML_RRG_CFGS(DML_CASE)
#undef DML_CASE
    default: dml_set_error("dml_conv_rrg: bad cfg"); return -1;
  }
  DML_CHECK_LAUNCH();
  return 0;
}
