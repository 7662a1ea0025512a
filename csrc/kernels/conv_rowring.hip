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
