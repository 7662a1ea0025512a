// conv_igemm_pt.hip — patch-stationary warp-specialised implicit-GEMM convolution for
// stride-1 kernels (3x3, 5x5, 1x7, 7x1, 1x3, 3x1; gfx950).
//
// Why: the implicit-GEMM tiles (conv_igemm_v2.hip, conv_igemm_ws.hip) DMA a fresh BM x BK
// activation block into LDS for EVERY (tap, channel chunk) K tile, so a 3x3 conv moves ~9x
// its input through L2 -> LDS, and the r4 phase probes put the 3x3 layers on that
// operand stream, not on the matrix cores (per CU, an L2-served LDS fill runs at ~70 GB/s,
// MI355X_MICROARCH.md "Indexed rows": a 256 x 128 tile's 48 KiB per K tile take longer than
// its 4.2 MFLOP of MFMAs).
//
// What: an M tile is a block of WHOLE output rows of one image (TH x Wo pixels, TH =
// BM / Wo), or TI = BM / (Ho*Wo) whole images when an image has fewer than BM pixels, so its
// input footprint is one rectangular patch per image — (TH + kh - 1) x (Wo + kw - 1) pixels,
// image borders zero-filled by the buffer range check. The loader waves DMA that patch ONCE
// per BK-channel chunk into one of two LDS patch buffers (the next chunk's patch lands while
// the current chunk's taps run) and stream only the weights through the K-tile ring. The MFMA
// waves read each tap's activation fragments from the patch at a per-tap row offset
// (r * PW + s): per K tile the CU fills BN weight rows plus ~PR / taps patch rows instead of
// BN + BM rows (a 256 x 128 tile at 3x3: ~21 1-KiB pieces instead of 48).
//
// K order: chunk-major, then tap (v2: tap-major) — numerically the same fp32 sums in another
// order, so outputs match the fp32 reference, not v2 bit for bit. Requires stride 1,
// dilation 1, Cin % BK == 0 (a chunk never straddles a tap: the v2 weight packing
// [Cout][tap][Cin] then gives every (tap, chunk) weight row contiguously), no split-K; the
// launcher refuses anything else (the tuner then skips the config).
//
// Reference compute: the Keras convolutions of models.py:23-44 / 48-69.
#include "conv_shared.h"

namespace dml {
namespace pt {

using convk::lds_void;
using convk::wait_vmcnt;

constexpr int lds_occupancy(int a, int b) { return 163840 / (a > b ? a : b); }

template <int BM, int BN, int WM, int WN, int NL_, int STAGES, int BK_, int PRMAX, int NPB = 2>
struct Cfg {
  static constexpr int NC = WM * WN;          // MFMA waves
  static constexpr int NL = NL_;              // loader waves
  static constexpr int NT = (NC + NL) * 64;
  static constexpr int NTC = NC * 64;
  static constexpr int WTP = BM / WM;
  static constexpr int WTC = BN / WN;
  static constexpr int FJ = WTP / 16;
  static constexpr int FI = WTC / 16;
  static constexpr int BK = BK_;
  using R = convk::Rows<BK>;
  static constexpr int ROWB = R::ROWB;
  static constexpr int RP = R::RP;
  static constexpr int WI = BN / RP / NL;                 // weight pieces per loader lane per K tile
  static constexpr int PP = (PRMAX + RP * NL - 1) / (RP * NL) * NL;  // patch pieces per chunk (whole rounds)
  static constexpr int PI = PP / NL;                      // patch pieces per loader lane per chunk
  static constexpr int PROWS = PP * RP;                   // patch rows (>= PRMAX: dummy pieces land here)
  static constexpr int WSTAGE = BN * ROWB;
  static constexpr int PATCH = PROWS * ROWB;
  static constexpr int PIPE_BYTES = STAGES * WSTAGE + NPB * PATCH;  // NPB 1: single-chunk convs only
  static constexpr int CROW = BN * 4 + 16;
  static constexpr bool EP_OK2 = (BM / 2) % 16 == 0 && ((BM * BN / 8) / NTC) % 2 == 0;
  static constexpr bool EP_OK4 = (BM / 4) % 16 == 0 && ((BM * BN / 8) / NTC) % 4 == 0;
  static constexpr int EP_MAX = EP_OK4 ? 4 : (EP_OK2 ? 2 : 1);
  static constexpr int OCC_BEST = lds_occupancy(PIPE_BYTES, (BM / EP_MAX) * CROW);
  static constexpr int EP = lds_occupancy(PIPE_BYTES, BM * CROW) >= OCC_BEST ? 1
                          : (EP_OK2 && lds_occupancy(PIPE_BYTES, (BM / 2) * CROW) >= OCC_BEST) ? 2 : EP_MAX;
  static constexpr int EPI_BYTES = (BM / EP) * CROW;
  static constexpr int LDS = PIPE_BYTES > EPI_BYTES ? PIPE_BYTES : EPI_BYTES;
  static_assert(WI >= 1 && BN % (RP * NL) == 0, "weight rows must split evenly over the loaders");
  static_assert(FI >= 1 && FJ >= 1 && WTP % 16 == 0 && WTC % 16 == 0, "wave tile");
  static_assert(STAGES >= 2 && (STAGES - 2) * WI + PI < 64, "vmcnt range");
  static_assert(LDS <= 163840, "LDS");
};

// M-tile geometry (identical in every thread; host launcher: pt_geometry)
struct Geo {
  int TI, TH, PH, PW, PR, tpi, mt;
};

__host__ __device__ inline Geo pt_geometry(const DmlConvArgs& a, int BM) {
  Geo g;
  const int HoWo = a.Ho * a.Wo;
  if (HoWo <= BM) {
    g.TI = BM / HoWo;
    g.TH = a.Ho;
    g.tpi = 1;
    g.mt = (a.N + g.TI - 1) / g.TI;
  } else {
    g.TI = 1;
    g.TH = a.Wo > 0 ? BM / a.Wo : 0;
    g.tpi = g.TH > 0 ? (a.Ho + g.TH - 1) / g.TH : 0;
    g.mt = a.N * g.tpi;
  }
  g.PH = g.TH + a.kh - 1;
  g.PW = a.Wo + a.kw - 1;
  g.PR = g.TI * g.PH * g.PW;
  return g;
}

template <int BM, int BN, int WM, int WN, int NL, int STAGES, bool RES, int BK, bool LATE, int PRMAX, int NPB>
__device__ __forceinline__ void conv_pt_tile(const DmlConvArgs& a, int Lb) {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK, PRMAX, NPB>;
  using RW = typename T::R;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const patch0 = smem + STAGES * T::WSTAGE;

  const Geo g = pt_geometry(a, BM);
  const int ntc = (a.Cout + BN - 1) / BN;
  const int tc = Lb % ntc, tm = Lb / ntc;
  const int c0 = tc * BN;
  const int HoWo = a.Ho * a.Wo;
  int n0, oh0, cnt;
  if (g.TI > 1 || g.tpi == 1) {
    n0 = tm * g.TI;
    oh0 = 0;
    cnt = min(g.TI, a.N - n0) * HoWo;
  } else {
    n0 = tm / g.tpi;
    oh0 = (tm - n0 * g.tpi) * g.TH;
    cnt = min(g.TH, a.Ho - oh0) * a.Wo;
  }
  const int m0 = n0 * HoWo + oh0 * a.Wo;
  const int taps = a.kh * a.kw;
  const int nchunk = a.Cin / BK;
  const int nk = taps * nchunk;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

  f32x4 acc[T::FI][T::FJ];
#pragma unroll
  for (int i = 0; i < T::FI; ++i)
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) acc[i][j] = (f32x4)(0.f);
  convk::Epilogue<BM, BN, T::NTC, RES, T::EP, LATE, true> epi;
  const int wc = wid % WN, wp = wid / WN;

  if (wid >= T::NC) {
    // ======================= loader wave =======================
    const int lw = wid - T::NC;
    const int lrow = RW::lane_row(lane);
    const int lchunk = RW::lane_chunk(lane);
    const unsigned OOB = 0x80000000u;
    // this lane's patch pixels (pieces lw, lw + NL, ...): element offset of its 8 channels of
    // chunk 0, or -1 (outside the image / a dummy row past the patch)
    int poff[T::PI];
    const int PHW = g.PH * g.PW;
#pragma unroll
    for (int i = 0; i < T::PI; ++i) {
      const int row = (lw + i * NL) * T::RP + lrow;
      const int ti = row / PHW;
      const int rem = row - ti * PHW;
      const int ph = rem / g.PW;
      const int pw = rem - ph * g.PW;
      const int n = n0 + ti, ih = oh0 - a.ph + ph, iw = pw - a.pw;
      const bool ok = row < g.PR && n < a.N && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      poff[i] = ok ? ((n * a.H + ih) * a.W + iw) * a.ldx + lchunk * 8 : -1;
    }
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
    const char* wrow = (const char*)a.w + ((long)(c0 + lw * T::WI * RW::RP + lrow) * a.Kpad + lchunk * 8) * 2;
    const long wstep_row = (long)RW::RP * a.Kpad * 2;

    auto issue_w = [&](int kt) {
      const int cb = kt / taps, t = kt - cb * taps;
      const long koff = ((long)t * a.Cin + (long)cb * BK) * 2;
      char* sw = smem + (kt % STAGES) * T::WSTAGE;
#pragma unroll
      for (int j = 0; j < T::WI; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(wrow + j * wstep_row + koff),
                                         (lds_void*)(sw + (lw * T::WI + j) * 1024), 16, 0, 0);
    };
    auto issue_p = [&](int cb) {
      char* dst = patch0 + (NPB > 1 ? (cb & 1) : 0) * T::PATCH;
#pragma unroll
      for (int i = 0; i < T::PI; ++i) {
        const unsigned off = poff[i] >= 0 ? (unsigned)(poff[i] + cb * BK) * 2u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void*)(dst + (lw + i * NL) * 1024), 16, off, 0, 0, 0);
      }
    };

    // issue stream: P0, W0 .. W(S-2); then per iteration kt (after barrier kt): P(cb+1) when kt
    // opens chunk cb (its buffer was last read by chunk cb-1, finished before this barrier),
    // then W(kt+S-1). P(c) precedes W(c*taps) in issue order when taps >= S-1 (the launcher
    // requires it), so the wait for W(kt) covers the patch of kt's chunk.
    issue_p(0);
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nk) issue_w(s);
    int ip = -(1 << 20);  // iteration of the last patch issue
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + STAGES - 2 < nk) {
        if (ip >= kt - STAGES + 2) wait_vmcnt<(STAGES - 2) * T::WI + T::PI>();
        else wait_vmcnt<(STAGES - 2) * T::WI>();
      } else {
        wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();  // K tile kt (and its chunk's patch) published
      const int cb = kt / taps;
      if (NPB > 1 && kt == cb * taps && cb + 1 < nchunk) {
        issue_p(cb + 1);
        ip = kt;
      }
      if (kt + STAGES - 1 < nk) issue_w(kt + STAGES - 1);
    }
  } else {
    // ======================= MFMA wave =======================
    epi.prefetch(a, m0, c0, m0 + cnt, tid);
    const int frow = lane & 15, fq = lane >> 4;
    constexpr int KSM = BK / 32;
    // patch row of each of this lane's pixel fragments (tap (0, 0)); rows past the tile read
    // patch row 0 (computed, never stored)
    int pb[T::FJ];
    const int TW = g.TH * a.Wo;
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) {
      const int r = wp * T::WTP + j * 16 + frow;
      const int ti = r / TW;
      const int rem = r - ti * TW;
      const int ohl = rem / a.Wo;
      const int ow = rem - ohl * a.Wo;
      pb[j] = r < cnt ? (ti * g.PH + ohl) * g.PW + ow : 0;
    }
    for (int kt = 0; kt < nk; ++kt) {
      __builtin_amdgcn_s_barrier();  // tile kt landed; stage kt-1 free for the refill
      const int cb = kt / taps, t = kt - cb * taps;
      const int tr = t / a.kw;
      const int toff = tr * g.PW + (t - tr * a.kw);
      const char* sw = smem + (kt % STAGES) * T::WSTAGE;
      const char* sx = patch0 + (NPB > 1 ? (cb & 1) : 0) * T::PATCH;
      bf16x8 fa[KSM][T::FI], fb[KSM][T::FJ];
#pragma unroll
      for (int ks = 0; ks < KSM; ++ks) {
        const int ch = ks * 4 + fq;
#pragma unroll
        for (int i = 0; i < T::FI; ++i) fa[ks][i] = *(const bf16x8*)(sw + RW::off(wc * T::WTC + i * 16 + frow, ch));
#pragma unroll
        for (int j = 0; j < T::FJ; ++j) fb[ks][j] = *(const bf16x8*)(sx + RW::off(pb[j] + toff, ch));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < KSM; ++ks)
#pragma unroll
        for (int i = 0; i < T::FI; ++i)
#pragma unroll
          for (int j = 0; j < T::FJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  epi.template store<16, T::FI, T::FJ, T::WTP, T::WTC>(a, smem, acc, wp, wc, lane, tid, wid < T::NC);
}

template <int BM, int BN, int WM, int WN, int NL, int STAGES, bool RES, int BK, bool LATE, int W, int PRMAX, int NPB>
__global__ __launch_bounds__((WM * WN + NL) * 64, W) void conv_pt_kernel(DmlConvArgs a) {
  conv_pt_tile<BM, BN, WM, WN, NL, STAGES, RES, BK, LATE, PRMAX, NPB>(a, xcd_remap(blockIdx.x, gridDim.x));
}

// host: can this config run this conv?
template <int BM, int BN, int NL, int STAGES, int BK, int PRMAX, int WM, int WN, int NPB>
static bool fits(const DmlConvArgs* a) {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK, PRMAX, NPB>;
  const int dh = a->dh > 0 ? a->dh : 1, dw = a->dw > 0 ? a->dw : 1;
  if (a->sh != 1 || a->sw != 1 || dh != 1 || dw != 1 || a->ksplit > 1) return false;
  if (a->Cin % BK || a->ldx % 8 || a->Wo > BM || a->Kpad < a->kh * a->kw * a->Cin) return false;
  if (a->kh * a->kw < STAGES - 1 && a->Cin / BK > 1) return false;  // patch issue order (see the loaders)
  if (NPB == 1 && a->Cin != BK) return false;                        // one patch buffer: one chunk
  const Geo g = pt_geometry(*a, BM);
  return g.TH >= 1 && g.PR <= T::PROWS && g.mt > 0;
}

template <int BM, int BN, int WM, int WN, int NL, int STAGES, int BK, bool LATE, int W, int PRMAX, int NPB>
static int launch(const DmlConvArgs* a, hipStream_t s) {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK, PRMAX, NPB>;
  if (!fits<BM, BN, NL, STAGES, BK, PRMAX, WM, WN, NPB>(a)) {
    dml_set_error("dml_conv_pt: needs stride 1, dilation 1, Cin % BK == 0, no split-K, Wo <= BM and a patch "
                  "that fits the config");
    return -1;
  }
  const Geo g = pt_geometry(*a, BM);
  const long tiles = (long)g.mt * ((a->Cout + BN - 1) / BN);
  if (a->res)
    hipLaunchKernelGGL((conv_pt_kernel<BM, BN, WM, WN, NL, STAGES, true, BK, LATE, W, PRMAX, NPB>),
                       dim3((unsigned)tiles), dim3(T::NT), T::LDS, s, *a);
  else
    hipLaunchKernelGGL((conv_pt_kernel<BM, BN, WM, WN, NL, STAGES, false, BK, false, W, PRMAX, NPB>),
                       dim3((unsigned)tiles), dim3(T::NT), T::LDS, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN, int NL, int STAGES, int BK, bool LATE, int W, int PRMAX, int NPB>
static int set_attr() {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK, PRMAX, NPB>;
  return (int)hipFuncSetAttribute(
             (const void*)conv_pt_kernel<BM, BN, WM, WN, NL, STAGES, true, BK, LATE, W, PRMAX, NPB>,
             hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS) |
         (int)hipFuncSetAttribute(
             (const void*)conv_pt_kernel<BM, BN, WM, WN, NL, STAGES, false, BK, false, W, PRMAX, NPB>,
             hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS);
}

}  // namespace pt
}  // namespace dml

// Patch-stationary tile configurations: id, BM, BN, WM x WN MFMA waves, NL loader waves,
// weight-ring STAGES, BK, RL (residual loaded in the epilogue), W (min waves/SIMD hint),
// PRMAX (patch rows per chunk), NPB (patch buffers: 2 = the next chunk's patch loads during
// this chunk's taps; 1 = Cin == BK only, half the LDS). Ids 140..159 are part of the tuner ABI (ops/tuning.py
// PT_CFGS), validated by dml_conv (conv_dispatch.hip).
#define DML_PT_TILES(X)                                                                             \
  X(140, 256, 128, 4, 2, 4, 3, 64, 1, 1, 416, 2) /* 8 (64x64) + 4 loaders, 152 KiB */                \
  X(141, 256, 64, 4, 1, 4, 3, 64, 0, 1, 416, 2)  /* 4 (64x64) + 4, 128 KiB */                         \
  X(142, 128, 128, 2, 2, 2, 3, 64, 0, 1, 240, 2) /* 4 + 2, 108 KiB */                                 \
  X(143, 128, 64, 2, 2, 2, 3, 64, 0, 1, 240, 2)  /* 4 (64x32) + 2, 84 KiB */                          \
  /* one patch buffer (single-chunk convs, Cin == 64): 2-3 workgroups per CU */                      \
  X(144, 256, 64, 4, 1, 2, 3, 64, 0, 3, 416, 1)  /* 4 (64x64) + 2, 76 KiB: 2 WG/CU */                 \
  X(145, 128, 64, 2, 2, 2, 3, 64, 0, 4, 240, 1)  /* 4 (64x32) + 2, 54 KiB: 3 WG/CU */                 \
  X(146, 128, 128, 2, 2, 2, 3, 64, 0, 2, 240, 1) /* 4 (64x64) + 2, 78 KiB: 2 WG/CU */                 \
  /* deeper weight rings (more operand bytes in flight per CU): smaller patches */                    \
  X(147, 256, 128, 4, 2, 4, 6, 64, 1, 1, 256, 2) /* 14x14 and 7x7 (TI 1 / 3 ... ), 160 KiB */        \
  X(148, 256, 128, 4, 2, 4, 4, 64, 1, 1, 352, 2) /* 56 / 28 / 14 rows, 152 KiB */                     \
  X(149, 256, 128, 4, 2, 4, 8, 32, 1, 1, 416, 2) /* BK 32: 8-stage ring, 116 KiB */

extern "C" int dml_conv_pt_init(void) {
  using namespace dml::pt;
  int rc = 0;
#define DML_SET(id, BM, BN, WM, WN, NL, ST, BK, RL, W, PR, NPB) rc |= set_attr<BM, BN, WM, WN, NL, ST, BK, RL, W, PR, NPB>();
  DML_PT_TILES(DML_SET)
#undef DML_SET
  if (rc) dml_set_error("dml_conv_pt_init: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  return rc ? -1 : 0;
}

extern "C" int dml_conv_pt(const DmlConvArgs* a, int cfg, hipStream_t s) {
  using namespace dml::pt;
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, NL, ST, BK, RL, W, PR, NPB) \
  case id: return launch<BM, BN, WM, WN, NL, ST, BK, RL, W, PR, NPB>(a, s);
    DML_PT_TILES(DML_CASE)
#undef DML_CASE
    default: dml_set_error("dml_conv_pt: bad cfg"); return -1;
  }
}

extern "C" int dml_conv_pt_bn(int cfg) {
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, NL, ST, BK, RL, W, PR, NPB) \
  case id: return BN;
    DML_PT_TILES(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}

// 1 if config `cfg` can run conv `a` (the tuner's candidate filter); 0 otherwise
extern "C" int dml_conv_pt_fits(const DmlConvArgs* a, int cfg) {
  using namespace dml::pt;
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, NL, ST, BK, RL, W, PR, NPB) \
  case id: return fits<BM, BN, NL, ST, BK, PR, WM, WN, NPB>(a) ? 1 : 0;
    DML_PT_TILES(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}
