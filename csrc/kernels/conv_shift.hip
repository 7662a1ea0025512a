// conv_shift.hip — shifted-pixel MFMA convolution for stride-1 "same" convs
// (ResNet50's 3x3 bottleneck convs; InceptionV3's 3x3 / 1x7 / 7x1 / 1x3 / 3x1).
//
// Why: the implicit-GEMM kernel (conv_igemm_v2.hip) fetches its activation
// operand per K tile, i.e. every input row once PER TAP: a 3x3 layer moves ~9x
// its input through L2 -> LDS, and on the 256x128 tile the activation side is
// 2/3 of all L2 -> LDS bytes (the stride-1 3x3s run at 27-28 % of
// bf16 peak, L2-fill bound).
//
// Observation: with stride 1, dilation 1 and "same" padding (ph = (kh-1)/2,
// pw = (kw-1)/2, Ho = H, Wo = W), output pixel m (flat NHW index) reads, at tap
// (r, s), flat input pixel m + (r - ph) * W + (s - pw) — a pure SHIFT in flat
// pixel space whenever the tap is inside the image. So a tile of BM consecutive
// output pixels reads, over all taps, one CONTIGUOUS span of input pixels:
//     [m0 - (ph*W + pw), m0 + BM + (ph*W + pw))          ("halo", HR rows)
// per channel chunk. The kernel loads that span into LDS ONCE per BK-channel
// chunk (LDS-DMA, hardware zero fill outside [0, M)), and runs every tap as an
// MFMA pass over the same halo with a per-lane row = tile pixel + r*W + s.
// A lane whose tap falls outside its image (row wrap, top/bottom padding, or
// the neighbouring image in flat space) reads a dedicated all-zero LDS row
// instead: one compare-select per fragment and tap, no padded copy of the input.
// Only the weight panel streams per tap (W column t*Cin + chunk, the same packed
// [Coutp][Kpad] layout as the implicit GEMM: k = (r*kw + s)*Cin + c).
//
// L2 -> LDS bytes per MFMA, 256x128 tile, 3x3: implicit GEMM (256 + 128) rows
// per tap-chunk; here 128 weight rows per tap-chunk + (256 + 2W + 2)/9 halo
// rows: 2.4-2.7x fewer.
//
// Pipeline: halo double-buffered across channel chunks (chunk c+1's halo is
// issued at the first tap of chunk c), weight panels in a STAGES-deep ring, one
// raw s_barrier per (chunk, tap) iteration with counted vmcnt waits (the halo
// DMA's count is included exactly when it is younger than the awaited panel).
// Epilogue: the implicit GEMM's (bias, residual, ReLU, segments, NHWC 16-B
// stores), staged through LDS.
#include "conv_shared.h"

namespace dml {
namespace shift {

using convk::lds_void;
using convk::wait_vmcnt;

constexpr int occ(int bytes) { return 163840 / bytes; }

template <int BM, int BN, int WM, int WN, int STAGES, int BK, int HALO>
struct Cfg {
  static constexpr int NW = WM * WN, NT = NW * 64;
  static constexpr int WTP = BM / WM, WTC = BN / WN;  // pixels / channels per wave
  static constexpr int FJ = WTP / 16, FI = WTC / 16;  // 16x16 fragments
  using R = convk::Rows<BK>;
  static constexpr int ROWB = R::ROWB;
  static constexpr int XH = HALO / (R::RP * NW);      // halo DMA instructions per wave
  static constexpr int WI = BN / (R::RP * NW);        // weight DMA instructions per wave per panel
  static constexpr int HALO_BYTES = HALO * ROWB;
  static constexpr int ZOFF = 2 * HALO_BYTES;         // the all-zero row
  static constexpr int WOFF = ZOFF + 128;
  static constexpr int PANEL = BN * ROWB;
  static constexpr int MAIN = WOFF + STAGES * PANEL;
  // epilogue staging passes: the fewest whose fp32 rows fit in the operand LDS
  static constexpr int CROW = BN * 4 + 16;
  static constexpr int EIT = BM * (BN / 8) / NT;
  static constexpr int EP = (BM * CROW <= MAIN) ? 1
                          : ((BM / 2) * CROW <= MAIN && EIT % 2 == 0 && (BM / 2) % 16 == 0) ? 2
                          : ((BM / 4) * CROW <= MAIN && EIT % 4 == 0 && (BM / 4) % 16 == 0) ? 4 : 8;
  static constexpr int LDS = MAIN;
  static_assert(XH >= 1 && XH * R::RP * NW == HALO, "halo rows must split evenly into DMA pieces");
  static_assert(WI >= 1 && WI * R::RP * NW == BN, "weight rows must split evenly into DMA pieces");
  static_assert(FI >= 1 && FJ >= 1 && WTP % 16 == 0 && WTC % 16 == 0, "wave tile");
  static_assert((STAGES - 2) * WI + XH < 64, "vmcnt range");
  static_assert(EP <= 4 || (BM / 8) % 16 == 0, "epilogue passes");
  static_assert(LDS <= 163840, "LDS");
};

template <int BM, int BN, int WM, int WN, int STAGES, int BK, int HALO, bool RES, bool LATE, int W>
__global__ __launch_bounds__(WM* WN * 64, W) void conv_shift_kernel(DmlConvArgs a) {
  using T = Cfg<BM, BN, WM, WN, STAGES, BK, HALO>;
  using RW = typename T::R;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int ntc = (a.Cout + BN - 1) / BN;
  const int Lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tc = Lb % ntc, tm = Lb / ntc;  // channel tiles fastest: an XCD's blocks share halo rows in L2
  const int m0 = tm * BM, c0 = tc * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid % WN, wp = wid / WN;
  const int frow = lane & 15, fq = lane >> 4;

  // the all-zero row read by out-of-image taps
  if (tid < 8) *(uint4*)(smem + T::ZOFF + tid * 16) = make_uint4(0, 0, 0, 0);
  __syncthreads();

  // ---- per-lane DMA bookkeeping ----
  const int lrow = RW::lane_row(lane), lchunk = RW::lane_chunk(lane);
  const int ctr = a.ph * a.W + a.pw;  // flat-pixel reach of the taps on each side
  const int hs = m0 - ctr;            // flat input pixel of halo row 0
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
  const unsigned OOB = 0x80000000u;
  const int hpix0 = hs + wid * T::XH * RW::RP + lrow;  // flat input pixel of this lane's first halo row
  const char* wbase = (const char*)a.w + ((long)(c0 + wid * T::WI * RW::RP + lrow) * a.Kpad + lchunk * 8) * 2;
  const long wstep_row = (long)RW::RP * a.Kpad * 2;

  const int taps = a.kh * a.kw;
  const int nch = a.Cin / BK;
  const int nk = nch * taps;

  auto issue_halo = [&](int c, int buf) {
    char* dst = smem + buf * T::HALO_BYTES;
#pragma unroll
    for (int j = 0; j < T::XH; ++j) {
      const int pix = hpix0 + j * RW::RP;
      const unsigned off = ((unsigned)pix < (unsigned)M) ? (unsigned)((pix * a.ldx + c * BK + lchunk * 8) * 2) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void*)(dst + (wid * T::XH + j) * 1024), 16, off, 0, 0, 0);
    }
  };
  // weight panel of iteration it = (chunk c, tap t): W columns t*Cin + c*BK ..
  int wi_c = 0, wi_t = 0;  // (chunk, tap) of the next panel to issue
  auto issue_w = [&](int stage) {
    const char* src = wbase + ((long)wi_t * a.Cin + (long)wi_c * BK) * 2;
    char* dst = smem + T::WOFF + stage * T::PANEL;
#pragma unroll
    for (int j = 0; j < T::WI; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(src + j * wstep_row), (lds_void*)(dst + (wid * T::WI + j) * 1024),
                                       16, 0, 0);
    if (++wi_t == taps) {
      wi_t = 0;
      ++wi_c;
    }
  };

  // ---- per-lane output geometry of the wave's pixel fragments ----
  int poh[T::FJ], pow_[T::FJ];
#pragma unroll
  for (int j = 0; j < T::FJ; ++j) {
    const int m = m0 + wp * T::WTP + j * 16 + frow;
    if (m < M) {
      const int n = m / HW, rem = m - n * HW;
      poh[j] = rem / a.W;
      pow_[j] = rem - poh[j] * a.W;
    } else {
      poh[j] = -(1 << 28);  // tail pixel: every tap reads the zero row
      pow_[j] = 0;
    }
  }

  f32x4 acc[T::FI][T::FJ];
#pragma unroll
  for (int i = 0; i < T::FI; ++i)
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) acc[i][j] = (f32x4)(0.f);

  // prologue: halo of chunk 0, panels 0 .. STAGES-2
  issue_halo(0, 0);
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue_w(s);

  convk::Epilogue<BM, BN, T::NT, RES, T::EP, LATE> epi;
  epi.prefetch(a, m0, c0, M, tid, 0);

  int c = 0, t = 0, r = 0, s = 0;
  for (int it = 0; it < nk; ++it) {
    // retire panel it (and, through it, the halo of chunk c); the halo of chunk
    // c+1 is younger than panel it exactly for taps 1 .. STAGES-1
    if (it + STAGES - 2 < nk) {
      if (t >= 1 && t <= STAGES - 1 && c + 1 < nch) wait_vmcnt<(STAGES - 2) * T::WI + T::XH>();
      else wait_vmcnt<(STAGES - 2) * T::WI>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (it + STAGES - 1 < nk) issue_w((it + STAGES - 1) % STAGES);
    if (t == 0 && c + 1 < nch) issue_halo(c + 1, (c + 1) & 1);

    const char* hb = smem + (c & 1) * T::HALO_BYTES;
    const char* wsb = smem + T::WOFF + (it % STAGES) * T::PANEL;
    const int toff = r * a.W + s;
    const int zrow = (c & 1) ? HALO : 2 * HALO;  // T::ZOFF as a row of this halo buffer
    const int dr = r - a.ph, ds = s - a.pw;
    int hrow[T::FJ];
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) {
      const bool ok = ((unsigned)(poh[j] + dr) < (unsigned)a.H) & ((unsigned)(pow_[j] + ds) < (unsigned)a.W);
      hrow[j] = ok ? wp * T::WTP + j * 16 + frow + toff : zrow;
    }
    constexpr int KSM = BK / 32;
    bf16x8 fa[KSM][T::FI], fb[KSM][T::FJ];
#pragma unroll
    for (int ks = 0; ks < KSM; ++ks) {
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < T::FI; ++i) fa[ks][i] = *(const bf16x8*)(wsb + RW::off(wc * T::WTC + i * 16 + frow, ch));
#pragma unroll
      for (int j = 0; j < T::FJ; ++j) fb[ks][j] = *(const bf16x8*)(hb + RW::off(hrow[j], ch));
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

    if (++s == a.kw) {
      s = 0;
      if (++r == a.kh) r = 0;
    }
    if (++t == taps) {
      t = 0;
      ++c;
    }
  }
  epi.template store<16, T::FI, T::FJ, T::WTP, T::WTC>(a, smem, acc, wp, wc, lane, tid);
}

template <int BM, int BN, int WM, int WN, int STAGES, int BK, int HALO, bool LATE, int W>
static int launch(const DmlConvArgs* a, hipStream_t st) {
  using T = Cfg<BM, BN, WM, WN, STAGES, BK, HALO>;
  const long M = (long)a->N * a->H * a->W;
  const long tiles = ((M + BM - 1) / BM) * ((a->Cout + BN - 1) / BN);
  if (a->res)
    hipLaunchKernelGGL((conv_shift_kernel<BM, BN, WM, WN, STAGES, BK, HALO, true, LATE, W>), dim3((unsigned)tiles),
                       dim3(T::NT), T::LDS, st, *a);
  else
    hipLaunchKernelGGL((conv_shift_kernel<BM, BN, WM, WN, STAGES, BK, HALO, false, false, W>), dim3((unsigned)tiles),
                       dim3(T::NT), T::LDS, st, *a);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN, int STAGES, int BK, int HALO, bool LATE, int W>
static int set_attr() {
  using T = Cfg<BM, BN, WM, WN, STAGES, BK, HALO>;
  return (int)hipFuncSetAttribute((const void*)conv_shift_kernel<BM, BN, WM, WN, STAGES, BK, HALO, true, LATE, W>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS) |
         (int)hipFuncSetAttribute((const void*)conv_shift_kernel<BM, BN, WM, WN, STAGES, BK, HALO, false, false, W>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS);
}

}  // namespace shift
}  // namespace dml

// Shifted-pixel configurations: id, BM (pixels), BN (channels), WM x WN waves,
// weight-ring STAGES, BK (channel chunk), HALO (LDS halo rows: the largest
// BM + 2*(ph*W + pw) served), LATE (residual loaded in the epilogue), W (min
// waves/SIMD register hint). Ids are
// ABI of the plan builder and the tuner (ops/tuning.py SHIFT_CFGS).
#define DML_SHIFT_TILES(X)                                                                \
  X(64, 256, 128, 4, 2, 3, 64, 384, 0, 1) /* 8 waves, 64x64 per wave, 144 KiB: 1 WG/CU */ \
  X(65, 256, 128, 4, 2, 3, 32, 384, 1, 4) /* 8 waves, 72 KiB: 2 WG/CU at <=128 VGPRs */   \
  X(66, 128, 128, 2, 2, 3, 32, 256, 1, 1) /* 4 waves, 56 KiB: 2 WG/CU */                  \
  X(67, 128, 128, 2, 2, 3, 64, 256, 0, 1) /* 4 waves, 112 KiB */                          \
  X(68, 256, 64, 4, 1, 3, 64, 384, 0, 1)  /* 4 waves, 64 ch tiles, 120 KiB */             \
  X(69, 128, 64, 2, 1, 3, 32, 256, 1, 1)  /* 2 waves, 38 KiB */

extern "C" int dml_conv_shift_init(void) {
  using namespace dml::shift;
  int rc = 0;
#define DML_SET(id, BM, BN, WM, WN, ST, BK, HALO, LATE, W) rc |= set_attr<BM, BN, WM, WN, ST, BK, HALO, LATE, W>();
  DML_SHIFT_TILES(DML_SET)
#undef DML_SET
  if (rc) dml_set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed (conv_shift)");
  return rc ? -1 : 0;
}

// channel-tile width of a shifted-pixel config (0: not one)
extern "C" int dml_conv_shift_bn(int cfg) {
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST, BK, HALO, LATE, W) \
  case id: return BN;
    DML_SHIFT_TILES(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}

// 0 if config cfg can run conv a; else an error message (host-side shape check:
// the kernel's halo, tap and chunk arithmetic assume exactly these)
extern "C" const char* dml_conv_shift_check(const DmlConvArgs* a, int cfg) {
  int bm = 0, bk = 0, halo = 0, st = 0;
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST, BK, HALO, LATE, W) \
  case id: bm = BM; bk = BK; halo = HALO; st = ST; break;
    DML_SHIFT_TILES(DML_CASE)
#undef DML_CASE
    default: return "conv_shift: not a shifted-pixel config";
  }
  if (a->sh != 1 || a->sw != 1 || (a->dh > 1) || (a->dw > 1))
    return "conv_shift: needs stride 1 and dilation 1";
  if ((a->kh & 1) == 0 || (a->kw & 1) == 0 || a->ph != (a->kh - 1) / 2 || a->pw != (a->kw - 1) / 2 ||
      a->Ho != a->H || a->Wo != a->W)
    return "conv_shift: needs odd kh, kw with same padding (Ho = H, Wo = W)";
  if (a->kh * a->kw < st) return "conv_shift: needs kh*kw >= STAGES (halo ordering of the vmcnt waits)";
  if (a->Cin % bk) return "conv_shift: needs Cin % BK == 0";
  if (a->K != a->kh * a->kw * a->Cin || a->Kpad < a->K) return "conv_shift: needs K = kh*kw*Cin";
  if (bm + 2 * (a->ph * a->W + a->pw) > halo) return "conv_shift: halo rows exceed the config's LDS halo";
  if (a->ksplit > 1 || a->rsub > 1) return "conv_shift: no split-K / subsampled residual";
  if ((long)a->N * a->H * a->W * a->ldx * 2 >= 0x7ffffff0L) return "conv_shift: input exceeds the buffer range";
  return 0;
}

extern "C" int dml_conv_shift(const DmlConvArgs* a, int cfg, hipStream_t s) {
  using namespace dml::shift;
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST, BK, HALO, LATE, W) \
  case id: return launch<BM, BN, WM, WN, ST, BK, HALO, LATE, W>(a, s);
    DML_SHIFT_TILES(DML_CASE)
#undef DML_CASE
    default: dml_set_error("dml_conv_shift: bad cfg"); return -1;
  }
}
