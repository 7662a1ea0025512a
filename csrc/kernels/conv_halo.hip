// conv_halo.hip — stride-1 convolution from halo tiles (gfx950).
//
// The generic implicit GEMM (conv_igemm_v2.hip) DMAs one 64-channel X tile per
// (tap, channel chunk): a 3x3 layer fetches every activation row 9 times from
// L2. On MI355X that fetch, not the MFMA, bounds the 3x3 layers (~17 TB/s of
// L2->LDS traffic at ~750 TF/s; the L2 gather ceiling is 17-19 TB/s).
//
// Here a workgroup owns BM consecutive output pixels (flattened n, oh, ow) and
// loads, once per 64-channel chunk, the HALO those pixels read: in the zero-
// padded image (Hq = Ho+kh-1 rows of Wq = Wo+kw-1 pixels per image, images
// stacked) output pixel (n, oh, ow) reads tap (r, s) at padded position
//     P(n, oh, ow) + r*Wq + s,   P(n, oh, ow) = (n*Hq + oh)*Wq + ow,
// so the BM pixels' taps all fall in ONE contiguous span of padded positions
// [P(m0), P(m_last) + (kh-1)*Wq + kw). The span is DMA'd to LDS (one 128-B row
// per position; padding positions and channels >= Cin come from the buffer
// range check as zeros), and each of the kh*kw taps is an MFMA pass whose pixel
// fragments are read at a per-lane row offset + a uniform tap offset. Only the
// weights stream per tap. X traffic drops from kh*kw x to ~(span/BM) x.
//
// K order of the weights is chunk-major: W[cout][chunk][tap][64] (host packs
// them so; `Kpad` = nch*kh*kw*64), so K tile kt = (chunk kt / T, tap kt % T)
// is contiguous and streamed exactly like v2's.
//
// Pipeline: W tiles in an S-stage ring; X halos double-buffered across channel
// chunks. X(c+1) is issued right after W(c*T+S-1) at the first tap of chunk c;
// counted vmcnt waits account for it (it is younger than W(kt) exactly for the
// taps 1..S-1 of chunk c). Requires T = kh*kw >= S.
#include "conv_shared.h"

namespace dml {
namespace halo {

using convk::lds_swz;
using convk::lds_void;
using convk::wait_vmcnt;

template <int BM, int BN, int WM, int WN, int S, int XP>
struct Cfg {
  static constexpr int NW = WM * WN;
  static constexpr int NT = NW * 64;
  static constexpr int WTP = BM / WM;
  static constexpr int WTC = BN / WN;
  static constexpr int FJ = WTP / 16;
  static constexpr int FI = WTC / 16;
  static constexpr int XROWS = XP * NW * 8;    // halo rows per X buffer
  static constexpr int XBYTES = XROWS * 128;
  static constexpr int WI = BN / 8 / NW;       // W DMA instructions per wave per tile
  static constexpr int WBYTES = BN * 128;
  static constexpr int EPI = BM * (BN * 4 + 16);
  static_assert(WI >= 1 && BN % (8 * NW) == 0, "W tile rows must split across waves");
  static_assert(FI >= 1 && FJ >= 1, "wave tile too small");
  static_assert((S - 2) * WI + XP < 64, "vmcnt overflow");
  static_assert(S >= 2, "at least double-buffered weights");
};

// padded flat position of output pixel m
__device__ __forceinline__ int pflat(int m, int HoWo, int Wo, int Hq, int Wq) {
  const int n = m / HoWo;
  const int r = m - n * HoWo;
  const int oh = r / Wo;
  return (n * Hq + oh) * Wq + (r - oh * Wo);
}

template <int BM, int BN, int WM, int WN, int S, int XP, bool RES>
__device__ __forceinline__ void conv_halo_body(const DmlConvArgs& a) {
  using C = Cfg<BM, BN, WM, WN, S, XP>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int M = a.N * a.Ho * a.Wo;
  const int HoWo = a.Ho * a.Wo;
  const int ntc = (a.Cout + BN - 1) / BN;
  const int Lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tc = Lb % ntc, tm = Lb / ntc;
  const int m0 = tm * BM, c0 = tc * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int Wq = a.Wo + a.kw - 1, Hq = a.Ho + a.kh - 1;
  const int T = a.kh * a.kw;
  const int nch = (a.Cin + 63) >> 6;
  const int nk = nch * T;
  const int P0 = pflat(m0, HoWo, a.Wo, Hq, Wq);
  const int mlast = (m0 + BM < M ? m0 + BM : M) - 1;
  const int span = pflat(mlast, HoWo, a.Wo, Hq, Wq) - P0 + (a.kh - 1) * Wq + a.kw;

  // ---- X halo DMA: piece q = wid*XP + j covers halo rows 8q .. 8q+7 ----
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  const unsigned OOB = 0x80000000u;
  unsigned xoff[XP];
#pragma unroll
  for (int j = 0; j < XP; ++j) {
    const int q = (wid * XP + j) * 8 + lrow;
    const int P = P0 + q;
    const int rowall = P / Wq;
    const int pc = P - rowall * Wq;
    const int n = rowall / Hq;
    const int ih = rowall - n * Hq - a.ph, iw = pc - a.pw;
    const bool ok = q < span && n < a.N && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    xoff[j] = ok ? (unsigned)((((n * a.H + ih) * a.W + iw) * a.ldx + lchunk * 8) * 2) : OOB;
  }
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
  const int nxb = nch > 1 ? 2 : 1;
  char* const wring = smem + nxb * C::XBYTES;

  auto issue_x = [&](int c) {
    char* xs = smem + (c & 1) * C::XBYTES;
    // channels >= Cin (Cin % 64 != 0) -> zeros; offsets stay < 2^31 so OOB|x is OOB
    const unsigned cmask = (c * 64 + lchunk * 8 < a.Cin) ? 0u : OOB;
    const unsigned cadd = (unsigned)c * 128u;
#pragma unroll
    for (int j = 0; j < XP; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void*)(xs + (wid * XP + j) * 1024), 16,
                                               (xoff[j] + cadd) | cmask, 0, 0, 0);
  };

  const char* wbase = (const char*)a.w + ((long)(c0 + wid * C::WI * 8 + lrow) * a.Kpad + lchunk * 8) * 2;
  const long wstep_row = (long)8 * a.Kpad * 2;
  auto issue_w = [&](int kt) {
    char* ws = wring + (kt % S) * C::WBYTES;
#pragma unroll
    for (int j = 0; j < C::WI; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(wbase + j * wstep_row + (long)kt * 128),
                                       (lds_void*)(ws + (wid * C::WI + j) * 1024), 16, 0, 0);
  };

  const int wc = wid % WN, wp = wid / WN;
  const int frow = lane & 15, fq = lane >> 4;
  // halo row of this lane's pixel in each pixel fragment (tap (0,0))
  int drow[C::FJ];
#pragma unroll
  for (int j = 0; j < C::FJ; ++j) {
    const int m = m0 + wp * C::WTP + j * 16 + frow;
    drow[j] = m < M ? pflat(m, HoWo, a.Wo, Hq, Wq) - P0 : 0;
  }

  f32x4 acc[C::FI][C::FJ];
#pragma unroll
  for (int i = 0; i < C::FI; ++i)
#pragma unroll
    for (int j = 0; j < C::FJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: X(0), then W tiles 0 .. S-2
  issue_x(0);
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue_w(s);

  convk::Epilogue<BM, BN, C::NT, RES> epi;
  epi.prefetch(a, m0, c0, M, tid);

  int c = 0, t = 0, ts = 0, toff = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // retire W(kt) (and, at t == 0, X(c)); X(c+1) may stay in flight when it
    // is younger than W(kt), i.e. for taps 1..S-1 of chunk c.
    if (kt + S - 2 < nk) {
      if (t >= 1 && t <= S - 1 && c + 1 < nch) wait_vmcnt<(S - 2) * C::WI + XP>();
      else wait_vmcnt<(S - 2) * C::WI>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (kt + S - 1 < nk) issue_w(kt + S - 1);
    if (t == 0 && c + 1 < nch) issue_x(c + 1);

    const char* xs = smem + (c & 1) * C::XBYTES;
    const char* ws = wring + (kt % S) * C::WBYTES;
    bf16x8 fa[2][C::FI], fb[2][C::FJ];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < C::FI; ++i) fa[ks][i] = *(const bf16x8*)(ws + lds_swz(wc * C::WTC + i * 16 + frow, ch));
#pragma unroll
      for (int j = 0; j < C::FJ; ++j) fb[ks][j] = *(const bf16x8*)(xs + lds_swz(drow[j] + toff, ch));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < C::FI; ++i)
#pragma unroll
        for (int j = 0; j < C::FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);

    // next tap (row-major over (r, s)), then next channel chunk
    ++toff;
    if (++ts == a.kw) {
      ts = 0;
      toff += Wq - a.kw;
    }
    if (++t == T) {
      t = 0;
      toff = 0;
      ++c;
    }
  }

  epi.template store<C::FI, C::FJ, C::WTP, C::WTC>(a, smem, acc, wp, wc, lane, tid);
}

template <int BM, int BN, int WM, int WN, int S, int XP, bool RES>
__global__ __launch_bounds__(WM* WN * 64) void conv_halo_kernel(DmlConvArgs a) {
  conv_halo_body<BM, BN, WM, WN, S, XP, RES>(a);
}

// Largest halo span over all tiles of this launch (host side, exact).
static long max_span(const DmlConvArgs* a, int BM) {
  const long M = (long)a->N * a->Ho * a->Wo, HoWo = (long)a->Ho * a->Wo;
  const long Wq = a->Wo + a->kw - 1, Hq = a->Ho + a->kh - 1;
  auto pf = [&](long m) {
    const long n = m / HoWo, r = m - n * HoWo, oh = r / a->Wo;
    return (n * Hq + oh) * Wq + (r - oh * a->Wo);
  };
  long best = 0;
  for (long m0 = 0; m0 < M; m0 += BM) {
    const long ml = (m0 + BM < M ? m0 + BM : M) - 1;
    const long sp = pf(ml) - pf(m0) + (a->kh - 1) * Wq + a->kw;
    if (sp > best) best = sp;
  }
  return best;
}

template <int BM, int BN, int WM, int WN, int S, int XP>
static int lds_bytes(const DmlConvArgs* a) {
  using C = Cfg<BM, BN, WM, WN, S, XP>;
  const int nch = (a->Cin + 63) / 64;
  const int pipe = (nch > 1 ? 2 : 1) * C::XBYTES + S * C::WBYTES;
  return pipe > C::EPI ? pipe : C::EPI;
}

template <int BM, int BN, int WM, int WN, int S, int XP>
static int check(const DmlConvArgs* a) {
  using C = Cfg<BM, BN, WM, WN, S, XP>;
  const int T = a->kh * a->kw;
  const int nch = (a->Cin + 63) / 64;
  if (a->sh != 1 || a->sw != 1 || (a->dh > 1) || (a->dw > 1)) return -1;
  if (T < S || a->Kpad != nch * T * 64) return -2;
  if (max_span(a, BM) > C::XROWS) return -4;
  if (lds_bytes<BM, BN, WM, WN, S, XP>(a) > 160 * 1024) return -5;
  return 0;
}

template <int BM, int BN, int WM, int WN, int S, int XP>
static int launch(const DmlConvArgs* a, hipStream_t s) {
  using C = Cfg<BM, BN, WM, WN, S, XP>;
  const int rc = check<BM, BN, WM, WN, S, XP>(a);
  if (rc) {
    static const char* why[] = {"", "needs stride 1 / dilation 1", "needs kh*kw >= stages and halo-packed weights",
                                "", "halo span exceeds the tile's LDS rows",
                                "LDS over 160 KiB"};
    dml_set_error(why[-rc]);
    return -1;
  }
  const long M = (long)a->N * a->Ho * a->Wo;
  const long tiles = ((M + BM - 1) / BM) * ((a->Cout + BN - 1) / BN);
  const int lds = lds_bytes<BM, BN, WM, WN, S, XP>(a);
  if (a->res)
    hipLaunchKernelGGL((conv_halo_kernel<BM, BN, WM, WN, S, XP, true>), dim3((unsigned)tiles), dim3(C::NT), lds, s,
                       *a);
  else
    hipLaunchKernelGGL((conv_halo_kernel<BM, BN, WM, WN, S, XP, false>), dim3((unsigned)tiles), dim3(C::NT), lds, s,
                       *a);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN, int S, int XP>
static int set_attr() {
  return (int)hipFuncSetAttribute((const void*)conv_halo_kernel<BM, BN, WM, WN, S, XP, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) |
         (int)hipFuncSetAttribute((const void*)conv_halo_kernel<BM, BN, WM, WN, S, XP, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

#define DML_HALO_CFGS(X)            \
  X(40, 128, 64, 2, 2, 3, 12)       \
  X(41, 128, 64, 2, 2, 3, 16)       \
  X(42, 256, 64, 4, 1, 3, 16)       \
  X(43, 128, 128, 2, 2, 2, 8)       \
  X(44, 128, 128, 2, 2, 2, 12)      \
  X(45, 128, 128, 2, 2, 3, 8)       \
  X(46, 64, 128, 1, 4, 3, 8)        \
  X(47, 256, 64, 4, 1, 3, 20)

}  // namespace halo
}  // namespace dml

extern "C" int dml_conv_halo_init(void) {
  using namespace dml::halo;
  int rc = 0;
#define X(id, bm, bn, wm, wn, s, xp) rc |= set_attr<bm, bn, wm, wn, s, xp>();
  DML_HALO_CFGS(X)
#undef X
  if (rc) dml_set_error("hipFuncSetAttribute(halo) failed");
  return rc ? -1 : 0;
}

// 0 if config `cfg` can run this conv, else <0 (host-side shape check only)
extern "C" int dml_conv_halo_ok(const DmlConvArgs* a, int cfg) {
  using namespace dml::halo;
  switch (cfg) {
#define X(id, bm, bn, wm, wn, s, xp) \
  case id: return check<bm, bn, wm, wn, s, xp>(a);
    DML_HALO_CFGS(X)
#undef X
    default: return -1;
  }
}

extern "C" int dml_conv_halo(const DmlConvArgs* a, int cfg, hipStream_t st) {
  using namespace dml::halo;
  switch (cfg) {
#define X(id, bm, bn, wm, wn, s, xp) \
  case id: return launch<bm, bn, wm, wn, s, xp>(a, st);
    DML_HALO_CFGS(X)
#undef X
    default: dml_set_error("dml_conv_halo: bad cfg"); return -1;
  }
}
