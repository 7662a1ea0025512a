// conv_igemm_ws.hip — warp-specialised LDS-DMA implicit-GEMM convolution (gfx950).
//
// Same GEMM view, LDS image, swizzle, epilogue and ABI (DmlConvArgs) as the v2 kernel
// (conv_igemm_v2.hip): D[c][m] = sum_k W[c][k] X[k][m], channels on the MFMA rows, so
// each v_mfma_f32_16x16x32_bf16 accumulator lane holds 4 consecutive output channels
// of one pixel. What changes is WHO does what inside the K loop (VERDICT r4 "next
// round" 1a/1b):
//
//  * NL loader waves issue every LDS-DMA of the operand ring (activations by
//    buffer_load ... lds with the hardware range check producing the im2col zero
//    padding, weights by global_load_lds) and own the per-lane im2col K walk and the
//    counted `s_waitcnt vmcnt`; they never touch the matrix pipe.
//  * NC = WM x WN MFMA waves only run ds_read_b128 fragment reads + MFMAs: no VMEM
//    issue (each LDS-DMA piece costs the issuing wave 60-185 cycles of its stream,
//    MI355X_MICROARCH.md cycle constants), no address math, no vmcnt waits.
//  * One raw s_barrier per K tile hands a landed stage from the loaders to the MFMA
//    waves and the consumed stage back (RAW: the loaders' vmcnt before barrier kt
//    retires tile kt; WAR: the stage refilled after barrier kt was last read in
//    iteration kt-1, whose reads every MFMA wave retired (its MFMAs consumed them)
//    before arriving). STAGES-1 tiles are in flight ahead of the MFMA waves.
//  * The loaders' K walk: with Cin % 64 == 0 (every ResNet50 conv, most InceptionV3
//    ones) a 64-deep K tile lies inside one tap, so advance() is one add and one
//    compare per K tile; the tap-straddling shapes (Cin 80 / 96 / 160 / 288, K tail)
//    take its loop, off the MFMA waves' critical path either way.
//
// Epilogue (conv_shared.h Epilogue): the MFMA waves stage their fp32 accumulators
// through LDS and write bias (+ residual) (+ ReLU) rows with 16-B NHWC stores; the
// loader waves only take part in its barriers.
//
// Reference compute this serves: the Keras convolutions of models.py:23-44 (InceptionV3)
// and models.py:48-69 (ResNet50) — SURVEY §2.7 "conv_igemm_bf16".
#include "conv_shared.h"
#include "pool_shared.h"

namespace dml {
namespace ws {

using convk::lds_void;
using convk::wait_vmcnt;

constexpr int lds_occupancy(int a, int b) { return 163840 / (a > b ? a : b); }

template <int BM, int BN, int WM, int WN, int NL_, int STAGES, int BK_>
struct Cfg {
  static constexpr int NC = WM * WN;          // MFMA waves
  static constexpr int NL = NL_;              // loader waves
  static constexpr int NT = (NC + NL) * 64;   // threads
  static constexpr int NTC = NC * 64;         // MFMA-wave threads (the epilogue's output threads)
  static constexpr int WTP = BM / WM;         // pixels per MFMA wave
  static constexpr int WTC = BN / WN;         // channels per MFMA wave
  static constexpr int MF = 16;               // v_mfma_f32_16x16x32_bf16 fragments
  static constexpr int FJ = WTP / MF;
  static constexpr int FI = WTC / MF;
  static constexpr int BK = BK_;
  using R = convk::Rows<BK>;
  static constexpr int ROWB = R::ROWB;
  static constexpr int XI = BM / R::RP / NL;  // X DMA pieces per loader wave per K tile
  static constexpr int WI = BN / R::RP / NL;  // W DMA pieces per loader wave per K tile
  static constexpr int L = XI + WI;           // vm ops per loader lane per K tile
  static constexpr int STAGE_BYTES = (BM + BN) * ROWB;
  static constexpr int PIPE_BYTES = STAGES * STAGE_BYTES;
  static constexpr int CROW = BN * 4 + 16;
  static constexpr bool EP_OK2 = (BM / 2) % MF == 0 && ((BM * BN / 8) / NTC) % 2 == 0;
  static constexpr bool EP_OK4 = (BM / 4) % MF == 0 && ((BM * BN / 8) / NTC) % 4 == 0;
  static constexpr int EP_MAX = EP_OK4 ? 4 : (EP_OK2 ? 2 : 1);
  static constexpr int OCC_BEST = lds_occupancy(PIPE_BYTES, (BM / EP_MAX) * CROW);
  static constexpr int EP = lds_occupancy(PIPE_BYTES, BM * CROW) >= OCC_BEST ? 1
                          : (EP_OK2 && lds_occupancy(PIPE_BYTES, (BM / 2) * CROW) >= OCC_BEST) ? 2 : EP_MAX;
  static constexpr int EPI_BYTES = (BM / EP) * CROW;
  static constexpr int LDS = PIPE_BYTES > EPI_BYTES ? PIPE_BYTES : EPI_BYTES;
  static_assert(XI >= 1 && WI >= 1, "each loader wave needs >= 1 DMA piece per operand");
  static_assert(BM % (R::RP * NL) == 0 && BN % (R::RP * NL) == 0, "tile rows must split evenly over the loaders");
  static_assert(FI >= 1 && FJ >= 1 && WTP % MF == 0 && WTC % MF == 0, "wave tile too small");
  static_assert(STAGES >= 2 && (STAGES - 2) * L < 64, "vmcnt range");
  static_assert(LDS <= 163840, "LDS");
};

template <int BM, int BN, int WM, int WN, int NL, int STAGES, bool RES, int BK, bool LATE>
__device__ __forceinline__ void conv_ws_tile(const DmlConvArgs& a, int Lb, int nblk) {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK>;
  using RW = typename T::R;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int M = a.N * a.Ho * a.Wo;
  const int ntc = (a.Cout + BN - 1) / BN;
  const int ksplit = a.ksplit > 1 ? a.ksplit : 1;
  int split = 0;
  if (ksplit > 1) {
    const int ntiles = nblk / ksplit;
    split = Lb / ntiles;
    Lb -= split * ntiles;
  }
  const int tc = Lb % ntc, tm = Lb / ntc;  // channel tiles fastest (v2: an XCD's blocks share activation rows)
  const int m0 = tm * BM, c0 = tc * BN;
  int nk = a.Kpad / T::BK, kbeg = 0;
  if (ksplit > 1) {
    const int nk_slice = (nk + ksplit - 1) / ksplit;
    kbeg = split * nk_slice;
    nk = max(0, min(nk_slice, nk - kbeg));
  }

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

  using Acc = f32x4;
  Acc acc[T::FI][T::FJ];
#pragma unroll
  for (int i = 0; i < T::FI; ++i)
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) acc[i][j] = (Acc)(0.f);
  convk::Epilogue<BM, BN, T::NTC, RES, T::EP, LATE, true> epi;
  const int wc = wid % WN, wp = wid / WN;

  if (wid >= T::NC) {
    // ======================= loader wave =======================
    const int lw = wid - T::NC;
    const int lrow = RW::lane_row(lane);
    const int lchunk = RW::lane_chunk(lane);
    int base[T::XI], ih0[T::XI], iw0[T::XI];
    const int HoWo = a.Ho * a.Wo;
#pragma unroll
    for (int j = 0; j < T::XI; ++j) {
      const int m = m0 + (lw * T::XI + j) * RW::RP + lrow;
      if (m < M) {
        const int n = m / HoWo;
        const int rem = m - n * HoWo;
        const int oh = rem / a.Wo;
        const int ow = rem - oh * a.Wo;
        ih0[j] = oh * a.sh - a.ph;
        iw0[j] = ow * a.sw - a.pw;
        base[j] = (n * a.H * a.W + ih0[j] * a.W + iw0[j]) * a.ldx;
      } else {
        base[j] = 0;
        ih0[j] = -(1 << 28);  // fails every bounds test: zero row
        iw0[j] = 0;
      }
    }
    const int dh = a.dh > 0 ? a.dh : 1, dw = a.dw > 0 ? a.dw : 1;
    const int step_s = dw * a.ldx;
    const int step_r = dh * a.W * a.ldx;
    int cc = lchunk * 8, ss = 0, rr = 0, dih = 0, diw = 0, koff = lchunk * 8;
    auto advance = [&](int by) {
      cc += by;
      koff += by;
      while (cc >= a.Cin) {
        cc -= a.Cin;
        koff += step_s - a.Cin;
        diw += dw;
        if (++ss == a.kw) {
          ss = 0;
          koff += step_r - a.kw * step_s;
          diw = 0;
          ++rr;
          dih = rr < a.kh ? dih + dh : (1 << 28);  // K tail: every row out of bounds -> zeros
        }
      }
    };
    advance(0);
    if (kbeg > 0) advance(kbeg * T::BK);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
    const unsigned OOB = 0x80000000u;
    const char* wbase =
        (const char*)a.w + ((long)(c0 + lw * T::WI * RW::RP + lrow) * a.Kpad + (long)kbeg * T::BK + lchunk * 8) * 2;
    const long wstep_row = (long)RW::RP * a.Kpad * 2;

    auto issue = [&](int kt, int stage) {
      char* sx = smem + stage * T::STAGE_BYTES;
      char* sw = sx + BM * T::ROWB;
#pragma unroll
      for (int j = 0; j < T::XI; ++j) {
        const int ih = ih0[j] + dih, iw = iw0[j] + diw;
        const unsigned ok = ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
        const unsigned msk = 0u - ok;
        const unsigned off = ((unsigned)((base[j] + koff) * 2) & msk) | (OOB & ~msk);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void*)(sx + (lw * T::XI + j) * 1024), 16, off, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < T::WI; ++j) {
        const char* src = wbase + j * wstep_row + (long)kt * T::BK * 2;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sw + (lw * T::WI + j) * 1024), 16, 0, 0);
      }
      advance(T::BK);
    };

#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nk) issue(s, s);
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + STAGES - 2 < nk) wait_vmcnt<(STAGES - 2) * T::L>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // tile kt published to the MFMA waves
      if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    }
  } else {
    // ======================= MFMA wave =======================
    epi.prefetch(a, m0, c0, M, tid, split);
    const int frow = lane & 15, fq = lane >> 4;
    constexpr int KSM = BK / 32;
    auto read = [&](int kt, bf16x8(&fa)[KSM][T::FI], bf16x8(&fb)[KSM][T::FJ]) __attribute__((always_inline)) {
      const char* sx = smem + (kt % STAGES) * T::STAGE_BYTES;
      const char* sw = sx + BM * T::ROWB;
#pragma unroll
      for (int ks = 0; ks < KSM; ++ks) {
        const int ch = ks * 4 + fq;
#pragma unroll
        for (int i = 0; i < T::FI; ++i) fa[ks][i] = *(const bf16x8*)(sw + RW::off(wc * T::WTC + i * 16 + frow, ch));
#pragma unroll
        for (int j = 0; j < T::FJ; ++j) fb[ks][j] = *(const bf16x8*)(sx + RW::off(wp * T::WTP + j * 16 + frow, ch));
      }
    };
    auto mfma = [&](bf16x8(&fa)[KSM][T::FI], bf16x8(&fb)[KSM][T::FJ]) __attribute__((always_inline)) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < KSM; ++ks)
#pragma unroll
        for (int i = 0; i < T::FI; ++i)
#pragma unroll
          for (int j = 0; j < T::FJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    for (int kt = 0; kt < nk; ++kt) {
      __builtin_amdgcn_s_barrier();  // tile kt landed (loaders' vmcnt), stage kt-1 free for the refill
      bf16x8 fa[KSM][T::FI], fb[KSM][T::FJ];
      read(kt, fa, fb);
      mfma(fa, fb);
    }
  }

  // every DMA retired (the loaders' last wait is vmcnt(0)); the epilogue's first
  // __syncthreads orders the last fragment reads before its staging writes
  epi.template store<16, T::FI, T::FJ, T::WTP, T::WTC>(a, smem, acc, wp, wc, lane, tid, wid < T::NC);
}

template <int BM, int BN, int WM, int WN, int NL, int STAGES, bool RES, int BK, bool LATE, int W>
__global__ __launch_bounds__((WM * WN + NL) * 64, W) void conv_ws_kernel(DmlConvArgs a) {
  conv_ws_tile<BM, BN, WM, WN, NL, STAGES, RES, BK, LATE>(a, xcd_remap(blockIdx.x, gridDim.x), gridDim.x);
}

template <int BM, int BN, int WM, int WN, int NL, int STAGES, int BK, bool LATE, int W>
static int launch(const DmlConvArgs* a, hipStream_t s) {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK>;
  const long M = (long)a->N * a->Ho * a->Wo;
  const long tiles = ((M + BM - 1) / BM) * ((a->Cout + BN - 1) / BN) * (a->ksplit > 1 ? a->ksplit : 1);
  if (a->res)
    hipLaunchKernelGGL((conv_ws_kernel<BM, BN, WM, WN, NL, STAGES, true, BK, LATE, W>), dim3((unsigned)tiles),
                       dim3(T::NT), T::LDS, s, *a);
  else
    hipLaunchKernelGGL((conv_ws_kernel<BM, BN, WM, WN, NL, STAGES, false, BK, false, W>), dim3((unsigned)tiles),
                       dim3(T::NT), T::LDS, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN, int NL, int STAGES, int BK, bool LATE, int W>
static int set_attr() {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK>;
  return (int)hipFuncSetAttribute((const void*)conv_ws_kernel<BM, BN, WM, WN, NL, STAGES, true, BK, LATE, W>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS) |
         (int)hipFuncSetAttribute((const void*)conv_ws_kernel<BM, BN, WM, WN, NL, STAGES, false, BK, false, W>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS);
}

}  // namespace ws
}  // namespace dml

// Warp-specialised tile configurations: id, BM (pixels), BN (channels), WM x WN MFMA
// waves, NL loader waves, ring STAGES, BK, RL (residual loaded in the epilogue), W (min
// waves/SIMD register hint). The fragment-prefetch forms (113..118, r5) never beat their bases
// and were removed in r6. Ids 100..139 are part of the plan-builder / tuner ABI
// (ops/tuning.py WS_CFGS); validated by dml_conv (conv_dispatch.hip).
#define DML_WS_TILES(X)                                                                         \
  X(100, 128, 128, 2, 2, 4, 3, 64, 0, 1)  /* 4 MFMA (64x64) + 4 loaders, 96 KiB, 1 WG/CU */      \
  X(101, 128, 128, 2, 2, 2, 4, 32, 0, 1)  /* 4 + 2, BK32 4-stage, 64 KiB: 2 WG/CU */             \
  X(102, 256, 128, 4, 2, 4, 3, 64, 1, 1)  /* 8 + 4, 144 KiB (residual form: late, else it spills) */ \
  X(103, 128, 64, 2, 2, 2, 3, 64, 0, 1)   /* 4 (64px x 32ch) + 2, 72 KiB: 2 WG/CU */             \
  X(104, 64, 128, 1, 4, 2, 3, 64, 0, 1)   /* 4 (64px x 32ch) + 2, 72 KiB: 2 WG/CU */             \
  X(105, 256, 64, 4, 1, 4, 3, 64, 0, 1)   /* 4 (64x64) + 4, 120 KiB */                           \
  X(106, 128, 128, 2, 2, 4, 4, 64, 0, 1)  /* 4 + 4, 128 KiB */                                   \
  X(107, 256, 128, 4, 2, 4, 4, 32, 0, 1)  /* 8 + 4, BK32 4-stage, 96 KiB */                      \
  X(108, 128, 256, 2, 4, 4, 3, 64, 1, 1)  /* 8 + 4, 144 KiB (residual form: late) */           \
  X(109, 128, 64, 2, 2, 2, 4, 32, 0, 1)   /* 4 + 2, BK32 4-stage, 48 KiB: 3 WG/CU */             \
  X(110, 64, 128, 1, 4, 2, 4, 32, 0, 1)   /* 4 + 2, BK32 4-stage, 48 KiB: 3 WG/CU */             \
  X(111, 128, 128, 2, 2, 2, 3, 64, 0, 1)  /* 4 + 2, 96 KiB */                                    \
  X(112, 128, 128, 2, 2, 4, 2, 64, 0, 1)  /* 4 + 4, 2-stage, 64 KiB: 2 WG/CU */                  \
  X(119, 256, 128, 4, 2, 4, 6, 32, 1, 1)  /* 8 + 4, BK32 6-stage, 144 KiB: 5 tiles in flight */

extern "C" int dml_conv_ws_init(void) {
  using namespace dml::ws;
  int rc = 0;
#define DML_SET(id, BM, BN, WM, WN, NL, ST, BK, RL, W) rc |= set_attr<BM, BN, WM, WN, NL, ST, BK, RL, W>();
  DML_WS_TILES(DML_SET)
#undef DML_SET
  if (rc) dml_set_error("dml_conv_ws_init: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  return rc ? -1 : 0;
}

extern "C" int dml_conv_ws(const DmlConvArgs* a, int cfg, hipStream_t s) {
  using namespace dml::ws;
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, NL, ST, BK, RL, W) \
  case id: return launch<BM, BN, WM, WN, NL, ST, BK, RL, W>(a, s);
    DML_WS_TILES(DML_CASE)
#undef DML_CASE
    default: dml_set_error("dml_conv_ws: bad cfg"); return -1;
  }
}

// channel-tile width of a warp-specialised config (0: not one)
extern "C" int dml_conv_ws_bn(int cfg) {
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, NL, ST, BK, RL, W) \
  case id: return BN;
    DML_WS_TILES(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}
