// conv_igemm_wsp.hip — PERSISTENT warp-specialised implicit-GEMM convolution (gfx950).
//
// The warp-specialised kernel (conv_igemm_ws.hip: NL loader waves own every LDS-DMA of
// the operand ring, WM x WN MFMA waves only read fragments and issue MFMAs, one raw
// s_barrier per K tile) made persistent: a grid of about CUs x workgroups-per-CU
// workgroups, each running a list of output tiles, and ONE operand ring over the
// flattened (tile, K tile) sequence. The loaders therefore keep STAGES-1 K tiles in
// flight ACROSS tile boundaries: while the MFMA waves run a tile's epilogue, the next
// tile's first K tiles are already landing. That is what the per-tile kernels cannot do
// — each of their workgroups starts with an empty ring and pays the operand latency
// (about 1 us from HBM / MALL) before its first MFMA — and it matters most for the short
// K loops of the 1x1 and 64-channel 3x3 layers (ResNet50 stage 2: 9 K tiles of 64 per
// tile), where that start-up is a large part of a tile's life.
//
// Tile order: XCD x (= blockIdx % 8 under the round-robin dispatch; speed only) owns
// the contiguous range [x*chunk, (x+1)*chunk) of the channel-fastest tile order, its
// workgroups interleaved over it, so the tiles an XCD runs at one time are neighbours
// that share activation rows (and weight panels) in its L2.
//
// Epilogue: wave-private, no workgroup barrier (the loaders never wait for it): each
// MFMA wave stages one 16-pixel row of its fp32 accumulator fragments at a time in its
// own LDS area (outside the ring), reads back 8 consecutive channels of one pixel per
// lane, adds bias (+ residual, loaded at the start of the epilogue) (+ ReLU) and writes
// 16-B NHWC rows — the same arithmetic, in the same order, as the shared Epilogue, so
// outputs are bit-identical to the v2 / warp-specialised tiles. Channel offsets, output
// segments (fused sibling 1x1 convs), fp32 output and the stride-2 subsampled residual
// are supported; split-K is not (the per-tile kernels serve it).
//
// Reference compute: the Keras convolutions of models.py:23-44 / 48-69.
#include "conv_shared.h"

namespace dml {
namespace wsp {

using convk::lds_void;
using convk::wait_vmcnt;

template <int BM, int BN, int WM, int WN, int NL_, int STAGES, int BK_>
struct Cfg {
  static constexpr int NC = WM * WN, NL = NL_, NT = (NC + NL) * 64;
  static constexpr int WTP = BM / WM, WTC = BN / WN;
  static constexpr int FJ = WTP / 16, FI = WTC / 16;
  static constexpr int BK = BK_;
  using R = convk::Rows<BK>;
  static constexpr int ROWB = R::ROWB;
  static constexpr int XI = BM / R::RP / NL, WI = BN / R::RP / NL, L = XI + WI;
  static constexpr int STAGE_BYTES = (BM + BN) * ROWB;
  static constexpr int PIPE_BYTES = STAGES * STAGE_BYTES;
  static constexpr int CGW = WTC / 8;           // 8-channel groups of a wave tile row
  static constexpr int PPR = 64 / CGW;          // pixels per read-back pass
  static constexpr int SROW = WTC * 4 + 16;     // fp32 staging row pitch (bytes)
  static constexpr int EPW = 16 * SROW;         // staging bytes per MFMA wave (one 16-pixel row)
  static constexpr int LDS = PIPE_BYTES + NC * EPW;
  static_assert(XI >= 1 && WI >= 1 && BM % (R::RP * NL) == 0 && BN % (R::RP * NL) == 0, "loader split");
  static_assert(FI >= 1 && FJ >= 1 && WTC % 16 == 0 && WTP % 16 == 0 && 16 % PPR == 0, "wave tile");
  static_assert(STAGES >= 2 && (STAGES - 2) * L < 64, "vmcnt range");
  static_assert(LDS <= 163840, "LDS");
};

template <int BM, int BN, int WM, int WN, int NL, int STAGES, int BK, bool RES>
__global__ __launch_bounds__((WM * WN + NL) * 64) void conv_wsp_kernel(DmlConvArgs a) {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK>;
  using RW = typename T::R;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int M = a.N * a.Ho * a.Wo;
  const int ntc = (a.Cout + BN - 1) / BN;
  const int ntiles = ((M + BM - 1) / BM) * ntc;
  const int nk = a.Kpad / BK;
  // this workgroup's tiles: XCD x's contiguous range, interleaved over its G / 8 workgroups
  const int G = gridDim.x, b = blockIdx.x;
  const int per = G >> 3, chunk = (ntiles + 7) >> 3;
  const int tbeg = (b & 7) * chunk + (b >> 3);
  const int tend = min(ntiles, ((b & 7) + 1) * chunk);
  const int nmine = tbeg < tend ? (tend - tbeg + per - 1) / per : 0;
  const int nsteps = nmine * nk;  // the flattened (tile, K tile) sequence of this workgroup

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

  if (wid >= T::NC) {
    // ============================ loader wave ============================
    const int lw = wid - T::NC;
    const int lrow = RW::lane_row(lane), lchunk = RW::lane_chunk(lane);
    const int HoWo = a.Ho * a.Wo;
    const int dh = a.dh > 0 ? a.dh : 1, dw = a.dw > 0 ? a.dw : 1;
    const int step_s = dw * a.ldx, step_r = dh * a.W * a.ldx;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
    const unsigned OOB = 0x80000000u;
    const long wstep_row = (long)RW::RP * a.Kpad * 2;
    int base[T::XI], ih0[T::XI], iw0[T::XI];
    int cc, ss, rr, dih, diw, koff, kt_i = 0, tile_i = tbeg;
    const char* wbase = nullptr;
    auto setup = [&](int t) __attribute__((always_inline)) {  // row bases and the K walk of tile t
      const int m0 = (t / ntc) * BM, c0 = (t % ntc) * BN;
#pragma unroll
      for (int j = 0; j < T::XI; ++j) {  // straight-line selects: the arrays stay in registers
        const int m = m0 + (lw * T::XI + j) * RW::RP + lrow;
        const bool in = m < M;
        const int mm = in ? m : 0;
        const int n = mm / HoWo, rem = mm - n * HoWo;
        const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
        const int h0 = oh * a.sh - a.ph, w0 = ow * a.sw - a.pw;
        ih0[j] = in ? h0 : -(1 << 28);  // a row past M fails every bounds test: zeros
        iw0[j] = in ? w0 : 0;
        base[j] = in ? (n * a.H * a.W + h0 * a.W + w0) * a.ldx : 0;
      }
      cc = lchunk * 8; ss = 0; rr = 0; dih = 0; diw = 0; koff = lchunk * 8;
      wbase = (const char*)a.w + ((long)(c0 + lw * T::WI * RW::RP + lrow) * a.Kpad + lchunk * 8) * 2;
    };
    auto advance = [&](int by) __attribute__((always_inline)) {
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
          dih = rr < a.kh ? dih + dh : (1 << 28);  // K tail: zeros
        }
      }
    };
    auto issue = [&](int stage) __attribute__((always_inline)) {  // the next (tile, K tile) into `stage`
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
        const char* src = wbase + j * wstep_row + (long)kt_i * BK * 2;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sw + (lw * T::WI + j) * 1024), 16, 0, 0);
      }
      if (++kt_i == nk) {  // next tile of this workgroup
        kt_i = 0;
        tile_i += per;
        if (tile_i < tend) {
          setup(tile_i);
          advance(0);
        }
      } else {
        advance(BK);
      }
    };
    if (nsteps > 0) {
      setup(tile_i);
      advance(0);
    }
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nsteps) issue(s);
    for (int f = 0; f < nsteps; ++f) {
      if (f + STAGES - 2 < nsteps) wait_vmcnt<(STAGES - 2) * T::L>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // step f published to the MFMA waves; step f-1's stage free
      if (f + STAGES - 1 < nsteps) issue((f + STAGES - 1) % STAGES);
    }
    return;
  }

  // ============================= MFMA wave =============================
  const int wc = wid % WN, wp = wid / WN;
  const int frow = lane & 15, fq = lane >> 4;
  char* stg = smem + T::PIPE_BYTES + wid * T::EPW;  // this wave's private staging rows
  const int cg = lane % T::CGW, pr = lane / T::CGW;  // read-back: channel group, pixel in pass
  int f = 0;
  for (int t = tbeg; t < tend; t += per) {
    const int m0 = (t / ntc) * BM, c0 = (t % ntc) * BN;
    f32x4 acc[T::FI][T::FJ];
#pragma unroll
    for (int i = 0; i < T::FI; ++i)
#pragma unroll
      for (int j = 0; j < T::FJ; ++j) acc[i][j] = (f32x4)(0.f);
    for (int kt = 0; kt < nk; ++kt, ++f) {
      __builtin_amdgcn_s_barrier();
      const char* sx = smem + (f % STAGES) * T::STAGE_BYTES;
      const char* sw = sx + BM * T::ROWB;
      constexpr int KSM = BK / 32;
      bf16x8 fa[KSM][T::FI], fb[KSM][T::FJ];
#pragma unroll
      for (int ks = 0; ks < KSM; ++ks) {
        const int ch = ks * 4 + fq;
#pragma unroll
        for (int i = 0; i < T::FI; ++i) fa[ks][i] = *(const bf16x8*)(sw + RW::off(wc * T::WTC + i * 16 + frow, ch));
#pragma unroll
        for (int j = 0; j < T::FJ; ++j) fb[ks][j] = *(const bf16x8*)(sx + RW::off(wp * T::WTP + j * 16 + frow, ch));
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

    // ---- epilogue (this wave only): lane -> channel group cg, pixels pr + PPR*q of each row ----
    const int ch = c0 + wc * T::WTC + cg * 8;
    const bool ch_ok = ch < a.Cout;
    float4 bias0 = make_float4(0.f, 0.f, 0.f, 0.f), bias1 = bias0;
    if (ch_ok) {
      bias0 = *(const float4*)(a.bias + ch);
      bias1 = *(const float4*)(a.bias + ch + 4);
    }
    void* ybase = a.y;
    int ldy = a.ldy, relu = a.relu, choff = ch;
    if (a.nseg > 0) {
      int sgi = 0;
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (q < a.nseg && ch >= a.seg_c0[q]) sgi = q;
      ybase = a.seg_y[sgi];
      ldy = a.seg_ldy[sgi];
      relu = a.seg_relu[sgi];
      choff = ch - a.seg_c0[sgi];
    }
    constexpr int NQ = 16 / T::PPR;  // read-back passes per 16-pixel row
    uint4 rpre[RES ? T::FJ * NQ : 1];
    if constexpr (RES) {  // the tile's residual rows, all in flight before the first use
      const unsigned short* __restrict__ rg = (const unsigned short*)a.res;
#pragma unroll
      for (int j = 0; j < T::FJ; ++j)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int m = m0 + wp * T::WTP + j * 16 + q * T::PPR + pr;
          long rp = m;
          if (a.rsub > 1) {
            const int hw = a.Ho * a.Wo;
            const int ni = m / hw, r = m - ni * hw;
            const int ho = r / a.Wo, wo = r - ho * a.Wo;
            rp = (long)ni * a.rHW + ((long)ho * a.rW + wo) * a.rsub;
          }
          rpre[j * NQ + q] = (ch_ok && m < M) ? *(const uint4*)(rg + rp * a.ldr + ch) : make_uint4(0, 0, 0, 0);
        }
    }
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) {
#pragma unroll
      for (int i = 0; i < T::FI; ++i)  // fragment (i, j): 4 channels of pixel frow per lane
        *(f32x4*)(stg + frow * T::SROW + (i * 16 + fq * 4) * 4) = acc[i][j];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int lp = q * T::PPR + pr;
        const int m = m0 + wp * T::WTP + j * 16 + lp;
        const float4 v0 = *(const float4*)(stg + lp * T::SROW + cg * 32);
        const float4 v1 = *(const float4*)(stg + lp * T::SROW + cg * 32 + 16);
        if (m >= M || !ch_ok) continue;
        float v[8] = {v0.x + bias0.x, v0.y + bias0.y, v0.z + bias0.z, v0.w + bias0.w,
                      v1.x + bias1.x, v1.y + bias1.y, v1.z + bias1.z, v1.w + bias1.w};
        if constexpr (RES) {
          const uint4 r = rpre[j * NQ + q];
          v[0] += bf2f(r.x & 0xffff); v[1] += bf2f(r.x >> 16);
          v[2] += bf2f(r.y & 0xffff); v[3] += bf2f(r.y >> 16);
          v[4] += bf2f(r.z & 0xffff); v[5] += bf2f(r.z >> 16);
          v[6] += bf2f(r.w & 0xffff); v[7] += bf2f(r.w >> 16);
        }
        if (relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (a.out_f32) {
          float* yp = (float*)ybase + (long)m * ldy + choff;
          *(float4*)yp = make_float4(v[0], v[1], v[2], v[3]);
          *(float4*)(yp + 4) = make_float4(v[4], v[5], v[6], v[7]);
        } else {
          *(uint4*)((unsigned short*)ybase + (long)m * ldy + choff) =
              make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
        }
      }
    }
  }
}

struct Occ {
  int cus = 0;
  int per_cu[64] = {0};
};

template <int BM, int BN, int WM, int WN, int NL, int STAGES, int BK>
static int launch(const DmlConvArgs* a, int id, hipStream_t s) {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK>;
  static Occ occ;  // CU count and resident workgroups per CU of this config (queried once)
  if (occ.cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&occ.cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  int& wpc = occ.per_cu[id & 63];
  if (wpc == 0) {
    int n = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)conv_wsp_kernel<BM, BN, WM, WN, NL, STAGES, BK, false>,
                                                 T::NT, T::LDS);
    wpc = n > 0 ? n : 1;
  }
  const long M = (long)a->N * a->Ho * a->Wo;
  const long tiles = ((M + BM - 1) / BM) * ((a->Cout + BN - 1) / BN);
  long G = (long)occ.cus * wpc;
  G = (G / 8) * 8;
  const long t8 = (tiles + 7) / 8 * 8;
  if (t8 < G) G = t8;
  if (G < 8) G = 8;
  if (a->res)
    hipLaunchKernelGGL((conv_wsp_kernel<BM, BN, WM, WN, NL, STAGES, BK, true>), dim3((unsigned)G), dim3(T::NT),
                       T::LDS, s, *a);
  else
    hipLaunchKernelGGL((conv_wsp_kernel<BM, BN, WM, WN, NL, STAGES, BK, false>), dim3((unsigned)G), dim3(T::NT),
                       T::LDS, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN, int NL, int STAGES, int BK>
static int set_attr() {
  using T = Cfg<BM, BN, WM, WN, NL, STAGES, BK>;
  return (int)hipFuncSetAttribute((const void*)conv_wsp_kernel<BM, BN, WM, WN, NL, STAGES, BK, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS) |
         (int)hipFuncSetAttribute((const void*)conv_wsp_kernel<BM, BN, WM, WN, NL, STAGES, BK, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS);
}

}  // namespace wsp
}  // namespace dml

// Persistent warp-specialised tile configurations: id, BM, BN, WM x WN MFMA waves, NL
// loader waves, ring STAGES, BK. Ids 120..139 (ABI of the tuner, ops/tuning.py WSP_CFGS).
#define DML_WSP_TILES(X)                                                             \
  X(120, 128, 64, 2, 2, 2, 4, 32)   /* 57 KiB: 2 WG/CU */                              \
  X(121, 128, 128, 2, 2, 2, 3, 32)  /* 65 KiB: 2 WG/CU */                              \
  X(122, 128, 128, 2, 2, 4, 3, 64)  /* 113 KiB */                                      \
  X(123, 256, 128, 4, 2, 4, 4, 32)  /* 131 KiB */                                      \
  X(124, 64, 128, 1, 4, 2, 4, 32)   /* 57 KiB: 2 WG/CU */                              \
  X(125, 256, 64, 4, 1, 4, 3, 64)   /* 137 KiB */                                      \
  X(126, 128, 64, 2, 2, 2, 2, 64)   /* 57 KiB: 2 WG/CU */                              \
  X(127, 128, 128, 2, 2, 4, 4, 64)  /* 145 KiB */                                      \
  X(128, 128, 64, 2, 2, 2, 3, 64)   /* 81 KiB */                                       \
  X(129, 64, 128, 1, 4, 2, 2, 64)   /* 57 KiB: 2 WG/CU */

extern "C" int dml_conv_wsp_init(void) {
  using namespace dml::wsp;
  int rc = 0;
#define DML_SET(id, BM, BN, WM, WN, NL, ST, BK) rc |= set_attr<BM, BN, WM, WN, NL, ST, BK>();
  DML_WSP_TILES(DML_SET)
#undef DML_SET
  if (rc) dml_set_error("dml_conv_wsp_init: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  return rc ? -1 : 0;
}

extern "C" int dml_conv_wsp(const DmlConvArgs* a, int cfg, hipStream_t s) {
  using namespace dml::wsp;
  if (a->ksplit > 1) {
    dml_set_error("dml_conv_wsp: the persistent tiles do not split K");
    return -1;
  }
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, NL, ST, BK) \
  case id: return launch<BM, BN, WM, WN, NL, ST, BK>(a, id, s);
    DML_WSP_TILES(DML_CASE)
#undef DML_CASE
    default: dml_set_error("dml_conv_wsp: bad cfg"); return -1;
  }
}

extern "C" int dml_conv_wsp_bn(int cfg) {
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, NL, ST, BK) \
  case id: return BN;
    DML_WSP_TILES(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}
