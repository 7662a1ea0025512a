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
// and while it runs the loaders fetch the 4 rows tile i + 1 adds (the ring then holds exactly
// both tiles' rows). Every input pixel is loaded ONCE per strip instead of 9 x per tap, the
// weights once per workgroup, and one barrier per tile covers 9 taps x 2 k-steps of MFMAs.
// 4 MFMA waves (2 x 2: 112 pixels x 32 channels each) + 2 loader waves; the epilogue is
// wave-private (8-pixel staging passes, no workgroup barrier), as in conv_igemm_wsp.hip.
//
// K order: tap-major then channel, as v2 (Cin = 64 is one chunk). The launcher refuses anything but 3x3 / pad 1 / stride 1, Cin 64, Cout <= 64,
// W = Wo = 56, no split-K.
//
// Reference compute: the Keras convolutions of models.py:48-69 (ResNet50).
#include "conv_shared.h"

namespace dml {
namespace rr {

using convk::lds_void;
using convk::wait_vmcnt;

constexpr int W56 = 56;                 // image width (= output width)
constexpr int TH = 4;                   // output rows per tile
constexpr int BM = TH * W56;            // 224 pixels per tile
constexpr int RING = 2 * TH + 2;        // image rows resident: a tile's 6 + the next tile's 4
constexpr int SLOT = 64;                // LDS rows per image row: zero column, 56 pixels, zero column, pad
constexpr int ROWB = 128;               // 64 channels of bf16
constexpr int WROWS = 9 * 64;           // weight LDS rows: [tap][cout]
constexpr int W_BYTES = WROWS * ROWB;   // 72 KiB
constexpr int RING_BYTES = RING * SLOT * ROWB;  // 80 KiB
constexpr int NC = 4, NL = 2, NT = (NC + NL) * 64;
constexpr int WTP = 112, WTC = 32, FJ = WTP / 16, FI = WTC / 16;
constexpr int SROW = WTC * 4 + 16;      // fp32 staging row pitch
constexpr int EPW = 8 * SROW;           // staging per MFMA wave: 8 pixels
constexpr int LDS = W_BYTES + RING_BYTES + NC * EPW;
static_assert(LDS <= 163840, "LDS");
constexpr int WPL = WROWS / 8 / NL;     // weight pieces (8 LDS rows) per loader lane
constexpr int RPL = TH * SLOT / 8 / NL; // ring pieces per loader lane per tile (4 image rows)

__device__ __forceinline__ int swz(int row, int ch) { return row * ROWB + ((ch ^ (row & 7)) << 4); }

// PROBE (timing probes only, cfg 156 / 157; wrong outputs): 1 = no output stores, 2 = no row
// loads after the strip's first tile
template <bool RES, bool PIPE, int PROBE = 0>
__global__ __launch_bounds__(NT) void conv_rr_kernel(DmlConvArgs a, int strips) {
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
    const unsigned OOB = 0x80000000u;
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
      if (PROBE != 2 && t + 1 < t1) rows((t + 1) * TH + 1, TH);  // tile t+1's new rows: the slots tile t-1 alone used
    }
    return;
  }

  // ================================== MFMA wave ==================================
  const int wc = wid & 1, wp = wid >> 1;
  const int frow = lane & 15, fq = lane >> 4;
  char* stg = smem + W_BYTES + RING_BYTES + wid * EPW;
  int ohl[FJ], col[FJ];
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int p = wp * WTP + j * 16 + frow;
    ohl[j] = p / W56;
    col[j] = p - ohl[j] * W56;  // LDS column of input pixel (ow - 1) = ow: the left zero column is 0
  }
  const int c0 = wc * WTC;
  const int cg = lane & 3, pr = lane >> 2;  // read-back: channel group (8 ch), pixel (0..15; < 8 used)
  const int ch = c0 + cg * 8;
  const bool ch_ok = ch < a.Cout;
  float4 bias0 = make_float4(0.f, 0.f, 0.f, 0.f), bias1 = bias0;
  if (ch_ok) {
    bias0 = *(const float4*)(a.bias + ch);
    bias1 = *(const float4*)(a.bias + ch + 4);
  }
  if constexpr (PIPE) {
    // fragment-pipelined taps (the next tap's 18 fragments load while this tap's 28 MFMAs run:
    // one MFMA wave per SIMD cannot hide a read latency behind another wave) and a direct
    // epilogue from the accumulators (no LDS round trip; lane: 4 channels of one pixel)
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
      uint2 rv[RES ? FI : 1][RES ? FJ : 1];
      if constexpr (RES) {  // residual rows of this tile: in flight during the MFMAs
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
      f32x4 acc[FI][FJ];
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = (f32x4)(0.f);
      __builtin_amdgcn_s_barrier();
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
      // the compiler otherwise reads each fragment just before its MFMA and waits on it (one
      // wave per SIMD: nothing hides that latency): pin the interleave — tap 0's reads, then
      // per tap one next-tap read after each of the first NR MFMAs
      constexpr int NR = 2 * (FI + FJ), NM = 2 * FI * FJ;
      __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (tap < 8) {
#pragma unroll
          for (int k = 0; k < NR; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int lp = wp * WTP + j * 16 + frow;
        if (PROBE == 1 || lp >= cnt) continue;
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
    }
    return;
  }
  for (int t = t0; t < t1; ++t) {
    f32x4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = (f32x4)(0.f);
    __builtin_amdgcn_s_barrier();
    const int r0 = t * TH;  // first output row of the tile
    const int s0 = (r0 - 1 - gbase) % RING;
#pragma unroll 1
    for (int r = 0; r < 3; ++r) {
      int rb[FJ];
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        int sl = s0 + ohl[j] + r;
        sl = sl >= RING ? sl - RING : sl;
        rb[j] = sl * SLOT + col[j];
      }
#pragma unroll
      for (int sx = 0; sx < 3; ++sx) {
        const char* wt = wl + (r * 3 + sx) * 64 * ROWB;
        bf16x8 fa[2][FI], fb[2][FJ];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int c = ks * 4 + fq;
#pragma unroll
          for (int i = 0; i < FI; ++i) fa[ks][i] = *(const bf16x8*)(wt + swz(c0 + i * 16 + frow, c));
#pragma unroll
          for (int j = 0; j < FJ; ++j) fb[ks][j] = *(const bf16x8*)(ring + swz(rb[j] + sx, c));
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < FI; ++i)
#pragma unroll
            for (int j = 0; j < FJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // ---- epilogue (this wave only), 8 pixels per staging pass ----
    const int m0 = n * HW + r0 * a.W;
    const int cnt = min(TH, a.Ho - r0) * a.W;
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if ((frow >> 3) == h) {
#pragma unroll
          for (int i = 0; i < FI; ++i) *(f32x4*)(stg + (frow & 7) * SROW + (i * 16 + fq * 4) * 4) = acc[i][j];
        }
        const int lp = wp * WTP + j * 16 + h * 8 + pr;  // tile pixel of this lane's read-back
        if (pr < 8 && lp < cnt && ch_ok) {
          const float4 v0 = *(const float4*)(stg + pr * SROW + cg * 32);
          const float4 v1 = *(const float4*)(stg + pr * SROW + cg * 32 + 16);
          const long m = m0 + lp;
          float v[8] = {v0.x + bias0.x, v0.y + bias0.y, v0.z + bias0.z, v0.w + bias0.w,
                        v1.x + bias1.x, v1.y + bias1.y, v1.z + bias1.z, v1.w + bias1.w};
          if constexpr (RES) {
            const uint4 rv = *(const uint4*)((const unsigned short*)a.res + m * a.ldr + ch);
            v[0] += bf2f(rv.x & 0xffff); v[1] += bf2f(rv.x >> 16);
            v[2] += bf2f(rv.y & 0xffff); v[3] += bf2f(rv.y >> 16);
            v[4] += bf2f(rv.z & 0xffff); v[5] += bf2f(rv.z >> 16);
            v[6] += bf2f(rv.w & 0xffff); v[7] += bf2f(rv.w >> 16);
          }
          if (a.relu) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          if (a.out_f32) {
            float* yp = (float*)a.y + m * a.ldy + ch;
            *(float4*)yp = make_float4(v[0], v[1], v[2], v[3]);
            *(float4*)(yp + 4) = make_float4(v[4], v[5], v[6], v[7]);
          } else {
            *(uint4*)((unsigned short*)a.y + m * a.ldy + ch) =
                make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
          }
        }
      }
    }
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
  const auto set = [](const void* f) { return (int)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS); };
  const int rc = set((const void*)conv_rr_kernel<true, false>) | set((const void*)conv_rr_kernel<false, false>) |
                 set((const void*)conv_rr_kernel<true, true>) | set((const void*)conv_rr_kernel<false, true>) |
                 set((const void*)conv_rr_kernel<false, true, 1>) | set((const void*)conv_rr_kernel<false, true, 2>);
  if (rc) dml_set_error("dml_conv_rr_init: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  return rc ? -1 : 0;
}

extern "C" int dml_conv_rr_fits(const DmlConvArgs* a) { return rr_fits(a) ? 1 : 0; }

// cfg 150 / 151 / 152: 2 / 1 / 4 strips per image (ResNet50 b128 at 2: 256 workgroups), LDS-staged
// epilogue; 153 / 154 / 155: the same with fragment-pipelined taps and the direct epilogue
extern "C" int dml_conv_rr(const DmlConvArgs* a, int cfg, hipStream_t s) {
  using namespace dml::rr;
  if (!rr_fits(a) || cfg < 150 || cfg > 157) {
    dml_set_error("dml_conv_rr: needs 3x3 pad 1 stride 1, Cin 64, Cout <= 64, width 56, no split-K / segments");
    return -1;
  }
  const int ntile = (a->Ho + TH - 1) / TH;
  const int v = cfg >= 156 ? 0 : (cfg - 150) % 3;
  const bool pipe = cfg >= 153;
  const int strips = v == 1 ? 1 : (v == 0 ? 2 : 4);
  const int sp = strips < ntile ? strips : ntile;
  const unsigned grid = (unsigned)(a->N * sp);
  const void* k = cfg == 156 ? (const void*)conv_rr_kernel<false, true, 1>
                : cfg == 157 ? (const void*)conv_rr_kernel<false, true, 2>
                : a->res ? (pipe ? (const void*)conv_rr_kernel<true, true> : (const void*)conv_rr_kernel<true, false>)
                         : (pipe ? (const void*)conv_rr_kernel<false, true> : (const void*)conv_rr_kernel<false, false>);
  DmlConvArgs args = *a;
  void* kargs[] = {(void*)&args, (void*)&sp};
  hipLaunchKernel(k, dim3(grid), dim3(NT), kargs, LDS, s);
  DML_CHECK_LAUNCH();
  return 0;
}
