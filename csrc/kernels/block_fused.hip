// block_fused.hip — a whole ResNet50 identity bottleneck block as ONE kernel (gfx950).
//
//   T1 = relu(W1 . X + b1)            1x1 reduce   C -> F      (convN_blockK_1_conv)
//   T2 = relu(W2 * T1 + b2)           3x3 'same'   F -> F      (convN_blockK_2_conv)
//   Y  = relu(W3 . T2 + b3 + X)       1x1 expand   F -> C, + identity shortcut
//
// (Keras ResNet50 v1, reference models.py:48-51; BN folded into W/b on the host.)
// Unfused, the block moves X (read by the reduce AND as the residual), T1 and T2
// (each written and read back) and Y through HBM: 4 C-channel + 4 F-channel
// tensor passes. Here a workgroup owns a 14x14 output tile of one image: it
// reduces the 16x16 halo of that tile into LDS (T1 never leaves the CU; padding
// pixels are exact zeros), runs the 3x3 from LDS with per-lane shifted-row
// addressing (a tap is a uniform LDS offset, no im2col), keeps T2 in registers
// and streams the expand + shortcut + ReLU straight to Y. HBM traffic: X once
// (its halo and shortcut re-reads hit L2 / the Infinity Cache) and Y once.
//
// Work split (4 waves, 2 workgroups per CU):
//  phase 1  wave w reduces halo rows 4w..4w+3 (4 pixel fragments of 16) x all F
//           channels; operands straight from global/L2 into VGPRs, 2-deep
//           register ring; epilogue: bias + ReLU + out-of-image mask -> bf16 T1
//           rows in LDS (16-B chunks XOR-swizzled by pixel: conflict-free reads)
//  barrier  (the only one: T1 complete, halo included)
//  phase 2  wave w owns output pixel fragments w, w+4, w+8, w+12 (13 fragments of
//           16 cover the 196 pixels) x all F channels: K = 9F, B fragments read
//           from T1 at (pixel + tap offset), W2 fragments from L2
//  phase 3  T2 -> this wave's LDS scratch -> B fragments in VGPRs; expand in
//           64-channel chunks, fp32 staging (per-wave scratch, 32-pixel passes)
//           -> each lane owns 8 channels of a pixel: bias + shortcut (16-B load)
//           + ReLU -> one 16-B store. Phases 2-3 are wave-private (no barrier).
#include <cstdlib>

#include "conv_shared.h"

namespace dml {
namespace blk {

template <int F_>
struct Cfg {
  static constexpr int F = F_, C = 4 * F_;
  static constexpr int TH = 14, TW = 14;        // output tile
  static constexpr int HH = TH + 2, HW = TW + 2; // halo tile
  static constexpr int HP = HH * HW;            // 256 halo pixels
  static constexpr int OP = TH * TW;            // 196 output pixels
  static constexpr int OF = (OP + 15) / 16;     // 13 output pixel fragments
  static constexpr int NW = 4, NT = NW * 64;
  static constexpr int FCH = F / 16;            // 16-channel fragments of F
  static constexpr int ROW = F * 2;             // bf16 T1 / T2 row bytes
  static constexpr int T1B = HP * ROW;
  static constexpr int PFW = 4;                 // pixel fragments per wave (phases 2-3)
  static constexpr int EPX = 32;                // pixels per expand epilogue pass
  static constexpr int SROW = 64 * 4 + 16;      // fp32 staging row (64 channels + pad)
  static constexpr int SCR_T2 = PFW * 16 * ROW;
  static constexpr int SCR_EP = EPX * SROW;
  static constexpr int SCR = SCR_T2 > SCR_EP ? SCR_T2 : SCR_EP;  // per-wave scratch
  static constexpr int LDS = T1B + NW * SCR;
  static constexpr int KS1 = C / 32, KS2 = 9 * F / 32, KS3 = F / 32;
  static_assert(HH == 4 * NW && HW == 16, "phase 1: wave w reduces halo rows 4w..4w+3, one fragment per row");
  static_assert(F % 32 == 0 && ROW >= 128, "T1 rows of >= 8 chunks (swizzle)");
};

// byte offset of 16-B chunk `ch` of bf16 row `px` (row pitch ROW): chunk XOR
// (px & 7), so 16 consecutive pixels reading one chunk hit distinct banks
template <int ROW>
__device__ __forceinline__ int toff(int px, int ch) { return px * ROW + ((ch ^ (px & 7)) << 4); }

__device__ __forceinline__ void wave_lds_sync() {
  // LDS ops of one wave complete in order; the asm keeps the compiler from
  // moving LDS accesses across the hand-off between lanes
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int F>
__global__ __launch_bounds__(256, 2) void block_fused_kernel(DmlBlockArgs a) {
  using T = Cfg<F>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* t1 = smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  char* scr = smem + T::T1B + wid * T::SCR;

  const int tiles_w = (a.W + T::TW - 1) / T::TW, tiles_h = (a.H + T::TH - 1) / T::TH;
  const int per_img = tiles_w * tiles_h;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int n = b / per_img, rem = b - n * per_img;
  const int th = rem / tiles_w, tw = rem - th * tiles_w;
  const int oh0 = th * T::TH, ow0 = tw * T::TW;
  const long img = (long)n * a.H * a.W;
  const bf16* __restrict__ x = (const bf16*)a.x;
  // diagnostics: wave 0 stamps the phase boundaries of its workgroup (real-time
  // 100 MHz clock + shader cycles) into a buffer nothing else reads
  long long* st = a.stamps ? a.stamps + (long)blockIdx.x * 8 : nullptr;
  auto stamp = [&](int i) {
    if (st != nullptr && tid == 0) {
      st[2 * i] = __builtin_amdgcn_s_memrealtime();
      st[2 * i + 1] = __builtin_amdgcn_s_memtime();
    }
  };
  stamp(0);

  // ------------------------------------------------------------- phase 1 --
  const bf16* xp[4];
  bool hv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int h = oh0 - 1 + 4 * wid + j, w = ow0 - 1 + frow;
    hv[j] = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
    const int hc = min(max(h, 0), a.H - 1), wc = min(max(w, 0), a.W - 1);  // any in-image row: result masked
    xp[j] = x + (img + (long)hc * a.W + wc) * a.ldx + fq * 8;
  }
  const bf16* __restrict__ w1p = (const bf16*)a.w1 + (long)frow * a.ldw1 + fq * 8;
  f32x4 acc[T::FCH][4];
#pragma unroll
  for (int i = 0; i < T::FCH; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  {
    // PD-deep register ring: k-steps ks+1 .. ks+PD-1 in flight under step ks's MFMAs
    // (the X rows come from HBM: one k-step of MFMAs is far shorter than the latency)
    constexpr int PD = 3;
    bf16x8 wa[PD][T::FCH], xb[PD][4];
    auto ld = [&](int ks, int buf) {
#pragma unroll
      for (int j = 0; j < 4; ++j) xb[buf][j] = *(const bf16x8*)(xp[j] + ks * 32);
#pragma unroll
      for (int i = 0; i < T::FCH; ++i) wa[buf][i] = *(const bf16x8*)(w1p + (long)i * 16 * a.ldw1 + ks * 32);
    };
#pragma unroll
    for (int s = 0; s < PD - 1; ++s) ld(s, s);
#pragma unroll
    for (int ks = 0; ks < T::KS1; ++ks) {
      if (ks + PD - 1 < T::KS1) ld(ks + PD - 1, (ks + PD - 1) % PD);
#pragma unroll
      for (int i = 0; i < T::FCH; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks % PD][i], xb[ks % PD][j], acc[i][j], 0, 0, 0);
    }
  }
  // bias + ReLU + padding mask -> bf16 T1 (lane: channels 16i + 4fq .. +3 of halo pixel (4w+j, frow))
#pragma unroll
  for (int i = 0; i < T::FCH; ++i) {
    const float4 bb = *(const float4*)(a.b1 + 16 * i + 4 * fq);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = acc[i][j];
      const float m = hv[j] ? 1.f : 0.f;
      const uint2 o = make_uint2(pack2(fmaxf(v[0] + bb.x, 0.f) * m, fmaxf(v[1] + bb.y, 0.f) * m),
                                 pack2(fmaxf(v[2] + bb.z, 0.f) * m, fmaxf(v[3] + bb.w, 0.f) * m));
      const int hp = (4 * wid + j) * T::HW + frow;
      const int ch = 16 * i + 4 * fq;
      *(uint2*)(t1 + toff<T::ROW>(hp, ch >> 3) + (ch & 7) * 2) = o;
    }
  }
  __syncthreads();
  stamp(1);

  // ------------------------------------------------------------- phase 2 --
  const bool has4 = wid + 12 < T::OF;  // wave-uniform: the 13th fragment belongs to wave 0
  int hb[T::PFW];
#pragma unroll
  for (int k = 0; k < T::PFW; ++k) {
    const int op = min(16 * (wid + 4 * k) + frow, T::OP - 1);  // junk lanes read a valid pixel
    const int r = op / T::TW, c = op - r * T::TW;
    hb[k] = r * T::HW + c;
  }
  const bf16* __restrict__ w2p = (const bf16*)a.w2 + (long)frow * a.ldw2 + fq * 8;
#pragma unroll
  for (int i = 0; i < T::FCH; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  {
    constexpr int HF = F / 32;  // 32-channel k-steps per tap
    constexpr int PD = 3;
    bf16x8 wa[PD][T::FCH];
    auto ldw = [&](int ks, int buf) {
#pragma unroll
      for (int i = 0; i < T::FCH; ++i) wa[buf][i] = *(const bf16x8*)(w2p + (long)i * 16 * a.ldw2 + ks * 32);
    };
#pragma unroll
    for (int s = 0; s < PD - 1; ++s) ldw(s, s);
#pragma unroll
    for (int ks = 0; ks < T::KS2; ++ks) {
      if (ks + PD - 1 < T::KS2) ldw(ks + PD - 1, (ks + PD - 1) % PD);
      const int t = ks / HF, hf = ks - t * HF;
      const int tap = (t / 3) * T::HW + (t % 3);
      const int chunk = hf * 4 + fq;
      bf16x8 xb[T::PFW];
#pragma unroll
      for (int k = 0; k < T::PFW; ++k) {
        const int hp = hb[k] + tap;
        xb[k] = *(const bf16x8*)(t1 + toff<T::ROW>(hp, chunk));
      }
#pragma unroll
      for (int i = 0; i < T::FCH; ++i)
#pragma unroll
        for (int k = 0; k < T::PFW; ++k)
          if (k < 3 || has4)
            acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks % PD][i], xb[k], acc[i][k], 0, 0, 0);
    }
  }
  // bias + ReLU -> bf16 T2 rows in this wave's scratch (pixel 16k + frow)
#pragma unroll
  for (int i = 0; i < T::FCH; ++i) {
    const float4 bb = *(const float4*)(a.b2 + 16 * i + 4 * fq);
#pragma unroll
    for (int k = 0; k < T::PFW; ++k) {
      const f32x4 v = acc[i][k];
      const uint2 o = make_uint2(pack2(fmaxf(v[0] + bb.x, 0.f), fmaxf(v[1] + bb.y, 0.f)),
                                 pack2(fmaxf(v[2] + bb.z, 0.f), fmaxf(v[3] + bb.w, 0.f)));
      const int ch = 16 * i + 4 * fq;
      *(uint2*)(scr + toff<T::ROW>(16 * k + frow, ch >> 3) + (ch & 7) * 2) = o;
    }
  }
  wave_lds_sync();
  bf16x8 tb[T::PFW][T::KS3];  // expand B fragments: pixel 16k + frow, K chunk s*4 + fq
#pragma unroll
  for (int k = 0; k < T::PFW; ++k)
#pragma unroll
    for (int s = 0; s < T::KS3; ++s) tb[k][s] = *(const bf16x8*)(scr + toff<T::ROW>(16 * k + frow, s * 4 + fq));
  wave_lds_sync();
  stamp(2);

  // ------------------------------------------------------------- phase 3 --
  // epilogue lane map: channel group cg (8 channels) of staging pixel (lane >> 3) + 8 * it
  const int cg = lane & 7;
  long opix[T::PFW * 16 / 8];  // output pixel (element row) of each epilogue item, -1 = not stored
#pragma unroll
  for (int q = 0; q < T::PFW * 2; ++q) {  // q = pass * 4 + it: staging pixel (lane >> 3) + 8 it of pass
    const int pass = q >> 2, it = q & 3;
    const int pxl = (lane >> 3) + 8 * it;            // 0..31 within the pass
    const int k = 2 * pass + (pxl >> 4);             // the wave's pixel fragment
    const int f = wid + 4 * k;
    const int op = 16 * f + (pxl & 15);
    const int r = op / T::TW, c = op - r * T::TW;
    const int oh = oh0 + r, ow = ow0 + c;
    const bool ok = f < T::OF && op < T::OP && oh < a.H && ow < a.W;
    opix[q] = ok ? img + (long)oh * a.W + ow : -1;
  }
  const bf16* __restrict__ w3p = (const bf16*)a.w3 + (long)frow * a.ldw3 + fq * 8;
  const unsigned short* __restrict__ xs = (const unsigned short*)a.x;
  unsigned short* __restrict__ y = (unsigned short*)a.y;
  // shortcut rows: chunk cc+1's are reloaded as soon as chunk cc's are consumed,
  // so they stream in under the next chunk's MFMAs
  uint4 rr[T::PFW * 2];
#pragma unroll
  for (int q = 0; q < T::PFW * 2; ++q)
    rr[q] = opix[q] >= 0 ? *(const uint4*)(xs + opix[q] * a.ldx + 8 * cg) : make_uint4(0, 0, 0, 0);
#pragma unroll 1
  for (int cc = 0; cc < T::C / 64; ++cc) {
    f32x4 e[4][T::PFW];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < T::PFW; ++k) e[i][k] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < T::KS3; ++s) {
      bf16x8 wa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) wa[i] = *(const bf16x8*)(w3p + (long)(64 * cc + 16 * i) * a.ldw3 + s * 32);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < T::PFW; ++k)
          if (k < 3 || has4) e[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i], tb[k][s], e[i][k], 0, 0, 0);
    }
    const float4 bb0 = *(const float4*)(a.b3 + 64 * cc + 8 * cg);
    const float4 bb1 = *(const float4*)(a.b3 + 64 * cc + 8 * cg + 4);
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          *(f32x4*)(scr + (16 * kk + frow) * T::SROW + (16 * i + 4 * fq) * 4) = e[i][2 * pass + kk];
      wave_lds_sync();
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int q = pass * 4 + it;
        const int pxl = (lane >> 3) + 8 * it;
        const float4 v0 = *(const float4*)(scr + pxl * T::SROW + cg * 32);
        const float4 v1 = *(const float4*)(scr + pxl * T::SROW + cg * 32 + 16);
        const uint4 r = rr[q];
        float f[8] = {v0.x + bb0.x + bf2f(r.x & 0xffff), v0.y + bb0.y + bf2f(r.x >> 16),
                      v0.z + bb0.z + bf2f(r.y & 0xffff), v0.w + bb0.w + bf2f(r.y >> 16),
                      v1.x + bb1.x + bf2f(r.z & 0xffff), v1.y + bb1.y + bf2f(r.z >> 16),
                      v1.z + bb1.z + bf2f(r.w & 0xffff), v1.w + bb1.w + bf2f(r.w >> 16)};
        if (opix[q] >= 0)
          *(uint4*)(y + opix[q] * a.ldy + 64 * cc + 8 * cg) =
              make_uint4(pack2(fmaxf(f[0], 0.f), fmaxf(f[1], 0.f)), pack2(fmaxf(f[2], 0.f), fmaxf(f[3], 0.f)),
                         pack2(fmaxf(f[4], 0.f), fmaxf(f[5], 0.f)), pack2(fmaxf(f[6], 0.f), fmaxf(f[7], 0.f)));
        if (cc + 1 < T::C / 64 && opix[q] >= 0) rr[q] = *(const uint4*)(xs + opix[q] * a.ldx + 64 * (cc + 1) + 8 * cg);
      }
      wave_lds_sync();
    }
  }
  stamp(3);
}

template <int F>
int launch(const DmlBlockArgs* a, hipStream_t s) {
  using T = Cfg<F>;
  const long blocks = (long)a->N * ((a->H + T::TH - 1) / T::TH) * ((a->W + T::TW - 1) / T::TW);
  hipLaunchKernelGGL((block_fused_kernel<F>), dim3((unsigned)blocks), dim3(T::NT), T::LDS, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int F>
int set_attr() {
  return (int)hipFuncSetAttribute((const void*)block_fused_kernel<F>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  Cfg<F>::LDS);
}


// ===================================================================================
// Persistent, warp-specialised form (the default): phase 1 of tile t+1 runs beside
// phases 2-3 of tile t in the SAME workgroup.
//
// The phase-serialised kernel above measured 283 us per 128 images (stage 2), every
// phase latency-bound: all resident workgroups start in phase 1 together, so HBM is
// read in bursts and idles while every CU sits in the 3x3 (profiles/r3_v1 stamps:
// phase 1 16 us, 3x3 12 us, expand 26 us per workgroup). Here one 768-thread
// workgroup per CU loops over tiles with two roles:
//   producers (waves 0-4)  reduce the halo of tile t+1 into T1 buffer (t+1) & 1:
//                          X straight from HBM into VGPRs (3-deep register ring)
//   consumers (waves 5-11) 3x3 over T1 buffer t & 1 + expand + shortcut + store Y
// and ONE s_barrier per tile (T1 is double-buffered), so the HBM read stream
// (producers) overlaps the MFMA work and the store stream (consumers) of the
// previous tile on every CU, all the time. Tile = 8 x 28 output pixels (14 pixel
// fragments, two per consumer wave), halo 10 x 30 (19 fragments over 5 producers).
// Tiles: each XCD owns a contiguous range, dealt round-robin to its workgroups, so
// neighbouring tiles (which share halo rows) run at the same time in one L2.
template <int F_>
struct WsCfg {
  static constexpr int F = F_, C = 4 * F_;
  static constexpr int TH = 8, TW = 28;            // output tile
  static constexpr int HH = TH + 2, HW = TW + 2;   // halo tile
  static constexpr int HP = HH * HW;               // 300 halo pixels
  static constexpr int HFR = (HP + 15) / 16;       // 19 halo fragments
  static constexpr int OP = TH * TW;               // 224 output pixels
  static constexpr int OF = OP / 16;               // 14 output fragments
  static constexpr int NP = 5, NQ = 7, NW = NP + NQ, NT = NW * 64;
  static constexpr int PF = (HFR + NP - 1) / NP;   // 4 halo fragments per producer wave
  static constexpr int QF = OF / NQ;               // 2 output fragments per consumer wave
  static constexpr int FCH = F / 16;
  static constexpr int ROW = F * 2;
  static constexpr int T1B = HFR * 16 * ROW;       // one T1 buffer (304 rows)
  static constexpr int SROW = 64 * 4 + 16, EPX = QF * 16;
  static constexpr int SCR_T2 = QF * 16 * ROW, SCR_EP = EPX * SROW;
  static constexpr int SCR = SCR_T2 > SCR_EP ? SCR_T2 : SCR_EP;
  static constexpr int LDS = 2 * T1B + NQ * SCR;
  static constexpr int KS1 = C / 32, KS2 = 9 * F / 32, KS3 = F / 32;
  static_assert(OP % 16 == 0 && OF % NQ == 0 && ROW >= 128, "tile / role split");
  static_assert(LDS <= 163840, "one workgroup per CU");
};

__device__ __forceinline__ void lds_barrier() {
  // producers' T1 writes (ds_write) done, then the rendezvous; global loads and
  // stores stay in flight across it (no vmcnt wait)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

template <int F>
__global__ __launch_bounds__(WsCfg<F>::NT, 1) void block_ws_kernel(DmlBlockArgs a, int total) {
  using T = WsCfg<F>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const bool producer = wid < T::NP;
  const int tiles_w = (a.W + T::TW - 1) / T::TW, tiles_h = (a.H + T::TH - 1) / T::TH;
  const int per_img = tiles_w * tiles_h;
  // contiguous tile range per XCD (workgroup b runs on XCD b % 8), dealt round-robin
  const int G = gridDim.x, x8 = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int gx = (G >> 3) + ((G & 7) > x8 ? 1 : 0);                  // workgroups on this XCD
  const int t_lo = (int)((long)total * x8 / 8), t_hi = (int)((long)total * (x8 + 1) / 8);
  const int my_tiles = slot < gx ? (t_hi - t_lo - slot + gx - 1) / gx : 0;
  // every workgroup runs the same iteration count (the barrier count must match):
  // the largest share; surplus iterations do no work
  const int per_xcd_max = (total + 7) / 8;
  const int iters = (per_xcd_max + (G >> 3) - 1) / max(G >> 3, 1);
  auto tile_of = [&](int j) { return j < my_tiles ? t_lo + slot + j * gx : -1; };

  const bf16* __restrict__ x = (const bf16*)a.x;
  const unsigned short* __restrict__ xs = (const unsigned short*)a.x;
  unsigned short* __restrict__ y = (unsigned short*)a.y;

  // ---------------------------------------------------------- producer --
  auto produce = [&](int t, char* t1) {
    const int n = t / per_img, rem = t - n * per_img;
    const int th = rem / tiles_w, tw = rem - th * tiles_w;
    const long img = (long)n * a.H * a.W;
    const bf16* __restrict__ w1p = (const bf16*)a.w1 + (long)frow * a.ldw1 + fq * 8;
    // two passes of PF / 2 halo fragments: half the accumulators and X ring live at
    // once (W1 is streamed from L2 twice), so the union with the consumer code fits
    // the 168 VGPRs of 3 waves per SIMD without spilling
    constexpr int PP = T::PF / 2;
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
      const bf16* xp[PP];
      float mk[PP];
      int hps[PP];
#pragma unroll
      for (int k = 0; k < PP; ++k) {
        const int hf = min(wid + T::NP * (PP * pass + k), T::HFR - 1);  // a duplicate when past the end: never stored
        const int hp = 16 * hf + frow;
        const int hr = hp / T::HW, hc = hp - hr * T::HW;
        const int h = th * T::TH - 1 + hr, w = tw * T::TW - 1 + hc;
        const bool ok = hp < T::HP && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        mk[k] = ok ? 1.f : 0.f;
        hps[k] = hp;
        const int hcl = min(max(h, 0), a.H - 1), wcl = min(max(w, 0), a.W - 1);
        xp[k] = x + (img + (long)hcl * a.W + wcl) * a.ldx + fq * 8;
      }
      f32x4 acc[T::FCH][PP];
#pragma unroll
      for (int i = 0; i < T::FCH; ++i)
#pragma unroll
        for (int k = 0; k < PP; ++k) acc[i][k] = (f32x4){0.f, 0.f, 0.f, 0.f};
      // k-steps in a rolled loop with explicit register buffers (a fully unrolled
      // ring lets the scheduler hoist every load: 129 VGPRs of spills measured);
      // X two k-steps ahead (HBM latency), W1 one ahead (L2)
      bf16x8 x0[PP], x1[PP], x2[PP], w0[T::FCH], w1[T::FCH];
      auto ldx = [&](bf16x8 (&d)[PP], int ks) {
#pragma unroll
        for (int k = 0; k < PP; ++k) d[k] = *(const bf16x8*)(xp[k] + ks * 32);
      };
      auto ldw = [&](bf16x8 (&d)[T::FCH], int ks) {
#pragma unroll
        for (int i = 0; i < T::FCH; ++i) d[i] = *(const bf16x8*)(w1p + (long)i * 16 * a.ldw1 + ks * 32);
      };
      ldx(x0, 0);
      ldx(x1, 1);
      ldw(w0, 0);
#pragma unroll 1
      for (int ks = 0; ks < T::KS1; ++ks) {
        if (ks + 2 < T::KS1) ldx(x2, ks + 2);
        if (ks + 1 < T::KS1) ldw(w1, ks + 1);
#pragma unroll
        for (int i = 0; i < T::FCH; ++i)
#pragma unroll
          for (int k = 0; k < PP; ++k)
            acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[i], x0[k], acc[i][k], 0, 0, 0);
#pragma unroll
        for (int k = 0; k < PP; ++k) {
          x0[k] = x1[k];
          x1[k] = x2[k];
        }
#pragma unroll
        for (int i = 0; i < T::FCH; ++i) w0[i] = w1[i];
      }
#pragma unroll
      for (int i = 0; i < T::FCH; ++i) {
        const float4 bb = *(const float4*)(a.b1 + 16 * i + 4 * fq);
#pragma unroll
        for (int k = 0; k < PP; ++k) {
          if (wid + T::NP * (PP * pass + k) >= T::HFR) continue;  // wave-uniform
          const f32x4 v = acc[i][k];
          const float m = mk[k];
          const uint2 o = make_uint2(pack2(fmaxf(v[0] + bb.x, 0.f) * m, fmaxf(v[1] + bb.y, 0.f) * m),
                                     pack2(fmaxf(v[2] + bb.z, 0.f) * m, fmaxf(v[3] + bb.w, 0.f) * m));
          const int ch = 16 * i + 4 * fq;
          *(uint2*)(t1 + toff<T::ROW>(hps[k], ch >> 3) + (ch & 7) * 2) = o;
        }
      }
    }
  };

  // ---------------------------------------------------------- consumer --
  const int q = wid - T::NP;
  char* scr = smem + 2 * T::T1B + (producer ? 0 : q) * T::SCR;
  auto consume = [&](int t, const char* t1) {
    const int n = t / per_img, rem = t - n * per_img;
    const int th = rem / tiles_w, tw = rem - th * tiles_w;
    const long img = (long)n * a.H * a.W;
    const int oh0 = th * T::TH, ow0 = tw * T::TW;
    int hb[T::QF];
#pragma unroll
    for (int k = 0; k < T::QF; ++k) {
      const int op = 16 * (T::QF * q + k) + frow;
      const int r = op / T::TW, c = op - r * T::TW;
      hb[k] = r * T::HW + c;
    }
    // 3x3 from T1 (per-lane shifted rows: a tap is a uniform offset)
    const bf16* __restrict__ w2p = (const bf16*)a.w2 + (long)frow * a.ldw2 + fq * 8;
    f32x4 acc[T::FCH][T::QF];
#pragma unroll
    for (int i = 0; i < T::FCH; ++i)
#pragma unroll
      for (int k = 0; k < T::QF; ++k) acc[i][k] = (f32x4){0.f, 0.f, 0.f, 0.f};
    {
      // rolled over the 9 taps; a tap's weights (HF k-steps) are loaded one tap ahead
      constexpr int HF = F / 32;
      bf16x8 wc[HF][T::FCH], wn[HF][T::FCH];
      auto ldw = [&](bf16x8 (&d)[HF][T::FCH], int tp) {
#pragma unroll
        for (int hf = 0; hf < HF; ++hf)
#pragma unroll
          for (int i = 0; i < T::FCH; ++i)
            d[hf][i] = *(const bf16x8*)(w2p + (long)i * 16 * a.ldw2 + (tp * HF + hf) * 32);
      };
      ldw(wc, 0);
#pragma unroll 1
      for (int tp = 0; tp < 9; ++tp) {
        if (tp + 1 < 9) ldw(wn, tp + 1);
        const int tap = (tp / 3) * T::HW + (tp % 3);
#pragma unroll
        for (int hf = 0; hf < HF; ++hf) {
          bf16x8 xb[T::QF];
#pragma unroll
          for (int k = 0; k < T::QF; ++k) xb[k] = *(const bf16x8*)(t1 + toff<T::ROW>(hb[k] + tap, hf * 4 + fq));
#pragma unroll
          for (int i = 0; i < T::FCH; ++i)
#pragma unroll
            for (int k = 0; k < T::QF; ++k)
              acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wc[hf][i], xb[k], acc[i][k], 0, 0, 0);
        }
#pragma unroll
        for (int hf = 0; hf < HF; ++hf)
#pragma unroll
          for (int i = 0; i < T::FCH; ++i) wc[hf][i] = wn[hf][i];
      }
    }
    // epilogue items: staging pixel (lane >> 3) + 8 it of the wave's 32, channel group lane & 7
    const int cg = lane & 7;
    long opix[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int pxl = (lane >> 3) + 8 * it;
      const int op = 16 * T::QF * q + pxl;
      const int r = op / T::TW, c = op - r * T::TW;
      const int oh = oh0 + r, ow = ow0 + c;
      opix[it] = (oh < a.H && ow < a.W) ? img + (long)oh * a.W + ow : -1;
    }
    // shortcut rows of chunk 0, issued now: in flight under the T2 round trip and chunk 0's MFMAs (loaded during the 3x3 they cost 24 VGPRs)
    uint4 rr[4];
#pragma unroll
    for (int it = 0; it < 4; ++it)
      rr[it] = opix[it] >= 0 ? *(const uint4*)(xs + opix[it] * a.ldx + 8 * cg) : make_uint4(0, 0, 0, 0);
    // T2 = bias + ReLU -> bf16 rows in this wave's scratch -> expand B fragments
#pragma unroll
    for (int i = 0; i < T::FCH; ++i) {
      const float4 bb = *(const float4*)(a.b2 + 16 * i + 4 * fq);
#pragma unroll
      for (int k = 0; k < T::QF; ++k) {
        const f32x4 v = acc[i][k];
        const uint2 o = make_uint2(pack2(fmaxf(v[0] + bb.x, 0.f), fmaxf(v[1] + bb.y, 0.f)),
                                   pack2(fmaxf(v[2] + bb.z, 0.f), fmaxf(v[3] + bb.w, 0.f)));
        const int ch = 16 * i + 4 * fq;
        *(uint2*)(scr + toff<T::ROW>(16 * k + frow, ch >> 3) + (ch & 7) * 2) = o;
      }
    }
    wave_lds_sync();
    bf16x8 tb[T::QF][T::KS3];
#pragma unroll
    for (int k = 0; k < T::QF; ++k)
#pragma unroll
      for (int s = 0; s < T::KS3; ++s) tb[k][s] = *(const bf16x8*)(scr + toff<T::ROW>(16 * k + frow, s * 4 + fq));
    wave_lds_sync();
    // expand in 64-channel chunks + shortcut + ReLU -> Y
    const bf16* __restrict__ w3p = (const bf16*)a.w3 + (long)frow * a.ldw3 + fq * 8;
#pragma unroll 1
    for (int cc = 0; cc < T::C / 64; ++cc) {
      f32x4 e[4][T::QF];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < T::QF; ++k) e[i][k] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < T::KS3; ++s) {
        bf16x8 wa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) wa[i] = *(const bf16x8*)(w3p + (long)(64 * cc + 16 * i) * a.ldw3 + s * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int k = 0; k < T::QF; ++k) e[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i], tb[k][s], e[i][k], 0, 0, 0);
      }
      const float4 bb0 = *(const float4*)(a.b3 + 64 * cc + 8 * cg);
      const float4 bb1 = *(const float4*)(a.b3 + 64 * cc + 8 * cg + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < T::QF; ++k)
          *(f32x4*)(scr + (16 * k + frow) * T::SROW + (16 * i + 4 * fq) * 4) = e[i][k];
      wave_lds_sync();
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int pxl = (lane >> 3) + 8 * it;
        const float4 v0 = *(const float4*)(scr + pxl * T::SROW + cg * 32);
        const float4 v1 = *(const float4*)(scr + pxl * T::SROW + cg * 32 + 16);
        const uint4 r = rr[it];
        float f[8] = {v0.x + bb0.x + bf2f(r.x & 0xffff), v0.y + bb0.y + bf2f(r.x >> 16),
                      v0.z + bb0.z + bf2f(r.y & 0xffff), v0.w + bb0.w + bf2f(r.y >> 16),
                      v1.x + bb1.x + bf2f(r.z & 0xffff), v1.y + bb1.y + bf2f(r.z >> 16),
                      v1.z + bb1.z + bf2f(r.w & 0xffff), v1.w + bb1.w + bf2f(r.w >> 16)};
        if (opix[it] >= 0)
          *(uint4*)(y + opix[it] * a.ldy + 64 * cc + 8 * cg) =
              make_uint4(pack2(fmaxf(f[0], 0.f), fmaxf(f[1], 0.f)), pack2(fmaxf(f[2], 0.f), fmaxf(f[3], 0.f)),
                         pack2(fmaxf(f[4], 0.f), fmaxf(f[5], 0.f)), pack2(fmaxf(f[6], 0.f), fmaxf(f[7], 0.f)));
        if (cc + 1 < T::C / 64 && opix[it] >= 0)
          rr[it] = *(const uint4*)(xs + opix[it] * a.ldx + 64 * (cc + 1) + 8 * cg);
      }
      wave_lds_sync();
    }
  };

  // ---------------------------------------------------------- schedule --
  // prologue: T1 of the first tile; then one barrier per tile. The two roles run
  // separate loops with the same barrier count, so each role's loop-invariant
  // values stay out of the other's register budget (one shared loop spilled 49
  // VGPRs although either role alone fits the 168 of 3 waves per SIMD).
  if (producer) {
    if (tile_of(0) >= 0) produce(tile_of(0), smem);
    lds_barrier();
#pragma unroll 1
    for (int j = 0; j < iters; ++j) {
      const int tn = tile_of(j + 1);
      if (tn >= 0) produce(tn, smem + ((j + 1) & 1) * T::T1B);
      lds_barrier();
    }
  } else {
    lds_barrier();
#pragma unroll 1
    for (int j = 0; j < iters; ++j) {
      const int t = tile_of(j);
      if (t >= 0) consume(t, smem + (j & 1) * T::T1B);
      lds_barrier();
    }
  }
}

static int cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <int F>
int launch_ws(const DmlBlockArgs* a, hipStream_t s) {
  using T = WsCfg<F>;
  const int total = a->N * ((a->H + T::TH - 1) / T::TH) * ((a->W + T::TW - 1) / T::TW);
  const int grid = max(8, min(cu_count(), ((total + 7) / 8) * 8));
  hipLaunchKernelGGL((block_ws_kernel<F>), dim3((unsigned)grid), dim3(T::NT), T::LDS, s, *a, total);
  DML_CHECK_LAUNCH();
  return 0;
}

}  // namespace blk
}  // namespace dml

extern "C" int dml_block_fused_init(void) {
  const int rc = dml::blk::set_attr<64>() |
                 (int)hipFuncSetAttribute((const void*)dml::blk::block_ws_kernel<64>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, dml::blk::WsCfg<64>::LDS);
  if (rc) dml_set_error("dml_block_fused_init: hipFuncSetAttribute failed");
  return rc ? -1 : 0;
}

extern "C" int dml_block_fused(const DmlBlockArgs* a, hipStream_t s) {
  const int F = a->F, C = 4 * a->F;
  if (F != 64 || a->N < 1 || a->H < 1 || a->W < 1 || a->ldx % 8 || a->ldx < C || a->ldy % 8 || a->ldy < C ||
      a->ldw1 % 8 || a->ldw1 < C || a->ldw2 % 8 || a->ldw2 < 9 * F || a->ldw3 % 8 || a->ldw3 < F ||
      a->x == a->y) {
    dml_set_error("dml_block_fused: unsupported shape (F = 64, C = 4F, 8-aligned strides, y != x)");
    return -1;
  }
  return a->kernel == 1 ? dml::blk::launch<64>(a, s) : dml::blk::launch_ws<64>(a, s);
}
