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

}  // namespace blk
}  // namespace dml

extern "C" int dml_block_fused_init(void) {
  const int rc = dml::blk::set_attr<64>();
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
  return dml::blk::launch<64>(a, s);
}
