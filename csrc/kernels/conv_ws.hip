// conv_ws.hip — persistent weight-stationary 1x1 convolution (gfx950).
//
// The v2 tile kernel (conv_igemm_v2.hip) waits on its global -> LDS operand stream
// (DESIGN.md §2 phase probes), and on a 1x1 conv every one of its workgroups
// (a) re-streams its channel tile's BN x K weight panel from L2 next to the
// activations and (b) starts its LDS ring from empty, K/64 = 1..16 tiles deep, so
// most of a workgroup's life is prologue latency. Here a grid of (CUs x
// workgroups per CU) persistent workgroups each:
//   * loads its BN x K weight panel into LDS ONCE (LDS-DMA, the v2 swizzle) and
//     keeps it resident: only activation rows stream afterwards;
//   * runs ONE continuous LDS-DMA ring over the flattened (pixel tile, K tile)
//     sequence of its tiles, so the next tile's first K tiles are in flight while
//     the current tile's last K tiles are multiplied;
//   * stores each finished tile straight from the accumulators (lane: 4
//     consecutive output channels of one pixel -> one 8-B store; bias, residual,
//     ReLU in registers), so the epilogue never touches the ring or a barrier.
// Same MFMA operand order and the same fp32 epilogue arithmetic as the v2 tiles:
// outputs are bit-identical to any v2 config (tests/test_conv_ws_gpu.py).
// Scope: 1x1 stride-1 unpadded convs with K = Cin a multiple of 64, bf16 output,
// no output segments / split-K / subsampled residual (dml_conv_ws_check); cfg ids
// 84.. (DML_WS_TILES) are tuner candidates of those convs (ops/tuning.py).
#include "conv_shared.h"

namespace dml {
namespace ws {

using convk::lds_swz;
using convk::lds_void;
using convk::wait_vmcnt;

constexpr int kLds = 163840;  // LDS per CU

template <int BM, int BN, int WM, int WN, int STAGES>
struct WsCfg {
  static constexpr int NW = WM * WN;
  static constexpr int NT = NW * 64;
  static constexpr int WTP = BM / WM;          // pixels per wave
  static constexpr int WTC = BN / WN;          // channels per wave
  static constexpr int FJ = WTP / 16;          // 16x16 fragments along pixels
  static constexpr int FI = WTC / 16;          // ... along channels
  static constexpr int XI = BM / 8 / NW;       // activation DMA wave-instructions per K tile
  static constexpr int STAGE_BYTES = BM * 128; // BM rows x 64 bf16
  static constexpr int RING = STAGES * STAGE_BYTES;
  static constexpr int NV = (STAGES - 2) * XI; // vm ops younger than the awaited K tile
  static_assert(STAGES >= 3, "ring depth");
  static_assert(XI >= 1 && BM % (8 * NW) == 0, "activation rows must split evenly across waves");
  static_assert(FI >= 1 && FJ >= 1 && WTP % 16 == 0 && WTC % 16 == 0, "wave tile");
  static_assert(BN % 8 == 0 && NV < 48, "weight pieces / vmcnt range");
  static int lds(int nk) { return RING + nk * BN * 128; }
};

template <int BM, int BN, int WM, int WN, int STAGES, bool RES>
__global__ __launch_bounds__(WM* WN * 64) void conv_ws_kernel(DmlConvArgs a) {
  using T = WsCfg<BM, BN, WM, WN, STAGES>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const wl = smem + T::RING;  // resident weight panel: K tile kt at wl + kt * BN * 128

  const int M = a.N * a.Ho * a.Wo;
  const int ntc = (a.Cout + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int G = gridDim.x, P = G / ntc;  // the launch makes G a multiple of ntc
  // XCD-aware: consecutive logical ids (the ntc channel tiles of one pixel-tile
  // stream) share an XCD and so the activation rows in its L2
  const int Lb = xcd_remap(blockIdx.x, G);
  const int tc = Lb % ntc, p = Lb / ntc;
  const int c0 = tc * BN;
  const int nk = a.Kpad >> 6;
  const int total = (p < ntm ? (ntm - 1 - p) / P + 1 : 0) * nk;  // K tiles this workgroup streams

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;  // v2 source-side swizzle (Rows<64>)
  const int wc = wid % WN, wp = wid / WN;
  const int frow = lane & 15, fq = lane >> 4;

  // bias of this lane's 4-channel groups, completed before the loop (the
  // compiler's wait for it must not land inside the K loop)
  float4 bias[T::FI];
#pragma unroll
  for (int i = 0; i < T::FI; ++i) {
    const int ch = c0 + wc * T::WTC + i * 16 + fq * 4;
    bias[i] = ch < a.Cout ? *(const float4*)(a.bias + ch) : make_float4(0.f, 0.f, 0.f, 0.f);
    asm volatile("" ::"v"(bias[i].x), "v"(bias[i].y), "v"(bias[i].z), "v"(bias[i].w));
  }

  // resident weights: nk x BN/8 one-KiB pieces dealt over the waves
  const int wpieces = nk * (BN / 8);
  for (int q = wid; q < wpieces; q += T::NW) {
    const int kt = q / (BN / 8), rg = q - kt * (BN / 8);
    const char* src = (const char*)a.w + ((long)(c0 + rg * 8 + lrow) * a.Kpad + kt * 64 + lchunk * 8) * 2;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(wl + kt * BN * 128 + rg * 1024), 16, 0, 0);
  }

  // activation stream: issue cursor (pixel tile is_tm, K tile is_kt)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
  const unsigned OOB = 0x80000000u;
  int is_tm = p, is_kt = 0;
  auto issue = [&](int stage) {
    char* sx = smem + stage * T::STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < T::XI; ++j) {
      const int m = is_tm * BM + (wid * T::XI + j) * 8 + lrow;
      const unsigned ok = m < M;
      const unsigned msk = 0u - ok;  // branch-free select (no exec split around the DMA)
      const unsigned off = ((unsigned)(m * a.ldx + is_kt * 64 + lchunk * 8) * 2u & msk) | (OOB & ~msk);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void*)(sx + (wid * T::XI + j) * 1024), 16, off, 0, 0, 0);
    }
    if (++is_kt == nk) {
      is_kt = 0;
      is_tm += P;
    }
  };
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < total) issue(s);

  f32x4 acc[T::FI][T::FJ];
#pragma unroll
  for (int i = 0; i < T::FI; ++i)
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) acc[i][j] = (f32x4)(0.f);

  const unsigned short* __restrict__ rg = (const unsigned short*)a.res;
  uint2 rres[RES ? T::FI : 1][RES ? T::FJ : 1];
  auto load_res = [&](int tm) {
#pragma unroll
    for (int i = 0; i < T::FI; ++i)
#pragma unroll
      for (int j = 0; j < T::FJ; ++j) {
        const int m = tm * BM + wp * T::WTP + j * 16 + frow, ch = c0 + wc * T::WTC + i * 16 + fq * 4;
        rres[i][j] = (m < M && ch < a.Cout) ? *(const uint2*)(rg + (long)m * a.ldr + ch) : make_uint2(0, 0);
      }
  };
  int tm = p, kt = 0;
  if constexpr (RES)
    if (total > 0) load_res(tm);

  for (int s = 0; s < total; ++s) {
    // K tile s landed (younger ops: the next STAGES-2 tiles' DMA, and stores /
    // residual loads of a tile boundary, which only make this wait stricter)
    if (s + STAGES - 2 < total) wait_vmcnt<T::NV>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (s + STAGES - 1 < total) issue((s + STAGES - 1) % STAGES);
    const char* sx = smem + (s % STAGES) * T::STAGE_BYTES;
    const char* sw = wl + kt * BN * 128;
    bf16x8 fa[2][T::FI], fb[2][T::FJ];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < T::FI; ++i) fa[ks][i] = *(const bf16x8*)(sw + lds_swz(wc * T::WTC + i * 16 + frow, ch));
#pragma unroll
      for (int j = 0; j < T::FJ; ++j) fb[ks][j] = *(const bf16x8*)(sx + lds_swz(wp * T::WTP + j * 16 + frow, ch));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < T::FI; ++i)
#pragma unroll
        for (int j = 0; j < T::FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);

    if (++kt == nk) {  // tile done: bias (+ residual) (+ ReLU) -> 8-B NHWC stores
#pragma unroll
      for (int j = 0; j < T::FJ; ++j) {
        const int m = tm * BM + wp * T::WTP + j * 16 + frow;
#pragma unroll
        for (int i = 0; i < T::FI; ++i) {
          const int ch = c0 + wc * T::WTC + i * 16 + fq * 4;
          float f0 = acc[i][j][0] + bias[i].x, f1 = acc[i][j][1] + bias[i].y;
          float f2 = acc[i][j][2] + bias[i].z, f3 = acc[i][j][3] + bias[i].w;
          if constexpr (RES) {
            const uint2 r = rres[i][j];
            f0 += bf2f(r.x & 0xffff);
            f1 += bf2f(r.x >> 16);
            f2 += bf2f(r.y & 0xffff);
            f3 += bf2f(r.y >> 16);
          }
          if (a.relu) {
            f0 = fmaxf(f0, 0.f);
            f1 = fmaxf(f1, 0.f);
            f2 = fmaxf(f2, 0.f);
            f3 = fmaxf(f3, 0.f);
          }
          if (m < M && ch < a.Cout)
            *(uint2*)((unsigned short*)a.y + (long)m * a.ldy + ch) = make_uint2(pack2(f0, f1), pack2(f2, f3));
          acc[i][j] = (f32x4)(0.f);
        }
      }
      kt = 0;
      tm += P;
      if constexpr (RES)
        if (s + 1 < total) load_res(tm);
    }
  }
}

}  // namespace ws
}  // namespace dml

// Configurations: id, BM (pixels), BN (channels), WM x WN waves, ring STAGES.
// LDS = STAGES x BM x 128 B ring + K x BN x 2 B resident weights (<= 160 KiB).
#define DML_WS_TILES(X)                                       \
  X(84, 128, 64, 2, 2, 3)   /* the reduce 1x1s (Cout 64) */   \
  X(85, 128, 64, 2, 2, 4)                                     \
  X(86, 64, 64, 1, 4, 4)                                      \
  X(87, 128, 128, 2, 2, 3)                                    \
  X(88, 64, 256, 1, 4, 4)                                     \
  X(89, 128, 256, 2, 4, 3)  /* 8 waves */                     \
  X(90, 256, 64, 4, 1, 3)

static int g_cus = 0;  // compute units of the device (dml_conv_ws_init)

static int ws_lds(int cfg, int nk) {
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST) \
  case id: return dml::ws::WsCfg<BM, BN, WM, WN, ST>::lds(nk);
    DML_WS_TILES(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}

extern "C" int dml_conv_ws_supported(int cfg) {
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST) \
  case id: return BN;
    DML_WS_TILES(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}

extern "C" const char* dml_conv_ws_check(const DmlConvArgs* a, int cfg) {
  const int bn = dml_conv_ws_supported(cfg);
  if (!bn) return "dml_conv_ws: not a weight-stationary cfg";
  if (a->kh != 1 || a->kw != 1 || a->sh != 1 || a->sw != 1 || a->ph || a->pw || a->dh > 1 || a->dw > 1 ||
      a->Ho != a->H || a->Wo != a->W)
    return "dml_conv_ws: 1x1 stride-1 unpadded convs only";
  if (a->Cin % 64 || a->K != a->Cin || a->Kpad != a->Cin)
    return "dml_conv_ws: K = Cin must be a multiple of 64";
  if (a->nseg || a->out_f32 || a->ksplit > 1 || a->rsub > 1)
    return "dml_conv_ws: no output segments, fp32 output, split-K or subsampled residual";
  if (a->ldx % 8 || a->Cout % 8 || a->ldy % 4 || (a->res && a->ldr % 4))
    return "dml_conv_ws: need ldx, Cout %8 == 0 and ldy, ldr %4 == 0";
  if ((a->Cout + bn - 1) / bn * bn > (a->Cout + 255) / 256 * 256)
    return "dml_conv_ws: the channel tiles of this cfg overrun the 256-row weight padding";
  if ((long)a->N * a->H * a->W * a->ldx * 2 >= 0x7ffffff0L) return "dml_conv_ws: input larger than 2 GiB";
  if (ws_lds(cfg, a->Kpad / 64) > dml::ws::kLds) return "dml_conv_ws: ring + weight panel exceed 160 KiB of LDS";
  return nullptr;
}

extern "C" int dml_conv_ws_init(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount,
                                                                 dev) != hipSuccess || g_cus <= 0)
    g_cus = 256;
  int rc = 0;
#define DML_SET(id, BM, BN, WM, WN, ST)                                                                        \
  rc |= (int)hipFuncSetAttribute((const void*)dml::ws::conv_ws_kernel<BM, BN, WM, WN, ST, false>,            \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, dml::ws::kLds);                 \
  rc |= (int)hipFuncSetAttribute((const void*)dml::ws::conv_ws_kernel<BM, BN, WM, WN, ST, true>,             \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, dml::ws::kLds);
  DML_WS_TILES(DML_SET)
#undef DML_SET
  return rc;
}

template <int BM, int BN, int WM, int WN, int ST>
static int launch_ws(const DmlConvArgs* a, hipStream_t s) {
  using T = dml::ws::WsCfg<BM, BN, WM, WN, ST>;
  const int lds = T::lds(a->Kpad / 64);
  const long M = (long)a->N * a->Ho * a->Wo;
  const long ntm = (M + BM - 1) / BM, ntc = (a->Cout + BN - 1) / BN;
  int occ = dml::ws::kLds / lds;
  if (occ * T::NW > 32) occ = 32 / T::NW;  // 8 waves per SIMD
  long G = (long)(g_cus > 0 ? g_cus : 256) * occ;
  if (G > ntm * ntc) G = ntm * ntc;
  G = G / ntc * ntc;
  if (G < ntc) G = ntc;
  if (a->res)
    hipLaunchKernelGGL((dml::ws::conv_ws_kernel<BM, BN, WM, WN, ST, true>), dim3((unsigned)G), dim3(T::NT), lds, s,
                       *a);
  else
    hipLaunchKernelGGL((dml::ws::conv_ws_kernel<BM, BN, WM, WN, ST, false>), dim3((unsigned)G), dim3(T::NT), lds, s,
                       *a);
  DML_CHECK_LAUNCH();
  return 0;
}

extern "C" int dml_conv_ws(const DmlConvArgs* a, int cfg, hipStream_t s) {
  const char* why = dml_conv_ws_check(a, cfg);
  if (why) {
    dml_set_error(why);
    return -1;
  }
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST) \
  case id: return launch_ws<BM, BN, WM, WN, ST>(a, s);
    DML_WS_TILES(DML_CASE)
#undef DML_CASE
    default: dml_set_error("dml_conv_ws: not a weight-stationary cfg"); return -1;
  }
}
