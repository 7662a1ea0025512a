// bottleneck_fused.hip — ResNet50 block boundary as ONE kernel (gfx950):
//
//   Y = relu(W3 . T + b3 + R)      block k's 1x1 expand (F -> C) + shortcut
//   Z = relu(W1 . Y + b1)          block k+1's 1x1 reduce (C -> F), F = C / 4
//
// Both are HBM-bound 1x1 GEMMs (Keras convN_blockK_3_conv / convN_blockK+1_1_conv,
// reference models.py:48-51). Unfused, Y is written by the expand and read back
// in full by the reduce; here a workgroup owns BM pixels x ALL C channels of Y,
// so the reduce reads Y from LDS. Stage 2 (C = 256, per 128 images):
//   HBM bytes  T 51 + R 205 + Y 205 + Z 51 MB  (vs 718 MB for the two launches)
// Instantiations: C = 256 (BM 64, 4 waves), 512 (BM 32, 8 waves), 1024 (BM 32,
// 16 waves); wave w owns Y channels 64w..64w+63 and Z channels 16w..16w+15.
// Measured (profiles/r1_v11, per 128 images): C = 256 130 us vs 153 us for the
// two launches — the engine default; C = 512 123-138 us vs 75-90 us and C = 1024
// 157 us vs 63 us — every workgroup re-reads both weight matrices (C^2 bytes,
// 3-6x its activation bytes at BM = 32) and the phase-serialised workgroup runs
// at 1-2 waves/SIMD, so those stay opt-in (DML_FUSED_BLOCKS_MAXC). BM = 32 / 128
// for C = 256 measured 175 us. An epilogue straight from the MFMA layout (no fp32
// staging tile, one barrier, 8-B residual loads / Y stores of 4 channels per lane)
// measured 176-182 us vs 131-135 us: the 32-B-per-pixel access pattern costs more
// than the staging round trip (profiles/r1_v11/op_times_direct_epilogue.json).
//  1. expand: the wave's 64-channel x BM-pixel tile, K = F, W3 and T fragments
//     loaded straight from global into VGPRs (no LDS ring: one pass over K); the
//     shortcut rows are prefetched first (16-B loads, one 8-channel group per
//     thread) so they stream under the MFMAs;
//  2. epilogue in BM/16 passes of 16 pixels through an fp32 LDS staging tile:
//     bias + shortcut + ReLU -> bf16 -> one coalesced 16-B store to Y AND a copy
//     into an LDS Y tile (row pitch 2C + 32 B: the reduce's fragment reads are
//     conflict-free);
//  Merged-shortcut variant (RES = false, KX = 2F; C = 256): after the projection-
//  shortcut merge (models/optimize.py) a stage's first expand reads the channel
//  concat [x ; s] (K = 2F) with no residual; same kernel, longer K loop. Measured
//  150 us vs 74 + 55 us for the two launches (profiles/r1_v15: the doubled expand K
//  runs inside the phase-serialised workgroup), so the engine keeps it opt-in.
//  3. reduce: the wave's 16 output channels for the BM pixels from the LDS Y
//     tile (K = C), W1 fragments in VGPRs in chunks of 8 k-steps (the first
//     chunk loaded during the epilogue), bias + ReLU -> 8-B stores.
#include <cstdlib>

#include "common.h"
#include "dml.h"

namespace dml {
namespace bneck {

template <int C_, int BM_, int KX_ = C_ / 4>
struct Cfg {
  static constexpr int C = C_, BM = BM_, F = C / 4, KX = KX_;
  static constexpr int NW = C / 64, NT = NW * 64;
  static constexpr int SROW = C * 4 + 16;         // fp32 staging row
  static constexpr int STAGE_BYTES = 16 * SROW;   // one pass = 16 pixels
  static constexpr int YROW = C * 2 + 32;         // bf16 Y tile row
  static constexpr int LDS = STAGE_BYTES + BM * YROW;
  static constexpr int CG = C / 8;                // 8-channel groups per pixel
  static constexpr int PR = NT / CG;              // pixel rows per epilogue sweep (8)
  static constexpr int EIT = BM / PR;             // epilogue pixels per thread
  static constexpr int JN = BM / 16;              // pixel fragments
  static constexpr int KS1 = KX / 32, KS2 = C / 32;
  static constexpr int KC = 8;                    // reduce k-steps per weight chunk
  static_assert(PR == 8 && BM % 16 == 0 && KS2 % KC == 0, "tile shape");
};

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = bf2f(v.x & 0xffff); f[1] = bf2f(v.x >> 16);
  f[2] = bf2f(v.y & 0xffff); f[3] = bf2f(v.y >> 16);
  f[4] = bf2f(v.z & 0xffff); f[5] = bf2f(v.z >> 16);
  f[6] = bf2f(v.w & 0xffff); f[7] = bf2f(v.w >> 16);
}

template <int C, int BM, int MINB, int KX = C / 4, bool RES = true>
__global__ __launch_bounds__(C, MINB) void expand_reduce_kernel(DmlExpandReduceArgs a) {
  using T = Cfg<C, BM, KX>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* stage = smem;
  char* ytile = smem + T::STAGE_BYTES;

  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const bf16* x = (const bf16*)a.x;
  const bf16* w3 = (const bf16*)a.w3;
  const bf16* w1 = (const bf16*)a.w1;
  const unsigned short* rg = (const unsigned short*)a.res;

  // shortcut rows + bias for the epilogue: thread owns channel group cg_t of pixels prow + 8*it
  const int cg_t = tid % T::CG, prow = tid / T::CG, ch_t = cg_t * 8;
  uint4 rpre[T::EIT];
#pragma unroll
  for (int it = 0; it < T::EIT; ++it) {
    const int m = min(m0 + prow + it * T::PR, a.M - 1);  // rows >= M are computed but never stored
    rpre[it] = RES ? *(const uint4*)(rg + (long)m * a.ldr + ch_t) : make_uint4(0, 0, 0, 0);
  }
  const float4 bias0 = *(const float4*)(a.b3 + ch_t), bias1 = *(const float4*)(a.b3 + ch_t + 4);

  // 1. expand: A = W3 rows (this wave's 64 channels), B = T rows (BM pixels), K = F
  f32x4 acc[4][T::JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < T::JN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < T::KS1; ++ks) {
    bf16x8 wa[4], xb[T::JN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      wa[i] = *(const bf16x8*)(w3 + (long)(wid * 64 + i * 16 + frow) * a.ldw3 + ks * 32 + fq * 8);
#pragma unroll
    for (int j = 0; j < T::JN; ++j) {
      const int m = min(m0 + j * 16 + frow, a.M - 1);
      xb[j] = *(const bf16x8*)(x + (long)m * a.ldx + ks * 32 + fq * 8);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < T::JN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i], xb[j], acc[i][j], 0, 0, 0);
  }

  // first reduce-weight chunk (in flight during the epilogue): this wave's 16 output channels
  const bf16* w1row = w1 + (long)(wid * 16 + frow) * a.ldw1 + fq * 8;
  bf16x8 w1f[T::KC];
#pragma unroll
  for (int k = 0; k < T::KC; ++k) w1f[k] = *(const bf16x8*)(w1row + k * 32);
  const float4 b1v = *(const float4*)(a.b1 + wid * 16 + fq * 4);

  // 2. epilogue: pass p stages pixel fragment j = p (16 pixels x C channels, fp32)
#pragma unroll
  for (int p = 0; p < T::JN; ++p) {
    __syncthreads();  // staging rows free
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *(f32x4*)(stage + frow * T::SROW + (wid * 64 + i * 16 + fq * 4) * 4) = acc[i][p];
    __syncthreads();
#pragma unroll
    for (int it = 2 * p; it < 2 * p + 2; ++it) {
      const int px = prow + it * T::PR;  // in [16p, 16p + 16)
      const int lp = px - 16 * p;
      const float4 v0 = *(const float4*)(stage + lp * T::SROW + cg_t * 32);
      const float4 v1 = *(const float4*)(stage + lp * T::SROW + cg_t * 32 + 16);
      float r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (RES) unpack8(rpre[it], r);
      float f[8] = {v0.x + bias0.x + r[0], v0.y + bias0.y + r[1], v0.z + bias0.z + r[2], v0.w + bias0.w + r[3],
                    v1.x + bias1.x + r[4], v1.y + bias1.y + r[5], v1.z + bias1.z + r[6], v1.w + bias1.w + r[7]};
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] = fmaxf(f[q], 0.f);
      const uint4 yv = make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
      const int m = m0 + px;
      long ym = m;
      bool keep = m < a.M;
      if (a.ysub > 1) {  // only the pixels a strided reader takes, stored compactly
        const int hw = a.yH * a.yW;
        const int ni = m / hw, r = m - ni * hw;
        const int hh = r / a.yW, ww = r - hh * a.yW;
        keep = keep && hh % a.ysub == 0 && ww % a.ysub == 0;
        ym = ((long)ni * (a.yH / a.ysub) + hh / a.ysub) * (a.yW / a.ysub) + ww / a.ysub;
      }
      if (keep) *(uint4*)((unsigned short*)a.y + ym * a.ldy + ch_t) = yv;
      *(uint4*)(ytile + px * T::YROW + cg_t * 16) = yv;
    }
  }
  __syncthreads();

  // 3. reduce from the LDS Y tile: A = W1 rows, B = Y rows, K = C
  f32x4 acc2[T::JN];
#pragma unroll
  for (int j = 0; j < T::JN; ++j) acc2[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < T::KS2; kc += T::KC) {
    if (kc) {
#pragma unroll
      for (int k = 0; k < T::KC; ++k) w1f[k] = *(const bf16x8*)(w1row + (kc + k) * 32);
    }
#pragma unroll
    for (int k = 0; k < T::KC; ++k) {
      bf16x8 pf[T::JN];
#pragma unroll
      for (int j = 0; j < T::JN; ++j)
        pf[j] = *(const bf16x8*)(ytile + (j * 16 + frow) * T::YROW + (kc + k) * 64 + fq * 16);
#pragma unroll
      for (int j = 0; j < T::JN; ++j)
        acc2[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[k], pf[j], acc2[j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < T::JN; ++j) {
    const int m = m0 + j * 16 + frow;
    if (m >= a.M) continue;
    const f32x4 v = acc2[j];
    *(uint2*)((unsigned short*)a.z + (long)m * a.ldz + wid * 16 + fq * 4) =
        make_uint2(pack2(fmaxf(v[0] + b1v.x, 0.f), fmaxf(v[1] + b1v.y, 0.f)),
                   pack2(fmaxf(v[2] + b1v.z, 0.f), fmaxf(v[3] + b1v.w, 0.f)));
  }
}

template <int C, int BM, int MINB, int KX = C / 4, bool RES = true>
int launch(const DmlExpandReduceArgs* a, hipStream_t s) {
  using T = Cfg<C, BM, KX>;
  const long blocks = ((long)a->M + BM - 1) / BM;
  hipLaunchKernelGGL((expand_reduce_kernel<C, BM, MINB, KX, RES>), dim3((unsigned)blocks), dim3(T::NT), T::LDS, s,
                     *a);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int C, int BM, int MINB, int KX = C / 4, bool RES = true>
int set_attr() {
  return (int)hipFuncSetAttribute((const void*)expand_reduce_kernel<C, BM, MINB, KX, RES>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, Cfg<C, BM, KX>::LDS);
}

}  // namespace bneck
}  // namespace dml

// Raise the dynamic-LDS limit of every instantiation (before any launch or graph
// capture); called from dml_conv_v2_init.
extern "C" int dml_expand_reduce_init(void) {
  using namespace dml::bneck;
  const int rc = set_attr<256, 64, 2>() | set_attr<512, 32, 2>() | set_attr<1024, 32, 1>() |
                 set_attr<256, 64, 2, 128, false>() | dml_chain_init();
  if (rc) dml_set_error("dml_expand_reduce_init: hipFuncSetAttribute failed");
  return rc ? -1 : 0;
}

extern "C" int dml_expand_reduce(const DmlExpandReduceArgs* a, hipStream_t s) {
  // the chained-GEMM kernel (expand_reduce_chain.hip) where it serves the shape (C = 512 / 1024
  // with a shortcut, merged C = 256 / 512); DML_ER_R1=1 keeps the phase-serialised r1 kernels
  // below (A/B)
  static const bool chain = [] { const char* e = getenv("DML_ER_R1"); return !(e && e[0] == '1'); }();
  if (chain && dml_chain_supported(a)) return dml_chain(a, s);
  if (a->fz > 0 && a->fz != a->C / 4) {  // a stage-end boundary: the chained kernel's form only
    dml_set_error("dml_expand_reduce: reduce width != C / 4 needs the chained kernel (DML_ER_R1 unset)");
    return -1;
  }
  // expand KX -> C channels (+ shortcut), reduce C -> F, F = C / 4, C in {256, 512, 1024};
  // KX = F with a shortcut, or KX = 2F without one (merged projection shortcut, C = 256)
  const int C = a->C, F = C / 4;
  const int kx = a->kx > 0 ? a->kx : F;
  const bool merged = a->res == nullptr;
  if ((C != 256 && C != 512 && C != 1024) || a->M < 1 || a->ldx % 8 || a->ldx < kx || a->ldw3 % 8 ||
      a->ldw3 < kx || (!merged && (a->ldr % 8 || a->ldr < C)) || a->ldy % 8 || a->ldy < C || a->ldw1 % 8 ||
      a->ldw1 < C || a->ldz % 4 || a->ldz < F || (merged ? (C != 256 || kx != 2 * F) : kx != F) ||
      (a->ysub > 1 && (a->yH % a->ysub || a->yW % a->ysub || (long)a->yH * a->yW < 1 ||
                       a->M % ((long)a->yH * a->yW)))) {
    dml_set_error("dml_expand_reduce: unsupported shape");
    return -1;
  }
  using namespace dml::bneck;
  if (merged) return launch<256, 64, 2, 128, false>(a, s);
  if (C == 256) return launch<256, 64, 2>(a, s);
  if (C == 512) return launch<512, 32, 2>(a, s);
  return launch<1024, 32, 1>(a, s);
}
