// bottleneck_fused.hip — ResNet50 stage-2 block boundary as ONE kernel (gfx950):
//
//   Y = relu(W3 . T + b3 + R)      block k's 1x1 expand (64 -> 256) + shortcut
//   Z = relu(W1 . Y + b1)          block k+1's 1x1 reduce (256 -> 64)
//
// Both are HBM-bound 1x1 GEMMs (Keras conv2_blockK_3_conv / conv2_blockK+1_1_conv,
// reference models.py:48-51). Unfused, Y (205 MB per 128 images) is written by
// the expand and read back in full by the reduce; here a workgroup owns 64
// pixels x ALL 256 channels of Y, so the reduce reads Y from LDS:
//   HBM bytes  T 51 + R 205 + Y 205 + Z 51 MB  (vs 718 MB for the two launches)
//  1. expand: the wave's 64-channel x 64-pixel tile, K = 64 (two k-steps), with
//     W3 and T fragments loaded straight from global into VGPRs (one K tile:
//     no LDS ring needed); the shortcut rows are prefetched first (16-B loads,
//     one 8-channel group per thread) so they stream under the MFMAs;
//  2. epilogue in 4 passes of 16 pixels through an fp32 LDS staging tile: bias +
//     shortcut + ReLU -> bf16 -> one coalesced 16-B store to Y AND a copy into
//     an LDS Y tile (544-B rows: the reduce's fragment reads are conflict-free);
//  3. reduce: wave w computes output channels 16w..16w+15 for the 64 pixels from
//     the LDS Y tile (K = 256, 8 k-steps), W1 fragments in VGPRs (loaded during
//     the epilogue), bias + ReLU -> 8-B stores.
#include "common.h"
#include "dml.h"

namespace dml {
namespace bneck {

constexpr int BM = 64, C = 256, F = 64;
constexpr int NT = 256;                       // 4 waves
constexpr int SROW = C * 4 + 16;              // fp32 staging row (1040 B)
constexpr int P = 4;                          // staging passes of 16 pixels
constexpr int STAGE_BYTES = (BM / P) * SROW;  // 16640
constexpr int YROW = C * 2 + 32;              // bf16 Y tile row (544 B)
constexpr int Y_BYTES = BM * YROW;            // 34816
constexpr int CG = C / 8;                     // 8-channel groups per pixel (32)
constexpr int EIT = BM * CG / NT;             // epilogue pixels per thread (8)

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = bf2f(v.x & 0xffff); f[1] = bf2f(v.x >> 16);
  f[2] = bf2f(v.y & 0xffff); f[3] = bf2f(v.y >> 16);
  f[4] = bf2f(v.z & 0xffff); f[5] = bf2f(v.z >> 16);
  f[6] = bf2f(v.w & 0xffff); f[7] = bf2f(v.w >> 16);
}

__global__ __launch_bounds__(NT, 2) void expand_reduce_kernel(DmlExpandReduceArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[STAGE_BYTES + Y_BYTES];
  char* stage = smem;
  char* ytile = smem + STAGE_BYTES;

  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const bf16* x = (const bf16*)a.x;
  const unsigned short* rg = (const unsigned short*)a.res;

  // shortcut rows + bias for the epilogue: thread owns channel group cg_t of pixels (tid>>5) + 8*it
  const int cg_t = tid & (CG - 1), ch_t = cg_t * 8;
  uint4 rpre[EIT];
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int m = min(m0 + (tid >> 5) + it * 8, a.M - 1);  // rows >= M are computed but never stored
    rpre[it] = *(const uint4*)(rg + (long)m * a.ldr + ch_t);
  }
  const float4 bias0 = *(const float4*)(a.b3 + ch_t), bias1 = *(const float4*)(a.b3 + ch_t + 4);

  // 1. expand: A = W3 rows (this wave's 64 channels), B = T rows (64 pixels), K = 64
  bf16x8 wa[4][2], xb[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      wa[i][ks] = *(const bf16x8*)((const bf16*)a.w3 + (long)(wid * 64 + i * 16 + frow) * a.ldw3 + ks * 32 + fq * 8);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = min(m0 + j * 16 + frow, a.M - 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) xb[j][ks] = *(const bf16x8*)(x + (long)m * a.ldx + ks * 32 + fq * 8);
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][ks], xb[j][ks], acc[i][j], 0, 0, 0);

  // reduce weights (in flight during the epilogue): this wave's 16 output channels, K = 256
  bf16x8 w1f[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
    w1f[ks] = *(const bf16x8*)((const bf16*)a.w1 + (long)(wid * 16 + frow) * a.ldw1 + ks * 32 + fq * 8);
  const float4 b1v = *(const float4*)(a.b1 + wid * 16 + fq * 4);

  // 2. epilogue: pass p stages pixel fragment j = p (16 pixels x 256 channels, fp32)
#pragma unroll
  for (int p = 0; p < P; ++p) {
    __syncthreads();  // staging rows free
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *(f32x4*)(stage + frow * SROW + (wid * 64 + i * 16 + fq * 4) * 4) = acc[i][p];
    __syncthreads();
#pragma unroll
    for (int it = 2 * p; it < 2 * p + 2; ++it) {
      const int px = (tid >> 5) + it * 8;  // in [16p, 16p + 16)
      const int lp = px - 16 * p;
      const float4 v0 = *(const float4*)(stage + lp * SROW + cg_t * 32);
      const float4 v1 = *(const float4*)(stage + lp * SROW + cg_t * 32 + 16);
      float r[8];
      unpack8(rpre[it], r);
      float f[8] = {v0.x + bias0.x + r[0], v0.y + bias0.y + r[1], v0.z + bias0.z + r[2], v0.w + bias0.w + r[3],
                    v1.x + bias1.x + r[4], v1.y + bias1.y + r[5], v1.z + bias1.z + r[6], v1.w + bias1.w + r[7]};
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] = fmaxf(f[q], 0.f);
      const uint4 yv = make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
      const int m = m0 + px;
      if (m < a.M) *(uint4*)((unsigned short*)a.y + (long)m * a.ldy + ch_t) = yv;
      *(uint4*)(ytile + px * YROW + cg_t * 16) = yv;
    }
  }
  __syncthreads();

  // 3. reduce from the LDS Y tile: A = W1 rows, B = Y rows, K = 256
  f32x4 acc2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc2[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    bf16x8 pf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pf[j] = *(const bf16x8*)(ytile + (j * 16 + frow) * YROW + ks * 64 + fq * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[ks], pf[j], acc2[j], 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + j * 16 + frow;
    if (m >= a.M) continue;
    const f32x4 v = acc2[j];
    *(uint2*)((unsigned short*)a.z + (long)m * a.ldz + wid * 16 + fq * 4) =
        make_uint2(pack2(fmaxf(v[0] + b1v.x, 0.f), fmaxf(v[1] + b1v.y, 0.f)),
                   pack2(fmaxf(v[2] + b1v.z, 0.f), fmaxf(v[3] + b1v.w, 0.f)));
  }
}

}  // namespace bneck
}  // namespace dml

extern "C" int dml_expand_reduce(const DmlExpandReduceArgs* a, hipStream_t s) {
  // hard-coded: expand 64 -> 256 channels (+ shortcut), reduce 256 -> 64
  if (a->M < 1 || a->ldx % 8 || a->ldx < 64 || a->ldw3 % 8 || a->ldw3 < 64 || a->ldr % 8 || a->ldr < 256 ||
      a->ldy % 8 || a->ldy < 256 || a->ldw1 % 8 || a->ldw1 < 256 || a->ldz % 4 || a->ldz < 64) {
    dml_set_error("dml_expand_reduce: unsupported shape");
    return -1;
  }
  using namespace dml::bneck;
  const long blocks = ((long)a->M + BM - 1) / BM;
  hipLaunchKernelGGL(dml::bneck::expand_reduce_kernel, dim3((unsigned)blocks), dim3(NT), 0, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}
