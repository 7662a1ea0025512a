// conv_pool.hip — 3x3 'same' convolution (32 -> 64 channels) + ReLU fused with the
// 3x3/2 'valid' max pool that consumes it (gfx950). InceptionV3 conv2d_3 +
// max_pooling2d_1 (Keras; reference models.py:26): unfused, the 147x147x64 conv
// output is written to HBM and read back by the pool (2 x 177 MB per 64 images).
//
// A workgroup owns an 8x8 block of pool outputs:
//  1. the 19x19 x 32-channel input patch the conv window needs (conv pad 1 ->
//     zeros), 16-B global loads into registers (all issued first, clamped
//     addresses, padding zeroed after) -> LDS rows of 96 B (64 B + 32-B pad: the
//     16 lanes of each ds_read_b128 lane group hit distinct banks; 80-B rows
//     measured 2-way conflicts, SQ_LDS_BANK_CONFLICT);
//  2. the 17x17 conv window (289 pixels = 19 MFMA fragments) with
//     v_mfma_f32_16x16x32_bf16: k-step t = tap (r, s) over 32 channels, one
//     ds_read_b128 per pixel fragment; wave w owns output channels 16w..16w+15,
//     its 16 x 288 weights in VGPRs;
//  3. bias + ReLU -> bf16 (the unfused rounding point) into an LDS tile that
//     reuses the patch region;
//  4. 3x3/2 max pool from LDS -> one 16-B NHWC store per 8 channels;
//  or, with a folded 1x1 conv (c4 > 0: InceptionV3 conv2d_4, 64 -> 80 + ReLU, the pool's only
//  reader), the pooled 64-pixel x 64-channel tile goes to LDS instead, and
//  5. y = relu(w4 . tile + b4) per 16-pixel fragment (one wave each; 2 k-steps x c4/16
//     MFMAs), staged through LDS for 16-B NHWC stores: the 64-channel pool output never
//     reaches HBM (its write and the 1x1 conv's re-read, 2 x 44 MB per 64 images).
#include "common.h"
#include "dml.h"

namespace dml {
namespace cpool {

constexpr int PB = 8;                        // pool outputs per block side
constexpr int CW = 2 * PB + 1;               // conv window 17 x 17
constexpr int NPX = CW * CW;                 // 289
constexpr int PW = CW + 2;                   // patch 19 x 19 (conv pad 1)
// The conv is computed over 17 rows x 19 columns in PATCH pitch (columns 17, 18
// of each row are junk, never stored): output q' = a*19 + b reads patch pixel
// q' + r*19 + s, so a fragment's 16 consecutive q' are 16 consecutive patch
// pixels for every tap — linear addresses (one base register + immediate
// offsets) and no row-wrap discontinuity, which made some 16-lane groups hit
// the same banks. +2 fragments of MFMA work buy conflict-free reads.
constexpr int NQ = CW * PW;                  // 323
constexpr int NF = (NQ + 15) / 16;           // 21 pixel fragments
constexpr int PROW = 32 * 2 + 32;            // patch pixel row: 32 bf16 + 32-B pad (96 B: the 16 lanes of
                                             // every ds_read_b128 lane group hit 16 distinct 4-bank windows)
constexpr int PATCH_BYTES = PW * PW * PROW;  // 28880
constexpr int TROW = 64 * 2 + 16;            // conv tile row: 64 bf16 + 16-B pad
constexpr int TILE_BYTES = NPX * TROW;       // 41616
constexpr int LDS_MAIN = PATCH_BYTES > TILE_BYTES ? PATCH_BYTES : TILE_BYTES;
constexpr int POOLT = LDS_MAIN;                 // folded 1x1: pooled tile [64 px][64 ch] bf16, 128-B rows
constexpr int LDS_BYTES = POOLT + PB * PB * 128;
constexpr int C4_MAX = 128;
constexpr int SROW4 = C4_MAX * 2 + 16;          // folded 1x1 output staging row (reuses the conv tile)
constexpr int NT = 256;
constexpr int CHUNKS = PW * PW * 4;          // 16-B input chunks of the patch (1444)
constexpr int FILL = (CHUNKS + NT - 1) / NT; // 6

// 16-B chunk `ch` of 128-B row `row` of the pooled tile, XOR-swizzled (conflict-free
// fragment reads of 16 consecutive rows)
__device__ __forceinline__ int convk_swz(int row, int ch) { return row * 128 + ((ch ^ (row & 7)) << 4); }

__global__ __launch_bounds__(NT, 3) void conv_pool_kernel(DmlConvPoolArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* patch = smem;
  char* tile = smem;  // after the conv (barrier in between)

  const int bpr = (a.Wo + PB - 1) / PB, bpc = (a.Ho + PB - 1) / PB;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int n = blk / (bpr * bpc);
  const int rem = blk - n * bpr * bpc;
  const int by = rem / bpr, bx = rem - by * bpr;
  const int py0 = by * PB, px0 = bx * PB;
  const int cy0 = 2 * py0, cx0 = 2 * px0;  // conv window origin (valid pool)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;

  // weights: this wave's 16 output channels, k-step t = tap (r, s), quarter fq = 8 channels
  bf16x8 wf[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
    wf[t] = *(const bf16x8*)((const bf16*)a.w + (long)(wid * 16 + frow) * a.ldw + t * 32 + fq * 8);
  const float4 bias = *(const float4*)(a.bias + wid * 16 + fq * 4);

  // 1. patch: pixel (i, j) = input (cy0 - 1 + i, cx0 - 1 + j), 4 chunks of 8 channels
  {
    const unsigned short* x = (const unsigned short*)a.x + (long)n * a.H * a.W * a.ldx;
    uint4 v[FILL];
    bool ok[FILL];
#pragma unroll
    for (int it = 0; it < FILL; ++it) {
      const int t = min(tid + it * NT, CHUNKS - 1);
      const int pix = t >> 2, c = t & 3;
      const int i = pix / PW, j = pix - i * PW;
      const int ih = cy0 - 1 + i, iw = cx0 - 1 + j;
      ok[it] = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const int ihc = min(max(ih, 0), a.H - 1), iwc = min(max(iw, 0), a.W - 1);
      v[it] = *(const uint4*)(x + ((long)ihc * a.W + iwc) * a.ldx + c * 8);
    }
#pragma unroll
    for (int it = 0; it < FILL; ++it) {
      const int t = tid + it * NT;
      if (t >= CHUNKS) continue;
      const int pix = t >> 2, c = t & 3;
      *(uint4*)(patch + pix * PROW + c * 16) = ok[it] ? v[it] : make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();

  // 2. conv over the window in patch pitch: fragment j = outputs q' = 16j .. 16j+15
  //    (q' >= 323 read past the patch into the same LDS allocation: junk, never stored)
  const char* pbase = patch + frow * PROW + fq * 16;
  f32x4 acc[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int toff = ((t / 3) * PW + (t % 3)) * PROW;
#pragma unroll
    for (int j0 = 0; j0 < NF; j0 += 4) {  // 4 fragments in flight at a time
      bf16x8 pf[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (j0 + q < NF) pf[q] = *(const bf16x8*)(pbase + (j0 + q) * 16 * PROW + toff);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (j0 + q < NF) acc[j0 + q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t], pf[q], acc[j0 + q], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  __syncthreads();  // every wave done reading the patch: the conv tile reuses it

  // 3. bias + ReLU -> bf16 conv tile (positions outside the conv image -> 0)
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int qp = j * 16 + frow;
    const int wa = qp / PW, wb = qp - wa * PW;
    if (qp >= NQ || wb >= CW) continue;  // junk columns / dummy outputs
    const int p = wa * CW + wb;          // conv tile (window) index
    const bool ok = (cy0 + wa < a.H) && (cx0 + wb < a.W);
    const f32x4 v = acc[j];
    const float f0 = ok ? fmaxf(v[0] + bias.x, 0.f) : 0.f, f1 = ok ? fmaxf(v[1] + bias.y, 0.f) : 0.f;
    const float f2 = ok ? fmaxf(v[2] + bias.z, 0.f) : 0.f, f3 = ok ? fmaxf(v[3] + bias.w, 0.f) : 0.f;
    *(uint2*)(tile + p * TROW + (wid * 16 + fq * 4) * 2) =
        make_uint2(pack2(f0, f1) & kNoSign2, pack2(f2, f3) & kNoSign2);  // +0 only: the pool maxes bits
  }
  __syncthreads();

  // 4. max pool 3x3/2 valid: item = (pool pixel, 8-channel group)
#pragma unroll
  for (int it = 0; it < PB * PB * 8 / NT; ++it) {
    // lanes 0-7 / 8-15 of a lane group read pool pixels lx and lx + 4: their conv
    // pixels are 8 x 144 B apart = 128 B mod 256, so the two 128-B reads never
    // share a bank (adjacent pool pixels, 288 B apart, overlapped: 2-way conflicts)
    const int t = tid + it * NT;
    const int cg = t & 7, half = (t >> 3) & 1, pr = t >> 4;
    const int ly = pr / (PB / 2), lx = pr - ly * (PB / 2) + half * (PB / 2);
    const int oy = py0 + ly, ox = px0 + lx;
    if (oy >= a.Ho || ox >= a.Wo) continue;
    uint4 pv = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
        pv = max_bf16x8_nonneg(pv, *(const uint4*)(tile + ((2 * ly + dy) * CW + 2 * lx + dx) * TROW + cg * 16));
    if (a.c4 > 0)
      *(uint4*)(smem + POOLT + convk_swz(ly * PB + lx, cg)) = pv;
    else
      *(uint4*)((unsigned short*)a.y + ((long)(n * a.Ho + oy) * a.Wo + ox) * a.ldy + cg * 8) = pv;
  }
  if (a.c4 <= 0) return;

  // 5. folded 1x1 conv: wave w owns pool pixels 16w .. 16w+15 (pool tile row-major, 8 wide)
  __syncthreads();  // pooled tile complete; pool rows outside the image hold junk, never stored
  const int nf4 = a.c4 / 16;
  f32x4 acc4[C4_MAX / 16];
#pragma unroll
  for (int o = 0; o < C4_MAX / 16; ++o) {
    if (o < nf4) {
      const float4 bb = *(const float4*)(a.b4 + 16 * o + 4 * fq);
      acc4[o] = (f32x4){bb.x, bb.y, bb.z, bb.w};
    }
  }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const bf16x8 pb = *(const bf16x8*)(smem + POOLT + convk_swz(16 * wid + frow, 4 * ks + fq));
#pragma unroll
    for (int o = 0; o < C4_MAX / 16; ++o) {
      if (o < nf4) {
        const bf16x8 wa = *(const bf16x8*)((const bf16*)a.w4 + (long)(16 * o + frow) * a.ldw4 + 32 * ks + 8 * fq);
        acc4[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, pb, acc4[o], 0, 0, 0);
      }
    }
  }
  // bias (in the accumulator start) + ReLU -> bf16 staging rows (the conv tile region is free:
  // every wave passed the barrier above after its last pool read)
#pragma unroll
  for (int o = 0; o < C4_MAX / 16; ++o) {
    if (o < nf4) {
      const f32x4 v = acc4[o];
      *(uint2*)(smem + (16 * wid + frow) * SROW4 + (16 * o + 4 * fq) * 2) =
          make_uint2(pack2(fmaxf(v[0], 0.f), fmaxf(v[1], 0.f)), pack2(fmaxf(v[2], 0.f), fmaxf(v[3], 0.f)));
    }
  }
  __syncthreads();
  const int cgs = a.c4 / 8;
  for (int t = tid; t < PB * PB * cgs; t += NT) {
    const int px = t / cgs, cg = t - px * cgs;
    const int oy = py0 + px / PB, ox = px0 + px % PB;
    if (oy >= a.Ho || ox >= a.Wo) continue;
    *(uint4*)((unsigned short*)a.y + ((long)(n * a.Ho + oy) * a.Wo + ox) * a.ldy + cg * 8) =
        *(const uint4*)(smem + px * SROW4 + cg * 16);
  }
}

}  // namespace cpool
}  // namespace dml

extern "C" int dml_conv3x3_pool(const DmlConvPoolArgs* a, hipStream_t s) {
  // hard-coded: conv 3x3 stride 1 pad 1, 32 -> 64 channels; max pool 3x3/2 valid
  const int cy = a->c4 > 0 ? a->c4 : 64;
  if (a->ldx % 8 || a->ldx < 32 || a->ldw % 8 || a->ldw < 288 || a->ldy % 8 || a->ldy < cy || a->N < 1 ||
      a->H < 3 || a->W < 3 || a->Ho != (a->H - 3) / 2 + 1 || a->Wo != (a->W - 3) / 2 + 1 ||
      (a->c4 > 0 && (a->c4 % 16 || a->c4 > dml::cpool::C4_MAX || !a->w4 || !a->b4 || a->ldw4 % 8 || a->ldw4 < 64))) {
    dml_set_error("dml_conv3x3_pool: unsupported shape");
    return -1;
  }
  using namespace dml::cpool;
  const long blocks = (long)a->N * ((a->Ho + PB - 1) / PB) * ((a->Wo + PB - 1) / PB);
  hipLaunchKernelGGL(dml::cpool::conv_pool_kernel, dim3((unsigned)blocks), dim3(NT), 0, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}
