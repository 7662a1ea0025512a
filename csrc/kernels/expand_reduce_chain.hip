// expand_reduce_chain.hip — ResNet50 block boundary as a CHAINED GEMM (gfx950):
//
//   Y = relu(W3 . T + b3 + R)      block k's 1x1 expand (F -> C = 4F) + shortcut
//   Z = relu(W1 . Y + b1)          block k+1's 1x1 reduce (C -> F)
//
// (Keras convN_blockK_3_conv / convN_blockK+1_1_conv, reference models.py:48-51.)
// The two HBM-bound 1x1 launches move T + R + Y (write) + Y (read back) + Z; here
// Y is written once and never read back, and the reduce consumes it from
// registers, chunk by chunk, like the second GEMM of fused attention:
//
//   for each 64-channel chunk c of Y:
//     GEMM1  Yc[64 ch][px] = W3[c rows] . T           (K = F; T in VGPRs)
//     epi    Yc = relu(Yc + b3 + R[c])  -> Y (HBM, 16-B rows) and VGPR B-operands
//     GEMM2  Zacc[F][px]  += W1[:, c cols] . Yc       (K = 64)
//   Z = relu(Zacc + b1)
//
// Layout: 8 waves, each owning 32 consecutive pixels (a workgroup: 256) and ALL
// channels of them, so the Y chunk a wave produces is exactly the B operand its
// own GEMM2 needs: the epilogue never crosses waves and needs no workgroup
// barrier. Per wave an 8 KiB LDS buffer: first T ([32 px][F], 256-B rows), then
// two halves [32 px][64 ch] (128-B rows) that alternate between chunks: R[c+2]
// streams into a half by LDS-DMA while chunk c+1 computes; the epilogue of chunk
// c overwrites R[c] in place with Y, reads its B operands and its 16-B rows for
// the coalesced Y stores out of it. Weight panels (W3: 64 rows x 64 k, W1: F rows
// x 64 k) stream through a 5-slot LDS-DMA ring, one raw s_barrier per panel.
// Every vmcnt wait is exact: the wave counts the VMEM ops it issued and waits for
// "issued - mark" (stores are buffer stores with out-of-range offsets for the
// rows not stored, so every counted op really issues).
//
// Why not the r1 expand_reduce_kernel<512> (bottleneck_fused.hip, removed in r5;
// git history): its workgroups of 32 pixels re-read both weight matrices per 32
// pixels straight into VGPRs and ran phase-serialised at 1-2 waves/SIMD (123-138 us
// vs 75-90 us for the two launches, per 128 images). This file now serves every
// block boundary the engine fuses (dml_expand_reduce == dml_chain).
#include <cstdlib>

#include "conv_shared.h"

namespace dml {
namespace chain {

using convk::lds_swz;
using convk::lds_void;
using convk::wait_vmcnt;

constexpr int CC = 64;                                     // Y channels per chunk
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// F: reduce width (C = 4F); NW waves per workgroup; FJ 16-pixel fragments per wave.
//  <128, 8, 2>: 256 pixels, 1 workgroup/CU; <128, 4, 2>: 128 pixels, 2 independent
//  workgroups per CU (one's epilogue VALU work overlaps the other's MFMAs);
//  <256, 4, 1>: stage 4 (C = 1024) - T (256 k) and the Z accumulators (256 channels)
//  of 16 pixels per wave fit in VGPRs.
//  BIG: 16-KiB panels (W3 64 rows x 128 k, W1 128 rows x 64 k: one barrier per GEMM of a chunk
//  at F = 128) in a 3-slot ring instead of 8-KiB ones (64 x 64) in 5 slots; the bias is read
//  from global memory so the 4-wave forms fit 80 KiB: two workgroups per CU.
//  KX: expand input width (F, or 2F for a stage's first block after the projection-shortcut
//  merge: T = [x ; s], no residual); RES: the expand adds the shortcut R.
template <int F_, int NW_, int FJ_, bool BIG_ = false, int KX_ = F_, bool RES_ = true>
struct Cfg {
  static constexpr int F = F_, NW = NW_, FJ = FJ_, NT = NW * 64, PXW = 16 * FJ, BM = NW * PXW;
  static constexpr int KX = KX_;
  static constexpr bool BIG = BIG_, RES = RES_;
  static constexpr int NS = BIG ? 3 : 5;               // weight panel ring slots
  static constexpr int SLOT = BIG ? 16384 : 8192;      // panel bytes
  static constexpr int KW3 = BIG ? (KX < 128 ? KX : 128) : 64;  // k columns of a W3 panel (64 rows)
  static constexpr int RW1 = BIG ? (F < 128 ? F : 128) : 64;     // rows of a W1 panel (64 k columns)
  static constexpr int C_MAX = 4 * F;
  static constexpr int KS1 = KX / 32;      // T fragments (k32 steps of GEMM1)
  static constexpr int FI1 = CC / 16;      // GEMM1 channel fragments
  static constexpr int KS2 = CC / 32;      // Y fragments per chunk (k32 steps of GEMM2)
  static constexpr int FI2 = F / 16;       // GEMM2 output-channel fragments
  static constexpr int P1 = KX / KW3;      // W3 panels per chunk
  static constexpr int P2 = F / RW1;       // W1 panels per chunk
  static constexpr int PPC = P1 + P2;
  static constexpr int PI = SLOT / 1024 / NW;  // DMA instructions per wave per panel
  static constexpr int TROW = KX * 2;      // T row bytes in the wave buffer
  static constexpr int ZROW = F * 2;       // Z row bytes (the Z epilogue reuses the wave buffer)
  static constexpr int TPR = 1024 / TROW;  // T rows per 1-KiB DMA piece
  static constexpr int TPC = PXW / TPR;    // T DMA pieces per wave
  static constexpr int HALF = PXW * 128;   // R / Y half: [PXW px][64 ch] bf16
  static constexpr int HPC = PXW / 8;      // R DMA pieces per wave (8 rows of 128 B each)
  static constexpr int WB1 = PXW * TROW > 2 * HALF ? PXW * TROW : 2 * HALF;
  static constexpr int WBUF = WB1 > PXW * ZROW ? WB1 : PXW * ZROW;  // per-wave buffer
  static constexpr int WBUF0 = NS * SLOT;
  static constexpr int BIAS = WBUF0 + NW * WBUF;  // b3 [C] then b1 [F], fp32 (not BIG)
  static constexpr int STAMPS = BIAS + (BIG ? 0 : (C_MAX + F) * 4);  // diagnostics: 40 x 8 B (not BIG)
  static constexpr int LDS = STAMPS + (BIG ? 0 : 40 * 8);
  static_assert(PI >= 1 && CC == 64 && F % 64 == 0 && TPC >= 1 && HPC >= 1, "DMA split");
  static_assert(LDS <= 163840, "LDS");
};

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (n >= 31: wait for 31, stricter)
__device__ __forceinline__ void wait_vm(int n) {
  n = __builtin_amdgcn_readfirstlane(n);
  switch (n < 0 ? 0 : n) {
#define W_(k) case k: wait_vmcnt<k>(); break;
    W_(0) W_(1) W_(2) W_(3) W_(4) W_(5) W_(6) W_(7) W_(8) W_(9) W_(10) W_(11) W_(12) W_(13) W_(14) W_(15)
    W_(16) W_(17) W_(18) W_(19) W_(20) W_(21) W_(22) W_(23) W_(24) W_(25) W_(26) W_(27) W_(28) W_(29) W_(30)
#undef W_
    default: wait_vmcnt<31>(); break;
  }
}

typedef short s16x2 __attribute__((ext_vector_type(2)));
// relu + round to bf16 of 4 floats: round first (RNE keeps the sign, and -0 maps to +0
// below), then one packed signed-16-bit max against 0 per pair (bf16 bits order like
// int16 for the comparison with 0) instead of four fmaxf
__device__ __forceinline__ uint2 relu_pack4(float f0, float f1, float f2, float f3) {
  const s16x2 z = {0, 0};
  const s16x2 lo = __builtin_elementwise_max(__builtin_bit_cast(s16x2, pack2(f0, f1)), z);
  const s16x2 hi = __builtin_elementwise_max(__builtin_bit_cast(s16x2, pack2(f2, f3)), z);
  return make_uint2(__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi));
}

// T / Z rows of ROWB bytes: 16-B chunk ^= row & 15 (256- and 512-B rows: 16 consecutive rows of
// one logical chunk hit 16 distinct 4-bank groups) or ^= row & 7 (128-B rows, = lds_swz)
template <int ROWB>
__device__ __forceinline__ int wswz(int row, int ch) {
  constexpr int K = ROWB / 16 >= 16 ? 15 : ROWB / 16 - 1;
  return row * ROWB + ((ch ^ (row & K)) << 4);
}

template <int F, int NW, int FJ, bool BIG, int KX, bool RES>
__global__ __launch_bounds__(NW * 64, 2) void chain_kernel(DmlExpandReduceArgs a) {
  using T = Cfg<F, NW, FJ, BIG, KX, RES>;
  constexpr int NT = T::NT, BM = T::BM, PXW = T::PXW, HALF = T::HALF, NS = T::NS, SLOT = T::SLOT;
  using RW = convk::Rows<64>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int mw = m0 + wid * PXW;              // this wave's first pixel
  const int C = a.C, nch = C / CC, nq = nch * T::PPC;
  char* wb = smem + T::WBUF0 + wid * T::WBUF;  // this wave's buffer
  float* b3s = (float*)(smem + T::BIAS);
  float* b1s = b3s + C;

  // diagnostics (a.stamps != null): wave 0 records s_memtime at phase boundaries into LDS
  // (BIG: straight to the stamp buffer), written to a buffer nothing else reads
  long long* stl = (long long*)(smem + T::STAMPS);
  const bool stamping = a.stamps != nullptr;
  auto stamp = [&](int i) {
    if (stamping && tid == 0) {
      if constexpr (BIG) a.stamps[(long)blockIdx.x * 40 + i] = __builtin_amdgcn_s_memtime();
      else stl[i] = __builtin_amdgcn_s_memtime();
    }
  };
  stamp(0);
  // biases -> LDS (read in the MFMA layout by every wave; visible after the loop's first barrier)
  if constexpr (!BIG)
    for (int i = tid; i < C + F; i += NT) b3s[i] = i < C ? a.b3[i] : a.b1[i - C];

  int issued = 0;  // VMEM ops this wave issued since here (LDS-DMA, buffer stores)
  const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.res, 0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, 0x7ffffff0, 0x00020000);
  const unsigned OOB = 0x80000000u;
  const int lrow = RW::lane_row(lane), lchunk = RW::lane_chunk(lane);  // 128-B-row DMA geometry

  // T: PXW rows x TROW B in 1-KiB pieces of TPR rows (lane -> row, physical chunk)
  {
    constexpr int CPRW = T::TROW / 16;  // 16-B chunks per row
    const int prow = lane / CPRW, pch = lane % CPRW;
#pragma unroll
    for (int p = 0; p < T::TPC; ++p) {
      const int row = p * T::TPR + prow, m = mw + row;
      constexpr int K = CPRW >= 16 ? 15 : CPRW - 1;
      const unsigned off = m < a.M ? (unsigned)(((long)m * a.ldx + (pch ^ (row & K)) * 8) * 2) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(trs, (lds_void*)(wb + p * 1024), 16, off, 0, 0, 0);
    }
    issued += T::TPC;
  }
  const int mark_t = issued;
  // R[c] -> half c & 1: PXW rows x 128 B, pieces of 8 rows (lds_swz layout)
  int mark_r0 = 0, mark_r1 = 0;  // marks of R[c] for the next two chunks (c, c+1)
  auto dma_res = [&](int c) {
    char* dst = wb + (c & 1) * HALF;
#pragma unroll
    for (int p = 0; p < T::HPC; ++p) {
      const int row = p * 8 + lrow, m = mw + row;
      const unsigned off = m < a.M ? (unsigned)(((long)m * a.ldr + c * CC + lchunk * 8) * 2) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rrs, (lds_void*)(dst + p * 1024), 16, off, 0, 0, 0);
    }
    issued += T::HPC;
  };

  // weight panels (64 rows x 64 k): q -> (chunk c, part); part < P1: W3 rows [c*64, +64) x
  // k [64 part, +64); else W1 rows [64 (part - P1), +64) x k [c*64, +64)
  int mk0 = 0, mk1 = 0, mk2 = 0, mk3 = 0;  // issue marks of the pending panels q .. q+NS-2, oldest first
  static_assert(NS == 5 || NS == 3, "mark FIFO depth");
  auto issue_panel = [&](int q) {
    const int c = q / T::PPC, part = q - c * T::PPC;
    char* dst = smem + (q % NS) * SLOT;
#pragma unroll
    for (int j = 0; j < T::PI; ++j) {
      const int pc = wid * T::PI + j;  // 1-KiB piece = 8 rows of one 64-k sub-panel
      const char* src;
      if (part < T::P1) {  // W3 rows [c*64, +64), k [part*KW3 + 64 sp, +64)
        const int sp = pc / 8, r = (pc % 8) * 8 + lrow;
        src = (const char*)a.w3 + ((long)(c * CC + r) * a.ldw3 + part * T::KW3 + sp * 64 + lchunk * 8) * 2;
      } else {             // W1 rows [(part - P1) * RW1, +RW1), k [c*64, +64)
        const int r = (part - T::P1) * T::RW1 + pc * 8 + lrow;
        src = (const char*)a.w1 + ((long)r * a.ldw1 + c * CC + lchunk * 8) * 2;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + pc * 1024), 16, 0, 0);
    }
    issued += T::PI;
  };

  // prologue panels 0 .. NS-2 (the host guarantees nq >= NS - 1)
  issue_panel(0);
  mk0 = issued;
  issue_panel(1);
  mk1 = issued;
  if constexpr (NS == 5) {
    issue_panel(2);
    mk2 = issued;
    issue_panel(3);
    mk3 = issued;
  }

  // T -> B-operand fragments (lane: pixel 16j + frow, k 32ks + 8fq .. +7)
  wait_vm(issued - mark_t);
  bf16x8 tf[T::KS1][FJ];
#pragma unroll
  for (int ks = 0; ks < T::KS1; ++ks)
#pragma unroll
    for (int j = 0; j < FJ; ++j) tf[ks][j] = *(const bf16x8*)(wb + wswz<T::TROW>(16 * j + frow, 4 * ks + fq));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // T read out before R[0], R[1] land on it
  stamp(1);
  if constexpr (RES) {
    dma_res(0);
    mark_r0 = issued;
    if (nch > 1) {
      dma_res(1);
      mark_r1 = issued;
    }
  }

  f32x4 acc1[T::FI1][FJ], acc2[T::FI2][FJ];
#pragma unroll
  for (int i = 0; i < T::FI1; ++i) {  // the accumulators start at the bias: no bias add in the epilogues
    const float4 bb = *(const float4*)(a.b3 + 16 * i + 4 * fq);
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc1[i][j] = (f32x4){bb.x, bb.y, bb.z, bb.w};
  }
#pragma unroll
  for (int i = 0; i < T::FI2; ++i) {
    const float4 bb = *(const float4*)(a.b1 + 16 * i + 4 * fq);
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc2[i][j] = (f32x4){bb.x, bb.y, bb.z, bb.w};
  }
  bf16x8 yb[T::KS2][FJ];

  for (int c = 0; c < nch; ++c) {
#pragma unroll
  for (int part = 0; part < T::PPC; ++part) {  // compile-time part: register arrays stay statically indexed
    const int q = c * T::PPC + part;
    wait_vm(issued - mk0);
    if constexpr (NS == 5) mk0 = mk1, mk1 = mk2, mk2 = mk3;
    else mk0 = mk1;
    __builtin_amdgcn_s_barrier();  // every wave's pieces of panel q landed; slot (q-1) % NS is free
    if (q + NS - 1 < nq) {
      issue_panel(q + NS - 1);
      if constexpr (NS == 5) mk3 = issued;
      else mk1 = issued;
    }
    const char* pan = smem + (q % NS) * SLOT;
    if (part < T::P1) {
      // ---- GEMM1: acc1[ch][px] += W3 panel (64 ch x KW3 k, as 64-k sub-panels) . T ----
#pragma unroll
      for (int sp = 0; sp < T::KW3 / 64; ++sp)
#pragma unroll
      for (int kl = 0; kl < 2; ++kl) {
        bf16x8 fa[T::FI1];
#pragma unroll
        for (int i = 0; i < T::FI1; ++i)
          fa[i] = *(const bf16x8*)(pan + sp * 8192 + lds_swz(16 * i + frow, 4 * kl + fq));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < T::FI1; ++i)
#pragma unroll
          for (int j = 0; j < FJ; ++j)
            acc1[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                fa[i], tf[(part * (T::KW3 / 64) + sp) * 2 + kl][j], acc1[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      if (part == T::P1 - 1) {
        // ---- epilogue of chunk c (this wave only): Y = relu(acc1 + b3 (+ R[c])) in place ----
        char* hb = wb + (c & 1) * HALF;
        if (c < 8) stamp(2 + 4 * c);
        if constexpr (RES) {
          wait_vm(issued - mark_r0);
          mark_r0 = mark_r1;
        }
        if (c < 8) stamp(3 + 4 * c);
#pragma unroll
        for (int i = 0; i < T::FI1; ++i) {
          // the next chunk's bias (the accumulators restart from it): LDS, or global memory (BIG)
          const float* bsrc = BIG ? a.b3 : b3s;
          const float4 nb = *(const float4*)(bsrc + (c + 1 < nch ? c + 1 : c) * CC + 16 * i + 4 * fq);
#pragma unroll
          for (int j = 0; j < FJ; ++j) {
            const int off = lds_swz(16 * j + frow, 2 * i + (fq >> 1)) + 8 * (fq & 1);
            const f32x4 v = acc1[i][j];
            if constexpr (RES) {
              const uint2 r = *(const uint2*)(hb + off);
              *(uint2*)(hb + off) =
                  relu_pack4(v[0] + __uint_as_float(r.x << 16), v[1] + __uint_as_float(r.x & 0xffff0000u),
                             v[2] + __uint_as_float(r.y << 16), v[3] + __uint_as_float(r.y & 0xffff0000u));
            } else {
              *(uint2*)(hb + off) = relu_pack4(v[0], v[1], v[2], v[3]);
            }
            acc1[i][j] = (f32x4){nb.x, nb.y, nb.z, nb.w};
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // Y complete in the half (this wave's lanes)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int ks = 0; ks < T::KS2; ++ks)
#pragma unroll
          for (int j = 0; j < FJ; ++j) yb[ks][j] = *(const bf16x8*)(hb + lds_swz(16 * j + frow, 4 * ks + fq));
        // Y rows -> HBM: item u = (row, 16-B chunk), 8 lanes per 128-B row
#pragma unroll
        for (int u = 0; u < PXW / 8; ++u) {
          const int row = u * 8 + (lane >> 3), ch = lane & 7, m = mw + row;
          const uint4 v = *(const uint4*)(hb + lds_swz(row, ch));
          long ym = m;
          bool keep = m < a.M;
          if (a.ysub > 1) {  // only the pixels a strided reader takes, stored compactly
            const int hw = a.yH * a.yW;
            const int ni = m / hw, rr = m - ni * hw;
            const int hh = rr / a.yW, ww = rr - hh * a.yW;
            keep = keep && hh % a.ysub == 0 && ww % a.ysub == 0;
            ym = ((long)ni * (a.yH / a.ysub) + hh / a.ysub) * (a.yW / a.ysub) + ww / a.ysub;
          }
          const unsigned off = keep ? (unsigned)((ym * a.ldy + c * CC + ch * 8) * 2) : OOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, off, 0, 0);
        }
        issued += PXW / 8;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // half read out before R[c+2] lands on it
        if (RES && c + 2 < nch) {
          dma_res(c + 2);
          mark_r1 = issued;
        }
        if (c < 8) stamp(4 + 4 * c);
      }
    } else {
      // ---- GEMM2: acc2[f][px] += W1 panel (RW1 output rows from (part-P1)*RW1, 64 k) . Y chunk c ----
      const int fb0 = (part - T::P1) * (T::RW1 / 16);  // compile-time after the unroll
#pragma unroll
      for (int kl = 0; kl < 2; ++kl)
#pragma unroll
      for (int g = 0; g < T::RW1 / 64; ++g) {  // 4 output-channel fragments at a time (VGPRs)
        bf16x8 fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = *(const bf16x8*)(pan + lds_swz(16 * (4 * g + i) + frow, 4 * kl + fq));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < FJ; ++j)
            acc2[fb0 + 4 * g + i][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], yb[kl][j], acc2[fb0 + 4 * g + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      if (c < 8 && part == T::PPC - 1) stamp(5 + 4 * c);
    }
  }
  }

  // ---- Z = relu(acc2 + b1) -> the wave buffer as [PXW px][F] (TROW-B rows) -> 16-B row stores ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no R DMA still landing in the buffer
#pragma unroll
  for (int i = 0; i < T::FI2; ++i) {
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int off = wswz<T::ZROW>(16 * j + frow, 2 * i + (fq >> 1)) + 8 * (fq & 1);
      const f32x4 v = acc2[i][j];
      *(uint2*)(wb + off) = relu_pack4(v[0], v[1], v[2], v[3]);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  constexpr int ZC = T::ZROW / 16;  // 16-B chunks per Z row
#pragma unroll
  for (int u = 0; u < PXW * ZC / 64; ++u) {
    const int row = u * (64 / ZC) + lane / ZC, ch = lane % ZC, m = mw + row;
    const uint4 v = *(const uint4*)(wb + wswz<T::ZROW>(row, ch));
    if (m < a.M) *(uint4*)((unsigned short*)a.z + (long)m * a.ldz + ch * 8) = v;
  }
  stamp(34);
  if (!BIG && stamping && tid < 40) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    a.stamps[(long)blockIdx.x * 40 + tid] = stl[tid];
  }
}

}  // namespace chain
}  // namespace dml

template <int F, int NW, int FJ, bool BIG = false, int KX = F, bool RES = true>
static int chain_attr() {
  using T = dml::chain::Cfg<F, NW, FJ, BIG, KX, RES>;
  return (int)hipFuncSetAttribute((const void*)dml::chain::chain_kernel<F, NW, FJ, BIG, KX, RES>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS);
}

template <int F, int NW, int FJ, bool BIG = false, int KX = F, bool RES = true>
static void chain_launch(const DmlExpandReduceArgs* a, hipStream_t s) {
  using T = dml::chain::Cfg<F, NW, FJ, BIG, KX, RES>;
  const long blocks = ((long)a->M + T::BM - 1) / T::BM;
  hipLaunchKernelGGL((dml::chain::chain_kernel<F, NW, FJ, BIG, KX, RES>), dim3((unsigned)blocks), dim3(T::NT),
                     T::LDS, s, *a);
}

extern "C" int dml_chain_init(void) {
  const int rc = chain_attr<128, 8, 2>() | chain_attr<128, 4, 2>() | chain_attr<128, 4, 2, true>() |
                 chain_attr<256, 4, 1>() | chain_attr<256, 8, 1>() | chain_attr<256, 4, 1, true>() |
                 chain_attr<64, 4, 2>() |
                 chain_attr<64, 4, 2, false, 128, false>() | chain_attr<128, 4, 2, false, 256, false>() |
                 chain_attr<128, 4, 2, false, 64, true>() | chain_attr<256, 4, 1, false, 128, true>();
  if (rc) dml_set_error("dml_chain_init: hipFuncSetAttribute failed");
  return rc ? -1 : 0;
}

static bool env_on(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '1';
}

// 1 if the chained kernel serves this block boundary, else 0 (the engine then keeps the two
// 1x1 launches): with a shortcut, F = 64 / C = 256 (stage 2: ResNet50 b256 90.3-90.9k vs
// 88.1-88.7k img/s with the r1 phase-serialised kernel, interleaved on one box, profiles/r3_v6),
// F = 128 / C = 512 or F = 256 / C = 1024; merged projection shortcut (T = [x ; s], K = 2F, no
// residual), F = 64 / C = 256 or F = 128 / C = 512
extern "C" int dml_chain_supported(const DmlExpandReduceArgs* a) {
  const int C = a->C, F = C / 4, FZ = a->fz > 0 ? a->fz : F;
  const bool merged = a->res == nullptr;
  const int kx = merged ? a->kx : F;
  // a stage's last boundary: expand F = 64 -> C = 256 (+ shortcut) feeding the next stage's
  // first reduce 256 -> 128 (template F = reduce width 128, KX = 64; a.C = 256 chunks), or
  // F = 128 -> C = 512 -> reduce 256 (16 pixels per wave: the 256 Z accumulators)
  if (FZ != F)
    return !merged && ((C == 256 && FZ == 128) || (C == 512 && FZ == 256)) && (a->kx == 0 || a->kx == F) &&
           a->M >= 1 && a->ldx % 8 == 0 &&
           a->ldx >= F && a->ldw3 % 8 == 0 && a->ldw3 >= F && a->ldr % 8 == 0 && a->ldr >= C &&
           a->ldy % 8 == 0 && a->ldy >= C && a->ldw1 % 8 == 0 && a->ldw1 >= C && a->ldz % 8 == 0 &&
           a->ldz >= FZ && (long)a->M * (a->ldr > a->ldy ? a->ldr : a->ldy) * 2 < 0x7ffffff0L;
  const long ld = a->ldx > a->ldr ? (a->ldx > a->ldy ? a->ldx : a->ldy) : (a->ldr > a->ldy ? a->ldr : a->ldy);
  const bool shape = merged ? ((F == 64 || F == 128) && a->kx == 2 * F)
                            : ((F == 64 || F == 128 || F == 256) && (a->kx == 0 || a->kx == F));
  return shape && a->M >= 1 && a->ldx % 8 == 0 && a->ldx >= kx && a->ldw3 % 8 == 0 && a->ldw3 >= kx &&
         (merged || (a->ldr % 8 == 0 && a->ldr >= C)) && a->ldy % 8 == 0 && a->ldy >= C && a->ldw1 % 8 == 0 &&
         a->ldw1 >= C && a->ldz % 8 == 0 && a->ldz >= F && (long)a->M * ld * 2 < 0x7ffffff0L;
}

// workgroup shape: 4 waves (two workgroups per CU) by default; DML_CHAIN_WAVES=8 (8 waves) and
// DML_CHAIN_BIG=1 (one barrier per GEMM of a chunk) are A/B variants of the C = 512 form
extern "C" int dml_chain(const DmlExpandReduceArgs* a, hipStream_t s) {
  if (!dml_chain_supported(a)) {
    dml_set_error("dml_chain: unsupported shape (C = 256 / 512 / 1024 with a shortcut, merged C = 256 / 512, "
                  "stage end C = 256 -> 128)");
    return -1;
  }
  static const int nw = [] { const char* e = getenv("DML_CHAIN_WAVES"); return e && atoi(e) == 8 ? 8 : 4; }();
  static const bool big = env_on("DML_CHAIN_BIG");
  const bool merged = a->res == nullptr;
  if (a->fz > 0 && a->fz != a->C / 4) {  // stage-end boundary
    if (a->C == 256) chain_launch<128, 4, 2, false, 64, true>(a, s);  // 64 -> 256 -> 128
    else chain_launch<256, 4, 1, false, 128, true>(a, s);             // 128 -> 512 -> 256
  } else if (merged) {
    if (a->C == 256) chain_launch<64, 4, 2, false, 128, false>(a, s);
    else chain_launch<128, 4, 2, false, 256, false>(a, s);
  } else if (a->C == 256) {
    chain_launch<64, 4, 2>(a, s);
  } else if (a->C == 512) {
    if (nw == 8) chain_launch<128, 8, 2>(a, s);
    else if (big) chain_launch<128, 4, 2, true>(a, s);
    else chain_launch<128, 4, 2>(a, s);
  } else {
    if (nw == 8) chain_launch<256, 8, 1>(a, s);
    else if (big) chain_launch<256, 4, 1, true>(a, s);
    else chain_launch<256, 4, 1>(a, s);
  }
  DML_CHECK_LAUNCH();
  return 0;
}

// The block-boundary entry of the plan executor (the r1 phase-serialised kernels of
// bottleneck_fused.hip were removed in r5; every shape the engine fuses runs chained).
extern "C" int dml_expand_reduce(const DmlExpandReduceArgs* a, hipStream_t s) {
  if (a->C != 256 && a->C != 512 && a->C != 1024) {
    dml_set_error("dml_expand_reduce: unsupported shape (expand width must be 256 / 512 / 1024)");
    return -1;
  }
  return dml_chain(a, s);
}

extern "C" int dml_expand_reduce_init(void) { return dml_chain_init(); }
