// conv_shared.h — pieces shared by the LDS-DMA convolution kernels
// (conv_igemm_v2.hip: implicit GEMM; expand_reduce_chain.hip: chained block boundary).
//
//  * counted vmcnt waits (LDS-DMA completes in issue order with other VMEM ops)
//  * the 16-B-chunk XOR swizzle of a 128-B LDS tile row
//  * the LDS-staged epilogue: fp32 accumulators -> LDS -> each thread owns one
//    8-channel group of a pixel: bias (+ residual, prefetched before the main
//    loop) (+ ReLU) -> one 16-B NHWC store at a channel offset, or into one of up
//    to 4 output segments (fused sibling convs).
#pragma once
#include "common.h"
#include "dml.h"

namespace dml {
namespace convk {

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// byte offset of 16-B chunk `chunk` (0..7) of 128-B tile row `row`
__device__ __forceinline__ int lds_swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

// 64-B tile rows (BK = 32): a ds_read_b128 lane group reads 16 rows; four rows
// share each 256-B bank window, so the chunk is XORed with a per-row-quad key.
// s(q) = {0, 2, 3, 1}[q], q = (row >> 2) & 3, makes all 4 lane groups of an MFMA
// fragment read (16 rows x chunk fq = lane >> 4) hit 64 distinct banks.
__device__ __forceinline__ int swz64_key(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }
__device__ __forceinline__ int lds_swz64(int row, int chunk) { return row * 64 + ((chunk ^ swz64_key(row)) << 4); }

// tile-row geometry for BK = 64 (128-B rows) or BK = 32 (64-B rows)
template <int BK>
struct Rows {
  static_assert(BK == 64 || BK == 32, "BK");
  static constexpr int ROWB = BK * 2;            // bytes per tile row
  static constexpr int CPR = ROWB / 16;          // 16-B chunks per row
  static constexpr int RP = 1024 / ROWB;         // rows per 1-KiB DMA wave-instruction
  static constexpr int KS = BK / 32;             // MFMA k-steps per tile
  __device__ static __forceinline__ int off(int row, int chunk) {
    return BK == 64 ? lds_swz(row, chunk) : lds_swz64(row, chunk);
  }
  // DMA: lane writes physical chunk (lane % CPR) of row (lane / CPR); it must
  // fetch the logical chunk that the read side expects there
  __device__ static __forceinline__ int lane_row(int lane) { return lane / CPR; }
  __device__ static __forceinline__ int lane_chunk(int lane) {
    const int r = lane / CPR;  // row within the piece; pieces start at multiples of RP (>= 8, aligned)
    return BK == 64 ? ((lane & 7) ^ (r & 7)) : ((lane & 3) ^ swz64_key(r));
  }
};

// Epilogue of a BM(pixels) x BN(channels) tile computed by NT threads, staged
// through LDS in P passes of BM/P pixels each (P > 1 keeps the fp32 staging
// buffer within the operand ring's LDS, so the epilogue does not set the
// kernel's LDS size and occupancy). LATE (RES only): the residual is loaded at
// the start of each pass instead of before the main loop, so its EIT x 4 VGPRs
// are not live across the K loop (the tiles whose residual prefetch costs a
// workgroup per CU).
// XT: the workgroup has threads beyond the NT output threads (the loader waves of
// conv_igemm_ws.hip), which skip the residual loads and the output rows.
template <int BM, int BN, int NT, bool RES, int P = 1, bool LATE = false, bool XT = false>
struct Epilogue {
  static constexpr int CG = BN / 8;            // 8-channel groups per pixel
  static constexpr int EIT = BM * CG / NT;     // pixels handled per thread
  static constexpr int CROW = BN * 4 + 16;     // fp32 staging row stride (+16 B pad)
  static constexpr int PB = BM / P;            // pixels per pass
  static constexpr int BYTES = PB * CROW;
  // BN >= 256: the 32+ channel-group lanes of one staging row read 32 B apart, so
  // lanes 16 apart hit the same banks (512 B = 128 dwords); the row's upper half is
  // shifted into the row pad by 16 B (4 banks). Row pitch and writer pattern unchanged.
  static constexpr int HALF = BN >= 256 ? BN * 2 : (1 << 30);
  __device__ __forceinline__ static int sw(int b) { return b + (b >= HALF ? 16 : 0); }
  static_assert(NT % CG == 0 && (BM * CG) % NT == 0, "epilogue mapping");
  static_assert(PB % 16 == 0 && EIT % P == 0, "epilogue passes");

  int cg_t, ch_t, m0, M;
  long yoff;                                    // split-K slice offset (elements, fp32 output)
  bool ch_ok;
  float4 bias0, bias1;
  uint4 rpre[RES ? EIT : 1];

  // Issue the bias / residual loads early: on memory-bound layers the residual
  // read then hides under the operand DMA instead of following the last MFMA.
  // Split-K slice `split` > 0 adds no bias (slice 0 does).
  __device__ __forceinline__ void prefetch(const DmlConvArgs& a, int m0_, int c0, int M_, int tid, int split = 0) {
    m0 = m0_;
    M = M_;
    cg_t = tid % CG;
    ch_t = c0 + cg_t * 8;
    ch_ok = ch_t < a.Cout;
    yoff = (long)split * a.split_ld;
    bias0 = make_float4(0.f, 0.f, 0.f, 0.f);
    bias1 = bias0;
    if (ch_ok && split == 0) {
      bias0 = *(const float4*)(a.bias + ch_t);
      bias1 = *(const float4*)(a.bias + ch_t + 4);
    }
    if constexpr (RES && !LATE) load_res(a, tid, 0, EIT);
  }

  // residual rows [it0, it1) of this thread's channel group -> rpre
  __device__ __forceinline__ void load_res(const DmlConvArgs& a, int tid, int it0, int it1) {
    if (XT && tid >= NT) return;  // wave-uniform: no output rows (a loader wave, conv_igemm_ws.hip)
    const unsigned short* __restrict__ rg = (const unsigned short*)a.res;
#pragma unroll
    for (int it = 0; it < EIT; ++it) {
      if (it < it0 || it >= it1) continue;  // compile-time after unrolling
      const int m = m0 + (tid + it * NT) / CG;
      long rp = m;
      if (a.rsub > 1) {  // shortcut read at stride rsub on its full-resolution grid
        const int hw = a.Ho * a.Wo;
        const int ni = m / hw, r = m - ni * hw;
        const int ho = r / a.Wo, wo = r - ho * a.Wo;
        rp = (long)ni * a.rHW + ((long)ho * a.rW + wo) * a.rsub;
      }
      rpre[it] = (ch_ok && m < M) ? *(const uint4*)(rg + rp * a.ldr + ch_t) : make_uint4(0, 0, 0, 0);
    }
  }

  // acc[i][j]: channel fragment i (MF ch) x pixel fragment j (MF px) of this
  // wave's (WTC x WTP) sub-tile at (wc, wp); MF = 16 (f32x4 accumulators of
  // v_mfma_f32_16x16x32_bf16: lane holds channels 4*(lane>>4)+0..3 of pixel
  // lane&15) or MF = 32 (f32x16 of v_mfma_f32_32x32x16_bf16: register group g
  // holds channels 8g+4*(lane>>5)+0..3 of pixel lane&31). Caller must have
  // retired all DMA. has_acc = false (wave-uniform): the calling wave holds no
  // accumulators (a loader wave of the warp-specialised kernel, conv_igemm_ws.hip) and
  // only takes part in the bias / residual / store half.
  template <int MF, int FI, int FJ, int WTP, int WTC, class Acc>
  __device__ __forceinline__ void store(const DmlConvArgs& a, char* smem, Acc (&acc)[FI][FJ], int wp, int wc,
                                        int lane, int tid, bool has_acc = true) {
    static_assert(MF == 16 || MF == 32, "MFMA fragment size");
    static_assert(PB % MF == 0, "an epilogue pass must hold whole pixel fragments");
    const int frow = lane & (MF - 1), fq = lane / MF;
    // destination of this thread's channel group: the plain output, or the
    // segment (fused sibling conv) that owns channel ch_t
    void* ybase = a.y;
    int ldy = a.ldy, relu = a.relu, choff = ch_t;
    if (a.nseg > 0) {
      int sgi = 0;
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (q < a.nseg && ch_t >= a.seg_c0[q]) sgi = q;
      ybase = a.seg_y[sgi];
      ldy = a.seg_ldy[sgi];
      relu = a.seg_relu[sgi];
      choff = ch_t - a.seg_c0[sgi];
    }
#pragma unroll
    for (int pass = 0; pass < P; ++pass) {
      // late residual: this pass's rows in flight while the accumulators are staged
      if constexpr (RES && LATE) load_res(a, tid, pass * (EIT / P), (pass + 1) * (EIT / P));
      __syncthreads();  // operand tiles (pass 0) / the previous pass's staging rows are free
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        if (!has_acc) break;                                       // wave-uniform
        if (P > 1 && (wp * WTP + j * MF) / PB != pass) continue;  // wave-uniform
        const int px = wp * WTP + j * MF + frow - pass * PB;
#pragma unroll
        for (int i = 0; i < FI; ++i) {
          if constexpr (MF == 16) {
            const int ch = wc * WTC + i * 16 + fq * 4;
            *(f32x4*)(smem + px * CROW + sw(ch * 4)) = acc[i][j];
          } else {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int ch = wc * WTC + i * 32 + g * 8 + fq * 4;
              *(f32x4*)(smem + px * CROW + sw(ch * 4)) =
                  (f32x4){acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
            }
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int it = pass * (EIT / P); it < (pass + 1) * (EIT / P); ++it) {
        if (XT && tid >= NT) break;  // a loader wave beyond the NT output threads (conv_igemm_ws.hip)
        const int px = (tid + it * NT) / CG;
        const int m = m0 + px;
        if (m >= M || !ch_ok) continue;
        const int lp = px - pass * PB;
        const float4 v0 = *(const float4*)(smem + lp * CROW + sw(cg_t * 32));
        const float4 v1 = *(const float4*)(smem + lp * CROW + sw(cg_t * 32) + 16);
        float f[8] = {v0.x + bias0.x, v0.y + bias0.y, v0.z + bias0.z, v0.w + bias0.w,
                      v1.x + bias1.x, v1.y + bias1.y, v1.z + bias1.z, v1.w + bias1.w};
        if constexpr (RES) {
          const uint4 r = rpre[it];
          f[0] += bf2f(r.x & 0xffff); f[1] += bf2f(r.x >> 16);
          f[2] += bf2f(r.y & 0xffff); f[3] += bf2f(r.y >> 16);
          f[4] += bf2f(r.z & 0xffff); f[5] += bf2f(r.z >> 16);
          f[6] += bf2f(r.w & 0xffff); f[7] += bf2f(r.w >> 16);
        }
        if (relu) {
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] = fmaxf(f[q], 0.f);
        }
        if (a.out_f32) {
          float* yp = (float*)ybase + yoff + (long)m * ldy + choff;
          *(float4*)yp = make_float4(f[0], f[1], f[2], f[3]);
          *(float4*)(yp + 4) = make_float4(f[4], f[5], f[6], f[7]);
        } else {
          *(uint4*)((unsigned short*)ybase + (long)m * ldy + choff) =
              make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
        }
      }
    }
  }
};

}  // namespace convk
}  // namespace dml
