// conv_igemm_v2.hip — LDS-DMA pipelined MFMA implicit-GEMM convolution (gfx950).
//
// Implicit-GEMM convolution over DmlConvArgs (validated and dispatched by
// conv_dispatch.hip). GEMM view, computed TRANSPOSED: D[c][m] = sum_k W[c][k] X[k][m]
// with c = output channel on the MFMA rows and m = output pixel on the columns:
// the v_mfma_f32_16x16x32_bf16 accumulator of lane l then holds 4 CONSECUTIVE
// output channels of one pixel (NHWC-friendly epilogue). Built around the CDNA4
// memory path:
//
//  * Operand tiles go global -> LDS by LDS-DMA (no VGPR round trip):
//      activations: buffer_load_dwordx4 ... lds through a raw buffer descriptor.
//        The implicit-im2col zero padding (out-of-image taps, K tail, M tail)
//        is produced by the hardware range check: such lanes get an offset past
//        num_records and the DMA writes zeros.
//      weights:     global_load_lds_dwordx4.
//    A wave-instruction writes 1 KiB = 8 tile rows of 128 B contiguously, so the
//    bank-conflict swizzle (16-B chunk ^= row & 7) is applied on the SOURCE side:
//    lane L always fetches logical chunk (L & 7) ^ (L >> 3) of its row.
//  * STAGES-deep LDS ring with counted `s_waitcnt vmcnt(N)` + raw s_barrier —
//    one barrier per 64-deep K tile, loads for tiles kt+1..kt+STAGES-2 stay in
//    flight across it (never __syncthreads() in the loop: its fence would drain
//    the DMA).
//  * Epilogue staged through LDS: fp32 accumulators -> LDS -> each thread
//    handles 8 consecutive output channels of one pixel: bias + residual (16-B
//    coalesced load) + ReLU -> one 16-B coalesced NHWC store. Rows of a pixel
//    are contiguous across 16 lanes, so stores/residual loads are full lines.
//  * XCD-aware bijective block remap; channel tiles fastest so the blocks on
//    one XCD share the activation rows in its L2.
#include "conv_shared.h"
#include "pool_shared.h"

#ifndef DML_V2_PROBE
#define DML_V2_PROBE 0  // A/B timing probes only (tools/build_variant.py, tools/conv_ab.py):
                        // 1 = no operand DMA (MFMAs on stale LDS), 2 = no fragment reads, 3 = no MFMAs,
                        // 4 = every DMA reads the same 16-KiB block (L2-resident: issue cost without
                        //     HBM latency / bandwidth), 5 = no per-lane K walk (advance() reduced to
                        //     one masked add: the address math's cost), 6 = no K-loop barrier
#endif

namespace dml {
namespace v2 {

using convk::lds_swz;
using convk::lds_void;
using convk::wait_vmcnt;

// workgroups per CU that the larger of two LDS regions allows (160 KiB per CU)
constexpr int lds_occupancy(int a, int b) { return 163840 / (a > b ? a : b); }

template <int BM, int BN, int WM, int WN, int STAGES, int BK_ = 64, int MF_ = 16>
struct Cfg {
  static constexpr int NW = WM * WN;          // waves
  static constexpr int NT = NW * 64;          // threads
  static constexpr int WTP = BM / WM;         // pixels per wave
  static constexpr int WTC = BN / WN;         // channels per wave
  static constexpr int MF = MF_;              // MFMA fragment: 16 (16x16x32) or 32 (32x32x16)
  static constexpr int FJ = WTP / MF;         // fragments along pixels
  static constexpr int FI = WTC / MF;         // fragments along channels
  static constexpr int BK = BK_;
  using R = convk::Rows<BK>;
  static constexpr int ROWB = R::ROWB;        // 128 B (BK 64) or 64 B (BK 32) per tile row
  static constexpr int XI = BM / R::RP / NW;  // X DMA instructions per wave per K tile
  static constexpr int WI = BN / R::RP / NW;  // W DMA instructions per wave per K tile
  static constexpr int L = XI + WI;           // vm ops per thread per K tile
  static constexpr int STAGE_BYTES = (BM + BN) * ROWB;
  static constexpr int PIPE_BYTES = STAGES * STAGE_BYTES;
  // Epilogue staging passes: the fewest (1, 2, 4) whose fp32 staging rows fit in
  // the operand ring, so the epilogue never raises the LDS size (occupancy).
  static constexpr int CROW = BN * 4 + 16;
  static constexpr bool EP_OK2 = (BM / 2) % MF == 0 && ((BM * BN / 8) / NT) % 2 == 0;
  static constexpr bool EP_OK4 = (BM / 4) % MF == 0 && ((BM * BN / 8) / NT) % 4 == 0;
  // most passes allowed, then back off to the fewest passes that keep that occupancy
  static constexpr int EP_MAX = EP_OK4 ? 4 : (EP_OK2 ? 2 : 1);
  static constexpr int OCC_BEST = lds_occupancy(PIPE_BYTES, (BM / EP_MAX) * CROW);
  static constexpr int EP = lds_occupancy(PIPE_BYTES, BM * CROW) >= OCC_BEST ? 1
                          : (EP_OK2 && lds_occupancy(PIPE_BYTES, (BM / 2) * CROW) >= OCC_BEST) ? 2 : EP_MAX;
  static constexpr int EPI_BYTES = (BM / EP) * CROW;  // = convk::Epilogue<BM, BN, NT, *, EP>::BYTES
  static constexpr int LDS = PIPE_BYTES > EPI_BYTES ? PIPE_BYTES : EPI_BYTES;
  static_assert(XI >= 1 && WI >= 1, "each wave needs >=1 DMA instruction per operand");
  static_assert(BM % (R::RP * NW) == 0 && BN % (R::RP * NW) == 0, "tile rows must split evenly across waves");
  static_assert(FI >= 1 && FJ >= 1 && WTP % MF == 0 && WTC % MF == 0, "wave tile too small");
  static_assert((STAGES - 2) * L < 64, "vmcnt overflow");
};

// One workgroup's tile: logical block Lb (already XCD-remapped) of a grid of
// nblk blocks that runs conv `a` (the plain kernel's whole grid, or one member
// of a grouped launch).
template <int BM, int BN, int WM, int WN, int STAGES, bool RES, int BK, int MF = 16, bool LATE = false>
__device__ __forceinline__ void conv_v2_tile(const DmlConvArgs& a, int Lb, int nblk) {
  using T = Cfg<BM, BN, WM, WN, STAGES, BK, MF>;
  using RW = typename T::R;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int M = a.N * a.Ho * a.Wo;
  const int ntc = (a.Cout + BN - 1) / BN;
  // split-K: the grid is ksplit slices of the tile grid; slice `split` runs K
  // tiles [kbeg, kbeg + nk) and writes its own fp32 partial output
  const int ksplit = a.ksplit > 1 ? a.ksplit : 1;
  int split = 0;
  if (ksplit > 1) {  // wave-uniform; the common path skips the division
    const int ntiles = nblk / ksplit;
    split = Lb / ntiles;
    Lb -= split * ntiles;
  }
  // channel tiles fastest: an XCD's blocks share activation rows (a
  // pixel-fastest order, sharing weight panels instead, measured neutral warm
  // and cold on the K-heavy stage-4/5 layers, profiles/r2_v31)
  const int tc = Lb % ntc, tm = Lb / ntc;
  const int m0 = tm * BM, c0 = tc * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

  // ---- per-lane DMA bookkeeping ----
  const int lrow = RW::lane_row(lane);         // row within an RP-row DMA piece
  const int lchunk = RW::lane_chunk(lane);     // logical K chunk this lane always fetches
  // X rows of this lane: piece q = wid*XI + j -> row RP*q + lrow
  // Element offset of (row, k) = base[row] + koff(k) with
  //   base[row] = (pix0 + ih0*W + iw0) * ldx          (per row, fixed)
  //   koff(k)   = (rr*dh*W + ss*dw) * ldx + cc        (per lane, row-independent)
  // so the K loop does one add per row (no multiplies); the bounds test uses the
  // running tap displacement (dih, diw).
  int base[T::XI], ih0[T::XI], iw0[T::XI];
  const int HoWo = a.Ho * a.Wo;
#pragma unroll
  for (int j = 0; j < T::XI; ++j) {
    const int m = m0 + (wid * T::XI + j) * RW::RP + lrow;
    if (m < M) {
      const int n = m / HoWo;
      const int rem = m - n * HoWo;
      const int oh = rem / a.Wo;
      const int ow = rem - oh * a.Wo;
      ih0[j] = oh * a.sh - a.ph;
      iw0[j] = ow * a.sw - a.pw;
      base[j] = (n * a.H * a.W + ih0[j] * a.W + iw0[j]) * a.ldx;
    } else {
      base[j] = 0;
      ih0[j] = -(1 << 28);  // fails every bounds test: zero row
      iw0[j] = 0;
    }
  }
  const int dh = a.dh > 0 ? a.dh : 1, dw = a.dw > 0 ? a.dw : 1;
  const int step_s = dw * a.ldx;                 // koff change for ss += 1
  const int step_r = dh * a.W * a.ldx;           // koff change for rr += 1
  int cc = lchunk * 8, ss = 0, rr = 0, dih = 0, diw = 0, koff = lchunk * 8;
  auto advance = [&](int by) {
    if (DML_V2_PROBE == 5) {  // stays inside the row's first 64 channels (Cin >= 64): in bounds
      koff = (koff + by) & 63;
      return;
    }
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
        dih = rr < a.kh ? dih + dh : (1 << 28);  // K tail: every row out of bounds -> zeros
      }
    }
  };
  advance(0);
  int nk = a.Kpad / T::BK, kbeg = 0;
  if (ksplit > 1) {
    const int nk_slice = (nk + ksplit - 1) / ksplit;
    kbeg = split * nk_slice;
    nk = max(0, min(nk_slice, nk - kbeg));
    if (kbeg > 0) advance(kbeg * T::BK);
  }

  // buffer descriptor over the activations (range check -> zero fill)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);
  const unsigned OOB = 0x80000000u;
  const char* wbase =
      (const char*)a.w + ((long)(c0 + wid * T::WI * RW::RP + lrow) * a.Kpad + (long)kbeg * T::BK + lchunk * 8) * 2;
  const long wstep_row = (long)RW::RP * a.Kpad * 2;  // next RP-row piece

  auto issue = [&](int kt, int stage) {
    if (DML_V2_PROBE == 1) return;
    char* sx = smem + stage * T::STAGE_BYTES;
    char* sw = sx + BM * T::ROWB;
#pragma unroll
    for (int j = 0; j < T::XI; ++j) {
      const int ih = ih0[j] + dih, iw = iw0[j] + diw;
      const unsigned ok = ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
      const unsigned msk = 0u - ok;  // branch-free select (no exec-mask split around the DMA)
      const unsigned off = DML_V2_PROBE == 4 ? ((unsigned)((base[j] + koff) * 2) & 0x3ff0u)
                                             : (((unsigned)((base[j] + koff) * 2) & msk) | (OOB & ~msk));
      // cache policy: default (a non-temporal stream, aux = 2, measured -1 % end to end: DESIGN §2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void*)(sx + (wid * T::XI + j) * 1024), 16, off, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < T::WI; ++j) {
      const char* src = DML_V2_PROBE == 4 ? (const char*)a.w + ((lrow * 128 + lchunk * 16) & 0x3ff0)
                                          : wbase + j * wstep_row + (long)kt * T::BK * 2;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sw + (wid * T::WI + j) * 1024), 16, 0, 0);
    }
    advance(T::BK);
  };

  using Acc = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  Acc acc[T::FI][T::FJ];
#pragma unroll
  for (int i = 0; i < T::FI; ++i)
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) acc[i][j] = (Acc)(0.f);

  const int wc = wid % WN, wp = wid / WN;
  // fragment lane map: row (lane & (MF-1)) of the fragment, 16-B K chunk
  // (lane / MF) of each MFMA k-step (32 deep for MF 16, 16 deep for MF 32)
  const int frow = lane & (MF - 1), fq = lane / MF;

  // prologue: tiles 0 .. STAGES-2 in flight
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s);

  // epilogue operands (bias, residual) prefetched behind the first DMA tiles
  convk::Epilogue<BM, BN, T::NT, RES, T::EP, LATE> epi;
  epi.prefetch(a, m0, c0, M, tid, split);

  for (int kt = 0; kt < nk; ++kt) {
    // retire tile kt (leave the younger STAGES-2 tiles in flight), then barrier
    if (kt + STAGES - 2 < nk) wait_vmcnt<(STAGES - 2) * T::L>();
    else wait_vmcnt<0>();
    if (DML_V2_PROBE != 6) __builtin_amdgcn_s_barrier();
    // Refill the stage freed by tile kt-1 right after the barrier, before the
    // fragment reads. A/B-measured (profiles/r1_v5/sched_ab_v*.json): issuing it
    // between the two k-steps, or interleaving it among the MFMAs with
    // sched_group_barrier, was 8-15 % slower on both 3x3 and 1x1 layers.
    if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    const char* sx = smem + (kt % STAGES) * T::STAGE_BYTES;
    const char* sw = sx + BM * T::ROWB;
    // Both 32-deep k-steps' fragments are read up front (separate registers), so
    // the second step's ds_reads are in flight while the first step's MFMAs run;
    // hipcc emits a counted lgkmcnt before each MFMA group.
    constexpr int KSM = BK / (512 / MF);  // MFMA k-steps per tile (32 or 16 deep)
    constexpr int CPS = 64 / MF;          // 16-B chunks per k-step (4 or 2)
    bf16x8 fa[KSM][T::FI], fb[KSM][T::FJ];
#pragma unroll
    for (int ks = 0; ks < KSM; ++ks) {
      const int ch = ks * CPS + fq;
#pragma unroll
      for (int i = 0; i < T::FI; ++i)
        fa[ks][i] = DML_V2_PROBE == 2 ? (bf16x8)(bf16)(float)(kt + i)
                                      : *(const bf16x8*)(sw + RW::off(wc * T::WTC + i * MF + frow, ch));
#pragma unroll
      for (int j = 0; j < T::FJ; ++j)
        fb[ks][j] = DML_V2_PROBE == 2 ? (bf16x8)(bf16)(float)(kt - j)
                                      : *(const bf16x8*)(sx + RW::off(wp * T::WTP + j * MF + frow, ch));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KSM; ++ks)
#pragma unroll
      for (int i = 0; i < T::FI; ++i)
#pragma unroll
        for (int j = 0; j < T::FJ; ++j) {
          if constexpr (DML_V2_PROBE == 3)
            acc[i][j][0] += (float)fa[ks][i][0] * (float)fb[ks][j][1];
          else if constexpr (MF == 16)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  }

  // all DMA retired (vmcnt(0) on the last tile); epilogue through LDS
  epi.template store<MF, T::FI, T::FJ, T::WTP, T::WTC>(a, smem, acc, wp, wc, lane, tid);
}

// W: minimum waves/SIMD asked of the register allocator (launch-bounds hint; 1 =
// none). Set per tile only where it reaches the LDS-limited occupancy without
// scratch (checked by tests/test_kernel_occupancy.py).
template <int BM, int BN, int WM, int WN, int STAGES, bool RES, int BK = 64, int MF = 16, bool LATE = false, int W = 1>
__global__ __launch_bounds__(WM* WN * 64, W) void conv_v2_kernel(DmlConvArgs a) {
  conv_v2_tile<BM, BN, WM, WN, STAGES, RES, BK, MF, LATE>(a, xcd_remap(blockIdx.x, gridDim.x), gridDim.x);
}

// Grouped launch: up to DML_CONV_GROUP_MAX independent convs (InceptionV3's
// parallel branch convs: different kh x kw, inputs and outputs) and up to
// DML_GROUP_POOL_MAX independent 3x3 pools of the same graph level share ONE
// grid; block -> member by the prefix block offsets. The conv tiles are
// XCD-remapped over their own block range; the pools' blocks come last, so they
// fill the conv tiles' tail instead of paying a launch and a drain of their own.
template <int BM, int BN, int WM, int WN, int STAGES, int BK = 64>
__global__ __launch_bounds__(WM* WN * 64) void conv_v2_group_kernel(DmlConvGroupArgs g) {
  const int b = blockIdx.x, nconv = g.off[g.n];
  if (b >= nconv) {
    // pool member: 256 work items per block, raw block order (dispatched last and
    // round-robin over the XCDs; an XCD-remapped range would put them all on one)
    const int nm = g.n + g.npool;
    int i = g.n;
#pragma unroll
    for (int q = 1; q < DML_GROUP_POOL_MAX; ++q)
      if (g.n + q < nm && b >= g.off[g.n + q]) i = g.n + q;
    i = __builtin_amdgcn_readfirstlane(i);
    const DmlPoolArgs& p = g.pool[i - g.n];
    const unsigned t = (unsigned)(b - g.off[i]) * 256u + threadIdx.x;
    if (t < (unsigned)poolk::pool_work(p)) {
      if (p.mode == 0) poolk::pool3x3_item<0, true>(p, t);
      else poolk::pool3x3_item<1, true>(p, t);
    }
    return;
  }
  // Conv tiles: every member is cut into 8 contiguous chunks, one per XCD
  // (block b runs on XCD b % 8), the members' remainder tiles rotating over the
  // XCDs so each XCD gets exactly its share of blocks. On each XCD the members
  // come in host order — longest K first (launch_group) — so the long tiles are
  // dispatched first (longest-processing-time order) and no XCD is left with
  // only the short member's tiles.
  const int x = b & 7;
  int j = b >> 3, i = 0, tile = 0, rot = 0;
  bool found = false;
#pragma unroll
  for (int q = 0; q < DML_CONV_GROUP_MAX; ++q) {
    if (q < g.n && !found) {
      const int t = g.off[q + 1] - g.off[q], qd = t >> 3, r = t & 7;
      const int cnt = qd + (((x - rot) & 7) < r ? 1 : 0);
      if (j < cnt) {
        int before = 0;  // XCDs before x holding one of this member's remainder tiles
        for (int k = 0; k < x; ++k) before += (((k - rot) & 7) < r) ? 1 : 0;
        i = q;
        tile = x * qd + before + j;
        found = true;
      } else {
        j -= cnt;
      }
      rot = (rot + r) & 7;
    }
  }
  i = __builtin_amdgcn_readfirstlane(i);
  tile = __builtin_amdgcn_readfirstlane(tile);
  conv_v2_tile<BM, BN, WM, WN, STAGES, false, BK>(g.a[i], tile, g.off[i + 1] - g.off[i]);
}

template <int BM, int BN, int WM, int WN, int STAGES, int BK = 64, int MF = 16, bool LATE = false, int W = 1>
static int launch(const DmlConvArgs* a, hipStream_t s) {
  using T = Cfg<BM, BN, WM, WN, STAGES, BK, MF>;
  const long M = (long)a->N * a->Ho * a->Wo;
  const long tiles = ((M + BM - 1) / BM) * ((a->Cout + BN - 1) / BN) * (a->ksplit > 1 ? a->ksplit : 1);
  if (a->res)
    hipLaunchKernelGGL((conv_v2_kernel<BM, BN, WM, WN, STAGES, true, BK, MF, LATE, W>), dim3((unsigned)tiles),
                       dim3(T::NT), T::LDS, s, *a);
  else
    hipLaunchKernelGGL((conv_v2_kernel<BM, BN, WM, WN, STAGES, false, BK, MF, false, LATE ? 1 : W>),
                       dim3((unsigned)tiles), dim3(T::NT), T::LDS, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN, int STAGES, int BK = 64>
static int launch_group(const DmlConvGroupArgs* g, hipStream_t s) {
  using T = Cfg<BM, BN, WM, WN, STAGES, BK>;
  static_assert(T::NT == 256, "pool members run 256 work items per block");
  DmlConvGroupArgs h = *g;
  // longest K first: the kernel dispatches each XCD's tiles in member order
  for (int i = 1; i < h.n; ++i)
    for (int k = i; k > 0 && h.a[k].Kpad > h.a[k - 1].Kpad; --k) {
      const DmlConvArgs t = h.a[k];
      h.a[k] = h.a[k - 1];
      h.a[k - 1] = t;
    }
  h.off[0] = 0;
  for (int i = 0; i < h.n; ++i) {
    const long M = (long)h.a[i].N * h.a[i].Ho * h.a[i].Wo;
    h.off[i + 1] = h.off[i] + (int)(((M + BM - 1) / BM) * ((h.a[i].Cout + BN - 1) / BN));
  }
  for (int j = 0; j < h.npool; ++j)
    h.off[h.n + j + 1] = h.off[h.n + j] + (int)((poolk::pool_work(h.pool[j]) + 255) / 256);
  hipLaunchKernelGGL((conv_v2_group_kernel<BM, BN, WM, WN, STAGES, BK>), dim3((unsigned)h.off[h.n + h.npool]),
                     dim3(T::NT), T::LDS, s, h);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN, int STAGES, int BK = 64>
static int set_attr_group() {
  using T = Cfg<BM, BN, WM, WN, STAGES, BK>;
  return (int)hipFuncSetAttribute((const void*)conv_v2_group_kernel<BM, BN, WM, WN, STAGES, BK>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS);
}

template <int BM, int BN, int WM, int WN, int STAGES, int BK = 64, int MF = 16, bool LATE = false, int W = 1>
static int set_attr() {
  using T = Cfg<BM, BN, WM, WN, STAGES, BK, MF>;
  return (int)hipFuncSetAttribute((const void*)conv_v2_kernel<BM, BN, WM, WN, STAGES, true, BK, MF, LATE, W>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS) |
         (int)hipFuncSetAttribute(
             (const void*)conv_v2_kernel<BM, BN, WM, WN, STAGES, false, BK, MF, false, LATE ? 1 : W>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS);
}

}  // namespace v2
}  // namespace dml

// Tile configurations: id, BM (pixels), BN (channels), WM x WN waves, ring
// STAGES, BK, MF (MFMA fragment: 16 = v_mfma_f32_16x16x32_bf16, 32 =
// v_mfma_f32_32x32x16_bf16), RL (residual load: 0 = prefetched before the K
// loop, 1 = in the epilogue), W (min waves/SIMD register hint; for an RL 1 twin
// it applies to the residual form only). The ids are the ABI of the plan builder and the tuner
// (ops/tuning.py); validated by dml_conv (conv_dispatch.hip).
#define DML_V2_TILES(X)                                                                            \
  X(10, 256, 128, 4, 2, 3, 64, 16, 0, 1)   /* 8 waves, 64x64 per wave */                                     \
  X(11, 128, 128, 2, 2, 2, 64, 16, 0, 1)   /* 4 waves, 64x64 per wave, 2 blocks/CU */                        \
  X(12, 256, 64, 4, 1, 2, 64, 16, 0, 1)    /* 4 waves, 64x64 per wave */                                     \
  X(13, 128, 256, 2, 4, 3, 64, 16, 0, 1)   /* 8 waves, 64x64 per wave */                                     \
  X(14, 64, 128, 1, 4, 2, 64, 16, 0, 1)    /* 4 waves, 64px x 32ch per wave */                               \
  X(15, 128, 64, 2, 2, 2, 64, 16, 0, 1)    /* 4 waves, 64px x 32ch per wave */                               \
  X(16, 256, 128, 4, 2, 2, 64, 16, 0, 1)   /* 8 waves, 2-stage */                                            \
  X(17, 128, 128, 2, 2, 3, 64, 16, 0, 1)   /* 4 waves, 3-stage */                                            \
  X(18, 256, 32, 4, 1, 2, 64, 16, 0, 1)    /* 4 waves (Cout = 32 layers) */                                  \
  X(19, 128, 128, 2, 4, 3, 64, 16, 0, 1)   /* 8 waves, 64px x 32ch per wave, 3-stage */                      \
  X(20, 128, 128, 4, 2, 3, 64, 16, 0, 1)   /* 8 waves, 32px x 64ch per wave, 3-stage */                      \
  X(21, 128, 256, 2, 4, 2, 64, 16, 0, 1)   /* 8 waves, 64x64 per wave, 2-stage */                            \
  X(22, 64, 256, 1, 4, 2, 64, 16, 0, 1)    /* 4 waves, 64px x 64ch per wave */                               \
  /* BK = 32 (64-B tile rows): half-size stages -> more workgroups per CU */                        \
  X(23, 64, 128, 1, 4, 2, 32, 16, 0, 1)                                                                      \
  X(24, 128, 64, 2, 2, 2, 32, 16, 0, 1)                                                                      \
  X(25, 128, 128, 2, 2, 2, 32, 16, 0, 1)                                                                     \
  X(26, 64, 128, 1, 4, 3, 32, 16, 0, 1)                                                                      \
  X(27, 128, 64, 2, 2, 3, 32, 16, 0, 1)                                                                      \
  X(28, 128, 128, 2, 2, 3, 32, 16, 0, 1)                                                                     \
  /* deeper rings (the epilogue no longer sets the LDS size: Cfg::EP passes) */                    \
  X(29, 128, 128, 2, 2, 4, 32, 16, 0, 1)   /* 64 KiB: 2 blocks/CU */                                         \
  X(30, 256, 128, 4, 2, 3, 32, 16, 0, 1)   /* 8 waves, 72 KiB */                                             \
  X(31, 128, 256, 2, 4, 3, 32, 16, 0, 1)   /* 8 waves, 72 KiB */                                             \
  X(32, 64, 128, 1, 4, 3, 64, 16, 0, 1)    /* 72 KiB: 2 blocks/CU */                                         \
  X(33, 64, 128, 1, 4, 4, 32, 16, 0, 1)    /* 48 KiB: 3 blocks/CU */                                         \
  /* 256x256: half the L2->LDS bytes per MFMA of 128x128 (the 3x3 layers are L2-bound); its */     \
  /* residual form spills at 2 waves/SIMD (not a tuner candidate for residual layers) */           \
  X(34, 256, 256, 2, 4, 3, 32, 16, 0, 1)   /* 8 waves, 128px x 64ch per wave, 96 KiB */                      \
  X(36, 128, 32, 2, 1, 3, 32, 16, 0, 1)    /* Cout = 32 layers (InceptionV3 stem): 2 waves, 30 KiB */        \
  X(37, 256, 32, 4, 1, 3, 64, 16, 0, 1)    /* 4 waves, 3-stage */                                     \
  /* 3-stage BK64 forms of the 64-channel tiles (the stride-1 Cout 64 / 192 layers' 2-stage */     \
  /* 128x64 tile waits on DRAM latency every K tile: one tap of 64 channels per stage) */         \
  X(38, 128, 64, 2, 2, 3, 64, 16, 0, 1)    /* 72 KiB: 2 blocks/CU */                                         \
  X(39, 256, 64, 4, 1, 3, 64, 16, 0, 1)    /* 120 KiB: 1 block/CU */                                         \
  /* v_mfma_f32_32x32x16_bf16 twins (MF 32: 32x32 fragments, f32x16 accumulators) of the two */   \
  /* most-picked tiles; kept as A/B probes, not tuner candidates: over all 64 ResNet50 / */        \
  /* InceptionV3 shapes x 8 tile pairs the MF 32 form ran a median 4-6 % slower (best on 2 */      \
  /* HBM-bound K=64 shapes, within noise; profiles/r2_v23/mf32_*.json) */                         \
  X(48, 64, 128, 1, 4, 2, 64, 32, 0, 1)    /* = 14 */                                                    \
  X(49, 128, 64, 2, 2, 2, 64, 32, 0, 1)    /* = 15 */                                                 \
  /* late-residual twins (RL 1: residual loaded in the epilogue, not across the K loop) of the */  \
  /* tiles whose residual prefetch costs occupancy; residual layers only (ops/tuning.py) */        \
  X(56, 256, 128, 4, 2, 3, 32, 16, 1, 4)  /* = 30 */                                                  \
  X(57, 128, 256, 2, 4, 3, 32, 16, 1, 1)  /* = 31 */                                                  \
  X(58, 128, 128, 2, 2, 2, 32, 16, 1, 1)  /* = 25 */                                                  \
  X(59, 128, 128, 2, 2, 3, 32, 16, 1, 1)  /* = 28 */                                                  \
  X(60, 64, 128, 1, 4, 2, 32, 16, 1, 1)   /* = 23 */
// (r2, measured and removed: 192x96 and 192x192 tiles with 64px x 96ch wave
// tiles for InceptionV3's Cout = 96/160/192 layers won no shape; conv2d_5 156 us
// vs 147 us on 128x64, profiles/r2_v8/cb_192.log. Deep BK64 rings (4-5 stages,
// 96-160 KiB, 1 workgroup/CU) for the long-K stage-4/5 layers were 1.3-1.9x
// slower than the 2-3 workgroups/CU tiles: co-resident workgroups hide the L2
// latency better than a deeper ring, profiles/r2_v11/cb_r50.log)

// the 4-wave tiles also instantiated as grouped launches (pool members run 256
// work items per block)
#define DML_V2_GROUP_TILES(X)                                                                      \
  X(11, 128, 128, 2, 2, 2, 64) X(12, 256, 64, 4, 1, 2, 64) X(14, 64, 128, 1, 4, 2, 64)             \
  X(15, 128, 64, 2, 2, 2, 64) X(17, 128, 128, 2, 2, 3, 64) X(22, 64, 256, 1, 4, 2, 64)             \
  X(23, 64, 128, 1, 4, 2, 32) X(24, 128, 64, 2, 2, 2, 32) X(25, 128, 128, 2, 2, 2, 32)             \
  X(26, 64, 128, 1, 4, 3, 32) X(27, 128, 64, 2, 2, 3, 32) X(28, 128, 128, 2, 2, 3, 32)             \
  X(29, 128, 128, 2, 2, 4, 32) X(32, 64, 128, 1, 4, 3, 64) X(33, 64, 128, 1, 4, 4, 32)

// Raise the dynamic-LDS limit of every v2 instantiation once (before any
// launch or graph capture). Called by the Python loader.
extern "C" int dml_conv_v2_init(void) {
  using namespace dml::v2;
  int rc = 0;
#define DML_SET(id, BM, BN, WM, WN, ST, BK, MF, RL, W) rc |= set_attr<BM, BN, WM, WN, ST, BK, MF, RL, W>();
  DML_V2_TILES(DML_SET)
#undef DML_SET
#define DML_SET(id, BM, BN, WM, WN, ST, BK) rc |= set_attr_group<BM, BN, WM, WN, ST, BK>();
  DML_V2_GROUP_TILES(DML_SET)
#undef DML_SET
  if (rc) dml_set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  if (!rc && dml_chain_init() != 0) return -1;  // chained block-boundary kernels (expand_reduce_chain.hip)
  if (!rc && dml_conv_ws_init() != 0) return -1;  // warp-specialised tiles (conv_igemm_ws.hip)
  if (!rc && dml_conv_wsp_init() != 0) return -1;  // persistent warp-specialised tiles (conv_igemm_wsp.hip)
  if (!rc && dml_conv_rr_init() != 0) return -1;   // row-ring 3x3 kernel (conv_rowring.hip)
  return rc ? -1 : 0;
}

extern "C" int dml_conv_v2(const DmlConvArgs* a, int cfg, hipStream_t s) {
  using namespace dml::v2;
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST, BK, MF, RL, W) \
  case id: return launch<BM, BN, WM, WN, ST, BK, MF, RL, W>(a, s);
    DML_V2_TILES(DML_CASE)
#undef DML_CASE
    default: dml_set_error("dml_conv_v2: bad cfg"); return -1;
  }
}

// channel-tile width of a config (0: not a config); ids 100..119: the warp-specialised
// tiles of conv_igemm_ws.hip, 120..139 their persistent form (conv_igemm_wsp.hip)
extern "C" int dml_conv_v2_bn(int cfg) {
  if (cfg >= 150) return cfg <= 152 ? 64 : 0;  // row-ring 3x3 kernel (conv_rowring.hip)
  if (cfg >= 120) return dml_conv_wsp_bn(cfg);
  if (cfg >= 100) return dml_conv_ws_bn(cfg);
  if (cfg < 10) return 0;
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST, BK, MF, RL, W) \
  case id: return BN;
    DML_V2_TILES(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}

// Grouped launch of independent convs (cfg: the tile config every member uses).
extern "C" int dml_conv_v2_group(const DmlConvGroupArgs* g, int cfg, hipStream_t s) {
  using namespace dml::v2;
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST, BK) \
  case id: return launch_group<BM, BN, WM, WN, ST, BK>(g, s);
    DML_V2_GROUP_TILES(DML_CASE)
#undef DML_CASE
    default: dml_set_error("dml_conv_group: cfg has no grouped instantiation (the 4-wave tiles)"); return -1;
  }
}

extern "C" int dml_conv_v2_group_supported(int cfg) {
  switch (cfg) {
#define DML_CASE(id, BM, BN, WM, WN, ST, BK) \
  case id: return 1;
    DML_V2_GROUP_TILES(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}
