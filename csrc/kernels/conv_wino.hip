// conv_wino.hip — Winograd F(2x2, 3x3) convolution on MFMA for stride-1 3x3 convs (gfx950).
//
// y = A^T [ U ⊙ V ] A per 2x2 output tile, with U = G g G^T (the filter transform,
// done once on the host: ops.pack_wino_weight) and V = B^T d B (the input
// transform of the tile's 4x4 input window, done here in registers). The 16
// element-wise products over the input channels are 16 independent GEMMs
//   M[p][cout][tile] = sum_cin U[p][cout][cin] * V[p][cin][tile],  p = 0..15,
// run on v_mfma_f32_16x16x32_bf16: 2.25x fewer MACs than the direct (implicit
// GEMM) 3x3 conv. The reference has no kernel of its own (its convs run inside
// Keras, models.py:26,51); this serves SURVEY §2.7's 3x3 stride-1 rows.
//
// Workgroup = 8 waves = 4 tile groups x 2 position halves; 64 tiles x 64 output
// channels. Wave (g, h) owns the 16 tiles of group g and positions 8h..8h+7
// (rows 2h, 2h+1 of the 4x4 transform), for all 64 channels: 8 x 4 accumulator
// fragments = 128 registers, so two waves share a SIMD (the pair (g, 0) / (g, 1)
// lands on one SIMD and reads the same input rows).
//
//  * Input transform in registers, straight into the MFMA B operand: lane
//    (tile = lane & 15, channels 8q..8q+7 of the 32-channel chunk, q = lane >> 4)
//    loads the 3 input rows its half needs (16-B buffer loads; image border and
//    channel tail come back as zeros from the buffer range check), converts to
//    fp32, applies B^T . B with adds only, and rounds ONCE to bf16 — which is
//    exactly the fragment layout of v_mfma_f32_16x16x32_bf16's B operand.
//  * Transformed weights stream through a 2-stage LDS ring by LDS-DMA
//    (global_load_lds_dwordx4): a chunk is 16 positions x 4 fragments x 1 KiB,
//    host-packed in fragment order, so every ds_read_b128 is lane-linear
//    (conflict-free). The chunk k+1 DMA is in flight while chunk k computes.
//  * Epilogue: the two halves of a tile group swap half of their accumulators
//    through LDS (the ring's 128 KiB), then each lane applies A^T . A to its 16
//    positions (fp32), + bias, ReLU, and stores 4 consecutive channels of each of
//    the tile's 4 output pixels (8-B stores; the 4 lanes of a 16-channel run write
//    32 contiguous bytes).
#include "common.h"
#include "dml.h"

namespace dml {
namespace wino {

typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int KC = 32;                        // input channels per chunk (one MFMA k-step)
constexpr int NW = 8;                         // waves
constexpr int NT = NW * 64;                   // threads
constexpr int TILES = 64;                     // 2x2 output tiles per workgroup (4 groups of 16)
constexpr unsigned OOB = 0x80000000u;         // buffer offset past num_records: the load returns zeros
#ifndef DML_WINO_PROBE
#define DML_WINO_PROBE 0  // A/B timing probes only (tools/build_variant.py): 1 = no transform, 2 = no MFMA
#endif

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ float lo_f(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// B^T d B for the two transform rows of half H, one channel. x[r][c]: the 3 input
// rows the half loads (H = 0: rows 0..2, H = 1: rows 1..3), 4 columns.
// Returns v[i][j] for transform rows 2H + i (i = 0, 1).
template <int H>
__device__ __forceinline__ void btdb(const float (&x)[3][4], float (&v)[2][4]) {
  float t[2][4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (H == 0) {
      t[0][c] = x[0][c] - x[2][c];  // row 0: d0 - d2
      t[1][c] = x[1][c] + x[2][c];  // row 1: d1 + d2
    } else {
      t[0][c] = x[1][c] - x[0][c];  // row 2: d2 - d1
      t[1][c] = x[0][c] - x[2][c];  // row 3: d1 - d3
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    v[i][0] = t[i][0] - t[i][2];
    v[i][1] = t[i][1] + t[i][2];
    v[i][2] = t[i][2] - t[i][1];
    v[i][3] = t[i][1] - t[i][3];
  }
}

// 8 channels (4 dwords) of 12 input pixels -> the B fragments of this half's 8 positions
template <int H>
__device__ __forceinline__ void transform(const u32x4 (&raw)[3][4], u32x4 (&vb)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float xl[3][4], xh[3][4], vl[2][4], vh[2][4];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        xl[r][c] = lo_f(raw[r][c][e]);
        xh[r][c] = hi_f(raw[r][c][e]);
      }
    btdb<H>(xl, vl);
    btdb<H>(xh, vh);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) vb[i * 4 + j][e] = pack2(vl[i][j], vh[i][j]);
  }
}

// Workgroup geometry of one configuration: NF 16-channel fragments (TN = 16 NF output
// channels), a STAGES-deep weight ring, input rows prefetched PREF chunks ahead.
template <int NF, int STAGES, int PREF>
struct WCfg {
  static constexpr int TN = 16 * NF;
  static constexpr int CHUNK = 16 * NF * 1024;   // one chunk of U: 16 positions x NF fragments x 1 KiB
  static constexpr int WI = 16 * NF / NW;        // weight DMA pieces per wave per chunk
  static constexpr int LDS = STAGES * CHUNK;
  static constexpr int FH = NF / 2;              // fragments each position half finalises
  // vm ops younger than chunk kc's input rows when chunk kc starts: the weight DMA and the
  // input rows issued by the chunk before (PREF 2) / the weight DMA of this chunk's predecessor
  static constexpr int VM_YOUNGER = PREF == 2 ? WI + 12 : 0;
  static_assert(NF % 2 == 0 && (16 * NF) % NW == 0, "fragments split over the two halves and the waves");
  static_assert(LDS <= 163840 && NW * 64 * 16 * 8 * FH <= LDS, "ring / epilogue exchange exceed the LDS");
  static_assert(PREF == 1 || STAGES >= 3, "prefetching inputs 2 chunks ahead wants the weights 2+ ahead");
};

template <int H, int NF, int STAGES, int PREF>
__device__ __forceinline__ void wino_body(const DmlConvArgs& a, char* smem, int ct, int tb, int nkc) {
  using T = WCfg<NF, STAGES, PREF>;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid & 3;
  const int col = lane & 15, q = lane >> 4;
  const int TH = (a.Ho + 1) >> 1, TW = (a.Wo + 1) >> 1;
  const int ntiles = a.N * TH * TW;
  const int tile = tb * TILES + grp * 16 + col;
  const bool tile_ok = tile < ntiles;
  int n = 0, ty = 0, tx = 0;
  if (tile_ok) {
    n = tile / (TH * TW);
    const int r = tile - n * TH * TW;
    ty = r / TW;
    tx = r - ty * TW;
  }
  // byte offsets of this lane's 3 x 4 input pixels (channel 8q of chunk 0); OOB -> zeros
  unsigned off[3][4];
  const int ih0 = 2 * ty - a.ph + H, iw0 = 2 * tx - a.pw;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int ih = ih0 + r, iw = iw0 + c;
      const bool ok = tile_ok && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      off[r][c] = ok ? (unsigned)((((n * a.H + ih) * a.W + iw) * a.ldx + q * 8) * 2) : OOB;
    }
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);

  // transformed weights: [kc][pos][nft][lane][8] (nft = all of the layer's 16-channel
  // fragments, padded to a multiple of 4): this workgroup's fragments ct*NF .. ct*NF+NF-1.
  // Piece j of a chunk (position j / NF, fragment j % NF) lands at LDS offset j KiB.
  const int nft = (a.Cout + 63) / 64 * 4;
  const char* ubase = (const char*)a.wu + lane * 16;
  auto issue_w = [&](int kc, int stage) {
    char* dst = smem + stage * T::CHUNK;
#pragma unroll
    for (int j = 0; j < T::WI; ++j) {
      const int piece = wid * T::WI + j, pos = piece / NF, f = piece % NF;
      const char* src = ubase + (((long)kc * 16 + pos) * nft + ct * NF + f) * 1024;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + piece * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[8][NF];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[p][f] = (f32x4)(0.f);

  // this lane's 12 input pixels of chunk kc (image border / channel tail -> zeros)
  auto load_x = [&](u32x4 (&raw)[3][4], int kc) {
    // branch-free: an OOB offset stays >= OOB after the add, and the channel tail
    // (Cin % 32 != 0) ORs OOB in — no exec-mask split around the loads
    const unsigned cadd = (unsigned)(kc * KC * 2);
    const unsigned ctail = (kc * KC + q * 8 < a.Cin) ? 0u : OOB;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        raw[r][c] = __builtin_amdgcn_raw_buffer_load_b128(xrs, (off[r][c] + cadd) | ctail, 0, 0);
  };
  auto last = [&](int kc) { return kc < nkc ? kc : nkc - 1; };  // clamp: no branch around a load

  // one chunk: the weights landed (STAGES-1 chunks ago) and its input rows (PREF chunks ago)
  auto chunk = [&](int kc, u32x4 (&raw)[3][4]) {
    // A compiler-visible wait (it then knows raw[] is ready and inserts no wait of its own)
    // for everything but the VM_YOUNGER youngest vm ops; the barrier covers the other
    // waves' weight pieces and frees the stage the next DMA overwrites.
    constexpr int V = T::VM_YOUNGER;
    __builtin_amdgcn_s_waitcnt(((V >> 4) << 14) | 0x0f70 | (V & 15));
    __builtin_amdgcn_s_barrier();
    // (past the last chunk the ring re-loads the last chunk into a free stage)
    issue_w(last(kc + STAGES - 1), (kc + STAGES - 1) % STAGES);
    u32x4 vb[8];
#if DML_WINO_PROBE == 1  // timing probe: no input transform (wrong results)
#pragma unroll
    for (int p = 0; p < 8; ++p) vb[p] = raw[p >> 2][p & 3];
#else
    transform<H>(raw, vb);
#endif
    // the rows PREF chunks ahead load into the registers just consumed, under the MFMAs
    load_x(raw, last(kc + PREF));
    const char* su = smem + (kc % STAGES) * T::CHUNK + (H * 8 * NF) * 1024 + lane * 16;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const bf16x8 bv = __builtin_bit_cast(bf16x8, vb[p]);
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const bf16x8 au = *(const bf16x8*)(su + (p * NF + f) * 1024);
#if DML_WINO_PROBE == 2  // timing probe: no MFMA (wrong results)
        acc[p][f][0] += (float)au[0] * (float)bv[0];
#else
        acc[p][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(au, bv, acc[p][f], 0, 0, 0);
#endif
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue, in the issue order the steady-state waits count on:
  // W(0) .. W(S-3), X(0), W(S-2), X(1)   (PREF 2)   /   W(0) .. W(S-2), X(0)   (PREF 1)
  u32x4 rawA[3][4];
  if constexpr (PREF == 2) {
    u32x4 rawB[3][4];
    for (int s = 0; s < STAGES - 2; ++s) issue_w(last(s), s);
    load_x(rawA, 0);
    issue_w(last(STAGES - 2), STAGES - 2);
    load_x(rawB, last(1));
    int kc = 0;
    for (; kc + 1 < nkc; kc += 2) {  // unrolled by 2: the two register sets alternate
      chunk(kc, rawA);
      chunk(kc + 1, rawB);
    }
    if (kc < nkc) chunk(kc, rawA);
  } else {
    for (int s = 0; s < STAGES - 1; ++s) issue_w(last(s), s);
    load_x(rawA, 0);
    for (int kc = 0; kc < nkc; ++kc) chunk(kc, rawA);
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): every DMA retired
  __syncthreads();  // every wave is done with the ring: it becomes the exchange buffer

  // ---- epilogue: swap half the accumulators with the partner half ----
  // wave (g, H) finalises fragments H*FH .. H*FH+FH-1; it sends the partner its positions of
  // the partner's fragments
  constexpr int XB = 8 * T::FH * 64 * 16;  // exchange bytes per wave
  f32x4* mine = (f32x4*)(smem + wid * XB) + lane;
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int k = 0; k < T::FH; ++k) mine[(p * T::FH + k) * 64] = acc[p][(1 - H) * T::FH + k];
  __syncthreads();
  const f32x4* theirs = (const f32x4*)(smem + (grp + 4 * (1 - H)) * XB) + lane;

#pragma unroll
  for (int k = 0; k < T::FH; ++k) {
    const int f = H * T::FH + k;
    const int c0 = ct * T::TN + f * 16 + q * 4;  // 4 consecutive output channels of this lane
    // m[pos][e]: all 16 positions of this lane's 4 channels
    f32x4 m[16];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      m[8 * H + p] = acc[p][f];
      m[8 * (1 - H) + p] = theirs[(p * T::FH + k) * 64];
    }
    const float4 bias = *(const float4*)(a.bias + c0);
    float y[4][4];  // [pixel (a, b) = 2a + b][e]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float u0[4], u1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        u0[j] = m[j][e] + m[4 + j][e] + m[8 + j][e];
        u1[j] = m[4 + j][e] - m[8 + j][e] - m[12 + j][e];
      }
      const float bb = e == 0 ? bias.x : e == 1 ? bias.y : e == 2 ? bias.z : bias.w;
      y[0][e] = u0[0] + u0[1] + u0[2] + bb;
      y[1][e] = u0[1] - u0[2] - u0[3] + bb;
      y[2][e] = u1[0] + u1[1] + u1[2] + bb;
      y[3][e] = u1[1] - u1[2] - u1[3] + bb;
    }
    if (!tile_ok || c0 >= a.Cout) continue;
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const int oy = 2 * ty + (px >> 1), ox = 2 * tx + (px & 1);
      if (oy >= a.Ho || ox >= a.Wo) continue;
      float v0 = y[px][0], v1 = y[px][1], v2 = y[px][2], v3 = y[px][3];
      if (a.relu) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      }
      *(uint2*)((unsigned short*)a.y + ((long)(n * a.Ho + oy) * a.Wo + ox) * a.ldy + c0) =
          make_uint2(pack2(v0, v1), pack2(v2, v3));
    }
  }
}

template <int NF, int STAGES, int PREF>
__global__ __launch_bounds__(NT) void conv_wino_kernel(DmlConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TN = 16 * NF;
  const int nct = (a.Cout + TN - 1) / TN;
  const int nkc = (a.Cin + KC - 1) / KC;
  // output-channel tiles fastest: the blocks of one XCD share input tiles in its L2
  const int Lb = xcd_remap(blockIdx.x, gridDim.x);
  const int ct = Lb % nct, tb = Lb / nct;
  if ((threadIdx.x >> 8) == 0) wino_body<0, NF, STAGES, PREF>(a, smem, ct, tb, nkc);  // waves 0..3: positions 0..7
  else wino_body<1, NF, STAGES, PREF>(a, smem, ct, tb, nkc);                           // waves 4..7: positions 8..15
}

// ---------------------------------------------------------------------------
// Patch kernel (cfg 82): the input patch of the workgroup's 64 tiles is DMA'd into
// LDS once per chunk (consecutive tiles = consecutive input rows: one contiguous pixel
// range), transformed ONCE per workgroup into V (LDS), and the GEMM phase reads V
// fragments from LDS and the weights straight from L2 into registers (each wave owns
// two of the 16 positions for all 64 tiles x 64 channels, so no weight is read by two
// waves). Per chunk: [wait patch] barrier, DMA next patch, transform (VALU + LDS),
// barrier, [wait weights] 32 MFMAs per wave, load the next chunk's weights.
// The first version's per-lane global loads re-read every input pixel ~47x (4
// overlapping tile windows x 2 position halves x every output-channel tile).
constexpr int P_TN = 64;                  // output channels per workgroup
constexpr int P_VBYTES = 16 * 4 * 1024;   // V: 16 positions x 4 tile fragments x 1 KiB

template <int NPW>  // patch DMA pieces (16 pixels x 64 B) per wave per chunk
struct PCfg {
  static constexpr int PIECES = NPW * NW;
  static constexpr int PATCH = PIECES * 1024;          // bytes per patch stage
  static constexpr int MAXPX = PIECES * 16;            // pixels per patch
  static constexpr int ZERO = P_VBYTES + 2 * PATCH;    // 16 zero bytes: out-of-image taps read here
  static constexpr int LDS = ZERO + 16;
  static_assert(LDS <= 163840, "LDS");
};

// LDS slot of 16-B unit q (channels 8q..8q+7 of the chunk) of patch pixel p: the quarter is
// rotated by pixel pair so the 16 tiles of a read (pixels 2 apart) spread over the banks
__device__ __forceinline__ int patch_off(int p, int q) { return ((p << 2) + (q ^ ((p >> 1) & 3))) << 4; }

template <int H, int NPW>
__device__ __forceinline__ void patch_body(const DmlConvArgs& a, char* smem, int ct, int tb, int nkc) {
  using T = PCfg<NPW>;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid & 3;
  const int col = lane & 15, q = lane >> 4;
  const int TH = (a.Ho + 1) >> 1, TW = (a.Wo + 1) >> 1, THW = TH * TW;
  const int ntiles = a.N * THW;
  // the workgroup's pixel range: input rows R0 .. R1-1 of the flattened (n, row) space
  const int t_first = tb * TILES, t_last = min(t_first + TILES, ntiles) - 1;
  const int n0 = t_first / THW, ty0 = (t_first - n0 * THW) / TW;
  const int n1 = t_last / THW, ty1 = (t_last - n1 * THW) / TW;
  const int R0 = n0 * a.H + max(0, 2 * ty0 - a.ph);
  const int R1 = n1 * a.H + min(a.H, 2 * ty1 + 4 - a.ph);
  const int P = (R1 - R0) * a.W;   // <= T::MAXPX (checked by the host)
  const int pix0 = R0 * a.W;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7ffffff0, 0x00020000);

  // ---- this lane's transform work: tile (group grp, column col), channels 8q.., half H ----
  const int tile = t_first + grp * 16 + col;
  const bool tile_ok = tile < ntiles;
  int n = 0, ty = 0, tx = 0;
  if (tile_ok) {
    n = tile / THW;
    const int r = tile - n * THW;
    ty = r / TW;
    tx = r - ty * TW;
  }
  int lds_px[3][4];  // LDS offsets (within a patch stage) of the 12 pixels, or the zero slot
  {
    const int ih0 = 2 * ty - a.ph + H, iw0 = 2 * tx - a.pw;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int ih = ih0 + r, iw = iw0 + c;
        const bool ok = tile_ok && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const int p = (n * a.H + ih) * a.W + iw - pix0;
        lds_px[r][c] = ok ? patch_off(p, q) : -1;
      }
  }
  // ---- patch DMA: piece j = wid*NPW + i, lane L -> unit j*64 + L (pixel u/4, slot u%4) ----
  unsigned dma_off[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const int u = (wid * NPW + i) * 64 + lane;
    const int p = u >> 2, q4 = (u & 3) ^ ((p >> 1) & 3);
    dma_off[i] = p < P ? (unsigned)((((long)(pix0 + p)) * a.ldx + q4 * 8) * 2) : OOB;
  }
  auto issue_patch = [&](int kc, int stage) {
    char* dst = smem + P_VBYTES + stage * T::PATCH + wid * NPW * 1024;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int u = (wid * NPW + i) * 64 + lane;
      const int q4 = (u & 3) ^ (((u >> 2) >> 1) & 3);
      const unsigned tail = (kc * KC + q4 * 8 < a.Cin) ? 0u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void*)(dst + i * 1024), 16,
                                              (dma_off[i] + (unsigned)(kc * KC * 2)) | tail, 0, 0, 0);
    }
  };

  // ---- GEMM work: positions 2*wid, 2*wid+1; all 4 tile fragments x 4 channel fragments ----
  const int nft = (a.Cout + 63) / 64 * 4;
  const char* ug = (const char*)a.wu + lane * 16;
  bf16x8 wreg[2][4];
  auto load_w = [&](int kc) {
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int f = 0; f < 4; ++f)
        wreg[pp][f] = *(const bf16x8*)(ug + (((long)kc * 16 + 2 * wid + pp) * nft + ct * 4 + f) * 1024);
  };
  f32x4 acc[2][4][4];  // [position][tile fragment][channel fragment]
#pragma unroll
  for (int pp = 0; pp < 2; ++pp)
#pragma unroll
    for (int tf = 0; tf < 4; ++tf)
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[pp][tf][f] = (f32x4)(0.f);

  if (tid == 0) *(uint4*)(smem + T::ZERO) = make_uint4(0, 0, 0, 0);
  // prologue: patch(0), then W(0) (issue order the waits below count on)
  issue_patch(0, 0);
  load_w(0);
  for (int kc = 0; kc < nkc; ++kc) {
    // patch(kc) landed (the 8 weight loads of W(kc) are younger), every wave is past the
    // previous chunk's GEMM (V and the other patch stage are free)
    __builtin_amdgcn_s_waitcnt(0x0070 | 8);  // vmcnt(8) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    issue_patch(kc + 1 < nkc ? kc + 1 : kc, (kc + 1) & 1);
    // ---- transform: 12 pixels from the patch -> this half's 8 positions of V ----
    {
      const char* ps = smem + P_VBYTES + (kc & 1) * T::PATCH;
      u32x4 raw[3][4];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          raw[r][c] = *(const u32x4*)(lds_px[r][c] >= 0 ? ps + lds_px[r][c] : smem + T::ZERO);
      u32x4 vb[8];
      transform<H>(raw, vb);
#pragma unroll
      for (int p = 0; p < 8; ++p) *(u32x4*)(smem + (((8 * H + p) * 4 + grp) * 64 + lane) * 16) = vb[p];
    }
    // W(kc) landed (the patch(kc+1) DMA is younger) and this wave's V writes are done; the raw
    // barrier then makes V complete (a __syncthreads() fence would also drain the DMA)
    static_assert(NPW < 16, "vmcnt field");
    __builtin_amdgcn_s_waitcnt(0x0070 | NPW);  // vmcnt(NPW) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int tf = 0; tf < 4; ++tf) {
        const bf16x8 bv = *(const bf16x8*)(smem + (((2 * wid + pp) * 4 + tf) * 64 + lane) * 16);
#pragma unroll
        for (int f = 0; f < 4; ++f)
          acc[pp][tf][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[pp][f], bv, acc[pp][tf][f], 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
    load_w(kc + 1 < nkc ? kc + 1 : kc);  // under the next chunk's DMA wait + transform
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  // ---- epilogue: per channel fragment, the 16 positions meet in LDS ----
  const int etf = tid >> 6;  // threads 0..255: tile fragment etf, lane = tile col + 16 x channel quad
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    __syncthreads();
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int tf = 0; tf < 4; ++tf)
        *(f32x4*)(smem + (((2 * wid + pp) * 4 + tf) * 64 + lane) * 16) = acc[pp][tf][f];
    __syncthreads();
    if (tid < 256) {
      f32x4 m[16];
#pragma unroll
      for (int p = 0; p < 16; ++p) m[p] = *(const f32x4*)(smem + ((p * 4 + etf) * 64 + lane) * 16);
      const int et = t_first + etf * 16 + col;
      const int c0 = ct * P_TN + f * 16 + q * 4;
      if (et < ntiles && c0 < a.Cout) {
        const int en = et / THW, er = et - en * THW, ety = er / TW, etx = er - ety * TW;
        const float4 bias = *(const float4*)(a.bias + c0);
        float y[4][4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float u0[4], u1[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            u0[j] = m[j][e] + m[4 + j][e] + m[8 + j][e];
            u1[j] = m[4 + j][e] - m[8 + j][e] - m[12 + j][e];
          }
          const float bb = e == 0 ? bias.x : e == 1 ? bias.y : e == 2 ? bias.z : bias.w;
          y[0][e] = u0[0] + u0[1] + u0[2] + bb;
          y[1][e] = u0[1] - u0[2] - u0[3] + bb;
          y[2][e] = u1[0] + u1[1] + u1[2] + bb;
          y[3][e] = u1[1] - u1[2] - u1[3] + bb;
        }
#pragma unroll
        for (int px = 0; px < 4; ++px) {
          const int oy = 2 * ety + (px >> 1), ox = 2 * etx + (px & 1);
          if (oy >= a.Ho || ox >= a.Wo) continue;
          float v0 = y[px][0], v1 = y[px][1], v2 = y[px][2], v3 = y[px][3];
          if (a.relu) {
            v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
          }
          *(uint2*)((unsigned short*)a.y + ((long)(en * a.Ho + oy) * a.Wo + ox) * a.ldy + c0) =
              make_uint2(pack2(v0, v1), pack2(v2, v3));
        }
      }
    }
  }
}

template <int NPW>
__global__ __launch_bounds__(NT) void conv_wino_patch_kernel(DmlConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nct = (a.Cout + P_TN - 1) / P_TN;
  const int nkc = (a.Cin + KC - 1) / KC;
  const int Lb = xcd_remap(blockIdx.x, gridDim.x);
  const int ct = Lb % nct, tb = Lb / nct;
  if ((threadIdx.x >> 8) == 0) patch_body<0, NPW>(a, smem, ct, tb, nkc);
  else patch_body<1, NPW>(a, smem, ct, tb, nkc);
}

// largest input patch (pixels) of any workgroup of conv a (host)
static inline long patch_pixels_max(const DmlConvArgs& a) {
  const long TH = (a.Ho + 1) / 2, TW = (a.Wo + 1) / 2, THW = TH * TW, nt = (long)a.N * THW;
  long best = 0;
  for (long t0 = 0; t0 < nt; t0 += TILES) {
    const long t1 = (t0 + TILES < nt ? t0 + TILES : nt) - 1;
    const long n0 = t0 / THW, ty0 = (t0 - n0 * THW) / TW, n1 = t1 / THW, ty1 = (t1 - n1 * THW) / TW;
    const long r0 = n0 * a.H + (2 * ty0 - a.ph > 0 ? 2 * ty0 - a.ph : 0);
    const long r1 = n1 * a.H + (2 * ty1 + 4 - a.ph < a.H ? 2 * ty1 + 4 - a.ph : a.H);
    const long p = (r1 - r0) * a.W;
    if (p > best) best = p;
  }
  return best;
}

// configurations: cfg id, NF, STAGES, PREF
#define DML_WINO_CFGS(X) \
  X(80, 2, 4, 2)   /* 32 channels, 4-stage ring, inputs 2 chunks ahead (the default) */ \
  X(81, 4, 2, 1)   /* 64 channels, 2-stage ring (r4 first version: latency-bound) */
// patch kernels: cfg id, pieces per wave (patch capacity = 128 x NPW pixels)
#define DML_WINO_PATCH_CFGS(X) X(82, 3) X(83, 5)

}  // namespace wino
}  // namespace dml

// host side ------------------------------------------------------------------

extern "C" const char* dml_conv_wino_check(const DmlConvArgs* a) {
  if (!a->wu) return "dml_conv_wino: no Winograd-transformed weights (DmlConvArgs.wu)";
  if (a->kh != 3 || a->kw != 3 || a->sh != 1 || a->sw != 1 || (a->dh > 1) || (a->dw > 1))
    return "dml_conv_wino: 3x3 stride-1 undilated convs only";
  if (a->ph < 0 || a->ph > 1 || a->pw < 0 || a->pw > 1 || a->Ho != a->H + 2 * a->ph - 2 ||
      a->Wo != a->W + 2 * a->pw - 2)
    return "dml_conv_wino: padding must be 'same' (1) or 'valid' (0)";
  if (a->res || a->nseg || a->out_f32 || a->ksplit > 1 || a->rsub > 1)
    return "dml_conv_wino: no residual, segments, fp32 output or split-K";
  if (a->Cin % 8 || a->ldx % 8 || a->Cout % 8 || a->ldy % 4)
    return "dml_conv_wino: need Cin, ldx, Cout %8 == 0 and ldy %4 == 0";
  const long last = ((long)a->N * a->H * a->W) * a->ldx * 2;
  if (last >= 0x7ffffff0L) return "dml_conv_wino: input larger than the 2 GiB buffer range";
  return nullptr;
}

extern "C" int dml_conv_wino_init(void) {
  using namespace dml::wino;
  int rc = 0;
#define DML_SET(id, NF, ST, PF)                                                                      \
  rc |= (int)hipFuncSetAttribute((const void*)conv_wino_kernel<NF, ST, PF>,                        \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, WCfg<NF, ST, PF>::LDS);
  DML_WINO_CFGS(DML_SET)
#undef DML_SET
#define DML_SET(id, NPW)                                                                           \
  rc |= (int)hipFuncSetAttribute((const void*)conv_wino_patch_kernel<NPW>,                         \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, PCfg<NPW>::LDS);
  DML_WINO_PATCH_CFGS(DML_SET)
#undef DML_SET
  return rc;
}

template <int NF, int STAGES, int PREF>
static int launch_wino(const DmlConvArgs* a, hipStream_t s) {
  using namespace dml::wino;
  using T = WCfg<NF, STAGES, PREF>;
  const long ntiles = (long)a->N * ((a->Ho + 1) / 2) * ((a->Wo + 1) / 2);
  const long blocks = (ntiles + TILES - 1) / TILES * ((a->Cout + T::TN - 1) / T::TN);
  hipLaunchKernelGGL((conv_wino_kernel<NF, STAGES, PREF>), dim3((unsigned)blocks), dim3(NT), T::LDS, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}

template <int NPW>
static int launch_wino_patch(const DmlConvArgs* a, hipStream_t s) {
  using namespace dml::wino;
  if (patch_pixels_max(*a) > PCfg<NPW>::MAXPX) {
    dml_set_error("dml_conv_wino: a workgroup's input patch exceeds this config's LDS patch");
    return -1;
  }
  const long ntiles = (long)a->N * ((a->Ho + 1) / 2) * ((a->Wo + 1) / 2);
  const long blocks = (ntiles + TILES - 1) / TILES * ((a->Cout + P_TN - 1) / P_TN);
  hipLaunchKernelGGL((conv_wino_patch_kernel<NPW>), dim3((unsigned)blocks), dim3(NT), PCfg<NPW>::LDS, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}

extern "C" int dml_conv_wino_supported(int cfg) {
  switch (cfg) {
#define DML_CASE(id, NF, ST, PF) case id: return 16 * NF;
    DML_WINO_CFGS(DML_CASE)
#undef DML_CASE
#define DML_CASE(id, NPW) case id: return 64;
    DML_WINO_PATCH_CFGS(DML_CASE)
#undef DML_CASE
    default: return 0;
  }
}

extern "C" int dml_conv_wino(const DmlConvArgs* a, int cfg, hipStream_t s) {
  const char* why = dml_conv_wino_check(a);
  if (why) {
    dml_set_error(why);
    return -1;
  }
  switch (cfg) {
#define DML_CASE(id, NF, ST, PF) case id: return launch_wino<NF, ST, PF>(a, s);
    DML_WINO_CFGS(DML_CASE)
#undef DML_CASE
#define DML_CASE(id, NPW) case id: return launch_wino_patch<NPW>(a, s);
    DML_WINO_PATCH_CFGS(DML_CASE)
#undef DML_CASE
    default: dml_set_error("dml_conv_wino: not a Winograd cfg"); return -1;
  }
}
