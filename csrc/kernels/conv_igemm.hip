// conv_igemm.hip — MFMA implicit-GEMM convolution for gfx950 (MI355X).
//
// Serves every convolution of ResNet50 / InceptionV3 and the FC layer
// (SURVEY §2.7 "conv_igemm_bf16"; the reference runs these inside Keras,
// models.py:26,51 — it has no kernel of its own).
//
// GEMM view, computed TRANSPOSED:  D[c][m] = sum_k W[c][k] * X[k][m]
//   c = output channel (MFMA "A" rows),  m = output pixel (MFMA "B" columns).
// Why transposed: with v_mfma_f32_16x16x32_bf16 the accumulator of lane l holds
// column (l & 15) and 4 consecutive rows 4*(l>>4)+r. Putting channels on the rows
// gives every lane 4 CONSECUTIVE output channels of one pixel — an 8-byte NHWC
// store (and an 8-byte residual load, a 16-byte bias load) per fragment instead
// of four scattered 2-byte stores.
//
// Tiling: BM pixels x BN channels x BK reduction per 256-thread workgroup
// (4 waves of 64 lanes). Operand tiles are staged global->VGPR->LDS with a
// one-tile register prefetch (issue next tile's loads before this tile's MFMAs,
// write them to the other LDS buffer after), one barrier per K-tile.
// LDS rows are XOR-swizzled per 16-byte chunk so the ds_read_b128 fragment reads
// are bank-conflict free (swizzle found by exhaustive search over the gfx950
// ds_read_b128 lane groups, see tools/lds_swizzle_search.py).
//
// Implicit im2col: each thread owns fixed tile rows (pixels) for the whole
// K loop; their (n, oh*sh-ph, ow*sw-pw) are computed once, and the (r, s, c)
// position of the thread's 8-channel chunk advances with a running counter —
// no division in the K loop. Requires Cin % 8 == 0 (the stem input is padded
// to 8 channels by the preprocess kernel) and 16-byte aligned channel offsets.
#include "common.h"
#include "dml.h"

namespace dml {

template <int BM, int BN, int BK>
struct ConvTile {
  static constexpr int WAVES_C = (BN >= 128) ? 2 : 1;
  static constexpr int WAVES_P = 4 / WAVES_C;
  static constexpr int WTC = BN / WAVES_C;  // channels per wave
  static constexpr int WTP = BM / WAVES_P;  // pixels per wave
  static constexpr int FI = WTC / 16;       // 16x16 fragments along channels
  static constexpr int FJ = WTP / 16;       // along pixels
  static constexpr int CPR = BK / 8;        // 16-byte chunks per LDS row
  static constexpr int XCH = BM * CPR / 256;  // X chunks per thread per K-tile
  static constexpr int WCH = BN * CPR / 256;  // W chunks per thread per K-tile
  static constexpr int ROWSTEP = 256 / CPR;
  static_assert(XCH >= 1 && WCH >= 1, "tile too small for 256 threads");
  static constexpr int LDS_X = BM * BK * 2;  // bytes per buffer
  static constexpr int LDS_W = BN * BK * 2;
};

template <int BK>
__device__ __forceinline__ int swz(int row, int chunk) {
  if constexpr (BK == 64) return chunk ^ (row & 7);
  else return chunk ^ ((row >> 1) & 3);  // BK == 32
}

template <int BK>
__device__ __forceinline__ int lds_off(int row, int chunk) {
  return row * (BK * 2) + swz<BK>(row, chunk) * 16;
}

template <int BM, int BN, int BK>
__global__ __launch_bounds__(256) void conv_igemm_kernel(DmlConvArgs a) {
  using T = ConvTile<BM, BN, BK>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* xs = smem;                      // [2][BM][BK]
  char* ws = smem + 2 * T::LDS_X;       // [2][BN][BK]

  const int M = a.N * a.Ho * a.Wo;
  const int ntiles_c = (a.Cout + BN - 1) / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tc = L % ntiles_c;
  const int tm = L / ntiles_c;
  const int m0 = tm * BM, c0 = tc * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wc = wid % T::WAVES_C;
  const int wp = wid / T::WAVES_C;

  // ---- per-thread im2col bookkeeping (fixed rows, one chunk column) ----
  const int kq = tid % T::CPR;
  const int rbase = tid / T::CPR;
  int pix0[T::XCH], ih0[T::XCH], iw0[T::XCH];
  const int HoWo = a.Ho * a.Wo;
#pragma unroll
  for (int i = 0; i < T::XCH; ++i) {
    const int m = m0 + rbase + i * T::ROWSTEP;
    if (m < M) {
      const int n = m / HoWo;
      const int rem = m - n * HoWo;
      const int oh = rem / a.Wo;
      const int ow = rem - oh * a.Wo;
      pix0[i] = n * a.H * a.W;
      ih0[i] = oh * a.sh - a.ph;
      iw0[i] = ow * a.sw - a.pw;
    } else {
      pix0[i] = 0;
      ih0[i] = -(1 << 28);  // forces the bounds test to fail: zero row
      iw0[i] = 0;
    }
  }
  // running (r, s, c) of this thread's chunk
  int cc = kq * 8, ss = 0, rr = 0;
  while (cc >= a.Cin) { cc -= a.Cin; if (++ss == a.kw) { ss = 0; ++rr; } }

  const bf16* __restrict__ xg = (const bf16*)a.x;
  const bf16* __restrict__ wg = (const bf16*)a.w;
  const int nk = a.Kpad / BK;
  const int dh = a.dh > 0 ? a.dh : 1, dw = a.dw > 0 ? a.dw : 1;

  uint4 xr[T::XCH], wr[T::WCH];

  auto load_tile = [&](int kt) {
    const bool kval = rr < a.kh;
#pragma unroll
    for (int i = 0; i < T::XCH; ++i) {
      const int ih = ih0[i] + rr * dh, iw = iw0[i] + ss * dw;
      const bool ok = kval && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      if (ok) {
        const long off = (long)(pix0[i] + ih * a.W + iw) * a.ldx + cc;
        xr[i] = *(const uint4*)(xg + off);
      } else {
        xr[i] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < T::WCH; ++i) {
      const int row = rbase + i * T::ROWSTEP;
      wr[i] = *(const uint4*)(wg + (long)(c0 + row) * a.Kpad + kt * BK + kq * 8);
    }
    // advance the chunk position by BK reduction elements
    cc += BK;
    while (cc >= a.Cin) { cc -= a.Cin; if (++ss == a.kw) { ss = 0; ++rr; } }
  };
  auto store_tile = [&](int buf) {
    char* xb = xs + buf * T::LDS_X;
    char* wb = ws + buf * T::LDS_W;
#pragma unroll
    for (int i = 0; i < T::XCH; ++i) {
      const int row = rbase + i * T::ROWSTEP;
      *(uint4*)(xb + lds_off<BK>(row, kq)) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < T::WCH; ++i) {
      const int row = rbase + i * T::ROWSTEP;
      *(uint4*)(wb + lds_off<BK>(row, kq)) = wr[i];
    }
  };

  f32x4 acc[T::FI][T::FJ];
#pragma unroll
  for (int i = 0; i < T::FI; ++i)
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int frow = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = (kt + 1) < nk;
    if (more) load_tile(kt + 1);
    const char* xb = xs + cur * T::LDS_X;
    const char* wb = ws + cur * T::LDS_W;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 fa[T::FI], fb[T::FJ];
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < T::FI; ++i)
        fa[i] = *(const bf16x8*)(wb + lds_off<BK>(wc * T::WTC + i * 16 + frow, ch));
#pragma unroll
      for (int j = 0; j < T::FJ; ++j)
        fb[j] = *(const bf16x8*)(xb + lds_off<BK>(wp * T::WTP + j * 16 + frow, ch));
#pragma unroll
      for (int i = 0; i < T::FI; ++i)
#pragma unroll
        for (int j = 0; j < T::FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- fused epilogue: bias (+ residual) (+ ReLU), NHWC store at channel offset ----
  const unsigned short* __restrict__ rg = (const unsigned short*)a.res;
#pragma unroll
  for (int i = 0; i < T::FI; ++i) {
    const int ch = c0 + wc * T::WTC + i * 16 + fq * 4;
    if (ch >= a.Cout) continue;
    const float4 b4 = *(const float4*)(a.bias + ch);
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) {
      const int m = m0 + wp * T::WTP + j * 16 + frow;
      if (m >= M) continue;
      float v0 = acc[i][j][0] + b4.x, v1 = acc[i][j][1] + b4.y;
      float v2 = acc[i][j][2] + b4.z, v3 = acc[i][j][3] + b4.w;
      if (rg) {
        const uint2 r = *(const uint2*)(rg + (long)m * a.ldr + ch);
        v0 += bf2f(r.x & 0xffff); v1 += bf2f(r.x >> 16);
        v2 += bf2f(r.y & 0xffff); v3 += bf2f(r.y >> 16);
      }
      if (a.relu) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      }
      if (a.out_f32) {
        *(float4*)((float*)a.y + (long)m * a.ldy + ch) = make_float4(v0, v1, v2, v3);
      } else {
        *(uint2*)((unsigned short*)a.y + (long)m * a.ldy + ch) = make_uint2(pack2(v0, v1), pack2(v2, v3));
      }
    }
  }
}

template <int BM, int BN, int BK>
static int launch_conv(const DmlConvArgs* a, hipStream_t s) {
  using T = ConvTile<BM, BN, BK>;
  const long M = (long)a->N * a->Ho * a->Wo;
  const long tiles = ((M + BM - 1) / BM) * ((a->Cout + BN - 1) / BN);
  const int lds = 2 * (T::LDS_X + T::LDS_W);
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK>), dim3((unsigned)tiles), dim3(256), lds, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}

}  // namespace dml

// Tile configurations (cfg ids are part of the ABI used by the plan builder).
//   0: 128 px x 128 ch x BK64   (large M, Cout >= 128)
//   1: 256 px x  64 ch x BK64   (large M, Cout = 64-ish)
//   2:  64 px x 128 ch x BK64   (small M, wide Cout)
//   3: 128 px x 128 ch x BK32   (short K)
//   4:  64 px x  64 ch x BK64   (tiny layers)
extern "C" int dml_conv_v2(const DmlConvArgs* a, int cfg, hipStream_t s);

extern "C" int dml_conv(const DmlConvArgs* a, int cfg, hipStream_t s) {
  if (cfg >= 10) {
    if (a->Cin % 8 || a->ldx % 8 || a->Cout % 8 || a->Kpad % 64 || a->ldy % 8 || (a->res && a->ldr % 8)) {
      dml_set_error("dml_conv(v2): need Cin, ldx, Cout, ldy, ldr %8==0 and Kpad%64==0");
      return -1;
    }
    if (a->nseg < 0 || a->nseg > 4) {
      dml_set_error("dml_conv(v2): nseg must be 0..4");
      return -1;
    }
    if (a->rsub > 1 && (!a->res || a->rW < a->Wo * a->rsub || a->rHW < a->rW * a->Ho * a->rsub)) {
      dml_set_error("dml_conv(v2): subsampled residual needs res and rW >= Wo*rsub, rHW >= rW*Ho*rsub");
      return -1;
    }
    if (a->ksplit > 1 && (cfg >= 40 || !a->out_f32 || a->res || a->nseg || a->relu || a->split_ld < 1)) {
      dml_set_error("dml_conv(v2): split-K needs a v2 config, fp32 output, no residual/segments/ReLU, split_ld");
      return -1;
    }
    if (a->kchunk && (cfg >= 40 || a->kchunk < 0 || a->kchunk % 64 || a->Cin % a->kchunk || a->dh > 1 ||
                      a->dw > 1)) {
      dml_set_error("dml_conv(v2): chunk-major K order needs a v2 config, kchunk%64==0, Cin%kchunk==0, no dilation");
      return -1;
    }
    return cfg >= 40 ? dml_conv_halo(a, cfg, s) : dml_conv_v2(a, cfg, s);
  }
  if (a->nseg > 0 || a->ksplit > 1 || a->rsub > 1 || a->kchunk) {
    dml_set_error("dml_conv: output segments / split-K / subsampled residual / chunk-major K need a v2 config (cfg >= 10)");
    return -1;
  }
  if (a->Cin % 8 || a->ldx % 8 || a->Cout % 4 || a->Kpad % 64) {
    dml_set_error("dml_conv: need Cin%8==0, ldx%8==0, Cout%4==0, Kpad%64==0");
    return -1;
  }
  switch (cfg) {
    case 0: return dml::launch_conv<128, 128, 64>(a, s);
    case 1: return dml::launch_conv<256, 64, 64>(a, s);
    case 2: return dml::launch_conv<64, 128, 64>(a, s);
    case 3: return dml::launch_conv<128, 128, 32>(a, s);
    case 4: return dml::launch_conv<64, 64, 64>(a, s);
    default: dml_set_error("dml_conv: bad cfg"); return -1;
  }
}

// Heuristic tile choice: keep >= ~2 waves of workgroups on the 256 CUs and
// avoid padding waste along Cout. (Measured refinements live in the Python
// autotuner, distributed_machine_learning_amd/ops/tuning.py.)
extern "C" int dml_conv_pick_cfg(const DmlConvArgs* a) {
  const long M = (long)a->N * a->Ho * a->Wo;
  const int C = a->Cout;
  const bool v2ok = !(a->Cin % 8 || a->ldx % 8 || C % 8 || a->ldy % 8 || (a->res && a->ldr % 8));
  if (v2ok) {  // measured defaults (tools/conv_bench.py); the engine autotunes per shape
    if (C <= 64) return 15;
    if (a->Kpad <= 512 || M < 16384) return 14;
    return 11;
  }
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((C + bn - 1) / bn); };
  if (C <= 64) return tiles(256, 64) >= 512 ? 1 : 4;
  if (tiles(128, 128) >= 512) return 0;
  if (tiles(64, 128) >= 256) return 2;
  return 4;
}
