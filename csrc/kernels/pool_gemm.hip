// pool_gemm.hip — max pool 3x3/2 (valid) + the 1x1 GEMM that is its only reader, ONE kernel
// (gfx950). InceptionV3: max_pooling2d_2 (71x71x192 -> 35x35x192) feeds only mixed0's four
// sibling 1x1 convs, which the graph rewrite already runs as one segmented GEMM
// (conv2d_6 | conv2d_7 | conv2d_9 | conv2d_12: 192 -> 64 + 48 + 64 + 32; reference models.py:26-44,
// Keras InceptionV3 mixed0). Unfused, the pooled tensor is written and read back and the chip
// drains once between the two launches. Here a workgroup owns 64 consecutive pooled pixels:
//
//  1. pool: item = (pixel, 8-channel group), the 3x3 window's nine 16-B rows loaded first, two
//     items per thread in flight, max -> bf16 into an LDS tile [64 px][C] (400-B rows for C =
//     192: 16 consecutive rows start on 16 distinct 4-bank groups, so the fragment reads below
//     are conflict-free);
//  2. GEMM: output-channel fragment f (16 channels) belongs to wave f % 4; each wave runs its
//     fragments x the 4 pixel fragments over K = C with v_mfma_f32_16x16x32_bf16, weights as A
//     fragments loaded from L2 into VGPRs before the pool phase (their latency hides under it;
//     every weight is read once per workgroup);
//  3. epilogue: bias (accumulator start) + per-segment ReLU -> 4 channels (8 B) per lane into the
//     segment's own destination (a concat slice or a branch buffer), as the v2 conv's segmented
//     epilogue does.
//
// The pooled values are rounded to bf16 before the GEMM, as the unfused pool writes them.
#include <string>

#include "common.h"
#include "dml.h"

namespace dml {
namespace pgemm {

constexpr int NT = 256, BMP = 64;  // threads, pooled pixels per workgroup
constexpr int FMAX = 4;            // output-channel fragments per wave (Cout <= 256)

__device__ __forceinline__ void max8(float* m, const uint4& v) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    m[2 * q] = fmaxf(m[2 * q], bf2f((unsigned short)(w[q] & 0xffff)));
    m[2 * q + 1] = fmaxf(m[2 * q + 1], bf2f((unsigned short)(w[q] >> 16)));
  }
}

template <int C>
__global__ __launch_bounds__(NT, 2) void pool_gemm_kernel(DmlPoolGemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const DmlPoolArgs& p = a.p;
  const DmlConvArgs& g = a.g;
  constexpr int CG = C / 8, KS = C / 32;
  constexpr int ROW = C * 2 + 16;  // LDS row bytes (pad: C * 2 = 384 -> 400 B)
  const int HWo = p.Ho * p.Wo, M = p.N * HWo;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BMP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const unsigned short* x = (const unsigned short*)p.x;
  const int NF = (g.Cout + 15) / 16;

  // this wave's weight fragments (all K) are loaded first: their L2 latency hides under the pool
  const bf16* w = (const bf16*)g.w;
  bf16x8 wa[FMAX][KS];
#pragma unroll
  for (int t = 0; t < FMAX; ++t) {
    const int f = min(wid + 4 * t, NF - 1);  // clamped (a wave past NF loads a valid row, never uses it)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wa[t][ks] = *(const bf16x8*)(w + (long)(16 * f + frow) * g.Kpad + 32 * ks + 8 * fq);
  }

  // 1. pool into LDS (rows of pixels past M are left as they are: never stored)
  const int items = BMP * CG;
  for (int t0 = tid; t0 < items; t0 += 2 * NT) {
    uint4 v[2][9];
    int px[2], cg[2];
    bool ok[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = t0 + u * NT;
      px[u] = t / CG;
      cg[u] = t - px[u] * CG;
      const int m = m0 + px[u];
      ok[u] = t < items && m < M;
      const int mm = ok[u] ? m : 0;  // clamped: every load is issued (no branch around a load)
      const int n = mm / HWo, rem = mm - n * HWo;
      const int i = rem / p.Wo, j = rem - i * p.Wo;
      const unsigned short* base = x + ((long)(n * p.H + 2 * i) * p.W + 2 * j) * p.ldx + (ok[u] ? cg[u] : 0) * 8;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) v[u][dy * 3 + dx] = *(const uint4*)(base + ((long)dy * p.W + dx) * p.ldx);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!ok[u]) continue;
      float m[8];
      {
        const unsigned w[4] = {v[u][0].x, v[u][0].y, v[u][0].z, v[u][0].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          m[2 * q] = bf2f((unsigned short)(w[q] & 0xffff));
          m[2 * q + 1] = bf2f((unsigned short)(w[q] >> 16));
        }
      }
#pragma unroll
      for (int k = 1; k < 9; ++k) max8(m, v[u][k]);
      *(uint4*)(smem + px[u] * ROW + cg[u] * 16) =
          make_uint4(pack2(m[0], m[1]), pack2(m[2], m[3]), pack2(m[4], m[5]), pack2(m[6], m[7]));
    }
  }
  __syncthreads();

  // 2. GEMM: fragments f = wid + 4t of the output channels, 4 pixel fragments
  f32x4 acc[FMAX][4];
#pragma unroll
  for (int t = 0; t < FMAX; ++t) {
    const int f = wid + 4 * t;
    float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
    if (f < NF) bb = *(const float4*)(g.bias + 16 * f + 4 * fq);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[t][j] = (f32x4){bb.x, bb.y, bb.z, bb.w};
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 pb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pb[j] = *(const bf16x8*)(smem + (16 * j + frow) * ROW + (4 * ks + fq) * 16);
#pragma unroll
    for (int t = 0; t < FMAX; ++t) {
      if (wid + 4 * t < NF) {  // wave-uniform
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[t][ks], pb[j], acc[t][j], 0, 0, 0);
      }
    }
  }

  // 3. epilogue: lane = 4 consecutive channels (16f + 4fq ..) of pixel 16j + frow
#pragma unroll
  for (int t = 0; t < FMAX; ++t) {
    const int f = wid + 4 * t;
    if (f >= NF) continue;
    const int c = 16 * f + 4 * fq;
    int s = 0;
    if (g.nseg > 0) {
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (q < g.nseg && c >= g.seg_c0[q]) s = q;
    }
    unsigned short* dst = (unsigned short*)(g.nseg > 0 ? g.seg_y[s] : g.y);
    const int ld = g.nseg > 0 ? g.seg_ldy[s] : g.ldy;
    const int cc = g.nseg > 0 ? c - g.seg_c0[s] : c;
    const bool relu = (g.nseg > 0 ? g.seg_relu[s] : g.relu) != 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + 16 * j + frow;
      if (m >= M || c >= g.Cout) continue;
      f32x4 v = acc[t][j];
      if (relu) v = (f32x4){fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f)};
      *(uint2*)(dst + (long)m * ld + cc) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
}

}  // namespace pgemm
}  // namespace dml

// 1 if the kernel serves this pool + 1x1 GEMM pair, else 0 (dml_last_error says why not).
extern "C" int dml_pool_gemm_supported(const DmlPoolGemmArgs* a) {
  const DmlPoolArgs& p = a->p;
  const DmlConvArgs& g = a->g;
  const char* why = nullptr;
  if (p.k != 3 || p.stride != 2 || p.pad != 0 || p.mode != 0 || p.relu) why = "pool must be max 3x3/2 valid";
  else if (p.Ho != (p.H - 3) / 2 + 1 || p.Wo != (p.W - 3) / 2 + 1 || p.N < 1) why = "pool output size";
  else if ((p.C != 64 && p.C != 128 && p.C != 192) || p.ldx % 8 || p.ldx < p.C) why = "pool channels (64 / 128 / 192)";
  else if (g.kh != 1 || g.kw != 1 || g.sh != 1 || g.sw != 1 || g.ph || g.pw || g.res || g.out_f32 || g.ksplit > 1)
    why = "GEMM must be a plain 1x1 stride-1 conv";
  else if (g.N != p.N || g.H != p.Ho || g.W != p.Wo || g.Ho != p.Ho || g.Wo != p.Wo || g.Cin != p.C)
    why = "GEMM input must be the pooled grid";
  else if (g.Cout < 16 || g.Cout % 16 || g.Cout > 16 * 4 * dml::pgemm::FMAX || g.Kpad < p.C || g.Kpad % 8)
    why = "GEMM output channels";
  else if (g.nseg > 4) why = "segments";
  if (!why && g.nseg > 0) {
    for (int s = 0; s < g.nseg && !why; ++s)
      if (g.seg_c0[s] % 16 || g.seg_ldy[s] % 4 || !g.seg_y[s] || (s > 0 && g.seg_c0[s] <= g.seg_c0[s - 1]))
        why = "segment layout (16-channel boundaries)";
    if (!why && g.seg_c0[0] != 0) why = "segment 0 starts at channel 0";
  } else if (!why && (g.ldy % 4 || !g.y || g.ldy < g.Cout)) {
    why = "output stride";
  }
  if (why) {
    dml_set_error((std::string("dml_pool_gemm: ") + why).c_str());
    return 0;
  }
  return 1;
}

extern "C" int dml_pool_gemm(const DmlPoolGemmArgs* a, hipStream_t s) {
  if (!dml_pool_gemm_supported(a)) return -1;
  using namespace dml::pgemm;
  const int lds = BMP * (a->p.C * 2 + 16);
  const long M = (long)a->p.N * a->p.Ho * a->p.Wo;
  const dim3 grid((unsigned)((M + BMP - 1) / BMP));
  if (a->p.C == 64) hipLaunchKernelGGL(pool_gemm_kernel<64>, grid, dim3(NT), lds, s, *a);
  else if (a->p.C == 128) hipLaunchKernelGGL(pool_gemm_kernel<128>, grid, dim3(NT), lds, s, *a);
  else hipLaunchKernelGGL(pool_gemm_kernel<192>, grid, dim3(NT), lds, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}
