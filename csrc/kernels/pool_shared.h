// pool_shared.h — the 3x3 pool body shared by the standalone pool kernel
// (misc.hip: pool3x3_fast_kernel) and the grouped conv launch
// (conv_igemm_v2.hip: conv_v2_group_kernel runs a level's pools in the same
// grid as its convs).
#pragma once
#include "common.h"
#include "dml.h"

namespace dml {
namespace poolk {

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = bf2f(v.x & 0xffff); f[1] = bf2f(v.x >> 16);
  f[2] = bf2f(v.y & 0xffff); f[3] = bf2f(v.y >> 16);
  f[4] = bf2f(v.z & 0xffff); f[5] = bf2f(v.z >> 16);
  f[6] = bf2f(v.w & 0xffff); f[7] = bf2f(v.w >> 16);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// work items (pixel, 8-channel group) of a 3x3 pool
__host__ __device__ inline long pool_work(const DmlPoolArgs& a) { return (long)a.N * a.Ho * a.Wo * (a.C / 8); }

// 3x3 pool, pad <= 1: work item t = one (pixel, 8-channel group), all nine 16-B
// tap loads issued before any is consumed (per-tap branches serialise them:
// max_pooling2d_2 of InceptionV3 ran at 1.9 TB/s that way). Out-of-image taps
// load the clamped edge pixel — for a 3-wide window with pad <= 1 that pixel
// lies inside the window, so max needs no mask; avg weights it 0 and divides by
// the in-image tap count (TF SAME semantics). 32-bit index math.
// LOW_REGS: the window is read one row (3 loads in flight) at a time instead of
// all nine loads up front — about half the live registers, for the pool path of
// the grouped conv kernel, whose register count (and so its occupancy) is the
// max over its conv and pool paths.
template <int MODE, bool LOW_REGS = false>
__device__ __forceinline__ void pool3x3_item(const DmlPoolArgs& a, unsigned t) {
  const unsigned C8 = (unsigned)a.C / 8;
  const unsigned cg = t % C8;
  unsigned p = t / C8;
  const int ow = (int)(p % (unsigned)a.Wo); p /= (unsigned)a.Wo;
  const int oh = (int)(p % (unsigned)a.Ho);
  const int n = (int)(p / (unsigned)a.Ho);
  const int h0 = oh * a.stride - a.pad, w0 = ow * a.stride - a.pad;
  const bf16* xb = (const bf16*)a.x + (long)n * a.H * a.W * a.ldx + cg * 8;
  int rows[3], cols[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    rows[r] = min(max(h0 + r, 0), a.H - 1);
    cols[r] = min(max(w0 + r, 0), a.W - 1);
  }
  float acc[8];
  if constexpr (LOW_REGS) {
    float rw[3], cw[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      rw[r] = (unsigned)(h0 + r) < (unsigned)a.H ? 1.f : 0.f;
      cw[r] = (unsigned)(w0 + r) < (unsigned)a.W ? 1.f : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = MODE == 0 ? -3.0e38f : 0.f;
#pragma unroll 1
    for (int r = 0; r < 3; ++r) {  // one window row (3 loads in flight) at a time
      uint4 v[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = *(const uint4*)(xb + (long)(rows[r] * a.W + cols[c]) * a.ldx);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float f[8];
        unpack8(v[c], f);
        const float wgt = rw[r] * cw[c];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = MODE == 0 ? fmaxf(acc[j], f[j]) : fmaf(wgt, f[j], acc[j]);
      }
    }
    if (MODE != 0) {
      const float inv = 1.f / fmaxf((rw[0] + rw[1] + rw[2]) * (cw[0] + cw[1] + cw[2]), 1.f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= inv;
    }
    if (a.relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaxf(acc[j], 0.f);
    }
    *(uint4*)((bf16*)a.y + ((long)(n * a.Ho + oh) * a.Wo + ow) * a.ldy + cg * 8) = pack8(acc);
    return;
  }
  uint4 v[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) v[r * 3 + c] = *(const uint4*)(xb + (long)(rows[r] * a.W + cols[c]) * a.ldx);
  if (MODE == 0) {
    unpack8(v[0], acc);
#pragma unroll
    for (int q = 1; q < 9; ++q) {
      float f[8];
      unpack8(v[q], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaxf(acc[j], f[j]);
    }
  } else {
    float rw[3], cw[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      rw[r] = (unsigned)(h0 + r) < (unsigned)a.H ? 1.f : 0.f;
      cw[r] = (unsigned)(w0 + r) < (unsigned)a.W ? 1.f : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float f[8];
        unpack8(v[r * 3 + c], f);
        const float wgt = rw[r] * cw[c];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(wgt, f[j], acc[j]);
      }
    const float inv = 1.f / fmaxf((rw[0] + rw[1] + rw[2]) * (cw[0] + cw[1] + cw[2]), 1.f);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= inv;
  }
  if (a.relu) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = fmaxf(acc[j], 0.f);
  }
  *(uint4*)((bf16*)a.y + ((long)(n * a.Ho + oh) * a.Wo + ow) * a.ldy + cg * 8) = pack8(acc);
}

// the conditions of the fast path (dml_pool) and of a pool member of a grouped launch
inline bool pool3x3_fast_ok(const DmlPoolArgs& a) {
  return a.k == 3 && a.pad >= 0 && a.pad <= 1 && a.H >= 1 && a.W >= 1 && a.C % 8 == 0 && a.ldx % 8 == 0 &&
         a.ldy % 8 == 0 && pool_work(a) < (1L << 31);
}

}  // namespace poolk
}  // namespace dml
