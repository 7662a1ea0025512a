// misc.hip — the memory-bound kernels around the convolutions (gfx950).
//
//   pool3x3   : max (ResNet pool1 / Inception stem, mixed3, mixed8) and
//               avg 'same' with padding excluded from the divisor (Inception
//               pool branches; TF SAME avg_pool semantics).
//   gap       : global average pool, NHWC -> [N][C].
//   softmax_top5 : row softmax over the classes + wave-level top-5 (replaces
//               Keras decode_predictions(top=5), reference models.py:42,67).
//   preprocess: uint8 RGB -> nearest resize -> caffe/tf normalisation -> bf16
//               NHWC with the channel dim padded to 8 (reference models.py:34-38,
//               59-63 do this per image on the CPU).
// All bf16 traffic is 16 bytes per lane (8 channels), per the CDNA4 guide's
// vectorisation rule; every kernel is a grid-stride loop capped near 8 blocks/CU.
#include "common.h"
#include "dml.h"
#include "pool_shared.h"
#include <cstdlib>

namespace dml {

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = bf2f(v.x & 0xffff); f[1] = bf2f(v.x >> 16);
  f[2] = bf2f(v.y & 0xffff); f[3] = bf2f(v.y >> 16);
  f[4] = bf2f(v.z & 0xffff); f[5] = bf2f(v.z >> 16);
  f[6] = bf2f(v.w & 0xffff); f[7] = bf2f(v.w >> 16);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

static inline unsigned grid_for(long work, int block) {
  long g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (unsigned)g;
}

__global__ __launch_bounds__(256) void pool3x3_kernel(DmlPoolArgs a) {
  const int C8 = a.C / 8;
  const long total = (long)a.N * a.Ho * a.Wo * C8;
  const bf16* x = (const bf16*)a.x;
  bf16* y = (bf16*)a.y;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % C8);
    long p = t / C8;
    const int ow = (int)(p % a.Wo); p /= a.Wo;
    const int oh = (int)(p % a.Ho);
    const int n = (int)(p / a.Ho);
    const int h0 = oh * a.stride - a.pad, w0 = ow * a.stride - a.pad;
    float acc[8];
    const float init = a.mode == 0 ? -3.0e38f : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = init;
    int cnt = 0;
    for (int r = 0; r < a.k; ++r) {
      const int ih = h0 + r;
      if ((unsigned)ih >= (unsigned)a.H) continue;
      for (int s = 0; s < a.k; ++s) {
        const int iw = w0 + s;
        if ((unsigned)iw >= (unsigned)a.W) continue;
        const uint4 v = *(const uint4*)(x + ((long)(n * a.H + ih) * a.W + iw) * a.ldx + cg * 8);
        float f[8];
        unpack8(v, f);
        if (a.mode == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = fmaxf(acc[j], f[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += f[j];
        }
        ++cnt;
      }
    }
    if (a.mode == 1) {
      const float inv = 1.f / (float)(cnt > 0 ? cnt : 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= inv;
    }
    if (a.relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaxf(acc[j], 0.f);
    }
    *(uint4*)(y + ((long)(n * a.Ho + oh) * a.Wo + ow) * a.ldy + cg * 8) = pack8(acc);
  }
}

// 3x3 pool, pad <= 1 (body: pool_shared.h, also run inside grouped conv grids)
template <int MODE>
__global__ __launch_bounds__(256) void pool3x3_fast_kernel(DmlPoolArgs a, unsigned total) {
  const unsigned t = blockIdx.x * 256u + threadIdx.x;
  if (t < total) poolk::pool3x3_item<MODE>(a, t);
}

// Global average pool. One workgroup per (image, 256-channel slab): 8 pixel
// lanes x 32 channel groups, each thread sums every 8th pixel of its 16-B
// channel group, then the 8 partial sums meet in LDS. N*ceil(C/256) workgroups
// (ResNet50 b128: 1024) and 8 independent 16-B loads in flight per lane-column,
// instead of one thread walking all HW pixels of a channel group.
__global__ __launch_bounds__(256) void gap_kernel(const bf16* x, bf16* y, int N, int HW, int C, int ldx) {
  __shared__ float part[8][32][9];  // +1 pad: the 8 partial rows of a group land in different banks
  const int n = blockIdx.x / ((C + 255) / 256);
  const int slab = blockIdx.x - n * ((C + 255) / 256);
  const int cgl = threadIdx.x & 31, py = threadIdx.x >> 5;
  const int cg = slab * 32 + cgl;
  const bool ok = cg * 8 < C;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (ok) {
    const bf16* base = x + (long)n * HW * ldx + cg * 8;
    for (int p = py; p < HW; p += 8) {
      float f[8];
      unpack8(*(const uint4*)(base + (long)p * ldx), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[py][cgl][j] = acc[j];
  __syncthreads();
  if (py == 0 && ok) {
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) t += part[q][cgl][j];
      acc[j] = t * inv;
    }
    *(uint4*)(y + (long)n * C + cg * 8) = pack8(acc);
  }
}

// One 256-thread workgroup per row (4 waves): thread t owns classes t, t+256, ...
// With nsplit > 1 the logits arrive as split-K partial slices (the classifier
// GEMM's K range cut over workgroups): they are summed here, in slice order
// (deterministic), and the summed row is written back to slice 0. Max / sum /
// 5 rounds of argmax (ties -> lower class id) reduce per wave with shuffles,
// then across the 4 waves through LDS.
__device__ __forceinline__ void argmax_merge(float& v, int& i, float ov, int oi) {
  if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
}

template <int PER_T>
__global__ __launch_bounds__(256) void softmax_top5_kernel(float* logits, int B, int classes, int ld, int nsplit,
                                                           int split_ld, float* probs, int* top_idx, float* top_p) {
  __shared__ float red_v[4];
  __shared__ int red_i[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int row = blockIdx.x;
  if (row >= B) return;
  float* lr = logits + (long)row * ld;
  float v[PER_T];
#pragma unroll
  for (int i = 0; i < PER_T; ++i) {
    const int c = tid + i * 256;
    v[i] = c < classes ? lr[c] : -3.0e38f;
  }
  if (nsplit > 1) {
#pragma unroll 4
    for (int sp = 1; sp < nsplit; ++sp) {
      const float* ls = lr + (long)sp * split_ld;
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int c = tid + i * 256;
        if (c < classes) v[i] += ls[c];
      }
    }
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = tid + i * 256;
      if (c < classes) lr[c] = v[i];
    }
  }
  // row max
  float mx = -3.0e38f;
#pragma unroll
  for (int i = 0; i < PER_T; ++i) mx = fmaxf(mx, v[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (lane == 0) red_v[w] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red_v[0], red_v[1]), fmaxf(red_v[2], red_v[3]));
  __syncthreads();
  // row sum of exp
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < PER_T; ++i) {
    const int c = tid + i * 256;
    if (c < classes) sum += __expf(v[i] - mx);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (lane == 0) red_v[w] = sum;
  __syncthreads();
  sum = (red_v[0] + red_v[1]) + (red_v[2] + red_v[3]);
  __syncthreads();
  const float inv = 1.f / sum;
  if (probs) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = tid + i * 256;
      if (c < classes) probs[(long)row * classes + c] = __expf(v[i] - mx) * inv;
    }
  }
  // top-5: 5 rounds of (thread-local argmax -> wave -> workgroup)
  unsigned taken = 0;
  for (int k = 0; k < 5; ++k) {
    float bv = -3.0e38f;
    int bi = 0x7fffffff, bslot = -1;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = tid + i * 256;
      if (c < classes && !(taken >> i & 1u) && v[i] > bv) { bv = v[i]; bi = c; bslot = i; }
    }
    float wv = bv;
    int wi = bi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) argmax_merge(wv, wi, __shfl_xor(wv, o), __shfl_xor(wi, o));
    if (lane == 0) { red_v[w] = wv; red_i[w] = wi; }
    __syncthreads();
    float gv = red_v[0];
    int gi = red_i[0];
#pragma unroll
    for (int q = 1; q < 4; ++q) argmax_merge(gv, gi, red_v[q], red_i[q]);
    __syncthreads();
    if (gi == bi && bslot >= 0) taken |= 1u << bslot;
    if (tid == 0) {
      top_idx[row * 5 + k] = gi;
      top_p[row * 5 + k] = __expf(gv - mx) * inv;
    }
  }
}

// One WAVE per row (4 rows per 256-thread workgroup), classes <= 1024: lane l owns classes
// l, l + 64, ... in registers; the split-K slices are summed in slice order (the same fp32
// additions, in the same order, as softmax_top5_kernel), max / sum / 5 argmax rounds reduce with
// wave shuffles only — no LDS, no barrier (the workgroup kernel above spends its time in 7
// barriers and 8 dependent slice loads per row).
__global__ __launch_bounds__(256) void softmax_top5_wave_kernel(float* logits, int B, int classes, int ld, int nsplit,
                                                                int split_ld, float* probs, int* top_idx,
                                                                float* top_p) {
  constexpr int PER = 16;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;  // wave-uniform
  float* lr = logits + (long)row * ld;
  float v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < classes ? lr[c] : -3.0e38f;
  }
  if (nsplit > 1) {
    for (int sp = 1; sp < nsplit; ++sp) {
      const float* ls = lr + (long)sp * split_ld;
      float u[PER];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = lane + 64 * i;
        u[i] = c < classes ? ls[c] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < PER; ++i) v[i] += u[i];
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c < classes) lr[c] = v[i];
    }
  }
  float mx = -3.0e38f;
#pragma unroll
  for (int i = 0; i < PER; ++i) mx = fmaxf(mx, v[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    if (c < classes) sum += __expf(v[i] - mx);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  const float inv = 1.f / sum;
  if (probs) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c < classes) probs[(long)row * classes + c] = __expf(v[i] - mx) * inv;
    }
  }
  unsigned taken = 0;
  for (int k = 0; k < 5; ++k) {
    float bv = -3.0e38f;
    int bi = 0x7fffffff, bslot = -1;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c < classes && !(taken >> i & 1u) && v[i] > bv) { bv = v[i]; bi = c; bslot = i; }
    }
    float wv = bv;
    int wi = bi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) argmax_merge(wv, wi, __shfl_xor(wv, o), __shfl_xor(wi, o));
    if (wi == bi && bslot >= 0) taken |= 1u << bslot;
    if (lane == 0) {
      top_idx[row * 5 + k] = wi;
      top_p[row * 5 + k] = __expf(wv - mx) * inv;
    }
  }
}

// Pillow NEAREST resize (Keras load_img default): src = floor((dst + 0.5) * Ssrc / Sdst).
__device__ __forceinline__ void preprocess_pixel(const DmlPreprocArgs& a, const unsigned char* src, int n, int oh,
                                                 int ow, float sy, float sx, float* f) {
  int iy = (int)(((float)oh + 0.5f) * sy), ix = (int)(((float)ow + 0.5f) * sx);
  iy = min(iy, a.Hs - 1);
  ix = min(ix, a.Ws - 1);
  const long img_n = a.idx ? (long)a.idx[n] : (long)n;  // an HBM arena slot (serving path) or n
  const unsigned char* px = src + ((img_n * a.Hs + iy) * a.Ws + ix) * 3;
  const float r = px[0], g = px[1], b = px[2];
  if (a.mode == 0) {  // caffe: RGB->BGR, subtract BGR mean, no scaling
    f[0] = b - 103.939f; f[1] = g - 116.779f; f[2] = r - 123.68f;
  } else {            // tf: scale to [-1, 1]
    f[0] = r / 127.5f - 1.f; f[1] = g / 127.5f - 1.f; f[2] = b / 127.5f - 1.f;
  }
}

// pair == 0: y[n][oh][ow][8] = (c0, c1, c2, 0 x5)
// pair == 1: y[n][oh][j][8] = (pixel j-lpad: c0..c2, 0, pixel j-lpad+1: c0..c2, 0), zero outside the
//            image — the stem conv then sees two horizontal taps per 16-byte chunk (dilation 2).
__global__ __launch_bounds__(256) void preprocess_kernel(DmlPreprocArgs a) {
  const int Wout = a.Wo + (a.pair ? a.lpad : 0);
  const long total = (long)a.N * a.Ho * Wout;
  const float sy = (float)a.Hs / (float)a.Ho, sx = (float)a.Ws / (float)a.Wo;
  const unsigned char* src = (const unsigned char*)a.src;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int j = (int)(t % Wout);
    long p = t / Wout;
    const int oh = (int)(p % a.Ho);
    const int n = (int)(p / a.Ho);
    float f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int ow = a.pair ? j - a.lpad : j;
    if (ow >= 0 && ow < a.Wo) preprocess_pixel(a, src, n, oh, ow, sy, sx, f);
    if (a.pair && ow + 1 >= 0 && ow + 1 < a.Wo) preprocess_pixel(a, src, n, oh, ow + 1, sy, sx, f + 4);
    *(uint4*)((bf16*)a.y + t * 8) = pack8(f);
  }
}

// dev[i] = host[i], i < n: the serving path's per-launch arena slot table, fetched from pinned
// host memory once per batch (system-scope loads) so that the stem kernels' workgroups read
// it from device memory (a host read per workgroup made the ResNet50 stem 3.8x slower:
// profiles/r4_service/stem_bench.log)
__global__ __launch_bounds__(1024) void index_fetch_kernel(const int* __restrict__ host, int* __restrict__ dev, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) dev[i] = dml_host_index(host, i);
}

// A staged window's decoded images (full resolution, packed) -> their arena slots, resized
// nearest-neighbour on the GPU (the store path's CPU decode pool only entropy-decodes; the two
// per-model resizes were 43 % of its CPU per image). pack: n records {src offset in 16-byte units
// (a pack may exceed 2 GiB: ADVICE r5), h, w, row-table offset, column-table offset, slot} (int32),
// then the int32 source row / column tables (computed on the host with Pillow's own float64 accumulation, so the
// result is byte-identical to Image.resize(NEAREST)), then the RGB pixels. One workgroup per
// (output row, image); dst = arena [slots][H][W][3].
__global__ __launch_bounds__(256) void resize_nearest_kernel(const unsigned char* __restrict__ pack, int n, int H,
                                                             int W, unsigned char* __restrict__ dst) {
  const int y = blockIdx.x, i = blockIdx.y;
  if (i >= n || y >= H) return;
  const int* rec = (const int*)pack + i * 6;
  const size_t off = (size_t)(unsigned)rec[0] << 4;
  const int w = rec[2], yt = rec[3], xt = rec[4], slot = rec[5];
  const int* tab = (const int*)(pack + (size_t)n * 24);
  const unsigned char* srow = pack + off + (size_t)tab[yt + y] * w * 3;
  unsigned char* drow = dst + ((size_t)slot * H + y) * W * 3;
  for (int x = threadIdx.x; x < W; x += blockDim.x) {
    const unsigned char* p = srow + (size_t)tab[xt + x] * 3;
    drow[x * 3] = p[0];
    drow[x * 3 + 1] = p[1];
    drow[x * 3 + 2] = p[2];
  }
}

}  // namespace dml

extern "C" int dml_resize_nearest(const void* pack, int n, int H, int W, void* dst, hipStream_t s) {
  if (n <= 0) return 0;
  if (H <= 0 || W <= 0 || H > 65535) {
    dml_set_error("dml_resize_nearest: bad output size");
    return -1;
  }
  hipLaunchKernelGGL(dml::resize_nearest_kernel, dim3(H, n), dim3(256), 0, s, (const unsigned char*)pack, n, H, W,
                     (unsigned char*)dst);
  DML_CHECK_LAUNCH();
  return 0;
}

extern "C" int dml_index_fetch(const int* host, int* dev, int n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(dml::index_fetch_kernel, dim3(1), dim3(n < 1024 ? ((n + 63) / 64) * 64 : 1024), 0, s, host, dev, n);
  DML_CHECK_LAUNCH();
  return 0;
}

extern "C" int dml_pool(const DmlPoolArgs* a, hipStream_t s) {
  static const bool generic = getenv("DML_POOL_GENERIC") != nullptr;  // A/B switch: the per-tap kernel
  if (a->C % 8 || a->ldx % 8 || a->ldy % 8) { dml_set_error("dml_pool: channels must be %8"); return -1; }
  const long work = dml::poolk::pool_work(*a);
  if (!generic && dml::poolk::pool3x3_fast_ok(*a)) {
    const unsigned blocks = (unsigned)((work + 255) / 256);
    if (a->mode == 0)
      hipLaunchKernelGGL(dml::pool3x3_fast_kernel<0>, dim3(blocks), dim3(256), 0, s, *a, (unsigned)work);
    else
      hipLaunchKernelGGL(dml::pool3x3_fast_kernel<1>, dim3(blocks), dim3(256), 0, s, *a, (unsigned)work);
  } else {
    hipLaunchKernelGGL(dml::pool3x3_kernel, dim3(dml::grid_for(work, 256)), dim3(256), 0, s, *a);
  }
  DML_CHECK_LAUNCH();
  return 0;
}

extern "C" int dml_global_avgpool(const void* x, void* y, int N, int HW, int C, int ldx, hipStream_t s) {
  if (C % 8 || ldx % 8) { dml_set_error("dml_global_avgpool: channels must be %8"); return -1; }
  hipLaunchKernelGGL(dml::gap_kernel, dim3((unsigned)(N * ((C + 255) / 256))), dim3(256), 0, s, (const bf16*)x,
                     (bf16*)y, N, HW, C, ldx);
  DML_CHECK_LAUNCH();
  return 0;
}

extern "C" int dml_softmax_top5_split(float* logits, int B, int classes, int ld, int nsplit, int split_ld,
                                      float* probs, int* top_idx, float* top_p, hipStream_t s) {
  const dim3 grid(B), block(256);
  if (nsplit < 1) nsplit = 1;
  static const bool wg = getenv("DML_SOFTMAX_WG") != nullptr;  // A/B switch: one workgroup per row
  if (!wg && classes <= 1024) {
    hipLaunchKernelGGL(dml::softmax_top5_wave_kernel, dim3((unsigned)((B + 3) / 4)), block, 0, s, logits, B, classes,
                       ld, nsplit, split_ld, probs, top_idx, top_p);
  } else if (classes <= 4 * 256) {
    hipLaunchKernelGGL(dml::softmax_top5_kernel<4>, grid, block, 0, s, logits, B, classes, ld, nsplit, split_ld,
                       probs, top_idx, top_p);
  } else if (classes <= 8 * 256) {
    hipLaunchKernelGGL(dml::softmax_top5_kernel<8>, grid, block, 0, s, logits, B, classes, ld, nsplit, split_ld,
                       probs, top_idx, top_p);
  } else {
    dml_set_error("dml_softmax_top5: classes > 2048");
    return -1;
  }
  DML_CHECK_LAUNCH();
  return 0;
}

extern "C" int dml_softmax_top5(const float* logits, int B, int classes, int ld, float* probs, int* top_idx,
                                float* top_p, hipStream_t s) {
  return dml_softmax_top5_split((float*)logits, B, classes, ld, 1, 0, probs, top_idx, top_p, s);
}

extern "C" int dml_preprocess(const DmlPreprocArgs* a, hipStream_t s) {
  const long work = (long)a->N * a->Ho * (a->Wo + (a->pair ? a->lpad : 0));
  hipLaunchKernelGGL(dml::preprocess_kernel, dim3(dml::grid_for(work, 256)), dim3(256), 0, s, *a);
  DML_CHECK_LAUNCH();
  return 0;
}
