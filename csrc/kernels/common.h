// common.h — device-side helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace dml {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(((unsigned)u) << 16); }

// RNE float -> bf16 bits (hipcc lowers the __bf16 cast to v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ unsigned short f2bf(float f) {
  bf16 h = (bf16)f;
  return __builtin_bit_cast(unsigned short, h);
}

__device__ __forceinline__ unsigned pack2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}

// Bijective XCD-aware block remap (MI355X: 8 XCDs, blocks dealt round-robin).
// Blocks that share an XCD (b % 8 equal) get a contiguous range of logical ids,
// so neighbouring tiles (which share operand panels) hit the same L2.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int xcd = b & 7, q = nb >> 3, r = nb & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (b >> 3);
}

// Max of 8 bf16 values that are all >= +0 (post-ReLU; the writer clears the sign bit, so no
// -0): for non-negative IEEE values the bit patterns order like the values, so the max is
// one packed 16-bit unsigned max per 2 channels (v_pk_max_u16) — no bf16 <-> fp32
// conversion, exact.
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint4 max_bf16x8_nonneg(uint4 a, uint4 b) {
  return __builtin_bit_cast(uint4, __builtin_elementwise_max(__builtin_bit_cast(u16x8, a),
                                                             __builtin_bit_cast(u16x8, b)));
}
constexpr unsigned kNoSign2 = 0x7fff7fffu;  // two bf16 with the sign bits cleared (-0 -> +0)

// Entry n of a table in pinned host memory that the host rewrites between launches (the
// serving path's arena slot table, misc.hip index_fetch_kernel): a system-scope vector load,
// never served from a stale cache line of an earlier launch.
__device__ __forceinline__ int dml_host_index(const int* idx, int n) {
  return __hip_atomic_load(idx + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace dml

// error plumbing for the host API (defined in runtime/errors.hip)
extern "C" void dml_set_error(const char* msg);
#define DML_CHECK_LAUNCH()                                        \
  do {                                                            \
    hipError_t _e = hipGetLastError();                            \
    if (_e != hipSuccess) {                                       \
      dml_set_error(hipGetErrorString(_e));                       \
      return -1;                                                  \
    }                                                             \
  } while (0)
