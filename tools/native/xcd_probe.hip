// xcd_probe.hip — where do a stream's workgroups run? Each block records its
// XCD (HW_REG_XCC_ID) and the raw HW_ID register of wave 0. Launched on CU-masked
// streams by tools/cu_mask_probe.py to learn how logical CU-mask bits map to XCDs.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(64) void xcd_probe_kernel(unsigned* out) {
  if (threadIdx.x == 0) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID, all 32 bits
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
  // keep the block resident a little so the dispatcher spreads the grid
  for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(1);
}

extern "C" int xcd_probe(unsigned* out_dev, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(xcd_probe_kernel, dim3(blocks), dim3(64), 0, s, out_dev);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
