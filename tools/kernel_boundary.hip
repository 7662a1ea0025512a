// kernel_boundary.hip — what a dependent kernel boundary costs inside a hipGraph on one
// stream (and with a second stream running the same chain concurrently):
//   empty   1 workgroup, no work                       -> CP launch + dependency latency
//   store   2048 x 256 threads, 16 B stored per thread  -> + end-of-kernel writeback of dirty lines
//   spin    2048 x 256 threads, ~SPIN cycles each       -> + ramp-up / tail of a full grid
// Prints microseconds per kernel for chains of N kernels (graph replay, best of R).
//   hipcc --offload-arch=gfx950 -O3 tools/kernel_boundary.hip -o /tmp/kb && /tmp/kb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_empty(int* p) {
  if (threadIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

__global__ void k_store(uint4* p) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  p[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

__global__ void k_spin(int* p, long cycles) {
  const long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < cycles) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

template <class F>
static float time_graph(int nstreams, int n, F launch) {
  hipStream_t s[2];
  for (int i = 0; i < 2; ++i) CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  hipGraph_t g;
  CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeGlobal));
  if (nstreams == 2) {
    CK(hipEventRecord(fork, s[0]));
    CK(hipStreamWaitEvent(s[1], fork, 0));
  }
  for (int k = 0; k < n; ++k)
    for (int j = 0; j < nstreams; ++j) launch(s[j], j);
  if (nstreams == 2) {
    CK(hipEventRecord(join, s[1]));
    CK(hipStreamWaitEvent(s[0], join, 0));
  }
  CK(hipStreamEndCapture(s[0], &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 7; ++r) {
    CK(hipEventRecord(a, s[0]));
    CK(hipGraphLaunch(ge, s[0]));
    CK(hipEventRecord(b, s[0]));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r > 0 && ms < best) best = ms;
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  for (int i = 0; i < 2; ++i) CK(hipStreamDestroy(s[i]));
  return best * 1000.f;  // us
}

int main() {
  int* flag;
  uint4* buf;
  const int WG = 2048, NT = 256;
  CK(hipMalloc(&flag, 64));
  CK(hipMemset(flag, 0, 64));
  CK(hipMalloc(&buf, 2L * WG * NT * sizeof(uint4)));
  const long spin_cycles[] = {2000, 20000};  // s_memtime = shader clock: ~0.8 / ~8 us at 2.4 GHz
  for (int ns = 1; ns <= 2; ++ns) {
    for (int n : {10, 100}) {
      const float te = time_graph(ns, n, [&](hipStream_t st, int) { k_empty<<<1, 64, 0, st>>>(flag); });
      const float tst = time_graph(ns, n, [&](hipStream_t st, int j) {
        k_store<<<WG, NT, 0, st>>>(buf + (long)j * WG * NT);
      });
      printf("streams %d n %3d: empty %.2f us/kernel, store(8 MiB) %.2f us/kernel\n", ns, n, te / n, tst / n);
      for (long c : spin_cycles) {
        const float tsp = time_graph(ns, n, [&](hipStream_t st, int) { k_spin<<<WG, NT, 0, st>>>(flag, c); });
        printf("streams %d n %3d: spin %ld ticks x %d WGs: %.2f us/kernel\n", ns, n, c, WG, tsp / n);
      }
    }
  }
  CK(hipFree(flag));
  CK(hipFree(buf));
  return 0;
}
