// runtime.hip — the native host runtime around the kernels.
//
//  * Plan executor: the model graph (built once by the Python planner from the
//    layer IR) is a flat vector of launch records replayed per batch. It can be
//    captured into a hipGraph so a forward is one graph launch (the reference
//    rebuilds the Keras model for every batch instead, models.py:18-21,84-91).
//  * Pinned staging ring: hipHostMalloc'd slots + one event per slot. A copy
//    stream moves batch k+1 host->HBM (hipMemcpyAsync) while the compute stream
//    runs batch k; the compute stream waits on the slot's event, not on the host.
//    This replaces the reference's per-image scp pull (worker.py:1365-1366,
//    file_service.py:116-124).
#include <hip/hip_runtime.h>
#include <string>
#include <vector>
#include <mutex>
#include <cstring>
#include "dml.h"

static thread_local std::string g_err;
extern "C" void dml_set_error(const char* msg) { g_err = msg ? msg : ""; }
extern "C" const char* dml_last_error(void) { return g_err.c_str(); }

#define HIP_OK(expr)                                       \
  do {                                                     \
    hipError_t _e = (expr);                                \
    if (_e != hipSuccess) {                                \
      g_err = std::string(#expr) + ": " + hipGetErrorString(_e); \
      return -1;                                           \
    }                                                      \
  } while (0)

extern "C" int dml_device_info(int* cus, int* arch_major, int* arch_minor) {
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  hipDeviceProp_t p;
  HIP_OK(hipGetDeviceProperties(&p, dev));
  *cus = p.multiProcessorCount;
  *arch_major = p.major;
  *arch_minor = p.minor;
  return 0;
}

// Argument-struct sizes, in the order of _native.ABI_STRUCTS: the Python
// bindings refuse a library whose structs do not match their ctypes mirrors.
extern "C" int dml_abi_sizes(int* out, int n) {
  const int sz[] = {(int)sizeof(DmlConvArgs), (int)sizeof(DmlPoolArgs), (int)sizeof(DmlConvGroupArgs),
                    (int)sizeof(DmlPreprocArgs), (int)sizeof(DmlStemArgs), (int)sizeof(DmlIncStemArgs),
                    (int)sizeof(DmlConvPoolArgs), (int)sizeof(DmlExpandReduceArgs)};
  const int m = (int)(sizeof(sz) / sizeof(sz[0]));
  for (int i = 0; i < n && i < m; ++i) out[i] = sz[i];
  return m;
}

// ----------------------------------------------------------------- plan ----
namespace {
enum OpKind { OP_CONV, OP_POOL, OP_GAP, OP_SMTOP5, OP_PREPROC, OP_STEM, OP_INC_STEM, OP_CONV_POOL, OP_EXP_RED,
              OP_CONV_GROUP };
struct GapArgs { const void* x; void* y; int N, HW, C, ldx; };
struct SmArgs { float* logits; int B, classes, ld, nsplit, split_ld; float* probs; int* idx; float* p; };
struct Op {
  OpKind kind;
  int cfg;
  DmlConvArgs conv;
  DmlPoolArgs pool;
  GapArgs gap;
  SmArgs sm;
  DmlPreprocArgs pre;
  DmlStemArgs stem;
  DmlIncStemArgs istem;
  DmlConvPoolArgs cpool;
  DmlExpandReduceArgs er;
  DmlConvGroupArgs grp;
};
struct Plan {
  std::vector<Op> ops;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  std::vector<hipGraph_t> part_graphs;      // dml_plan_capture_parts: one graph per op range
  std::vector<hipGraphExec_t> part_execs;
  void clear_parts() {
    for (auto e : part_execs) (void)hipGraphExecDestroy(e);
    for (auto g : part_graphs) (void)hipGraphDestroy(g);
    part_execs.clear();
    part_graphs.clear();
  }
  ~Plan() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    clear_parts();
  }
};

int run_op(const Op& o, hipStream_t s) {
  switch (o.kind) {
    case OP_CONV: return dml_conv(&o.conv, o.cfg, s);
    case OP_POOL: return dml_pool(&o.pool, s);
    case OP_GAP: return dml_global_avgpool(o.gap.x, o.gap.y, o.gap.N, o.gap.HW, o.gap.C, o.gap.ldx, s);
    case OP_SMTOP5:
      return dml_softmax_top5_split(o.sm.logits, o.sm.B, o.sm.classes, o.sm.ld, o.sm.nsplit, o.sm.split_ld,
                                    o.sm.probs, o.sm.idx, o.sm.p, s);
    case OP_PREPROC: return dml_preprocess(&o.pre, s);
    case OP_STEM: return dml_stem_resnet(&o.stem, s);
    case OP_INC_STEM: return dml_stem_inception(&o.istem, s);
    case OP_CONV_POOL: return dml_conv3x3_pool(&o.cpool, s);
    case OP_EXP_RED: return dml_expand_reduce(&o.er, s);
    case OP_CONV_GROUP: return dml_conv_group(&o.grp, o.cfg, s);
  }
  return -1;
}
}  // namespace

extern "C" void* dml_plan_create(void) { return new Plan(); }
extern "C" void dml_plan_destroy(void* p) { delete (Plan*)p; }
extern "C" int dml_plan_size(void* p) { return (int)((Plan*)p)->ops.size(); }

extern "C" int dml_plan_add_conv(void* p, const DmlConvArgs* a, int cfg) {
  Op o{};
  o.kind = OP_CONV;
  o.conv = *a;
  o.cfg = cfg < 0 ? dml_conv_pick_cfg(a) : cfg;
  if (dml_conv_v2_bn(o.cfg) <= 0) { g_err = "dml_plan_add_conv: no tile config for this conv"; return -1; }
  ((Plan*)p)->ops.push_back(o);
  return o.cfg;
}
extern "C" int dml_plan_add_pool(void* p, const DmlPoolArgs* a) {
  Op o{};
  o.kind = OP_POOL;
  o.pool = *a;
  ((Plan*)p)->ops.push_back(o);
  return 0;
}
extern "C" int dml_plan_add_gap(void* p, const void* x, void* y, int N, int HW, int C, int ldx) {
  Op o{};
  o.kind = OP_GAP;
  o.gap = GapArgs{x, y, N, HW, C, ldx};
  ((Plan*)p)->ops.push_back(o);
  return 0;
}
extern "C" int dml_plan_add_softmax_top5_split(void* p, float* logits, int B, int classes, int ld, int nsplit,
                                               int split_ld, float* probs, int* idx, float* pr) {
  Op o{};
  o.kind = OP_SMTOP5;
  o.sm = SmArgs{logits, B, classes, ld, nsplit, split_ld, probs, idx, pr};
  ((Plan*)p)->ops.push_back(o);
  return 0;
}
extern "C" int dml_plan_add_softmax_top5(void* p, const float* logits, int B, int classes, int ld, float* probs,
                                         int* idx, float* pr) {
  return dml_plan_add_softmax_top5_split(p, (float*)logits, B, classes, ld, 1, 0, probs, idx, pr);
}
extern "C" int dml_plan_add_preprocess(void* p, const DmlPreprocArgs* a) {
  Op o{};
  o.kind = OP_PREPROC;
  o.pre = *a;
  ((Plan*)p)->ops.push_back(o);
  return 0;
}
extern "C" int dml_plan_add_stem(void* p, const DmlStemArgs* a) {
  Op o{};
  o.kind = OP_STEM;
  o.stem = *a;
  ((Plan*)p)->ops.push_back(o);
  return 0;
}
extern "C" int dml_plan_add_inc_stem(void* p, const DmlIncStemArgs* a) {
  Op o{};
  o.kind = OP_INC_STEM;
  o.istem = *a;
  ((Plan*)p)->ops.push_back(o);
  return 0;
}
extern "C" int dml_plan_add_conv_pool(void* p, const DmlConvPoolArgs* a) {
  Op o{};
  o.kind = OP_CONV_POOL;
  o.cpool = *a;
  ((Plan*)p)->ops.push_back(o);
  return 0;
}
extern "C" int dml_plan_add_conv_group(void* p, const DmlConvGroupArgs* g, int cfg) {
  if (dml_conv_group_validate(g, cfg) != 0) return -1;
  Op o{};
  o.kind = OP_CONV_GROUP;
  o.grp = *g;
  o.cfg = cfg;
  ((Plan*)p)->ops.push_back(o);
  return cfg;
}

extern "C" int dml_plan_add_expand_reduce(void* p, const DmlExpandReduceArgs* a) {
  Op o{};
  o.kind = OP_EXP_RED;
  o.er = *a;
  ((Plan*)p)->ops.push_back(o);
  return 0;
}

extern "C" int dml_plan_run_range(void* p, int begin, int end, hipStream_t s) {
  Plan* pl = (Plan*)p;
  if (end < 0 || end > (int)pl->ops.size()) end = (int)pl->ops.size();
  for (int i = begin; i < end; ++i)
    if (run_op(pl->ops[i], s)) return -1 - i;
  return 0;
}
extern "C" int dml_plan_run(void* p, hipStream_t s) { return dml_plan_run_range(p, 0, -1, s); }

extern "C" int dml_plan_capture(void* p, hipStream_t s) {
  Plan* pl = (Plan*)p;
  if (pl->exec) { (void)hipGraphExecDestroy(pl->exec); pl->exec = nullptr; }
  if (pl->graph) { (void)hipGraphDestroy(pl->graph); pl->graph = nullptr; }
  HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  int rc = dml_plan_run(p, s);
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(s, &g);
  if (rc) return rc;
  if (e != hipSuccess) { g_err = hipGetErrorString(e); return -1; }
  pl->graph = g;
  HIP_OK(hipGraphInstantiate(&pl->exec, g, nullptr, nullptr, 0));
  return 0;
}
// Capture ops [bounds[i], bounds[i+1]) as graph i (i < nparts): the forward can
// then be replayed in pieces, e.g. to stagger sub-batches on two streams.
extern "C" int dml_plan_capture_parts(void* p, const int* bounds, int nparts, hipStream_t s) {
  Plan* pl = (Plan*)p;
  pl->clear_parts();
  for (int i = 0; i < nparts; ++i) {
    if (bounds[i] < 0 || bounds[i] > bounds[i + 1] || bounds[i + 1] > (int)pl->ops.size()) {
      g_err = "dml_plan_capture_parts: bad bounds";
      return -1;
    }
    HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int rc = dml_plan_run_range(p, bounds[i], bounds[i + 1], s);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(s, &g);
    if (rc) return rc;
    if (e != hipSuccess) { g_err = hipGetErrorString(e); return -1; }
    hipGraphExec_t x = nullptr;
    HIP_OK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    pl->part_graphs.push_back(g);
    pl->part_execs.push_back(x);
  }
  return 0;
}
extern "C" int dml_plan_replay_part(void* p, int i, hipStream_t s) {
  Plan* pl = (Plan*)p;
  if (i < 0 || i >= (int)pl->part_execs.size()) { g_err = "dml_plan_replay_part: not captured"; return -1; }
  HIP_OK(hipGraphLaunch(pl->part_execs[i], s));
  return 0;
}
extern "C" int dml_plan_replay(void* p, hipStream_t s) {
  Plan* pl = (Plan*)p;
  if (!pl->exec) { g_err = "dml_plan_replay: not captured"; return -1; }
  HIP_OK(hipGraphLaunch(pl->exec, s));
  return 0;
}

// One batch launch of the serving loop in one call (GpuRankBackend.launch): the sequence of
// event records, stream waits, index-table fetches and graph replays that Engine / SplitEngine
// .run issue one Python call each (8-10 HIP calls a batch, ~0.8 ms of serve-loop time under the
// decode pool's GIL traffic). ops: n records of 5 int64 {kind, a, b, c, d}:
//   0 record event a on stream b        1 stream a waits on event b
//   2 replay plan a on stream b         3 replay part b of plan a on stream c
//   4 index fetch host a -> device b, c entries, on stream d
// Returns 0, or -1 - i for the first op i that failed.
extern "C" int dml_launch_seq(const int64_t* ops, int n) {
  for (int i = 0; i < n; ++i) {
    const int64_t* o = ops + 5 * i;
    int rc = 0;
    switch (o[0]) {
      case 0: rc = hipEventRecord((hipEvent_t)o[1], (hipStream_t)o[2]) == hipSuccess ? 0 : -1; break;
      case 1: rc = hipStreamWaitEvent((hipStream_t)o[1], (hipEvent_t)o[2], 0) == hipSuccess ? 0 : -1; break;
      case 2: rc = dml_plan_replay((void*)o[1], (hipStream_t)o[2]); break;
      case 3: rc = dml_plan_replay_part((void*)o[1], (int)o[2], (hipStream_t)o[3]); break;
      case 4: rc = dml_index_fetch((const int*)o[1], (int*)o[2], (int)o[3], (hipStream_t)o[4]); break;
      default: g_err = "dml_launch_seq: bad op"; rc = -1;
    }
    if (rc) {
      if (o[0] <= 1) g_err = "dml_launch_seq: event op failed";
      return -1 - i;
    }
  }
  return 0;
}

// Re-point conv op i at tile config cfg (joint tuning of co-scheduled
// sub-batch plans). Returns the previous cfg, or -1 if op i is not a conv or
// cfg is not a tile config. A captured graph must be re-captured.
// tile config of a conv or grouped-conv op (co-tuning: tools/cotune*.py)
extern "C" int dml_plan_set_cfg(void* p, int i, int cfg) {
  Plan* pl = (Plan*)p;
  if (i < 0 || i >= (int)pl->ops.size() || (pl->ops[i].kind != OP_CONV && pl->ops[i].kind != OP_CONV_GROUP)) {
    g_err = "dml_plan_set_cfg: not a conv op";
    return -1;
  }
  Op& o = pl->ops[i];
  if (o.kind == OP_CONV_GROUP) {
    if (dml_conv_group_validate(&o.grp, cfg) != 0) return -1;
  } else if (dml_conv_v2_bn(cfg) <= 0) {
    g_err = "dml_plan_set_cfg: not a tile config";
    return -1;
  }
  const int prev = o.cfg;
  o.cfg = cfg;
  return prev;
}
extern "C" int dml_plan_get_cfg(void* p, int i) {
  Plan* pl = (Plan*)p;
  if (i < 0 || i >= (int)pl->ops.size() || (pl->ops[i].kind != OP_CONV && pl->ops[i].kind != OP_CONV_GROUP)) return -1;
  return pl->ops[i].cfg;
}

extern "C" int dml_plan_time_ops(void* p, hipStream_t s, float* ms_out, int n) {
  Plan* pl = (Plan*)p;
  const int cnt = (int)pl->ops.size() < n ? (int)pl->ops.size() : n;
  std::vector<hipEvent_t> ev(cnt + 1);
  for (auto& e : ev) HIP_OK(hipEventCreate(&e));
  HIP_OK(hipEventRecord(ev[0], s));
  for (int i = 0; i < cnt; ++i) {
    if (run_op(pl->ops[i], s)) return -1;
    HIP_OK(hipEventRecord(ev[i + 1], s));
  }
  HIP_OK(hipEventSynchronize(ev[cnt]));
  for (int i = 0; i < cnt; ++i) HIP_OK(hipEventElapsedTime(&ms_out[i], ev[i], ev[i + 1]));
  for (auto& e : ev) (void)hipEventDestroy(e);
  return 0;
}

// ---------------------------------------------------------- staging ring ----
namespace {
struct Ring {
  std::vector<void*> host;
  std::vector<hipEvent_t> ev;
  size_t slot_bytes = 0;
};
}  // namespace

extern "C" void* dml_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) { g_err = "hipHostMalloc failed"; return nullptr; }
  return p;
}
extern "C" void dml_host_free(void* p) { if (p) (void)hipHostFree(p); }

extern "C" int dml_memcpy_h2d_async(void* dst, const void* src, size_t bytes, hipStream_t s) {
  HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
  return 0;
}
extern "C" int dml_memcpy_d2h_async(void* dst, const void* src, size_t bytes, hipStream_t s) {
  HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
  return 0;
}

extern "C" void* dml_ring_create(int slots, size_t slot_bytes) {
  Ring* r = new Ring();
  r->slot_bytes = slot_bytes;
  for (int i = 0; i < slots; ++i) {
    void* h = dml_host_alloc(slot_bytes);
    hipEvent_t e;
    if (!h || hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      for (void* q : r->host) dml_host_free(q);
      delete r;
      return nullptr;
    }
    r->host.push_back(h);
    r->ev.push_back(e);
  }
  return r;
}
extern "C" void dml_ring_destroy(void* rp) {
  Ring* r = (Ring*)rp;
  if (!r) return;
  for (auto e : r->ev) (void)hipEventSynchronize(e), (void)hipEventDestroy(e);
  for (void* h : r->host) dml_host_free(h);
  delete r;
}
extern "C" void* dml_ring_slot(void* rp, int slot) { return ((Ring*)rp)->host[slot]; }
extern "C" int dml_ring_h2d(void* rp, int slot, void* dst, size_t bytes, hipStream_t cs) {
  Ring* r = (Ring*)rp;
  if (bytes > r->slot_bytes) { g_err = "dml_ring_h2d: bytes > slot"; return -1; }
  HIP_OK(hipMemcpyAsync(dst, r->host[slot], bytes, hipMemcpyHostToDevice, cs));
  HIP_OK(hipEventRecord(r->ev[slot], cs));
  return 0;
}
extern "C" int dml_ring_wait(void* rp, int slot, hipStream_t s) {
  HIP_OK(hipStreamWaitEvent(s, ((Ring*)rp)->ev[slot], 0));
  return 0;
}
extern "C" int dml_ring_sync(void* rp, int slot) {
  HIP_OK(hipEventSynchronize(((Ring*)rp)->ev[slot]));
  return 0;
}
