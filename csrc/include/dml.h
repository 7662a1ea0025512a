// dml.h — shared declarations for the MI355X-native inference runtime.
//
// Everything here is plain C ABI so the Python side can bind it with ctypes
// (no torch headers, no pybind: the .so is built by one hipcc line in seconds
// and resolves libamdhip64.so.7 to the copy torch already loaded).
//
// Layout conventions (all kernels):
//   activations : NHWC bf16, with an explicit per-pixel channel stride (ld*) so
//                 that Inception's channel concat is a strided write into one
//                 buffer (no concat kernel) and a branch can read a channel slice.
//   weights     : [Cout_pad][K_pad] bf16, K ordered (r, s, c) — one output channel
//                 per row, BatchNorm already folded in on the host.
//   bias        : fp32 [Cout_pad] (folded BN shift / conv bias).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Implicit-GEMM convolution (GEMM view: M = N*Ho*Wo pixels, N = Cout, K = kh*kw*Cin)
// with fused epilogue  y = act(acc + bias[c] (+ res[m, c])).
typedef struct {
  const void* x;      // bf16 NHWC input, already offset to the first input channel
  const void* w;      // bf16 [Coutp][Kpad]
  const float* bias;  // fp32 [Coutp]
  const void* res;    // optional bf16 residual (same pixel grid as y), or null
  void* y;            // output (bf16 or fp32), already offset to the first output channel
  int N, H, W, Cin, ldx;
  int kh, kw, sh, sw, ph, pw;
  int Ho, Wo, Cout, K, Kpad;
  int ldy, ldr;
  int relu, out_f32;
  int dh, dw;         // tap dilation (0 is treated as 1); dw = 2 serves the pair-packed stem
  // Output segments (v2 kernels only): when nseg > 0, output channels
  // [seg_c0[s], seg_c0[s+1]) go to seg_y[s] (+ channel - seg_c0[s]) with row
  // stride seg_ldy[s] and ReLU flag seg_relu[s] — sibling 1x1 convs that read the
  // same input run as ONE GEMM scattering into their own destinations.
  int nseg;
  int seg_c0[4];
  int seg_ldy[4];
  int seg_relu[4];
  void* seg_y[4];
  // Split-K (v2 kernels only; 0/1 = off): the K loop is cut into `ksplit`
  // contiguous ranges, one per workgroup slice; slice s writes its fp32 partial
  // sum to y + s * split_ld (elements) and only slice 0 adds the bias. The
  // consumer sums the slices (dml_softmax_top5_split does, for the classifier).
  int ksplit;
  int split_ld;
  // Subsampled residual (0/1 = off): output pixel
  // (n, ho, wo) adds res pixel n*rHW + (ho*rW + wo)*rsub — the shortcut read at
  // stride rsub from its full-resolution grid (rW = its width, rHW = H*W), used
  // when a stride-2 consumer has been pushed up into the block (models/optimize.py).
  int rsub, rW, rHW;
} DmlConvArgs;



typedef struct {
  const void* x;  // bf16 NHWC
  void* y;        // bf16 NHWC
  int N, H, W, C, ldx;
  int Ho, Wo, ldy;
  int k, stride, pad;  // square window
  int mode;            // 0 = max (padding never wins), 1 = avg with padding excluded from the divisor
  int relu;            // apply ReLU to the pooled value (avg-pool after a pre-pool 1x1 conv)
} DmlPoolArgs;

// Grouped launch (dml_conv_group): up to DML_CONV_GROUP_MAX independent convs
// (residual-free, all on one tile config) and up to DML_GROUP_POOL_MAX
// independent 3x3 pools (pad <= 1) in ONE grid. off[] is filled by the launcher
// (prefix block offsets: convs, then pools; off[n + npool] = grid size).
#define DML_CONV_GROUP_MAX 4
#define DML_GROUP_POOL_MAX 2
typedef struct {
  int n;      // convs (>= 1)
  int npool;  // pools
  int off[DML_CONV_GROUP_MAX + DML_GROUP_POOL_MAX + 1];
  DmlConvArgs a[DML_CONV_GROUP_MAX];
  DmlPoolArgs pool[DML_GROUP_POOL_MAX];
} DmlConvGroupArgs;

typedef struct {
  const void* src;  // uint8 [N][Hs][Ws][3] RGB
  void* y;          // bf16 NHWC, C = 8 (RGB/BGR + 5 zero channels)
  int N, Hs, Ws, Ho, Wo;
  int mode;         // 0 = caffe (BGR, minus ImageNet mean), 1 = tf (x/127.5 - 1)
  int pair;         // 1: channels 4..6 hold the NEXT pixel's 3 values (pair-packed stem input)
  int lpad;         // pair mode: zero columns on the left; output width = Wo + lpad
  const int* idx;   // optional (device memory): image n is src image idx[n] (an arena slot); null: n
} DmlPreprocArgs;

// Fused ResNet50 stem (csrc/kernels/stem_fused.hip): uint8 image -> preprocess ->
// conv 7x7/2 pad 3 (64 ch, folded BN) + ReLU -> max pool 3x3/2 pad 1, one kernel.
typedef struct {
  const void* src;    // uint8 [N][Hs][Ws][3] RGB
  const void* w;      // bf16 [>=64][ldw]: pair-packed 7x7 kernel, K = (row r, pair tap s', 8 ch), 224 used
  const float* bias;  // fp32 [64]
  void* y;            // bf16 NHWC [N][Ho][Wo][ldy] (pooled)
  int N, Hs, Ws;      // source images
  int H, W;           // network input size (nearest resize target)
  int mode;           // 0 = caffe, 1 = tf
  int ldw;
  int Hc, Wc;         // conv output size
  int Ho, Wo, ldy;    // pool output size / channel stride
  // optional folded 1x1 conv on the pooled tile (ResNet50 conv2_block1_1: 64 -> 64 + ReLU, the
  // next op reading exactly the pool output), z = relu(w4 . pool + b4); c4 = 0: off. The pooled
  // tensor y is still written (the merged projection shortcut reads it).
  const void* w4;     // bf16 [>=64][ldw4], K = 64 used
  const float* b4;    // fp32 [64]
  void* z;            // bf16 NHWC [N][Ho][Wo][ldz]
  int c4, ldw4, ldz;
  const int* idx;     // optional (device memory): image n is src image idx[n] (an arena slot); null: n
} DmlStemArgs;

// Fused InceptionV3 stem (csrc/kernels/stem_fused.hip): uint8 image -> preprocess ->
// conv 3x3/2 valid (3 -> 32) + ReLU -> conv 3x3/1 valid (32 -> 32) + ReLU, one kernel.
typedef struct {
  const void* src;     // uint8 [N][Hs][Ws][3] RGB
  const void* w1;      // bf16 [>=32][ldw1]: pair-packed 3x3 kernel, K = (row r, pair tap s', 8 ch), 48 used
  const float* b1;     // fp32 [32]
  const void* w2;      // bf16 [>=32][ldw2]: K = (r, s, 32 ch), 288 used
  const float* b2;     // fp32 [32]
  void* y;             // bf16 NHWC [N][H2][W2][ldy]
  int N, Hs, Ws, H, W, mode;
  int ldw1, ldw2;
  int H1, W1;          // conv1 output size
  int H2, W2, ldy;     // conv2 output size / channel stride
  const int* idx;      // optional (device memory): image n is src image idx[n] (an arena slot); null: n
} DmlIncStemArgs;

// Fused 3x3 'same' conv (32 -> 64 ch, folded BN) + ReLU + 3x3/2 'valid' max pool
// (csrc/kernels/conv_pool.hip; InceptionV3 conv2d_3 + max_pooling2d_1).
typedef struct {
  const void* x;       // bf16 NHWC [N][H][W][ldx] (32 channels used)
  const void* w;       // bf16 [>=64][ldw]: K = (r, s, 32 ch), 288 used
  const float* bias;   // fp32 [64]
  void* y;             // bf16 NHWC [N][Ho][Wo][ldy]
  int N, H, W, ldx, ldw;
  int Ho, Wo, ldy;     // pool output (or, with c4 > 0, the folded 1x1 conv's output)
  // optional folded 1x1 conv on the pooled tile (InceptionV3 conv2d_4: 64 -> 80, ReLU):
  // y = relu(w4 . pool + b4) with c4 output channels (c4 % 16 == 0, <= 128); c4 = 0: off
  const void* w4;      // bf16 [>=c4][ldw4], K = 64 used
  const float* b4;     // fp32 [c4]
  int c4, ldw4;
} DmlConvPoolArgs;

// Fused ResNet50 block boundary (csrc/kernels/expand_reduce_chain.hip), F = C / 4:
//   y = relu(w3 . x + b3 + res)  (1x1 expand F -> C + shortcut)
//   z = relu(w1 . y + b1)        (next block's 1x1 reduce C -> F)
typedef struct {
  const void* x;     // bf16 [M][ldx] (F channels)
  const void* w3;    // bf16 [>=C][ldw3], K = F used
  const float* b3;   // fp32 [C]
  const void* res;   // bf16 [M][ldr] (C channels)
  void* y;           // bf16 [M][ldy] (C channels)
  const void* w1;    // bf16 [>=F][ldw1], K = C used
  const float* b1;   // fp32 [F]
  void* z;           // bf16 [M][ldz] (F channels)
  int M, ldx, ldw3, ldr, ldy, ldw1, ldz;
  int C;             // expand width: 256, 512 or 1024 (reduce width F = C / 4)
  int kx;            // expand K: 0/F with res, 2F with res == null (merged projection shortcut, C = 256)
  // Subsampled Y store (0/1 = off): when Y's only other reader takes every ysub-th
  // pixel (a shortcut after the stride pushdown), pixel (n, h, w) of the yH x yW grid
  // is stored only for h, w % ysub == 0, compactly at n*(yH/ysub)*(yW/ysub) + ...
  int ysub, yH, yW;
  long long* stamps;  // diagnostics only (null in the engine): chained kernel, per workgroup 40 x s_memtime
  // reduce width (0 = F = C / 4). 2F at a stage's last boundary, where the expand's output feeds
  // the next stage's first reduce (ResNet50 conv2_block3_3 -> conv3_block1_1: 256 -> 128;
  // chained kernel only)
  int fz;
} DmlExpandReduceArgs;

// ---- single-op launches (used by tests and by the plan executor) ----
int dml_stem_resnet(const DmlStemArgs* a, hipStream_t s);
int dml_stem_inception(const DmlIncStemArgs* a, hipStream_t s);
int dml_conv3x3_pool(const DmlConvPoolArgs* a, hipStream_t s);
// chained-GEMM block boundary (expand_reduce_chain.hip); dml_expand_reduce is the same entry
int dml_expand_reduce(const DmlExpandReduceArgs* a, hipStream_t s);
int dml_chain(const DmlExpandReduceArgs* a, hipStream_t s);
int dml_chain_supported(const DmlExpandReduceArgs* a);
int dml_chain_init(void);
int dml_expand_reduce_init(void);
int dml_conv(const DmlConvArgs* a, int cfg, hipStream_t s);
int dml_conv_v2(const DmlConvArgs* a, int cfg, hipStream_t s);
int dml_conv_v2_init(void);
int dml_conv_pick_cfg(const DmlConvArgs* a);
int dml_conv_group(const DmlConvGroupArgs* g, int cfg, hipStream_t s);
int dml_conv_v2_group(const DmlConvGroupArgs* g, int cfg, hipStream_t s);
int dml_conv_v2_group_supported(int cfg);
int dml_conv_v2_bn(int cfg);  // channel-tile width of any tile config (v2 or warp-specialised), 0: none
// warp-specialised implicit GEMM (conv_igemm_ws.hip; cfg ids 100..119): loader waves + MFMA waves
int dml_conv_ws(const DmlConvArgs* a, int cfg, hipStream_t s);
int dml_conv_ws_bn(int cfg);
int dml_conv_ws_init(void);
// persistent warp-specialised implicit GEMM (conv_igemm_wsp.hip; cfg ids 120..139): one operand
// ring over each workgroup's whole tile list (no split-K)
int dml_conv_wsp(const DmlConvArgs* a, int cfg, hipStream_t s);
int dml_conv_wsp_bn(int cfg);
int dml_conv_wsp_init(void);
// row-ring 3x3 convolution of ResNet50 stage 2 (conv_rowring.hip; cfg ids 150..152 = 2 / 1 / 4
// strips per image): weights LDS-resident, input rows streamed through a 10-row ring; refuses
// anything but 3x3 pad 1 stride 1, Cin 64, Cout <= 64, width 56
int dml_conv_rr(const DmlConvArgs* a, int cfg, hipStream_t s);
int dml_conv_rr_fits(const DmlConvArgs* a);
int dml_conv_rr_init(void);
int dml_conv_rr_stamped(const DmlConvArgs* a, int cfg, void* stamps, hipStream_t s);  // phase probe
// baseline JPEG decode on the GPU fused with the Pillow-exact nearest resize into arena slots
// (jpeg_decode.hip): host parse + un-stuffing into one buffer, then three kernels
long dml_jpeg_prepare(int n, const unsigned char* const* datas, const long* lens, int outH, int outW, void* buf,
                      long cap, int* status, long* info);
void dml_jpeg_set_slot(void* buf, int i, int slot);
void dml_jpeg_set_slots(void* buf, const int* idx, const int* slots, int n);
int dml_jpeg_decode_resize(const void* dbuf, int n, int maxblk, long maxstream, void* dwork, int H, int W,
                           void* arena, hipStream_t s);
int dml_jpeg_launch(const void* host, void* dev, long used, void* dwork, long coef_bytes, int n, int maxblk,
                    long maxstream, int H, int W, void* arena, hipStream_t s);   // H2D + zero + decode_resize
int dml_jpeg_init(void);
long dml_jpeg_desc_size(void);
long dml_jpeg_head_size(void);
void dml_jpeg_retarget(void* dst, const void* src, int outH, int outW, long base);
void dml_jpeg_retarget_many(void* dst, const void* const* srcs, const long* bases, int n, int outH, int outW);
int dml_jpeg_resize_only(const void* dbuf, int n, int H, int W, void* arena, hipStream_t s);
int dml_jpeg_decode_host(const unsigned char* data, long len, unsigned char* out, int* hw);
int dml_conv_group_validate(const DmlConvGroupArgs* g, int cfg);
int dml_pool(const DmlPoolArgs* a, hipStream_t s);
int dml_global_avgpool(const void* x, void* y, int N, int HW, int C, int ldx, hipStream_t s);
int dml_softmax_top5(const float* logits, int B, int classes, int ld, float* probs_out,
                     int* top_idx, float* top_p, hipStream_t s);
// logits given as `nsplit` fp32 partial slices (split-K classifier): row r of
// slice s at logits + s*split_ld + r*ld; the summed logits are written back to
// slice 0 before the softmax.
int dml_softmax_top5_split(float* logits, int B, int classes, int ld, int nsplit, int split_ld,
                           float* probs_out, int* top_idx, float* top_p, hipStream_t s);
int dml_preprocess(const DmlPreprocArgs* a, hipStream_t s);
int dml_index_fetch(const int* host, int* dev, int n, hipStream_t s);  // pinned host table -> device
// packed full-resolution RGB images -> arena slots, nearest resize (misc.hip resize_nearest_kernel)
int dml_resize_nearest(const void* pack, int n, int H, int W, void* dst, hipStream_t s);

int dml_abi_sizes(int* out, int n);

// ---- plan executor (C++ runtime, csrc/runtime/runtime.hip) ----
void* dml_plan_create(void);
void dml_plan_destroy(void* plan);
int dml_plan_add_conv(void* plan, const DmlConvArgs* a, int cfg);
int dml_plan_add_conv_group(void* plan, const DmlConvGroupArgs* g, int cfg);
int dml_plan_add_pool(void* plan, const DmlPoolArgs* a);
int dml_plan_add_gap(void* plan, const void* x, void* y, int N, int HW, int C, int ldx);
int dml_plan_add_softmax_top5(void* plan, const float* logits, int B, int classes, int ld,
                              float* probs, int* idx, float* p);
int dml_plan_add_softmax_top5_split(void* plan, float* logits, int B, int classes, int ld, int nsplit,
                                    int split_ld, float* probs, int* idx, float* p);
int dml_plan_add_preprocess(void* plan, const DmlPreprocArgs* a);
int dml_plan_add_stem(void* plan, const DmlStemArgs* a);
int dml_plan_add_inc_stem(void* plan, const DmlIncStemArgs* a);
int dml_plan_add_conv_pool(void* plan, const DmlConvPoolArgs* a);
int dml_plan_add_expand_reduce(void* plan, const DmlExpandReduceArgs* a);
int dml_plan_size(void* plan);
int dml_plan_run(void* plan, hipStream_t s);
int dml_plan_run_range(void* plan, int begin, int end, hipStream_t s);
int dml_plan_capture(void* plan, hipStream_t s);   // capture the whole plan into a hipGraph
int dml_plan_replay(void* plan, hipStream_t s);    // launch the captured graph
// capture op ranges [bounds[i], bounds[i+1]) as separate graphs / launch graph i
int dml_plan_capture_parts(void* plan, const int* bounds, int nparts, hipStream_t s);
int dml_plan_replay_part(void* plan, int i, hipStream_t s);
// a batch's event records / stream waits / index fetches / graph replays in one call (5 int64 per op)
int dml_launch_seq(const int64_t* ops, int n);
int dml_plan_time_ops(void* plan, hipStream_t s, float* ms_out, int n);  // per-op hipEvent timing
int dml_plan_set_cfg(void* plan, int i, int cfg);  // re-point conv op i at config cfg; returns the old one
int dml_plan_get_cfg(void* plan, int i);

// ---- pinned-host staging ring (csrc/runtime/staging.cpp) ----
void* dml_ring_create(int slots, size_t slot_bytes);
void dml_ring_destroy(void* ring);
void* dml_ring_slot(void* ring, int slot);
int dml_ring_h2d(void* ring, int slot, void* dst, size_t bytes, hipStream_t copy_stream);
int dml_ring_wait(void* ring, int slot, hipStream_t compute_stream);  // compute waits for copy
int dml_ring_sync(void* ring, int slot);                               // host waits (slot reusable)
void* dml_host_alloc(size_t bytes);
void dml_host_free(void* p);
int dml_memcpy_h2d_async(void* dst, const void* src, size_t bytes, hipStream_t s);
int dml_memcpy_d2h_async(void* dst, const void* src, size_t bytes, hipStream_t s);

const char* dml_last_error(void);
int dml_device_info(int* cus, int* arch_major, int* arch_minor);

#ifdef __cplusplus
}
#endif
