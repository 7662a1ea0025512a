// host_checks.cpp — host-side checks of the native runtime, built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host code only
// (-Xarch_host -fsanitize=...; GPU sanitizers are not available on this
// pool) and run on a CPU-only machine: every path exercised here is host code
// (plan recording / teardown, argument validation, error plumbing) that must
// not touch the device. tests/test_native_host.py builds and runs it.
#include <cstdio>
#include <cstring>
#include <string>
#include "dml.h"

extern "C" void dml_set_error(const char* msg);

static int failures = 0;
#define CHECK(cond)                                                   \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s (last error: %s)\n", __FILE__, __LINE__, #cond, \
                   dml_last_error());                                 \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

static DmlConvArgs conv_args(int cin, int cout, int kh, int kw) {
  DmlConvArgs a;
  std::memset(&a, 0, sizeof a);
  a.x = (const void*)0x1000; a.w = (const void*)0x2000; a.bias = (const float*)0x3000; a.y = (void*)0x4000;
  a.N = 2; a.H = 14; a.W = 14; a.Cin = cin; a.ldx = cin;
  a.kh = kh; a.kw = kw; a.sh = 1; a.sw = 1; a.ph = kh / 2; a.pw = kw / 2;
  a.Ho = 14; a.Wo = 14; a.Cout = cout; a.K = kh * kw * cin; a.Kpad = (a.K + 63) / 64 * 64;
  a.ldy = cout; a.dh = 1; a.dw = 1;
  return a;
}

int main() {
  // ---- plan recording and teardown (no launches) ----
  for (int rep = 0; rep < 3; ++rep) {
    void* plan = dml_plan_create();
    CHECK(plan != nullptr);
    int n = 0;
    for (int i = 0; i < 500; ++i) {
      DmlConvArgs a = conv_args(64 + 8 * (i % 7), 64 + 64 * (i % 5), 1 + 2 * (i % 2), 1 + 2 * (i % 2));
      const int cfg = dml_plan_add_conv(plan, &a, -1);  // heuristic pick: pure host code
      CHECK(cfg >= 0);
      ++n;
      DmlPoolArgs p;
      std::memset(&p, 0, sizeof p);
      p.N = 2; p.H = 14; p.W = 14; p.C = 64; p.ldx = 64; p.Ho = 7; p.Wo = 7; p.ldy = 64; p.k = 3; p.stride = 2;
      CHECK(dml_plan_add_pool(plan, &p) == 0);
      ++n;
    }
    CHECK(dml_plan_add_gap(plan, (void*)0x10, (void*)0x20, 2, 49, 2048, 2048) == 0);
    CHECK(dml_plan_add_softmax_top5_split(plan, (float*)0x30, 2, 1000, 1000, 8, 2000, nullptr, (int*)0x40,
                                          (float*)0x50) == 0);
    DmlPreprocArgs pr;
    std::memset(&pr, 0, sizeof pr);
    CHECK(dml_plan_add_preprocess(plan, &pr) == 0);
    DmlStemArgs st;
    std::memset(&st, 0, sizeof st);
    CHECK(dml_plan_add_stem(plan, &st) == 0);
    DmlIncStemArgs ist;
    std::memset(&ist, 0, sizeof ist);
    CHECK(dml_plan_add_inc_stem(plan, &ist) == 0);
    DmlConvPoolArgs cp;
    std::memset(&cp, 0, sizeof cp);
    CHECK(dml_plan_add_conv_pool(plan, &cp) == 0);
    DmlExpandReduceArgs er;
    std::memset(&er, 0, sizeof er);
    CHECK(dml_plan_add_expand_reduce(plan, &er) == 0);
    DmlConvGroupArgs grp;
    std::memset(&grp, 0, sizeof grp);
    grp.n = 3;
    grp.a[0] = conv_args(64, 96, 5, 5);
    grp.a[1] = conv_args(64, 96, 3, 3);
    grp.a[2] = conv_args(64, 64, 1, 1);
    CHECK(dml_plan_add_conv_group(plan, &grp, 14) == 14);
    CHECK(dml_plan_add_conv_group(plan, &grp, 10) != 0);   // no grouped instantiation of tile 10
    CHECK(std::string(dml_last_error()).find("grouped") != std::string::npos);
    n += 8;
    CHECK(dml_plan_size(plan) == n);
    // error paths that must return before any device call
    CHECK(dml_plan_replay(plan, nullptr) != 0);
    CHECK(std::string(dml_last_error()).find("not captured") != std::string::npos);
    CHECK(dml_plan_replay_part(plan, 0, nullptr) != 0);
    CHECK(dml_plan_replay_part(plan, -1, nullptr) != 0);
    int bad[2] = {5, 2};
    CHECK(dml_plan_capture_parts(plan, bad, 1, nullptr) != 0);
    int oob[2] = {0, n + 1};
    CHECK(dml_plan_capture_parts(plan, oob, 1, nullptr) != 0);
    dml_plan_destroy(plan);
  }

  // ---- launch-argument validation (rejected on the host) ----
  DmlConvArgs a = conv_args(3, 64, 3, 3);  // Cin % 8 != 0 is illegal for every config
  CHECK(dml_conv(&a, 11, nullptr) != 0);
  CHECK(dml_conv(&a, 0, nullptr) != 0);
  a = conv_args(64, 64, 3, 3);
  CHECK(dml_conv(&a, 99, nullptr) != 0);        // unknown config
  CHECK(dml_conv(&a, 35, nullptr) != 0);        // an unassigned id inside 10..63
  CHECK(dml_conv(&a, 90, nullptr) != 0);        // past the table
  CHECK(std::string(dml_last_error()).find("tile config") != std::string::npos);
  CHECK(dml_conv_v2_bn(64) == 0 && dml_conv_v2_bn(68) == 0);   // the removed shifted-pixel ids
  CHECK(dml_conv(&a, 64, nullptr) != 0);
  CHECK(dml_conv(&a, 80, nullptr) != 0);        // the removed Winograd ids
  CHECK(dml_conv(&a, 99, nullptr) != 0);        // an unassigned id
  CHECK(dml_conv(&a, 139, nullptr) != 0);       // an unassigned persistent id
  CHECK(std::string(dml_last_error()).find("tile config") != std::string::npos);
  CHECK(dml_conv_v2_bn(100) == 128 && dml_conv_v2_bn(103) == 64 && dml_conv_v2_bn(120) == 64 &&
        dml_conv_v2_bn(122) == 128);
  // row-ring 3x3 kernel (conv_rowring.hip): ResNet50 stage 2 only
  CHECK(dml_conv_v2_bn(150) == 64 && dml_conv_v2_bn(152) == 64);
  {
    DmlConvArgs s2 = conv_args(64, 64, 3, 3);
    s2.H = s2.W = s2.Ho = s2.Wo = 56;
    CHECK(dml_conv_rr_fits(&s2) == 1);
    s2.Cout = 48; s2.ldy = 48;
    CHECK(dml_conv_rr_fits(&s2) == 1);
    s2.Cout = 128; s2.ldy = 128;                                      // > 64 output channels: refused
    CHECK(dml_conv_rr_fits(&s2) == 0);
    DmlConvArgs s3 = conv_args(128, 128, 3, 3);                       // stage 3 (28 x 28, Cin 128): refused
    s3.H = s3.W = s3.Ho = s3.Wo = 28;
    CHECK(dml_conv_rr_fits(&s3) == 0);
    CHECK(dml_conv(&s3, 150, nullptr) != 0);
    CHECK(std::string(dml_last_error()).find("dml_conv_rr") != std::string::npos);
  }
  a = conv_args(64, 64, 3, 3);
  a.nseg = 5;
  CHECK(dml_conv(&a, 11, nullptr) != 0);        // too many output segments
  a.nseg = 2;
  CHECK(dml_conv(&a, 0, nullptr) != 0);         // not a tile config
  a = conv_args(64, 64, 1, 1);
  a.ksplit = 4; a.split_ld = 1 << 20;
  CHECK(dml_conv(&a, 14, nullptr) != 0);        // split-K needs fp32 output
  a.out_f32 = 1; a.relu = 1;
  CHECK(dml_conv(&a, 14, nullptr) != 0);        // ... and no ReLU
  a.relu = 0;
  CHECK(dml_conv(&a, 40, nullptr) != 0);        // ... and a tile config
  CHECK(dml_conv(&a, 2, nullptr) != 0);
  a = conv_args(64, 64, 3, 3);
  DmlConvGroupArgs g;
  std::memset(&g, 0, sizeof g);
  CHECK(dml_conv_group(&g, 14, nullptr) != 0);  // no members
  g.n = DML_CONV_GROUP_MAX + 1;
  CHECK(dml_conv_group(&g, 14, nullptr) != 0);  // too many members
  g.n = 2;
  g.a[0] = conv_args(64, 64, 3, 3);
  g.a[1] = conv_args(64, 64, 1, 1);
  g.a[1].res = (const void*)0x100; g.a[1].ldr = 64;
  CHECK(dml_conv_group(&g, 14, nullptr) != 0);  // members are residual-free
  CHECK(std::string(dml_last_error()).find("residual-free") != std::string::npos);
  g.a[1] = conv_args(12, 64, 1, 1);
  CHECK(dml_conv_group(&g, 14, nullptr) != 0);  // every member passes dml_conv's validation
  g.a[1] = conv_args(64, 64, 1, 1);
  g.npool = 3;
  CHECK(dml_conv_group(&g, 14, nullptr) != 0);  // at most DML_GROUP_POOL_MAX pools
  g.npool = 1;
  g.pool[0].N = 2; g.pool[0].H = 14; g.pool[0].W = 14; g.pool[0].C = 64; g.pool[0].ldx = 64;
  g.pool[0].Ho = 14; g.pool[0].Wo = 14; g.pool[0].ldy = 64; g.pool[0].k = 5; g.pool[0].stride = 1; g.pool[0].pad = 2;
  CHECK(dml_conv_group(&g, 14, nullptr) != 0);  // pool members: 3x3, pad <= 1
  CHECK(std::string(dml_last_error()).find("pool members") != std::string::npos);
  a = conv_args(8, 64, 3, 3);
  CHECK(dml_conv_pick_cfg(&a) == 15);
  a = conv_args(3, 64, 3, 3);
  CHECK(dml_conv_pick_cfg(&a) == -1);           // nothing can run Cin % 8 != 0
  DmlPoolArgs p;
  std::memset(&p, 0, sizeof p);
  p.C = 12; p.ldx = 12; p.ldy = 12;
  CHECK(dml_pool(&p, nullptr) != 0);
  CHECK(dml_global_avgpool(nullptr, nullptr, 1, 1, 12, 12, nullptr) != 0);
  CHECK(dml_softmax_top5_split(nullptr, 1, 4096, 4096, 1, 0, nullptr, nullptr, nullptr, nullptr) != 0);
  // fused stem: only conv 7x7/2 pad 3 + pool 3x3/2 pad 1 geometry, K >= 224, 64 channels
  DmlStemArgs st;
  std::memset(&st, 0, sizeof st);
  st.N = 1; st.Hs = 224; st.Ws = 224; st.H = 224; st.W = 224; st.ldw = 256;
  st.Hc = 112; st.Wc = 112; st.Ho = 56; st.Wo = 56; st.ldy = 64;
  st.ldw = 128;
  CHECK(dml_stem_resnet(&st, nullptr) != 0);    // weights shorter than K = 224
  st.ldw = 256; st.Ho = 55;
  CHECK(dml_stem_resnet(&st, nullptr) != 0);    // pool size not 3x3/2 pad 1 of the conv
  st.Ho = 56; st.Hc = 111;
  CHECK(dml_stem_resnet(&st, nullptr) != 0);    // conv size not 7x7/2 pad 3 of the input
  CHECK(std::string(dml_last_error()).find("unsupported shape") != std::string::npos);
  DmlIncStemArgs ist;
  std::memset(&ist, 0, sizeof ist);
  ist.N = 1; ist.Hs = 299; ist.Ws = 299; ist.H = 299; ist.W = 299; ist.ldw1 = 64; ist.ldw2 = 320;
  ist.H1 = 149; ist.W1 = 149; ist.H2 = 147; ist.W2 = 147; ist.ldy = 32;
  ist.ldw2 = 256;
  CHECK(dml_stem_inception(&ist, nullptr) != 0);  // conv2 weights shorter than K = 288
  ist.ldw2 = 320; ist.H2 = 149;
  CHECK(dml_stem_inception(&ist, nullptr) != 0);  // conv2 size not 3x3 valid of conv1
  DmlConvPoolArgs cp;
  std::memset(&cp, 0, sizeof cp);
  cp.N = 1; cp.H = 147; cp.W = 147; cp.ldx = 32; cp.ldw = 320; cp.Ho = 73; cp.Wo = 73; cp.ldy = 64;
  cp.ldx = 16;
  CHECK(dml_conv3x3_pool(&cp, nullptr) != 0);     // fewer than 32 input channels
  cp.ldx = 32; cp.Wo = 74;
  CHECK(dml_conv3x3_pool(&cp, nullptr) != 0);     // pool size not 3x3/2 valid of the conv
  DmlExpandReduceArgs er;
  std::memset(&er, 0, sizeof er);
  er.C = 128;
  er.M = 100; er.ldx = 64; er.ldw3 = 64; er.ldr = 256; er.ldy = 256; er.ldw1 = 256; er.ldz = 64;
  CHECK(dml_expand_reduce(&er, nullptr) != 0);    // expand width not 256 / 512 / 1024
  er.C = 256;
  er.M = 100; er.ldx = 64; er.ldw3 = 64; er.ldr = 256; er.ldy = 256; er.ldw1 = 256; er.ldz = 64;
  er.ldw1 = 128;
  CHECK(dml_expand_reduce(&er, nullptr) != 0);    // reduce weights shorter than K = 256
  er.ldw1 = 256; er.ldr = 64;
  CHECK(dml_expand_reduce(&er, nullptr) != 0);    // shortcut narrower than 256 channels
  er.ldr = 256; er.fz = 96; er.ldz = 128;
  er.res = (const void*)&er;                       // a shortcut (never dereferenced by the checks)
  CHECK(dml_chain_supported(&er) == 0);            // stage-end reduce width: 128 only
  CHECK(dml_expand_reduce(&er, nullptr) != 0);    // ... so dml_expand_reduce refuses it
  er.fz = 128;
  CHECK(dml_chain_supported(&er) == 1);            // 64 -> 256 (+ shortcut) -> 128
  er.ldz = 64;
  CHECK(dml_chain_supported(&er) == 0);            // Z rows narrower than the reduce width
  er.fz = 0; er.ldz = 64; er.res = nullptr;
  {  // tile-config ids: dml_conv refuses what no config serves
    DmlConvArgs w{};
    char buf[64];
    w.x = buf; w.y = buf; w.N = 2; w.H = w.W = 14; w.Cin = 64; w.ldx = 64; w.kh = w.kw = 3; w.sh = w.sw = 1;
    w.ph = w.pw = 1; w.Ho = w.Wo = 14; w.Cout = 64; w.ldy = 64; w.K = 576; w.Kpad = 576;
    CHECK(dml_conv(&w, 80, nullptr) != 0);                     // the removed Winograd ids are no config
    CHECK(std::string(dml_last_error()).find("tile config") != std::string::npos);
    CHECK(dml_conv_v2_bn(80) == 0 && dml_conv_v2_bn(15) == 64 && dml_conv_v2_bn(9) == 0);
  }
  dml_set_error(nullptr);
  CHECK(std::string(dml_last_error()).empty());

  if (failures) {
    std::fprintf(stderr, "%d host check(s) failed\n", failures);
    return 1;
  }
  std::printf("host checks passed\n");
  return 0;
}
