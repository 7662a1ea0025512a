// conv_dispatch.hip — argument validation, dispatch and default tile choice of
// the MFMA implicit-GEMM convolution (the kernel: conv_igemm_v2.hip).
//
// Serves every convolution of ResNet50 / InceptionV3 and the FC layer
// (SURVEY §2.7 "conv_igemm_bf16"; the reference runs these inside Keras,
// models.py:26,51 — it has no kernel of its own). cfg ids 10..63 select a v2
// tile configuration (dml_conv_v2), ids 100..119 a warp-specialised one (loader +
// MFMA waves, dml_conv_ws, conv_igemm_ws.hip), ids 120..139 its persistent form
// (dml_conv_wsp, conv_igemm_wsp.hip), ids 150..152 the row-ring 3x3 kernel of ResNet50 stage 2
// (dml_conv_rr, conv_rowring.hip); they are part of the ABI the plan builder and the
// autotuner (ops/tuning.py) use.
//
// Removed (measured never faster, kept only as history in DESIGN.md and
// profiles/): the register-staged v1 kernel (cfg 0..4, r1, profiles/r1_v2), the
// stride-1 halo-tile kernel (cfg 40..47, r2, profiles/r1_v5/halo_vs_v2_*.json: won
// 0 of 217 tuned shapes), the shifted-pixel stride-1 kernel (cfg 64..69, r4:
// never picked by the cold tuner, profiles/r3_v2/shift_vs_igemm.json) and the
// persistent weight-stationary 1x1 kernel (cfg 84..90, r4, commit f96f4b1: parity at
// best, profiles/r4_probes/ws) and the Winograd F(2x2, 3x3) kernel (cfg 80..83, r4,
// removed in r5: slower than the direct tiles on every shape, profiles/r4_wino) and the
// patch-stationary stride-1 tiles (cfg 140..149, r5: slower on every shape, profiles/r5_ws;
// removed in r6).
#include "common.h"
#include "dml.h"
#include "pool_shared.h"

static int validate(const DmlConvArgs* a, int cfg) {
  const int bn = dml_conv_v2_bn(cfg);
  if (bn <= 0) {
    dml_set_error("dml_conv: cfg must be a tile config (v2: 10..63, warp-specialised: 100..119, persistent: "
                  "120..139, row-ring: 150..152)");
    return -1;
  }
  // weights are packed with Cout padded to a multiple of 256 rows; a 96- or
  // 192-wide channel tile must not run past them
  if ((a->Cout + bn - 1) / bn * bn > (a->Cout + 255) / 256 * 256) {
    dml_set_error("dml_conv: the channel tiles of this cfg overrun the 256-row weight padding");
    return -1;
  }
  if (a->Cin % 8 || a->ldx % 8 || a->Cout % 8 || a->Kpad % 64 || a->ldy % 8 || (a->res && a->ldr % 8)) {
    dml_set_error("dml_conv: need Cin, ldx, Cout, ldy, ldr %8==0 and Kpad%64==0");
    return -1;
  }
  if (a->nseg < 0 || a->nseg > 4) {
    dml_set_error("dml_conv: nseg must be 0..4");
    return -1;
  }
  if (a->rsub > 1 && (!a->res || a->rW < a->Wo * a->rsub || a->rHW < a->rW * a->Ho * a->rsub)) {
    dml_set_error("dml_conv: subsampled residual needs res and rW >= Wo*rsub, rHW >= rW*Ho*rsub");
    return -1;
  }
  if (a->ksplit > 1 && (!a->out_f32 || a->res || a->nseg || a->relu || a->split_ld < 1)) {
    dml_set_error("dml_conv: split-K needs fp32 output, no residual/segments/ReLU, split_ld");
    return -1;
  }
  return 0;
}

extern "C" int dml_conv(const DmlConvArgs* a, int cfg, hipStream_t s) {
  if (validate(a, cfg) != 0) return -1;
  if (cfg >= 150) return dml_conv_rr(a, cfg, s);
  if (cfg >= 120) return dml_conv_wsp(a, cfg, s);
  return cfg >= 100 ? dml_conv_ws(a, cfg, s) : dml_conv_v2(a, cfg, s);
}

extern "C" int dml_conv_group_validate(const DmlConvGroupArgs* g, int cfg) {
  if (!g || g->n < 1 || g->n > DML_CONV_GROUP_MAX || g->npool < 0 || g->npool > DML_GROUP_POOL_MAX) {
    dml_set_error("dml_conv_group: 1..4 convs and 0..2 pools");
    return -1;
  }
  for (int j = 0; j < g->npool; ++j) {
    if (!dml::poolk::pool3x3_fast_ok(g->pool[j])) {
      dml_set_error("dml_conv_group: pool members must be 3x3, pad <= 1, channels %8");
      return -1;
    }
  }
  if (!dml_conv_v2_group_supported(cfg)) {
    dml_set_error("dml_conv_group: cfg has no grouped instantiation (the 4-wave tiles)");
    return -1;
  }
  for (int i = 0; i < g->n; ++i) {
    if (validate(&g->a[i], cfg) != 0) return -1;
    if (g->a[i].res || g->a[i].ksplit > 1) {
      dml_set_error("dml_conv_group: members must be residual-free and without split-K");
      return -1;
    }
  }
  return 0;
}

extern "C" int dml_conv_group(const DmlConvGroupArgs* g, int cfg, hipStream_t s) {
  if (dml_conv_group_validate(g, cfg) != 0) return -1;
  return dml_conv_v2_group(g, cfg, s);
}

// Measured default tile per shape class (tools/conv_bench.py); the engine
// autotunes every shape (ops/tuning.py). -1: no config can run this conv.
extern "C" int dml_conv_pick_cfg(const DmlConvArgs* a) {
  const long M = (long)a->N * a->Ho * a->Wo;
  const int C = a->Cout;
  if (a->Cin % 8 || a->ldx % 8 || C % 8 || a->ldy % 8 || (a->res && a->ldr % 8)) return -1;
  if (C <= 64) return 15;
  if (a->Kpad <= 512 || M < 16384) return 14;
  return 11;
}
