#!/usr/bin/env python3
"""Launch conv shapes of tools/conv_ws_ab.py with given tile configs back to back, warm, for
rocprofv3 counter passes (--pmc + --kernel-trace only): each (shape, cfg) is one kernel
symbol in the trace.

  rocprofv3 --pmc SQ_WAVE_CYCLES ... --kernel-trace -- python3 tools/conv_pmc_run.py \
      --shapes r50_3x3_s4 --cfgs 102,140 --iters 5
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from conv_ws_ab import SHAPES  # noqa: E402
from distributed_machine_learning_amd import _native as N, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="r50_3x3_s4")
    ap.add_argument("--cfgs", default="102,140")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    N.ensure_device_init()
    L, s = N.lib(), N.stream_ptr()
    want = set(a.shapes.split(","))
    for name, B, h, w, cin, cout, kh, kw, st, ph, pw, res in SHAPES:
        if name not in want:
            continue
        ho, wo = (h + 2 * ph - kh) // st + 1, (w + 2 * pw - kw) // st + 1
        x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
        wp, K, kp = ops.pack_weight(torch.randn(cout, cin, kh, kw) * 0.05)
        wp = wp.cuda()
        bias = torch.zeros(wp.shape[0], device="cuda")
        y = torch.empty(B, ho, wo, cout, device="cuda", dtype=torch.bfloat16)
        ar = N.ConvArgs(x.data_ptr(), wp.data_ptr(), bias.data_ptr(), None, y.data_ptr(), B, h, w, cin, cin, kh, kw,
                        st, st, ph, pw, ho, wo, cout, K, kp, cout, 0, 1, 0, 1, 1)
        for cfg in (int(c) for c in a.cfgs.split(",")):
            for _ in range(a.iters):
                if L.dml_conv(C.byref(ar), cfg, C.c_void_p(s)) != 0:
                    print("refused", name, cfg, flush=True)
                    break
            torch.cuda.synchronize()
            print("ran", name, cfg, flush=True)


if __name__ == "__main__":
    main()
