"""HBM-bound 1x1 convs of ResNet50 (128-image sub-batch) vs a plain device copy
moving the same bytes: how close the conv kernel gets to the achievable
streaming rate. Writes gpurun_out/bw_probe.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402
from distributed_machine_learning_amd.ops import tuning  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    N.ensure_device_init()
    flush = torch.empty(512 * 1024 * 1024, dtype=torch.uint8, device="cuda")  # > Infinity Cache
    rows = []
    for (n, hw, cin, cout, res) in [(128, 56, 256, 64, False), (128, 56, 64, 256, True), (128, 56, 64, 64, False),
                                    (128, 28, 512, 128, False), (128, 28, 128, 512, True)]:
        x = torch.randn(n, hw, hw, cin, device="cuda").to(torch.bfloat16)
        r = torch.randn(n, hw, hw, cout, device="cuda").to(torch.bfloat16) if res else None
        w = torch.randn(cout, cin, 1, 1) * cin ** -0.5
        wp = ops.pack_weight(w)[0].cuda()
        b = torch.zeros(cout, device="cuda")
        y = torch.empty(n, hw, hw, cout, device="cuda", dtype=torch.bfloat16)
        nbytes = x.numel() * 2 + y.numel() * 2 + (r.numel() * 2 if res else 0)
        best = None
        per = {}
        for cfg in tuning.V2_CFGS:
            if res and cfg in tuning.NO_RES_CFGS:
                continue
            def run():
                flush.zero_()
                ops.conv2d_nhwc(x, wp, b, cout, 1, 1, residual=r, out=y, relu=True, cfg=cfg)
            t = timeit(run) - timeit(lambda: flush.zero_())
            per[cfg] = round(t * 1e3, 1)
            best = min(best or (t, cfg), (t, cfg))
        src = torch.empty(nbytes // 4, dtype=torch.uint8, device="cuda")
        dst = torch.empty_like(src)
        def cp():
            flush.zero_()
            dst.copy_(src)
        tcopy = timeit(cp) - timeit(lambda: flush.zero_())  # copy of half the bytes read + written = nbytes/2 moved
        row = {"shape": f"{hw}x{hw} {cin}->{cout}{' +res' if res else ''}", "MB": round(nbytes / 1e6, 1),
               "conv_us": round(best[0] * 1e3, 1), "cfg": best[1], "conv_TBs": round(nbytes / best[0] / 1e9, 2),
               "copy_TBs": round(nbytes / 2 / tcopy / 1e9, 2), "us_per_cfg": per}
        print(json.dumps(row), flush=True)
        rows.append(row)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(rows, open("gpurun_out/bw_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
