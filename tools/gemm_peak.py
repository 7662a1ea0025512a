"""Mainloop ceiling of the implicit-GEMM conv kernel: a large 1x1 conv (a plain
GEMM, M = 65536 pixels, N = K = 4096) on every tile config vs torch.matmul
(hipBLASLt) of the same bf16 GEMM, random data. Separates the kernel's MFMA
pipeline efficiency from the shape / fill effects of the real layers."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402


def timeit(fn, iters=10):
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
    out = []
    for (n, hw, K, Co) in [(16, 64, 4096, 4096), (16, 64, 1152, 128), (16, 64, 2304, 256), (64, 28, 1152, 128)]:
        M = n * hw * hw
        x = torch.randn(n, hw, hw, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(Co, K, 1, 1) * K ** -0.5
        wp = ops.pack_weight(w)[0].cuda()
        b = torch.zeros(Co, device="cuda")
        flop = 2.0 * M * K * Co
        row = {"M": M, "N": Co, "K": K}
        for cfg in (10, 11, 13, 16, 17, 21, 28, 29, 30, 31, 34):
            try:
                y = torch.empty(n, hw, hw, Co, device="cuda", dtype=torch.bfloat16)
                ms = timeit(lambda: ops.conv2d_nhwc(x, wp, b, Co, 1, 1, out=y, cfg=cfg))
                row[f"cfg{cfg}_tflops"] = round(flop / ms / 1e9, 1)
            except N.NativeError as e:
                row[f"cfg{cfg}_tflops"] = None
        a2 = x.view(M, K)
        w2 = wp[:Co, :K].contiguous()
        ms = timeit(lambda: torch.matmul(a2, w2.t()))
        row["hipblaslt_tflops"] = round(flop / ms / 1e9, 1)
        print(json.dumps(row), flush=True)
        out.append(row)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/gemm_peak.json", "w"), indent=1)


if __name__ == "__main__":
    main()
