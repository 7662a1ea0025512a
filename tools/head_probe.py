"""Isolated time of the classifier head kernels at the bench sub-batch sizes:
softmax+top-5 over 8 split-K fp32 partial slices (ResNet50 128 rows, InceptionV3
64 rows, 1000 classes) and the global average pool."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N  # noqa: E402


def timeit(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return round(best * 1e3, 1)


L = N.lib()
s = N.stream_ptr()
for B in (128, 64):
    for ks in (1, 8):
        parts = torch.randn(ks, B, 1000, device="cuda")
        probs = torch.empty(B, 1000, device="cuda")
        idx = torch.empty(B, 5, device="cuda", dtype=torch.int32)
        p = torch.empty(B, 5, device="cuda")
        t = timeit(lambda: L.dml_softmax_top5_split(C.c_void_p(parts.data_ptr()), B, 1000, 1000, ks, B * 1000,
                                                    C.c_void_p(probs.data_ptr()), C.c_void_p(idx.data_ptr()),
                                                    C.c_void_p(p.data_ptr()), C.c_void_p(s)))
        print(f"softmax_top5 rows {B} nsplit {ks}: {t} us")
    x = torch.randn(B, 7, 7, 2048, device="cuda").to(torch.bfloat16)
    y = torch.empty(B, 2048, device="cuda", dtype=torch.bfloat16)
    print(f"gap {B}x7x7x2048: {timeit(lambda: L.dml_global_avgpool(C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), B, 49, 2048, 2048, C.c_void_p(s)))} us")
