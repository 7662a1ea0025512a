"""Practical HBM bandwidth ceilings on this GPU (torch kernels, 1 GiB tensors):
copy (read+write), read-only reduction, write-only fill. Prints TB/s."""
import json
import sys

import torch

n = (1 << 30) // 2
a = torch.randn(n, device="cuda").to(torch.bfloat16)
b = torch.empty_like(a)


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters / 1e3


res = {"copy_TBps": 2 * a.numel() * 2 / t(lambda: b.copy_(a)) / 1e12,
       "read_TBps": a.numel() * 2 / t(lambda: a.sum(dtype=torch.float32)) / 1e12,
       "write_TBps": a.numel() * 2 / t(lambda: b.fill_(1.0)) / 1e12}
print(json.dumps({k: round(v, 2) for k, v in res.items()}))
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"))
