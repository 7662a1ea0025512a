"""Runs each fused stem / conv+pool kernel a few times at the bench sub-batch
sizes (ResNet50 128 images, InceptionV3 64) and prints its time: a short,
deterministic program for rocprofv3 --pmc passes over these kernels.

  python tools/fused_kernels_probe.py [--iters 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_machine_learning_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=5)
args = ap.parse_args()


def bench(name, fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(args.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / args.iters * 1e3:.1f} us", flush=True)


r50 = torch.randint(0, 256, (128, 224, 224, 3), dtype=torch.uint8, device="cuda")
inc = torch.randint(0, 256, (64, 299, 299, 3), dtype=torch.uint8, device="cuda")
w7 = (torch.randn(256, 256, device="cuda") * 0.05).to(torch.bfloat16)
w1 = (torch.randn(256, 64, device="cuda") * 0.1).to(torch.bfloat16)
w2 = (torch.randn(256, 320, device="cuda") * 0.05).to(torch.bfloat16)
w3 = (torch.randn(256, 320, device="cuda") * 0.05).to(torch.bfloat16)
b64 = torch.zeros(64, device="cuda")
b32 = torch.zeros(32, device="cuda")
x3 = torch.rand(64, 147, 147, 32, device="cuda").to(torch.bfloat16)
bench("resnet_stem b128", lambda: ops.resnet_stem(r50, w7, b64))
bench("inception_stem b64", lambda: ops.inception_stem(inc, w1, b32, w2, b32, (299, 299), "tf"))
bench("conv3x3_pool b64", lambda: ops.conv3x3_pool(x3, w3, b64))
