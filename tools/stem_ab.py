"""Time the fused stem kernels alone at the bench sub-batch sizes (ResNet50 128
images 224x224, InceptionV3 64 images 299x299, identity resize): run once with
the default library and once with DML_LIB=<variant .so> for an A/B."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402


def timeit(fn, iters=30):
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
    return best * 1e3


N.ensure_device_init()
g = torch.Generator().manual_seed(0)
x = torch.randint(0, 256, (128, 224, 224, 3), dtype=torch.uint8, generator=g).cuda()
w = (torch.randn(64, 224) * 0.05).to(torch.bfloat16).cuda()
b = torch.zeros(64)
print("resnet_stem_us", round(timeit(lambda: ops.resnet_stem(x, w, b)), 1))
xi = torch.randint(0, 256, (64, 299, 299, 3), dtype=torch.uint8, generator=g).cuda()
w1 = (torch.randn(32, 64) * 0.05).to(torch.bfloat16).cuda()
w2 = (torch.randn(32, 288) * 0.05).to(torch.bfloat16).cuda()
print("inception_stem_us", round(timeit(lambda: ops.inception_stem(xi, w1, torch.zeros(32), w2, torch.zeros(32))), 1))
