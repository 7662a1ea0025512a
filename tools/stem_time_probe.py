import os, sys, json, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from distributed_machine_learning_amd import ops
B = 128
imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda")
wp = torch.randn(256, 256, device="cuda").to(torch.bfloat16)
b = torch.zeros(64, device="cuda")
for _ in range(3): ops.resnet_stem(imgs, wp, b)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
e0.record()
for _ in range(20): ops.resnet_stem(imgs, wp, b)
e1.record(); torch.cuda.synchronize()
print(os.environ.get("DML_LIB"), round(e0.elapsed_time(e1) / 20 * 1000, 1), "us")
