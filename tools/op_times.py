"""Per-op device times (best of 5 timed passes) of one sub-batch forward at the
bench configuration (ResNet50 128 images, InceptionV3 64 images), in the format
of ``bench.py --op-times`` (input of tools/roofline.py).

python tools/op_times.py --out-dir gpurun_out/ops
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd.models import build_model  # noqa: E402
from distributed_machine_learning_amd.models.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out-dir", default="gpurun_out/ops")
    ap.add_argument("--passes", type=int, default=5)
    ap.add_argument("--runs", default="ResNet50:128,InceptionV3:64",
                    help="model:batch list, e.g. InceptionV3:64,InceptionV3:128")
    a = ap.parse_args()
    os.makedirs(a.out_dir, exist_ok=True)
    for run in a.runs.split(","):
        model, batch = run.split(":")[0], int(run.split(":")[1])
        g, w = build_model(model, seed=0, calibrate=False)
        eng = Engine(g, w, batch=batch)
        eng.run()
        torch.cuda.synchronize()
        best = None
        for _ in range(a.passes):
            t = eng.time_ops()
            best = t if best is None else [(n, min(x, y)) for (n, x), (_, y) in zip(best, t)]
        rec = {"model": model, "batch": batch, "ops": best, "cfg": eng.op_cfg,
               "total_ms": sum(t for _, t in best)}
        with open(os.path.join(a.out_dir, f"op_times_{model}_b{batch}.json"), "w") as f:
            json.dump(rec, f, indent=1)
        print(model, batch, "ops", len(best), "total_ms", round(rec["total_ms"], 3), flush=True)
        del eng


if __name__ == "__main__":
    main()
