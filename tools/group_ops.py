"""Per-op device time of InceptionV3 (batch 64 = one sub-batch of the served
b128) with grouped branch convs vs conv-by-conv: which groups the tuner kept
and what each saves. Writes gpurun_out/groups/ops.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd.models import build_model  # noqa: E402
from distributed_machine_learning_amd.models.engine import Engine  # noqa: E402


def main():
    g, w = build_model("InceptionV3", seed=0, calibrate=False)
    out = {}
    for grouped in (True, False):
        eng = Engine(g, w, batch=64, conv_groups=grouped)
        eng.run()
        torch.cuda.synchronize()
        best = None
        for _ in range(5):
            t = eng.time_ops()
            best = t if best is None else [(n, min(a, b)) for (n, a), (_, b) in zip(best, t)]
        out["grouped" if grouped else "single"] = {"total_ms": sum(t for _, t in best), "ops": best,
                                                   "group_cfg": getattr(eng, "group_cfg", {})}
        del eng
    single = dict(out["single"]["ops"])
    rows = []
    for name, t in out["grouped"]["ops"]:
        if "|" in name:
            alone = sum(single.get(m, 0.0) for m in name.split("|"))
            rows.append((name, t, alone))
            print(f"{name:40s} grouped {t * 1e3:8.1f} us   alone {alone * 1e3:8.1f} us   {alone / t:5.2f}x")
    print("total grouped %.3f ms, single %.3f ms" % (out["grouped"]["total_ms"], out["single"]["total_ms"]))
    out["groups"] = rows
    os.makedirs("gpurun_out/groups", exist_ok=True)
    with open("gpurun_out/groups/ops.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
