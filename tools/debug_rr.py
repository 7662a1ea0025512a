"""Debug: SplitEngine(splits=4, streams=2) graph vs eager vs per-quarter Engine."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_machine_learning_amd.models import build_model
from distributed_machine_learning_amd.models.engine import Engine, SplitEngine

g, w = build_model("ResNet50", seed=5, calibrate=False)
imgs = torch.randint(0, 256, (8, 224, 224, 3), dtype=torch.uint8, device="cuda")
e2 = Engine(g, w, batch=2)
ref = []
for q in range(4):
    e2.infer(imgs[2 * q: 2 * q + 2]); torch.cuda.synchronize(); ref.append(e2.result.clone())
ref = torch.cat(ref, dim=1)
for streams in (2, 4, 1):
    for use_graph in (False, True):
        se = SplitEngine(g, w, batch=8, splits=4, streams=streams, src_slots=2)
        s = torch.cuda.Stream()
        se.srcs[0].copy_(imgs)
        for rep in range(2):
            with torch.cuda.stream(s):
                se.run(s, use_graph=use_graph, slot=0)
            s.synchronize()
            rows = [bool(torch.equal(se.result[:, r], ref[:, r])) for r in range(8)]
            print(f"streams={streams} graph={use_graph} rep={rep} rows equal: {rows}", flush=True)
            if not all(rows):
                bad = [r for r in range(8) if not rows[r]]
                for r in bad[:2]:
                    print("  got", se.result[0, r].tolist(), "ref", ref[0, r].tolist())
                    lg = se.engines[r // 2].buf[g.logits][r % 2]
                    print("  logits[:4]", lg[:4].tolist())
