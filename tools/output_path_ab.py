#!/usr/bin/env python3
"""where should a batch's output file be rendered at world 8 - on the rank
that ran it (the product: parallel/service.OutputWriter, then a bundled PUT into the replicated
store), or on the coordinator after an RCCL gather of the packed top-5 (40 B per image over
xGMI)? The gather itself is ~10 KB per b256 batch, nothing for xGMI; the question is the host
work that would then land on ONE process: rendering 8 x 360 b256 documents/s (~169 KB each)
plus initiating every PUT. This measures the native renderer (serving/output.BatchRenderer,
byte-identical to the reference's json.dump(indent=4)) per batch on 1..T threads (its ctypes
call releases the GIL) and prints the coordinator-centric capacity against the requirement.

  python tools/output_path_ab.py [--world 8] [--rate 360] [--threads 4] [--out f.json]
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from distributed_machine_learning_amd.serving.output import BatchRenderer  # noqa: E402


def rate(r: BatchRenderer, threads: int, seconds: float = 2.0) -> float:
    rng = np.random.default_rng(0)
    names = [f"synthetic:{i}" for i in range(256)]
    idx = rng.integers(0, 1000, (256, 5)).astype(np.int32)
    p = rng.random((256, 5)).astype(np.float32)
    r.render(names, idx, p)
    done = [0] * threads
    stop = time.perf_counter() + seconds

    def work(k):
        while time.perf_counter() < stop:
            r.render(names, idx, p)
            done[k] += 1
    ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return sum(done) / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rate", type=float, default=360.0, help="b256 batches/s per rank (one MI355X)")
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    r = BatchRenderer()
    need = a.world * a.rate
    res = {"renderer_native": r.native, "required_batches_per_s_world": need,
           "per_rank_required": a.rate, "render_batches_per_s": {}}
    for t in range(1, a.threads + 1):
        res["render_batches_per_s"][t] = round(rate(r, t), 1)
    one = res["render_batches_per_s"][1]
    res["coordinator_centric_margin_1_thread"] = round(one / need, 3)
    res["per_rank_render_share_of_one_thread"] = round(a.rate / one, 3)
    res["verdict"] = ("per-rank rendering: each rank renders only its own batches; the coordinator-centric "
                      "design needs %.2fx one thread's render rate on one process before any PUT" % (need / one))
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
