#!/usr/bin/env python3
"""BASELINE configs 4 and 5 on GPUs, standalone: concurrent ResNet50 +
InceptionV3 jobs served by the elastic collective service (one process per GPU,
replicated coordinator, SWIM liveness, fair-share with preemption, outputs
written by the ranks), optionally with injected rank kills. The same run is the
``service`` sub-record of ``bench.py`` (parallel/service_bench.py).

  torchrun --nproc-per-node N tools/serve_bench.py --resnet-images 20480 --inception-images 10240 \\
      [--kill 3:100 --kill 6:200]      # rank 3 dies after 100 completed batches, rank 6 after 200
  python tools/serve_bench.py ...      # N = 1

Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--resnet-images", type=int, default=20480)
    ap.add_argument("--inception-images", type=int, default=10240)
    ap.add_argument("--resnet-batch", type=int, default=256)
    ap.add_argument("--inception-batch", type=int, default=128)
    ap.add_argument("--kill", action="append", default=[],
                    help="rank:batches (the rank exits 17 once that many batches completed; the pass then "
                         "runs in child processes, service_bench.run_in_children)")
    ap.add_argument("--out-dir", default="", help="output files ('' = outputs off)")
    ap.add_argument("--comm", default="gloo", choices=("nccl", "gloo"))
    ap.add_argument("--depth", type=int, default=0, help="0: service.auto_depth")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    from distributed_machine_learning_amd.parallel import service_bench
    from distributed_machine_learning_amd.parallel.dataplane import init_process_group

    rank, world, local = init_process_group(backend="gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    rdzv, port = service_bench.agree(rank)
    dist.destroy_process_group()
    bs = {"ResNet50": a.resnet_batch, "InceptionV3": a.inception_batch}
    kills = service_bench.parse_kills(a.kill)
    if kills:  # a killed rank exits 17: never the launcher's worker itself
        rec = service_bench.run_in_children(rank, world, local, rdzv, port, a.resnet_images, a.inception_images,
                                            bs, kills)
    else:
        rec = service_bench.run(rank, world, dev, rdzv, port, a.resnet_images, a.inception_images, bs,
                                a.out_dir or None, comm=a.comm, depth=a.depth)
    if rank == 0 and rec is not None:
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
