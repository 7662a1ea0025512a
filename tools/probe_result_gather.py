#!/usr/bin/env python3
"""GPU probe of the result collect's RCCL branch at world 1 (gloo control group, RCCL data and
result groups): the gather on a side stream, the pinned copy-out and the event the serve loop
polls - the steps of CollectiveService._collect / _drain_gathers, with every exception shown."""
import os
import sys
import tempfile
import time
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_machine_learning_amd.parallel.elastic import ElasticGroup  # noqa: E402


def main():
    rdzv = tempfile.mkdtemp(prefix="dml_probe_")
    dev = torch.device("cuda", 0)
    eg = ElasticGroup(0, 1, store_path=os.path.join(rdzv, "rdzv"), backend="gloo", timeout_s=60,
                      data_backend="nccl", shm_exchange=True)
    print("groups", eg.data_group, eg.result_group, flush=True)
    buf = np.arange(2 * 8 * 10, dtype=np.int32).reshape(2, 8, 10)
    try:
        st = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(st):
            t = torch.from_numpy(buf).to(dev)
            outs = [torch.empty_like(t)]
            w = eg.gather_result_async(t, outs, 0)
            print("issued", w, flush=True)
            w.wait()
            host = torch.empty((1,) + tuple(buf.shape), dtype=torch.int32, pin_memory=True)
            host[0].copy_(outs[0], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        t0 = time.monotonic()
        while not ev.query():
            if time.monotonic() - t0 > 20:
                print("event never completed; work completed:", w.is_completed(), flush=True)
                return 1
            time.sleep(0.001)
        ok = np.array_equal(host.numpy()[0], buf)
        print("gather ok" if ok else "gather WRONG", round(time.monotonic() - t0, 4), "s", flush=True)
        return 0 if ok else 1
    except Exception:
        traceback.print_exc()
        return 1
    finally:
        eg.close()


if __name__ == "__main__":
    sys.exit(main())
