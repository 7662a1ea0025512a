"""RCCL data plane: batch dispatch and result collection over xGMI.

One process per GPU (rank r <-> GPU r). The coordinator runs on rank 0.

* dispatch  — rank 0 broadcasts a small int64 descriptor table
  ``[world, DESC_FIELDS]`` = (job_id, batch_id, model_id, image_start, count,
  epoch) for every worker; each rank reads its own row. Issued on a dedicated
  (idle) stream so the broadcast never queues behind the previous batch's
  compute — the next batch is dispatched while the current one runs.
  Reference equivalent: the WORKER_TASK_REQUEST UDP datagram carrying image
  names + replica locations (worker.py:297, 428, 480; ~260 B/image, overflows
  the 32 KiB frame at ~122 images — here it is 48 bytes per worker).
* gather    — every rank's packed top-5 result ``[2, B, 5]`` int32 (class ids +
  fp32 probability bits, 40 B/image) is gathered to rank 0 in one collective.
  Reference equivalent: the worker PUTs an indent-4 JSON per batch into SDFS and
  ACKs the leader (worker.py:518-537); the client later merges the JSONs
  (worker.py:1617-1627).

Failure semantics: RCCL is not elastic. The host SWIM detector
(cluster.membership) is the source of truth for liveness; on a membership
change the coordinator bumps ``epoch`` and the communicator is rebuilt over the
survivors (``rebuild``) before the next dispatch.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

DESC_FIELDS = 6  # job_id, batch_id, model_id, image_start, count, epoch
F_JOB, F_BATCH, F_MODEL, F_START, F_COUNT, F_EPOCH = range(DESC_FIELDS)


def init_process_group(backend: Optional[str] = None, timeout_s: int = 600) -> tuple:
    """Initialise torch.distributed from torchrun env (or a 1-rank group).
    Returns (rank, world, local_rank)."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", 0))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if "MASTER_ADDR" not in os.environ:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
    if "MASTER_PORT" not in os.environ:
        import socket

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        kw["device_id"] = torch.device("cuda", local_rank)
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s),
                            **kw)
    return rank, world, local_rank


class DataPlane:
    RING = 3  # descriptor buffers in flight (dispatch lookahead 2 + the one being read)

    def __init__(self, device: torch.device, result_shape=(2, 256, 5), group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device
        self.is_cuda = device.type == "cuda"
        self.dispatch_stream = torch.cuda.Stream(device) if self.is_cuda else None
        self.desc = [torch.zeros((self.world, DESC_FIELDS), dtype=torch.int64, device=device)
                     for _ in range(self.RING)]
        if self.is_cuda:  # pinned staging: table upload and row readback never block the host
            self.host_table = [torch.zeros((self.world, DESC_FIELDS), dtype=torch.int64).pin_memory()
                               for _ in range(self.RING)]
            self.host_row = [torch.zeros(DESC_FIELDS, dtype=torch.int64).pin_memory() for _ in range(self.RING)]
            self.row_ready = [torch.cuda.Event() for _ in range(self.RING)]
        self._next = 0
        self.result_shape = tuple(result_shape)
        self.gather_bufs: List[torch.Tensor] = (
            [torch.empty(self.result_shape, dtype=torch.int32, device=device) for _ in range(self.world)]
            if self.rank == 0 else []
        )
        self.epoch = 0

    # ------------------------------------------------------------ dispatch --
    def issue_dispatch(self, table: Optional[np.ndarray]) -> int:
        """Enqueue the broadcast of rank 0's descriptor table and the readback
        of this rank's row on the dispatch stream; returns a handle for
        ``wait_dispatch``. Nothing here waits on the GPU: the serving pipeline
        issues the table of step k+2 while step k computes, and reads it one step
        later, so the host never blocks behind the forward it just enqueued
        (a blocking read here cost a ~260 us GPU bubble per step,
        profiles/r2_v1/resnet50_kernel_stats.csv trace analysis in DESIGN.md)."""
        h = self._next
        self._next = (self._next + 1) % self.RING
        d = self.desc[h]
        if self.is_cuda:
            with torch.cuda.stream(self.dispatch_stream):
                if self.rank == 0:
                    self.host_table[h].numpy()[...] = np.asarray(table, dtype=np.int64)
                    d.copy_(self.host_table[h], non_blocking=True)
                dist.broadcast(d, src=0, group=self.group)
                self.host_row[h].copy_(d[self.rank], non_blocking=True)
                self.row_ready[h].record(self.dispatch_stream)
        else:
            if self.rank == 0:
                d.copy_(torch.as_tensor(table, dtype=torch.int64))
            dist.broadcast(d, src=0, group=self.group)
        return h

    def wait_dispatch(self, h: int) -> np.ndarray:
        """This rank's row of the dispatch issued as ``h`` (host numpy copy)."""
        if self.is_cuda:
            self.row_ready[h].synchronize()
            return self.host_row[h].numpy().copy()
        return self.desc[h][self.rank].clone().numpy()

    def dispatch(self, table: Optional[np.ndarray]) -> np.ndarray:
        """Broadcast the descriptor table from rank 0; return this rank's row (host)."""
        return self.wait_dispatch(self.issue_dispatch(table))

    # -------------------------------------------------------------- gather --
    def gather(self, result: torch.Tensor) -> Optional[List[torch.Tensor]]:
        """Gather every rank's packed result to rank 0 (enqueued on the current
        stream, after whatever produced `result` there)."""
        assert tuple(result.shape) == self.result_shape, (result.shape, self.result_shape)
        if self.rank == 0:
            dist.gather(result, self.gather_bufs, dst=0, group=self.group)
            return self.gather_bufs
        dist.gather(result, None, dst=0, group=self.group)
        return None

    def barrier(self) -> None:
        if self.is_cuda:
            dist.barrier(group=self.group, device_ids=[self.device.index])
        else:
            dist.barrier(group=self.group)

    def max_over_ranks(self, value: float) -> float:
        t = torch.tensor([value], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def rebuild(self, survivors: List[int]) -> "DataPlane":
        """New epoch: a sub-communicator over the surviving ranks (collective
        over the current group; survivors must all call it)."""
        self.epoch += 1
        grp = dist.new_group(ranks=sorted(survivors))
        dp = DataPlane(self.device, self.result_shape, group=grp)
        dp.epoch = self.epoch
        return dp


def unpack_results(packed: torch.Tensor):
    """[2, B, 5] int32 -> (class ids int32 [B,5], probs fp32 [B,5]) (host numpy)."""
    a = packed.cpu().numpy()
    return a[0], a[1].view(np.float32)
