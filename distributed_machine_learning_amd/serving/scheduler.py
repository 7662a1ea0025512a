"""Fair-share, preempting batch scheduler (pure function; the coordinator applies it).

Reference (worker.py:255-495):
 * one model has queued work -> give a queued batch to every free worker;
 * both have work -> over the online workers n, enumerate splits (n-k, k),
   predict each model's rate ``vm_count * batch / time(batch)`` and choose the
   split minimising the % difference between the two rates; fill each model's
   share from free workers first, then STEAL workers running the other model;
   a stolen worker's batch is PREEMPTED back to the front of its queue.
 * ``online`` there was "membership minus H1/H2"; here it is the alive workers.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from .cost_model import CostModel


@dataclass
class Assignment:
    worker: str
    model: str
    preempt: Optional[Tuple[str, tuple]] = None  # (model, batch key) taken off this worker


def best_split(n: int, rate_a: float, rate_b: float) -> Tuple[int, int]:
    """Workers (a, b) with a + b = n, a, b >= 1, minimising |Ra - Rb| / max(Ra, Rb)
    where R = count * per-worker rate (ties -> the first, i.e. most workers to a)."""
    if n < 2:
        return (n, 0)
    best, best_d = (n - 1, 1), float("inf")
    for k in range(1, n):
        ra, rb = (n - k) * rate_a, k * rate_b
        d = abs(ra - rb) / max(ra, rb) * 100.0
        if d < best_d - 1e-12:
            best, best_d = (n - k, k), d
    return best


def plan(queued: Dict[str, int], free: Sequence[str], running: Dict[str, Tuple[str, tuple]],
         online: Sequence[str], cost: CostModel, batch_sizes: Dict[str, int],
         models: Sequence[str] = ("InceptionV3", "ResNet50"), preempt: bool = True) -> List[Assignment]:
    """Decide which worker runs what next.

    queued:  model -> number of queued batches
    free:    idle alive workers
    running: worker -> (model, batch key) currently executing
    online:  all alive workers
    preempt: steal workers running the other model (the reference's policy);
             the collective service's per-rank queues only fill free slots
    """
    free = sorted(free)
    active = [m for m in models if queued.get(m, 0) > 0]
    out: List[Assignment] = []
    if not active:
        return out
    if len(active) == 1:
        m = active[0]
        for w in free[: queued[m]]:
            out.append(Assignment(w, m))
        return out
    a, b = models[0], models[1]
    n = len(online)
    ca, cb = best_split(n, cost.rate_per_worker(a, batch_sizes[a]), cost.rate_per_worker(b, batch_sizes[b]))
    want = {a: ca, b: cb}
    run_by = {m: sorted(w for w, (mm, _) in running.items() if mm == m) for m in models}
    pool = list(free)
    budget = dict(queued)
    for m, other in ((a, b), (b, a)):
        have = len(run_by[m])
        # free workers first
        while have < want[m] and pool and budget[m] > 0:
            out.append(Assignment(pool.pop(), m))
            have += 1
            budget[m] -= 1
        # then steal from the other model's running workers beyond its own share
        while preempt and have < want[m] and budget[m] > 0 and len(run_by[other]) > want[other]:
            w = run_by[other].pop()
            out.append(Assignment(w, m, preempt=(other, running[w][1])))
            have += 1
            budget[m] -= 1
    # leftover free workers: keep them busy with whatever is still queued
    for w in pool:
        for m in sorted(models, key=lambda mm: -budget.get(mm, 0)):
            if budget.get(m, 0) > 0:
                out.append(Assignment(w, m))
                budget[m] -= 1
                break
    return out
