"""C1 / C2 metrics.

Reference (worker.py:989-1001, 1394-1428, 1744-1797):
 * counters on every worker ACK: ``query_count += image_count`` and
   ``query_rate_list.append((t_now, t_now - start_time, image_count))`` where
   ``start_time`` comes from the WORKER's clock (cross-host skew leaks in);
 * C2: per model, samples = batch_time / image_count -> mean, stdev,
   statistics.quantiles(n=4);
 * C1: cumulative query count and "query rate [10 s]" derived from the
   scheduler's predicted rate, not measured.

Here: batch durations are measured on the coordinator's clock (dispatch ->
ACK) plus the worker-reported service time; C1's rate is a true sliding 10 s
window of completed images; C2 adds p50/p90/p99 per-image and per-query
latency next to the reference's mean/stdev/quartiles.
"""
from __future__ import annotations

import statistics
import time
from collections import deque
from dataclasses import dataclass
from typing import Deque, Dict, List, Optional


@dataclass
class BatchRecord:
    t_done: float
    latency: float       # coordinator clock: dispatch -> ACK (a query's latency)
    service: float       # worker-measured compute+IO time for the batch
    images: int


def _pct(xs: List[float], q: float) -> float:
    if not xs:
        return 0.0
    s = sorted(xs)
    k = (len(s) - 1) * q
    lo = int(k)
    hi = min(lo + 1, len(s) - 1)
    return s[lo] + (s[hi] - s[lo]) * (k - lo)


class Metrics:
    def __init__(self, window: float = 10.0, max_records: int = 100000, clock=time.monotonic):
        self.window = window
        self.clock = clock
        self.records: Dict[str, Deque[BatchRecord]] = {}
        self.query_count: Dict[str, int] = {}
        self.max_records = max_records

    def record(self, model: str, latency: float, service: float, images: int, t_done: Optional[float] = None) -> None:
        t = self.clock() if t_done is None else t_done
        dq = self.records.setdefault(model, deque(maxlen=self.max_records))
        dq.append(BatchRecord(t, latency, service, images))
        self.query_count[model] = self.query_count.get(model, 0) + images

    # ------------------------------------------------------------------ C1 --
    def c1(self, now: Optional[float] = None) -> Dict[str, Dict[str, float]]:
        now = self.clock() if now is None else now
        out = {}
        for m, dq in self.records.items():
            recent = sum(r.images for r in dq if now - r.t_done <= self.window)
            out[m] = {"query_count": self.query_count.get(m, 0),
                      f"query_rate_{int(self.window)}s": recent / self.window}
        return out

    # ------------------------------------------------------------------ C2 --
    def c2(self) -> Dict[str, Dict[str, object]]:
        out = {}
        for m, dq in self.records.items():
            per_img = [r.service / r.images for r in dq if r.images]
            lat = [r.latency for r in dq]
            if not per_img:
                continue
            d = {
                "per_image_avg": statistics.fmean(per_img),
                "per_image_std": statistics.stdev(per_img) if len(per_img) > 1 else 0.0,
                "per_image_quartiles": statistics.quantiles(per_img, n=4) if len(per_img) > 1 else [per_img[0]] * 3,
                "per_image_p50": _pct(per_img, 0.5), "per_image_p90": _pct(per_img, 0.9),
                "per_image_p99": _pct(per_img, 0.99),
                "query_latency_p50": _pct(lat, 0.5), "query_latency_p90": _pct(lat, 0.9),
                "query_latency_p99": _pct(lat, 0.99),
                "batches": len(per_img),
            }
            out[m] = d
        return out

    # reference GET_C2_COMMAND_ACK payload keys (worker.py:1044)
    def c2_reference_payload(self) -> dict:
        c2 = self.c2()
        p = {}
        for m, key in (("InceptionV3", "inceptionv3"), ("ResNet50", "resnet50")):
            d = c2.get(m)
            p[f"{key}_avg"] = d["per_image_avg"] if d else 0
            p[f"{key}_std"] = d["per_image_std"] if d else 0
            p[f"{key}_quantiles"] = d["per_image_quartiles"] if d else []
        return p
