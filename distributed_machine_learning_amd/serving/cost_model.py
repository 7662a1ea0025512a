"""Per-batch cost model used by the fair-share scheduler.

Reference (models.py:128-139, worker.py:57-84): a static model
``time(batch) = download*b + load + first + each*(b-1)`` with constants from
test.py notes — Inception (1, 5.6, 2, 0.325), ResNet (1, 3.5, 1, 0.25) —
and ``SET_BATCH_SIZE`` recomputing ResNet's time with Inception's parameters
(worker.py:1035 defect).

Here: the static model is kept as the prior, and replaced online by an EWMA of
MEASURED batch service times per (model, batch size) reported by workers.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Tuple


@dataclass
class ModelParameters:
    download_time: float
    model_load_time: float
    first_image_predict_time: float
    each_image_predict_time: float
    batch_size: int = 10

    def execution_time_per_vm(self, batch_size: int = None) -> float:
        b = self.batch_size if batch_size is None else batch_size
        return (self.download_time * b + self.model_load_time + self.first_image_predict_time
                + self.each_image_predict_time * (b - 1))


REFERENCE_PARAMS = {
    "InceptionV3": ModelParameters(1.0, 5.6, 2.0, 0.325),
    "ResNet50": ModelParameters(1.0, 3.5, 1.0, 0.25),
}


class CostModel:
    def __init__(self, prior: Dict[str, ModelParameters] = None, alpha: float = 0.3):
        self.prior = dict(prior or REFERENCE_PARAMS)
        self.alpha = alpha
        self.measured: Dict[Tuple[str, int], float] = {}

    def observe(self, model: str, batch_size: int, seconds: float) -> None:
        k = (model, batch_size)
        old = self.measured.get(k)
        self.measured[k] = seconds if old is None else (1 - self.alpha) * old + self.alpha * seconds

    def batch_time(self, model: str, batch_size: int) -> float:
        m = self.measured.get((model, batch_size))
        if m is not None:
            return m
        # scale a measurement at another batch size linearly before falling back to the prior
        others = [(b, t) for (mm, b), t in self.measured.items() if mm == model]
        if others:
            b, t = max(others)
            return t * batch_size / b
        prior = self.prior[model].execution_time_per_vm(batch_size)
        # no measurement for this model yet: scale its prior by how far the
        # measured models deviate from theirs (keeps the two models' rates
        # comparable when one runs on GPUs and the prior is CPU-VM seconds)
        ratios = [t / self.prior[mm].execution_time_per_vm(b) for (mm, b), t in self.measured.items()
                  if mm in self.prior]
        if ratios:
            return prior * sorted(ratios)[len(ratios) // 2]
        return prior

    def rate_per_worker(self, model: str, batch_size: int) -> float:
        """images / s one worker sustains."""
        return batch_size / self.batch_time(model, batch_size)
