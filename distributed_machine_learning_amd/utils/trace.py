"""Tracing: host spans + HIP-event GPU spans -> Chrome trace JSON.

The reference has no tracing, only ad-hoc wall-clock log lines around the
download and inference phases of a task (worker.py:1357-1359, 1363-1384) and
per-command runtimes (worker.py:673, 1708, 1818, ...). SURVEY §5 asks for
per-stage timestamps (queue wait, H2D, preprocess, forward, gather) with
hipEvent timing and a Chrome-trace export; that is this module.

* Host spans use ``time.perf_counter_ns`` on the thread that opened them.
* GPU spans are a pair of ``torch.cuda.Event(enable_timing=True)`` recorded on
  a stream; they are resolved lazily at export (no host sync on the hot path)
  and placed on the host timeline through one anchor event recorded at
  ``Tracer.__init__`` / first GPU use (``elapsed_time`` is relative between
  events on one device).
* Async spans (``begin_async``/``end_async``) follow one object across
  threads/coroutines, e.g. a batch from dispatch to ACK on the coordinator.

A disabled tracer (the default global one) costs one attribute check per call
site. Enable with ``set_tracer(Tracer())`` or ``DML_TRACE=<path>`` (the file is
written at interpreter exit).
"""
from __future__ import annotations

import atexit
import contextlib
import json
import os
import threading
import time
from typing import Any, Dict, List, Optional, Tuple


class _NullSpan:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NULL = _NullSpan()


class Tracer:
    def __init__(self, enabled: bool = True, process_name: str = "dml", pid: Optional[int] = None):
        self.enabled = enabled
        self.pid = os.getpid() if pid is None else pid
        self.process_name = process_name
        self._t0 = time.perf_counter_ns()
        self._events: List[Dict[str, Any]] = []
        self._gpu: List[Tuple[str, str, Any, Any, str, Dict[str, Any]]] = []
        self._anchor = None          # (event, host ns when recorded)
        self._lock = threading.Lock()
        self._tids: Dict[int, int] = {}
        self._lanes: Dict[str, int] = {}

    # --------------------------------------------------------------- util --
    def _now_us(self) -> float:
        return (time.perf_counter_ns() - self._t0) / 1e3

    def _tid(self) -> int:
        ident = threading.get_ident()
        with self._lock:
            if ident not in self._tids:
                self._tids[ident] = len(self._tids) + 1
            return self._tids[ident]

    def _lane(self, name: str) -> int:
        with self._lock:
            if name not in self._lanes:
                self._lanes[name] = 1000 + len(self._lanes)
            return self._lanes[name]

    def _emit(self, ev: Dict[str, Any]) -> None:
        with self._lock:
            self._events.append(ev)

    # --------------------------------------------------------- host spans --
    @contextlib.contextmanager
    def _span(self, name: str, cat: str, args: Dict[str, Any]):
        t = self._now_us()
        try:
            yield self
        finally:
            self._emit({"name": name, "cat": cat, "ph": "X", "ts": t, "dur": self._now_us() - t,
                        "pid": self.pid, "tid": self._tid(), "args": args})

    def span(self, name: str, cat: str = "host", **args):
        """Context manager timing a host-side region."""
        if not self.enabled:
            return _NULL
        return self._span(name, cat, args)

    def instant(self, name: str, cat: str = "host", **args) -> None:
        if self.enabled:
            self._emit({"name": name, "cat": cat, "ph": "i", "s": "t", "ts": self._now_us(),
                        "pid": self.pid, "tid": self._tid(), "args": args})

    def counter(self, name: str, **values: float) -> None:
        if self.enabled:
            self._emit({"name": name, "ph": "C", "ts": self._now_us(), "pid": self.pid, "args": values})

    def begin_async(self, name: str, key: Any, cat: str = "async", **args) -> None:
        if self.enabled:
            self._emit({"name": name, "cat": cat, "ph": "b", "id": str(key), "ts": self._now_us(),
                        "pid": self.pid, "tid": self._tid(), "args": args})

    def end_async(self, name: str, key: Any, cat: str = "async", **args) -> None:
        if self.enabled:
            self._emit({"name": name, "cat": cat, "ph": "e", "id": str(key), "ts": self._now_us(),
                        "pid": self.pid, "tid": self._tid(), "args": args})

    # ---------------------------------------------------------- GPU spans --
    def _ensure_anchor(self, stream) -> None:
        if self._anchor is None:
            import torch

            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
            ev.synchronize()  # once: pins the GPU clock to the host timeline
            self._anchor = (ev, self._now_us())

    @contextlib.contextmanager
    def _gpu_span(self, name: str, stream, lane: str, args: Dict[str, Any]):
        import torch

        self._ensure_anchor(stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        try:
            yield self
        finally:
            e1.record(stream)
            with self._lock:
                self._gpu.append((name, "gpu", e0, e1, lane, args))

    def gpu_span(self, name: str, stream, lane: Optional[str] = None, **args):
        """Context manager timing the work enqueued on ``stream`` inside it
        (HIP events; resolved at export without stalling the stream)."""
        if not self.enabled:
            return _NULL
        return self._gpu_span(name, stream, lane or f"stream {getattr(stream, 'stream_id', 0)}", args)

    def add_gpu_ops(self, ops: List[Tuple[str, float]], lane: str = "ops", start_us: Optional[float] = None) -> None:
        """Lay out per-op device times (``[(name, ms)]``, e.g. Engine.time_ops)
        back to back on their own lane."""
        if not self.enabled:
            return
        t = self._now_us() if start_us is None else start_us
        tid = self._lane(lane)
        for name, ms in ops:
            self._emit({"name": name, "cat": "op", "ph": "X", "ts": t, "dur": ms * 1e3, "pid": self.pid,
                        "tid": tid, "args": {"ms": ms}})
            t += ms * 1e3

    def _resolve_gpu(self) -> List[Dict[str, Any]]:
        out = []
        if not self._gpu:
            return out
        anchor_ev, anchor_us = self._anchor
        with self._lock:
            pending, self._gpu = self._gpu, []
        for name, cat, e0, e1, lane, args in pending:
            e1.synchronize()
            ts = anchor_us + anchor_ev.elapsed_time(e0) * 1e3
            dur = e0.elapsed_time(e1) * 1e3
            out.append({"name": name, "cat": cat, "ph": "X", "ts": ts, "dur": dur, "pid": self.pid,
                        "tid": self._lane(lane), "args": args})
        return out

    # ------------------------------------------------------------- export --
    def events(self) -> List[Dict[str, Any]]:
        gpu = self._resolve_gpu()
        with self._lock:
            self._events.extend(gpu)
            evs = list(self._events)
        meta = [{"name": "process_name", "ph": "M", "pid": self.pid, "args": {"name": self.process_name}}]
        for ident, tid in self._tids.items():
            meta.append({"name": "thread_name", "ph": "M", "pid": self.pid, "tid": tid,
                         "args": {"name": f"host thread {tid}"}})
        for lane, tid in self._lanes.items():
            meta.append({"name": "thread_name", "ph": "M", "pid": self.pid, "tid": tid, "args": {"name": lane}})
        return meta + sorted(evs, key=lambda e: e.get("ts", 0.0))

    def summary(self) -> Dict[str, Dict[str, float]]:
        """Per span name: count, total and mean duration (ms)."""
        out: Dict[str, Dict[str, float]] = {}
        for e in self.events():
            if e.get("ph") != "X":
                continue
            d = out.setdefault(e["name"], {"count": 0, "total_ms": 0.0})
            d["count"] += 1
            d["total_ms"] += e["dur"] / 1e3
        for d in out.values():
            d["mean_ms"] = d["total_ms"] / d["count"]
        return out

    def export_chrome(self, path: str) -> str:
        """Write a chrome://tracing / Perfetto-loadable JSON file."""
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events(), "displayTimeUnit": "ms"}, f)
        return path


def merge_chrome(paths: List[str], out: str) -> str:
    """Merge per-rank trace files (distinct pids) into one."""
    evs: List[Dict[str, Any]] = []
    for p in paths:
        with open(p) as f:
            evs.extend(json.load(f)["traceEvents"])
    with open(out, "w") as f:
        json.dump({"traceEvents": evs, "displayTimeUnit": "ms"}, f)
    return out


_global = Tracer(enabled=False)


def get_tracer() -> Tracer:
    return _global


def set_tracer(t: Tracer) -> Tracer:
    global _global
    _global = t
    return t


if os.environ.get("DML_TRACE"):
    _path = os.environ["DML_TRACE"]
    set_tracer(Tracer(process_name=f"dml rank {os.environ.get('RANK', '0')}"))
    atexit.register(lambda: _global.export_chrome(_path.replace("{rank}", os.environ.get("RANK", "0"))))
