"""Append-only job journal for coordinator restart (SURVEY §5 checkpoint/resume).

The reference keeps job state in memory only; its sole durability is the H2
standby's partial mirror (worker.py:887-897, 965-985), so losing H1 and H2
together lost every queued job. Here the active coordinator writes every state
transition it relays to the standby (submit, dispatch, requeue, complete,
batch_size) as one JSON line; a coordinator started on the same journal
replays it through the standby-mirror apply path and resumes the queues.
In-progress batches at the crash are requeued at the front (at-least-once, as
after a standby takeover; a late ACK of such a batch is dropped as stale by
``JobManager.complete``).

Compaction: ``compact(snapshot)`` rewrites the file as one ``snapshot`` line
(``JobManager.snapshot()``) so the journal stays O(live state).
"""
from __future__ import annotations

import json
import os
import threading
from typing import Callable, Iterator, Optional


class JobJournal:
    def __init__(self, path: str, fsync: bool = False, compact_every: int = 10000):
        self.path = path
        self.fsync = fsync
        self.compact_every = compact_every
        self.appended = 0
        self._lock = threading.Lock()
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._f = open(path, "a", encoding="utf-8")

    def append(self, op: str, **kw) -> None:
        line = json.dumps({"op": op, **kw}, separators=(",", ":"))
        with self._lock:
            self._f.write(line + "\n")
            self._f.flush()
            if self.fsync:
                os.fsync(self._f.fileno())
            self.appended += 1

    def entries(self) -> Iterator[dict]:
        """Every well-formed line (a torn last line from a crash is skipped)."""
        try:
            with open(self.path, encoding="utf-8") as f:
                for line in f:
                    line = line.strip()
                    if not line:
                        continue
                    try:
                        yield json.loads(line)
                    except ValueError:
                        continue
        except FileNotFoundError:
            return

    def replay(self, apply: Callable[[dict], None]) -> int:
        n = 0
        for e in self.entries():
            apply(e)
            n += 1
        return n

    def compact(self, snapshot: dict) -> None:
        tmp = f"{self.path}.tmp"
        with self._lock:
            with open(tmp, "w", encoding="utf-8") as f:
                f.write(json.dumps({"op": "snapshot", "state": snapshot}, separators=(",", ":")) + "\n")
                f.flush()
                os.fsync(f.fileno())
            self._f.close()
            os.replace(tmp, self.path)
            self._f = open(self.path, "a", encoding="utf-8")
            self.appended = 0

    def maybe_compact(self, snapshot_fn: Callable[[], dict]) -> bool:
        if self.appended >= self.compact_every:
            self.compact(snapshot_fn())
            return True
        return False

    def close(self) -> None:
        with self._lock:
            if not self._f.closed:
                self._f.close()


def open_journal(path: Optional[str], **kw) -> Optional[JobJournal]:
    return JobJournal(path, **kw) if path else None
