"""Leader-side store metadata: global file map, replica placement, request
tracking and re-replication planning.

Reference (leader.py:7-181): ``global_file_dict[node][name] = [versions]``;
placement = sha256(name) + random probing until 4 distinct ALIVE nodes — which
loops forever when fewer than 4 are alive (leader.py:60); W = all replicas;
``check_if_request_falied`` compares against the misspelt 'Falied' so failures
were never reported (leader.py:132).

Here: deterministic placement on the sha256-ordered alive ring, bounded by the
number of alive nodes; explicit request states with the failure path working.
"""
from __future__ import annotations

import fnmatch
import hashlib
from typing import Dict, Iterable, List, Optional, Tuple

REPLICATION_FACTOR = 4
WAITING, SUCCESS, FAILED = "Waiting", "Success", "Failed"


class StoreMetadata:
    def __init__(self, replication: int = REPLICATION_FACTOR):
        self.replication = replication
        self.file_map: Dict[str, Dict[str, List[int]]] = {}   # node -> name -> versions
        self.requests: Dict[str, Dict[str, str]] = {}          # name -> node -> status

    # --------------------------------------------------------------- map --
    def set_node_files(self, node: str, files: Dict[str, List[int]]) -> None:
        self.file_map[node] = {k: sorted(int(x) for x in v) for k, v in files.items()}

    def update_node_files(self, node: str, files: Dict[str, List[int]]) -> None:
        """Merge a replica's report about SOME of its files (the names it just stored,
        deleted or re-replicated): name -> its versions there now ([] = gone)."""
        fm = self.file_map.setdefault(node, {})
        for k, v in files.items():
            if v:
                fm[k] = sorted(int(x) for x in v)
            else:
                fm.pop(k, None)

    def remove_node(self, node: str) -> Dict[str, List[int]]:
        return self.file_map.pop(node, {})

    def holders(self, name: str) -> Dict[str, List[int]]:
        return {n: list(f[name]) for n, f in self.file_map.items() if name in f}

    def all_names(self) -> List[str]:
        return sorted({k for f in self.file_map.values() for k in f})

    def matching(self, pattern: str) -> List[str]:
        return [n for n in self.all_names() if fnmatch.fnmatch(n, pattern)]

    def latest_version(self, name: str) -> int:
        vs = [max(v) for v in self.holders(name).values() if v]
        return max(vs) if vs else 0

    # ----------------------------------------------------------- placement --
    def place(self, name: str, alive: Iterable[str], k: Optional[int] = None) -> List[str]:
        """The k replica nodes for a NEW file: consecutive nodes on the alive
        ring starting at sha256(name) (bounded: min(k, #alive))."""
        ring = sorted(alive)
        if not ring:
            return []
        k = min(k or self.replication, len(ring))
        h = int.from_bytes(hashlib.sha256(name.encode()).digest()[:8], "big")
        start = h % len(ring)
        return [ring[(start + i) % len(ring)] for i in range(k)]

    def targets_for_put(self, name: str, alive: Iterable[str]) -> List[str]:
        alive = list(alive)
        cur = [n for n in self.holders(name) if n in alive]
        if cur:
            extra = [n for n in self.place(name, alive, len(alive)) if n not in cur]
            return (cur + extra)[: min(self.replication, len(alive))]
        return self.place(name, alive)

    def under_replicated(self, alive: Iterable[str]) -> List[Tuple[str, str, List[str]]]:
        """[(name, source holder, new nodes)] to restore the replication factor."""
        alive = sorted(alive)
        out = []
        for name in self.all_names():
            hs = [n for n in self.holders(name) if n in alive]
            want = min(self.replication, len(alive))
            if hs and len(hs) < want:
                cands = [n for n in self.place(name, alive, len(alive)) if n not in hs]
                out.append((name, hs[0], cands[: want - len(hs)]))
        return out

    # ------------------------------------------------------------ requests --
    def begin(self, name: str, nodes: Iterable[str]) -> bool:
        if self.in_progress(name):
            return False
        self.requests[name] = {n: WAITING for n in nodes}
        return True

    def in_progress(self, name: str) -> bool:
        st = self.requests.get(name)
        return st is not None and any(v == WAITING for v in st.values())

    def update(self, name: str, node: str, ok: bool) -> Optional[str]:
        """Record one replica's outcome; return SUCCESS/FAILED once decided (W = all)."""
        st = self.requests.get(name)
        if st is None or node not in st:
            return None
        st[node] = SUCCESS if ok else FAILED
        if any(v == FAILED for v in st.values()):
            return FAILED
        if all(v == SUCCESS for v in st.values()):
            return SUCCESS
        return None

    def finish(self, name: str) -> None:
        self.requests.pop(name, None)

    def replace_node_in_requests(self, dead: str, alive: Iterable[str]) -> List[Tuple[str, str]]:
        """In-flight PUTs waiting on a dead replica: pick a substitute
        (the reference's condition was inverted so it never re-routed, worker.py:1264)."""
        out = []
        alive = list(alive)
        for name, st in self.requests.items():
            if st.get(dead) == WAITING:
                del st[dead]
                cands = [n for n in self.place(name, alive, len(alive)) if n not in st]
                if cands:
                    st[cands[0]] = WAITING
                    out.append((name, cands[0]))
        return out
