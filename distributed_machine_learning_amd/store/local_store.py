"""Per-node versioned file store (the SDFS replica's local half).

Reference (file_service.py:13-124): files live in SDFS_LOCATION as
``<name>_version<N>`` with at most MAX_FILE_VERSIONS=5 (oldest evicted), the
index is rebuilt from disk at startup, and bytes move by asyncssh scp.
Here bytes move over the blob server (store/blob.py); this class is purely the
on-disk versioned store with an in-memory index, safe for concurrent readers
(writes go to a temp file + atomic rename).
"""
from __future__ import annotations

import fnmatch
import os
import re
import threading
from typing import Dict, List, Optional, Tuple

MAX_FILE_VERSIONS = 5
_VER = re.compile(r"^(?P<name>.+)_version(?P<v>\d+)$")


class LocalFileStore:
    def __init__(self, root: str, max_versions: int = MAX_FILE_VERSIONS):
        self.root = root
        self.max_versions = max_versions
        os.makedirs(root, exist_ok=True)
        self._lock = threading.Lock()
        self.index: Dict[str, List[int]] = {}
        self._load()

    def _load(self) -> None:
        for fn in os.listdir(self.root):
            m = _VER.match(fn)
            if m:
                self.index.setdefault(m.group("name"), []).append(int(m.group("v")))
        for v in self.index.values():
            v.sort()

    def _path(self, name: str, version: int) -> str:
        if "/" in name or name.startswith(".."):
            raise ValueError(f"bad sdfs name {name!r}")
        return os.path.join(self.root, f"{name}_version{version}")

    # ---------------------------------------------------------------- API --
    def put_bytes(self, name: str, data: bytes, version: Optional[int] = None) -> int:
        with self._lock:
            vers = self.index.setdefault(name, [])
            v = version if version is not None else (vers[-1] + 1 if vers else 1)
            path = self._path(name, v)
            tmp = path + ".tmp"
            with open(tmp, "wb") as f:
                f.write(data)
            os.replace(tmp, path)
            if v not in vers:
                vers.append(v)
                vers.sort()
            while len(vers) > self.max_versions:
                old = vers.pop(0)
                try:
                    os.remove(self._path(name, old))
                except FileNotFoundError:
                    pass
            return v

    def put_link(self, name: str, src_path: str, version: Optional[int] = None) -> int:
        """Store ``src_path`` (a file on this filesystem) as a version of ``name`` by a
        hard link: the same-node replica path of a bundle PUT (store/service.py) — the
        bytes were written once by the client into its spool, every replica on the node
        adds a directory entry of its own, and the file lives while any replica keeps it.
        The store never rewrites a file in place (new versions are new files), so
        replicas sharing an inode never see each other's changes."""
        with self._lock:
            vers = self.index.setdefault(name, [])
            v = version if version is not None else (vers[-1] + 1 if vers else 1)
            path = self._path(name, v)
            tmp = path + ".lnk"
            try:
                os.remove(tmp)
            except FileNotFoundError:
                pass
            os.link(src_path, tmp)
            os.replace(tmp, path)
            if v not in vers:
                vers.append(v)
                vers.sort()
            while len(vers) > self.max_versions:
                old = vers.pop(0)
                try:
                    os.remove(self._path(name, old))
                except FileNotFoundError:
                    pass
            return v

    def put_links(self, items: List[Tuple[str, str, Optional[int]]]) -> Dict[str, int]:
        """put_link for a whole bundle: every link made by ONE native call (store/fastio.py)
        instead of three Python syscalls per file. Returns name -> stored version; a file whose
        link failed is missing from the result."""
        from .fastio import link_many

        with self._lock:
            plan = []
            for name, src, version in items:
                vers = self.index.setdefault(name, [])
                v = version if version is not None else (vers[-1] + 1 if vers else 1)
                plan.append((name, src, v, self._path(name, v)))
            st = link_many([(src, path) for _, src, _, path in plan])
            out: Dict[str, int] = {}
            for (name, _, v, _), rc in zip(plan, st):
                if rc != 0:
                    continue
                vers = self.index[name]
                if v not in vers:
                    vers.append(v)
                    vers.sort()
                while len(vers) > self.max_versions:
                    old = vers.pop(0)
                    try:
                        os.remove(self._path(name, old))
                    except FileNotFoundError:
                        pass
                out[name] = v
            return out

    def put_file(self, name: str, src_path: str) -> int:
        with open(src_path, "rb") as f:
            return self.put_bytes(name, f.read())

    def has(self, name: str, version: Optional[int] = None) -> bool:
        vers = self.index.get(name)
        return bool(vers) and (version is None or version in vers)

    def versions(self, name: str) -> List[int]:
        return list(self.index.get(name, []))

    def latest(self, name: str) -> Optional[int]:
        v = self.index.get(name)
        return v[-1] if v else None

    def get_bytes(self, name: str, version: Optional[int] = None) -> bytes:
        v = version if version is not None else self.latest(name)
        if v is None or not self.has(name, v):
            raise FileNotFoundError(f"{name} v{version}")
        with open(self._path(name, v), "rb") as f:
            return f.read()

    def path(self, name: str, version: Optional[int] = None) -> str:
        v = version if version is not None else self.latest(name)
        if v is None:
            raise FileNotFoundError(name)
        return self._path(name, v)

    def delete(self, name: str) -> bool:
        with self._lock:
            vers = self.index.pop(name, None)
            if not vers:
                return False
            for v in vers:
                try:
                    os.remove(self._path(name, v))
                except FileNotFoundError:
                    pass
            return True

    def list(self, pattern: str = "*") -> Dict[str, List[int]]:
        return {n: list(v) for n, v in sorted(self.index.items()) if fnmatch.fnmatch(n, pattern)}

    def all_files(self) -> Dict[str, List[int]]:
        """The reference's ``all_files`` payload (name -> versions), sent on join/ACKs."""
        return self.list("*")
