"""In-tree build of the native HIP library (``libdml_hip.so``) for gfx950.

One hipcc line per translation unit (compiled in parallel), then one link.
The .so lands next to this file so it travels with the repo snapshot to the GPU
box (a JIT cache under ~/.cache would not). No torch headers are involved: the
library exposes a plain C ABI (csrc/include/dml.h) bound with ctypes, and its
NEEDED ``libamdhip64.so.7`` resolves to the HIP runtime torch already loaded.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
LIB_PATH = PKG_DIR / "libdml_hip.so"
BUILD_DIR = REPO / "build" / "hip"
ARCH = os.environ.get("DML_OFFLOAD_ARCH", "gfx950")

SOURCES = [
    CSRC / "kernels" / "conv_dispatch.hip",
    CSRC / "kernels" / "conv_igemm_v2.hip",
    CSRC / "kernels" / "conv_igemm_ws.hip",
    CSRC / "kernels" / "conv_igemm_wsp.hip", CSRC / "kernels" / "conv_rowring.hip",
    CSRC / "kernels" / "misc.hip",
    CSRC / "kernels" / "jpeg_decode.hip",
    CSRC / "kernels" / "stem_fused.hip",
    CSRC / "kernels" / "conv_pool.hip",
    CSRC / "kernels" / "expand_reduce_chain.hip",
    CSRC / "runtime" / "runtime.hip",
]
HEADERS = [CSRC / "include" / "dml.h"] + sorted((CSRC / "kernels").glob("*.h"))  # every header the stamp covers


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.exists(cand) or cand == "hipcc"):
            return cand
    raise RuntimeError("hipcc not found")


def _flags() -> list[str]:
    return [
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-mcode-object-version=5",
        "-munsafe-fp-atomics",
        f"-I{CSRC / 'include'}",
        f"-I{CSRC / 'kernels'}",
    ]


def _stamp() -> str:
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        h.update(f.read_bytes())
    h.update(" ".join(_flags()).encode())
    return h.hexdigest()[:16]


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile csrc/ into LIB_PATH if sources changed; return the library path.
    Serialised with a file lock: every rank of a multi-GPU launch calls this."""
    import fcntl

    stamp_file = PKG_DIR / ".libdml_hip.stamp"
    stamp = _stamp()
    if not force and LIB_PATH.exists() and stamp_file.exists() and stamp_file.read_text() == stamp:
        return LIB_PATH
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    with open(BUILD_DIR / ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if not force and LIB_PATH.exists() and stamp_file.exists() and stamp_file.read_text() == stamp:
                return LIB_PATH  # another rank built it while we waited
            return _build_locked(stamp, stamp_file, verbose)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(stamp: str, stamp_file: Path, verbose: bool) -> Path:
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()

    def compile_one(src: Path) -> Path:
        obj = BUILD_DIR / (src.stem + ".o")
        cmd = [hipcc, *_flags(), "-x", "hip", "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    stamp_file.write_text(stamp)
    return LIB_PATH


# ---------------------------------------------------------------- host library --
# Pure C++ host runtime pieces (no HIP): built with g++ in a second, tiny library
# so that CPU-only processes (the CLI, the coordinator, tests) load it without
# the HIP runtime, and so a kernel edit never rebuilds it.
HOST_SOURCES = [CSRC / "host" / "output_json.cpp", CSRC / "host" / "shm_exchange.cpp", CSRC / "host" / "store_io.cpp"]
HOST_LIB_PATH = PKG_DIR / "libdml_host.so"


def _host_flags() -> list[str]:
    return ["-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-lrt"]


def build_host(force: bool = False, verbose: bool = False) -> Path:
    import fcntl

    h = hashlib.sha256()
    for f in HOST_SOURCES:
        h.update(f.read_bytes())
    h.update(" ".join(_host_flags()).encode())
    stamp = h.hexdigest()[:16]
    stamp_file = PKG_DIR / ".libdml_host.stamp"
    if not force and HOST_LIB_PATH.exists() and stamp_file.exists() and stamp_file.read_text() == stamp:
        return HOST_LIB_PATH
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    with open(BUILD_DIR / ".lock_host", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if not force and HOST_LIB_PATH.exists() and stamp_file.exists() and stamp_file.read_text() == stamp:
                return HOST_LIB_PATH
            cxx = os.environ.get("CXX", "g++")
            tmp = HOST_LIB_PATH.with_suffix(".so.tmp")
            cmd = [cxx, *_host_flags(), *map(str, HOST_SOURCES), "-o", str(tmp)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"host library build failed:\n{r.stderr}")
            os.replace(tmp, HOST_LIB_PATH)
            stamp_file.write_text(stamp)
            return HOST_LIB_PATH
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


if __name__ == "__main__":
    print(build_host(force="--force" in sys.argv, verbose=True))
    print(build(force="--force" in sys.argv, verbose=True))
