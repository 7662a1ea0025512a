"""Race/memory checking of the native runtime's host code (SURVEY §5 'race
detection / sanitizers'): csrc/ is rebuilt with AddressSanitizer (+ leak
check) and UndefinedBehaviorSanitizer on the HOST side only (-Xarch_host
-fsanitize=...; GPU sanitizers are not available on this pool) and
csrc/tests/host_checks.cpp drives every host-only path — plan recording and
teardown, launch-argument validation, error plumbing — on a CPU-only machine.
"""
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)
# every translation unit of libdml_hip.so (the build's own list) plus the host driver
from distributed_machine_learning_amd import _build  # noqa: E402

SOURCES = [os.path.relpath(str(p), os.path.join(ROOT, "csrc")) for p in _build.SOURCES] + ["tests/host_checks.cpp"]
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-omit-frame-pointer"]


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_host_runtime_under_asan_ubsan(tmp_path):
    inc = [f"-I{ROOT}/csrc/include", f"-I{ROOT}/csrc/kernels"]

    def compile_one(src):
        obj = tmp_path / (os.path.basename(src).rsplit(".", 1)[0] + ".o")
        cmd = [HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", *SAN, *inc, "-x", "hip", "-c",
               os.path.join(ROOT, "csrc", src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        return str(obj)

    with ThreadPoolExecutor(max_workers=3) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    exe = str(tmp_path / "host_checks")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", *SAN[:4], *objs, "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "host checks passed" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out
