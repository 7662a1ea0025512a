"""Build a variant of libdml_hip.so where ONE translation unit is compiled with extra
-D flags (kernel A/B probes), reusing the other objects of the in-tree build.

python tools/build_variant.py <tag> <source, e.g. kernels/conv_igemm_v2.hip> [-DFOO=1 ...]
-> variants/libdml_<tag>.so (git-ignored, shipped to the GPU box by gpurun)
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_machine_learning_amd import _build  # noqa: E402

tag, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
_build.build()
out_dir = _build.REPO / "variants"
out_dir.mkdir(exist_ok=True)
src_path = _build.CSRC / src
obj = out_dir / f"{src_path.stem}_{tag}.o"
subprocess.run([_build._hipcc(), *_build._flags(), *defs, "-x", "hip", "-c", str(src_path), "-o", str(obj)],
               check=True)
objs = [str(obj) if s == src_path else str(_build.BUILD_DIR / (s.stem + ".o")) for s in _build.SOURCES]
lib = out_dir / f"libdml_{tag}.so"
subprocess.run([_build._hipcc(), f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-Wl,-Bsymbolic", *objs, "-o", str(lib)],
               check=True)
print(lib)
