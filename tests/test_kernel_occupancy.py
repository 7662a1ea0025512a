"""Occupancy guard for the conv kernels (CPU: hipcc cross-compiles gfx950).

A kernel's occupancy is min(LDS-limited, register-limited). A few extra VGPRs
once pushed the 256x128 BK32 tile from 128 to 134 VGPRs — 1 workgroup/CU
instead of 2 — and the ResNet50 stage-3 layers tuned to it ran 41 -> 58 us
(DESIGN.md §3). This test compiles csrc/kernels/conv_igemm_v2.hip with the
resource-usage remarks and checks the waves/SIMD of the tile configs the tuner
actually picks (and of the grouped kernel) against floors equal to their
LDS-limited occupancy."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)

# (BM, BN, WM, WN, STAGES, RES, BK) -> minimum waves/SIMD (= LDS-limited occupancy)
PLAIN_FLOORS = {
    (256, 128, 4, 2, 3, 0, 32): 4,   # cfg 30: 2 workgroups/CU
    (128, 256, 2, 4, 3, 0, 32): 4,   # cfg 31
    (64, 128, 1, 4, 2, 0, 64): 3,    # cfg 14: 3 workgroups/CU (48 KiB)
    (128, 64, 2, 2, 2, 0, 64): 3,    # cfg 15
    (64, 128, 1, 4, 2, 0, 32): 5,    # cfg 23
    (128, 64, 2, 2, 2, 0, 32): 5,    # cfg 24
    (64, 128, 1, 4, 3, 0, 32): 4,    # cfg 26 (36 KiB: 4 workgroups/CU)
    (128, 64, 2, 2, 3, 0, 32): 4,    # cfg 27
    (64, 128, 1, 4, 3, 1, 32): 4,    # cfg 26, residual epilogue
    (128, 64, 2, 2, 3, 1, 32): 4,    # cfg 27, residual epilogue
    (128, 128, 2, 2, 2, 0, 64): 2,   # cfg 11 (64 KiB)
    (256, 64, 4, 1, 2, 0, 64): 2,    # cfg 12 (80 KiB)
    (128, 64, 2, 2, 3, 0, 64): 2,    # cfg 38 (72 KiB: 2 workgroups/CU)
    (256, 64, 4, 1, 3, 0, 64): 1,    # cfg 39 (120 KiB)
}
LATE_FLOORS = {  # late-residual twins (residual form): the occupancy their non-residual base has
    (256, 128, 4, 2, 3, 1, 32): 4,   # cfg 56 (min-waves hint 4: 128 VGPRs, no scratch)
    (128, 256, 2, 4, 3, 1, 32): 4,   # cfg 57
    (64, 128, 1, 4, 2, 1, 32): 5,    # cfg 60
}
GROUP_FLOORS = {  # (BM, BN, WM, WN, STAGES, BK): the grouped kernel must keep its conv path's occupancy
    (64, 128, 1, 4, 2, 32): 5,
    (128, 64, 2, 2, 2, 32): 5,
    (64, 128, 1, 4, 2, 64): 3,
    (128, 64, 2, 2, 2, 64): 3,
}


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_conv_tile_occupancy_floors(tmp_path):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/csrc/include", f"-I{ROOT}/csrc/kernels",
           "-c", os.path.join(ROOT, "csrc", "kernels", "conv_igemm_v2.hip"), "-o", str(tmp_path / "k.o"),
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    occ, cur, spills = {}, None, []
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            continue
        m = re.search(r"Occupancy \[waves/SIMD\]: (\d+)", line)
        if m and cur:
            occ[cur] = int(m.group(1))
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and cur and int(m.group(1)) and "ILi256ELi256E" not in cur:  # the 256x256 residual form is known to spill
            spills.append(cur)
    plain, group, late = {}, {}, {}
    for name, w in occ.items():
        m = re.search(r"conv_v2_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELi(\d+)ELi(\d+)ELb(\d)E", name)
        if m and m.group(8) == "16":  # MF = 16 (v_mfma_f32_16x16x32_bf16) tiles
            (late if m.group(9) == "1" else plain)[tuple(int(x) for x in m.groups()[:7])] = w
        m = re.search(r"conv_v2_group_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", name)
        if m:
            group[tuple(int(x) for x in m.groups())] = w
    assert plain and group and late, "no resource-usage remarks parsed"
    assert not spills, f"conv kernels with scratch (register spills): {spills}"
    bad = [(k, plain.get(k), f) for k, f in PLAIN_FLOORS.items() if plain.get(k, 0) < f]
    bad += [(("group",) + k, group.get(k), f) for k, f in GROUP_FLOORS.items() if group.get(k, 0) < f]
    bad += [(("late",) + k, late.get(k), f) for k, f in LATE_FLOORS.items() if late.get(k, 0) < f]
    assert not bad, f"occupancy below the LDS-limited floor (config, waves/SIMD, floor): {bad}"
