"""Python model of conv_v2_group_kernel's block -> (member, tile) map
(csrc/kernels/conv_igemm_v2.hip): every member cut into 8 contiguous per-XCD
chunks with the remainder tiles rotating over the XCDs. Checked here for
bijectivity (every tile of every member run exactly once, no block idle) and
balance (each XCD runs each member's tile count within one of t/8) over random
groups — the GPU tests check the numerics of the same map."""
import random


def block_map(tiles, b):
    x, j, rot = b & 7, b >> 3, 0
    for q, t in enumerate(tiles):
        qd, r = t >> 3, t & 7
        cnt = qd + (1 if ((x - rot) & 7) < r else 0)
        if j < cnt:
            before = sum(1 for k in range(x) if ((k - rot) & 7) < r)
            return q, x * qd + before + j
        j -= cnt
        rot = (rot + r) & 7
    return None


def test_group_block_map_bijective_and_balanced():
    rng = random.Random(0)
    cases = [[1], [1, 1], [8, 8], [7, 9, 3], [1, 1, 1, 1], [5]]
    cases += [[rng.randint(1, 400) for _ in range(rng.randint(1, 4))] for _ in range(2000)]
    for tiles in cases:
        seen, per_xcd = set(), {}
        for b in range(sum(tiles)):
            m = block_map(tiles, b)
            assert m is not None and 0 <= m[1] < tiles[m[0]], (tiles, b, m)
            seen.add(m)
            per_xcd.setdefault((b & 7, m[0]), 0)
            per_xcd[(b & 7, m[0])] += 1
        assert len(seen) == sum(tiles), tiles
        for (x, q), c in per_xcd.items():
            assert tiles[q] // 8 <= c <= tiles[q] // 8 + 1, (tiles, x, q, c)


def test_group_block_map_member_order_within_xcd():
    """On every XCD a member's tiles all come before the next member's (the host
    puts the longest-K member first: longest-processing-time dispatch)."""
    tiles = [37, 200, 5]
    for x in range(8):
        members = [block_map(tiles, b)[0] for b in range(x, sum(tiles), 8)]
        assert members == sorted(members), (x, members)


def test_tuner_candidates_are_built_tile_configs():
    """Every config the tuner may pick exists in the library's tile table (host
    functions only, no GPU): plain candidates, late-residual twins (offered to
    residual convs only) and grouped-launch tiles."""
    from distributed_machine_learning_amd import _native as N
    from distributed_machine_learning_amd.ops import tuning

    L = N.lib()
    for c in tuning.V2_CFGS + tuning.LATE_RES_CFGS:
        assert L.dml_conv_v2_bn(c) > 0, c
    for c in tuning.GROUP_CFGS:
        assert L.dml_conv_v2_group_supported(c), c
    a = N.ConvArgs()
    a.Cin = a.ldx = a.Cout = a.ldy = 64
    plain = tuning.valid_cfgs(a)
    assert not set(tuning.LATE_RES_CFGS) & set(plain)
    a.res = 1
    withres = tuning.valid_cfgs(a)
    assert set(tuning.LATE_RES_CFGS) <= set(withres) and not set(tuning.NO_RES_CFGS) & set(withres)
