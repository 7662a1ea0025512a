"""Per-shape tile selection for the implicit-GEMM conv kernel.

Different layers want different tiles (measured on MI355X, tools/conv_bench.py):
the 3x3 convs of ResNet50 run best on 128x128 (2 blocks/CU), the memory-bound
1x1 convs with narrow K on 64x128 / 128x64 tiles (more workgroups in flight).
``autotune`` times every candidate config on the engine's real buffers once
per unique shape (a few hundred launches, well under a second) and caches the
winners in a JSON table keyed by the shape signature, so later processes load
it instead of re-timing. Candidates are timed cold by default (each launch after
overwriting 512 MiB, so weights and activations come from HBM as inside a
forward): the warm back-to-back timing picked tiles that lose in the engine
(DESIGN.md §3 "Cold-cache tuning").
"""
from __future__ import annotations

import ctypes as C
import json
import os
import threading
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from .. import _native as N

V2_CFGS = (10, 11, 12, 13, 14, 15, 16, 18, 21, 22, 23, 24, 26, 27, 28, 29, 30, 31, 32, 33, 34, 36, 37,
           38, 39)  # 23..37: BK32; 38 / 39: 3-stage BK64 64-channel tiles (r3)
# warp-specialised tiles (csrc/kernels/conv_igemm_ws.hip: loader waves + MFMA waves, r5)
WS_CFGS = tuple(range(100, 113)) + (119,)  # 113..118 (fragment prefetch) removed in r6
# their persistent form (csrc/kernels/conv_igemm_wsp.hip: one operand ring over a workgroup's
# whole tile list; no split-K)
WSP_CFGS = tuple(range(120, 130))
# the row-ring 3x3 kernel of ResNet50 stage 2 (csrc/kernels/conv_rowring.hip: weights resident in
# LDS, input rows streamed once per strip; 2 / 1 / 4 strips per image, r5)
RR_CFGS = (150, 151, 152)
CACHE_PATH = os.environ.get(
    "DML_TUNING_CACHE",
    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "conv_tuning.json"))
_lock = threading.Lock()


# Cache entries are only valid for the candidate set, kernel build and timing
# method they were timed with. "c4la": the late-residual twins joined the
# candidates of residual convs. "c5rt": every shape re-timed warm (10 back-to-back
# launches). "c5cold": every shape timed cold (time_cfg), the engine's situation:
# a forward's weights and most activations are out of L2/MALL when their layer
# runs; same-box A/B ResNet50 83.2-83.7k vs 81.9-82.1k img/s (profiles/r2_v31).
# DML_TUNING_TAG selects another tag (A/B of tables).
CAND_TAG = os.environ.get("DML_TUNING_TAG", "c5cold")


def shape_key(a: N.ConvArgs) -> str:
    """Cache key of a conv shape."""
    return (f"n{a.N}_h{a.H}_w{a.W}_c{a.Cin}_ld{a.ldx}_k{a.kh}x{a.kw}_s{a.sh}x{a.sw}_p{a.ph}x{a.pw}"
            f"_o{a.Cout}_K{a.Kpad}_r{int(bool(a.res))}_f{a.out_f32}_d{max(a.dh, 1)}x{max(a.dw, 1)}"
            + (f"_ks{a.ksplit}" if a.ksplit > 1 else "")
            + (f"_rs{a.rsub}" if a.rsub > 1 else "")
            + "_" + CAND_TAG)


def load_cache(path: str = CACHE_PATH) -> Dict[str, int]:
    try:
        with open(path) as f:
            return {k: int(v) for k, v in json.load(f).items()}
    except (OSError, ValueError):
        return {}


def save_cache(table: Dict[str, int], path: str = CACHE_PATH) -> None:
    with _lock:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        cur = load_cache(path)  # entries of other tags stay (A/B via DML_TUNING_TAG); lookups match the tag
        cur.update(table)
        tmp = f"{path}.{os.getpid()}.tmp"  # ranks of one node may tune concurrently
        with open(tmp, "w") as f:
            json.dump(dict(sorted(cur.items())), f, indent=0)
        os.replace(tmp, path)


NO_RES_CFGS = (34,)  # the residual-epilogue instantiation spills (256x256 tile)
# late-residual twins (residual loaded in the epilogue; identical to their base
# tile on residual-free convs, so timed on residual layers only)
LATE_RES_CFGS = (56, 57, 58, 59, 60)


def _excluded() -> set:
    """DML_TUNE_EXCLUDE=<cfg,cfg,...>: configs the tuner must not pick (A/B)."""
    v = os.environ.get("DML_TUNE_EXCLUDE", "")
    return {int(c) for c in v.split(",") if c.strip()}


def rr_fits(a: N.ConvArgs) -> bool:
    """The shapes conv_rowring.hip runs (mirrors its launcher's check)."""
    return (a.kh == 3 and a.kw == 3 and a.ph == 1 and a.pw == 1 and a.sh == 1 and a.sw == 1
            and max(a.dh, 1) == 1 and max(a.dw, 1) == 1 and a.Cin == 64 and a.Cout <= 64
            and a.W == 56 and a.Wo == 56 and a.Ho == a.H and a.ksplit <= 1 and a.nseg == 0
            and a.rsub <= 1 and a.Kpad >= 576)


def valid_cfgs(a: N.ConvArgs) -> List[int]:
    if a.Cout % 8 or a.Cin % 8 or a.ldx % 8 or a.ldy % 8:
        return []
    ex = _excluded()
    cands = [c for c in V2_CFGS if not (a.res and c in NO_RES_CFGS)] + (list(LATE_RES_CFGS) if a.res else [])
    cands += list(WS_CFGS) + ([] if a.ksplit > 1 else list(WSP_CFGS))
    if rr_fits(a):
        cands += list(RR_CFGS)
    return [c for c in cands if c not in ex]


def _added() -> List[int]:
    """DML_TUNE_ADD=<cfg,...>: configs new to the table. A cached shape re-times its cached
    config against these (cold, same method) and switches only when one is >= 3 % faster,
    so the pipeline-co-tuned entries (tools/cotune_pipe.py) stay unless a new kernel clearly
    beats them alone."""
    v = os.environ.get("DML_TUNE_ADD", "")
    return [int(c) for c in v.split(",") if c.strip()]


_scrub = None


def _release_scrub() -> None:
    global _scrub
    _scrub = None  # the 512 MiB eviction buffer is only needed while timing


def _cold() -> bool:
    return os.environ.get("DML_TUNE_COLD", "1") == "1"


def time_cfg(a: N.ConvArgs, cfg: int, iters: int = 10) -> float:
    """Mean time of one launch. Default (DML_TUNE_COLD=1): every launch timed
    alone after overwriting a 512 MiB buffer (L2 and MALL evicted: weights and
    activations come from HBM, as inside a forward). DML_TUNE_COLD=0:
    back-to-back launches (L2/MALL warm)."""
    import torch

    global _scrub
    L = N.lib()
    s = N.stream_ptr()
    N.check(L.dml_conv(C.byref(a), cfg, s), "conv warmup")
    if _cold():
        if _scrub is None:
            _scrub = torch.zeros(128 << 20, device=torch.cuda.current_device())
        ms = 0.0
        for _ in range(iters):
            _scrub.add_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.dml_conv(C.byref(a), cfg, s)
            e1.record()
            e1.synchronize()
            ms += e0.elapsed_time(e1)
        return ms / iters
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        L.dml_conv(C.byref(a), cfg, s)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def autotune(args: Iterable[N.ConvArgs], cache: Optional[Dict[str, int]] = None, persist: bool = True
             ) -> Dict[str, int]:
    """Return {shape_key: best cfg} for every ConvArgs (timing the uncached ones)."""
    args = list(args)
    cache = dict(load_cache() if cache is None else cache)
    new: Dict[str, int] = {}
    added = _added()
    for a in args:
        k = shape_key(a)
        if k in new:
            continue
        if k in cache and cache[k] in valid_cfgs(a):
            adds = [c for c in added if c in valid_cfgs(a) and c != cache[k]]
            if not adds:
                continue  # a cached cfg that is no longer a candidate (removed / excluded) is re-timed
            try:
                cur = time_cfg(a, cache[k])
            except N.NativeError:
                cur = float("inf")
            best = (cur, cache[k])
            for cfg in adds:
                try:
                    t = time_cfg(a, cfg)
                except N.NativeError:
                    continue
                if t < 0.97 * best[0]:
                    best = (t, cfg)
            if best[1] != cache[k]:
                new[k] = best[1]
            continue
        best: Tuple[float, int] = (float("inf"), -1)
        for cfg in valid_cfgs(a):
            try:
                t = time_cfg(a, cfg)
            except N.NativeError:
                continue
            best = min(best, (t, cfg))
        new[k] = best[1]
    if new and persist:
        try:
            save_cache(new)
        except OSError:
            pass
    cache.update(new)
    _release_scrub()
    return cache


# ---------------------------------------------------------- grouped convs --
GROUP_CFGS = (11, 12, 14, 15, 17, 22, 23, 24, 25, 26, 27, 28, 29, 32, 33)  # 4-wave tiles (dml_conv_v2_group)


def pool_key(p: N.PoolArgs) -> str:
    return f"pool{p.mode}_n{p.N}_h{p.H}_w{p.W}_c{p.C}_o{p.Ho}x{p.Wo}_s{p.stride}_p{p.pad}"


# bumped when the grouped kernel or the timing changes (r2: XCD-balanced LPT
# order; low-register pool path; grp4: cold-cache timing). DML_GROUP_TAG: A/B.
GROUP_TAG = os.environ.get("DML_GROUP_TAG", "grp4")


def group_key(args: List[N.ConvArgs], pools: Sequence[N.PoolArgs] = ()) -> str:
    return (GROUP_TAG + "_" + "|".join([shape_key(a)[:-len(CAND_TAG) - 1] for a in args] + [pool_key(p) for p in pools])
            + "_" + CAND_TAG)


def group_args(args: List[N.ConvArgs], pools: Sequence[N.PoolArgs] = ()) -> N.ConvGroupArgs:
    g = N.ConvGroupArgs()
    g.n, g.npool = len(args), len(pools)
    for i, a in enumerate(args):
        g.a[i] = a
    for i, p in enumerate(pools):
        g.pool[i] = p
    return g


def _time(fn, iters: int) -> float:
    """Mean time of ``fn``'s launches: cold (each call timed alone after the
    L2/MALL scrub, as time_cfg) unless DML_TUNE_COLD=0."""
    import torch

    global _scrub
    fn()
    if _cold():
        if _scrub is None:
            _scrub = torch.zeros(128 << 20, device=torch.cuda.current_device())
        ms = 0.0
        for _ in range(iters):
            _scrub.add_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ms += e0.elapsed_time(e1)
        return ms / iters
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def autotune_group(args: List[N.ConvArgs], cfgs: List[int], pools: Sequence[N.PoolArgs] = (),
                   cache: Optional[Dict[str, int]] = None, persist: bool = True, iters: int = 20) -> int:
    """Best tile for launching ``args`` (and the 3x3 ``pools``) as ONE grouped
    grid, or -1 when running them one after another, each conv on its own tuned
    tile ``cfgs``, is faster."""
    k = group_key(args, pools)
    cache = load_cache() if cache is None else cache
    if k in cache and (cache[k] == -1 or cache[k] in GROUP_CFGS):  # -1: grouping measured slower; a removed tile is re-timed
        return cache[k]
    L, s = N.lib(), N.stream_ptr()
    best: Tuple[float, int] = (float("inf"), -1)
    if all(c >= 0 for c in cfgs):
        def seq():
            for a, c in zip(args, cfgs):
                N.check(L.dml_conv(C.byref(a), c, s), "conv")
            for p in pools:
                N.check(L.dml_pool(C.byref(p), s), "pool")
        best = (_time(seq, iters), -1)
    g = group_args(args, pools)
    for cfg in GROUP_CFGS:
        try:
            t = _time(lambda: N.check(L.dml_conv_group(C.byref(g), cfg, s), "conv group"), iters)
        except N.NativeError:
            continue
        best = min(best, (t, cfg))
    cache[k] = best[1]
    _release_scrub()
    if persist:
        try:
            save_cache({k: best[1]})
        except OSError:
            pass
    return best[1]
