"""The MI355X inference engine: layer IR -> native launch plan.

Lowering (SURVEY §7.1 "C++/HIP graph executor"):

* BatchNorm is folded into the conv weights/bias once, on the host
  (``weights.fold_conv``); weights become bf16 ``[Cout_pad][K_pad]`` with K in
  (r, s, c) order, resident in HBM for the life of the process (the reference
  rebuilds the Keras model per batch, models.py:84-91).
* Every tensor is an NHWC bf16 buffer; Inception concats are channel-offset
  writes into one buffer; a liveness pass reuses buffers.
* The forward is recorded once into the native plan (csrc/runtime/runtime.hip):
  preprocess -> convs/pools -> global-avg-pool -> FC (1x1 implicit GEMM, fp32
  out) -> softmax+top-5, and can be captured into a hipGraph.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import _native as N
from .graph import Conv, Dense, FusedConv, Graph, GlobalAvgPool, Pool, node_outputs
from .weights import Weights, fold_conv


def _r(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def pair_pack_kernel(kernel_hwio: np.ndarray) -> np.ndarray:
    """[kh, kw, 3, cout] -> [kh, ceil(kw/2), 8, cout]: tap s' holds taps 2s' (channels 0-2)
    and 2s'+1 (channels 4-6) to match the pair-packed stem input."""
    kh, kw, cin, cout = kernel_hwio.shape
    assert cin <= 4
    kw2 = (kw + 1) // 2
    out = np.zeros((kh, kw2, 8, cout), np.float32)
    for s in range(kw):
        out[:, s // 2, 4 * (s % 2): 4 * (s % 2) + cin, :] = kernel_hwio[:, s]
    return out


def pack_conv_weight(kernel_hwio: np.ndarray, cin_eff: int, cout_pad: int, k_pad: int) -> np.ndarray:
    kh, kw, cin, cout = kernel_hwio.shape
    k = np.zeros((kh, kw, cin_eff, cout), np.float32)
    k[:, :, :cin, :] = kernel_hwio
    k = k.transpose(3, 0, 1, 2).reshape(cout, kh * kw * cin_eff)
    out = np.zeros((cout_pad, k_pad), np.float32)
    out[:cout, : k.shape[1]] = k
    return out


class Engine:
    """Batch-``batch`` executor of ``graph`` on the current CUDA (HIP) device."""

    def __init__(self, graph: Graph, weights: Weights, batch: int, device: str = "cuda",
                 src_hw: Optional[Tuple[int, int]] = None, cfg_overrides: Optional[Dict[str, int]] = None,
                 src_slots: int = 1, reuse_buffers: bool = True, autotune: bool = True, optimize: bool = True,
                 share: Optional["Engine"] = None, src_tensors: Optional[List[torch.Tensor]] = None,
                 result_views: Optional[List[torch.Tensor]] = None, fuse_stem: bool = True,
                 fuse_blocks: bool = True, conv_groups: Optional[bool] = None,
                 ext_buffers: Optional[Dict[str, List[torch.Tensor]]] = None,
                 tune_range: Optional[Tuple[Optional[str], Optional[str]]] = None,
                 src_index: Optional[List[torch.Tensor]] = None):
        """``share``: reuse another engine's (optimized) graph and resident weights
        (sub-batch engines of a SplitEngine); ``src_tensors`` / ``result_views``:
        external uint8 source slots / per-slot [2, batch, 5] result rows to use
        instead of allocating them. ``src_index``: per slot, an int32 [batch] table in
        device memory (rewritten by the caller before each run, in stream order): image n
        of the batch is image src_index[slot][n] of that slot's source tensor — the
        serving path's HBM arena, read in place by the stem kernel instead of gathered
        into a batch buffer first. ``fuse_stem=False`` (or DML_FUSED_STEM=0) keeps the
        ResNet stem as three launches (preprocess, conv, pool); ``fuse_blocks=False``
        (or DML_FUSED_BLOCKS=0) keeps every bottleneck 1x1 conv its own launch;
        ``conv_groups=False`` (or DML_CONV_GROUPS=0) launches InceptionV3's
        independent branch convs one by one instead of as grouped grids.
        ``ext_buffers``: {tensor: [flat bf16 storage per source slot]} — tensors this engine
        reads / writes in caller-owned memory instead of its own buffers (the merge tensors of
        a split-head / merged-tail SplitEngine: each head writes its rows of the tail's
        buffer), never recycled for another tensor. ``tune_range``: (first node, stop node) names
        (None = graph start / end): only those convs are autotuned (the part of the graph this
        engine will run); the others get the default tile."""
        if conv_groups is None:
            conv_groups = os.environ.get("DML_CONV_GROUPS", "1") != "0"
        if share is not None:
            graph = share.g
        elif optimize:  # graph rewrites: conv-before-avgpool, sibling 1x1 fusion (models/optimize.py)
            from .optimize import optimize as _opt

            merge = os.environ.get("DML_SHORTCUT_MERGE", "1") != "0"
            graph = _opt(graph, stride_push=os.environ.get("DML_STRIDE_PUSH") != "0",
                         weights=weights if merge else None,
                         shortcut_min_cout=int(os.environ.get("DML_SHORTCUT_MERGE_MINC", "0")))
            if conv_groups:  # independent convs side by side (models/optimize.py rewrite 5)
                from .optimize import level_order

                graph = level_order(graph)
        self.g, self.batch, self.device = graph, batch, torch.device(device)
        self.src_slots = src_slots
        self.reuse_buffers = reuse_buffers
        self.autotune = autotune
        self.lib = N.lib()
        self.src_hw = src_hw or graph.input_hw
        self.cfg_overrides = cfg_overrides or {}
        self._keep = []  # keep ctypes structs / tensors alive
        # Pair-packed stem: if the only consumer of the 3-channel input is one conv,
        # the preprocess kernel writes two horizontally adjacent pixels per 16-byte
        # chunk and that conv runs with dilation 2 over half as many taps — K drops
        # from kh*kw*8 to kh*ceil(kw/2)*8 (ResNet50 7x7: 392 -> 224).
        readers = [n for n in graph.nodes if getattr(n, "inp", None) == graph.input]
        self.stem = readers[0] if (len(readers) == 1 and isinstance(readers[0], Conv) and readers[0].cin == 3
                                   and readers[0].in_coff == 0 and readers[0].kw > 1) else None
        self.stem_lpad = self.stem.pw if self.stem is not None else 0
        # ResNet stem: preprocess + 7x7/2 conv + 3x3/2 max pool run as ONE kernel
        # (csrc/kernels/stem_fused.hip) when the pool is the conv's only consumer.
        self.stem_pool = self._fusable_stem_pool(fuse_stem)
        # ... with the 1x1 conv reading exactly the pooled tensor folded in (ResNet50 conv2_block1_1)
        self.stem_1x1 = self._foldable_stem_1x1(fuse_stem)
        # InceptionV3 stem: preprocess + conv 3x3/2 + conv 3x3 as ONE kernel
        self.stem_conv2 = self._fusable_inception_stem(fuse_stem) if self.stem_pool is None else None
        # conv 3x3 (32 -> 64) + the 3x3/2 max pool reading it as ONE kernel (csrc/kernels/conv_pool.hip),
        # with the 1x1 conv that is the pool's only reader folded in (InceptionV3 conv2d_4)
        self.conv_pools = self._fusable_conv_pools(fuse_stem)
        self.conv_pool_1x1 = self._foldable_pool_1x1(fuse_stem)
        # ResNet block boundaries: expand (+ shortcut) and the next block's reduce as ONE
        # kernel (csrc/kernels/expand_reduce_chain.hip)
        self.exp_red = self._fusable_expand_reduce(fuse_blocks)
        # fused pairs whose Y is otherwise only read at stride 2 store just those pixels
        self.ysub = self._subsampled_y()
        # a stage's last expand (its shortcut stored compactly by the pair above) chained with
        # the next stage's first reduce
        self.exp_red.update(self._fusable_stage_end(fuse_blocks))
        # independent residual-free convs of one graph level -> one grouped grid each
        self.conv_groups = self._conv_group_candidates() if conv_groups else []
        self._src_tensors, self._result_views = src_tensors, result_views
        self.src_index = src_index
        if src_index is not None:
            assert len(src_index) == src_slots and all(t.dtype == torch.int32 and t.numel() >= batch
                                                       and t.is_contiguous() for t in src_index)
        self._ext = ext_buffers or {}
        self._tune_range = tune_range
        self.op_range: Optional[Tuple[int, int]] = None
        if share is not None:
            self.wdev = share.wdev
        else:
            self._upload_weights(weights)
        self._alloc_buffers()
        self._build_plan()

    # ------------------------------------------------------------ weights ----
    def _upload_weights(self, w: Weights) -> None:
        self.wdev: Dict[str, Tuple[torch.Tensor, torch.Tensor, int, int, int]] = {}
        for n in self.g.nodes:
            if isinstance(n, Conv):
                k, b = fold_conv(n, w)
                if n is self.stem:
                    k = pair_pack_kernel(k)
                    kw = k.shape[1]
                    cin_eff = 8
                    K = n.kh * kw * cin_eff
                else:
                    cin_eff = _r(n.cin, 8)
                    K = n.kh * n.kw * cin_eff
                coutp, kpad = _r(n.cout, 256), _r(K, 64)
                wk = pack_conv_weight(k, cin_eff, coutp, kpad)
            elif isinstance(n, Dense):
                k = w[f"{n.name}/kernel"][None, None]  # 1x1xCinxCout
                b = w[f"{n.name}/bias"]
                cin_eff = _r(n.cin, 8)
                K = cin_eff
                coutp, kpad = _r(n.cout, 256), _r(K, 64)
                wk = pack_conv_weight(k, cin_eff, coutp, kpad)
            elif isinstance(n, FusedConv):
                # members' folded 1x1 kernels concatenated along Cout (segment order)
                folded = [fold_conv(m, w) for m in n.members]
                k = np.concatenate([f[0] for f in folded], axis=3)
                b = np.concatenate([f[1] for f in folded])
                cin_eff = _r(n.cin, 8)
                K = cin_eff
                coutp, kpad = _r(n.cout, 256), _r(K, 64)
                wk = pack_conv_weight(k, cin_eff, coutp, kpad)
            else:
                continue
            bias = np.zeros(coutp, np.float32)
            bias[: len(b)] = b
            self.wdev[n.name] = (
                torch.from_numpy(wk).to(self.device, torch.bfloat16).contiguous(),
                torch.from_numpy(bias).to(self.device),
                K, kpad, cin_eff,
            )

    def _foldable_stem_1x1(self, enabled: bool) -> Optional[Conv]:
        """The 1x1 conv (64 -> 64, stride 1, ReLU, no residual) that reads exactly the fused stem's
        pooled tensor — ResNet50's conv2_block1_1, which after the projection-shortcut merge reads
        the s slice of stage 2's [x ; s] buffer — applied by the stem kernel to the pooled tile in
        LDS (csrc/kernels/stem_fused.hip step 5). The pooled tensor is still written (the merged
        expand reads it). DML_FOLD_STEM_1X1=0: off (A/B)."""
        p = self.stem_pool
        if not enabled or p is None or os.environ.get("DML_FOLD_STEM_1X1", "1") == "0":
            return None
        nodes = self.g.nodes
        i = nodes.index(p)
        k = nodes[i + 1] if i + 1 < len(nodes) else None
        if not (isinstance(k, Conv) and k.inp == p.out and k.in_coff == p.out_coff and k.cin == 64
                and k.cout == 64 and k.kh == k.kw == 1 and k.sh == k.sw == 1 and k.ph == k.pw == 0 and k.relu
                and k.residual is None and not k.out_f32 and k.out_coff == 0 and max(getattr(k, "dh", 1), 1) == 1):
            return None
        return k

    def _fusable_stem_pool(self, enabled: bool) -> Optional[Pool]:
        """The max pool that the fused stem kernel can absorb together with the
        stem conv (conv 7x7/2 pad 3 -> 64 ch + ReLU, then pool 3x3/2 pad 1), else None."""
        s = self.stem
        if not enabled or s is None or self.device.type != "cuda" or os.environ.get("DML_FUSED_STEM") == "0":
            return None
        if not (s.kh == s.kw == 7 and s.sh == s.sw == 2 and s.ph == s.pw == 3 and s.cout == 64 and s.relu
                and s.residual is None and not s.out_f32 and s.out_coff == 0):
            return None
        users = [n for n in self.g.nodes if s.out in (getattr(n, "inp", None), getattr(n, "residual", None))]
        if len(users) != 1 or not isinstance(users[0], Pool):
            return None
        p = users[0]
        if (p.mode, p.k, p.stride, p.pad, p.relu) != ("max", 3, 2, 1, False) or p.out_coff % 8:
            return None
        return p

    def _fusable_inception_stem(self, enabled: bool) -> Optional[Conv]:
        """The second conv that the fused InceptionV3 stem kernel absorbs together
        with the stem conv (conv 3x3/2 valid 3 -> 32, then conv 3x3 valid 32 -> 32,
        both + ReLU), else None."""
        s = self.stem
        if not enabled or s is None or self.device.type != "cuda" or os.environ.get("DML_FUSED_STEM") == "0":
            return None
        if not (s.kh == s.kw == 3 and s.sh == s.sw == 2 and s.ph == s.pw == 0 and s.cout == 32 and s.relu
                and s.residual is None and not s.out_f32 and s.out_coff == 0):
            return None
        users = [n for n in self.g.nodes if s.out in (getattr(n, "inp", None), getattr(n, "residual", None))]
        if len(users) != 1 or not isinstance(users[0], Conv):
            return None
        c = users[0]
        if not (c.kh == c.kw == 3 and c.sh == c.sw == 1 and c.ph == c.pw == 0 and c.cin == 32 and c.cout == 32
                and c.relu and c.residual is None and not c.out_f32 and c.in_coff == 0):
            return None
        return c

    def _fusable_conv_pools(self, enabled: bool) -> Dict[str, Pool]:
        """{conv name: pool} for 3x3 stride-1 pad-1 convs (32 -> 64 channels, ReLU)
        whose only consumer is a 3x3/2 valid max pool (InceptionV3 conv2d_3)."""
        if not enabled or self.device.type != "cuda" or os.environ.get("DML_FUSED_STEM") == "0":
            return {}
        out: Dict[str, Pool] = {}
        for c in self.g.nodes:
            if not (isinstance(c, Conv) and c is not self.stem and c.kh == c.kw == 3 and c.sh == c.sw == 1
                    and c.ph == c.pw == 1 and c.cin == 32 and c.cout == 64 and c.relu and c.residual is None
                    and not c.out_f32 and c.in_coff == 0 and c.out_coff == 0):
                continue
            users = [n for n in self.g.nodes if c.out in (getattr(n, "inp", None), getattr(n, "residual", None))]
            if len(users) == 1 and isinstance(users[0], Pool):
                p = users[0]
                if (p.mode, p.k, p.stride, p.pad, p.out_coff, p.relu) == ("max", 3, 2, 0, 0, False):
                    out[c.name] = p
        return out

    def _foldable_pool_1x1(self, enabled: bool) -> Dict[str, Conv]:
        """{conv name: 1x1 conv} for fused conv+pool pairs whose pool output is read only by
        a 1x1 stride-1 conv (64 -> c4, c4 % 16 == 0, <= 128, ReLU, no residual): the conv_pool
        kernel applies it to the pooled tile in LDS. DML_FOLD_POOL_1X1=0: off (A/B)."""
        if not enabled or os.environ.get("DML_FOLD_POOL_1X1", "1") == "0":
            return {}
        out: Dict[str, Conv] = {}
        for c_name, p in self.conv_pools.items():
            users = [n for n in self.g.nodes if p.out in (getattr(n, "inp", None), getattr(n, "residual", None))]
            if len(users) != 1 or not isinstance(users[0], Conv):
                continue
            k = users[0]
            if (k.kh == k.kw == 1 and k.sh == k.sw == 1 and k.ph == k.pw == 0 and k.cin == 64 and k.relu
                    and k.residual is None and not k.out_f32 and k.in_coff == 0 and k.out_coff == 0
                    and k.cout % 16 == 0 and k.cout <= 128 and max(getattr(k, "dh", 1), 1) == 1):
                out[c_name] = k
        return out

    def cbuf_of(self, name: str) -> int:
        return _r(self.g.tensors[name].c, 8)

    def _fusable_expand_reduce(self, enabled: bool) -> Dict[str, Conv]:
        """{expand conv name: reduce conv} for adjacent node pairs expand (1x1 s1,
        F -> C, shortcut, ReLU) -> reduce (1x1 s1 reading the expand output, C -> F,
        ReLU), F = C / 4 — ResNet50's convN_blockK_3 / convN_blockK+1_1, run by the chained
        kernel (expand_reduce_chain.hip) for C in {256, 512} (C = 1024 with DML_CHAIN=2: no
        faster than its two launches), with the shortcut or merged (K = 2F, no residual)."""
        if not enabled or self.device.type != "cuda" or os.environ.get("DML_FUSED_BLOCKS") == "0":
            return {}
        maxc = int(os.environ.get("DML_FUSED_BLOCKS_MAXC", "256"))
        out: Dict[str, Conv] = {}
        nodes = self.g.nodes
        in_block = {t.name for trip in getattr(self, "blocks", {}).values() for t in trip}
        for e, r in zip(nodes, nodes[1:]):
            if not (isinstance(e, Conv) and isinstance(r, Conv)) or e.name in in_block or r.name in in_block:
                continue
            # with its shortcut (K = F), or a merged projection shortcut (K = 2F, no residual; C = 256)
            shortcut = e.residual and e.res_sub == 1 and e.cin * 4 == e.cout
            # merged: the chained kernel (ResNet50 b256 91.2-91.3k vs 88.1-89.3k img/s interleaved on
            # one box, profiles/r3_v9; DML_CHAIN_MERGED=0: off)
            chain_m = os.environ.get("DML_CHAIN_MERGED", "1") == "1"
            merged = e.residual is None and e.cin * 2 == e.cout and e.cout in (256, 512) and chain_m
            # the chained-GEMM kernel (expand_reduce_chain.hip): the C = 512 boundaries (stage 3) by
            # default (ResNet50 b256 87.8-88.3k vs 85.4-86.1k img/s, profiles/r3_v3); DML_CHAIN=2 also
            # C = 1024 (stage 4: no faster than its two launches), DML_CHAIN=0 none
            ch = os.environ.get("DML_CHAIN", "1")
            chain = merged or (shortcut and ((e.cout == 512 and ch in ("1", "2")) or (e.cout == 1024 and ch == "2")))
            if not (e.kh == e.kw == 1 and e.sh == e.sw == 1 and e.cout in (256, 512, 1024) and (e.cout <= maxc or chain)
                    and (shortcut or merged)
                    and e.relu and e.in_coff == 0 and e.out_coff == 0 and not e.out_f32):
                continue
            if not (r.inp == e.out and r.kh == r.kw == 1 and r.sh == r.sw == 1 and r.cin == e.cout
                    and r.cout * 4 == e.cout
                    and r.relu and r.residual is None and r.in_coff == 0 and r.out_coff == 0 and not r.out_f32):
                continue
            out[e.name] = r
        return out

    def _fusable_stage_end(self, enabled: bool) -> Dict[str, Conv]:
        """{expand name: reduce} for a stage's last block boundary, chained (expand_reduce_chain.hip):
        the expand (1x1 F -> C = 4F, + the shortcut, which the previous fused boundary stored
        compactly: ``ysub``) writes its C channels into the next stage's ``[x ; s]`` concat buffer,
        and the next stage's first reduce (C -> 2F) reads exactly that slice. ResNet50:
        conv2_block3_3 -> conv3_block1_1 (64 -> 256 -> 128 at 28x28). DML_CHAIN_STAGE_END=2 also
        stage 3's end (128 -> 512 -> 256 at 14x14, 16 pixels per wave: its 256 reduce accumulators;
        exact, neutral in the pipeline: 90.4-91.1k vs 90.5-90.9k img/s, profiles/r3_v11); 0: off."""
        if (not enabled or self.device.type != "cuda" or os.environ.get("DML_FUSED_BLOCKS") == "0"
                or os.environ.get("DML_CHAIN_STAGE_END", "1") == "0"):
            return {}
        out: Dict[str, Conv] = {}
        nodes = self.g.nodes
        taken = set(self.exp_red) | {r.name for r in self.exp_red.values()}
        taken |= {t.name for trip in getattr(self, "blocks", {}).values() for t in trip}
        for e, r in zip(nodes, nodes[1:]):
            if not (isinstance(e, Conv) and isinstance(r, Conv)) or e.name in taken or r.name in taken:
                continue
            shapes = {(64, 256)} | ({(128, 512)} if os.environ.get("DML_CHAIN_STAGE_END") == "2" else set())
            if not (e.kh == e.kw == 1 and e.sh == e.sw == 1 and (e.cin, e.cout) in shapes and e.relu
                    and e.residual in self.ysub and e.in_coff == 0 and not e.out_f32):
                continue
            if not (r.inp == e.out and r.in_coff == e.out_coff and r.cin == e.cout and r.cout == 2 * e.cin
                    and r.kh == r.kw == 1 and r.sh == r.sw == 1 and r.relu and r.residual is None
                    and r.out_coff == 0 and not r.out_f32):
                continue
            out[e.name] = r
        return out

    def _conv_group_candidates(self) -> List[list]:
        """Runs of consecutive groupable convs / 3x3 pools of one ASAP level (the
        level order puts them side by side), at most GROUP_MAX convs and
        GROUP_POOL_MAX pools per group. Whether a group really
        launches as one grid is decided by timing at plan time (``_build_plan``)."""
        from .optimize import conv_group_runs

        taken = {t.name for t in (self.stem, self.stem_conv2, self.stem_pool, self.stem_1x1) if t is not None}
        taken |= set(self.conv_pools) | {p.name for p in self.conv_pools.values()}
        taken |= {k.name for k in self.conv_pool_1x1.values()}
        taken |= set(self.exp_red) | {r.name for r in self.exp_red.values()}
        return conv_group_runs(self.g, taken, N.GROUP_MAX, N.GROUP_POOL_MAX)

    def _subsampled_y(self) -> Dict[str, int]:
        """{tensor: 2} for fused expand+reduce outputs Y whose readers besides the fused
        reduce all take it as a stride-2 shortcut (``res_sub == 2``, left by the stride
        pushdown): the kernel then stores only those pixels, compactly (a quarter of the
        Y bytes), and the readers address it as a same-grid residual. The compact tensor
        sits at the start of Y's full-size buffer (``view`` shows it in the first quarter)."""
        if os.environ.get("DML_YSUB", "1") == "0":
            return {}
        out: Dict[str, int] = {}
        for e_name, r in self.exp_red.items():
            e = next(n for n in self.g.nodes if getattr(n, "name", None) == e_name)
            h, w, _ = self.g.shape(e.out)
            users = [n for n in self.g.nodes if n is not r and e.out in (getattr(n, "inp", None),
                                                                          getattr(n, "residual", None))]
            if (users and h % 2 == 0 and w % 2 == 0 and e.out != self.g.logits
                    and all(isinstance(u, Conv) and u.inp != e.out and u.residual == e.out and u.res_sub == 2
                            for u in users)):
                out[e.out] = 2
        return out

    # ------------------------------------------------------------ buffers ----
    def _fc_split(self) -> int:
        """Split-K slices of the classifier GEMM: M = batch rows and N = 1000
        classes give only a few dozen output tiles on 256 CUs, so the K = 2048
        loop is cut into slices (fp32 partials, summed by the softmax kernel)."""
        env = os.environ.get("DML_FC_KSPLIT")
        dense = [n for n in self.g.nodes if isinstance(n, Dense)]
        if not dense or self.device.type != "cuda":
            return 1
        nk = self.wdev[dense[0].name][3] // 64
        ks = int(env) if env else (8 if nk >= 16 else max(1, nk // 2))
        return max(1, min(ks, nk))

    def _alloc_buffers(self) -> None:
        g, B = self.g, self.batch
        self.fc_ksplit = self._fc_split()
        nodes = g.nodes
        first_def, last_use = {g.input: -1}, {}
        for i, n in enumerate(nodes):
            for o in node_outputs(n):
                first_def.setdefault(o, i)
            for src in (n.inp, getattr(n, "residual", None)):
                if src:
                    last_use[src] = i
        last_use[g.logits] = len(nodes)
        # A fused pair (first, second) runs as ONE kernel at the first node's
        # position: the first node's inputs stay live through the second node, so
        # the second's output can never be handed a buffer the kernel still reads.
        index = {getattr(n, "name", None): i for i, n in enumerate(nodes)}
        pairs = {**self.conv_pools, **self.exp_red}
        for c_name, k in self.conv_pool_1x1.items():  # conv + pool + folded 1x1 end at the 1x1
            pairs[c_name] = k
            first_def[k.out] = min(first_def[k.out], index[c_name])
        if self.stem_1x1 is not None:  # the fused stem writes the folded 1x1's output at its own position
            first_def[self.stem_1x1.out] = min(first_def[self.stem_1x1.out], index[self.stem.name])
            last_use[self.stem_pool.out] = max(last_use.get(self.stem_pool.out, 0), index[self.stem_1x1.name])
        for first_name, second in pairs.items():
            first = nodes[index[first_name]]
            for src in (first.inp, getattr(first, "residual", None)):
                if src:
                    last_use[src] = max(last_use[src], index[second.name])
        # a conv group runs at its first member's position: every member's input
        # stays live through the last member
        for grp in self.conv_groups:
            for m in grp:
                last_use[m.inp] = max(last_use[m.inp], index[grp[-1].name])
        self.cbuf = {name: _r(t.c, 8) for name, t in g.tensors.items()}
        self.cbuf[g.input] = 8
        self.buf: Dict[str, torch.Tensor] = {}
        free: Dict[int, List[torch.Tensor]] = {}
        order = sorted(first_def.items(), key=lambda kv: kv[1])
        release_at: Dict[int, List[str]] = {}
        for name, lu in last_use.items():
            release_at.setdefault(lu, []).append(name)
        pending_release: List[str] = []
        idx = 0
        for step in range(-1, len(nodes) + 1):
            # tensors whose last use was before this step can be recycled
            for name in pending_release if self.reuse_buffers else []:
                if name in self._ext:  # caller-owned storage is never recycled
                    continue
                t = self.buf[name]
                free.setdefault(t.numel(), []).append(t)
            pending_release = release_at.get(step, [])
            while idx < len(order) and order[idx][1] == step:
                name = order[idx][0]
                idx += 1
                t = g.tensors[name]
                numel = B * t.h * t.w * self.cbuf[name]
                if name == g.input and self.stem is not None:
                    numel = B * t.h * (t.w + self.stem_lpad) * 8
                if name in (g.logits,):
                    # [ksplit][B][classes]: split-K partials; slice 0 holds the summed logits
                    self.logit_parts = torch.empty((self.fc_ksplit, B, t.c), device=self.device,
                                                   dtype=torch.float32)
                    self.buf[name] = self.logit_parts[0]
                    continue
                if name in self._ext:
                    assert all(t.numel() == numel and t.dtype == torch.bfloat16 for t in self._ext[name]), name
                    self.buf[name] = self._ext[name][0]
                    continue
                lst = free.get(numel)
                buf = lst.pop() if lst else torch.empty(numel, device=self.device, dtype=torch.bfloat16)
                self.buf[name] = buf
        # uint8 source slots (double-buffered: the copy stream fills slot k+1
        # while the compute stream consumes slot k)
        if self._src_tensors is not None:
            assert len(self._src_tensors) == self.src_slots
            self.srcs = list(self._src_tensors)
        else:
            self.srcs = [torch.zeros((B, self.src_hw[0], self.src_hw[1], 3), device=self.device, dtype=torch.uint8)
                         for _ in range(self.src_slots)]
        self.src = self.srcs[0]
        # one packed result tensor [2][B][5] per source slot: top-5 class ids
        # (int32) and their probabilities (fp32 bits) -> a single RCCL gather per
        # batch. Per slot, so the forward of batch k+1 may run while batch k's
        # result is still being gathered.
        if self._result_views is not None:
            assert len(self._result_views) == self.src_slots
            self.results = list(self._result_views)
        else:
            self.results = [torch.zeros((2, B, 5), device=self.device, dtype=torch.int32)
                            for _ in range(self.src_slots)]
        self._select_result(0)
        self.probs = torch.zeros((B, g.classes), device=self.device, dtype=torch.float32)

    def _select_result(self, slot: int) -> None:
        """result / top_idx / top_p name the result rows of the last-run slot (the views made
        once per slot: a serving loop selects per batch, and each tensor view was a ~60 us torch
        call next to the decode pool's threads)."""
        self.result, self.top_idx, self.top_p = _result_views(self, slot)

    def view(self, name: str) -> torch.Tensor:
        """NHWC view of a tensor buffer (for tests / debugging)."""
        t = self.g.tensors[name]
        if name == self.g.logits:
            return self.buf[name]
        if name == self.g.input and self.stem is not None:
            return self.buf[name].view(self.batch, t.h, t.w + self.stem_lpad, 8)
        return self.buf[name].view(self.batch, t.h, t.w, self.cbuf[name])

    # --------------------------------------------------------------- plan ----
    def _build_plan(self) -> None:
        from ..ops import tuning

        self.tuned: Dict[str, int] = {}
        lo, hi = 0, len(self.g.nodes)
        if self._tune_range is not None:
            idx = {n.name: i for i, n in enumerate(self.g.nodes)}
            lo = idx[self._tune_range[0]] if self._tune_range[0] else 0
            hi = idx[self._tune_range[1]] if self._tune_range[1] else len(self.g.nodes)
        active = {n.name for n in self.g.nodes[lo:hi]}
        if self.autotune and self.device.type == "cuda":
            cnodes = [n for n in self.g.nodes if isinstance(n, (Conv, Dense, FusedConv)) and n.name in active]
            convs = [self._conv_args(n) for n in cnodes]
            table = tuning.autotune(convs)
            for n, a in zip(cnodes, convs):
                self.tuned[n.name] = table.get(tuning.shape_key(a), -1)
        # grouped launches: the timed best grouped tile, or -1 where the members
        # run faster one by one on their own tuned tiles (no timing: group iff the
        # largest member's default tile has a grouped instantiation)
        self.group_cfg: Dict[str, int] = {}
        for grp in self.conv_groups:
            convs = [m for m in grp if not isinstance(m, Pool)]
            args = [self._conv_args(m) for m in convs]
            pools = [self._pool_args(m) for m in grp if isinstance(m, Pool)]
            cfgs = [self.cfg_overrides.get(m.name, self.tuned.get(m.name, -1)) for m in convs]
            if any(m.name in self.cfg_overrides for m in grp):
                cfg = -1
            elif self.autotune and self.device.type == "cuda" and grp[0].name in active:
                cfg = tuning.autotune_group(args, cfgs, pools)
            else:
                big = max(range(len(args)), key=lambda i: args[i].N * args[i].Ho * args[i].Wo * args[i].Cout
                          * args[i].Kpad)
                c = cfgs[big] if cfgs[big] >= 0 else self.lib.dml_conv_pick_cfg(C.byref(args[big]))
                cfg = c if c in tuning.GROUP_CFGS else -1
            if cfg >= 0:
                self.group_cfg[grp[0].name] = cfg
        self.plans = []
        for i in range(self.src_slots):
            for name, ts in self._ext.items():
                self.buf[name] = ts[i]
            self.plans.append(self._build_one_plan(self.srcs[i], self.results[i],
                                                   self.src_index[i] if self.src_index is not None else None))
        for name, ts in self._ext.items():
            self.buf[name] = ts[0]
        self.plan = self.plans[0]
        self.graph_captured = [False] * self.src_slots

    def _build_one_plan(self, src: torch.Tensor, result: torch.Tensor, idx: Optional[torch.Tensor] = None):
        g, B, L = self.g, self.batch, self.lib
        idx_ptr = idx.data_ptr() if idx is not None else None
        plan = L.dml_plan_create()
        self.op_names: List[str] = []
        self.op_cfg: Dict[str, int] = {}
        mode = 0 if g.preprocess == "caffe" else 1
        skip = set()
        if self.stem_pool is not None:
            s, p = self.stem, self.stem_pool
            wk, bias, _, kpad, _ = self.wdev[s.name]
            hc, wc, _ = g.shape(s.out)
            ho, wo, _ = g.shape(p.out)
            y = self.buf[p.out].data_ptr() + 2 * p.out_coff  # may be a channel slice (shortcut merge)
            sa = N.StemArgs(src.data_ptr(), wk.data_ptr(), bias.data_ptr(), y, B,
                            self.src_hw[0], self.src_hw[1], g.input_hw[0], g.input_hw[1], mode, kpad, hc, wc,
                            ho, wo, self.cbuf[p.out])
            k = self.stem_1x1
            if k is not None:
                w4, b4, _, kp4, _ = self.wdev[k.name]
                sa.w4, sa.b4, sa.z, sa.c4, sa.ldw4, sa.ldz = (w4.data_ptr(), b4.data_ptr(), self.buf[k.out].data_ptr(),
                                                              k.cout, kp4, self.cbuf[k.out])
            sa.idx = idx_ptr
            N.check(L.dml_plan_add_stem(plan, C.byref(sa)), "plan stem")
            self._keep.append(sa)
            self.op_names.append(f"preprocess+{s.name}+{p.name}" + (f"+{k.name}" if k is not None else ""))
            skip = {s.name, p.name} | ({k.name} if k is not None else set())
        elif self.stem_conv2 is not None:
            s, c = self.stem, self.stem_conv2
            w1, b1, _, kp1, _ = self.wdev[s.name]
            w2, b2, _, kp2, _ = self.wdev[c.name]
            h1, wd1, _ = g.shape(s.out)
            h2, wd2, _ = g.shape(c.out)
            ia = N.IncStemArgs(src.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
                               self.buf[c.out].data_ptr() + 2 * c.out_coff, B, self.src_hw[0], self.src_hw[1],
                               g.input_hw[0], g.input_hw[1], mode, kp1, kp2, h1, wd1, h2, wd2, self.cbuf[c.out])
            ia.idx = idx_ptr
            N.check(L.dml_plan_add_inc_stem(plan, C.byref(ia)), "plan inception stem")
            self.op_names.append(f"preprocess+{s.name}+{c.name}")
            skip = {s.name, c.name}
        else:
            pa = N.PreprocArgs(src.data_ptr(), self.buf[g.input].data_ptr(), B, self.src_hw[0], self.src_hw[1],
                               g.input_hw[0], g.input_hw[1], mode, int(self.stem is not None), self.stem_lpad)
            pa.idx = idx_ptr
            N.check(L.dml_plan_add_preprocess(plan, C.byref(pa)), "plan preprocess")
            self.op_names.append("preprocess")
        skip |= {p.name for p in self.conv_pools.values()}
        skip |= {k.name for k in self.conv_pool_1x1.values()}
        skip |= {r.name for r in self.exp_red.values()}
        groups = {grp[0].name: grp for grp in self.conv_groups if grp[0].name in self.group_cfg}
        for grp in groups.values():
            skip |= {m.name for m in grp[1:]}
        for n in g.nodes:
            if n.name in skip:
                continue
            if n.name in groups:
                grp, cfg = groups[n.name], self.group_cfg[n.name]
                ga = N.ConvGroupArgs()
                convs = [m for m in grp if not isinstance(m, Pool)]
                pools = [m for m in grp if isinstance(m, Pool)]
                ga.n, ga.npool = len(convs), len(pools)
                for i, m in enumerate(convs):
                    ga.a[i] = self._conv_args(m)
                for i, m in enumerate(pools):
                    ga.pool[i] = self._pool_args(m)
                N.check(L.dml_plan_add_conv_group(plan, C.byref(ga), cfg), f"plan conv group {n.name}")
                for m in grp:
                    self.op_cfg[m.name] = cfg
                self._keep.append(ga)
                self.op_names.append("|".join(m.name for m in grp))
                continue
            if n.name in self.exp_red:
                r = self.exp_red[n.name]
                w3, b3, _, kp3, _ = self.wdev[n.name]
                w1, b1, _, kp1, _ = self.wdev[r.name]
                h, w, _ = g.shape(n.out)
                res = self.buf[n.residual].data_ptr() if n.residual else None
                ldr = self.cbuf[n.residual] if n.residual else 0
                ea = N.ExpandReduceArgs(self.buf[n.inp].data_ptr(), w3.data_ptr(), b3.data_ptr(),
                                        res, self.buf[n.out].data_ptr() + 2 * n.out_coff,
                                        w1.data_ptr(), b1.data_ptr(), self.buf[r.out].data_ptr(), B * h * w,
                                        self.cbuf[n.inp], kp3, ldr, self.cbuf[n.out], kp1,
                                        self.cbuf[r.out], n.cout, n.cin)
                ea.fz = r.cout
                if n.out in self.ysub:
                    ea.ysub, ea.yH, ea.yW = self.ysub[n.out], h, w
                N.check(L.dml_plan_add_expand_reduce(plan, C.byref(ea)), "plan expand+reduce")
                self.op_names.append(f"{n.name}+{r.name}")
                continue
            if n.name in self.conv_pools:
                p = self.conv_pools[n.name]
                wk, bias, _, kpad, _ = self.wdev[n.name]
                h, w, _ = g.shape(n.inp)
                ho, wo, _ = g.shape(p.out)
                k = self.conv_pool_1x1.get(n.name)
                out = k.out if k is not None else p.out
                ca = N.ConvPoolArgs(self.buf[n.inp].data_ptr(), wk.data_ptr(), bias.data_ptr(),
                                    self.buf[out].data_ptr(), B, h, w, self.cbuf[n.inp], kpad, ho, wo,
                                    self.cbuf[out])
                if k is not None:
                    w4, b4, _, kp4, _ = self.wdev[k.name]
                    ca.w4, ca.b4, ca.c4, ca.ldw4 = w4.data_ptr(), b4.data_ptr(), k.cout, kp4
                N.check(L.dml_plan_add_conv_pool(plan, C.byref(ca)), "plan conv+pool")
                self._keep.append(ca)
                self.op_names.append(f"{n.name}+{p.name}" + (f"+{k.name}" if k is not None else ""))
                continue
            if isinstance(n, (Conv, Dense, FusedConv)):
                cfg = self.cfg_overrides.get(n.name, self.tuned.get(n.name, -1))
                a = self._conv_args(n)
                used = N.check(L.dml_plan_add_conv(plan, C.byref(a), cfg), f"plan conv {n.name}")
                self.op_cfg[n.name] = used
                self._keep.append(a)
            elif isinstance(n, Pool):
                N.check(L.dml_plan_add_pool(plan, C.byref(self._pool_args(n))), "plan pool")
            elif isinstance(n, GlobalAvgPool):
                h, w, c = g.shape(n.inp)
                N.check(L.dml_plan_add_gap(plan, self.buf[n.inp].data_ptr(), self.buf[n.out].data_ptr(),
                                           B, h * w, c, self.cbuf[n.inp]), "plan gap")
            self.op_names.append(n.name)
        N.check(L.dml_plan_add_softmax_top5_split(plan, self.buf[g.logits].data_ptr(), B, g.classes, g.classes,
                                                  self.fc_ksplit, B * g.classes, self.probs.data_ptr(),
                                                  result[0].data_ptr(), result[1].data_ptr()),
                "plan softmax_top5")
        self.op_names.append("softmax_top5")
        return plan

    def _pool_args(self, n: Pool) -> N.PoolArgs:
        g = self.g
        h, w, c = g.shape(n.inp)
        ho, wo, _ = g.shape(n.out)
        y = self.buf[n.out].data_ptr() + 2 * n.out_coff
        return N.PoolArgs(self.buf[n.inp].data_ptr(), y, self.batch, h, w, c, self.cbuf[n.inp], ho, wo,
                          self.cbuf[n.out], n.k, n.stride, n.pad, 0 if n.mode == "max" else 1, int(n.relu))

    def _conv_args(self, n) -> N.ConvArgs:
        g, B = self.g, self.batch
        wk, bias, K, kpad, cin_eff = self.wdev[n.name]
        if isinstance(n, Dense):
            x = self.buf[n.inp]
            a = N.ConvArgs(x.data_ptr(), wk.data_ptr(), bias.data_ptr(), None, self.buf[n.out].data_ptr(),
                           B, 1, 1, cin_eff, self.cbuf[n.inp], 1, 1, 1, 1, 0, 0, 1, 1, n.cout, K, kpad,
                           n.cout, 0, 0, 1, 1, 1)
            if n.out == g.logits and self.fc_ksplit > 1:
                a.ksplit, a.split_ld = self.fc_ksplit, B * n.cout
            return a
        if isinstance(n, FusedConv):
            m0 = n.members[0]
            h, w, _ = g.shape(n.inp)
            ho, wo, _ = g.shape(m0.out)
            a = N.ConvArgs(self.buf[n.inp].data_ptr(), wk.data_ptr(), bias.data_ptr(), None,
                           self.buf[m0.out].data_ptr() + 2 * m0.out_coff, B, h, w, cin_eff, self.cbuf[n.inp],
                           1, 1, m0.sh, m0.sw, 0, 0, ho, wo, n.cout, K, kpad, self.cbuf[m0.out], 0, int(m0.relu), 0,
                           1, 1)
            a.nseg = len(n.members)
            c0 = 0
            for s, m in enumerate(n.members):
                a.seg_c0[s] = c0
                a.seg_ldy[s] = self.cbuf[m.out]
                a.seg_relu[s] = int(m.relu)
                a.seg_y[s] = self.buf[m.out].data_ptr() + 2 * m.out_coff
                c0 += m.cout
            return a
        h, w, _ = g.shape(n.inp)
        ho, wo, _ = g.shape(n.out)
        x = self.buf[n.inp].data_ptr() + 2 * n.in_coff
        y = self.buf[n.out].data_ptr() + 2 * n.out_coff
        res = self.buf[n.residual].data_ptr() if n.residual else None
        ldr = self.cbuf[n.residual] if n.residual else 0
        kw, pw, dw, ldx = n.kw, n.pw, 1, self.cbuf[n.inp]
        if n is self.stem:  # pair-packed input: physical col = logical col + lpad, 2 taps per chunk
            kw, pw, dw, w, ldx = (n.kw + 1) // 2, n.pw - self.stem_lpad, 2, w + self.stem_lpad, 8
        a = N.ConvArgs(x, wk.data_ptr(), bias.data_ptr(), res, y, B, h, w, cin_eff, ldx,
                       n.kh, kw, n.sh, n.sw, n.ph, pw, ho, wo, n.cout, K, kpad,
                       self.cbuf[n.out], ldr, int(n.relu), int(n.out_f32), 1, dw)
        if n.residual and n.res_sub > 1 and n.residual not in self.ysub:  # strided shortcut (models/optimize.py)
            rh, rw, _ = g.shape(n.residual)
            a.rsub, a.rW, a.rHW = n.res_sub, rw, rh * rw
        return a

    # ---------------------------------------------------------------- run ----
    def op_node_span(self, i: int) -> Tuple[int, int]:
        """(first, last) graph-node index that op ``i`` of the plan covers (op names join the
        covered nodes' names with '+' / '|'; 'preprocess' counts as node 0, 'softmax_top5' as the
        last node)."""
        index: Dict[str, int] = {}
        for k, n in enumerate(self.g.nodes):
            index[n.name] = k
            for m in getattr(n, "members", []):
                index[m.name] = k
        name = self.op_names[i]
        if name in index:
            return index[name], index[name]
        ks = [index[x] for x in name.replace("|", "+").split("+") if x in index]
        if not ks:  # 'preprocess' opens the forward, 'softmax_top5' closes it
            ks = [0] if name == "preprocess" else [len(self.g.nodes) - 1]
        return min(ks), max(ks)

    def set_op_range(self, begin: int, end: int) -> None:
        """From now on ``run`` executes only plan ops [begin, end) (split-head / merged-tail
        serving: the heads stop at the merge point, the tail starts there)."""
        if not (0 <= begin <= end <= len(self.op_names)):
            raise ValueError(f"bad op range {begin}..{end} of {len(self.op_names)}")
        self.op_range = (begin, end)
        self.graph_captured = [False] * self.src_slots

    def run(self, stream=None, use_graph: bool = False, slot: int = 0) -> None:
        s = N.stream_ptr(stream)
        plan = self.plans[slot]
        self._select_result(slot)
        if self.op_range is not None:
            b, e = self.op_range
            if use_graph:
                if not self.graph_captured[slot]:
                    self.capture_parts([b, e], stream, slot)
                    self.graph_captured[slot] = True
                N.check(self.lib.dml_plan_replay_part(plan, 0, s), "plan replay_part")
            else:
                N.check(self.lib.dml_plan_run_range(plan, b, e, s), "plan run_range")
            return
        if use_graph:
            if not self.graph_captured[slot]:
                N.check(self.lib.dml_plan_capture(plan, s), "plan capture")
                self.graph_captured[slot] = True
            N.check(self.lib.dml_plan_replay(plan, s), "plan replay")
        else:
            N.check(self.lib.dml_plan_run(plan, s), "plan run")

    def select(self, slot: int) -> None:
        self._select_result(slot)

    def launch_ops(self, stream, slot: int = 0) -> Optional[List[tuple]]:
        """``run(stream, use_graph=True, slot=slot)`` as dml_launch_seq records (the graph
        replay only), or None while that slot's graph is not captured."""
        if not self.graph_captured[slot]:
            return None
        s = N.stream_ptr(stream)
        plan = int(self.plans[slot])
        if self.op_range is not None:
            return [(3, plan, 0, s, 0)]
        return [(2, plan, s, 0, 0)]

    def capture(self, stream=None) -> None:
        """Capture every source slot's forward as a hipGraph NOW, with the device
        idle, on ``stream`` — pass the stream the graphs will be replayed on.
        Serving loops call this before their first collective: a capture begun
        later, while RCCL work is in flight, can meet the process-group watchdog
        querying an event on a capturing stream (hipErrorCapturedEvent; seen with
        8 sub-batch engines in the bench). No new stream is created here: an extra
        stream shifts which HIP streams share a hardware queue, and a private
        capture stream measured the concurrent service 11 % slower."""
        if all(self.graph_captured):
            return
        torch.cuda.synchronize(self.device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        for slot in range(self.src_slots):
            if not self.graph_captured[slot]:
                if self.op_range is not None:
                    self.capture_parts(list(self.op_range), s, slot)
                else:
                    N.check(self.lib.dml_plan_capture(self.plans[slot], N.stream_ptr(s)), "plan capture")
                self.graph_captured[slot] = True
        torch.cuda.synchronize(self.device)

    def capture_parts(self, bounds: List[int], stream=None, slot: int = 0) -> None:
        """Capture the forward of source slot ``slot`` as len(bounds)-1 graphs over
        op ranges [bounds[i], bounds[i+1]) (op indices as in ``op_names``)."""
        arr = (C.c_int * len(bounds))(*bounds)
        N.check(self.lib.dml_plan_capture_parts(self.plans[slot], arr, len(bounds) - 1, N.stream_ptr(stream)),
                "plan capture_parts")

    def run_part(self, i: int, stream=None, slot: int = 0) -> None:
        N.check(self.lib.dml_plan_replay_part(self.plans[slot], i, N.stream_ptr(stream)), "plan replay_part")

    def run_from_preprocessed(self, stream=None) -> None:
        if self.stem_pool is not None or self.stem_conv2 is not None:
            raise RuntimeError("the fused stem reads the uint8 source; build the Engine with fuse_stem=False")
        N.check(self.lib.dml_plan_run_range(self.plan, 1, -1, N.stream_ptr(stream)), "plan run_range")

    def infer(self, images_u8: torch.Tensor, stream=None):
        """images_u8: [B, Hs, Ws, 3] uint8 (any device). Returns (top_idx, top_p) on device."""
        if self.src_index is not None:
            raise RuntimeError("infer: this engine reads an arena through its index table; fill it and run()")
        self.src.copy_(images_u8, non_blocking=True)
        self.run(stream)
        return self.top_idx, self.top_p

    def time_ops(self, stream=None) -> List[Tuple[str, float]]:
        n = len(self.op_names)
        arr = (C.c_float * n)()
        N.check(self.lib.dml_plan_time_ops(self.plan, N.stream_ptr(stream), arr, n), "time_ops")
        return list(zip(self.op_names, list(arr)))

    def __del__(self):
        try:
            for p in getattr(self, "plans", []):
                self.lib.dml_plan_destroy(p)
            self.plans = []
            self.plan = None
        except Exception:
            pass


# Split-head / merged-tail serving (SplitEngine(merge_at=...)): the first node of the full-batch
# tail per model (None: two half-batch engines end to end). Measured slower for both models
# (profiles/r3_v7, interleaved on one box: InceptionV3 b128 46.4k merged from mixed4 / 47.6k from
# mixed8 vs 48.3-48.5k; ResNet50 b256 82.2k from stage 4 / 86.2k from stage 5 vs 90.0-90.3k): the
# caller's stream then runs a head AND the tail per batch while the extra stream runs one head, so
# the two streams no longer carry equal work. Kept as an option. DML_MERGE_AT overrides it:
# "InceptionV3=<node>,ResNet50=<node>" (a model left out keeps its default), "0" = off for all.
MERGE_AT: Dict[str, Optional[str]] = {"ResNet50": None, "InceptionV3": None}


def _result_views(eng, slot: int) -> tuple:
    """(result, top-5 ids, top-5 probs as fp32) of ``eng.results[slot]``, cached per slot (the
    cache follows the tensor object, so a replaced result tensor gets new views)."""
    cache = eng.__dict__.setdefault("_views", {})
    r = eng.results[slot]
    hit = cache.get(slot)
    if hit is None or hit[0] is not r:
        hit = cache[slot] = (r, r[0], r[1].view(torch.float32))
    return hit


def _extra_stream(device) -> "torch.cuda.Stream":
    """A sub-batch stream of a SplitEngine, at the caller's stream priority (a higher one
    for the extra streams measured 5 % slower)."""
    return torch.cuda.Stream(device, priority=serve_stream_priority())


def serve_stream_priority() -> int:
    """DML_SERVE_STREAM_PRIO (A/B; default 0 = the default priority): the priority of the
    serving engines' streams, e.g. -1 (high) to run the model ahead of the GPU JPEG decodes
    sharing the device in a store-image pass."""
    return int(os.environ.get("DML_SERVE_STREAM_PRIO", "0"))


def merge_point(model: str) -> Optional[str]:
    env = os.environ.get("DML_MERGE_AT")
    if env is None:
        return MERGE_AT.get(model)
    if env.strip() in ("", "0"):
        return None
    for item in env.split(","):
        k, _, v = item.partition("=")
        if k.strip() == model:
            return v.strip() or None
    return MERGE_AT.get(model)


class SplitEngine:
    """The per-worker batch served as ``splits`` sub-batches, each its own
    Engine (own activations, own hipGraph) on its own HIP stream, all sharing
    one set of resident weights. ``run(stream)`` forks from ``stream`` and joins
    back into it, so callers see one batch on one stream; inside, one
    sub-batch's memory-bound layers overlap the other's compute-bound ones and
    each kernel's tail is filled (measured: ResNet50 b256 +7 %, InceptionV3
    b128 +5 %, profiles/r1_v5/overlap_*.json). Same interface as Engine for
    the serving pipeline: srcs, result, batch, src_slots, device, run."""

    def __init__(self, graph: Graph, weights: Weights, batch: int, device: str = "cuda", splits: int = 2,
                 src_slots: int = 1, src_hw: Optional[Tuple[int, int]] = None, streams: int = 0,
                 merge_at: Optional[str] = None, src_tensors: Optional[List[torch.Tensor]] = None,
                 src_index: Optional[List[torch.Tensor]] = None, result_views: Optional[List[torch.Tensor]] = None,
                 **kw):
        """``streams``: concurrent streams (default = splits); sub-batch i runs on
        stream i % streams, so splits=4, streams=2 runs two half-size sub-batches
        back to back on each of two streams (smaller per-layer working sets that
        stay in the 256 MiB Infinity Cache between producer and consumer).
        ``merge_at`` (a node name of the optimized graph; splits = 2): split head, merged
        tail — the two half-batch engines run the graph up to that node on two streams and
        ONE full-batch engine runs the rest (the late, small-grid layers at twice the grid),
        see ``_init_merged``. ``src_tensors`` / ``src_index`` / ``result_views``: as
        Engine's, for the whole batch (with ``src_index`` every sub-batch engine reads the
        full source tensor through its rows of the index table)."""
        if batch % splits:
            raise ValueError(f"batch {batch} not divisible by splits {splits}")
        sub = batch // splits
        self.batch, self.splits, self.src_slots = batch, splits, src_slots
        self.nstreams = max(1, min(streams or splits, splits))
        self.device = torch.device(device)
        hw = src_hw or graph.input_hw
        self.srcs = (list(src_tensors) if src_tensors is not None else
                     [torch.zeros((batch, hw[0], hw[1], 3), device=self.device, dtype=torch.uint8)
                      for _ in range(src_slots)])
        self.src = self.srcs[0]
        self.src_index = src_index
        self.results = (list(result_views) if result_views is not None else
                        [torch.zeros((2, batch, 5), device=self.device, dtype=torch.int32)
                         for _ in range(src_slots)])
        self._select_result(0)
        self.tails: List[Engine] = []
        if merge_at:
            self._init_merged(graph, weights, hw, merge_at, kw)
            return
        self.engines: List[Engine] = []
        for i in range(splits):
            rows = slice(i * sub, (i + 1) * sub)
            self.engines.append(Engine(graph, weights if i == 0 else None, batch=sub, device=device,
                                       src_slots=src_slots, src_hw=hw, share=self.engines[0] if i else None,
                                       **self._sub_src(rows), result_views=[r[:, rows] for r in self.results],
                                       **kw))
        self.g = self.engines[0].g
        # stream 0 is the caller's stream: only nstreams-1 extra streams.
        # Measured in the serving pipeline (copy / compute / dispatch / RCCL
        # streams already live): 2 extra streams 49.1k img/s, 1 extra 58.3k.
        self.streams = [_extra_stream(self.device) for _ in range(self.nstreams - 1)]
        self._fork = torch.cuda.Event()
        self._join = [torch.cuda.Event() for _ in range(self.nstreams - 1)]

    def _sub_src(self, rows: slice) -> dict:
        """Source arguments of the sub-batch engine of ``rows``: its rows of the batch
        buffers, or (index mode) the whole source tensor + its rows of the index table."""
        if self.src_index is None:
            return {"src_tensors": [t[rows] for t in self.srcs]}
        return {"src_tensors": list(self.srcs), "src_index": [t[rows] for t in self.src_index]}

    def _init_merged(self, graph: Graph, weights: Weights, hw, merge_at: str, kw) -> None:
        """Split head, merged tail. Two half-batch HEAD engines run ops up to ``merge_at`` (the
        first tail node), one on the caller's stream and one on the extra stream; a full-batch
        TAIL engine runs the rest on the caller's stream. Every tensor live across the cut (the
        merge tensors) is stored in the tail's buffers: head i writes rows [i*B/2, (i+1)*B/2) of
        them (``Engine(ext_buffers=...)``). There is one tail engine per source slot, so the
        extra stream can run the head of batch k+1 while the caller's stream still runs the
        tail of batch k (the merge tensors are double-buffered; a head waits only for the tail
        two batches back). Motivation (InceptionV3, serial per-op times, profiles/r3_v7): the
        17x17 / 8x8 layers take 1454 us at 128 images vs 2 x 936 us at 64 — their grids are a
        few hundred tiles for 256 CUs, so a 128-image grid costs 1.55x, not 2x, a 64-image one."""
        if self.splits != 2:
            raise ValueError("merge_at needs splits = 2")
        B, sub = self.batch, self.batch // 2
        for s in range(self.src_slots):
            self.tails.append(Engine(graph, weights if s == 0 else None, batch=B, device=str(self.device),
                                     src_slots=1, src_hw=hw, share=self.tails[0] if s else None,
                                     src_tensors=[self.srcs[s]], result_views=[self.results[s]],
                                     src_index=[self.src_index[s]] if self.src_index is not None else None,
                                     tune_range=(merge_at, None), **kw))
        t0 = self.tails[0]
        g = t0.g
        names = [n.name for n in g.nodes]
        if merge_at not in names:
            raise ValueError(f"merge_at: no node {merge_at!r} in the optimized graph")
        cut = names.index(merge_at)
        self.merge_tensors = self.live_across(g, cut)

        def rows(t: Engine, name: str, i: int) -> torch.Tensor:
            per = t.buf[name].numel() // B
            return t.buf[name][i * sub * per:(i + 1) * sub * per]

        self.engines = []
        for i in range(2):
            ext = {name: [rows(self.tails[s], name, i) for s in range(self.src_slots)] for name in self.merge_tensors}
            self.engines.append(Engine(graph, None, batch=sub, device=str(self.device), src_slots=self.src_slots,
                                       src_hw=hw, share=t0, **self._sub_src(slice(i * sub, (i + 1) * sub)),
                                       result_views=[r[:, i * sub:(i + 1) * sub] for r in self.results],
                                       ext_buffers=ext, tune_range=(None, merge_at), **kw))
        for e in self.engines:
            e.set_op_range(0, self._op_cut(e, cut))
        for t in self.tails:
            t.set_op_range(self._op_cut(t, cut), len(t.op_names))
        self.g = g
        self.merge_at = merge_at
        self.streams = [_extra_stream(self.device)]
        self._fork = torch.cuda.Event()
        self._join = [torch.cuda.Event()]
        self._head_done = torch.cuda.Event()
        self._tail_done = [torch.cuda.Event() for _ in range(self.src_slots)]
        cur = torch.cuda.current_stream(self.device)
        for ev in self._tail_done:  # recorded once, so the first waits are well defined
            ev.record(cur)

    @staticmethod
    def live_across(g: Graph, cut: int) -> List[str]:
        """Tensors written before node ``cut`` and read at or after it."""
        first_def: Dict[str, int] = {}
        last_use: Dict[str, int] = {}
        for i, n in enumerate(g.nodes):
            for o in node_outputs(n):
                first_def.setdefault(o, i)
            for src in (getattr(n, "inp", None), getattr(n, "residual", None)):
                if src:
                    last_use[src] = i
        return sorted(t for t, d in first_def.items() if d < cut and last_use.get(t, -1) >= cut)

    @staticmethod
    def _op_cut(e: "Engine", cut: int) -> int:
        """Index of the first op of ``e`` at or after graph node ``cut``; no op may straddle it."""
        spans = [e.op_node_span(i) for i in range(len(e.op_names))]
        p = next((i for i, (lo, _) in enumerate(spans) if lo >= cut), len(spans))
        bad = [e.op_names[i] for i in range(len(spans)) if (i < p and spans[i][1] >= cut) or (i >= p and spans[i][0] < cut)]
        if bad:
            raise ValueError(f"merge point inside fused ops {bad}")
        return p

    @property
    def op_cfg(self) -> Dict[str, int]:
        return self.engines[0].op_cfg

    def capture(self, stream=None) -> None:
        """Capture every sub-batch engine's graphs now (Engine.capture), each on
        the stream ``run`` replays it on (``stream`` = the caller's stream)."""
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        lanes = [main] + self.streams
        for i, e in enumerate(self.engines):
            e.capture(lanes[i % self.nstreams])
        for t in self.tails:
            t.capture(main)

    def _select_result(self, slot: int) -> None:
        self.result, self.top_idx, self.top_p = _result_views(self, slot)

    def run(self, stream=None, use_graph: bool = False, slot: int = 0,
            deps: Optional[List[torch.cuda.Event]] = None) -> None:
        """Forward of source slot ``slot``; returns with ``stream`` joined on
        every sub-batch. ``deps=None``: the extra streams fork from ``stream``.
        ``deps`` = the events this forward really depends on (source slot
        filled, previous reader of this slot's result done): the extra streams
        wait on those only, so the next batch's sub-batches start as soon as
        their own inputs are ready instead of behind the caller stream's tail
        (gather / host copies of the previous batch) — no drain bubble between
        batches on the extra streams."""
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        self._select_result(slot)
        for e in self.engines:
            e._select_result(slot)
        if self.tails:
            self._run_merged(main, use_graph, slot, deps)
            return
        lanes = [main] + self.streams
        if deps is None:
            self._fork.record(main)
            deps = [self._fork]
        for s in self.streams:
            for ev in deps:
                s.wait_event(ev)
        for i in range(1, self.splits):  # extra streams' sub-batches first, then the caller's
            if i % self.nstreams:
                self.engines[i].run(lanes[i % self.nstreams], use_graph=use_graph, slot=slot)
        for i in range(0, self.splits, self.nstreams):
            self.engines[i].run(main, use_graph=use_graph, slot=slot)
        for s, ev in zip(self.streams, self._join):
            ev.record(s)
            main.wait_event(ev)

    def launch_ops(self, stream, slot: int = 0) -> Optional[List[tuple]]:
        """``run(stream, use_graph=True, slot=slot)`` (deps None) as dml_launch_seq records:
        the same event records, stream waits and graph replays in the same order; None while
        a graph is not captured. The events are created here (a torch Event's handle exists
        from its first record)."""
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        evs = [self._fork] + list(self._join) + ([self._head_done] if self.tails else [])
        for ev in evs:
            if ev.cuda_event == 0:
                ev.record(main)
        ptr = lambda ev: int(ev.cuda_event)  # noqa: E731
        sp = lambda st: int(st.cuda_stream)  # noqa: E731
        ops: List[tuple] = []
        if self.tails:
            x = self.streams[0]
            if self._tail_done[slot].cuda_event == 0:
                return None
            h1 = self.engines[1].launch_ops(x, slot)
            h0 = self.engines[0].launch_ops(main, slot)
            tl = self.tails[slot].launch_ops(main, 0)
            if h1 is None or h0 is None or tl is None:
                return None
            ops += [(0, ptr(self._fork), sp(main), 0, 0), (1, sp(x), ptr(self._fork), 0, 0),
                    (1, sp(x), ptr(self._tail_done[slot]), 0, 0)]
            ops += h1 + [(0, ptr(self._head_done), sp(x), 0, 0)]
            ops += h0 + [(1, sp(main), ptr(self._head_done), 0, 0)]
            ops += tl + [(0, ptr(self._tail_done[slot]), sp(main), 0, 0)]
            return ops
        lanes = [main] + self.streams
        ops.append((0, ptr(self._fork), sp(main), 0, 0))
        for st in self.streams:
            ops.append((1, sp(st), ptr(self._fork), 0, 0))
        for i in range(1, self.splits):
            if i % self.nstreams:
                o = self.engines[i].launch_ops(lanes[i % self.nstreams], slot)
                if o is None:
                    return None
                ops += o
        for i in range(0, self.splits, self.nstreams):
            o = self.engines[i].launch_ops(main, slot)
            if o is None:
                return None
            ops += o
        for st, ev in zip(self.streams, self._join):
            ops += [(0, ptr(ev), sp(st), 0, 0), (1, sp(main), ptr(ev), 0, 0)]
        return ops

    def select(self, slot: int) -> None:
        """The result views of source slot ``slot`` (what ``run`` selects first)."""
        self._select_result(slot)
        for e in self.engines:
            e._select_result(slot)

    def _run_merged(self, main, use_graph: bool, slot: int, deps) -> None:
        """Head 1 on the extra stream (after its inputs and the tail that last read this slot's
        merge tensors), head 0 then the merged tail on the caller's stream."""
        x = self.streams[0]
        if deps is None:
            self._fork.record(main)
            deps = [self._fork]
        for ev in deps:
            x.wait_event(ev)
        x.wait_event(self._tail_done[slot])
        self.engines[1].run(x, use_graph=use_graph, slot=slot)
        self._head_done.record(x)
        self.engines[0].run(main, use_graph=use_graph, slot=slot)
        main.wait_event(self._head_done)
        self.tails[slot].run(main, use_graph=use_graph, slot=0)
        self._tail_done[slot].record(main)

    def infer(self, images_u8: torch.Tensor, stream=None):
        if self.src_index is not None:
            raise RuntimeError("infer: this engine reads an arena through its index table; fill it and run()")
        self.src.copy_(images_u8, non_blocking=True)
        self.run(stream)
        return self.top_idx, self.top_p

    def time_ops(self, stream=None) -> List[Tuple[str, float]]:
        """Per-op times of ONE sub-batch engine (ops of the split run overlap)."""
        return self.engines[0].time_ops(stream)
