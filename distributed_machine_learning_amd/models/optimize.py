"""Graph-level rewrites applied before lowering to the native plan.

1. ``conv_before_avgpool`` — Inception's pool branch is AvgPool3x3(s1, same)
   -> Conv1x1(+BN) -> ReLU. A 1x1 conv is a per-pixel linear map, so it commutes
   with spatial averaging; the folded-BN bias is constant per channel and the
   padding-excluded average of a constant is that constant. Hence
       relu(conv(avgpool(x)) + b) == relu(avgpool(conv(x) + b))
   exactly in real arithmetic. Running the conv first makes the pool touch
   ``cout`` channels instead of ``cin`` (192/256/288/768/1280/2048 -> 32..192).
2. ``fuse_sibling_1x1`` — 1x1 convs that read the same full input tensor
   (every Inception mixed block has 3-4: the 1x1 branch, the reductions of the
   5x5/3x3/7x7 branches and — after rewrite 1 — the pool branch's conv) become
   one GEMM with N = sum of their Couts whose epilogue scatters each column
   segment to its own destination (concat buffer at an offset, or a temporary).
   One read of the input, one launch, wider N.

3. ``push_stride_up`` — a tensor whose EVERY consumer is a 1x1 stride-2 conv
   (ResNet50's stage-boundary shortcut + first reduce, conv{3,4,5}_block1_{0,1},
   reading conv{2,3,4}_blockK_out) only ever has its even pixels read. The
   producer then only computes those: a 1x1 s1 producer becomes 1x1 s2 (its own
   input gets the same treatment next iteration) and a 'same'-padded k x k s1
   producer becomes k x k s2 with the same top/left padding (output (i, j) reads
   rows 2i-p..2i+p, exactly the s1 conv's even outputs). The consumers become s1
   and the producer's shortcut is read at stride 2 (``Conv.res_sub``). For
   ResNet50 this removes 3/4 of the work of each stage's last 1x1 expand and
   3x3 conv (and 3/4 of their activation traffic) at three stage boundaries.

4. ``merge_projection_shortcut`` — a projection shortcut (1x1 conv + BN, no ReLU) is a
   linear map whose output is only added into a block's last 1x1 expand, so
       expand(x) + shortcut(s) == [W_e | W_s] . [x ; s] + (b_e + b_s)
   — one GEMM over the channel concatenation of x and s (K = F + C_s) with no
   residual. x's producer and s's producer write into one buffer at channel
   offsets 0 and F (the Inception concat mechanism) and s's other readers read
   the slice. Same MACs; the C_out-channel shortcut tensor is never written or
   read back (ResNet50: 256/512/1024/2048 channels at the four stage entries).
   Needs the folded weights: the merged conv's kernel/bias are ADDED to the
   weights dict under "<expand>+<shortcut>" (BN folded, ``bn=False``).

5. ``level_order`` — a topological re-order by ASAP level (level = 1 + the
   deepest writer of any channel range the node reads; concat tensors have
   several writers). Nodes of one level are mutually independent: InceptionV3's
   branch convs (5x5 next to 3x3, 1x7 next to 7x1, 1x3 / 3x1 / 3x3) and the
   pool-branch avg pool / reduction max pool land side by side, groupable nodes
   first, so the engine can launch each level's convs and 3x3 pools as ONE
   grouped grid (dml_conv_group). Pure re-order: outputs are unchanged.

Rewrites 1-3 keep the weights dict unchanged (members keep their names); the
fp32 oracle can execute the rewritten graph too (tests compare both forms).
"""
from __future__ import annotations

import copy
from dataclasses import replace
from typing import Dict, List, Optional

import numpy as np

from .graph import Conv, FusedConv, Graph, Pool, Tensor, node_outputs


def _consumers(g: Graph) -> Dict[str, List[object]]:
    out: Dict[str, List[object]] = {}
    for n in g.nodes:
        for src in (getattr(n, "inp", None), getattr(n, "residual", None)):
            if src:
                out.setdefault(src, []).append(n)
    return out


def conv_before_avgpool(g: Graph) -> Graph:
    g = copy.deepcopy(g)
    cons = _consumers(g)
    nodes = list(g.nodes)
    for i, p in enumerate(list(nodes)):
        if not (isinstance(p, Pool) and p.mode == "avg" and p.stride == 1 and p.out_coff == 0 and not p.relu):
            continue
        users = cons.get(p.out, [])
        if len(users) != 1 or not isinstance(users[0], Conv):
            continue
        c = users[0]
        ph, pw, pc = g.shape(p.out)
        if not (c.kh == c.kw == 1 and c.sh == c.sw == 1 and c.ph == c.pw == 0 and c.in_coff == 0
                and c.cin == pc and c.residual is None and not c.out_f32):
            continue
        tmp = f"{c.name}_prepool"
        g.tensor(tmp, ph, pw, c.cout)
        c2 = replace(c, inp=p.inp, out=tmp, out_coff=0, relu=False)
        p2 = replace(p, inp=tmp, out=c.out, out_coff=c.out_coff, relu=c.relu)
        j = nodes.index(c)
        nodes[nodes.index(p)] = c2
        nodes[j] = p2
    g.nodes = nodes
    g.validate()
    return g


def fuse_sibling_1x1(g: Graph, max_members: int = 4) -> Graph:
    g = copy.deepcopy(g)
    groups: Dict[tuple, List[Conv]] = {}
    for n in g.nodes:
        if (isinstance(n, Conv) and n.kh == n.kw == 1 and n.ph == n.pw == 0
                and n.in_coff == 0 and n.residual is None and not n.out_f32 and n.cin == g.shape(n.inp)[2]
                and n.cout % 8 == 0 and n.out_coff % 8 == 0):
            # same input and same stride (ResNet's projection shortcut + first 1x1 of a stage)
            groups.setdefault((n.inp, n.sh, n.sw), []).append(n)
    fused_of: Dict[str, FusedConv] = {}
    for (inp, _, _), ms in groups.items():
        if len(ms) < 2:
            continue
        for k in range(0, len(ms), max_members):
            chunk = ms[k:k + max_members]
            if len(chunk) < 2:
                continue
            f = FusedConv(name="+".join(m.name for m in chunk), inp=inp, cin=chunk[0].cin, members=chunk)
            for m in chunk:
                fused_of[m.name] = f
    nodes: List[object] = []
    placed = set()
    for n in g.nodes:
        f = fused_of.get(getattr(n, "name", None)) if isinstance(n, Conv) else None
        if f is None:
            nodes.append(n)
        elif f.name not in placed:
            nodes.append(f)  # at the first member's position (all inputs exist by then)
            placed.add(f.name)
    g.nodes = nodes
    g.validate()
    return g


def push_stride_up(g: Graph) -> Graph:
    g = copy.deepcopy(g)
    while True:
        cons = _consumers(g)
        prod = {o: n for n in g.nodes for o in node_outputs(n)}
        for tname, users in cons.items():
            p = prod.get(tname)
            if tname in (g.input, g.logits) or not isinstance(p, Conv) or p.out_coff or p.out_f32:
                continue
            h, w, c = g.shape(tname)
            if h % 2 or w % 2 or c != p.cout or p.sh != 1 or p.sw != 1 or p.res_sub != 1:
                continue
            if not all(isinstance(u, Conv) and u.inp == tname and u.residual != tname and u.kh == u.kw == 1
                       and u.sh == u.sw == 2 and u.ph == u.pw == 0 for u in users):
                continue
            if not (p.kh % 2 and p.kw % 2 and p.ph == p.kh // 2 and p.pw == p.kw // 2):
                continue  # only 'same'-padded odd kernels keep the even outputs at stride 2
            p.sh = p.sw = 2
            if p.residual:
                p.res_sub = 2
            g.tensors[tname] = Tensor(tname, h // 2, w // 2, c)
            for u in users:
                u.sh = u.sw = 1
            break
        else:
            break
    g.validate()
    return g


def merge_projection_shortcut(g: Graph, w: Dict[str, np.ndarray], min_cout: int = 0) -> Graph:
    from .weights import fold_conv

    g = copy.deepcopy(g)
    while True:
        cons = _consumers(g)
        prod = {o: n for n in g.nodes for o in node_outputs(n)}
        for e in g.nodes:
            if not (isinstance(e, Conv) and e.residual and e.kh == e.kw == 1 and e.sh == e.sw == 1
                    and e.ph == e.pw == 0 and e.res_sub == 1 and e.in_coff == 0 and not e.out_f32
                    and e.cout >= min_cout):
                continue
            sc, q = prod.get(e.residual), prod.get(e.inp)
            if not (isinstance(sc, Conv) and sc.kh == sc.kw == 1 and sc.sh == sc.sw == 1 and sc.ph == sc.pw == 0
                    and not sc.relu and sc.residual is None and sc.in_coff == 0 and sc.out_coff == 0
                    and not sc.out_f32 and cons.get(e.residual) == [e]):
                continue
            S, X = sc.inp, e.inp
            pS = prod.get(S)
            if not (isinstance(q, Conv) and q.out_coff == 0 and cons.get(X) == [e] and g.shape(X)[2] == e.cin
                    and isinstance(pS, (Conv, Pool)) and pS.out_coff == 0 and S != g.input
                    and g.shape(S)[:2] == g.shape(X)[:2] and g.shape(S)[2] == sc.cin
                    and all(isinstance(u, Conv) and u.inp == S and u.residual != S and u.in_coff == 0
                            for u in cons.get(S, []))):
                continue
            if e.cin % 8 or sc.cin % 8:
                continue
            ke, be = fold_conv(e, w)
            ks, bs = fold_conv(sc, w)
            name = f"{e.name}+{sc.name}"
            w[f"{name}/kernel"] = np.concatenate([ke, ks], axis=2)
            w[f"{name}/bias"] = (be + bs).astype(np.float32)
            h, wd, _ = g.shape(X)
            g.tensors[X] = Tensor(X, h, wd, e.cin + sc.cin)
            pS.out, pS.out_coff = X, e.cin
            for u in cons.get(S, []):
                if u is not sc:
                    u.inp, u.in_coff = X, e.cin
            m = replace(e, name=name, cin=e.cin + sc.cin, residual=None, bias=True, bn=False)
            g.nodes = [m if n is e else n for n in g.nodes if n is not sc]
            del g.tensors[S], g.tensors[e.residual]
            break
        else:
            break
    g.validate()
    return g


def _writes(g: Graph, n) -> List[tuple]:
    """(tensor, c0, c1) channel ranges node ``n`` writes."""
    if isinstance(n, FusedConv):
        return [(m.out, m.out_coff, m.out_coff + m.cout) for m in n.members]
    if isinstance(n, Conv):
        return [(n.out, n.out_coff, n.out_coff + n.cout)]
    if isinstance(n, Pool):
        return [(n.out, n.out_coff, n.out_coff + g.shape(n.inp)[2])]
    return [(n.out, 0, g.shape(n.out)[2])]


def _reads(g: Graph, n) -> List[tuple]:
    out = []
    if isinstance(n, Conv):
        out.append((n.inp, n.in_coff, n.in_coff + n.cin))
    else:
        out.append((n.inp, 0, g.shape(n.inp)[2]))
    if getattr(n, "residual", None):
        out.append((n.residual, 0, g.shape(n.residual)[2]))
    return out


def levels(g: Graph) -> Dict[str, int]:
    """{node name: ASAP level}; the graph input is level 0. Dependencies are
    channel-range exact: a tensor written in slices (Inception concat, ResNet's
    merged [x ; shortcut] buffer) makes a reader wait only for the writers of
    the channels it reads."""
    writers: Dict[str, List[tuple]] = {}
    for n in g.nodes:
        for t, c0, c1 in _writes(g, n):
            writers.setdefault(t, []).append((n, c0, c1))
    lv: Dict[str, int] = {}
    for n in g.nodes:  # the node order is topological: producers come first
        deps = [lv[w.name] for t, r0, r1 in _reads(g, n) for w, c0, c1 in writers.get(t, [])
                if w is not n and c0 < r1 and r0 < c1]
        lv[n.name] = 1 + max(deps, default=0)
    return lv


def groupable_conv(n) -> bool:
    """A conv the grouped launch can run: plain or sibling-fused, no residual, bf16 out."""
    return isinstance(n, (Conv, FusedConv)) and getattr(n, "residual", None) is None and not getattr(n, "out_f32", False)


def groupable_pool(n) -> bool:
    """A pool the grouped launch can run beside its level's convs (3x3, pad <= 1)."""
    return isinstance(n, Pool) and n.k == 3 and 0 <= n.pad <= 1


def groupable(n) -> bool:
    return groupable_conv(n) or groupable_pool(n)


def level_order(g: Graph) -> Graph:
    lv = levels(g)
    pos = {n.name: i for i, n in enumerate(g.nodes)}
    g = copy.copy(g)
    g.nodes = sorted(g.nodes, key=lambda n: (lv[n.name], not groupable(n), pos[n.name]))
    g.validate()
    return g


def conv_group_runs(g: Graph, exclude: set = frozenset(), max_convs: int = 4, max_pools: int = 2
                    ) -> List[List[object]]:
    """Runs of consecutive groupable nodes of one level (not in ``exclude``): at
    most ``max_convs`` convs and ``max_pools`` 3x3 pools, at least one conv and two
    members — the members of one grouped launch. Consecutive + same level makes a
    run independent in any node order."""
    lv = levels(g)
    runs: List[List[object]] = []
    run: List[object] = []

    def flush():
        if len(run) > 1 and any(groupable_conv(m) for m in run):
            runs.append(list(run))
        run.clear()

    for n in list(g.nodes) + [None]:
        ok = n is not None and groupable(n) and n.name not in exclude
        if run and ok:
            nc = sum(groupable_conv(m) for m in run) + groupable_conv(n)
            npl = sum(groupable_pool(m) for m in run) + groupable_pool(n)
            if lv[n.name] != lv[run[0].name] or nc > max_convs or npl > max_pools:
                flush()
        elif run:
            flush()
        if ok:
            run.append(n)
    return runs


def optimize(g: Graph, pool_reorder: bool = True, fuse: bool = True, stride_push: bool = True,
             weights: Optional[Dict[str, np.ndarray]] = None, shortcut_min_cout: int = 0) -> Graph:
    if stride_push:
        g = push_stride_up(g)
    if weights is not None:  # adds the merged convs' folded weights to `weights`
        g = merge_projection_shortcut(g, weights, shortcut_min_cout)
    if pool_reorder:
        g = conv_before_avgpool(g)
    if fuse:
        g = fuse_sibling_1x1(g)
    return g
