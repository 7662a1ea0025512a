"""Layer-graph IR for the CNN classifiers.

A model is an ordered list of nodes over named NHWC tensors (per image: H, W, C).
The same IR drives two executors:

* ``models.oracle``  — plain-PyTorch fp32 NCHW, BatchNorm applied unfused (the
  numerics reference for every test);
* ``models.engine``  — the MI355X executor: BN folded into bf16 weights, every
  node lowered to a hand-written gfx950 kernel launch recorded in the native plan.

Channel concatenation (Inception) is not a node: a conv/pool writes into its
destination tensor at ``out_coff`` (the kernel's channel-offset store), and a node
may read a channel slice of a tensor through ``in_coff``/``cin``.

Reference parity: the reference never defines layers itself — it instantiates
``tf.keras.applications.ResNet50/InceptionV3`` (models.py:26, models.py:51). The
graphs in ``resnet50.py`` / ``inception_v3.py`` transcribe those Keras definitions.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple


@dataclass
class Tensor:
    name: str
    h: int
    w: int
    c: int  # total channels of the buffer (concat buffers hold all branches)


@dataclass
class Conv:
    name: str
    inp: str
    out: str
    cin: int
    cout: int
    kh: int
    kw: int
    sh: int = 1
    sw: int = 1
    ph: int = 0
    pw: int = 0
    in_coff: int = 0
    out_coff: int = 0
    bias: bool = True          # conv has its own bias term
    bn: bool = True            # followed by BatchNorm
    bn_scale: bool = True      # BN has gamma (Inception uses scale=False)
    bn_eps: float = 1e-3
    relu: bool = True
    residual: Optional[str] = None  # tensor added before the ReLU (ResNet shortcut)
    out_f32: bool = False
    res_sub: int = 1           # residual read at this stride from its full-resolution grid


@dataclass
class Pool:
    name: str
    inp: str
    out: str
    mode: str      # "max" | "avg"
    k: int = 3
    stride: int = 2
    pad: int = 0   # symmetric; max: zero pad == ignored (inputs are post-ReLU), avg: excluded
    out_coff: int = 0
    relu: bool = False  # ReLU after pooling (set when a 1x1 conv is moved in front of an avg pool)


@dataclass
class FusedConv:
    """Sibling 1x1 convs that read the same input, run as one GEMM whose output
    channels are scattered to each member's destination (models/optimize.py)."""
    name: str
    inp: str
    cin: int
    members: List["Conv"] = field(default_factory=list)

    @property
    def out(self) -> str:
        return self.members[0].out

    @property
    def outs(self) -> List[str]:
        return [m.out for m in self.members]

    @property
    def cout(self) -> int:
        return sum(m.cout for m in self.members)


@dataclass
class GlobalAvgPool:
    name: str
    inp: str
    out: str


@dataclass
class Dense:
    name: str
    inp: str
    out: str
    cin: int
    cout: int


@dataclass
class Graph:
    name: str
    input_hw: Tuple[int, int]
    preprocess: str  # "caffe" | "tf"
    tensors: Dict[str, Tensor] = field(default_factory=dict)
    nodes: List[object] = field(default_factory=list)
    input: str = "input"
    logits: str = "logits"
    classes: int = 1000

    # ---- builder helpers ----
    def tensor(self, name: str, h: int, w: int, c: int) -> str:
        if name in self.tensors:
            t = self.tensors[name]
            assert (t.h, t.w, t.c) == (h, w, c), f"tensor {name} redefined {t} vs {(h, w, c)}"
        else:
            self.tensors[name] = Tensor(name, h, w, c)
        return name

    def shape(self, name: str) -> Tuple[int, int, int]:
        t = self.tensors[name]
        return t.h, t.w, t.c

    def add(self, node):
        self.nodes.append(node)
        return node

    def conv_nodes(self) -> List[Conv]:
        return [n for n in self.nodes if isinstance(n, Conv)]

    def param_count(self) -> int:
        """Parameters as Keras counts them (conv kernel+bias, BN gamma/beta/mean/var, dense)."""
        total = 0
        for n in self.nodes:
            if isinstance(n, Conv):
                total += n.kh * n.kw * n.cin * n.cout + (n.cout if n.bias else 0)
                if n.bn:
                    total += n.cout * (4 if n.bn_scale else 3)
            elif isinstance(n, Dense):
                total += n.cin * n.cout + n.cout
        return total

    def macs_per_image(self) -> int:
        total = 0
        for n in self.nodes:
            if isinstance(n, Conv):
                ho, wo, _ = self.shape(n.out)
                total += ho * wo * n.cout * n.kh * n.kw * n.cin
            elif isinstance(n, Dense):
                total += n.cin * n.cout
        return total

    def validate(self) -> None:
        produced = {self.input}
        for n in self.nodes:
            src = getattr(n, "inp")
            assert src in produced, f"{n.name}: input {src} not yet produced"
            if isinstance(n, Conv):
                h, w, c = self.shape(n.inp)
                ho, wo, co = self.shape(n.out)
                assert n.in_coff + n.cin <= c, n.name
                assert n.out_coff + n.cout <= co, n.name
                eh = (h + 2 * n.ph - n.kh) // n.sh + 1
                ew = (w + 2 * n.pw - n.kw) // n.sw + 1
                assert (eh, ew) == (ho, wo), f"{n.name}: spatial {(eh, ew)} != {(ho, wo)}"
                if n.residual:
                    rs = n.res_sub
                    assert n.residual in produced and self.shape(n.residual)[:2] == (ho * rs, wo * rs), n.name
            elif isinstance(n, Pool):
                h, w, c = self.shape(n.inp)
                ho, wo, co = self.shape(n.out)
                eh = (h + 2 * n.pad - n.k) // n.stride + 1
                assert eh == ho, f"{n.name}: {eh} != {ho}"
                assert n.out_coff + c <= co, n.name
            produced.update(node_outputs(n))
        assert self.logits in produced


def node_outputs(n) -> List[str]:
    return list(n.outs) if isinstance(n, FusedConv) else [n.out]


def same_pad(k: int) -> int:
    """Keras 'same' padding for stride 1 and odd kernels (symmetric)."""
    assert k % 2 == 1
    return k // 2
