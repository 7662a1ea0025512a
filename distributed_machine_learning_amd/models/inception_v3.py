"""InceptionV3 (Keras applications definition) as a layer graph.

Reference: models.py:23-26 instantiates ``tf.keras.applications.InceptionV3(
weights='imagenet')``; inputs are 299x299 'tf'-preprocessed (x/127.5 - 1,
models.py:34-38). Every ``conv2d_bn`` = Conv (no bias) + BN(scale=False, eps=1e-3)
+ ReLU. Branch outputs are written straight into the mixed block's concat buffer
at their channel offset (no concat op). AvgPool 3x3/1 'same' excludes padding from
the divisor (TF semantics). Keras parameter count: 23,851,784.
"""
from __future__ import annotations

from .graph import Conv, Dense, Graph, GlobalAvgPool, Pool, same_pad


class _B:
    def __init__(self, g: Graph):
        self.g = g
        self.n = 0

    def conv(self, x, out, filters, kh, kw, stride=1, padding="same", in_coff=0, out_coff=0, cin=None, name=None):
        g = self.g
        h, w, c = g.shape(x)
        cin = c if cin is None else cin
        if padding == "same":
            assert stride == 1
            ph, pw = same_pad(kh), same_pad(kw)
        else:
            ph = pw = 0
        ho = (h + 2 * ph - kh) // stride + 1
        wo = (w + 2 * pw - kw) // stride + 1
        if out not in g.tensors:
            g.tensor(out, ho, wo, filters)
        self.n += 1
        nm = name or f"conv2d_{self.n}"
        g.add(Conv(nm, x, out, cin, filters, kh, kw, stride, stride, ph, pw, in_coff=in_coff, out_coff=out_coff,
                   bias=False, bn=True, bn_scale=False, bn_eps=1e-3, relu=True))
        return out


def build_inception_v3(classes: int = 1000) -> Graph:
    g = Graph(name="InceptionV3", input_hw=(299, 299), preprocess="tf", classes=classes)
    g.tensor("input", 299, 299, 3)
    b = _B(g)
    x = b.conv("input", "stem1", 32, 3, 3, stride=2, padding="valid")    # 149
    x = b.conv(x, "stem2", 32, 3, 3, padding="valid")                     # 147
    x = b.conv(x, "stem3", 64, 3, 3)                                      # 147
    g.tensor("stem_pool1", 73, 73, 64)
    g.add(Pool("max_pooling2d_1", x, "stem_pool1", "max", 3, 2, 0))
    x = b.conv("stem_pool1", "stem4", 80, 1, 1, padding="valid")          # 73
    x = b.conv(x, "stem5", 192, 3, 3, padding="valid")                    # 71
    g.tensor("stem_pool2", 35, 35, 192)
    g.add(Pool("max_pooling2d_2", x, "stem_pool2", "max", 3, 2, 0))
    x = "stem_pool2"

    # mixed 0, 1, 2: 35x35
    for i, pool_c in enumerate([32, 64, 64]):
        out = g.tensor(f"mixed{i}", 35, 35, 224 + pool_c)
        b.conv(x, out, 64, 1, 1, out_coff=0)
        t = b.conv(x, f"mixed{i}_b5_1", 48, 1, 1)
        b.conv(t, out, 64, 5, 5, out_coff=64)
        t = b.conv(x, f"mixed{i}_b3_1", 64, 1, 1)
        t = b.conv(t, f"mixed{i}_b3_2", 96, 3, 3)
        b.conv(t, out, 96, 3, 3, out_coff=128)
        h, w, c = g.shape(x)
        p = g.tensor(f"mixed{i}_pool", h, w, c)
        g.add(Pool(f"mixed{i}_avgpool", x, p, "avg", 3, 1, 1))
        b.conv(p, out, pool_c, 1, 1, out_coff=224)
        x = out

    # mixed 3: 35 -> 17
    out = g.tensor("mixed3", 17, 17, 768)
    b.conv(x, out, 384, 3, 3, stride=2, padding="valid", out_coff=0)
    t = b.conv(x, "mixed3_b3_1", 64, 1, 1)
    t = b.conv(t, "mixed3_b3_2", 96, 3, 3)
    b.conv(t, out, 96, 3, 3, stride=2, padding="valid", out_coff=384)
    g.add(Pool("mixed3_maxpool", x, out, "max", 3, 2, 0, out_coff=480))
    x = out

    # mixed 4..7: 17x17
    for i, c7 in zip(range(4, 8), [128, 160, 160, 192]):
        out = g.tensor(f"mixed{i}", 17, 17, 768)
        b.conv(x, out, 192, 1, 1, out_coff=0)
        t = b.conv(x, f"mixed{i}_b7_1", c7, 1, 1)
        t = b.conv(t, f"mixed{i}_b7_2", c7, 1, 7)
        b.conv(t, out, 192, 7, 1, out_coff=192)
        t = b.conv(x, f"mixed{i}_b7d_1", c7, 1, 1)
        t = b.conv(t, f"mixed{i}_b7d_2", c7, 7, 1)
        t = b.conv(t, f"mixed{i}_b7d_3", c7, 1, 7)
        t = b.conv(t, f"mixed{i}_b7d_4", c7, 7, 1)
        b.conv(t, out, 192, 1, 7, out_coff=384)
        p = g.tensor(f"mixed{i}_pool", 17, 17, 768)
        g.add(Pool(f"mixed{i}_avgpool", x, p, "avg", 3, 1, 1))
        b.conv(p, out, 192, 1, 1, out_coff=576)
        x = out

    # mixed 8: 17 -> 8
    out = g.tensor("mixed8", 8, 8, 1280)
    t = b.conv(x, "mixed8_b3_1", 192, 1, 1)
    b.conv(t, out, 320, 3, 3, stride=2, padding="valid", out_coff=0)
    t = b.conv(x, "mixed8_b7_1", 192, 1, 1)
    t = b.conv(t, "mixed8_b7_2", 192, 1, 7)
    t = b.conv(t, "mixed8_b7_3", 192, 7, 1)
    b.conv(t, out, 192, 3, 3, stride=2, padding="valid", out_coff=320)
    g.add(Pool("mixed8_maxpool", x, out, "max", 3, 2, 0, out_coff=512))
    x = out

    # mixed 9, 10: 8x8
    for i in (9, 10):
        out = g.tensor(f"mixed{i}", 8, 8, 2048)
        b.conv(x, out, 320, 1, 1, out_coff=0)
        t = b.conv(x, f"mixed{i}_b3_1", 384, 1, 1)
        b.conv(t, out, 384, 1, 3, out_coff=320)
        b.conv(t, out, 384, 3, 1, out_coff=704)
        t = b.conv(x, f"mixed{i}_b3d_1", 448, 1, 1)
        t = b.conv(t, f"mixed{i}_b3d_2", 384, 3, 3)
        b.conv(t, out, 384, 1, 3, out_coff=1088)
        b.conv(t, out, 384, 3, 1, out_coff=1472)
        h, w, c = g.shape(x)
        p = g.tensor(f"mixed{i}_pool", h, w, c)
        g.add(Pool(f"mixed{i}_avgpool", x, p, "avg", 3, 1, 1))
        b.conv(p, out, 192, 1, 1, out_coff=1856)
        x = out

    g.tensor("avg_pool", 1, 1, 2048)
    g.add(GlobalAvgPool("avg_pool", x, "avg_pool"))
    g.tensor("logits", 1, 1, classes)
    g.add(Dense("predictions", "avg_pool", "logits", 2048, classes))
    g.validate()
    return g
