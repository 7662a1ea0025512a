"""ResNet50 (Keras applications v1 definition) as a layer graph.

Reference: models.py:48-51 instantiates ``tf.keras.applications.ResNet50(weights=
'imagenet')``; inputs are 224x224 'caffe'-preprocessed (models.py:59-63).
Structure: ZeroPad 3 -> Conv7x7/2 (+bias) -> BN -> ReLU -> ZeroPad 1
-> MaxPool 3/2; four stacks of bottleneck blocks [3, 4, 6, 3] with the stride on
the FIRST 1x1 conv and on the projection shortcut (Keras v1), every conv with
bias, BN eps 1.001e-5; GlobalAvgPool -> Dense 1000 -> softmax.
Keras parameter count: 25,636,712 (checked by tests/test_models.py).
"""
from __future__ import annotations

from .graph import Conv, Dense, Graph, GlobalAvgPool, Pool

EPS = 1.001e-5


def build_resnet50(classes: int = 1000) -> Graph:
    g = Graph(name="ResNet50", input_hw=(224, 224), preprocess="caffe", classes=classes)
    g.tensor("input", 224, 224, 3)
    g.tensor("conv1", 112, 112, 64)
    g.add(Conv("conv1_conv", "input", "conv1", 3, 64, 7, 7, 2, 2, 3, 3, bn_eps=EPS))
    g.tensor("pool1", 56, 56, 64)
    g.add(Pool("pool1_pool", "conv1", "pool1", "max", k=3, stride=2, pad=1))
    x, h, cin = "pool1", 56, 64
    for si, (filters, blocks, stride1) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]):
        stage = si + 2
        for b in range(blocks):
            stride = stride1 if b == 0 else 1
            pre = f"conv{stage}_block{b + 1}"
            ho = (h - 1) // stride + 1
            if b == 0:
                sc = g.tensor(f"{pre}_0", ho, ho, 4 * filters)
                g.add(Conv(f"{pre}_0_conv", x, sc, cin, 4 * filters, 1, 1, stride, stride, relu=False, bn_eps=EPS))
            else:
                sc = x
            t1 = g.tensor(f"{pre}_1", ho, ho, filters)
            g.add(Conv(f"{pre}_1_conv", x, t1, cin, filters, 1, 1, stride, stride, bn_eps=EPS))
            t2 = g.tensor(f"{pre}_2", ho, ho, filters)
            g.add(Conv(f"{pre}_2_conv", t1, t2, filters, filters, 3, 3, 1, 1, 1, 1, bn_eps=EPS))
            out = g.tensor(f"{pre}_out", ho, ho, 4 * filters)
            g.add(Conv(f"{pre}_3_conv", t2, out, filters, 4 * filters, 1, 1, residual=sc, relu=True, bn_eps=EPS))
            x, h, cin = out, ho, 4 * filters
    g.tensor("avg_pool", 1, 1, 2048)
    g.add(GlobalAvgPool("avg_pool", x, "avg_pool"))
    g.tensor("logits", 1, 1, classes)
    g.add(Dense("predictions", "avg_pool", "logits", 2048, classes))
    g.validate()
    return g
