"""Fused stem kernels alone, cold and warm: the ResNet50 stem (uint8 224x224 -> conv 7x7/2
-> max pool -> folded 1x1, b128), the InceptionV3 stem (uint8 299x299 -> conv 3x3/2 -> conv
3x3, b64) and the InceptionV3 conv 3x3 + pool + 1x1 kernel (147x147x32, b64), on the main
library and on variant builds (tools/build_variant.py: A/B probes).

python tools/stem_bench.py [--lib variants/libdml_x.so,...] [--iters 20] [--out f.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N  # noqa: E402


def bf(*shape, scale=0.05):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16).contiguous()


def cases():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    out = []
    # ResNet50 stem + folded conv2_block1_1
    B = 128
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev, generator=g)
    w, b = bf(64, 224), torch.zeros(64, device=dev)
    y, z = torch.empty(B, 56, 56, 64, device=dev, dtype=torch.bfloat16), torch.empty(B, 56, 56, 64, device=dev,
                                                                                     dtype=torch.bfloat16)
    w4, b4 = bf(64, 64), torch.zeros(64, device=dev)
    sa = N.StemArgs(img.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), B, 224, 224, 224, 224, 0, 224,
                    112, 112, 56, 56, 64)
    sa.w4, sa.b4, sa.z, sa.c4, sa.ldw4, sa.ldz = w4.data_ptr(), b4.data_ptr(), z.data_ptr(), 64, 64, 64
    out.append(("resnet_stem_b128", "dml_stem_resnet", sa, (img, w, b, y, z, w4, b4)))
    sn = N.StemArgs(img.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), B, 224, 224, 224, 224, 0, 224,
                    112, 112, 56, 56, 64)
    out.append(("resnet_stem_no1x1", "dml_stem_resnet", sn, (img, w, b, y)))
    # the serving form: images read from a 4x larger arena through an index table, the table
    # in pinned host memory (GpuRankBackend) or in device memory
    arena = torch.randint(0, 256, (4 * B, 224, 224, 3), dtype=torch.uint8, device=dev, generator=g)
    perm = torch.randperm(4 * B, generator=torch.Generator().manual_seed(1))[:B].to(torch.int32)
    for where, t in (("host", perm.pin_memory()), ("dev", perm.to(dev))):
        sb = N.StemArgs(arena.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), B, 224, 224, 224, 224, 0, 224,
                        112, 112, 56, 56, 64)
        sb.w4, sb.b4, sb.z, sb.c4, sb.ldw4, sb.ldz = w4.data_ptr(), b4.data_ptr(), z.data_ptr(), 64, 64, 64
        sb.idx = t.data_ptr()
        out.append((f"resnet_stem_idx_{where}", "dml_stem_resnet", sb, (arena, t, w, b, y, z, w4, b4)))
    # InceptionV3 stem
    B = 64
    img2 = torch.randint(0, 256, (B, 299, 299, 3), dtype=torch.uint8, device=dev, generator=g)
    w1, b1, w2, b2 = bf(32, 64), torch.zeros(32, device=dev), bf(32, 288), torch.zeros(32, device=dev)
    y2 = torch.empty(B, 147, 147, 32, device=dev, dtype=torch.bfloat16)
    ia = N.IncStemArgs(img2.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), y2.data_ptr(),
                       B, 299, 299, 299, 299, 1, 64, 288, 149, 149, 147, 147, 32)
    out.append(("inception_stem_b64", "dml_stem_inception", ia, (img2, w1, b1, w2, b2, y2)))
    # InceptionV3 conv2d_3 (3x3 same 32 -> 64) + max pool 3x3/2 + folded conv2d_4 (1x1 64 -> 80)
    x3 = bf(B, 147, 147, 32, scale=1.0)
    w3, b3 = bf(64, 288), torch.zeros(64, device=dev)
    w5, b5 = bf(80, 64), torch.zeros(80, device=dev)
    y3 = torch.empty(B, 73, 73, 80, device=dev, dtype=torch.bfloat16)
    ca = N.ConvPoolArgs(x3.data_ptr(), w3.data_ptr(), b3.data_ptr(), y3.data_ptr(), B, 147, 147, 32, 288, 73, 73, 80)
    ca.w4, ca.b4, ca.c4, ca.ldw4 = w5.data_ptr(), b5.data_ptr(), 80, 64
    out.append(("inc_convpool_b64", "dml_conv3x3_pool", ca, (x3, w3, b3, w5, b5, y3)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    N.ensure_device_init()
    libs = [("main", N.lib())]
    for p in [x for x in a.lib.split(",") if x]:
        L2 = C.CDLL(p)
        L2.dml_conv_v2_init()
        libs.append((os.path.basename(p), L2))
    scrub = torch.zeros(128 << 20, device="cuda")
    s = N.stream_ptr()
    rows = []
    for name, fn, args, keep in cases():
        row = {"kernel": name, "us": {}}
        for ln, L in libs:
            f = getattr(L, fn)

            def run():
                rc = f(C.byref(args), C.c_void_p(s))
                if rc != 0:
                    raise RuntimeError(f"{ln}:{fn} rc {rc}")
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            e1.synchronize()
            warm = e0.elapsed_time(e1) / a.iters * 1e3
            cold = 0.0
            for _ in range(a.iters):
                scrub.add_(1.0)
                e0.record()
                run()
                e1.record()
                e1.synchronize()
                cold += e0.elapsed_time(e1)
            row["us"][ln] = {"warm": round(warm, 2), "cold": round(cold / a.iters * 1e3, 2)}
        rows.append(row)
        print(f"{name:22s} " + "  ".join(f"{k} {v['warm']:.1f}/{v['cold']:.1f}" for k, v in row["us"].items()),
              flush=True)
    if a.out:
        with open(a.out, "w") as fo:
            json.dump(rows, fo, indent=1)


if __name__ == "__main__":
    main()
