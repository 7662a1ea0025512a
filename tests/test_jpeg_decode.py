"""JPEG decoder of the store-image path (csrc/kernels/jpeg_decode.hip), CPU side: the same
__host__ __device__ decode code run on the host is byte-identical to Pillow's decode
(libjpeg-turbo: islow IDCT, h2v2 fancy upsampling incl. its narrow-image box fallback, jdcolor
tables) over sizes 1x1 .. 300x300, qualities 30-95, 4:2:0 / 4:4:4 / grayscale, optimised
Huffman tables; the parser hands progressive, 4:2:2, restart-marker and truncated files to the
CPU decode; the descriptors carry Pillow's NEAREST index tables (rank_backend.nearest_index)."""
import ctypes as C
import io

import numpy as np
import pytest
from PIL import Image

from distributed_machine_learning_amd import _native as N
from distributed_machine_learning_amd.parallel.rank_backend import nearest_index
from distributed_machine_learning_amd.parallel.service_bench import make_jpegs


def _jpeg(arr: np.ndarray, mode: str = "RGB", **kw) -> bytes:
    b = io.BytesIO()
    Image.fromarray(arr).convert(mode).save(b, "JPEG", **kw)
    return b.getvalue()


def _host_decode(data: bytes):
    out = np.zeros(max(len(data) * 64, 1 << 20), np.uint8)
    hw = (C.c_int * 2)()
    rc = N.lib().dml_jpeg_decode_host(data, len(data), out.ctypes.data, hw)
    if rc != 0:
        return None
    return out[:hw[0] * hw[1] * 3].reshape(hw[0], hw[1], 3)


def _cases():
    g = np.random.default_rng(7)
    out = [(f"bench{i}", d) for i, (_, d) in enumerate(make_jpegs(24, seed=11))]
    for h, w in [(1, 1), (2, 3), (5, 5), (64, 1), (64, 2), (64, 3), (64, 5), (7, 13), (17, 33), (40, 120), (300, 169)]:
        noise = g.integers(0, 256, (h, w, 3), dtype=np.uint8)
        ramp = (np.linspace(0, 255, w)[None, :, None] * np.ones((h, 1, 3))).astype(np.uint8)
        for arr in (noise, ramp):
            for kw in (dict(quality=75), dict(quality=95, subsampling=0), dict(quality=30),
                       dict(quality=90, optimize=True)):
                out.append((f"{h}x{w} {kw}", _jpeg(arr, **kw)))
            out.append((f"{h}x{w} gray", _jpeg(arr, "L", quality=80)))
    return out


@pytest.mark.parametrize("name,data", _cases())
def test_host_decode_is_byte_identical_to_pillow(name, data):
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    got = _host_decode(data)
    if got is None:   # > 60 KiB of entropy data (the noise images at q95 4:4:4): the CPU path
        assert len(data) > 60 * 1024, name
        return
    assert got.shape == ref.shape and np.array_equal(got, ref), name


def test_unsupported_files_take_the_cpu_path():
    g = np.random.default_rng(1)
    arr = g.integers(0, 256, (48, 64, 3), dtype=np.uint8)
    good = _jpeg(arr, quality=80)
    cases = {"progressive": _jpeg(arr, quality=80, progressive=True),
             "422": _jpeg(arr, quality=80, subsampling=1),
             "truncated": good[:len(good) // 2],
             "junk": b"definitely not a jpeg"}
    for name, data in cases.items():
        assert _host_decode(data) is None, name
    L = N.lib()
    datas = [good] + list(cases.values())
    n = len(datas)
    buf = np.zeros(16 + n * L.dml_jpeg_desc_size() + sum(len(d) + 32 for d in datas) + 256, np.uint8)
    keep = [bytes(d) for d in datas]
    status = (C.c_int * n)()
    info = (C.c_long * 4)()
    used = L.dml_jpeg_prepare(n, (C.c_char_p * n)(*keep), (C.c_long * n)(*[len(d) for d in keep]), 224, 224,
                              buf.ctypes.data, len(buf), status, info)
    assert used > 0 and list(status) == [1, 0, 0, 0, 0]
    assert info[2] == 6 * 8 + 2 * 3 * 4 and 0 < info[3] < len(good)   # 4:2:0 48x64: 6x8 Y + 2 x 3x4 chroma blocks
    assert info[1] > 0 and info[0] > info[1]


def test_descriptors_carry_pillows_nearest_tables():
    L = N.lib()
    data = _jpeg(np.zeros((250, 169, 3), np.uint8), quality=80)
    buf = np.zeros(16 + L.dml_jpeg_desc_size() + len(data) + 256, np.uint8)
    status = (C.c_int * 1)()
    info = (C.c_long * 4)()
    assert L.dml_jpeg_prepare(1, (C.c_char_p * 1)(data), (C.c_long * 1)(len(data)), 299, 224, buf.ctypes.data,
                              len(buf), status, info) > 0
    # DmljImage layout: 37 int32 (+ 4 B alignment), 7 int64, 4 int32, then rowtab[320], coltab[320]
    off = 16 + 37 * 4 + 4 + 7 * 8 + 4 * 4
    row = buf[off:off + 640].view(np.int16)[:299]
    col = buf[off + 640:off + 1280].view(np.int16)[:224]
    assert np.array_equal(row, nearest_index(250, 299)) and np.array_equal(col, nearest_index(169, 224))


def _par_and_serial(data: bytes):
    cap = 1 << 22
    par = np.zeros(cap, np.int16)
    ser = np.zeros(cap, np.int16)
    info = (C.c_long * 3)()
    rc = N.lib().dml_jpeg_parallel_host(data, len(data), par.ctypes.data, ser.ctypes.data, cap, info)
    return rc, par[:info[0]], ser[:info[0]], info[1], info[2]


@pytest.mark.parametrize("name,data", _cases())
def test_parallel_entropy_decode_equals_the_serial_one(name, data):
    """The self-synchronising segment decode (jpeg_huff_par_kernel's algorithm, replayed on the
    CPU with the same __host__ __device__ code): every coefficient of every block equals the
    serial decoder's, including the DC predictions rebuilt by the prefix sum; the Jacobi rounds
    converge in a few rounds."""
    rc, par, ser, rounds, nseg = _par_and_serial(data)
    if rc == -1:
        assert len(data) > 60 * 1024 or _host_decode(data) is None, name
        return
    assert rc == 0 and par.size > 0
    assert np.array_equal(par, ser), (name, int((par != ser).sum()), rounds, nseg)
    assert rounds <= max(6, nseg), (name, rounds, nseg)
