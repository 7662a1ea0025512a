"""JPEG decode worker processes (parallel/decode_worker.py): byte-identical to the in-process
decode (= serving.inference.load_image before its resize) for RGB and grayscale JPEGs and a
PNG with alpha, undecodable bytes reported as None, concurrent callers, clean shutdown."""
import io
from concurrent.futures import ThreadPoolExecutor

import numpy as np
from PIL import Image

from distributed_machine_learning_amd.parallel.decode_worker import DecodeProcs
from distributed_machine_learning_amd.parallel.service_bench import make_jpegs


def _here(data: bytes) -> np.ndarray:
    im = Image.open(io.BytesIO(data))
    if im.mode != "RGB":
        im = im.convert("RGB")
    return np.asarray(im, dtype=np.uint8)


def _encode(arr: np.ndarray, fmt: str, mode: str) -> bytes:
    b = io.BytesIO()
    Image.fromarray(arr).convert(mode).save(b, fmt)
    return b.getvalue()


def test_decode_procs_match_in_process_decode():
    files = make_jpegs(24, seed=3)
    g = np.random.default_rng(0).integers(0, 255, (37, 51, 3), dtype=np.uint8)
    files += [("gray.jpeg", _encode(g, "JPEG", "L")), ("alpha.png", _encode(g, "PNG", "RGBA")),
              ("junk.jpeg", b"not an image at all")]
    dp = DecodeProcs(2)
    try:
        with ThreadPoolExecutor(4) as ex:   # several callers share the workers
            parts = list(ex.map(dp.decode_many, [files[i::4] for i in range(4)]))
        got = {k: v for p in parts for k, v in p.items()}
        assert set(got) == {n for n, _ in files}
        assert got["junk.jpeg"] is None
        for n, data in files:
            if n == "junk.jpeg":
                continue
            ref = _here(data)
            assert got[n].shape == ref.shape and got[n].dtype == np.uint8, n
            assert np.array_equal(got[n], ref), n
    finally:
        dp.close()
    assert all(p.poll() is not None for p in dp.procs)
