"""GPU nearest resize of a staged window (parallel/rank_backend._Pack + misc.hip
resize_nearest_kernel): every decoded image lands in its arena slot byte-identical to Pillow's
Image.resize(NEAREST); other slots untouched."""
import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu


class _Be:
    def __init__(self):
        from distributed_machine_learning_amd.parallel.rank_backend import nearest_index
        self.nearest = nearest_index
        self.freed = 0

    def pinned(self, n):
        return torch.empty(n, dtype=torch.uint8).pin_memory()

    def unpin(self, b):
        self.freed += 1


def test_pack_resize_into_slots():
    from distributed_machine_learning_amd import _native as N
    from distributed_machine_learning_amd.parallel.rank_backend import _Pack

    N.ensure_device_init()
    rng = np.random.default_rng(1)
    imgs = [rng.integers(0, 256, size=(h, 300, 3), dtype=np.uint8) for h in (169, 300, 211, 250)]
    imgs[3] = rng.integers(0, 256, size=(3, 40000, 3), dtype=np.uint8)   # column index > 32767
    for H, W in ((224, 224), (299, 299)):
        arena = torch.full((8, H, W, 3), 7, dtype=torch.uint8, device="cuda")
        be = _Be()
        p = _Pack(be, ["a", "b", "c", "d"], imgs, (H, W))
        s = torch.cuda.Stream()
        p.launch([5, 1, 6, 2], arena, s)
        s.synchronize()
        p.release()
        got = arena.cpu().numpy()
        for im, slot in zip(imgs, [5, 1, 6, 2]):
            ref = np.asarray(Image.fromarray(im).resize((W, H), Image.NEAREST))
            assert np.array_equal(got[slot], ref)
        for slot in (0, 3, 4, 7):
            assert np.all(got[slot] == 7)
        assert be.freed == 1
