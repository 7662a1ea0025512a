"""The GPU nearest resize of the store path (misc.hip resize_nearest_kernel) gathers with
index tables computed on the host (parallel/rank_backend.nearest_index); they must reproduce
Pillow's Image.resize(NEAREST) — Keras load_img(target_size) — byte for byte, for every source
size the store serves (here: 300 x 150-310 images to 224 and 299)."""
import numpy as np
from PIL import Image

from distributed_machine_learning_amd.parallel.rank_backend import nearest_index


def test_nearest_index_matches_pillow():
    rng = np.random.default_rng(0)
    for h in list(range(150, 311, 7)) + [224, 299, 300, 75, 17]:
        w = 300
        img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        for H, W in ((224, 224), (299, 299), (17, 40)):
            ref = np.asarray(Image.fromarray(img).resize((W, H), Image.NEAREST))
            got = img[nearest_index(h, H)[:, None], nearest_index(w, W)[None, :]]
            assert np.array_equal(ref, got), (h, w, H, W)
