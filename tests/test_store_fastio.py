"""Batched native file reads of the image store's local fast path (store/fastio.read_many,
csrc/host/store_io.cpp dml_read_many): contents, empty files, order, missing-file errors."""
import os

import pytest

from distributed_machine_learning_amd.store import fastio


def test_read_many_contents_and_errors(tmp_path):
    paths, want = [], []
    for i in range(7):
        p = tmp_path / f"img{i}.jpeg"
        data = bytes((i * 31 + j) & 255 for j in range(i * 997))   # includes an empty file
        p.write_bytes(data)
        paths.append(str(p))
        want.append(data)
    got = fastio.read_many(paths[::-1])
    assert [bytes(m) for m in got] == want[::-1]
    with pytest.raises(OSError):
        fastio.read_many([paths[0], os.path.join(str(tmp_path), "missing.jpeg")])
