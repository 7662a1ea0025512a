"""Per-rank inference backends of the collective service (parallel/service.py).

A backend runs one batch (a list of image names) of one model on this rank:
``launch(model, names, slot)`` returns ``(rows, event)`` where ``rows`` is a
[2, cap, 5] int32 tensor (top-5 class ids; the fp32 probabilities bit-cast into
the second plane) that is valid once ``event`` has fired (``None`` = already
valid). Rows of images that could not be fetched or decoded carry class id -1.
GPU backends launch asynchronously into one of ``SLOTS`` result slots and copy
the rows into pinned host memory in stream order, so the service polls an
event instead of waiting on the GPU.

Image names: ``synthetic:<i>`` (seeded arena images), ``<name>`` or
``<name>@<version>`` (a store image pinned to one version by the coordinator at
submit time, so a later PUT of a new version never changes what a queued job
reads; reference worker.py:1323-1366 fetched the latest version at task time).
"""
from __future__ import annotations

import hashlib
import logging
import os
import time
from collections import OrderedDict
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..serving.jobs import MODELS, SYNTH, SynthNames
from ..serving.output import VERSION_SEP

log = logging.getLogger(__name__)
MODEL_IDS = {m: i for i, m in enumerate(MODELS)}
SLOTS = 2   # batches a GPU rank has launched at once (engine source / result slots)


def synthetic_names(n: int) -> SynthNames:
    """SYNTH + str(i), i < n, as a lazy sequence (serving/jobs.SynthNames)."""
    return SynthNames(0, n)


def split_version(name: str) -> Tuple[str, Optional[int]]:
    """'3.jpeg@2' -> ('3.jpeg', 2); '3.jpeg' -> ('3.jpeg', None)."""
    head, sep, tail = name.rpartition(VERSION_SEP)
    if sep and tail.isdigit():
        return head, int(tail)
    return name, None


class RankBackend:
    cap: int = 256
    device = torch.device("cpu")
    slots: int = SLOTS      # batches launched at once (GPU: the engines' source / result slots)

    def launch(self, model: str, names: Sequence[str], slot: int):
        raise NotImplementedError

    def run(self, model: str, names: Sequence[str]) -> torch.Tensor:
        res, ev = self.launch(model, names, 0)
        if ev is not None:
            ev.synchronize()
        self.finalize(0)
        return res

    def _launch_ops(self, model: str, slot: int) -> Optional[np.ndarray]:
        """(model, slot)'s launch after the window waits, as dml_launch_seq records: the index
        fetch, the engine's replays (Engine/SplitEngine.launch_ops), the slot's done event.
        Built once; None (the Python path) while a graph is not captured."""
        key = (model, slot)
        ops = self._lops.get(key)
        if ops is None:
            eng, s = self.engines[model], self.stream
            sp = int(s.cuda_stream)
            eo = eng.launch_ops(s, slot)
            if eo is None:
                return None
            if self.ev_done[slot].cuda_event == 0:
                self.ev_done[slot].record(s)
            hidx, didx = self.idx[model][slot], self.idx_dev[model][slot]
            rows = [(4, hidx.data_ptr(), didx.data_ptr(), eng.batch, sp)] + eo + \
                [(0, int(self.ev_done[slot].cuda_event), sp, 0, 0)]
            ops = self._lops[key] = np.asarray(rows, np.int64)
        return ops

    def finalize(self, slot: int) -> None:
        """(serve loop, after the slot's launch event completed, before its rows are read)"""

    # staging hooks (parallel/image_store.py): every rank calls stage / release /
    # reset_staging at the same points of the replicated job state; backends that fetch
    # their images at launch keep these no-ops
    def attach(self, eg) -> None:
        """A new communicator epoch (group rank / size, data group)."""

    def stage(self, model: str, batches, where: Optional[Dict[tuple, int]] = None) -> bool:
        """Stage these batches' images (in order) ahead of their launch on the rank
        ``where[batch.key]`` (a GLOBAL rank: the one it was dispatched to, or its affinity);
        False if the arena could not take all of them yet."""
        return True

    def progress(self) -> None:
        """Advance staging without blocking (serve loop, every poll)."""

    def ready(self, model: str, names: Sequence[str]) -> bool:
        return True

    def release(self, model: str, key, names: Sequence[str]) -> None:
        """A batch completed: its images are no longer pinned."""

    def reset_staging(self) -> None:
        """Epoch change: forget every staged window (identically on every rank)."""

    def drain(self) -> None:
        """Wait for every launched batch (failure recovery reuses the slots)."""


class _ArenaStaging:
    """Window staging over per-model HbmImageStores (shared by StoreRankBackend and
    GpuRankBackend): decisions from the replicated state, data movement asynchronous."""

    arenas: Dict[str, "object"]
    staged: Dict[tuple, Tuple[str, List[str], int]]   # batch key -> (model, images, destination group rank)

    def _init_staging(self, loader, decode_threads: int = 8) -> None:
        from concurrent.futures import ThreadPoolExecutor

        from .image_store import Stager

        self.loader = loader
        self.staged = {}
        self.pool = ThreadPoolExecutor(max_workers=decode_threads)
        self.stager = Stager()   # one window order (one collective order) for every model's store
        self.epoch = 0

    def _adopt(self, model: str, arena) -> None:
        arena.stager = self.stager
        arena.loader = lambda ns, m=model: self._load(m, ns)

    def attach(self, eg) -> None:
        self.epoch = eg.epoch
        self.members = list(eg.members)
        self.stager.attach(eg.rank, eg.world, self.pool, eg if eg.world > 1 else None,
                           getattr(self, "stage_stream", None), poll_dead=eg._poll_dead)

    def stage(self, model, batches, where=None) -> bool:
        arena = self.arenas[model]
        members = getattr(self, "members", [0])
        for b in batches:
            g = (where or {}).get(b.key, members[0])
            dst = members.index(g) if g in members else 0
            st = self.staged.get(b.key)
            if st is not None and st[2] == dst:
                continue
            if arena.plan(b.images, self.epoch, dst) is None:
                return False  # later batches wait for completions to free arena slots
            if st is None:
                arena.pin(b.images)   # a batch re-targeted to another rank stays pinned once
            self.staged[b.key] = (model, list(b.images), dst)
        return True

    def progress(self) -> None:
        if self.stager.queue:
            self.stager.progress()

    def ready(self, model, names) -> bool:
        return self.arenas[model].ready(names)

    def release(self, model, key, names) -> None:
        st = self.staged.pop(key, None)
        if st is not None:
            self.arenas[st[0]].unpin(st[1])

    def reset_staging(self) -> None:
        self.stager.drain()
        for a in self.arenas.values():
            a.reset()
        self.staged.clear()


class HostRankBackend(RankBackend):
    """A serving.inference backend (fake / cpu) behind the rank interface:
    decode-once per image name (LRU cache), synchronous predict. The same
    backend classes as the host cluster's workers, so both serving modes produce
    identical outputs for the same images. Synthetic names decode from their own
    name bytes; failed images get class id -1 in their result row."""

    slots = 8   # synchronous: a launch has finished when it returns

    def __init__(self, backend, loader: Optional[Callable] = None, cap: int = 256, delay_per_image: float = 0.0,
                 cache_images: int = 4096):
        self.be, self.loader, self.cap, self.delay = backend, loader, cap, delay_per_image
        self.cache: "OrderedDict[Tuple[str, str], np.ndarray]" = OrderedDict()
        self.cache_images = cache_images

    def _blobs(self, names: List[str]) -> Dict[str, Optional[bytes]]:
        out = {n: n.encode() for n in names if n.startswith(SYNTH)}
        rest = [n for n in names if not n.startswith(SYNTH)]
        if rest:
            out.update(self.loader(rest) if self.loader else {n: None for n in rest})
        return out

    def launch(self, model, names, slot):
        if len(names) > self.cap:
            raise ValueError(f"batch of {len(names)} exceeds the result capacity {self.cap}")
        if self.delay:
            time.sleep(self.delay * len(names))
        missing = [n for n in dict.fromkeys(names) if (model, n) not in self.cache]
        if missing:
            blobs = self._blobs(missing)
            for n in missing:  # keyed by the full (versioned) name: a new version is a new entry
                b = blobs.get(n)
                try:
                    self.cache[(model, n)] = self.be.decode_batch(model, [b])[0] if b is not None else None
                except Exception as e:
                    log.warning("decode of %s failed: %s", n, e)
                    self.cache[(model, n)] = None
            while len(self.cache) > self.cache_images:
                self.cache.popitem(last=False)
        imgs, ok = [], []
        for i, n in enumerate(names):
            im = self.cache.get((model, n))
            if im is not None:
                self.cache.move_to_end((model, n))
                imgs.append(im)
                ok.append(i)
        out = torch.zeros((2, self.cap, 5), dtype=torch.int32)
        out[0, :len(names)] = -1
        if ok:
            idx, p = self.be.predict(model, np.stack(imgs))
            rows = torch.tensor(ok, dtype=torch.long)
            out[0, rows] = torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int32))
            out[1, rows] = torch.from_numpy(np.ascontiguousarray(p, dtype=np.float32)).view(torch.int32)
        return out, None


class FakeRankBackend(HostRankBackend):
    """Deterministic pseudo-results (serving.inference.FakeBackend), optional
    per-image delay (CPU tests)."""

    def __init__(self, cap: int = 16, delay_per_image: float = 0.0, loader: Optional[Callable] = None):
        from ..serving.inference import FakeBackend

        super().__init__(FakeBackend(), loader=loader, cap=cap, delay_per_image=delay_per_image)


class _Deadline:
    """A launch 'event' that fires at a given monotonic time (PacedRankBackend)."""

    def __init__(self, t: float):
        self.t = t

    def query(self) -> bool:
        return time.monotonic() >= self.t

    def synchronize(self) -> None:
        d = self.t - time.monotonic()
        if d > 0:
            time.sleep(d)


class PacedRankBackend(RankBackend):
    """A GPU stand-in for host-path capacity runs (tools/store_capacity.py): batches
    complete at a fixed rate per rank (``batches_per_s``, serialised like one GPU's
    stream, SLOTS in flight) and their rows come from a precomputed random top-5 table,
    so everything measured is the host side: control exchange, result rendering and the
    replicated output store. Synthetic image names only."""

    slots = SLOTS

    def __init__(self, cap: int = 256, batches_per_s: float = 370.0, seed: int = 0):
        self.cap, self.dt = cap, 1.0 / batches_per_s
        g = np.random.default_rng(seed)
        self.ids = g.integers(0, 1000, size=(4096, 5), dtype=np.int32)
        p = np.sort(g.random((4096, 5), dtype=np.float32), axis=1)[:, ::-1]
        self.p = np.ascontiguousarray(p / p.sum(1, keepdims=True)).view(np.int32)
        self.busy_until = 0.0
        self.launched = 0
        self.idle_s, self.idle_n, self.first, self.real = 0.0, 0, 0.0, 0   # gaps the "GPU" sat idle (capacity runs)

    def reset_stats(self) -> None:
        """(service_bench, after the untimed warm-up launches) idle accounting starts here."""
        self.idle_s, self.idle_n, self.real = 0.0, 0, 0

    def launch(self, model, names, slot):
        if len(names) > self.cap:
            raise ValueError(f"batch of {len(names)} exceeds the result capacity {self.cap}")
        k = len(names)
        i0 = (self.launched * 131) % (4096 - self.cap)
        out = np.zeros((2, self.cap, 5), np.int32)   # numpy: no torch call (GIL hand-off) per launch
        out[0, :k] = self.ids[i0:i0 + k]
        out[1, :k] = self.p[i0:i0 + k]
        now = time.monotonic()
        if self.real == 0:
            self.first = max(now, self.busy_until)
        elif now > self.busy_until:
            self.idle_s += now - self.busy_until
            self.idle_n += 1
        self.real += 1
        self.busy_until = max(now, self.busy_until) + self.dt
        self.launched += 1
        return out, _Deadline(self.busy_until)


class StoreRankBackend(_ArenaStaging, RankBackend):
    """CPU stand-in of GpuRankBackend's data path for multi-rank tests: the same
    window-staged image store (parallel/image_store.py, on a CPU device, shipments and
    flags over the gloo data group) feeding a deterministic 'classifier' of the image bytes
    (top-5 = a hash of the pixels). Exercises decode-once staging, arena eviction,
    version pinning and rejoin re-staging without a GPU."""

    slots = 8   # synchronous

    def __init__(self, loader: Optional[Callable] = None, cap: int = 16, hw=(8, 8), arena_images: int = 512,
                 n_synth: int = 16, delay_per_image: float = 0.0):
        from .image_store import HbmImageStore

        self.cap, self.delay = cap, delay_per_image
        self.arenas = {m: HbmImageStore(arena_images, hw, torch.device("cpu"), n_synth=n_synth,
                                        seed=1000 + MODEL_IDS[m]) for m in MODELS}
        self._init_staging(loader)
        for m, a in self.arenas.items():
            self._adopt(m, a)
        self.launched = 0
        self.loads = 0

    def _load(self, model: str, names: List[str]) -> Dict[str, Optional[np.ndarray]]:
        hw = self.arenas[model].hw
        blobs = self.loader(names) if self.loader else {}
        self.loads += len(names)
        out: Dict[str, Optional[np.ndarray]] = {}
        for n in names:
            b = blobs.get(n)
            if b is None:
                out[n] = None
                continue
            h = hashlib.sha256(b).digest()
            out[n] = np.frombuffer((h * (hw[0] * hw[1] * 3 // 32 + 1))[:hw[0] * hw[1] * 3],
                                   np.uint8).reshape(*hw, 3).copy()
        return out

    @staticmethod
    def classify(img: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        h = hashlib.sha256(img.tobytes()).digest()
        ids = np.frombuffer(h[:20], np.uint32) % 1000
        p = np.sort(np.frombuffer(h[12:32], np.uint8).astype(np.float32) / 1275.0)[::-1][:5]
        return ids[:5].astype(np.int32), p.copy()

    def launch(self, model, names, slot):
        if len(names) > self.cap:
            raise ValueError(f"batch of {len(names)} exceeds the result capacity {self.cap}")
        if self.delay:
            time.sleep(self.delay * len(names))
        arena = self.arenas[model]
        slots, failed = arena.slots(list(names))
        bad = set(failed)
        out = torch.zeros((2, self.cap, 5), dtype=torch.int32)
        for i, (n, s) in enumerate(zip(names, slots)):
            if n in bad:
                out[0, i] = -1
                continue
            ids, p = self.classify(arena.arena[s].numpy())
            out[0, i] = torch.from_numpy(ids)
            out[1, i] = torch.from_numpy(p).view(torch.int32)
        self.launched += 1
        return out, None


def nearest_index(n_in: int, n_out: int) -> np.ndarray:
    """Source index of each output row / column of Pillow's NEAREST resize, byte-identical
    to Image.resize: Pillow walks the output with a float64 accumulator started at half a
    step (sequential adds, then truncation) — np.add.accumulate adds in the same order."""
    a = n_in / n_out
    steps = np.full(n_out, a, np.float64)
    steps[0] = a * 0.5
    return np.add.accumulate(steps).astype(np.int32)


class _PackedImages(dict):
    """A window's decodes (name -> full-resolution RGB, None = failed) plus ``pack``: the
    decoded images in one pinned buffer, resized into their arena slots by one kernel."""

    pack = None


class _Pack:
    """Full-resolution images of one window in a pinned host buffer (built in the decode
    pool): n records {pixel offset / 16, h, w, row-table offset, column-table offset, slot}
    (int32: the offset in 16-byte units, so a pack of large images may pass 2 GiB), the int32
    nearest-index tables (sources wider or taller than 32767 pixels), the pixels. ``launch`` (serve loop, staging stream) fills in
    the slots, copies it to the device once and resizes every image into its slot
    (misc.hip resize_nearest_kernel); ``release`` returns the buffer after the window's event."""

    def __init__(self, backend: "GpuRankBackend", names: List[str], imgs: List[np.ndarray], hw: Tuple[int, int]):
        self.be, self.names, self.hw = backend, names, hw
        n = len(names)
        H, W = hw
        tabs: Dict[Tuple[int, int], int] = {}
        tab_parts: List[np.ndarray] = []
        t_len = 0
        recs = np.zeros((n, 6), np.int32)
        for i, im in enumerate(imgs):
            h, w = im.shape[:2]
            for key, out in (((h, H), 3), ((w, W), 4)):
                if key not in tabs:
                    tabs[key] = t_len
                    t = backend.nearest(*key)
                    tab_parts.append(t)
                    t_len += len(t)
                recs[i, out] = tabs[key]
            recs[i, 1], recs[i, 2] = h, w
        pix0 = (n * 24 + t_len * 4 + 15) // 16 * 16
        off = pix0
        offs = []
        for i, im in enumerate(imgs):
            offs.append(off)
            recs[i, 0] = off >> 4
            off += (im.nbytes + 15) // 16 * 16
        if off >> 4 >= 1 << 31:
            raise ValueError(f"image pack of {off} bytes exceeds the 32 GiB record range")
        self.nbytes = off
        self.buf = backend.pinned(self.nbytes)
        b = self.buf.numpy()
        self.recs = b[:n * 24].view(np.int32).reshape(n, 6)
        self.recs[...] = recs
        if t_len:
            b[n * 24:n * 24 + t_len * 4].view(np.int32)[...] = np.concatenate(tab_parts)
        for i, im in enumerate(imgs):
            o = offs[i]
            b[o:o + im.nbytes] = np.ascontiguousarray(im).reshape(-1)
        self.dev = None

    def launch(self, slots: List[int], arena: torch.Tensor, stream) -> None:
        from .. import _native as N

        self.recs[:, 5] = slots
        H, W = self.hw
        with torch.cuda.stream(stream):
            self.dev = torch.empty(self.nbytes, dtype=torch.uint8, device=arena.device)
            self.dev.copy_(self.buf[:self.nbytes], non_blocking=True)
            N.check(N.lib().dml_resize_nearest(self.dev.data_ptr(), len(self.names), H, W, arena.data_ptr(),
                                               stream.cuda_stream), "dml_resize_nearest")

    def release(self) -> None:
        self.dev = None
        if self.buf is not None:
            self.be.unpin(self.buf)
            self.buf = None


class _JpegPack:
    """The GPU-decodable JPEGs of one window (csrc/kernels/jpeg_decode.hip): built in the decode
    pool — one native call parses every header and un-stuffs every entropy segment into a pinned
    buffer of fixed-size descriptors (with the model size's Pillow-exact nearest tables) and
    entropy bytes. ``launch`` (serve loop, staging stream) copies it to the device and runs the
    Huffman, IDCT and colour + resize kernels straight into the arena slots — bit-exact with
    Pillow's decode + NEAREST resize (tests/test_jpeg_decode.py). ``unsupported``: the names the
    parser left to the CPU decode (progressive, 4:2:2, restart markers, ...)."""

    def __init__(self, backend: "GpuRankBackend", names: List[str], datas: List[bytes], hw: Tuple[int, int]):
        import ctypes as C

        from .. import _native as N

        self.be, self.hw = backend, hw
        L = N.lib()
        n = len(names)
        cap = 16 + n * L.dml_jpeg_desc_size() + sum(len(d) + 32 for d in datas) + 256
        self.buf = backend.pinned(cap)
        keep = [bytes(d) for d in datas]
        ptrs = (C.c_char_p * n)(*keep)
        lens = (C.c_long * n)(*[len(d) for d in keep])
        status = (C.c_int * n)()
        info = (C.c_long * 4)()
        used = L.dml_jpeg_prepare(n, ptrs, lens, hw[0], hw[1], C.c_void_p(self.buf.data_ptr()), cap, status, info)
        if used < 0:
            raise RuntimeError("dml_jpeg_prepare: buffer too small")
        self.used, self.n = int(used), n
        self.work_bytes, self.coef_bytes, self.maxblk, self.maxstream = (int(v) for v in info)
        self.idx = [i for i in range(n) if status[i]]
        self.names = [names[i] for i in self.idx]
        self.unsupported = [names[i] for i in range(n) if not status[i]]
        self.dev = None
        self.done = None   # the decode's completion event (set at launch)
        self.desc = L.dml_jpeg_desc_size()
        # the device work buffer now (coefficients, then the sample planes the other model's
        # window re-uses: GpuRankBackend.planes_for)
        self.work = torch.empty(max(self.work_bytes, 256), dtype=torch.uint8, device=backend.device)
        # and the device copy of the pack (here, not on the serve loop at launch)
        self.dev = torch.empty(max(self.used, 256), dtype=torch.uint8, device=backend.device)
        # the stream `work` was allocated on (this pool thread's): the side stream waits on this
        # event only - waiting on the serve loop's current stream (the staging stream, which has
        # waited on every earlier window's decode) chained all decodes one after the other
        # (rocprofv3: 400 Huffman launches on 8 queues, zero overlap, profiles/r5_store)
        self.alloc_ev = torch.cuda.Event()
        self.alloc_ev.record(torch.cuda.current_stream(backend.device))

    def launch(self, slots: List[int], arena: torch.Tensor, stream) -> None:
        import ctypes as C

        from .. import _native as N

        L = N.lib()
        idx = np.asarray(self.idx, np.int32)
        sl = np.asarray(slots, np.int32)
        L.dml_jpeg_set_slots(C.c_void_p(self.buf.data_ptr()), idx.ctypes.data, sl.ctypes.data, len(sl))
        H, W = self.hw
        # on a side stream of its own: the serial Huffman decode of one window (one wave per
        # image, milliseconds) overlaps the next windows' instead of queueing behind it on the
        # staging stream, which only waits for it before the window's event
        # (no wait on `stream` - the current stream here: it has waited on the previous windows'
        # decodes, which would chain them again; nothing before this on `stream` touches this
        # window's slots or buffers)
        side = self.be.jpeg_stream()
        side.wait_event(self.alloc_ev)
        for ev in getattr(self, "after", ()):   # image_store: earlier windows writing these slots
            side.wait_event(ev)
        # H2D copy of the pack, zeroed coefficients and the decode kernels: one native call
        N.check(L.dml_jpeg_launch(C.c_void_p(self.buf.data_ptr()), C.c_void_p(self.dev.data_ptr()), self.used,
                                  C.c_void_p(self.work.data_ptr()), self.coef_bytes, self.n, self.maxblk,
                                  self.maxstream, H, W, C.c_void_p(arena.data_ptr()), C.c_void_p(side.cuda_stream)),
                "dml_jpeg_launch")
        done = torch.cuda.Event()
        done.record(side)
        stream.wait_event(done)
        # the caching allocator must not hand these buffers out before `side` is done with them
        self.dev.record_stream(side)
        self.work.record_stream(side)
        self.done = done
        # the re-target reads only each descriptor's head (dml_jpeg_head_size): one strided copy
        # of the heads instead of a 37 KB copy per image in the serve loop
        b = self.buf.numpy()
        head = L.dml_jpeg_head_size()
        heads = b[16:16 + self.n * self.desc].reshape(self.n, self.desc)[self.idx, :head]
        self.be.remember_planes(self, {nm: heads[j] for j, nm in enumerate(self.names)})

    def release(self) -> None:
        self.dev = None   # `work` stays while the plane cache holds this window
        if self.buf is not None:
            self.be.unpin(self.buf)
            self.buf = None


class _ResizePack:
    """The other model's window over images a _JpegPack already decoded on this GPU: their
    descriptors re-targeted to this model's size (dml_jpeg_retarget: NEAREST tables, absolute
    plane addresses) and one colour + resize launch after those decodes' events — each image
    is decoded once for both models."""

    def __init__(self, backend: "GpuRankBackend", names: List[str], entries: list, hw: Tuple[int, int]):
        import ctypes as C

        from .. import _native as N

        L = N.lib()
        self.be, self.hw, self.names = backend, hw, names
        desc = L.dml_jpeg_desc_size()
        self.used = 16 + len(names) * desc
        self.buf = backend.pinned(self.used)
        b = self.buf.numpy()
        b[:16].view(np.int64)[:] = (len(names), 0)
        self.packs, self.works = [], []
        srcs = np.fromiter((rec.ctypes.data for rec, _, _ in entries), np.uint64, len(entries))
        bases = np.fromiter((work.data_ptr() for _, _, work in entries), np.int64, len(entries))
        L.dml_jpeg_retarget_many(C.c_void_p(self.buf.data_ptr()), srcs.ctypes.data, bases.ctypes.data, len(entries),
                                 hw[0], hw[1])
        seen = set()
        for _, pk, work in entries:
            if id(pk) not in seen:
                seen.add(id(pk))
                self.packs.append(pk)
                self.works.append(work)
        self.desc, self.dev = desc, None

    def launch(self, slots: List[int], arena: torch.Tensor, stream) -> None:
        import ctypes as C

        from .. import _native as N

        L = N.lib()
        sl = np.asarray(slots, np.int32)
        L.dml_jpeg_set_slots(C.c_void_p(self.buf.data_ptr()), None, sl.ctypes.data, len(sl))
        with torch.cuda.stream(stream):
            for pk, work in zip(self.packs, self.works):
                stream.wait_event(pk.done)
                work.record_stream(stream)   # an eviction from the cache must not free it under us
            self.dev = torch.empty(self.used, dtype=torch.uint8, device=arena.device)
            self.dev.copy_(self.buf[:self.used], non_blocking=True)
            N.check(L.dml_jpeg_resize_only(self.dev.data_ptr(), len(self.names), self.hw[0], self.hw[1],
                                           arena.data_ptr(), stream.cuda_stream), "dml_jpeg_resize_only")

    def release(self) -> None:
        self.dev = None
        self.packs, self.works = [], []
        if self.buf is not None:
            self.be.unpin(self.buf)
            self.buf = None


class _Packs:
    """Several packs of one window (the GPU-decoded JPEGs and the CPU-decoded rest) behind the
    one-pack interface the image store uses."""

    def __init__(self, packs: list):
        self.packs = [p for p in packs if p is not None and p.names]
        self.names = [n for p in self.packs for n in p.names]

    def launch(self, slots: List[int], arena: torch.Tensor, stream) -> None:
        o = 0
        for p in self.packs:
            p.after = getattr(self, "after", [])
            p.launch(slots[o:o + len(p.names)], arena, stream)
            o += len(p.names)

    def release(self) -> None:
        for p in self.packs:
            p.release()


class GpuRankBackend(_ArenaStaging, RankBackend):
    """Native engines for both models resident in this GPU's HBM, fed from per-model
    HBM image stores (parallel/image_store.py: store images staged in windows ahead of
    dispatch, decoded once per job by the rank that runs them and shipped HBM to HBM over
    the data group — RCCL — only to another rank that re-uses them; plus seeded synthetic
    images). A batch is never gathered: the engines' stem
    kernels read its images in place from the arena through a per-slot index table
    (Engine ``src_index``: written into pinned host memory, fetched into device memory by
    one tiny kernel in stream order — a host-memory read per stem workgroup made the stem
    3.8x slower), and the top-5 kernel writes the result rows straight into the slot's
    pinned host buffer (Engine ``result_views``) — a launch is the index fetch, one graph
    replay and one event; no gather, no copy.
    The compute stream waits on the events of the windows that staged the batch's
    images. A batch larger than the engine's batch runs as several engine passes, one
    after the other (the host collects each pass's rows; a rare, blocking path).

    Arena writes (window scatters) run on ``stage_stream``; a launch makes the compute
    stream wait for the windows of its images. A slot is only re-assigned after every
    batch pinning its old image completed, so a scatter never overtakes a forward that
    still reads the old image."""

    def __init__(self, device: torch.device, batch_sizes: Dict[str, int], cap: int = 0, arena_images: int = 8192,
                 n_synth: int = 512, seed: int = 0, models: Sequence[str] = MODELS, splits: int = 2,
                 loader: Optional[Callable] = None, decode_threads: int = 8):
        from ..models import build_model
        from ..models.engine import Engine, SplitEngine, merge_point
        from .image_store import HbmImageStore

        self.device = device
        self.cap = cap or max(batch_sizes.values())
        self.engines, self.arenas, self.idx, self.idx_dev = {}, {}, {}, {}
        from .. import _native as N

        self._fetch = N.lib().dml_index_fetch
        # DML_NATIVE_LAUNCH=0: a batch launch issues its HIP calls one Python call each (A/B)
        self.native_launch = os.environ.get("DML_NATIVE_LAUNCH", "1") != "0"
        self._launch_seq = N.lib().dml_launch_seq
        self._lops: Dict[Tuple[str, int], np.ndarray] = {}
        from ..models.engine import serve_stream_priority
        self.stream = torch.cuda.Stream(device, priority=serve_stream_priority())
        self.stage_stream = torch.cuda.Stream(device)
        # the staging pool (a window's fetch + GPU-JPEG prepare each) shares the interpreter with
        # the serve loop: 4 threads, not decode_threads (51,200-distinct pass on one box, 2 rounds:
        # 4 threads 54.6k / 55.0k images/s, serve-loop launch phase 0.18 s; 32 threads 53.7k /
        # 51.2k, 0.35-0.40 s; profiles/r6_n). DML_STAGING_THREADS overrides; the CPU decode pool
        # (_jpool, decode worker processes behind it) keeps decode_threads
        self._init_staging(loader, int(os.environ.get("DML_STAGING_THREADS", "4")))
        import threading

        self._dcache: "OrderedDict[str, np.ndarray]" = OrderedDict()   # name -> full-res RGB (both models)
        self._nprocs, self._dprocs = int(os.environ.get("DML_DECODE_PROCS", "12")), None
        self._dbytes, self.decode_hits, self._dlock = 0, 0, threading.Lock()
        self.plane_hits = 0     # images a window took from another model's GPU decode (resize only)
        # decode-pool seconds per window phase (summed over windows; the store-image pass reports them)
        self.load_s = {"fetch": 0.0, "gpu_prepare": 0.0, "cpu_decode": 0.0, "windows": 0}
        self.gpu_decodes = 0    # images decoded on the GPU (jpeg_decode.hip)
        self._nn: Dict[Tuple[int, int], np.ndarray] = {}    # (n_in, n_out) -> nearest-index table
        self._pins: List[torch.Tensor] = []                  # free pinned pack buffers
        self._jstreams: List[torch.cuda.Stream] = []         # side streams of the GPU JPEG decodes
        self._jnext = 0
        self._planes: "OrderedDict[str, tuple]" = OrderedDict()   # name -> (descriptor, decoded window)
        self._plane_packs: "OrderedDict[int, object]" = OrderedDict()
        self._plane_bytes = 0
        # DML_GPU_RESIZE=0: the decode pool resizes on the CPU (Pillow) as before (A/B)
        self.gpu_resize = os.environ.get("DML_GPU_RESIZE", "1") != "0"
        # DML_GPU_JPEG=0: every JPEG decodes on the CPU (the decode workers), as before (A/B)
        self.gpu_jpeg = self.gpu_resize and os.environ.get("DML_GPU_JPEG", "1") != "0"
        # a window's images are decoded DECODE_CHUNK per task by this pool, each task handing its
        # chunk to a decode worker PROCESS (parallel/decode_worker.py; in-process threads held
        # the GIL for ~0.3 ms per image: ~3.5k img/s on the 51,200-distinct run with 32 threads)
        from concurrent.futures import ThreadPoolExecutor
        self.decode_threads = decode_threads
        self._jpool = ThreadPoolExecutor(max_workers=decode_threads, thread_name_prefix="jpeg")
        self.host = [torch.zeros((2, self.cap, 5), dtype=torch.int32).pin_memory() for _ in range(SLOTS)]
        self.host_np = [h.numpy() for h in self.host]   # the serve loop reads rows without a torch call
        self.ev_done = [torch.cuda.Event() for _ in range(SLOTS)]
        self.fail_rows: List[Optional[List[int]]] = [None] * SLOTS
        for m in models:
            g, w = build_model(m, seed=seed, calibrate=True)
            b = batch_sizes[m]
            if b > self.cap:
                raise ValueError(f"{m}: engine batch {b} exceeds the result capacity {self.cap}")
            # arena_images counts the slots windows can use: the seeded synthetic images come on
            # top (plan() never hands those out), so the staging room is what the caller sized
            arena = HbmImageStore(n_synth + max(arena_images, 2 * self.cap), g.input_hw, device,
                                  n_synth=n_synth, seed=1000 + MODEL_IDS[m])
            assert arena.capacity - arena.n_synth >= arena_images
            self.arenas[m] = arena
            self._adopt(m, arena)
            self.idx[m] = [torch.zeros(b, dtype=torch.int32).pin_memory() for _ in range(SLOTS)]
            self.idx_dev[m] = [torch.zeros(b, dtype=torch.int32, device=device) for _ in range(SLOTS)]
            src = dict(src_tensors=[arena.arena] * SLOTS, src_index=self.idx_dev[m],
                       result_views=[h[:, :b] for h in self.host])
            if splits > 1 and b % splits == 0:
                self.engines[m] = SplitEngine(g, w, batch=b, device=str(device), src_slots=SLOTS, splits=splits,
                                              merge_at=merge_point(m) if splits == 2 else None, **src)
            else:
                self.engines[m] = Engine(g, w, batch=b, device=str(device), src_slots=SLOTS, **src)
            self.engines[m].capture(self.stream)  # graphs now, before the service's first collective
        if self.gpu_jpeg:
            N.check(N.lib().dml_jpeg_init(), "dml_jpeg_init")
        if self.loader is not None:
            self._procs()   # the decode workers start (and import Pillow) now, not inside a timed pass
            # and the windows' pinned buffers: pinning host memory mid-pass (64 MB at a time) held
            # up the serve loop's launches for 20-50 ms
            self._pins = [torch.empty(self.PIN_BYTES, dtype=torch.uint8).pin_memory()
                          for _ in range(self.PIN_PREALLOC)]
            if self.gpu_jpeg:
                # and the device work buffers of the GPU decodes: one block the caching allocator
                # keeps and splits, so no window allocates device memory from the driver mid-pass
                # (each hipMalloc also stalls the serve loop's HIP calls)
                reserve = torch.empty(self.PLANE_CACHE_BYTES + (512 << 20), dtype=torch.uint8, device=device)
                del reserve

    DECODE_CACHE_BYTES = 1 << 30
    DECODE_CHUNK = 8
    PIN_BYTES = 16 << 20   # a GPU-JPEG window of 256 images needs ~9.5 MB (descriptors + entropy bytes)
    PIN_PREALLOC = 16      # pinned buffers allocated with the store loader (host-pinning stalls every HIP call)

    def nearest(self, n_in: int, n_out: int) -> np.ndarray:
        t = self._nn.get((n_in, n_out))
        if t is None:
            t = self._nn[(n_in, n_out)] = nearest_index(n_in, n_out)
        return t

    # side streams of the GPU JPEG decodes (DML_JPEG_STREAMS: A/B). 2, not 8: fewer decodes in
    # flight at once leave the model kernels more of the GPU; the 51,200-distinct pass measured
    # 58.0-58.9k images/s with 2 against 57.1-57.9k with 8 over 4 interleaved rounds
    # (profiles/r6_ah, r6_ai), the window bench with 4 windows on 4 streams being its own setup
    JPEG_STREAMS = int(os.environ.get("DML_JPEG_STREAMS", "2"))
    # device work buffers of decoded windows kept for the other model (DML_PLANE_CACHE_GB). A
    # 256-image window holds ~90 MB (coefficients + planes): 4 GiB kept ~11k images, so on the
    # 51,200-distinct run the second job re-decoded every image the first had decoded long before
    # (decode cache hits 0, 76,800 decodes for 51,200 images); 24 GiB (of 288 GB HBM) keeps ~68k
    PLANE_CACHE_BYTES = int(float(os.environ.get("DML_PLANE_CACHE_GB", "24")) * (1 << 30))

    def remember_planes(self, pack: "_JpegPack", recs: Dict[str, np.ndarray]) -> None:
        """(serve loop, after a GPU decode's launch) the window's planes serve the other
        model's windows of the same images (planes_for); least recently decoded windows go first."""
        with self._dlock:
            self._plane_packs[id(pack)] = pack
            self._plane_bytes += pack.work.numel()
            for nm, rec in recs.items():
                self._planes[nm] = (rec, pack)
                self._planes.move_to_end(nm)
            while self._plane_bytes > self.PLANE_CACHE_BYTES and self._plane_packs:
                old_id, old = next(iter(self._plane_packs.items()))
                del self._plane_packs[old_id]
                self._plane_bytes -= old.work.numel()
                for nm in [k for k, (_, pk) in self._planes.items() if pk is old]:
                    del self._planes[nm]
                old.work = None

    def planes_for(self, names: List[str]) -> Dict[str, tuple]:
        """(decode pool) {name: (descriptor, decoded window)} for the names a launched GPU decode
        already holds on this device."""
        with self._dlock:   # (descriptor, window, its work tensor: held, an eviction cannot free it)
            return {nm: (self._planes[nm][0], self._planes[nm][1], self._planes[nm][1].work)
                    for nm in names if nm in self._planes and self._planes[nm][1].work is not None}

    def jpeg_stream(self) -> torch.cuda.Stream:
        """(serve loop) the next of JPEG_STREAMS side streams for GPU JPEG decodes."""
        if not self._jstreams:
            self._jstreams = [torch.cuda.Stream(self.device) for _ in range(self.JPEG_STREAMS)]
        self._jnext = (self._jnext + 1) % len(self._jstreams)
        return self._jstreams[self._jnext]

    def pinned(self, nbytes: int) -> torch.Tensor:
        """(decode pool) a pinned buffer of at least nbytes: a free one of the pool or a new one."""
        with self._dlock:
            for i, b in enumerate(self._pins):
                if b.numel() >= nbytes:
                    return self._pins.pop(i)
        return torch.empty(max(nbytes, self.PIN_BYTES), dtype=torch.uint8).pin_memory()

    def unpin(self, buf: torch.Tensor) -> None:
        with self._dlock:
            if len(self._pins) < 32:
                self._pins.append(buf)

    def _cached(self, name: str) -> Optional[np.ndarray]:
        """The full-resolution RGB decode of one store image if this rank holds it (shared by
        both models' windows: Keras load_img decodes, converts to RGB, then resizes — the same
        steps in the same order, so the result is byte-identical to
        serving.inference.load_image)."""
        with self._dlock:
            hit = self._dcache.get(name)
            if hit is not None:
                self._dcache.move_to_end(name)
                self.decode_hits += 1
            return hit

    def _remember(self, name: str, img: np.ndarray) -> None:
        with self._dlock:
            self._dcache[name] = img
            self._dbytes += img.nbytes
            while self._dbytes > self.DECODE_CACHE_BYTES and self._dcache:
                _, old = self._dcache.popitem(last=False)
                self._dbytes -= old.nbytes

    @staticmethod
    def _decode_here(data: bytes) -> np.ndarray:
        import io

        from PIL import Image

        im = Image.open(io.BytesIO(data))
        if im.mode != "RGB":   # load_img's convert; an RGB JPEG needs no copy
            im = im.convert("RGB")
        return np.asarray(im, dtype=np.uint8)

    def _procs(self):
        """The decode worker processes (parallel/decode_worker.py), started with a store loader
        (before any timed work) or on first use: DML_DECODE_PROCS (default 12; 0 = decode in
        this process's threads)."""
        if self._dprocs is None and self._nprocs > 0:
            with self._dlock:
                if self._dprocs is None:
                    from .decode_worker import DecodeProcs
                    self._dprocs = DecodeProcs(self._nprocs)
        return self._dprocs

    def _load(self, model: str, names: List[str]) -> Dict[str, Optional[np.ndarray]]:
        """(decode pool thread) fetch + decode this rank's share of a window. Baseline JPEGs
        decode on the GPU (_JpegPack; DML_GPU_JPEG=0 turns it off); the rest decode on the CPU
        (decode workers): with GPU resize (the default) their full-resolution decodes go into
        one pinned pack that the staging stream resizes into the arena slots (_Pack); else
        Pillow NEAREST here, as load_img(target_size)."""
        from PIL import Image

        t0 = time.perf_counter()
        blobs = self.loader(names) if self.loader else {}
        t1 = time.perf_counter()
        t_fetch = t1 - t0
        hw = self.arenas[model].hw
        out = _PackedImages() if self.gpu_resize else {}
        jp = rp = None
        if self.gpu_jpeg:
            # decoded on this GPU already (the other model's window): colour + resize only
            cached = self.planes_for([n for n in names if blobs.get(n) is not None])
            if cached:
                hit = [n for n in names if n in cached]
                rp = _ResizePack(self, hit, [cached[n] for n in hit], hw)
                self.plane_hits += len(hit)
                for n in hit:
                    out[n] = True
                names = [n for n in names if n not in cached]
            # GPU decode (jpeg_decode.hip) for every other baseline JPEG; the CPU decodes the rest
            have = [n for n in names if blobs.get(n) is not None]
            if have:
                try:
                    jp = _JpegPack(self, have, [blobs[n] for n in have], hw)
                except Exception as e:   # never fatal: the CPU path takes the window
                    log.warning("GPU JPEG prepare failed (%s); decoding on the CPU", e)
                    jp = None
            t2 = time.perf_counter()
            with self._dlock:
                self.load_s["gpu_prepare"] += t2 - t1
            t1 = t2
            if jp is not None:
                self.gpu_decodes += len(jp.names)
                for n in jp.names:
                    out[n] = True   # decoded on the device at launch (the window only needs "ok")
                gone = set(jp.names)
                names = [n for n in names if n not in gone]

        def decode(chunk):
            res, miss = [], []
            for n in chunk:
                b = blobs.get(n)
                if b is None:
                    res.append((n, None))
                    continue
                hit = self._cached(n)
                if hit is not None:
                    res.append((n, hit))
                else:
                    miss.append((n, b))
            got: Dict[str, Optional[np.ndarray]] = {}
            procs = self._procs() if miss else None
            if procs is not None:
                try:
                    got = procs.decode_many(miss)
                except Exception as e:   # a dead worker: this chunk decodes here
                    log.warning("decode worker failed (%s); decoding in-process", e)
                    got = {}
            for n, b in miss:
                try:
                    img = got[n] if n in got else self._decode_here(b)
                    if img is None:
                        raise ValueError("undecodable image")
                    self._remember(n, img)
                    if not self.gpu_resize and img.shape[:2] != tuple(hw):
                        img = np.asarray(Image.fromarray(img).resize((hw[1], hw[0]), Image.NEAREST), dtype=np.uint8)
                    res.append((n, img))
                except Exception as e:  # undecodable file -> reported as failed
                    log.warning("decode of %s failed: %s", n, e)
                    res.append((n, None))
            return res
        k = min(self.decode_threads, len(names) // self.DECODE_CHUNK)
        if k > 1:   # cached names cost nothing, so round-robin chunks balance the uncached ones
            for f in [self._jpool.submit(decode, names[i::k]) for i in range(k)]:
                out.update(f.result())
        else:
            out.update(decode(names))
        if self.gpu_resize:
            ok = [n for n in names if out.get(n) is not None]
            cpu = _Pack(self, ok, [out[n] for n in ok], hw) if ok else None
            out.pack = _Packs([rp, jp, cpu]) if (jp is not None or rp is not None) else cpu
        t3 = time.perf_counter()
        with self._dlock:
            self.load_s["fetch"] += t_fetch
            self.load_s["cpu_decode"] += t3 - t1
            self.load_s["windows"] += 1
        return out

    def launch(self, model, names, slot):
        if len(names) > self.cap:
            raise ValueError(f"batch of {len(names)} exceeds the result capacity {self.cap}")
        eng, arena = self.engines[model], self.arenas[model]
        s = self.stream
        B = eng.batch
        slots, failed = arena.slots(list(names))
        bad = set(failed)
        self.fail_rows[slot] = [i for i, n in enumerate(names) if n in bad] if bad else None
        hidx, didx = self.idx[model][slot], self.idx_dev[model][slot]
        iv = hidx.numpy()   # the slot's previous launch has finished: free to rewrite
        host = self.host[slot]
        sp = s.cuda_stream

        def fetch():  # host table -> the device table the stems read (stream order)
            if self._fetch(hidx.data_ptr(), didx.data_ptr(), B, sp) != 0:
                raise RuntimeError("dml_index_fetch failed")
        if len(slots) <= B and self.native_launch:
            ops = self._launch_ops(model, slot)
            if ops is not None:
                iv[:len(slots)] = slots
                iv[len(slots):] = slots[0] if slots else 0   # padding rows: computed, never reported
                waits = [(1, sp, int(ev.cuda_event), 0, 0) for ev in arena.events(names) if ev.cuda_event]
                seq = np.asarray(waits, np.int64).reshape(-1, 5)
                seq = np.concatenate([seq, ops]) if len(waits) else ops
                eng.select(slot)
                rc = self._launch_seq(seq.ctypes.data, len(seq))
                if rc != 0:
                    N.check(rc, "dml_launch_seq")
                return self.host_np[slot], self.ev_done[slot]
        with torch.cuda.stream(s):
            for ev in arena.events(names):  # the windows that staged these images
                s.wait_event(ev)
            if len(slots) <= B:
                iv[:len(slots)] = slots
                iv[len(slots):] = slots[0] if slots else 0   # padding rows: computed, never reported
                fetch()
                eng.run(s, use_graph=True, slot=slot)
            else:  # larger than the engine batch: passes one after the other, rows collected here
                rows = []
                for off in range(0, len(slots), B):
                    chunk = slots[off:off + B]
                    iv[:len(chunk)] = chunk
                    iv[len(chunk):] = chunk[0]
                    fetch()
                    eng.run(s, use_graph=True, slot=slot)
                    s.synchronize()
                    rows.append(host[:, :len(chunk)].clone())
                host[:, :len(slots)] = torch.cat(rows, 1)
            self.ev_done[slot].record(s)
        return self.host_np[slot], self.ev_done[slot]

    def finalize(self, slot: int) -> None:
        """(after the slot's event) unfetchable / undecodable images: class id -1 marks the row failed."""
        rows = self.fail_rows[slot]
        if rows:
            self.host_np[slot][0, rows] = -1
            self.fail_rows[slot] = None

    def drain(self) -> None:
        # the compute stream only ever waits on window events that had completed (ready()),
        # so this returns even when a peer died mid-staging; the staging stream is released by
        # the communicator abort of the rebuild, never waited for here
        self.stream.synchronize()
