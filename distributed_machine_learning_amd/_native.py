"""ctypes binding of the native HIP library (csrc/ -> libdml_hip.so).

``lib()`` loads the in-tree library (building it first if the sources changed
and hipcc is available). On a machine with a GPU the native path is the ONLY
path: every op raises if the library cannot be loaded rather than silently
falling back to PyTorch.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import _build

_lock = threading.Lock()
_lib = None


class ConvArgs(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("w", C.c_void_p), ("bias", C.c_void_p), ("res", C.c_void_p), ("y", C.c_void_p),
        ("N", C.c_int), ("H", C.c_int), ("W", C.c_int), ("Cin", C.c_int), ("ldx", C.c_int),
        ("kh", C.c_int), ("kw", C.c_int), ("sh", C.c_int), ("sw", C.c_int), ("ph", C.c_int), ("pw", C.c_int),
        ("Ho", C.c_int), ("Wo", C.c_int), ("Cout", C.c_int), ("K", C.c_int), ("Kpad", C.c_int),
        ("ldy", C.c_int), ("ldr", C.c_int),
        ("relu", C.c_int), ("out_f32", C.c_int),
        ("dh", C.c_int), ("dw", C.c_int),
        ("nseg", C.c_int), ("seg_c0", C.c_int * 4), ("seg_ldy", C.c_int * 4), ("seg_relu", C.c_int * 4),
        ("seg_y", C.c_void_p * 4),
        ("ksplit", C.c_int), ("split_ld", C.c_int),
        ("rsub", C.c_int), ("rW", C.c_int), ("rHW", C.c_int),
    ]


class PoolArgs(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("y", C.c_void_p),
        ("N", C.c_int), ("H", C.c_int), ("W", C.c_int), ("C", C.c_int), ("ldx", C.c_int),
        ("Ho", C.c_int), ("Wo", C.c_int), ("ldy", C.c_int),
        ("k", C.c_int), ("stride", C.c_int), ("pad", C.c_int), ("mode", C.c_int), ("relu", C.c_int),
    ]


GROUP_MAX = 4       # DML_CONV_GROUP_MAX
GROUP_POOL_MAX = 2  # DML_GROUP_POOL_MAX


class ConvGroupArgs(C.Structure):
    _fields_ = [("n", C.c_int), ("npool", C.c_int), ("off", C.c_int * (GROUP_MAX + GROUP_POOL_MAX + 1)),
                ("a", ConvArgs * GROUP_MAX), ("pool", PoolArgs * GROUP_POOL_MAX)]


class PreprocArgs(C.Structure):
    _fields_ = [
        ("src", C.c_void_p), ("y", C.c_void_p),
        ("N", C.c_int), ("Hs", C.c_int), ("Ws", C.c_int), ("Ho", C.c_int), ("Wo", C.c_int), ("mode", C.c_int),
        ("pair", C.c_int), ("lpad", C.c_int), ("idx", C.c_void_p),
    ]


class StemArgs(C.Structure):
    _fields_ = [
        ("src", C.c_void_p), ("w", C.c_void_p), ("bias", C.c_void_p), ("y", C.c_void_p),
        ("N", C.c_int), ("Hs", C.c_int), ("Ws", C.c_int), ("H", C.c_int), ("W", C.c_int), ("mode", C.c_int),
        ("ldw", C.c_int), ("Hc", C.c_int), ("Wc", C.c_int), ("Ho", C.c_int), ("Wo", C.c_int), ("ldy", C.c_int),
        ("w4", C.c_void_p), ("b4", C.c_void_p), ("z", C.c_void_p), ("c4", C.c_int), ("ldw4", C.c_int),
        ("ldz", C.c_int), ("idx", C.c_void_p),
    ]


class IncStemArgs(C.Structure):
    _fields_ = [
        ("src", C.c_void_p), ("w1", C.c_void_p), ("b1", C.c_void_p), ("w2", C.c_void_p), ("b2", C.c_void_p),
        ("y", C.c_void_p),
        ("N", C.c_int), ("Hs", C.c_int), ("Ws", C.c_int), ("H", C.c_int), ("W", C.c_int), ("mode", C.c_int),
        ("ldw1", C.c_int), ("ldw2", C.c_int), ("H1", C.c_int), ("W1", C.c_int), ("H2", C.c_int), ("W2", C.c_int),
        ("ldy", C.c_int), ("idx", C.c_void_p),
    ]


class ConvPoolArgs(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("w", C.c_void_p), ("bias", C.c_void_p), ("y", C.c_void_p),
        ("N", C.c_int), ("H", C.c_int), ("W", C.c_int), ("ldx", C.c_int), ("ldw", C.c_int),
        ("Ho", C.c_int), ("Wo", C.c_int), ("ldy", C.c_int),
        ("w4", C.c_void_p), ("b4", C.c_void_p), ("c4", C.c_int), ("ldw4", C.c_int),
    ]


class ExpandReduceArgs(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("w3", C.c_void_p), ("b3", C.c_void_p), ("res", C.c_void_p), ("y", C.c_void_p),
        ("w1", C.c_void_p), ("b1", C.c_void_p), ("z", C.c_void_p),
        ("M", C.c_int), ("ldx", C.c_int), ("ldw3", C.c_int), ("ldr", C.c_int), ("ldy", C.c_int),
        ("ldw1", C.c_int), ("ldz", C.c_int), ("C", C.c_int), ("kx", C.c_int),
        ("ysub", C.c_int), ("yH", C.c_int), ("yW", C.c_int), ("stamps", C.c_void_p), ("fz", C.c_int),
    ]


_SIGS = {
    "dml_expand_reduce": (C.c_int, [C.POINTER(ExpandReduceArgs), C.c_void_p]),
    "dml_chain_supported": (C.c_int, [C.POINTER(ExpandReduceArgs)]),
    "dml_plan_add_expand_reduce": (C.c_int, [C.c_void_p, C.POINTER(ExpandReduceArgs)]),
    "dml_conv3x3_pool": (C.c_int, [C.POINTER(ConvPoolArgs), C.c_void_p]),
    "dml_plan_add_conv_pool": (C.c_int, [C.c_void_p, C.POINTER(ConvPoolArgs)]),
    "dml_stem_resnet": (C.c_int, [C.POINTER(StemArgs), C.c_void_p]),
    "dml_stem_inception": (C.c_int, [C.POINTER(IncStemArgs), C.c_void_p]),
    "dml_plan_add_inc_stem": (C.c_int, [C.c_void_p, C.POINTER(IncStemArgs)]),
    "dml_plan_add_stem": (C.c_int, [C.c_void_p, C.POINTER(StemArgs)]),
    "dml_conv": (C.c_int, [C.POINTER(ConvArgs), C.c_int, C.c_void_p]),
    "dml_conv_group": (C.c_int, [C.POINTER(ConvGroupArgs), C.c_int, C.c_void_p]),
    "dml_plan_add_conv_group": (C.c_int, [C.c_void_p, C.POINTER(ConvGroupArgs), C.c_int]),
    "dml_conv_pick_cfg": (C.c_int, [C.POINTER(ConvArgs)]),
    "dml_conv_v2_bn": (C.c_int, [C.c_int]),
    "dml_conv_v2_init": (C.c_int, []),
    "dml_pool": (C.c_int, [C.POINTER(PoolArgs), C.c_void_p]),
    "dml_global_avgpool": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "dml_softmax_top5": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p]),
    "dml_softmax_top5_split": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p]),
    "dml_preprocess": (C.c_int, [C.POINTER(PreprocArgs), C.c_void_p]),
    "dml_index_fetch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "dml_resize_nearest": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "dml_jpeg_prepare": (C.c_long, [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_long,
                                    C.c_void_p, C.c_void_p]),
    "dml_jpeg_set_slot": (None, [C.c_void_p, C.c_int, C.c_int]),
    "dml_jpeg_set_slots": (None, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "dml_jpeg_decode_resize": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_long, C.c_void_p, C.c_int, C.c_int,
                                         C.c_void_p, C.c_void_p]),
    "dml_jpeg_init": (C.c_int, []),
    "dml_jpeg_launch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_long, C.c_void_p, C.c_long, C.c_int, C.c_int, C.c_long,
                                  C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "dml_jpeg_retarget": (None, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_long]),
    "dml_jpeg_retarget_many": (None, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]),
    "dml_jpeg_resize_only": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "dml_jpeg_desc_size": (C.c_long, []),
    "dml_jpeg_head_size": (C.c_long, []),
    "dml_jpeg_decode_host": (C.c_int, [C.c_char_p, C.c_long, C.c_void_p, C.POINTER(C.c_int)]),
    "dml_jpeg_parallel_host": (C.c_int, [C.c_char_p, C.c_long, C.c_void_p, C.c_void_p, C.c_long,
                                         C.POINTER(C.c_long)]),
    "dml_plan_create": (C.c_void_p, []),
    "dml_plan_destroy": (None, [C.c_void_p]),
    "dml_plan_add_conv": (C.c_int, [C.c_void_p, C.POINTER(ConvArgs), C.c_int]),
    "dml_plan_add_pool": (C.c_int, [C.c_void_p, C.POINTER(PoolArgs)]),
    "dml_plan_add_gap": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]),
    "dml_plan_add_softmax_top5": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_void_p]),
    "dml_plan_add_softmax_top5_split": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                                  C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "dml_plan_add_preprocess": (C.c_int, [C.c_void_p, C.POINTER(PreprocArgs)]),
    "dml_plan_size": (C.c_int, [C.c_void_p]),
    "dml_plan_run": (C.c_int, [C.c_void_p, C.c_void_p]),
    "dml_plan_run_range": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "dml_plan_capture": (C.c_int, [C.c_void_p, C.c_void_p]),
    "dml_plan_replay": (C.c_int, [C.c_void_p, C.c_void_p]),
    "dml_launch_seq": (C.c_int, [C.c_void_p, C.c_int]),
    "dml_plan_capture_parts": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.c_int, C.c_void_p]),
    "dml_plan_replay_part": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "dml_plan_time_ops": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_float), C.c_int]),
    "dml_plan_set_cfg": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "dml_plan_get_cfg": (C.c_int, [C.c_void_p, C.c_int]),
    "dml_ring_create": (C.c_void_p, [C.c_int, C.c_size_t]),
    "dml_ring_destroy": (None, [C.c_void_p]),
    "dml_ring_slot": (C.c_void_p, [C.c_void_p, C.c_int]),
    "dml_ring_h2d": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p]),
    "dml_ring_wait": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "dml_ring_sync": (C.c_int, [C.c_void_p, C.c_int]),
    "dml_host_alloc": (C.c_void_p, [C.c_size_t]),
    "dml_host_free": (None, [C.c_void_p]),
    "dml_memcpy_h2d_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "dml_memcpy_d2h_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "dml_last_error": (C.c_char_p, []),
    "dml_abi_sizes": (C.c_int, [C.POINTER(C.c_int), C.c_int]),
    "dml_device_info": (C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
}


class NativeError(RuntimeError):
    pass


ABI_STRUCTS = ("ConvArgs", "PoolArgs", "ConvGroupArgs", "PreprocArgs", "StemArgs", "IncStemArgs", "ConvPoolArgs",
               "ExpandReduceArgs")


def _check_abi(L) -> None:
    """The library's argument structs must match their ctypes mirrors byte for byte."""
    f = getattr(L, "dml_abi_sizes", None)
    if f is None:
        return
    n = len(ABI_STRUCTS)
    out = (C.c_int * n)()
    f(out, n)
    for i, name in enumerate(ABI_STRUCTS):
        want = C.sizeof(globals()[name])
        if out[i] != want:
            raise NativeError(f"ABI mismatch: sizeof(Dml{name}) = {out[i]} in the library, {want} in _native.py")


def lib():
    """Load (building if needed) libdml_hip.so. Raises NativeError on failure."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  -- load torch's libamdhip64.so.7 first so ours binds to it

        path = _build.LIB_PATH
        if os.environ.get("DML_LIB"):  # explicit library (A/B experiments between kernel variants)
            from pathlib import Path

            path = Path(os.environ["DML_LIB"])
        elif os.environ.get("DML_SKIP_BUILD") != "1":
            try:
                path = _build.build()
            except Exception as e:  # hipcc missing on a runtime-only box: use the shipped .so
                if not path.exists():
                    raise NativeError(f"cannot build libdml_hip.so: {e}") from e
        if not path.exists():
            raise NativeError(f"{path} missing; run python -m distributed_machine_learning_amd._build")
        L = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name, None)
            if f is None and os.environ.get("DML_LIB"):  # an older variant library: bind what it has
                continue
            if f is None:
                raise NativeError(f"{path} lacks {name}; rebuild")
            f.restype = res
            f.argtypes = args
        _check_abi(L)
        _lib = L
        return _lib


_inited = False


def ensure_device_init() -> None:
    """Per-process device-side setup (kernel attributes); call before launching."""
    global _inited
    if not _inited:
        check(lib().dml_conv_v2_init(), "dml_conv_v2_init")
        _inited = True


def check(rc: int, what: str) -> int:
    if rc != 0 and rc is not None and not (isinstance(rc, int) and rc > 0):
        msg = lib().dml_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed (rc={rc}): {msg}")
    return rc


def stream_ptr(stream=None) -> int:
    import torch

    ensure_device_init()
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False
