"""ctypes binding of libofdmsync.so (the C ABI declared in include/ofdmsync.h).

PyTorch is used only as plumbing: device memory, the current HIP stream, host<->device
copies.  Every metric is computed by the HIP kernels in ``csrc/ofdmsync.hip``.  There is
no CPU fallback: if the library or a GPU is missing, calls raise.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_int32, c_int64, c_void_p

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libofdmsync.so")       # the in-tree build (no environment override)
TUNING_BUILD = None          # set by use_tuning_library(): name of the tools/variants.py build in use
_TUNING_PATH = None

# input formats / precisions / status (include/ofdmsync.h)
C64, C128, CI16, CP12 = 0, 1, 2, 3
FP32, FP64 = 0, 1

_lib = None

_CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
_HDR = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "ofdmsync.h")


def source_files() -> list[str]:
    """The sources libofdmsync.so is compiled from (csrc .hip/.h + the ABI header)."""
    if not os.path.isdir(_CSRC):
        return []
    fs = sorted(os.path.join(_CSRC, f) for f in os.listdir(_CSRC) if f.endswith((".hip", ".h")))
    return fs + ([_HDR] if os.path.exists(_HDR) else [])


# hipcc flags of every translation unit (__graft_entry__.build_hip); part of the source hash, so a
# flag change (arch, -O level, a -D knob) invalidates an existing library like a source edit
BUILD_FLAGS = ("--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC")


def source_hash() -> str:
    """sha256 (16 hex digits) over the sources' names and bytes and the build flags: baked into
    the library at build time (OFS_SOURCE_HASH) and checked at load, so a library built from
    other sources or flags than the ones next to it is refused instead of silently run."""
    import hashlib
    h = hashlib.sha256(" ".join(BUILD_FLAGS).encode() + b"\0")
    for f in source_files():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _declare(lib):
    P = c_void_p
    sig = {
        "ofs_version": (c_int32, []),
        "ofs_source_hash": (ctypes.c_char_p, []),
        "ofs_status_string": (ctypes.c_char_p, [c_int32]),
        "ofs_aa_detect": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32, P, P, P,
                                    P, c_int32, c_double, c_int32, c_double, c_int32, P, P, P, P]),
        "ofs_aa_plan": (c_int32, [c_int32, c_int32, c_int32, c_int64, c_int32]),
        "ofs_sc_metric": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32,
                                    c_int32, P, P, P, P]),
        "ofs_minn_metric": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32,
                                      P, P, P, P]),
        "ofs_minn_rtl": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32, c_int32,
                                   c_int64, c_int32, P, P, P, P, P, P, P, P, c_int32, c_int32,
                                   c_int32, c_int32, P, P, P, P]),
        "ofs_minn_rtl_gate": (c_int32, [P, P, P, c_int64, c_int64, c_int32, c_int32, c_int32, P, P,
                                        P, P]),
        "ofs_cp_cfo": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, P, c_int32, c_int32,
                                 c_double, P, P, P]),
        "ofs_cp_search": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, P, c_int32, c_int32, c_int32,
                                    c_int32, c_double, P, P, P, P, P]),
        "ofs_fft_used": (c_int32, [c_int32, P, c_int64, c_int64, c_int32, c_int32, P, P, P]),
        "ofs_cdiv_eps": (c_int32, [P, c_int64, c_int64, P, c_int64, c_double, P, P]),
        "ofs_common_phase": (c_int32, [P, c_int64, c_int64, P, c_int64, P, P, P]),
        "ofs_align_gain": (c_int32, [P, c_int64, c_int64, P, c_int64, c_double, P, P, P]),
        "ofs_evm": (c_int32, [P, c_int64, c_int64, P, c_int64, P, P, P]),
        "ofs_phase_slope": (c_int32, [P, c_int64, c_int32, P, c_int32, P, P, P]),
        "ofs_apply_cfo": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, P, c_double, P, P]),
        "ofs_quantize_adc": (c_int32, [c_int32, P, c_int64, c_double, c_int32, c_int32, P, P]),
        "ofs_rx_backend": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32, c_double, P, P,
                                     P, c_int32, P, P, c_int64, P, c_int64, P, P, P, P, P, P, P, P, P]),
        "ofs_synth_batch": (c_int32, [P, c_int64, c_int32, c_int64, c_int64, c_int32, c_double, c_double, c_double,
                                      c_double, c_double, ctypes.c_uint64, c_int32, c_double, P, P, P]),
        "ofs_synth_frames": (c_int32, [P, c_int64, P, c_int64, c_int32, c_int32, c_int32, c_int32, c_int32,
                                       c_int32, P, c_int32, c_int32, c_int64, c_int64, c_int64, c_int32,
                                       c_double, c_double, c_double, c_double, c_double, c_double,
                                       ctypes.c_uint64, c_int32, P, P, P, P]),
        "ofs_park_metric": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32, P, P,
                                      P, P]),
        "ofs_zc_correlate": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, P, c_int32, c_double,
                                       c_int32, P, P, P, P]),
        "ofs_zc_freq_metric": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32,
                                         c_int32, c_int32, P, P, c_double, P, P]),
        "ofs_sc_minn_metric": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32, P, P,
                                         P, P, P, P, P]),
        "ofs_win_plan": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_int64, c_int32]),
        "ofs_rtl_plan": (c_int32, [c_int32, c_int32, c_int64, c_int32]),
        "ofs_trailing_average": (c_int32, [c_int32, P, c_int64, c_int64, c_int32, c_int32, P, P]),
        "ofs_plateau_end": (c_int32, [c_int32, P, c_int64, c_int64, c_int32, c_int32, c_int32, P, P, P,
                                      P]),
        "ofs_minn_peak": (c_int32, [P, c_int64, c_int64, c_double, c_int64, c_int64, P, P, P, P, P]),
        "ofs_sc_gate": (c_int32, [c_int32, P, c_int64, c_int64, c_double, P, P, P]),
        "ofs_segment_peak": (c_int32, [P, P, c_int64, c_int64, c_int64, c_int64, P, P, P]),
        "ofs_zc_freq_plan": (c_int32, [c_int32, c_int32, c_int64, c_int32, c_int32]),
        "ofs_zc_freq_partial": (c_int32, [c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32, c_int32,
                                          c_int32, c_int32, P, P, c_int32, P, P]),
        "ofs_zc_freq_finish": (c_int32, [P, c_int64, c_int64, c_double, c_int32, P, P]),
        "ofs_zc_fft_plan_create": (c_int32, [c_int32, c_int32, c_int64, c_int64, P,
                                             ctypes.POINTER(ctypes.c_size_t)]),
        "ofs_zc_fft_plan_create2": (c_int32, [c_int32, c_int32, c_int64, c_int64, c_int32, P,
                                              ctypes.POINTER(ctypes.c_size_t)]),
        "ofs_zc_fft_plan_create3": (c_int32, [c_int32, c_int32, c_int64, c_int64, c_int32, c_int64, P,
                                              ctypes.POINTER(ctypes.c_size_t)]),
        "ofs_zc_fft_plan_create_rows": (c_int32, [c_int32, c_int32, c_int32, c_int64, c_int64, c_int64, c_int32, P,
                                                  ctypes.POINTER(ctypes.c_size_t)]),
        "ofs_zc_fft_plan_chunk": (c_int64, [P]),
        "ofs_zc_fft_plan_destroy": (c_int32, [P]),
        "ofs_zc_freq_metric_fft": (c_int32, [P, c_int32, P, c_int64, c_int32, c_int64, c_int32, c_int32,
                                             c_int32, P, P, c_double, P, P, P, P, P, P]),
        "ofs_zc_mf_plan_create": (c_int32, [P, c_int32, c_int64, c_int32, c_int64, c_int32, P,
                                            ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]),
        "ofs_zc_mf_plan_destroy": (c_int32, [P]),
        "ofs_zc_correlate_fft": (c_int32, [P, c_int32, P, c_int64, c_int32, c_int64, c_double, c_int32, P, P, P,
                                           P, P]),
        "ofs_row_argmax": (c_int32, [c_int32, P, c_int64, c_int64, P, P, P]),
        "ofs_zc_detect": (c_int32, [P, c_int64, c_int64, c_int32, c_int64, c_int32, c_double, c_int32,
                                    c_int32, P, P, P, P, P, P, c_int32, P, P, P, P]),
        "ofs_zc_gate": (c_int32, [P, P, P, c_int64, c_int64, c_int32, c_int32, P, c_int32, P, P, P,
                                  P]),
        "ofs_debug_set_variant": (c_int32, [ctypes.c_char_p, c_int64]),
        "ofs_debug_get_variant": (c_int64, [ctypes.c_char_p]),
        "ofs_debug_reset_variants": (c_int32, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def _baked_hash(l) -> str:
    fn = getattr(l, "ofs_source_hash", None)                # absent in libraries older than the check
    if fn is None:
        return "<none>"
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    return fn().decode()


def lib():
    """Load libofdmsync.so (after torch, so both share torch's HIP runtime).  The library must carry
    the hash of the sources next to it (source_hash()); the one other library accepted is a tuning
    build named explicitly through use_tuning_library()."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
                "from the repository root (hipcc --offload-arch=gfx950)")
        l = ctypes.CDLL(LIB_PATH)
        if source_files():
            built, want = _baked_hash(l), source_hash()
            if built != want:
                raise ImportError(f"{LIB_PATH} was built from other sources (hash {built}, sources {want}); "
                                  "rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
        _declare(l)
        _lib = l
    return _lib


def use_tuning_library(path: str) -> str:
    """Measurement tools only: load a tuning build of tools/variants.py (the sources compiled with
    extra -D flags; its baked hash reads ``variant-<name>``) instead of the in-tree library.  Must
    run before the library is first used; any other library is refused.  Returns the build name."""
    global _lib, TUNING_BUILD, _TUNING_PATH
    path = os.path.abspath(path)
    if _lib is not None and _TUNING_PATH == path:
        return TUNING_BUILD                                  # the same build again: already in use
    if _lib is not None:
        raise RuntimeError("use_tuning_library() must run before the library is first loaded")
    l = ctypes.CDLL(path)
    built = _baked_hash(l)
    if not built.startswith("variant-"):
        raise ImportError(f"{path} is not a tools/variants.py tuning build (hash {built})")
    _declare(l)
    _lib, TUNING_BUILD, _TUNING_PATH = l, built[len("variant-"):], path
    return TUNING_BUILD


# ------------------------------------------------------------------------------------------
# debug / A-B variants (include/ofdmsync.h ofs_debug_set_variant): the library reads no
# environment; tests and measurement tools force an alternative kernel through this entry only
# ------------------------------------------------------------------------------------------
VARIANT_UNSET = -(1 << 63)


def set_variant(name: str, value) -> None:
    """Force (value: int) or clear (value None) one debug variant, e.g. set_variant("EXACT", 0)."""
    rc = lib().ofs_debug_set_variant(name.encode(), VARIANT_UNSET if value is None else int(value))
    if rc != 0:
        raise ValueError(f"unknown variant {name!r}")


def get_variant(name: str):
    v = lib().ofs_debug_get_variant(name.encode())
    return None if v == VARIANT_UNSET else int(v)


def reset_variants() -> None:
    lib().ofs_debug_reset_variants()


class variants:
    """Context manager: ``with variants(EXACT=0, FAST_E=4): ...`` sets the variants for the block
    and restores the previous values after it."""

    def __init__(self, **kw):
        self.kw = kw
        self.prev = {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.prev[k] = get_variant(k)
            set_variant(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.prev.items():
            set_variant(k, v)
        return False


def require_gpu() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("ofdm_sync_amd needs a ROCm GPU (MI355X / gfx950); no CPU fallback exists")
    lib()
    return torch.device("cuda", torch.cuda.current_device())


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().ofs_status_string(rc).decode()
        if rc in (-1, -4):
            raise ValueError(f"{what}: {msg}")
        raise RuntimeError(f"{what}: {msg} (status {rc})")


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


# ------------------------------------------------------------------------------------------
# input normalisation
# ------------------------------------------------------------------------------------------
class Batch:
    """A device tensor of samples laid out [B][n_branch][T] plus its ABI format code."""

    def __init__(self, data: torch.Tensor, fmt: int, B: int, nb: int, T: int, from_numpy: bool,
                 exact_default: bool):
        self.data, self.fmt, self.B, self.nb, self.T = data, fmt, B, nb, T
        self.from_numpy = from_numpy
        self.exact_default = exact_default


def as_batch(x, batched: bool, *, complex_cast: bool = False) -> Batch:
    """Normalise reference-style inputs.

    Unbatched (drop-in) semantics follow the reference: 1-D -> one branch, 2-D -> branches on
    axis 0 (summed).  Batched inputs are [B, n_branch, T] (2-D means [B, T]).  ``int16``
    inputs carry I/Q in a trailing axis of size 2 (OFS_CI16).  ``complex_cast`` forces
    complex128 (minn_rtl.py:680 casts to complex128).
    """
    dev = require_gpu()
    from_numpy = not isinstance(x, torch.Tensor)
    if from_numpy:
        a = np.asarray(x)
        if a.dtype == np.uint8 and a.ndim >= 2 and a.shape[-1] % 3 == 0:
            t = torch.from_numpy(np.ascontiguousarray(a))
        elif a.dtype == np.int16 and a.ndim >= 1 and a.shape[-1] == 2:
            t = torch.from_numpy(np.ascontiguousarray(a))
        else:
            if complex_cast or not np.iscomplexobj(a) or a.dtype not in (np.complex64, np.complex128):
                a = a.astype(np.complex128)
            t = torch.from_numpy(np.ascontiguousarray(a))
        t = t.to(dev, non_blocking=False)
    else:
        t = x
        if t.device.type != "cuda":
            t = t.to(dev)
        packed = t.dtype == torch.uint8 and t.dim() >= 2 and t.shape[-1] % 3 == 0
        if complex_cast and t.dtype != torch.complex128 and t.dtype != torch.int16 and not packed:
            t = t.to(torch.complex128)
        if not (t.is_complex() or (t.dtype == torch.int16 and t.shape[-1] == 2) or packed):
            t = t.to(torch.complex128)
    if t.dtype == torch.uint8:
        # packed 12-bit AXIS words [.., T, 3 * n_ch] (OFS_CP12): channels live in the last axis
        fmt = CP12
        n_ch = t.shape[-1] // 3
        lead = tuple(t.shape[:-2])
        Tn = t.shape[-2]
        if batched:
            if len(lead) != 1:
                raise ValueError("batched packed input must be [B, T, 3 * n_ch] uint8")
            return Batch(t.contiguous(), fmt, lead[0], n_ch, Tn, from_numpy, True)
        if len(lead) != 0:
            raise ValueError("packed input must be [T, 3 * n_ch] uint8")
        return Batch(t.contiguous(), fmt, 1, n_ch, Tn, from_numpy, True)
    if t.dtype == torch.int16:
        fmt = CI16
        core_shape = tuple(t.shape[:-1])
    elif t.dtype == torch.complex64:
        fmt = C64
        core_shape = tuple(t.shape)
    elif t.dtype == torch.complex128:
        fmt = C128
        core_shape = tuple(t.shape)
    else:
        raise TypeError(f"unsupported sample dtype {t.dtype}")
    if batched:
        if len(core_shape) == 2:
            B, nb, T = core_shape[0], 1, core_shape[1]
        elif len(core_shape) == 3:
            B, nb, T = core_shape
        else:
            raise ValueError("batched input must be [B, T] or [B, n_branch, T]")
    else:
        if len(core_shape) == 1:
            B, nb, T = 1, 1, core_shape[0]
        elif len(core_shape) == 2:
            B, nb, T = 1, core_shape[0], core_shape[1]
        else:
            raise ValueError("input must be 1-D (T,) or 2-D (branches, T)")
    t = t.contiguous()
    exact_default = fmt in (C128, CI16)
    return Batch(t, fmt, B, nb, T, from_numpy, exact_default)


def resolve_precision(batch: Batch, precision) -> int:
    if precision is None:
        return FP64 if batch.exact_default else FP32
    if precision in ("fp64", "float64", FP64):
        return FP64
    if precision in ("fp32", "float32", FP32):
        return FP32
    raise ValueError(f"precision must be None, 'fp32' or 'fp64', got {precision!r}")


def out_real(shape, prec: int, dev) -> torch.Tensor:
    return torch.empty(shape, dtype=torch.float64 if prec == FP64 else torch.float32, device=dev)


def out_cplx(shape, prec: int, dev) -> torch.Tensor:
    return torch.empty(shape, dtype=torch.complex128 if prec == FP64 else torch.complex64, device=dev)


class _DeviceBlock:
    """A raw HIP allocation exposed through __cuda_array_interface__ (freed with the object)."""

    def __init__(self, nbytes: int, flags: int):
        self._hip = ctypes.CDLL("libamdhip64.so")
        p = ctypes.c_void_p()
        rc = self._hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flags))
        if rc != 0 or not p.value:
            raise MemoryError(f"hipExtMallocWithFlags({nbytes}, {flags:#x}) failed: {rc}")
        self.ptr, self.nbytes = p.value, nbytes
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                         "version": 2, "strides": None}

    def __del__(self):
        if getattr(self, "ptr", None):
            self._hip.hipFree(ctypes.c_void_p(self.ptr))
            self.ptr = None


HIP_MALLOC_CONTIGUOUS = 0x4           # hipDeviceMallocContiguous (hip_runtime_api.h)


def arena(dev, specs, contiguous: bool = False, gap: int = 0):
    """Carve several output tensors out of ONE device allocation.

    specs: list of (shape, dtype) or None.  Buffers of >= 2 MiB start on 2 MiB boundaries,
    smaller ones on 256 B.  One mapping per batch (one hipMalloc instead of four) with every
    stream 2 MiB-aligned.  Measured (tools/aa_ab.py --realloc, tools/arena_probe.py): the
    headline kernel runs either ~0.275 or ~0.322 ms depending on the box/allocation, with
    separate buffers and with this arena alike; the layout does not select the mode.
    """
    big = 2 << 20
    offs, total = [], 0
    for sp in specs:
        if sp is None:
            offs.append(None)
            continue
        shape, dtype = sp
        n = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
        al = big if n >= big else 256
        total = (total + al - 1) // al * al
        offs.append((total, n, shape, dtype))
        total += n + (gap if n >= big else 0)
    if total == 0:
        return [None if o is None else torch.empty(o[2], dtype=o[3], device=dev) for o in offs]
    if contiguous:
        # physically contiguous backing (hipDeviceMallocContiguous): measured 4 % faster than a
        # plain hipMalloc for the first batch a process allocates
        with torch.cuda.device(dev):
            blk = _DeviceBlock(total + big, HIP_MALLOC_CONTIGUOUS)
            buf = torch.as_tensor(blk, device=dev)
        buf._ofs_block = blk                                     # keep the allocation alive
    else:
        buf = torch.empty(total + big, dtype=torch.uint8, device=dev)
    shift = (-buf.data_ptr()) % big
    out = []
    for o in offs:
        if o is None:
            out.append(None)
            continue
        off, n, shape, dtype = o
        out.append(buf[shift + off:shift + off + n].view(dtype).view(shape))
    return out


def to_host(t: torch.Tensor, dtype=None) -> np.ndarray:
    a = t.detach().cpu().numpy()
    return a if dtype is None else a.astype(dtype, copy=False)
