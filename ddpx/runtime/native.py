"""ctypes bindings to the ddpx native libraries (HIP kernels + C++ runtime).

The libraries expose a plain C ABI (see ``csrc/``).  Tensors are passed as raw
device pointers and every launch takes the caller's HIP stream, so kernels
issued here are ordered with PyTorch's own work and are captured by HIP graphs
exactly like torch kernels.

Loud failure: on a machine with a GPU the native path is the only path for the
ops that have one; if the library cannot be loaded (and cannot be built in
tree) :func:`kernels` raises instead of silently falling back to eager torch.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported first: provides libamdhip64 / librccl)

from . import build as _build

_lock = threading.Lock()
_K = None
_R = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_uint64 = ctypes.c_uint64
c_size_t = ctypes.c_size_t
c_float = ctypes.c_float
c_double = ctypes.c_double
c_char_p = ctypes.c_char_p


class NativeError(RuntimeError):
    pass


def _sig(lib, name, restype, *argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = list(argtypes)


def _declare_kernels(lib):
    P, I, I64, F = c_void_p, c_int, c_int64, c_float
    _sig(lib, "ddpx_sgd_flat", I, P, P, P, I, P, I64, P, F, F, F, F, I, I, P, P, P)
    _sig(lib, "ddpx_cast_f32_bf16", I, P, P, I64, P)
    _sig(lib, "ddpx_colsum_bf16", I, P, P, I, I, I, F, I, P)
    _sig(lib, "ddpx_scale_f32", I, P, I64, F, P)
    _sig(lib, "ddpx_lr_advance", I, P, I, P, P, P)
    _sig(lib, "ddpx_gemm_pipe", I, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, P, P, P, P, F, F, I, P,
         I64, P, P, I, P, P)
    _sig(lib, "ddpx_gemm_pipe_tiles_m", I, I, I, I, I, I, I)
    _sig(lib, "ddpx_gemm_tile_dims", None, I, ctypes.POINTER(c_int), ctypes.POINTER(c_int))
    _sig(lib, "ddpx_gemm_pipe_plan", I, I, I, I, I, I, I, ctypes.POINTER(c_int), ctypes.POINTER(c_int64),
         ctypes.POINTER(c_int))
    _sig(lib, "ddpx_mx8_quant", I, P, I, I, I, P, I, P, P, I, P, I, P)
    _sig(lib, "ddpx_mx8_probe", I, P, P, P, P, P, I, I, P)
    _sig(lib, "ddpx_gemm_mx8", I, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, F, P, P, P, P, F, F, P)
    _sig(lib, "ddpx_head_fwd_scratch", I64, I, I)
    _sig(lib, "ddpx_head_fwd_tickets", I64, I)
    _sig(lib, "ddpx_head_fwd", I, P, P, P, P, I, I, I, I, F, P, P, P, P, P, P, P, I, P, P, P)
    _sig(lib, "ddpx_head_bwd", I, P, P, P, P, I, I, I, I, P, I, F, P, P, P, I, I, P, P, P, P, P, P, P, P, P, P,
         F, F, P)
    _sig(lib, "ddpx_accuracy", I, P, P, I, I, P, P)
    _sig(lib, "ddpx_augment", I, P, P, P, I, I, I, I, I, c_uint64, I, I, P, P, P)
    _sig(lib, "ddpx_augment_cursor", I, P, P, P, I, I, I, I, I, I, c_uint64, I, I, P, P, P, P)
    _sig(lib, "ddpx_conv_weight_prep", I, P, I, I, I, P, P, P)
    _sig(lib, "ddpx_bn_set_merge", None, I)
    _sig(lib, "ddpx_conv_set_rowcache", None, I)
    _sig(lib, "ddpx_conv_fwd_tiles_m", I, I, I, I, I)
    _sig(lib, "ddpx_conv_fwd_tile_rows", I, I, I, I, I)
    _sig(lib, "ddpx_conv_fwd", I, P, P, P, P, I, I, I, I, I, I, P)
    _sig(lib, "ddpx_conv_dgrad", I, P, P, P, I, I, I, I, I, I, P)
    _sig(lib, "ddpx_conv_fwd_act", I, P, P, P, P, I, I, I, I, I, I, P)
    _sig(lib, "ddpx_conv_dgrad_tiles_m", I, I, I, I, I, I, I)
    _sig(lib, "ddpx_conv_dgrad_act", I, P, P, P, I, I, I, I, I, I, P, P, P)
    _sig(lib, "ddpx_colsum_ws_floats", ctypes.c_longlong, I, I)
    _sig(lib, "ddpx_colsum_finish", I, P, I, I, P, P, I, I, P, P, P, P, F, F, P)
    _sig(lib, "ddpx_conv_dgrad_parts", I, I, I, I, I, I, I)
    _sig(lib, "ddpx_conv_dgrad_bn", I, P, P, P, I, I, I, I, I, I, P, P, P, P, P, I, P, P)
    _sig(lib, "ddpx_conv_wgrad_splits", I, I, I, I, I)
    _sig(lib, "ddpx_conv_wgrad", I, P, P, P, I, I, I, I, I, I, I, P)
    _sig(lib, "ddpx_conv_wgrad_reduce", I, P, I, I, I, I, P, I, I, P, P, P, P, F, F, P, P, P)
    _sig(lib, "ddpx_bn_finalize", I, P, I, I, I, I, P, P, P, P, P, F, F, I, P, P, P, P, P)
    _sig(lib, "ddpx_bn_apply", I, P, P, P, I, I, I, I, I, I, P, P)
    _sig(lib, "ddpx_bn_local_stats", I, P, I, I, I, I, P, P)
    _sig(lib, "ddpx_bn_bwd_sums", I, P, P, P, P, P, P, I, I, I, I, I, I, P, P, P, P, I, I, P)
    _sig(lib, "ddpx_bn_bwd_apply", I, P, P, P, P, P, P, P, P, I, I, I, I, I, I, P, P)
    _sig(lib, "ddpx_bn_bwd_blocks", I, I, I, I, I)
    _sig(lib, "ddpx_bn_bwd", I, P, P, P, P, P, P, I, I, I, I, I, I, P, P, P, P, P, I, I, P, P, P, P, P, P, F, F, P)
    _sig(lib, "ddpx_bn_bwd_sums_from_part", I, P, I, I, P, P, P, I, I, P)
    _sig(lib, "ddpx_bn_bwd_tail", I, P, P, P, P, P, P, I, I, I, I, I, I, P, I, P, P, P, P, I, I, P, P, P, P, P, P, F, F,
         P)
    _sig(lib, "ddpx_bias_act_bwd", I, P, P, P, P, P, I, I, I, I, I, I, P, P, P, P, I, I, P, P)
    _sig(lib, "ddpx_bf16_nchw_flatten", I, P, I, I, I, I, P, P)
    _sig(lib, "ddpx_dropout_fwd", I, P, P, I64, F, P, P, P)
    _sig(lib, "ddpx_avgpool", I, P, I, I, I, P, P)
    _sig(lib, "ddpx_avgpool_bwd", I, P, I, I, I, P, P)
    _sig(lib, "ddpx_debug_spin_wait", I, P, I, c_double, P, P)
    for extra in _EXTRA_KERNEL_SIGS:
        if hasattr(lib, extra[0]):
            _sig(lib, *extra)


# Additional kernels registered by other modules (conv/bn/pool/fp8 ...).
_EXTRA_KERNEL_SIGS: list = []


def register_kernel_sig(name, restype, *argtypes):
    _EXTRA_KERNEL_SIGS.append((name, restype, *argtypes))
    if _K is not None and hasattr(_K, name):
        _sig(_K, name, restype, *argtypes)


def _declare_rt(lib):
    P, I, D, S = c_void_p, c_int, c_double, c_size_t
    _sig(lib, "ddpx_comm_unique_id", I, ctypes.c_char * 128, I)
    _sig(lib, "ddpx_comm_version", I)
    _sig(lib, "ddpx_comm_create", P, c_char_p, I, I, I, I, D, ctypes.POINTER(c_int))
    _sig(lib, "ddpx_comm_create2", P, c_char_p, I, I, I, I, D, I, I, ctypes.POINTER(c_int))
    _sig(lib, "ddpx_comm_stream", P, P)
    _sig(lib, "ddpx_comm_renew_stream", I, P)
    _sig(lib, "ddpx_comm_error", I, P)
    _sig(lib, "ddpx_comm_destroy", I, P, I)
    _sig(lib, "ddpx_comm_allreduce", I, P, P, P, S, I, I, P)
    _sig(lib, "ddpx_comm_broadcast", I, P, P, P, S, I, I, P)
    _sig(lib, "ddpx_comm_reduce_scatter", I, P, P, P, S, I, I, P)
    _sig(lib, "ddpx_comm_allgather", I, P, P, P, S, I, P)
    _sig(lib, "ddpx_comm_track", I, P, P, c_char_p)
    _sig(lib, "ddpx_comm_tracked", c_int64, P)
    _sig(lib, "ddpx_comm_set_timeout", I, P, D, I)
    _sig(lib, "ddpx_hostflag_create", I, ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p))
    _sig(lib, "ddpx_hostflag_set", None, P, I)
    _sig(lib, "ddpx_hostflag_destroy", I, P)
    _sig(lib, "ddpx_comm_group_start", I, P)
    _sig(lib, "ddpx_comm_group_end", I, P)
    _sig(lib, "ddpx_reducer_create", P, P, I, I)
    _sig(lib, "ddpx_reducer_set_bucket", I, P, I, P, S, I, I, I)
    _sig(lib, "ddpx_reducer_set_gather", I, P, I, P, S, I)
    _sig(lib, "ddpx_reducer_gather", I, P, I, P)
    _sig(lib, "ddpx_reducer_wait_gather", I, P, I, P)
    _sig(lib, "ddpx_reducer_mark_backward_end", I, P, P)
    _sig(lib, "ddpx_reducer_comm_stats", I, P, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float))
    _sig(lib, "ddpx_reducer_prepare", I, P)
    _sig(lib, "ddpx_reducer_mark_ready", I, P, I, I, P)
    _sig(lib, "ddpx_reducer_wait_bucket", I, P, I, P)
    _sig(lib, "ddpx_reducer_finalize", I, P, P)
    _sig(lib, "ddpx_reducer_destroy", I, P)


def _load(path):
    return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def _ensure_built():
    need = not (os.path.exists(_build.KERNELS_LIB) and os.path.exists(_build.RT_LIB))
    if need or os.environ.get("DDPX_REBUILD") == "1":
        _build.build(verbose=bool(os.environ.get("DDPX_VERBOSE_BUILD")))


def kernels():
    """Return the loaded kernel library (building it in tree if absent)."""
    global _K
    if _K is None:
        with _lock:
            if _K is None:
                try:
                    _ensure_built()
                    lib = _load(_build.KERNELS_LIB)
                    _declare_kernels(lib)
                except Exception as e:  # pragma: no cover - depends on toolchain
                    raise NativeError(f"ddpx native kernels unavailable: {e}") from e
                _K = lib
    return _K


def runtime():
    """Return the loaded C++ runtime library (RCCL communicator + reducer)."""
    global _R
    if _R is None:
        with _lock:
            if _R is None:
                try:
                    _ensure_built()
                    lib = _load(_build.RT_LIB)
                    _declare_rt(lib)
                except Exception as e:  # pragma: no cover
                    raise NativeError(f"ddpx native runtime unavailable: {e}") from e
                _R = lib
    return _R


def available() -> bool:
    try:
        kernels()
        return True
    except NativeError:
        return False


def loaded_libraries() -> list:
    """Paths of ddpx native libraries mapped into this process."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libddpx" in line:
                    p = line.split()[-1]
                    if p not in out:
                        out.append(p)
    except OSError:
        pass
    return out


def stream_handle(stream: "torch.cuda.Stream | None" = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def sgd_args(sgd):
    """(p, buf, shadow, lr, mom, wd) tuple of tensors/floats -> C argument tuple (nulls when None)."""
    if sgd is None:
        return (None, None, None, None, 0.0, 0.0)
    p, buf, sh, lr, mom, wd = sgd
    return (p.data_ptr(), ptr(buf), ptr(sh), lr.data_ptr(), float(mom), float(wd))


def check(rc: int, what: str):
    if rc != 0:
        raise NativeError(f"{what} failed with code {rc}")
