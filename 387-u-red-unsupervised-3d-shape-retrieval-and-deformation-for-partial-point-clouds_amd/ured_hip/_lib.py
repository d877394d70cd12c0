"""ctypes loader for libured_hip.so (the C-ABI declared in include/ured_hip.h).

There is no CPU fallback: if the library is missing, or a tensor is not on a
ROCm device, the call raises. torch is imported *before* the library is
dlopen'ed so that the library's libamdhip64.so.7 dependency binds to the HIP
runtime torch already loaded (one runtime per process).
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libured_hip.so"
# URED_LIB: an alternative build of the same ABI (A/B kernel experiments, tools/)
LIB_PATH = os.environ.get("URED_LIB") or os.path.join(_HERE, LIB_NAME)
ABI_VERSION = 9

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_SZ = ctypes.c_size_t

# name -> argtypes (all functions return int status, 0 = ok)
_SIGNATURES = {
    "ured_nn_fwd": [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P],
    "ured_nn_bwd": [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "ured_nn_bwd_set": [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "ured_nn_seg_fwd": [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P],
    "ured_nn_fwd_workspace": [_I, _I, _I, _I, _I, _I],
    "ured_seg_aabb": [_P, _P, _I, _P, _P],
    "ured_part_rows_bwd": [_P, _P, _P, _P, _I, _I, _I, _P, _P],
    "ured_part_rows_bwd_add": [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P],
    "ured_get_shape_fwd": [_P, _P, _I, _I, _P, _P],
    "ured_get_shape_bwd": [_P, _P, _I, _I, _P, _P],
    "ured_get_shape_src_fwd": [_P, _P, _I, _P, _P, ctypes.c_float, _I, _I, _P, _P],
    "ured_get_shape_src_bwd": [_P, _P, _I, _P, ctypes.c_float, _I, _I, _P, _P],
    "ured_emd_workspace": [_I, _I],
    "ured_emd_fwd": [_P, _P, _I, _I, _F, _I, _P, _P, _P, _SZ, _P],
    "ured_emd_bwd": [_P, _P, _I, _I, _P, _P, _P, _P],
    "ured_nn_fwd_ws": [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _SZ, _P],
    "ured_nn_seg_fwd_ws": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _SZ, _P],
    "ured_nn_seg_bwd": [_P, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "ured_dcd": [_P, _P, _P, _P, _I, _I, _I, _F, _I, _F, _F, _P, _P, _P, _P],
}

# entry points that return a value instead of a status (see query())
_RESTYPES = {"ured_nn_fwd_workspace": _SZ, "ured_emd_workspace": _SZ}

_lib = None


class UredError(RuntimeError):
    """A libured_hip.so entry point returned a non-zero status."""


def lib():
    """Load (once) and return the ctypes handle; raises ImportError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is not built. Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` from the repo root.")
    handle = ctypes.CDLL(LIB_PATH)
    handle.ured_abi_version.restype = ctypes.c_int
    handle.ured_abi_version.argtypes = []
    handle.ured_last_error.restype = ctypes.c_char_p
    handle.ured_last_error.argtypes = []
    got = handle.ured_abi_version()
    if got != ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: ABI version {got}, expected {ABI_VERSION}")
    for name, argtypes in _SIGNATURES.items():
        fn = getattr(handle, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    _lib = handle
    return _lib


def register(sigs):
    """Add entry points (name -> argtypes); applied now if the library is loaded."""
    _SIGNATURES.update(sigs)
    if _lib is not None:
        for name, argtypes in sigs.items():
            fn = getattr(_lib, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int


def exported_symbols():
    return ["ured_abi_version", "ured_last_error"] + list(_SIGNATURES)


def call(name, *args):
    """Call entry point `name`; raise UredError with the library's message on failure."""
    handle = lib()
    rc = getattr(handle, name)(*args)
    if rc != 0:
        msg = handle.ured_last_error().decode(errors="replace")
        raise UredError(f"{name} failed (status {rc}): {msg}")


def query(name, *args):
    """Call a value-returning entry point (e.g. a workspace size query)."""
    return getattr(lib(), name)(*args)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


# the raw handle of torch's current stream (honours torch.cuda.stream contexts and graph capture)
# without building a Stream object: ~0.3 us instead of ~7 us per launch, which matters for the
# eager step's host issue rate (~1100 launches through here per config-2 step)
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(t):
    """The current torch stream on t's device, as a hipStream_t handle."""
    if _RAW_STREAM is not None and t.device.index is not None:
        return ctypes.c_void_p(_RAW_STREAM(t.device.index))
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def current_stream():
    """The current torch stream on the current device, as a hipStream_t handle."""
    if _RAW_STREAM is not None:
        return ctypes.c_void_p(_RAW_STREAM(torch.cuda.current_device()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def require_device(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(
                "ured_hip ops run on the MI355X only (GPU tensors only, like the reference "
                "chamfer3D extension); got a tensor on " + str(t.device))
