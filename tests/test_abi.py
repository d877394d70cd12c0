"""CPU-side checks of the drop-in boundary: the C-ABI library builds for gfx950,
loads, and exports every symbol include/ured_hip.h declares (no compute calls)."""
import ctypes
import os
import re

from conftest import ROOT


def _declared():
    hdr = open(os.path.join(ROOT, "include", "ured_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(ured_\w+)\s*\(", hdr, re.M)))


def test_header_symbols_exported(built):
    from ured_hip import _lib
    handle = _lib.lib()
    names = _declared()
    assert len(names) >= 6
    for n in names:
        assert hasattr(handle, n), n
        assert n in _lib.exported_symbols(), f"{n} declared in ured_hip.h but not bound in _lib.py"
    assert handle.ured_abi_version() == _lib.ABI_VERSION
    assert handle.ured_last_error() == b""


def test_invalid_args_report_error_without_gpu(built):
    """Argument validation happens before any device work, so it is testable on CPU."""
    from ured_hip import _lib
    import pytest
    with pytest.raises(_lib.UredError, match="negative size"):
        _lib.call("ured_nn_fwd", None, None, -1, 4, 4, 3, None, None, None, None, None)
    with pytest.raises(_lib.UredError, match="dirs"):
        _lib.call("ured_nn_seg_fwd", None, None, None, 1, 4, 4, 9, None, None, None, None, None)
    import ured_hip.attn  # noqa: F401  (binds the attention entry points)
    with pytest.raises(_lib.UredError, match="nsets"):
        _lib.call("ured_attn_fwd_sets", 3, None, None)


def test_library_is_gfx950(built):
    from ured_hip import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
