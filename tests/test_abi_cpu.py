"""The ctypes signature table (ops/_lib.py _SIGS) against the extern "C" entry points in csrc/:
every declared function exists with the same parameter count (ctypes would pass a surplus
argument through as a C vararg and shift the trailing stream handle), and the loaded library
refuses a call with the wrong count."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _decls():
    src = ""
    for pat in ("csrc/**/*.hip", "csrc/**/*.cpp", "csrc/*.h"):
        for f in glob.glob(os.path.join(ROOT, pat), recursive=True):
            with open(f) as fh:
                src += fh.read()
    out = {}
    for m in re.finditer(r'extern "C" [\w\s\*]+?\b(r2_\w+)\s*\(([^)]*)\)\s*\{', src):
        a = m.group(2).strip()
        out[m.group(1)] = 0 if a in ("", "void") else len(a.split(","))
    return out


def test_ctypes_table_matches_sources():
    from pytorch_r2d2_amd.ops._lib import _SIGS
    d = _decls()
    assert not [k for k in _SIGS if k not in d]
    assert not [(k, len(v), d[k]) for k, v in _SIGS.items() if d[k] != len(v)]


def test_strict_wrapper_refuses_wrong_arg_count():
    from pytorch_r2d2_amd.ops import _lib
    if not _lib.available():
        pytest.skip("kernel library not built")
    k = _lib.kernels()
    with pytest.raises(TypeError):
        k.r2_gemm5_set_mode(0, 1)
    assert k.r2_gemm5_set_mode(0) == 0
