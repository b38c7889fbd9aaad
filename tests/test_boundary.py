"""The C-ABI boundary: libdisq_gpu.so loads and exports every symbol include/disq_gpu.h declares;
the host-side mirror raises the reference's errors before touching the device."""
import ctypes
import os
import re

import pytest

from disq_amd import _build, _lib
from disq_amd.storage import HtsjdkReadsRddStorage, HtsjdkReadsTraversalParameters

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "disq_gpu.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(dq_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_build.gpu_lib_path())
    names = header_functions()
    assert len(names) >= 16
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.EXPORTS)


def test_version_string():
    assert b"gfx950" in _lib.lib().dq_version()


def test_mapped_only_traversal_rejected(golden):
    st = HtsjdkReadsRddStorage.makeDefault().splitSize(40000)
    with pytest.raises(ValueError, match="mapped reads only"):
        st.read(os.path.join(golden, "1.bam"), HtsjdkReadsTraversalParameters(None, False))


def test_unknown_format_rejected(tmp_path):
    p = tmp_path / "x.txt"
    p.write_text("hello")
    with pytest.raises(ValueError, match="format"):
        HtsjdkReadsRddStorage.makeDefault().read(str(p))


def test_structs_match_header_layout():
    # dq_opts 32 bytes, dq_chunk 40, dq_traversal 40, dq_stats 120
    assert ctypes.sizeof(_lib.DqOpts) == 32
    assert ctypes.sizeof(_lib.DqChunk) == 40
    assert ctypes.sizeof(_lib.DqTraversal) == 40
    assert ctypes.sizeof(_lib.DqStats) == 120
