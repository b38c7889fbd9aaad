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


def test_structs_match_header_layout(tmp_path):
    """ctypes mirrors of the C structs have the header's sizes and field offsets (gcc on the
    header itself)."""
    import subprocess
    structs = {"dq_opts": _lib.DqOpts, "dq_chunk": _lib.DqChunk, "dq_batch": _lib.DqBatch,
               "dq_traversal": _lib.DqTraversal, "dq_header_info": _lib.DqHeaderInfo,
               "dq_stats": _lib.DqStats}
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "disq_gpu.h"', "int main(void){"]
    for name, cls in structs.items():
        src.append(f'printf("{name} %zu\\n", sizeof({name}));')
        for f, _ in cls._fields_:
            src.append(f'printf("{name}.{f} %zu\\n", offsetof({name}, {f}));')
    src.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", "-I", inc, "-o", str(exe), str(c)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                       text=True).stdout.splitlines())
    for name, cls in structs.items():
        assert int(got[name]) == ctypes.sizeof(cls), name
        for f, _ in cls._fields_:
            assert int(got[f"{name}.{f}"]) == getattr(cls, f).offset, (name, f)
