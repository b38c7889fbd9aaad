"""Synthetic BAM workloads via libdisq_synth.so.

Generator only: it writes inputs for tests and bench.py; it is not part of the read path.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

from . import _build

WGS, ANYSAM, LONGREAD = 0, 1, 2


class _Opts(C.Structure):
    _fields_ = [
        ("n_records", C.c_int64),
        ("seed", C.c_uint64),
        ("shape", C.c_int32),
        ("level", C.c_int32),
        ("nthreads", C.c_int32),
        ("write_bai", C.c_int32),
        ("sbi_granularity", C.c_int64),
        ("records_per_chunk", C.c_int64),
        ("unplaced_fraction", C.c_double),
        ("chunk_lo", C.c_int64),
        ("chunk_hi", C.c_int64),
    ]


class _Res(C.Structure):
    _fields_ = [
        ("bam", C.c_void_p),
        ("bam_len", C.c_int64),
        ("bai", C.c_void_p),
        ("bai_len", C.c_int64),
        ("sbi", C.c_void_p),
        ("sbi_len", C.c_int64),
        ("n_records", C.c_int64),
        ("n_blocks", C.c_int64),
        ("record_bytes", C.c_int64),
        ("n_chunks", C.c_int64),
    ]


_lib = None


def _L():
    global _lib
    if _lib is None:
        _lib = C.CDLL(_build.synth_lib_path())
        _lib.dq_synth_bam.argtypes = [C.POINTER(_Opts), C.POINTER(_Res)]
        _lib.dq_synth_free.argtypes = [C.POINTER(_Res)]
    return _lib


def chunk_count(n_records: int, shape: int = WGS, records_per_chunk: int = 0) -> int:
    """Chunks of the logical file generate(n_records, ...) describes (synth_bam.cpp)."""
    if shape == ANYSAM:
        n_records = 2 * n_records + 2 if n_records > 0 else 0
    per = records_per_chunk if records_per_chunk > 0 else (2000 if shape == LONGREAD else 20000)
    return max(1, (n_records + per - 1) // per)


@dataclass
class SynthBam:
    bam: bytes
    bai: bytes | None
    sbi: bytes | None
    n_records: int
    n_blocks: int
    record_bytes: int

    def write(self, path: str) -> str:
        with open(path, "wb") as f:
            f.write(self.bam)
        if self.bai is not None:
            with open(path + ".bai", "wb") as f:
                f.write(self.bai)
        if self.sbi is not None:
            with open(path + ".sbi", "wb") as f:
                f.write(self.sbi)
        return path


def generate(n_records: int, seed: int = 1, shape: int = WGS, level: int = 5, nthreads: int = 0,
             bai: bool = False, sbi_granularity: int = 0, records_per_chunk: int = 0,
             unplaced_fraction: float = 0.005, as_buffer: bool = False,
             chunks: tuple | None = None):
    """Generate a coordinate-sorted synthetic BAM.

    shape=ANYSAM follows T/AnySamTestUtil.java:37-105 with n_records = numPairs.
    as_buffer=True returns (ctypes address, length, free-callback) without copying (bench path).
    chunks=(lo, hi) generates only chunks [lo, hi) of the logical file: the file's bytes starting
    at the total length of chunks [0, lo) (see n_chunks / chunk_count()).
    """
    lo, hi = chunks if chunks is not None else (0, 0)
    o = _Opts(n_records, seed, shape, level, nthreads or min(16, os.cpu_count() or 1), int(bai),
              sbi_granularity, records_per_chunk, unplaced_fraction, lo, hi)
    r = _Res()
    rc = _L().dq_synth_bam(C.byref(o), C.byref(r))
    if rc != 0:
        raise RuntimeError(f"dq_synth_bam failed: {rc}")
    if as_buffer:
        def free():
            _L().dq_synth_free(C.byref(r))
        return r, free
    def copy(ptr, n):
        # (ctypes.string_at takes a C int size: a file past 2 GiB needs the array view)
        return bytes((C.c_ubyte * n).from_address(ptr)) if n else b""
    try:
        return SynthBam(
            copy(r.bam, r.bam_len),
            copy(r.bai, r.bai_len) if r.bai else None,
            copy(r.sbi, r.sbi_len) if r.sbi else None,
            r.n_records, r.n_blocks, r.record_bytes)
    finally:
        _L().dq_synth_free(C.byref(r))
