"""ctypes binding of libdisq_gpu.so (include/disq_gpu.h).

This is the same C ABI a JNI / Panama shim binds.  The library is required:
there is no CPU fallback, so a missing or unloadable library raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import weakref

import numpy as np

from . import _build

DQ_OK, DQ_EIO, DQ_EFORMAT, DQ_EINVAL, DQ_EDEVICE, DQ_ENOMEM = 0, -1, -2, -3, -4, -5


class DqOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("split_size", C.c_int32), ("use_nio", C.c_int32),
                ("verify_crc", C.c_int32), ("stringency", C.c_int32),
                ("full_traversal", C.c_int32),
                ("hadoop_block_size", C.c_int64), ("compat", C.c_int32), ("reserved", C.c_int32)]


COMPAT_DISQ_EXACT, COMPAT_DEDUPE = 0, 1
# export modes (the with_raw argument; include/disq_gpu.h)
EXPORT_FIELDS, EXPORT_RAW, EXPORT_LEAN = 0, 1, 2
ABI_VERSION = 2  # DQ_ABI_VERSION this binding maps dq_batch for


class DqChunk(C.Structure):
    _fields_ = [("split_start", C.c_int64), ("split_end", C.c_int64), ("vstart", C.c_uint64),
                ("vend", C.c_uint64), ("has_chunk", C.c_int32), ("reserved", C.c_int32)]


class DqBatch(C.Structure):
    _fields_ = [("n_records", C.c_int64),
                ("voffset", C.POINTER(C.c_uint64)),
                ("block_size", C.POINTER(C.c_int32)),
                ("ref_id", C.POINTER(C.c_int32)),
                ("pos", C.POINTER(C.c_int32)),
                ("l_seq", C.POINTER(C.c_int32)),
                ("next_ref_id", C.POINTER(C.c_int32)),
                ("next_pos", C.POINTER(C.c_int32)),
                ("tlen", C.POINTER(C.c_int32)),
                ("flag", C.POINTER(C.c_uint16)),
                ("bin", C.POINTER(C.c_uint16)),
                ("n_cigar", C.POINTER(C.c_uint16)),
                ("mapq", C.POINTER(C.c_uint8)),
                ("l_read_name", C.POINTER(C.c_uint8)),
                ("hash", C.POINTER(C.c_uint64)),
                ("raw_offset", C.POINTER(C.c_int64)),
                ("raw", C.POINTER(C.c_uint8)),
                ("raw_len", C.c_int64),
                ("n_partitions", C.c_int64),
                ("part_offset", C.POINTER(C.c_int64)),
                ("part_digest", C.POINTER(C.c_uint64)),
                ("in_arena", C.c_int32), ("reserved", C.c_int32), ("arena_hold", C.c_void_p)]


class DqTextBatch(C.Structure):
    _fields_ = [("n_lines", C.c_int64),
                ("line_offset", C.POINTER(C.c_int64)),
                ("line_len", C.POINTER(C.c_int32)),
                ("hash", C.POINTER(C.c_uint64)),
                ("data_offset", C.POINTER(C.c_int64)),
                ("data", C.POINTER(C.c_uint8)),
                ("n_bytes", C.c_int64),
                ("n_partitions", C.c_int64),
                ("part_offset", C.POINTER(C.c_int64)),
                ("part_digest", C.POINTER(C.c_uint64))]


class DqTraversal(C.Structure):
    _fields_ = [("ref", C.POINTER(C.c_int32)), ("start", C.POINTER(C.c_int32)),
                ("end", C.POINTER(C.c_int32)), ("n", C.c_int64), ("has_intervals", C.c_int32),
                ("traverse_unplaced_unmapped", C.c_int32)]


class DqHeaderInfo(C.Structure):
    _fields_ = [("n_ref", C.c_int32), ("reserved", C.c_int32),
                ("first_record_voffset", C.c_uint64), ("header_bytes", C.c_int64)]


class DqStats(C.Structure):
    _fields_ = [("compressed_bytes", C.c_int64), ("decompressed_bytes", C.c_int64),
                ("n_blocks", C.c_int64), ("n_records", C.c_int64), ("n_partitions", C.c_int64),
                ("ms_total", C.c_double), ("ms_scan", C.c_double), ("ms_inflate", C.c_double),
                ("ms_records", C.c_double), ("ms_filter", C.c_double), ("ms_plan", C.c_double),
                ("digest", C.c_uint64), ("ms_crc", C.c_double), ("deflate_bytes", C.c_int64),
                ("n_filtered", C.c_int64), ("h2d_bytes", C.c_int64),
                ("owned_bytes", C.c_int64), ("blocks_inflated", C.c_int64),
                ("ms_span", C.c_double)]


class DqMultiResult(C.Structure):
    _fields_ = [("n_devices", C.c_int32), ("reserved", C.c_int32), ("n_partitions", C.c_int64),
                ("n_records", C.c_int64), ("compressed_bytes", C.c_int64),
                ("decompressed_bytes", C.c_int64), ("digest", C.c_uint64), ("ms_wall", C.c_double),
                ("ms_shard_wall_max", C.c_double), ("ms_device_max", C.c_double)]


# Every symbol include/disq_gpu.h declares.
EXPORTS = ("dq_ctx_create", "dq_ctx_destroy", "dq_last_error", "dq_version", "dq_open_memory",
           "dq_open_path", "dq_set_index", "dq_read_header", "dq_plan", "dq_decode",
           "dq_decode_filtered", "dq_read", "dq_run_resident", "dq_debug_inflated",
           "dq_batch_free", "dq_free", "dq_open_shard", "dq_header_from_prefix",
           "dq_set_splitting_index", "dq_write_sbi", "dq_open_shard_device", "dq_decode_chunk",
           "dq_get_stats", "dq_partition_digests", "dq_open_shard_path",
           "dq_decode_chunk_filtered", "dq_debug_guess_all", "dq_text_open_memory",
           "dq_text_open_path", "dq_text_run", "dq_text_read", "dq_text_batch_free",
           "dq_bgzf_compress", "dq_bgzf_compress_resident", "dq_bgzf_fetch",
           "dq_text_set_index", "dq_text_set_intervals", "dq_decode_file_multi",
           "dq_set_export_arena", "dq_checked_report", "dq_abi_version")

_lib = None
_lock = threading.Lock()


def lib():
    """Load libdisq_gpu.so (raises if it is not built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same soname as
        # /opt/rocm's), and whichever is loaded first serves both.  Loading torch first keeps the
        # runtime torch was built against, so torch.cuda and this library share devices and
        # memory (the multi-GPU path hands torch device tensors to dq_open_shard_device).
        import torch  # noqa: F401
        L = C.CDLL(_build.gpu_lib_path())
        P = C.POINTER
        vp = C.c_void_p
        L.dq_ctx_create.argtypes = [P(vp), P(DqOpts)]
        L.dq_ctx_destroy.argtypes = [vp]
        L.dq_last_error.restype = C.c_char_p
        L.dq_last_error.argtypes = [vp]
        L.dq_version.restype = C.c_char_p
        L.dq_abi_version.restype = C.c_int32
        if L.dq_abi_version() != ABI_VERSION:  # dq_batch's layout is what this binding maps
            raise RuntimeError(f"{_build.gpu_lib_path()}: ABI {L.dq_abi_version()}, binding expects "
                               f"{ABI_VERSION}")
        L.dq_open_memory.argtypes = [vp, vp, C.c_int64]
        L.dq_open_path.argtypes = [vp, C.c_char_p]
        L.dq_set_index.argtypes = [vp, vp, C.c_int64]
        L.dq_set_splitting_index.argtypes = [vp, vp, C.c_int64, C.c_int32]
        L.dq_write_sbi.argtypes = [vp, C.c_int64, P(P(C.c_uint8)), P(C.c_int64)]
        L.dq_open_shard.argtypes = [vp, vp, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                    vp, C.c_int64]
        L.dq_open_shard_device.argtypes = [vp, vp, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                           C.c_int64, vp, C.c_int64]
        L.dq_open_shard_path.argtypes = [vp, C.c_char_p, C.c_int64, C.c_int64, C.c_int64,
                                         C.c_int64, vp, C.c_int64]
        L.dq_decode_chunk.argtypes = [vp, C.c_char_p, C.c_uint64, C.c_uint64, C.c_int32,
                                      P(P(DqBatch))]
        L.dq_decode_chunk_filtered.argtypes = [vp, C.c_char_p, C.c_uint64, C.c_uint64,
                                               P(DqTraversal), C.c_int32, P(P(DqBatch))]
        L.dq_get_stats.argtypes = [vp, P(DqStats)]
        L.dq_partition_digests.argtypes = [vp, P(C.c_int64), P(C.c_uint64), C.c_int64,
                                           P(C.c_int64)]
        L.dq_header_from_prefix.argtypes = [vp, vp, C.c_int64, vp, C.c_int64, P(C.c_int64)]
        L.dq_read_header.argtypes = [vp, P(DqHeaderInfo), vp, C.c_int64]
        L.dq_plan.argtypes = [vp, P(P(DqChunk)), P(C.c_int64)]
        L.dq_decode.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_int32, P(P(DqBatch))]
        L.dq_decode_filtered.argtypes = [vp, C.c_uint64, C.c_uint64, P(DqTraversal), C.c_int32,
                                         P(P(DqBatch))]
        L.dq_read.argtypes = [vp, P(DqTraversal), C.c_int32, P(P(DqBatch))]
        L.dq_run_resident.argtypes = [vp, P(DqTraversal), P(DqStats)]
        L.dq_decode_file_multi.argtypes = [vp, C.c_char_p, P(C.c_int32), C.c_int32, P(DqMultiResult)]
        L.dq_debug_inflated.argtypes = [vp, vp, C.c_int64, P(C.c_int64)]
        L.dq_debug_guess_all.argtypes = [vp, vp, C.c_int64, P(C.c_int64)]
        L.dq_batch_free.argtypes = [P(DqBatch)]
        L.dq_set_export_arena.argtypes = [vp, C.c_int64]
        L.dq_checked_report.argtypes = [P(C.c_uint64)]
        L.dq_text_open_memory.argtypes = [vp, vp, C.c_int64]
        L.dq_text_open_path.argtypes = [vp, C.c_char_p]
        L.dq_text_run.argtypes = [vp, C.c_int32, P(DqStats)]
        L.dq_text_read.argtypes = [vp, C.c_int32, P(P(DqTextBatch))]
        L.dq_text_batch_free.argtypes = [P(DqTextBatch)]
        L.dq_text_set_index.argtypes = [vp, vp, C.c_int64]
        L.dq_text_set_intervals.argtypes = [vp, P(C.c_char_p), P(C.c_int32), P(C.c_int32),
                                            C.c_int64]
        L.dq_bgzf_compress.argtypes = [vp, vp, C.c_int64, P(C.c_void_p), P(C.c_int64)]
        L.dq_bgzf_compress_resident.argtypes = [vp, P(C.c_int64), P(C.c_double)]
        L.dq_bgzf_fetch.argtypes = [vp, vp, C.c_int64]
        L.dq_free.argtypes = [vp]
        _lib = L
        return L


class DqError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _copy_out(ptr, n):
    """n bytes at a library-owned address as bytes (ctypes.string_at takes a C int size, so a
    buffer past 2 GiB needs the array view)."""
    return bytes((C.c_ubyte * n).from_address(ptr)) if n else b""


def check(ctx, rc):
    if rc != DQ_OK:
        raise DqError(rc, lib().dq_last_error(ctx).decode(errors="replace") if ctx else "")
    return rc


FIELDS = (("voffset", np.uint64), ("block_size", np.int32), ("ref_id", np.int32),
          ("pos", np.int32), ("l_seq", np.int32), ("next_ref_id", np.int32),
          ("next_pos", np.int32), ("tlen", np.int32), ("flag", np.uint16), ("bin", np.uint16),
          ("n_cigar", np.uint16), ("mapq", np.uint8), ("l_read_name", np.uint8),
          ("hash", np.uint64), ("raw_offset", np.int64))


def export_mode(with_raw):
    """True / False / "lean" (or the DQ_EXPORT_* value) -> the C ABI's export mode."""
    if isinstance(with_raw, str):
        if with_raw != "lean":
            raise ValueError(f"unknown export mode {with_raw!r}")
        return EXPORT_LEAN
    if isinstance(with_raw, (bool, np.bool_)):
        return EXPORT_RAW if with_raw else EXPORT_FIELDS
    return int(with_raw)


# the fixed fields of a BAM record as its first 36 raw bytes hold them (SAMv1 section 4.2), parsed
# the way htsjdk's BAMRecordCodec.decode reads them (H/BAMFileReader2.java:929-931)
LEAN_HEAD = np.dtype([("block_size", "<i4"), ("ref_id", "<i4"), ("pos", "<i4"),
                      ("l_read_name", "u1"), ("mapq", "u1"), ("bin", "<u2"), ("n_cigar", "<u2"),
                      ("flag", "<u2"), ("l_seq", "<i4"), ("next_ref_id", "<i4"),
                      ("next_pos", "<i4"), ("tlen", "<i4")])


def parse_lean(raw, n):
    """A DQ_EXPORT_LEAN batch's records as a consumer reads them: walk the raw bytes (record i + 1
    starts 4 + block_size bytes after record i) and take the fixed fields from each record's first
    36 bytes.  Returns (raw_offset, fields) with fields a dict of arrays like a full batch's.  A
    plain loop over the block sizes: for tests and small batches (a JVM consumer walks the same
    way in BAMRecordCodec.decode)."""
    raw = np.asarray(raw, np.uint8)
    off = np.zeros(n, np.int64)
    o = 0
    bs = raw.view(np.uint8)
    for i in range(n):
        off[i] = o
        o += 4 + int.from_bytes(bs[o:o + 4].tobytes(), "little")
    if o != len(raw):
        raise ValueError(f"lean batch: {n} records end at byte {o}, raw holds {len(raw)}")
    idx = off[:, None] + np.arange(36)[None, :]
    head = raw[idx].copy().view(LEAN_HEAD).reshape(n)
    return off, {k: head[k].copy() for k in LEAN_HEAD.names}


class _BatchOwner:
    """Frees a dq_batch once no numpy view of its arrays is left.  An arena batch's arrays live in
    its context's pinned export arena (dq_set_export_arena); the C ABI keeps that arena alive for
    the batch even past dq_ctx_destroy and releases it in dq_batch_free."""

    def __init__(self, bp):
        self.bp = bp

    def __del__(self):
        try:
            lib().dq_batch_free(self.bp)
        except Exception:
            pass


_CT = {np.uint64: C.c_uint64, np.int64: C.c_int64, np.int32: C.c_int32, np.uint16: C.c_uint16,
       np.uint8: C.c_uint8}


def batch_to_numpy(bp, ctx=None):
    """The arrays of a dq_batch as numpy views of the library's memory (no copy: a batch of a
    whole file is tens of GB); the batch is freed when the last view is gone.  The views of an
    arena batch are read-only, and `ctx` refuses to overwrite or free its arena while any of them
    is alive (Context._arena_guard)."""
    b = bp.contents
    owner = _BatchOwner(bp)
    arena = bool(b.in_arena)
    if arena and ctx is not None:
        ctx._arena_ref = weakref.ref(owner)

    def view(ptr, n, dt):
        if not n or not ptr:
            return np.zeros(0, dt)
        ct = (_CT[dt] * n).from_address(C.cast(ptr, C.c_void_p).value)
        ct._owner = owner
        a = np.ctypeslib.as_array(ct)
        if arena:
            a.flags.writeable = False
        return a
    n = b.n_records
    out = {name: view(getattr(b, name), n, dt) for name, dt in FIELDS}
    out["raw"] = view(b.raw, b.raw_len, np.uint8) if (b.raw and b.raw_len) else None
    npart = b.n_partitions
    out["part_offset"] = view(b.part_offset, npart + 1, np.int64)
    out["part_digest"] = view(b.part_digest, npart, np.uint64) if npart else np.zeros(0, np.uint64)
    return out


class Context:
    """One dq_ctx (own HIP stream) with a resident BAM."""

    def __init__(self, split_size=0, use_nio=False, verify_crc=False, device=0,
                 hadoop_block_size=0, stringency=0, full_traversal=False,
                 compat=COMPAT_DISQ_EXACT):
        self._h = C.c_void_p()
        o = DqOpts(device, split_size, int(use_nio), int(verify_crc), stringency,
                   int(full_traversal), hadoop_block_size, int(compat), 0)
        rc = lib().dq_ctx_create(C.byref(self._h), C.byref(o))
        if rc != DQ_OK:
            msg = lib().dq_last_error(self._h).decode() if self._h else ""
            if self._h:
                lib().dq_ctx_destroy(self._h)
            self._h = None
            raise DqError(rc, msg)
        self._keep = None
        self._arena_ref = None

    def _arena_live(self):
        r = self._arena_ref
        return r() if r is not None else None

    def _arena_guard(self, what):
        """The library writes every batch of an arena context into the same pinned memory and
        refuses (DQ_EINVAL) a new one while the previous arena batch is alive; this raises the same
        refusal before any device work."""
        if self._arena_live() is not None:
            raise DqError(DQ_EINVAL, f"{what}: the previous batch of this context lives in its "
                          "export arena and is still referenced; drop it (or copy its arrays) "
                          "before the next batch")

    def close(self):
        if self._h:  # (a live arena batch keeps its arena: dq_ctx_destroy leaves it to the batch)
            lib().dq_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def open_bytes(self, data):
        buf = np.frombuffer(data, np.uint8)
        check(self._h, lib().dq_open_memory(self._h, buf.ctypes.data, len(buf)))

    def open_shard(self, data, base, file_len, p0, p1, header):
        """Byte-range shard [base, base + len(data)) owning partitions [p0, p1) (dq_open_shard)."""
        self._shard = np.frombuffer(data, np.uint8)
        self._hdr = np.frombuffer(header, np.uint8).copy()
        check(self._h, lib().dq_open_shard(self._h, self._shard.ctypes.data, len(self._shard),
                                           base, file_len, p0, p1, self._hdr.ctypes.data,
                                           len(self._hdr)))

    def open_shard_device(self, dev_ptr, length, base, file_len, p0, p1, header):
        """Shard bytes already in device memory (dq_open_shard_device): dev_ptr must stay valid,
        with 4096 zero bytes after `length`."""
        self._hdr = np.frombuffer(header, np.uint8).copy()
        check(self._h, lib().dq_open_shard_device(self._h, dev_ptr, length, base, file_len, p0,
                                                  p1, self._hdr.ctypes.data, len(self._hdr)))

    def open_shard_path(self, path, base, length, p0, p1, header):
        """Shard bytes [base, base + length) read from `path` by the library (dq_open_shard_path)."""
        self._hdr = np.frombuffer(header, np.uint8).copy()
        check(self._h, lib().dq_open_shard_path(self._h, os.fsencode(path), base, length, p0, p1,
                                                self._hdr.ctypes.data, len(self._hdr)))

    def decode_chunk(self, path, vstart, vend, with_raw=True, traversal=None):
        """BamSource.getIterator (or createIndexIterator with a traversal) for one task: only the
        chunk's bytes -- or its .bai span -- are read (dq_decode_chunk[_filtered])."""
        self._arena_guard("decode_chunk")
        bp = C.POINTER(DqBatch)()
        if traversal is None:
            check(self._h, lib().dq_decode_chunk(self._h, os.fsencode(path), vstart, vend,
                                                 export_mode(with_raw), C.byref(bp)))
        else:
            t, keep = self._traversal(traversal)
            check(self._h, lib().dq_decode_chunk_filtered(self._h, os.fsencode(path), vstart, vend,
                                                          C.byref(t), export_mode(with_raw), C.byref(bp)))
        return batch_to_numpy(bp, self)

    def stats(self):
        st = DqStats()
        check(self._h, lib().dq_get_stats(self._h, C.byref(st)))
        return st

    def partition_digests(self):
        """(counts, digests) per partition of the last pipeline run, in partition order."""
        n = C.c_int64()
        check(self._h, lib().dq_partition_digests(self._h, None, None, 0, C.byref(n)))
        cnt = np.zeros(max(1, n.value), np.int64)
        dig = np.zeros(max(1, n.value), np.uint64)
        check(self._h, lib().dq_partition_digests(
            self._h, cnt.ctypes.data_as(C.POINTER(C.c_int64)),
            dig.ctypes.data_as(C.POINTER(C.c_uint64)), n.value, C.byref(n)))
        return cnt[:n.value], dig[:n.value]

    def header_from_prefix(self, data):
        """Decompressed BAM header from the first bytes of a file (dq_header_from_prefix)."""
        buf = np.frombuffer(data, np.uint8)
        n = C.c_int64()
        out = np.zeros(1 << 20, np.uint8)
        check(self._h, lib().dq_header_from_prefix(self._h, buf.ctypes.data, len(buf),
                                                   out.ctypes.data, len(out), C.byref(n)))
        if n.value > len(out):
            out = np.zeros(n.value, np.uint8)
            check(self._h, lib().dq_header_from_prefix(self._h, buf.ctypes.data, len(buf),
                                                       out.ctypes.data, len(out), C.byref(n)))
        return bytes(out[: n.value])

    def open_path(self, path):
        check(self._h, lib().dq_open_path(self._h, path.encode()))

    # ---- BGZF compression (write path)
    def bgzf_compress(self, data) -> bytes:
        """BGZF blocks of `data` (65280 bytes each, no EOF terminator), compressed on the GPU."""
        buf = np.frombuffer(data, np.uint8)
        out, n = C.c_void_p(), C.c_int64()
        check(self._h, lib().dq_bgzf_compress(self._h, buf.ctypes.data if len(buf) else None,
                                              len(buf), C.byref(out), C.byref(n)))
        try:
            return _copy_out(out.value, n.value)
        finally:
            lib().dq_free(out)

    def bgzf_compress_resident(self):
        """Compress the open file's resident decompressed stream; (compressed length, device ms)."""
        n, ms = C.c_int64(), C.c_double()
        check(self._h, lib().dq_bgzf_compress_resident(self._h, C.byref(n), C.byref(ms)))
        return n.value, ms.value

    def bgzf_fetch(self, n) -> np.ndarray:
        out = np.zeros(max(1, n), np.uint8)
        check(self._h, lib().dq_bgzf_fetch(self._h, out.ctypes.data, n))
        return out[:n]

    # ---- BGZF text (VCF) path
    def text_open_bytes(self, data):
        buf = np.frombuffer(data, np.uint8)
        check(self._h, lib().dq_text_open_memory(self._h, buf.ctypes.data, len(buf)))

    def text_open_path(self, path):
        check(self._h, lib().dq_text_open_path(self._h, path.encode()))

    def text_set_index(self, tbi_bytes):
        """The tabix index of the open text file (the .tbi as on disk, gzip-decompressed here, as
        htsjdk's IndexFactory does when it loads it); None clears it."""
        if tbi_bytes is None:
            check(self._h, lib().dq_text_set_index(self._h, None, 0))
            return
        import gzip
        d = bytes(tbi_bytes)
        if d[:2] == b"\x1f\x8b":
            d = gzip.decompress(d)
        self._tbi = np.frombuffer(d, np.uint8).copy()
        check(self._h, lib().dq_text_set_index(self._h, self._tbi.ctypes.data, len(self._tbi)))

    def text_set_intervals(self, intervals):
        """[(contig, start, end)] 1-based closed, or None for no interval filter."""
        if intervals is None:
            check(self._h, lib().dq_text_set_intervals(self._h, None, None, None, -1))
            return
        n = len(intervals)
        names = (C.c_char_p * max(1, n))(*[c.encode() for c, _, _ in intervals])
        st = np.array([a for _, a, _ in intervals], np.int32)
        en = np.array([b for _, _, b in intervals], np.int32)
        self._tiv = (names, st, en)  # alive for the call
        check(self._h, lib().dq_text_set_intervals(
            self._h, names, st.ctypes.data_as(C.POINTER(C.c_int32)),
            en.ctypes.data_as(C.POINTER(C.c_int32)), n))

    def text_run(self, drop_header_lines=True):
        st = DqStats()
        check(self._h, lib().dq_text_run(self._h, int(drop_header_lines), C.byref(st)))
        return st

    def text_read(self, drop_header_lines=True):
        """The lines of every split, in partition order: dict of numpy arrays (line_offset,
        line_len, hash, data_offset, data, part_offset, part_digest)."""
        bp = C.POINTER(DqTextBatch)()
        check(self._h, lib().dq_text_read(self._h, int(drop_header_lines), C.byref(bp)))
        try:
            b = bp.contents
            n, npart = b.n_lines, b.n_partitions

            def arr(ptr, k, dt):
                if not k or not ptr:
                    return np.zeros(0, dt)
                return np.ctypeslib.as_array(ptr, shape=(k,)).astype(dt, copy=True)
            return {"line_offset": arr(b.line_offset, n, np.int64),
                    "line_len": arr(b.line_len, n, np.int32),
                    "hash": arr(b.hash, n, np.uint64),
                    "data_offset": arr(b.data_offset, n + 1, np.int64),
                    "data": arr(b.data, b.n_bytes, np.uint8),
                    "part_offset": arr(b.part_offset, npart + 1, np.int64),
                    "part_digest": arr(b.part_digest, npart, np.uint64)}
        finally:
            lib().dq_text_batch_free(bp)

    def set_index(self, bai_bytes):
        if bai_bytes is None:
            check(self._h, lib().dq_set_index(self._h, None, 0))
            return
        self._bai = np.frombuffer(bai_bytes, np.uint8).copy()
        check(self._h, lib().dq_set_index(self._h, self._bai.ctypes.data, len(self._bai)))

    def set_splitting_index(self, sbi_bytes, use_for_planning=False):
        """.sbi bytes (dq_set_splitting_index); planning uses them only if use_for_planning."""
        if sbi_bytes is None:
            check(self._h, lib().dq_set_splitting_index(self._h, None, 0, 0))
            return
        self._sbi = np.frombuffer(sbi_bytes, np.uint8).copy()
        check(self._h, lib().dq_set_splitting_index(self._h, self._sbi.ctypes.data,
                                                    len(self._sbi), int(use_for_planning)))

    def write_sbi(self, granularity=4096):
        """BAMSBIIndexer.createIndex of the open file (dq_write_sbi): the .sbi file's bytes."""
        p = C.POINTER(C.c_uint8)()
        n = C.c_int64()
        check(self._h, lib().dq_write_sbi(self._h, granularity, C.byref(p), C.byref(n)))
        out = _copy_out(C.cast(p, C.c_void_p).value, n.value)
        lib().dq_free(C.cast(p, C.c_void_p))
        return out

    def header(self):
        info = DqHeaderInfo()
        check(self._h, lib().dq_read_header(self._h, C.byref(info), None, 0))
        buf = np.zeros(max(1, info.header_bytes), np.uint8)
        check(self._h, lib().dq_read_header(self._h, C.byref(info), buf.ctypes.data, len(buf)))
        return info, bytes(buf[: info.header_bytes])

    def plan(self):
        p = C.POINTER(DqChunk)()
        n = C.c_int64()
        check(self._h, lib().dq_plan(self._h, C.byref(p), C.byref(n)))
        out = [(p[i].split_start, p[i].split_end,
                (p[i].vstart, p[i].vend) if p[i].has_chunk else None) for i in range(n.value)]
        lib().dq_free(C.cast(p, C.c_void_p))
        return out

    @staticmethod
    def _traversal(tr):
        if tr is None:
            return None, None
        ivs, unplaced = tr
        if ivs is None:
            t = DqTraversal(None, None, None, 0, 0, int(unplaced))
            return t, None
        r = np.array([i[0] for i in ivs], np.int32)
        s = np.array([i[1] for i in ivs], np.int32)
        e = np.array([i[2] for i in ivs], np.int32)
        P = C.POINTER(C.c_int32)
        t = DqTraversal(r.ctypes.data_as(P), s.ctypes.data_as(P), e.ctypes.data_as(P), len(ivs),
                        1, int(unplaced))
        return t, (r, s, e)

    def decode(self, vstart, vend, with_raw=True, traversal=None):
        self._arena_guard("decode")
        bp = C.POINTER(DqBatch)()
        if traversal is None:
            check(self._h, lib().dq_decode(self._h, vstart, vend, export_mode(with_raw), C.byref(bp)))
        else:
            t, keep = self._traversal(traversal)
            check(self._h, lib().dq_decode_filtered(self._h, vstart, vend, C.byref(t),
                                                    export_mode(with_raw), C.byref(bp)))
        return batch_to_numpy(bp, self)

    def set_export_arena(self, nbytes):
        """dq_set_export_arena: later batches of this context land in `nbytes` of pinned host
        memory by DMA; an arena batch's arrays are valid until the next batch of the context
        (a streaming consumer's recycled buffers)."""
        self._arena_guard("set_export_arena")
        check(self._h, lib().dq_set_export_arena(self._h, int(nbytes)))

    def read(self, with_raw=True, traversal=None):
        self._arena_guard("read")
        bp = C.POINTER(DqBatch)()
        t, keep = self._traversal(traversal)
        check(self._h, lib().dq_read(self._h, C.byref(t) if t is not None else None,
                                     export_mode(with_raw), C.byref(bp)))
        return batch_to_numpy(bp, self)

    def run_resident(self, traversal=None):
        st = DqStats()
        t, keep = self._traversal(traversal)
        check(self._h, lib().dq_run_resident(self._h, C.byref(t) if t is not None else None,
                                             C.byref(st)))
        return st

    def decode_file_multi(self, path, devices):
        """dq_decode_file_multi: the file's partitions sharded over `devices` (one context and
        host thread each, records left in HBM); returns DqMultiResult."""
        dv = (C.c_int32 * len(devices))(*devices)
        r = DqMultiResult()
        check(self._h, lib().dq_decode_file_multi(self._h, os.fsencode(path), dv, len(devices),
                                                  C.byref(r)))
        return r

    def inflated(self):
        n = C.c_int64()
        check(self._h, lib().dq_debug_inflated(self._h, None, 0, C.byref(n)))
        out = np.zeros(max(1, n.value), np.uint8)
        check(self._h, lib().dq_debug_inflated(self._h, out.ctypes.data, n.value, C.byref(n)))
        return out[: n.value]

    def guess_all(self):
        """Virtual offsets where the GPU record guesser fires, over every decompressed position
        of the resident file (dq_debug_guess_all)."""
        n = C.c_int64()
        check(self._h, lib().dq_debug_guess_all(self._h, None, 0, C.byref(n)))
        out = np.zeros(max(1, n.value), np.uint64)
        check(self._h, lib().dq_debug_guess_all(self._h, out.ctypes.data, n.value, C.byref(n)))
        return out[: n.value]


CHECK_UNITS = ("K1/K3 kernels", "K2 inflate", "text", "deflate")
CHECK_SITES = ("K1 candidate slot", "K2 bit reader word", "K2 image store", "K2 second-level table",
               "K2 per-lane arrays", "K2 match bitmap", "K2 resolve next pointer",
               "K2 resolve source", "K3 record staging", "K2 last_start",
               "deflate bucket-list slot", "deflate staged symbol", "deflate image word",
               "K3 segment speculation")


def checked_report():
    """dq_checked_report of the current device: (is_checked_build, {unit: (failed checks, [sites],
    largest excess reported)})
    -- the device bounds-checked build (-DDQ_CHECKED)."""
    w = (C.c_uint64 * 4)()
    checked = lib().dq_checked_report(w) == 1
    out = {}
    for name, v in zip(CHECK_UNITS, w):
        n, excess, bits = int(v) >> 32, (int(v) >> 16) & 0xffff, int(v) & 0xffff
        if n or bits:
            out[name] = (n, [CHECK_SITES[i] for i in range(len(CHECK_SITES)) if bits >> i & 1],
                         excess)
    return checked, out
