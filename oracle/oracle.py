"""ctypes wrapper for the CPU restatement of Disq's BAM read path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker.  The product (disq_amd/, libdisq_gpu.so) never imports it.

Every function mirrors a reference method; see oracle/disq_oracle.c for file:line citations.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libdisq_oracle.so")

REC_DTYPE = np.dtype(
    [
        ("voffset", "<u8"),
        ("lin", "<i8"),
        ("block_size", "<i4"),
        ("ref_id", "<i4"),
        ("pos", "<i4"),
        ("l_seq", "<i4"),
        ("next_ref_id", "<i4"),
        ("next_pos", "<i4"),
        ("tlen", "<i4"),
        ("align_end", "<i4"),
        ("flag", "<u2"),
        ("bin", "<u2"),
        ("n_cigar", "<u2"),
        ("mapq", "u1"),
        ("l_read_name", "u1"),
        ("hash", "<u8"),
    ],
    align=True,
)

HADOOP_LOCAL_BLOCK_SIZE = 32 * 1024 * 1024  # fs.local.block.size default (Hadoop 2.7)


def build() -> str:
    # DQ_ORACLE_LIB: another build of the same sources (tools/oracle_asan.sh: the ASan/UBSan one)
    if os.environ.get("DQ_ORACLE_LIB"):
        return os.environ["DQ_ORACLE_LIB"]
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
        os.path.join(_HERE, "disq_oracle.c")
    ):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        L = _lib
        P = C.POINTER
        L.dqo_open_mem.restype = C.c_void_p
        L.dqo_open_mem.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        L.dqo_close.argtypes = [C.c_void_p]
        L.dqo_last_error.restype = C.c_char_p
        L.dqo_last_error.argtypes = [C.c_void_p]
        L.dqo_path_splits.restype = C.c_int64
        L.dqo_path_splits.argtypes = [C.c_int64, C.c_int32, C.c_int, C.c_int64,
                                      P(C.c_int64), P(C.c_int64), C.c_int64]
        L.dqo_guess_next_bgzf.argtypes = [C.c_void_p, C.c_int64, C.c_int64, P(C.c_int64),
                                          P(C.c_int32), P(C.c_int32)]
        L.dqo_split_blocks.restype = C.c_int64
        L.dqo_split_blocks.argtypes = [C.c_void_p, C.c_int64, C.c_int64, P(C.c_int64),
                                       P(C.c_int32), P(C.c_int32), C.c_int64]
        L.dqo_read_header.argtypes = [C.c_void_p, P(C.c_int32), P(C.c_uint64), P(C.c_int32),
                                      C.c_int32]
        L.dqo_ref_index.restype = C.c_int32
        L.dqo_ref_index.argtypes = [C.c_void_p, C.c_char_p]
        L.dqo_check_record_start.argtypes = [C.c_void_p, C.c_uint64]
        L.dqo_scan_record_starts.restype = C.c_int64
        L.dqo_scan_record_starts.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p,
                                             C.c_int64]
        L.dqo_first_read_in_split.argtypes = [C.c_void_p, C.c_int64, C.c_int64, P(C.c_uint64),
                                              P(C.c_uint64)]
        for fn in (L.dqo_read_chunk,):
            fn.restype = C.c_int64
            fn.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int64]
        L.dqo_read_unmapped.restype = C.c_int64
        L.dqo_read_unmapped.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_int64]
        L.dqo_read_all.restype = C.c_int64
        L.dqo_read_all.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.dqo_bai_info.argtypes = [C.c_void_p, C.c_int64, P(C.c_int32), P(C.c_int64),
                                   P(C.c_int64)]
        L.dqo_bai_span.restype = C.c_int64
        L.dqo_bai_span.argtypes = [C.c_void_p, C.c_int64] + [P(C.c_int32)] * 3 + [
            C.c_int64, C.c_uint64, C.c_uint64, P(C.c_uint64), P(C.c_uint64), C.c_int64]
        L.dqo_optimize_intervals.restype = C.c_int64
        L.dqo_optimize_intervals.argtypes = [P(C.c_int32)] * 3 + [C.c_int64]
        L.dqo_record_overlaps.argtypes = [C.c_void_p] + [P(C.c_int32)] * 3 + [C.c_int64]
        L.dqo_text_split_lines.restype = C.c_int64
        L.dqo_text_split_lines.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_void_p,
                                           C.c_void_p, C.c_int64]
        L.dqo_record_hash.restype = C.c_uint64
        L.dqo_record_hash.argtypes = [C.c_void_p, C.c_int64]
        L.dqo_stream_digest.restype = C.c_uint64
        L.dqo_stream_digest.argtypes = [C.c_void_p, C.c_int64, C.c_uint64]
        L.dqo_inflate_file.restype = C.c_int64
        L.dqo_inflate_file.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.dqo_run_partitions.argtypes = [C.c_void_p, C.c_int64, P(C.c_int64), P(C.c_int64),
                                         C.c_int64, C.c_int, P(C.c_int64), P(C.c_uint64),
                                         P(C.c_int64)]
        L.dqo_run_partitions_window.argtypes = [
            C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_int64, P(C.c_int64),
            P(C.c_int64), C.c_int64, C.c_int, P(C.c_int64), P(C.c_uint64), P(C.c_int64)]
        L.dqo_run_partitions_traversal.argtypes = [
            C.c_void_p, C.c_int64, P(C.c_int64), P(C.c_int64), C.c_int64, C.c_int, C.c_void_p,
            C.c_int64, P(C.c_int32), P(C.c_int32), P(C.c_int32), C.c_int64, C.c_int, C.c_int,
            P(C.c_int64), P(C.c_uint64)]
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class OracleError(RuntimeError):
    pass


def path_splits(file_len, split_size, nio=False, local_block_size=HADOOP_LOCAL_BLOCK_SIZE):
    """PathSplitSource.getPathSplits for one file -> list of (start, end)."""
    L = lib()
    n = L.dqo_path_splits(file_len, split_size, int(nio), local_block_size, None, None, 0)
    if n < 0:
        raise OracleError("invalid split size")
    s = np.zeros(max(n, 1), np.int64)
    e = np.zeros(max(n, 1), np.int64)
    L.dqo_path_splits(file_len, split_size, int(nio), local_block_size, _p(s, C.c_int64),
                      _p(e, C.c_int64), n)
    return list(zip(s[:n].tolist(), e[:n].tolist()))


class OracleBam:
    """A BAM held in memory, read with Disq + htsjdk semantics."""

    def __init__(self, data: bytes, verify_crc: bool = False):
        self._buf = np.frombuffer(data, np.uint8).copy()
        self.len = len(self._buf)
        self._h = lib().dqo_open_mem(self._buf.ctypes.data, self.len, int(verify_crc))
        self._header = None

    @classmethod
    def from_path(cls, path, verify_crc=False):
        with open(path, "rb") as fh:
            return cls(fh.read(), verify_crc)

    def close(self):
        if self._h:
            lib().dqo_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, rc):
        return OracleError(f"oracle error {rc}: {lib().dqo_last_error(self._h).decode()}")

    # a2/a3
    def guess_next_bgzf(self, p, end):
        pos, cs, us = C.c_int64(), C.c_int32(), C.c_int32()
        if lib().dqo_guess_next_bgzf(self._h, p, end, C.byref(pos), C.byref(cs), C.byref(us)):
            return (pos.value, cs.value, us.value)
        return None

    def split_blocks(self, start, end):
        cap = max(16, (end - start) // 16 + 16)
        pos = np.zeros(cap, np.int64)
        cs = np.zeros(cap, np.int32)
        us = np.zeros(cap, np.int32)
        n = lib().dqo_split_blocks(self._h, start, end, _p(pos, C.c_int64), _p(cs, C.c_int32),
                                   _p(us, C.c_int32), cap)
        assert n <= cap
        return list(zip(pos[:n].tolist(), cs[:n].tolist(), us[:n].tolist()))

    # a10
    def header(self):
        if self._header is None:
            nr, first = C.c_int32(), C.c_uint64()
            lens = np.zeros(1 << 16, np.int32)
            rc = lib().dqo_read_header(self._h, C.byref(nr), C.byref(first), _p(lens, C.c_int32),
                                       len(lens))
            if rc != 0:
                raise self._err(rc)
            self._header = {"n_ref": nr.value, "first_record": first.value,
                            "ref_lengths": lens[: nr.value].copy()}
        return self._header

    def ref_index(self, name):
        self.header()
        return lib().dqo_ref_index(self._h, name.encode())

    # a5
    def check_record_start(self, vpos):
        self.header()
        rc = lib().dqo_check_record_start(self._h, vpos)
        if rc < 0:
            raise self._err(rc)
        return bool(rc)

    def scan_record_starts(self, start, end):
        """BamRecordGuesserChecker, granularity 1: guesser hits over one split's blocks."""
        self.header()
        cap = 1 << 20
        out = np.zeros(cap, np.uint64)
        n = lib().dqo_scan_record_starts(self._h, start, end, out.ctypes.data, cap)
        if n < 0:
            raise self._err(n)
        return out[:n].copy()

    # a4
    def first_read_in_split(self, start, end):
        self.header()
        vs, ve = C.c_uint64(), C.c_uint64()
        rc = lib().dqo_first_read_in_split(self._h, start, end, C.byref(vs), C.byref(ve))
        if rc < 0:
            raise self._err(rc)
        return (vs.value, ve.value) if rc == 1 else None

    def _recs(self, fn, *args):
        self.header()
        n = fn(self._h, *args, None, 0)
        if n < 0:
            raise self._err(n)
        out = np.zeros(n, REC_DTYPE)
        m = fn(self._h, *args, out.ctypes.data, n)
        assert m == n
        return out

    # a6-a8
    def read_chunk(self, vstart, vend):
        return self._recs(lib().dqo_read_chunk, vstart, vend)

    def read_unmapped(self, start):
        return self._recs(lib().dqo_read_unmapped, start)

    def read_all(self):
        return self._recs(lib().dqo_read_all)

    def inflate_all(self):
        n = lib().dqo_inflate_file(self._h, None, 0)
        if n < 0:
            raise self._err(n)
        out = np.zeros(n, np.uint8)
        lib().dqo_inflate_file(self._h, out.ctypes.data, n)
        return out

    # L2/L3: AbstractBinarySamSource.getReads over BamSource.getPathChunks
    def plan(self, split_size=0, nio=False, local_block_size=HADOOP_LOCAL_BLOCK_SIZE):
        """getPathChunks: one (split_start, split_end, vstart, vend) or None per split."""
        out = []
        for s, e in path_splits(self.len, split_size, nio, local_block_size):
            out.append((s, e, self.first_read_in_split(s, e)))
        return out

    def read_partitions(self, split_size=0, nio=False, local_block_size=HADOOP_LOCAL_BLOCK_SIZE,
                        traversal=None, bai=None, spans=False):
        """Records per partition, as Disq's RDD would hold them.

        traversal: None, or (intervals, traverse_unplaced_unmapped) where intervals is None or
        a list of (ref_index, start, end) (1-based closed, already converted from contig names).
        spans=True reads only the .bai span of the intervals clipped to each partition chunk
        (AbstractBinarySamSource.java:102-112, as Disq does); False reads the whole chunk.  With a
        complete index both select the same records.
        """
        if traversal is not None:
            ivs, unplaced = traversal
            if ivs is None and not unplaced:
                raise ValueError("Traversing mapped reads only is not supported.")
        parts = []
        plan = self.plan(split_size, nio, local_block_size)
        if traversal is not None:
            if bai is None:
                raise ValueError("Intervals set but no index file found")
            solb, ncc = bai_info(bai)
            q = optimize_intervals(ivs) if ivs else []
        for s, e, ch in plan:
            if ch is None:
                continue  # empty partition (no chunk)
            recs = self.read_chunk(*ch)
            if traversal is None:
                parts.append(recs)
                continue
            if ivs and spans:
                recs = np.concatenate([self.read_chunk(a, b) for a, b in bai_span(bai, q, *ch)]
                                      or [recs[:0]])
            if ivs:
                keep = np.array([overlaps(r, q) for r in recs], bool)
                sel = recs[keep] if len(recs) else recs
            else:
                sel = recs[:0]
            if unplaced and solb != -1 and ncc >= 1 and ch[0] <= solb < ch[1]:
                sel = np.concatenate([sel, self.read_unmapped(solb)])
            parts.append(sel)
        return parts


    # SBI (f1): BAMSBIIndexer.createIndex (M/htsjdk/samtools/BAMSBIIndexer.java:45-66)
    def sbi_final_pointer(self):
        """BlockCompressedInputStream.getFilePointer after the last record of a well-formed file
        (the record stream ends at the end of the last non-empty block): the start of the block
        after it (the EOF block), or the file length (BAMSBIIndexer.java:52-62)."""
        blocks = self.split_blocks(0, self.len)
        last = max((i for i, b in enumerate(blocks) if b[2] > 0), default=-1)
        if last + 1 < len(blocks):
            return blocks[last + 1][0] << 16
        return self.len << 16

    def write_sbi(self, granularity=4096):
        recs = self.read_all()
        return sbi_write(recs["voffset"], self.sbi_final_pointer(), self.len, granularity)

    # SBI planning: getPathChunks with a .sbi honoured (BamSource.java:69-87 as intended)
    def plan_sbi(self, sbi_bytes, split_size=0, nio=False,
                 local_block_size=HADOOP_LOCAL_BLOCK_SIZE):
        offs = sbi_offsets(sbi_bytes)
        return [(s, e, sbi_get_chunk(offs, s, e))
                for s, e in path_splits(self.len, split_size, nio, local_block_size)]

    def read_partitions_sbi(self, sbi_bytes, split_size=0, nio=False,
                            local_block_size=HADOOP_LOCAL_BLOCK_SIZE):
        return [self.read_chunk(*ch) for _, _, ch in
                self.plan_sbi(sbi_bytes, split_size, nio, local_block_size) if ch is not None]


class OracleText:
    """A BGZF-compressed text file (VCF) read as Disq's VcfSource reads it: Hadoop TextInputFormat
    with Disq's splittable BGZF codec (BGZFCodec.java:57-68, BGZFSplitCompressionInputStream.java),
    LineRecordReader per split, lines starting with '#' dropped (VcfSource.java:103-113)."""

    def __init__(self, data: bytes):
        self._buf = np.frombuffer(data, np.uint8).copy()
        self.len = len(self._buf)
        self._h = lib().dqo_open_mem(self._buf.ctypes.data, self.len, 1)
        self._u = None

    def __del__(self):
        try:
            if self._h:
                lib().dqo_close(self._h)
                self._h = None
        except Exception:
            pass

    def inflated(self):
        if self._u is None:
            n = lib().dqo_inflate_file(self._h, None, 0)
            if n < 0:
                raise OracleError(f"oracle error {n}: {lib().dqo_last_error(self._h).decode()}")
            out = np.zeros(n, np.uint8)
            lib().dqo_inflate_file(self._h, out.ctypes.data, n)
            self._u = out
        return self._u

    def split_lines(self, start, end, drop_hash=True):
        """(value offsets in the decompressed stream, value lengths) of split [start, end)."""
        n = lib().dqo_text_split_lines(self._h, start, end, int(drop_hash), None, None, 0)
        if n < 0:
            raise OracleError(f"oracle error {n}: {lib().dqo_last_error(self._h).decode()}")
        vs = np.zeros(max(n, 1), np.int64)
        vl = np.zeros(max(n, 1), np.int64)
        m = lib().dqo_text_split_lines(self._h, start, end, int(drop_hash), vs.ctypes.data,
                                       vl.ctypes.data, n)
        assert m == n
        return vs[:n], vl[:n]

    def read_partitions(self, split_size=0, drop_hash=True, nio=False,
                        local_block_size=HADOOP_LOCAL_BLOCK_SIZE):
        return [self.split_lines(s, e, drop_hash)
                for s, e in path_splits(self.len, split_size, nio, local_block_size)]

    def lines(self, part):
        u = self.inflated()
        vs, vl = part
        return [bytes(u[a:a + b]) for a, b in zip(vs.tolist(), vl.tolist())]

    def read_partitions_intervals(self, split_size, intervals, tbi_bytes, nio=False,
                                  local_block_size=HADOOP_LOCAL_BLOCK_SIZE):
        """VcfSource.getVariants with intervals (D/impl/formats/vcf/VcfSource.java:88-113,
        144-168): TribbleIndexIntervalFilteringTextInputFormat keeps the splits overlapping an
        index block of some interval (TribbleIndexIntervalFilteringTextInputFormat.java:32-68;
        TabixIndex.getBlocks restated as the bins' chunks optimized against the linear index, the
        same rule as the .bai, via dqo_bai_span on the tabix records); each kept split's lines,
        '#' dropped, filtered by OverlapDetector.overlapsAny on (CHROM, POS, end) with end =
        POS + len(REF) - 1 or INFO END.  intervals: [(contig, start, end)] 1-based closed.
        Returns [(split index, (offsets, lengths))] for the kept splits."""
        names, fake_bai = tabix_as_bai(tbi_bytes)
        blocks = []
        for c, a, b in intervals:
            if c not in names:
                continue
            blocks += bai_span(fake_bai, [(names.index(c), a, b)], 0, (1 << 64) - 1)

        def ov(a, b, a2, b2):  # TribbleIndexIntervalFilteringTextInputFormat.overlaps
            return (a <= a2 <= b) or (a <= b2 <= b) or (a >= a2 and b <= b2)
        u = self.inflated()
        out = []
        for k, (s, e) in enumerate(path_splits(self.len, split_size, nio, local_block_size)):
            if not any(ov(s << 16, e << 16, cb, ce) for cb, ce in blocks):
                continue
            vs, vl = self.split_lines(s, e, True)
            keep = [i for i, (a, n) in enumerate(zip(vs.tolist(), vl.tolist()))
                    if vcf_overlaps(bytes(u[a:a + n]), intervals)]
            out.append((k, (vs[keep], vl[keep])))
        return out


def tabix_as_bai(tbi_bytes):
    """(sequence names, the same per-reference index records as .bai bytes) of a tabix index
    (gzip-compressed or not)."""
    import gzip
    import struct
    d = bytes(tbi_bytes)
    if d[:2] == b"\x1f\x8b":
        d = gzip.decompress(d)
    if d[:4] != b"TBI\x01":
        raise OracleError("not a tabix index")
    n_ref = struct.unpack_from("<i", d, 4)[0]
    l_nm = struct.unpack_from("<i", d, 32)[0]
    names = [x.decode() for x in d[36:36 + l_nm].split(b"\x00")[:n_ref]]
    return names, b"BAI\x01" + struct.pack("<i", n_ref) + d[36 + l_nm:]


def vcf_overlaps(line, intervals):
    """OverlapDetector.overlapsAny(VCFCodec.decode(line)) for a data line: contig CHROM, start
    POS, end POS + len(REF) - 1 or the INFO END value (htsjdk AbstractVCFCodec)."""
    f = line.split(b"\t")
    if len(f) < 4:
        return False
    try:
        pos = int(f[1])
    except ValueError:
        return False
    end = pos + len(f[3]) - 1
    if len(f) >= 8:
        for kv in f[7].split(b";"):
            if kv.startswith(b"END="):
                try:
                    end = int(kv[4:])
                except ValueError:
                    pass
                break
    c = f[0].decode(errors="replace")
    return any(c == ic and pos <= ie and end >= ist for ic, ist, ie in intervals)


def sbi_offsets(sbi_bytes):
    """SBIIndex.readIndex (M/htsjdk/samtools/SBIIndex.java:123-144): the virtual offsets."""
    d = bytes(sbi_bytes)
    if d[:4] != b"SBI\x01":
        raise OracleError("Invalid file header in SBI")
    n = int.from_bytes(d[60:68], "little")
    offs = np.frombuffer(d, "<u8", count=n, offset=68)
    if n > 1 and np.any(offs[1:].astype(np.int64) < offs[:-1].astype(np.int64)):
        raise OracleError("Invalid SBI; offsets not in order")
    return offs


def sbi_get_chunk(offs, split_start, split_end):
    """SBIIndex.getChunk (M/htsjdk/samtools/SBIIndex.java:244-264) with ceiling (:266-280)."""
    if split_start >= split_end:
        raise ValueError("Split start must be less than end")
    max_end = int(offs[-1]) >> 16
    vs = min(split_start, max_end) << 16
    ve = min(split_end, max_end) << 16
    a = int(offs[int(np.searchsorted(offs, np.uint64(vs), side="left"))])
    b = int(offs[int(np.searchsorted(offs, np.uint64(ve), side="left"))])
    return None if a == b else (a, b)


def sbi_write(voffsets, final_pointer, file_len, granularity=4096):
    """SBIIndexWriter.processRecord / finish (M/htsjdk/samtools/SBIIndexWriter.java:84-151) with
    no MD5 and no UUID: every granularity-th record's virtual offset, then the final pointer."""
    ent = [int(v) for v in np.asarray(voffsets, np.uint64)[::granularity]] + [int(final_pointer)]
    out = bytearray(b"SBI\x01")
    out += int(file_len).to_bytes(8, "little") + bytes(32)
    for x in (len(voffsets), granularity, len(ent)):
        out += int(x).to_bytes(8, "little")
    for v in ent:
        out += v.to_bytes(8, "little")
    return bytes(out)


def bai_info(bai_bytes):
    b = np.frombuffer(bai_bytes, np.uint8)
    nr, solb, ncc = C.c_int32(), C.c_int64(), C.c_int64()
    rc = lib().dqo_bai_info(b.ctypes.data, len(b), C.byref(nr), C.byref(solb), C.byref(ncc))
    if rc != 0:
        raise OracleError("bad .bai")
    return solb.value, ncc.value


def bai_span(bai_bytes, q, vstart, vend):
    """getFileSpan(optimized intervals q) clipped to the partition chunk [vstart, vend):
    [(begin, end)] virtual-offset chunks in file order (dqo_bai_span)."""
    b = np.frombuffer(bai_bytes, np.uint8)
    r = np.array([i[0] for i in q], np.int32)
    s = np.array([i[1] for i in q], np.int32)
    e = np.array([i[2] for i in q], np.int32)
    args = (b.ctypes.data, len(b), _p(r, C.c_int32), _p(s, C.c_int32), _p(e, C.c_int32), len(q),
            vstart, vend)
    n = lib().dqo_bai_span(*args, None, None, 0)
    if n < 0:
        raise OracleError("bad .bai")
    ob = np.zeros(max(1, n), np.uint64)
    oe = np.zeros(max(1, n), np.uint64)
    lib().dqo_bai_span(*args, _p(ob, C.c_uint64), _p(oe, C.c_uint64), n)
    return list(zip(ob[:n].tolist(), oe[:n].tolist()))


def optimize_intervals(ivs):
    n = len(ivs)
    if n == 0:
        return []
    r = np.array([i[0] for i in ivs], np.int32)
    s = np.array([i[1] for i in ivs], np.int32)
    e = np.array([i[2] for i in ivs], np.int32)
    m = lib().dqo_optimize_intervals(_p(r, C.c_int32), _p(s, C.c_int32), _p(e, C.c_int32), n)
    return list(zip(r[:m].tolist(), s[:m].tolist(), e[:m].tolist()))


def overlaps(rec, q):
    r = np.array([i[0] for i in q], np.int32)
    s = np.array([i[1] for i in q], np.int32)
    e = np.array([i[2] for i in q], np.int32)
    one = np.array([rec], REC_DTYPE)
    return bool(lib().dqo_record_overlaps(one.ctypes.data, _p(r, C.c_int32), _p(s, C.c_int32),
                                          _p(e, C.c_int32), len(q)))


def record_hash(b: bytes) -> int:
    a = np.frombuffer(b, np.uint8)
    return int(lib().dqo_record_hash(a.ctypes.data, len(a)))


def stream_digest(hashes, start_index=0) -> int:
    h = np.ascontiguousarray(hashes, np.uint64)
    return int(lib().dqo_stream_digest(h.ctypes.data, len(h), start_index))


def run_partitions(data: bytes, splits, nthreads):
    """CPU baseline: per-partition (count, digest, bytes) on nthreads threads."""
    buf = np.frombuffer(data, np.uint8)
    n = len(splits)
    s = np.array([a for a, _ in splits], np.int64)
    e = np.array([b for _, b in splits], np.int64)
    cnt = np.zeros(n, np.int64)
    dig = np.zeros(n, np.uint64)
    ub = np.zeros(n, np.int64)
    rc = lib().dqo_run_partitions(buf.ctypes.data, len(buf), _p(s, C.c_int64), _p(e, C.c_int64),
                                  n, nthreads, _p(cnt, C.c_int64), _p(dig, C.c_uint64),
                                  _p(ub, C.c_int64))
    if rc != 0:
        raise OracleError("run_partitions failed")
    return cnt, dig, ub


def run_partitions_window(window, base: int, file_len: int, header: bytes, splits, nthreads):
    """run_partitions over a shard window: `window` holds the file's bytes [base, base + len)
    (a rank's resident bytes + its halo), `header` the file's decompressed BAM header.  Raises
    OracleError("window too short") when a partition needed bytes past the window."""
    buf = np.frombuffer(window, np.uint8)
    hb = np.frombuffer(header, np.uint8)
    n = len(splits)
    s = np.array([a for a, _ in splits] or [0], np.int64)
    e = np.array([b for _, b in splits] or [0], np.int64)
    cnt = np.zeros(max(n, 1), np.int64)
    dig = np.zeros(max(n, 1), np.uint64)
    ub = np.zeros(max(n, 1), np.int64)
    rc = lib().dqo_run_partitions_window(buf.ctypes.data, base, len(buf), file_len, hb.ctypes.data,
                                         len(hb), _p(s, C.c_int64), _p(e, C.c_int64), n, nthreads,
                                         _p(cnt, C.c_int64), _p(dig, C.c_uint64), _p(ub, C.c_int64))
    if rc == -6:
        raise OracleError("window too short")
    if rc != 0:
        raise OracleError(f"run_partitions_window failed ({rc})")
    return cnt[:n], dig[:n], ub[:n]


def run_partitions_traversal(data: bytes, splits, nthreads, bai: bytes, intervals,
                             unplaced=False, spans=True):
    """Interval traversal of every partition (count, digest) on nthreads threads, as
    OracleBam.read_partitions(traversal=(intervals, unplaced), bai=..., spans=...) followed by
    stream_digest per partition, but in C: the bench-scale parity of the GPU span runs."""
    buf = np.frombuffer(data, np.uint8)
    b = np.frombuffer(bai, np.uint8)
    q = optimize_intervals(intervals) if intervals else []
    r = np.array([i[0] for i in q] or [0], np.int32)
    s = np.array([i[1] for i in q] or [0], np.int32)
    e = np.array([i[2] for i in q] or [0], np.int32)
    n = len(splits)
    st = np.array([a for a, _ in splits], np.int64)
    en = np.array([x for _, x in splits], np.int64)
    cnt = np.zeros(n, np.int64)
    dig = np.zeros(n, np.uint64)
    rc = lib().dqo_run_partitions_traversal(
        buf.ctypes.data, len(buf), _p(st, C.c_int64), _p(en, C.c_int64), n, nthreads,
        b.ctypes.data, len(b), _p(r, C.c_int32), _p(s, C.c_int32), _p(e, C.c_int32), len(q),
        int(unplaced), int(spans), _p(cnt, C.c_int64), _p(dig, C.c_uint64))
    if rc != 0:
        raise OracleError("run_partitions_traversal failed")
    return cnt, dig
