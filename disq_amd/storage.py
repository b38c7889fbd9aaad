"""Host-side mirror of Disq's reads API over the MI355X path.

Mirrors, with the same names, argument meaning and error behaviour:
  HtsjdkReadsRddStorage      D/HtsjdkReadsRddStorage.java:17-131 (read side)
  HtsjdkReadsRdd             D/HtsjdkReadsRdd.java:16-38
  HtsjdkReadsTraversalParameters  D/HtsjdkReadsTraversalParameters.java:13-30
  getReads (AbstractBinarySamSource.java:42-136) with BamSource's planning/iteration
  (BamSource.java:61-182) executed by libdisq_gpu.so.

There is no Spark here: the "RDD" is the ordered list of partitions Spark would hold, each a
structure-of-arrays batch of records (plus each record's raw 4 + block_size bytes).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib


class ValidationStringency:
    STRICT = 0
    LENIENT = 1
    SILENT = 2
    DEFAULT_STRINGENCY = STRICT


@dataclass(frozen=True)
class Interval:
    """htsjdk.samtools.util.Interval (1-based, closed)."""
    contig: str
    start: int
    end: int

    def getContig(self):
        return self.contig

    def getStart(self):
        return self.start

    def getEnd(self):
        return self.end


class HtsjdkReadsTraversalParameters:
    def __init__(self, intervalsForTraversal: Optional[Sequence[Interval]],
                 traverseUnplacedUnmapped: bool):
        self._intervals = None if intervalsForTraversal is None else list(intervalsForTraversal)
        self._unplaced = bool(traverseUnplacedUnmapped)

    def getIntervalsForTraversal(self):
        return self._intervals

    def getTraverseUnplacedUnmapped(self):
        return self._unplaced


@dataclass
class SAMFileHeader:
    text: str
    sequences: List[tuple]  # (name, length)
    raw: bytes = b""        # the BAM header as stored (BAMFileWriter.writeHeader's bytes)

    def getSequenceDictionary(self):
        return self.sequences

    def getSequenceIndex(self, name):
        for i, (n, _) in enumerate(self.sequences):
            if n == name:
                return i
        return -1


@dataclass
class ReadsPartition:
    """Records of one Spark partition, as structure-of-arrays."""
    fields: dict
    raw: Optional[np.ndarray]
    digest: int
    path: str = ""

    def __len__(self):
        return len(self.fields["voffset"])

    def record_bytes(self, i):
        o = int(self.fields["raw_offset"][i])
        n = 4 + int(self.fields["block_size"][i])
        return bytes(self.raw[o:o + n])


@dataclass
class ReadsRDD:
    partitions: List[ReadsPartition] = field(default_factory=list)

    def count(self):
        return sum(len(p) for p in self.partitions)

    def getNumPartitions(self):
        return len(self.partitions)

    def field(self, name):
        arrs = [p.fields[name] for p in self.partitions]
        return np.concatenate(arrs) if arrs else np.zeros(0)

    def hashes(self):
        return self.field("hash").astype(np.uint64)


class HtsjdkReadsRdd:
    def __init__(self, header: SAMFileHeader, reads: ReadsRDD):
        self._header = header
        self._reads = reads

    def getHeader(self):
        return self._header

    def getReads(self):
        return self._reads


def _parse_header(raw: bytes) -> SAMFileHeader:
    import struct
    l_text = struct.unpack_from("<i", raw, 4)[0]
    text = raw[8:8 + l_text].decode(errors="replace")
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", raw, p)[0]
    p += 4
    seqs = []
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", raw, p)[0]
        name = raw[p + 4:p + 4 + ln - 1].decode()
        length = struct.unpack_from("<i", raw, p + 4 + ln)[0]
        seqs.append((name, length))
        p += 8 + ln
    return SAMFileHeader(text, seqs, bytes(raw[:p]))


def _is_hidden(name):  # HiddenFileFilter (D/impl/file/HiddenFileFilter.java)
    return name.startswith("_") or name.startswith(".")


class HtsjdkReadsRddStorage:
    """Builder + read() of Disq's reads entry point, backed by libdisq_gpu.so."""

    def __init__(self, device: int = 0):
        self._split_size = 0
        self._stringency = ValidationStringency.DEFAULT_STRINGENCY
        self._use_nio = False
        self._reference = None
        self._device = device
        self._verify_crc = False
        self._use_sbi = False

    @staticmethod
    def makeDefault(device: int = 0) -> "HtsjdkReadsRddStorage":
        return HtsjdkReadsRddStorage(device)

    def splitSize(self, splitSize: int):
        self._split_size = int(splitSize)
        return self

    def validationStringency(self, s: int):
        self._stringency = s
        return self

    def useNio(self, useNio: bool):
        self._use_nio = bool(useNio)
        return self

    def referenceSourcePath(self, p):
        self._reference = p
        return self

    def verifyCrc(self, v: bool):
        """Extension: check every BGZF block's CRC32 (htsjdk's default does not)."""
        self._verify_crc = bool(v)
        return self

    def useSplittingIndex(self, v: bool):
        """Extension: plan partitions from path.sbi (SBIIndex.getChunk) when it exists.  Disq
        itself loads the .sbi and discards the result (BamSource.java:69-87), so the default
        (False) only validates it and plans by record guessing."""
        self._use_sbi = bool(v)
        return self

    def _files(self, path):
        if os.path.isdir(path):
            names = sorted(n for n in os.listdir(path) if not _is_hidden(n))
            return [os.path.join(path, n) for n in names]
        return [path]

    def read(self, path: str, traversalParameters: Optional[HtsjdkReadsTraversalParameters] = None
             ) -> HtsjdkReadsRdd:
        files = self._files(path)
        if not files:
            raise ValueError(f"No files found in {path}")
        first = files[0]
        if not first.endswith(".bam"):
            raise ValueError(f"Cannot find format extension for {path}")
        tp = traversalParameters
        if tp is not None and tp.getIntervalsForTraversal() is None and \
                not tp.getTraverseUnplacedUnmapped():
            # AbstractBinarySamSource.java:50-54
            raise ValueError("Traversing mapped reads only is not supported.")
        header = None
        parts: List[ReadsPartition] = []
        for f in files:
            with _lib.Context(split_size=self._split_size, use_nio=self._use_nio,
                              verify_crc=self._verify_crc, device=self._device,
                              stringency=self._stringency) as ctx:
                ctx.open_path(f)
                sbi = f + ".sbi"  # SBIIndex.FILE_EXTENSION, BamSource.java:69-72
                if os.path.exists(sbi):
                    with open(sbi, "rb") as fh:
                        ctx.set_splitting_index(fh.read(), self._use_sbi)
                _, hraw = ctx.header()
                h = _parse_header(hraw)
                if header is None:
                    header = h
                trav = None
                if tp is not None:
                    bai = self._find_index(f)
                    if bai is None:
                        raise ValueError(f"Intervals set but no index file found for {f}")
                    with open(bai, "rb") as fh:
                        ctx.set_index(fh.read())
                    ivs = tp.getIntervalsForTraversal()
                    conv = None
                    if ivs is not None:
                        conv = []
                        for iv in ivs:  # BoundedTraversalUtil.convertSimpleIntervalToQueryInterval
                            if iv is None:
                                raise ValueError("interval may not be null")
                            idx = h.getSequenceIndex(iv.getContig())
                            if idx == -1:
                                raise ValueError(f"Contig {iv.getContig()} not present in reads "
                                                 "sequence dictionary")
                            conv.append((idx, iv.getStart(), iv.getEnd()))
                    trav = (conv, tp.getTraverseUnplacedUnmapped())
                b = ctx.read(with_raw=True, traversal=trav)
                po = b["part_offset"]
                for p in range(len(po) - 1):
                    lo, hi = int(po[p]), int(po[p + 1])
                    fields = {k: b[k][lo:hi] for k, _ in _lib.FIELDS}
                    raw = None
                    if b["raw"] is not None and hi > lo:
                        r0 = int(fields["raw_offset"][0])
                        r1 = int(fields["raw_offset"][-1]) + 4 + int(fields["block_size"][-1])
                        raw = b["raw"][r0:r1]
                        fields["raw_offset"] = fields["raw_offset"] - r0
                    parts.append(ReadsPartition(fields, raw, int(b["part_digest"][p]), f))
        return HtsjdkReadsRdd(header, ReadsRDD(parts))

    def write(self, rdd: HtsjdkReadsRdd, path: str, tempPartsDirectory: Optional[str] = None):
        """BamSink.save (D/impl/formats/bam/BamSink.java:32-69) with GPU BGZF compression: each
        partition's records as a headerless BGZF part (HeaderlessBamOutputFormat, no terminator),
        the header as its own BGZF blocks, the 28-byte EOF block, then the parts merged in
        partition order (Merger.mergeParts) into `path`; the temporary parts directory is deleted
        after the merge (BamSink.java:67-68).  The header bytes are the ones the file was read
        with (header.raw), not re-encoded from a SAMFileHeader as BAMFileWriter.writeHeader does:
        for a header read by this package they are the same BAM header."""
        header = rdd.getHeader()
        if not header.raw:
            raise ValueError("header has no BAM encoding")
        eof = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
        with _lib.Context(device=self._device) as ctx:
            pieces = [ctx.bgzf_compress(header.raw)]
            for p in rdd.getReads().partitions:
                raw = b"" if p.raw is None else p.raw.tobytes()
                pieces.append(ctx.bgzf_compress(raw))
        pieces.append(eof)
        if tempPartsDirectory:
            os.makedirs(tempPartsDirectory, exist_ok=True)
            names = ["header"] + [f"part-r-{i:05d}" for i in range(len(pieces) - 2)] + ["terminator"]
            for n, d in zip(names, pieces):
                with open(os.path.join(tempPartsDirectory, n), "wb") as fh:
                    fh.write(d)
        with open(path, "wb") as fh:
            for d in pieces:
                fh.write(d)
        if tempPartsDirectory:  # fileSystemWrapper.delete(tempPartsDirectory)
            import shutil
            shutil.rmtree(tempPartsDirectory, ignore_errors=True)
        return path

    @staticmethod
    def _find_index(path):
        # AbstractSamSource.findIndex (D/impl/formats/sam/AbstractSamSource.java:92-108)
        cand = [path + ".bai"]
        if path.endswith(".bam"):
            cand.append(path[: -len(".bam")] + ".bai")
        for c in cand:
            if os.path.exists(c):
                return c
        return None


class VariantsPartition(list):
    """The variant lines of one Spark partition (bytes, terminators excluded)."""


class VariantsRDD:
    def __init__(self, partitions):
        self.partitions = partitions

    def count(self):
        return sum(len(p) for p in self.partitions)

    def getNumPartitions(self):
        return len(self.partitions)

    def collect(self):
        return [l for p in self.partitions for l in p]


class HtsjdkVariantsRdd:
    def __init__(self, header_lines, variants: VariantsRDD):
        self._header = header_lines
        self._variants = variants

    def getHeader(self):
        """The '#' lines of the file (VCFHeader source text)."""
        return self._header

    def getVariants(self):
        """The data lines per partition, as VcfSource hands them to VCFCodec.decode."""
        return self._variants


class HtsjdkVariantsRddStorage:
    """Builder + read() of Disq's variants entry point (D/HtsjdkVariantsRddStorage.java:25-83,
    VcfSource.getVariants D/impl/formats/vcf/VcfSource.java:88-113) for BGZF-compressed VCF on the
    GPU text path.  Lines are returned undecoded: VCFCodec record parsing stays with the caller."""

    def __init__(self, device: int = 0):
        self._split_size = 0
        self._device = device

    @staticmethod
    def makeDefault(device: int = 0) -> "HtsjdkVariantsRddStorage":
        return HtsjdkVariantsRddStorage(device)

    def splitSize(self, splitSize: int):
        self._split_size = int(splitSize)
        return self

    def read(self, path: str, intervals: Optional[Sequence[Interval]] = None) -> HtsjdkVariantsRdd:
        if not (path.endswith(".gz") or path.endswith(".bgz")):
            raise ValueError(f"{path}: the GPU text path reads BGZF-compressed VCF (.vcf.gz/.vcf.bgz)")
        with _lib.Context(split_size=self._split_size, device=self._device) as ctx:
            ctx.text_open_path(path)
            if intervals is not None:
                tbi = path + ".tbi"  # TabixUtils.STANDARD_INDEX_EXTENSION (VcfSource.java:147)
                if not os.path.exists(tbi):
                    raise ValueError(f"Intervals set but no index file found for {path} at {tbi}")
                with open(tbi, "rb") as fh:
                    ctx.text_set_index(fh.read())
                ctx.text_set_intervals([(iv.getContig(), iv.getStart(), iv.getEnd())
                                        for iv in intervals])
            b = ctx.text_read(True)
        d, do, ln, po = b["data"], b["data_offset"], b["line_len"], b["part_offset"]
        parts = [VariantsPartition(bytes(d[do[k]:do[k] + ln[k]]) for k in range(po[p], po[p + 1]))
                 for p in range(len(po) - 1)]
        return HtsjdkVariantsRdd(vcf_header_lines(path), VariantsRDD(parts))


def vcf_header_lines(path: str):
    """The leading '#' lines of a BGZF VCF, read from a prefix of the file: BGZF members are
    inflated from the start (on the driver, as VcfSource.getVCFCodec reads the header through
    htsjdk, D/impl/formats/vcf/VcfSource.java:60-86) only until the first line that does not start
    with '#' (or the end of the file: no byte cap, however many contig/sample lines there are).  Terminators as Hadoop's LineReader: LF, CR LF, lone CR; a UTF-8 BOM on the first
    line is dropped (LineRecordReader.skipUtfByteOrderMark)."""
    import struct
    import zlib
    lines, buf, first, read = [], b"", True, 0
    with open(path, "rb") as fh:
        while True:
            hdr = fh.read(12)
            if len(hdr) < 12:
                break
            if hdr[:4] != b"\x1f\x8b\x08\x04":
                raise ValueError(f"{path}: not a BGZF member at {read}")
            xlen = struct.unpack_from("<H", hdr, 10)[0]
            extra = fh.read(xlen)
            bsize, k = None, 0
            while k + 4 <= len(extra):  # the BC subfield holds BSIZE
                si1, si2, slen = extra[k], extra[k + 1], struct.unpack_from("<H", extra, k + 2)[0]
                if si1 == 66 and si2 == 67 and slen == 2:
                    bsize = struct.unpack_from("<H", extra, k + 4)[0] + 1
                k += 4 + slen
            if bsize is None:
                raise ValueError(f"{path}: BGZF member without a BC subfield at {read}")
            body = fh.read(bsize - 12 - xlen)
            read += bsize
            buf += zlib.decompress(body[:-8], -15)
            if first and buf.startswith(b"\xef\xbb\xbf"):
                buf = buf[3:]
            first = False if buf else first
            # complete lines (a CR at the very end may be the first half of a CR LF)
            pos = 0
            while True:
                i = min([x for x in (buf.find(b"\n", pos), buf.find(b"\r", pos)) if x >= 0],
                        default=-1)
                if i < 0 or (buf[i:i + 1] == b"\r" and i + 1 == len(buf)):
                    break
                line = buf[pos:i]
                if not line.startswith(b"#"):
                    return lines
                lines.append(line)
                pos = i + (2 if buf[i:i + 2] == b"\r\n" else 1)
            buf = buf[pos:]
            if buf and not buf.startswith(b"#"):
                return lines
    if buf.startswith(b"#"):  # a header line that runs to the end of the file
        lines.append(buf.rstrip(b"\r"))
    return lines


class BAMSBIIndexer:
    """htsjdk BAMSBIIndexer (M/htsjdk/samtools/BAMSBIIndexer.java:20-66) on the GPU read path."""

    @staticmethod
    def createIndex(bamFile: str, granularity: int = 4096, device: int = 0) -> str:
        with _lib.Context(device=device) as ctx:
            ctx.open_path(bamFile)
            data = ctx.write_sbi(granularity)
        out = bamFile + ".sbi"
        with open(out, "wb") as fh:
            fh.write(data)
        return out
