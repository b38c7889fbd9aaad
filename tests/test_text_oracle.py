"""BGZF text (VCF) path, oracle side: the restatement of Hadoop's
LineRecordReader over Disq's BGZFCodec / BGZFSplitCompressionInputStream
(oracle/disq_oracle.c, dqo_text_split_lines) against the reference's VCF fixtures.

Pinning: the reference's tests (T/HtsjdkVariantsRddTest.java:38-70) assert that the RDD holds
every variant of test.vcf.bgz and HiSeq.10000.vcf.bgz (htsjdk's count) at splitSize 128 KiB; the
plain-text twin test.vcf and the decompressed stream give the exact variant lines.  Which split
a line lands in is pinned only by the restatement (no reference test observes partitions).
"""
import gzip
import os

import numpy as np
import pytest

from oracle import oracle as O
import textutil as T


def variant_lines(text):
    return [l for l in T.split_lines(text) if not l.startswith(b"#")]


def all_lines(ot, split, drop_hash=True):
    parts = ot.read_partitions(split, drop_hash)
    return parts, [l for p in parts for l in ot.lines(p)]


def test_test_vcf_bgz(golden):
    d = open(os.path.join(golden, "test.vcf.bgz"), "rb").read()
    want = variant_lines(open(os.path.join(golden, "test.vcf"), "rb").read())
    assert len(want) == 5
    _, got = all_lines(O.OracleText(d), 128 * 1024)
    assert got == want


@pytest.mark.parametrize("split", [0, 128 * 1024, 100000, 70000, 65536])
def test_hiseq_vcf_every_variant_once(golden, split):
    d = open(os.path.join(golden, "HiSeq.10000.vcf.bgz"), "rb").read()
    want = variant_lines(gzip.decompress(d))
    parts, got = all_lines(O.OracleText(d), split)
    assert got == want
    assert len(got) == 9965
    if split == 128 * 1024:
        assert [len(p[0]) for p in parts] == [2577, 2586, 2631, 2171]


def test_split_without_a_block_start_fails_like_the_reference(golden):
    """A split holding no block start streams from its end, inside a block: htsjdk fails."""
    d = open(os.path.join(golden, "test.vcf.bgz"), "rb").read()
    with pytest.raises(O.OracleError):
        O.OracleText(d).read_partitions(100)


@pytest.mark.parametrize("newline", ["lf", "crlf", "cr", "mixed"])
@pytest.mark.parametrize("bom", [False, True])
def test_synthetic_every_line_once(newline, bom):
    """LF and CR LF files: every line in exactly one partition.  With lone-CR terminators Hadoop
    2.7 can read a line twice: a split whose stream ends on a CR that a fill boundary separates
    from the next byte sets needAdditionalRecord (CompressedSplitLineReader.fillBuffer) and reads
    one more line, which the next split -- whose first block starts with that CR -- reads again
    after dropping the empty line the CR ends.  Then the duplicate is exactly that: the last line
    of one partition repeated as the first line of the next."""
    text = T.make_text(3000, seed=7, newline=newline, bom=bom, hash_every=97)
    bam = T.bgzf_text(text, block_u=3000, cuts=T.corner_cuts(text))
    ot = O.OracleText(bam)
    want = T.split_lines(text)
    if bom:
        want[0] = want[0][3:]
    want = [l for l in want if not l.startswith(b"#")]
    for split in (0, 40000, 25000, 17000):
        parts, got = all_lines(ot, split)
        if newline in ("lf", "crlf"):
            assert got == want, (newline, bom, split)
            continue
        dedup, dups = [], 0
        for p in parts:
            offs = p[0].tolist()
            for i, (o, l) in enumerate(zip(offs, ot.lines(p))):
                if i == 0 and dedup and dedup[-1][0] == o:
                    dups += 1
                    continue
                dedup.append((o, l))
        assert [l for _, l in dedup] == want, (newline, bom, split)


def test_hiseq_interval_keeps_one_partition(golden):
    """T/HtsjdkVariantsRddTest.java:124-149: splitSize 128 KiB, interval chr1:2700000-2800000 ->
    exactly 1 partition (the tabix index filter), holding every overlapping variant."""
    d = open(os.path.join(golden, "HiSeq.10000.vcf.bgz"), "rb").read()
    tbi = open(os.path.join(golden, "HiSeq.10000.vcf.bgz.tbi"), "rb").read()
    iv = [("chr1", 2700000, 2800000)]
    ot = O.OracleText(d)
    parts = ot.read_partitions_intervals(128 * 1024, iv, tbi)
    assert len(parts) == 1
    want = [l for l in variant_lines(gzip.decompress(d)) if O.vcf_overlaps(l, iv)]
    assert ot.lines(parts[0][1]) == want
    assert len(want) == 243


def test_vcf_overlap_uses_info_end():
    text = T.make_vcf(600, seed=2)
    lines = [l for l in T.split_lines(text) if not l.startswith(b"#")]
    f = lines[0].split(b"\t")
    assert f[7].startswith(b"SVTYPE=DEL;END=")
    pos, end = int(f[1]), int(f[7].split(b";")[1][4:])
    assert O.vcf_overlaps(lines[0], [("chr1", end, end)])
    assert not O.vcf_overlaps(lines[0], [("chr1", end + 1, end + 10)])
    assert not O.vcf_overlaps(lines[0], [("chr2", pos, end)])


def test_vcf_header_lines_from_a_prefix():
    """HtsjdkVariantsRddStorage.read's header: the leading '#' lines, read by inflating only the
    first BGZF members (no second full-file read), equal the plain VCF's '#' lines."""
    import os
    from disq_amd.storage import vcf_header_lines
    g = os.path.join(os.path.dirname(__file__), "golden")
    plain = open(os.path.join(g, "test.vcf"), "rb").read().split(b"\n")
    want = []
    for ln in plain:
        if not ln.startswith(b"#"):
            break
        want.append(ln.rstrip(b"\r"))
    assert vcf_header_lines(os.path.join(g, "test.vcf.bgz")) == want
    hs = vcf_header_lines(os.path.join(g, "HiSeq.10000.vcf.bgz"))
    assert hs[0].startswith(b"##fileformat") and hs[-1].startswith(b"#CHROM")


def test_vcf_header_lines_no_byte_cap(tmp_path):
    """A header larger than any fixed prefix (a 64 MB cap truncated it silently): 80 MB
    of '##contig' lines over ~1300 BGZF members, then one variant line."""
    import bamutil as B
    from disq_amd.storage import vcf_header_lines
    n = 800_000
    head = [b"##fileformat=VCFv4.2"] + [b"##contig=<ID=ctg%07d,length=%d,assembly=synthetic_%s>"
                                        % (i, 1000 + i, b"x" * 40) for i in range(n)]
    head.append(b"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO")
    text = b"\n".join(head) + b"\nctg0000001\t5\t.\tA\tC\t.\t.\t.\n"
    assert len(text) > 64 << 20
    p = tmp_path / "big_header.vcf.bgz"
    p.write_bytes(B.bgzf(text, level=1))
    got = vcf_header_lines(str(p))
    assert len(got) == len(head) and got[-1] == head[-1] and got[n // 2] == head[n // 2]
