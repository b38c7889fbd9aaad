"""The oracle (CPU restatement) pinned to the reference's own fixtures and test assertions.

Reference tests mirrored here:
  BgzfBlockSourceTest.testFindAllBlocks      T/impl/formats/bgzf/BgzfBlockSourceTest.java:19-36
  BamRecordGuesserCheckerTest (3 tests)      T/impl/formats/bam/BamRecordGuesserCheckerTest.java:16-70
  HtsjdkReadsRddTest.testReadAndWrite count  T/HtsjdkReadsRddTest.java:42-64 (read side)
  HtsjdkReadsRddTest.testReadUsingSBIIndex   T/HtsjdkReadsRddTest.java:88-102
"""
import json
import os
import struct

import numpy as np
import pytest

from oracle import oracle as O

SPLIT = 128 * 1024


def sbi_offsets(path):
    d = open(path, "rb").read()
    assert d[:4] == b"SBI\x01"
    n = struct.unpack_from("<q", d, 60)[0]
    return np.frombuffer(d, "<u8", count=n, offset=68)


@pytest.fixture(scope="module")
def bam1(golden):
    return O.OracleBam.from_path(os.path.join(golden, "1.bam"))


@pytest.mark.parametrize("nio", [False, True])
def test_find_all_blocks(bam1, nio):
    blocks = []
    for s, e in O.path_splits(bam1.len, SPLIT, nio=nio):
        blocks += bam1.split_blocks(s, e)
    assert len(blocks) == 26
    assert blocks[0] == (0, 14146, 65498)


def test_guesser_all_correct_granularity_one(bam1, golden):
    """Guesser fires exactly at the 4917 SBI record starts and nowhere else."""
    offs = sbi_offsets(os.path.join(golden, "1-with-splitting-index.bam.sbi"))
    hits = np.concatenate([bam1.scan_record_starts(s, e)
                           for s, e in O.path_splits(bam1.len, SPLIT)])
    assert np.array_equal(np.unique(hits), offs[:-1])
    assert len(offs) - 1 == 4917
    # final pointer is the EOF block address with offset 0 (end-of-block normalisation)
    assert (int(offs[-1]) >> 16, int(offs[-1]) & 0xffff) == (597454, 0)


def test_guesser_false_positive_and_negative_detected(bam1, golden):
    """Doctored index: offset[0] + 1 -> exactly one FALSE_POSITIVE and one FALSE_NEGATIVE."""
    offs = sbi_offsets(os.path.join(golden, "1-with-splitting-index.bam.sbi")).copy()
    missing = int(offs[0])
    offs[0] = missing + 1
    actual = set(int(x) for x in offs[:-1])
    mism = []
    for s, e in O.path_splits(bam1.len, SPLIT):
        for blk in bam1.split_blocks(s, e):
            pos, _, us = blk
            hits = set(int(x) for x in bam1.scan_record_starts(pos, pos))  # this block only
            for up in range(us):
                v = (pos << 16) | up
                a, g = v in actual, v in hits
                if a != g:
                    mism.append((v, "FALSE_POSITIVE" if g else "FALSE_NEGATIVE"))
            break  # first block of the split suffices: the doctored offset is in block 0
    mism.sort()
    assert mism == [(missing, "FALSE_POSITIVE"), (missing + 1, "FALSE_NEGATIVE")]


def test_counts_match_sbi(bam1):
    assert len(bam1.read_all()) == 4917
    for ss in (SPLIT, 40000, 0):
        for nio in ((False, True) if ss else (False,)):
            parts = bam1.read_partitions(ss, nio=nio)
            assert sum(len(p) for p in parts) == 4917


def test_partition_counts_and_duplicate_quirk(bam1, golden):
    g = json.load(open(os.path.join(golden, "golden.json")))["1.bam"]
    assert [len(p) for p in bam1.read_partitions(SPLIT)] == [1093, 1030, 1237, 1031, 526]
    assert [len(p) for p in bam1.read_partitions(40000)] == g["partitions_40000"]
    # a block starting exactly on a split boundary is read by both partitions
    # (BgzfBlockSource.java:70 `start > splitEnd`, BamSource.java:140 chunk end (splitEnd, 0xffff))
    assert sum(len(p) for p in bam1.read_partitions(14146)) == 5123
    assert sum(len(p) for p in bam1.read_partitions(19687)) == 4917


def test_records_match_golden(bam1, golden):
    ref = np.load(os.path.join(golden, "1.bam.records.npz"))
    recs = bam1.read_all()
    for k in ("voffset", "block_size", "ref_id", "pos", "flag", "hash"):
        assert np.array_equal(recs[k], ref[k]), k
    sbi = sbi_offsets(os.path.join(golden, "1-with-splitting-index.bam.sbi"))
    assert np.array_equal(recs["voffset"], sbi[:-1])


def test_hiseq_part_without_eof_block(golden):
    b = O.OracleBam.from_path(os.path.join(golden, "hiseq_part-r-00000.bam"))
    blocks = b.split_blocks(0, b.len)
    assert blocks[-1][2] != 0  # no 28-byte EOF terminator: reader must not require one
    recs = b.read_all()
    assert len(recs) == 837 and int((recs["ref_id"] == -1).sum()) == 12
    ref = np.load(os.path.join(golden, "hiseq.records.npz"))
    assert np.array_equal(recs["hash"], ref["hash"])


def test_record_hash_definition():
    # 8-byte little-endian words, zero padded
    assert O.record_hash(b"") == O.record_hash(b"")
    assert O.record_hash(b"\x01") != O.record_hash(b"\x01\x00")  # length is mixed in
    h1 = O.record_hash(bytes(range(40)))
    h2 = O.record_hash(bytes(range(39)) + b"\x00")
    assert h1 != h2
    assert O.stream_digest([1, 2]) != O.stream_digest([2, 1])  # order-dependent


def test_inflate_matches_zlib(bam1):
    import zlib
    d = open(os.path.join(os.path.dirname(__file__), "golden", "1.bam"), "rb").read()
    out, p = [], 0
    while p < len(d):
        bs = struct.unpack_from("<H", d, p + 16)[0] + 1
        out.append(zlib.decompress(d[p + 18:p + bs - 8], -15))
        p += bs
    assert np.array_equal(bam1.inflate_all(), np.frombuffer(b"".join(out), np.uint8))
