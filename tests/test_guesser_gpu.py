"""The GPU record guesser at every decompressed position, checked the way the reference's
BamRecordGuesserCheckerTest does (T/impl/formats/bam/BamRecordGuesserCheckerTest.java:16-70): the
SBI index of granularity 1 is the ground truth for record starts, so every position where the
guesser and the index disagree is a FALSE_POSITIVE (guesser fires, no record) or a FALSE_NEGATIVE
(record, guesser silent) -- BamRecordGuesserChecker.java:104-120.

Bar: no mismatch on 1.bam against the reference's own .sbi fixture; exactly the two mismatches of
the doctored index (offset[0] + 1); and on synthetic files the GPU guesser fires at exactly the
positions where the oracle's restatement fires (true starts and any data-dependent false hits).
"""
import os
import struct

import numpy as np
import pytest

from disq_amd import _lib, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SPLIT = 128 * 1024  # BamRecordGuesserCheckerTest.SPLIT_SIZE


def sbi_offsets(path):
    d = open(path, "rb").read()
    assert d[:4] == b"SBI\x01"
    assert struct.unpack_from("<q", d, 52)[0] == 1  # granularity 1: every record start
    n = struct.unpack_from("<q", d, 60)[0]
    return np.frombuffer(d, "<u8", count=n, offset=68).copy()


def mismatches(guessed, index_offsets):
    """BamRecordGuesserChecker.check over every position of every block: the final offset of the
    index (the end-of-records pointer) is not a record start."""
    g, a = set(int(x) for x in guessed), set(int(x) for x in index_offsets[:-1])
    out = [(v, "FALSE_POSITIVE") for v in g - a] + [(v, "FALSE_NEGATIVE") for v in a - g]
    return sorted(out)


@pytest.fixture(scope="module")
def guessed_1bam(golden):
    with _lib.Context(split_size=SPLIT) as c:
        c.open_path(os.path.join(golden, "1.bam"))
        return c.guess_all()


def test_all_correct_granularity_one(guessed_1bam, golden):
    offs = sbi_offsets(os.path.join(golden, "1-with-splitting-index.bam.sbi"))
    assert mismatches(guessed_1bam, offs) == []
    assert len(guessed_1bam) == 4917


def test_false_positive_and_false_negative_detected(guessed_1bam, golden):
    offs = sbi_offsets(os.path.join(golden, "1-with-splitting-index.bam.sbi"))
    missing = int(offs[0])
    offs[0] = missing + 1  # the doctored index of the reference test
    assert mismatches(guessed_1bam, offs) == [(missing, "FALSE_POSITIVE"),
                                              (missing + 1, "FALSE_NEGATIVE")]


def oracle_all_hits(ob, split):
    return np.unique(np.concatenate([ob.scan_record_starts(s, e)
                                     for s, e in O.path_splits(ob.len, split)]))


@pytest.mark.parametrize("shape,n,seed", [(synth.WGS, 3000, 3), (synth.ANYSAM, 1000, 0),
                                          (synth.LONGREAD, 60, 9)])
def test_gpu_guesser_equals_oracle_everywhere(tmp_path, shape, n, seed):
    r = synth.generate(n, seed=seed, shape=shape, nthreads=8)
    ob = O.OracleBam(r.bam)
    want = oracle_all_hits(ob, 64 * 1024)
    with _lib.Context(split_size=64 * 1024) as c:
        c.open_bytes(r.bam)
        got = c.guess_all()
    assert np.array_equal(got, want)
    # every true record start is found (no false negatives)
    starts = ob.read_all()["voffset"].astype(np.uint64)
    assert np.isin(starts, got).all()
