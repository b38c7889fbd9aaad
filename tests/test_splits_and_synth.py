"""Split arithmetic (a1), synthetic inputs and interval semantics on the oracle (CPU only)."""
import numpy as np
import pytest

from disq_amd import synth
from oracle import oracle as O


def test_hadoop_splits():
    # Hadoop 2.7 FileInputFormat.getSplits: SPLIT_SLOP 1.1, split = min(splitSize, blockSize)
    assert O.path_splits(597482, 128 * 1024) == [
        (0, 131072), (131072, 262144), (262144, 393216), (393216, 524288), (524288, 597482)]
    assert len(O.path_splits(597482, 40000)) == 15
    assert O.path_splits(597482, 0) == [(0, 597482)]  # one 32 MiB local block
    # slop: a 1.05x remainder stays in the last split
    assert O.path_splits(105, 100) == [(0, 105)]
    assert O.path_splits(111, 100) == [(0, 100), (100, 111)]
    assert O.path_splits(0, 100) == [(0, 0)]
    n = O.path_splits(10 * 2 ** 30, 0)
    assert len(n) == 320 and n[0] == (0, 32 * 2 ** 20)


def test_nio_splits():
    assert O.path_splits(597482, 128 * 1024, nio=True)[-1] == (524288, 597482)
    assert O.path_splits(100, 100, nio=True) == [(0, 100)]
    assert O.path_splits(0, 100, nio=True) == []
    with pytest.raises(O.OracleError):
        O.path_splits(100, 0, nio=True)


@pytest.fixture(scope="module")
def wgs():
    return synth.generate(6000, seed=7, bai=True, sbi_granularity=1, records_per_chunk=2500)


def test_synth_guesser_exact(wgs):
    b = O.OracleBam(wgs.bam)
    sbi = np.frombuffer(wgs.sbi, "<u8", offset=68)
    recs = b.read_all()
    assert len(recs) == wgs.n_records
    assert np.array_equal(recs["voffset"], sbi[:-1])
    hits = np.concatenate([b.scan_record_starts(s, e) for s, e in O.path_splits(b.len, 65536)])
    assert np.array_equal(np.unique(hits), sbi[:-1])


def test_synth_partitions_cover_stream(wgs):
    b = O.OracleBam(wgs.bam)
    allr = b.read_all()
    for ss in (0, 65536, 30000, 100000):
        parts = b.read_partitions(ss)
        cat = np.concatenate(parts)
        # no split starts exactly on a block here -> no duplicates, full coverage, in order
        assert len(cat) >= len(allr)
        assert np.array_equal(np.unique(cat["voffset"]), allr["voffset"])


def test_synth_deterministic():
    a = synth.generate(500, seed=3)
    b = synth.generate(500, seed=3)
    c = synth.generate(500, seed=4)
    assert a.bam == b.bam and a.bam != c.bam


ANYSAM_CASES = [
    # T/HtsjdkReadsRddTest.java:164-301 with AnySamTestUtil.writeAnySamFile(1000, coordinate)
    ([("chr21", 5000, 9999), ("chr21", 20000, 22999)], False, 16),
    ([("chr21", 1, 1000135)], False, 2000),
    ([("chr21", 5000, 9999), ("chr21", 20000, 22999)], True, 18),
    (None, True, 2),
    ([], True, 2),
]


@pytest.fixture(scope="module")
def anysam():
    return synth.generate(1000, shape=synth.ANYSAM, bai=True)


@pytest.mark.parametrize("ivs,unplaced,expected", ANYSAM_CASES)
@pytest.mark.parametrize("split", [40000, 8000])
def test_anysam_interval_counts(anysam, ivs, unplaced, expected, split):
    b = O.OracleBam(anysam.bam)
    conv = None if ivs is None else [(b.ref_index(c), s, e) for c, s, e in ivs]
    parts = b.read_partitions(split, traversal=(conv, unplaced), bai=anysam.bai)
    assert sum(len(p) for p in parts) == expected


def test_mapped_only_fails(anysam):
    b = O.OracleBam(anysam.bam)
    with pytest.raises(ValueError):
        b.read_partitions(40000, traversal=(None, False), bai=anysam.bai)


def test_optimize_intervals():
    q = O.optimize_intervals([(0, 10, 20), (0, 21, 30), (0, 5, 8), (1, 1, 5), (0, 25, 40)])
    assert q == [(0, 5, 8), (0, 10, 40), (1, 1, 5)]
    assert O.optimize_intervals([(0, 10, 20), (0, 22, 30)]) == [(0, 10, 20), (0, 22, 30)]


def test_longread_oracle():
    s = synth.generate(60, seed=5, shape=synth.LONGREAD, sbi_granularity=1)
    b = O.OracleBam(s.bam)
    recs = b.read_all()
    sbi = np.frombuffer(s.sbi, "<u8", offset=68)
    assert np.array_equal(recs["voffset"], sbi[:-1])
    parts = b.read_partitions(65536)
    # partitions whose split holds no record start are empty; the stream is still complete
    assert np.array_equal(np.unique(np.concatenate(parts)["voffset"]), recs["voffset"])
