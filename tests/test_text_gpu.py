"""BGZF text (VCF) path on the GPU: dq_text_* against the oracle's
restatement of LineRecordReader over Disq's BGZFCodec (oracle/disq_oracle.c), partition by
partition -- value offsets, lengths, bytes and hashes -- on the reference's VCF fixtures and on
synthetic files that put block boundaries at the reader's corners (after a CR, between CR and
LF, on a line start), with LF / CR LF / lone-CR terminators, a UTF-8 BOM and '#' lines."""
import gzip
import os

import numpy as np
import pytest

from disq_amd import _lib
from oracle import oracle as O
import textutil as T

pytestmark = pytest.mark.gpu


def assert_text_parity(data, split, drop_hash=True):
    ot = O.OracleText(data)
    parts = ot.read_partitions(split, drop_hash)
    with _lib.Context(split_size=split, verify_crc=True) as c:
        c.text_open_bytes(data)
        st = c.text_run(drop_hash)
        b = c.text_read(drop_hash)
    po = b["part_offset"]
    assert len(po) - 1 == len(parts)
    u = ot.inflated()
    n = 0
    for i, (vs, vl) in enumerate(parts):
        lo, hi = int(po[i]), int(po[i + 1])
        assert hi - lo == len(vs), (split, i)
        assert np.array_equal(b["line_offset"][lo:hi], vs), (split, i)
        assert np.array_equal(b["line_len"][lo:hi], vl), (split, i)
        want = O.stream_digest([O.record_hash(bytes(u[a:a + l])) for a, l in zip(vs, vl)])
        assert int(b["part_digest"][i]) == want, (split, i)
        n += len(vs)
    assert st.n_records == n == len(b["line_len"])
    # the exported bytes are the values
    d, do = b["data"], b["data_offset"]
    for k in np.linspace(0, n - 1, num=min(n, 40), dtype=int) if n else []:
        a, l = int(b["line_offset"][k]), int(b["line_len"][k])
        assert bytes(d[do[k]:do[k] + l]) == bytes(u[a:a + l])
    return b


@pytest.mark.parametrize("split", [0, 128 * 1024, 100000, 70000, 65536])
def test_hiseq_vcf(golden, split):
    d = open(os.path.join(golden, "HiSeq.10000.vcf.bgz"), "rb").read()
    b = assert_text_parity(d, split)
    assert len(b["line_len"]) == 9965


def test_test_vcf(golden):
    d = open(os.path.join(golden, "test.vcf.bgz"), "rb").read()
    b = assert_text_parity(d, 128 * 1024)
    want = [l for l in T.split_lines(open(os.path.join(golden, "test.vcf"), "rb").read())
            if not l.startswith(b"#")]
    got = [bytes(b["data"][b["data_offset"][k]:b["data_offset"][k] + b["line_len"][k]])
           for k in range(len(b["line_len"]))]
    assert got == want


def test_keep_header_lines(golden):
    d = open(os.path.join(golden, "HiSeq.10000.vcf.bgz"), "rb").read()
    b = assert_text_parity(d, 128 * 1024, drop_hash=False)
    assert len(b["line_len"]) == len(T.split_lines(gzip.decompress(d)))


@pytest.mark.parametrize("newline", ["lf", "crlf", "cr", "mixed"])
@pytest.mark.parametrize("bom", [False, True])
def test_synthetic_corners(newline, bom):
    text = T.make_text(3000, seed=7, newline=newline, bom=bom, hash_every=97)
    data = T.bgzf_text(text, block_u=3000, cuts=T.corner_cuts(text))
    for split in (0, 40000, 25000, 17000):
        assert_text_parity(data, split)


def test_long_lines_span_many_blocks():
    text = T.make_text(400, seed=3, newline="lf", long_every=50, long_len=300000)
    data = T.bgzf_text(text)
    for split in (0, 200000, 90000):
        assert_text_parity(data, split)


def test_split_without_block_start_fails(golden):
    d = open(os.path.join(golden, "test.vcf.bgz"), "rb").read()
    with pytest.raises(O.OracleError):
        O.OracleText(d).read_partitions(100)
    with _lib.Context(split_size=100) as c:
        c.text_open_bytes(d)
        with pytest.raises(_lib.DqError, match="no BGZF block starts"):
            c.text_run()


def assert_interval_parity(data, split, intervals, tbi):
    ot = O.OracleText(data)
    want = ot.read_partitions_intervals(split, intervals, tbi)
    with _lib.Context(split_size=split, verify_crc=True) as c:
        c.text_open_bytes(data)
        c.text_set_index(tbi)
        c.text_set_intervals(intervals)
        st = c.text_run()
        b = c.text_read()
    po = b["part_offset"]
    assert len(po) - 1 == len(want) == st.n_partitions
    for i, (_, (vs, vl)) in enumerate(want):
        lo, hi = int(po[i]), int(po[i + 1])
        assert np.array_equal(b["line_offset"][lo:hi], vs), i
        assert np.array_equal(b["line_len"][lo:hi], vl), i
    return b, want


@pytest.mark.parametrize("intervals,nparts", [
    ([("chr1", 2700000, 2800000)], 1),   # T/HtsjdkVariantsRddTest.java:127: one partition
    ([("chr1", 1, 100000)], None),
    ([("chr1", 2700000, 2800000), ("chr1", 4000000, 4100000), ("chr1", 4050000, 4060000)], None),
    ([("chr2", 1, 1000000)], 0),          # a contig the index does not know: no split
    ([("chr1", 1, 300000000)], 4),
])
def test_hiseq_vcf_intervals(golden, intervals, nparts):
    d = open(os.path.join(golden, "HiSeq.10000.vcf.bgz"), "rb").read()
    tbi = open(os.path.join(golden, "HiSeq.10000.vcf.bgz.tbi"), "rb").read()
    b, want = assert_interval_parity(d, 128 * 1024, intervals, tbi)
    if nparts is not None:
        assert len(want) == nparts
    txt = gzip.decompress(d)
    exp = [l for l in T.split_lines(txt) if not l.startswith(b"#") and O.vcf_overlaps(l, intervals)]
    assert len(b["line_len"]) == len(exp)


def test_synthetic_vcf_intervals_with_info_end():
    text = T.make_vcf(6000, seed=4)
    data = T.bgzf_text(text, block_u=8000)
    tbi = T.whole_file_tabix(["chr1", "chr2", "chrX"], len(data))
    rng = np.random.default_rng(9)
    ivs = [(("chr1", "chr2", "chrX", "chr7")[int(rng.integers(0, 4))], int(a), int(a) + int(rng.integers(0, 3000)))
           for a in rng.integers(1, 400000, size=40)]
    for split in (0, 30000):
        b, want = assert_interval_parity(data, split, ivs, tbi)
        assert sum(len(p[0]) for _, p in want) > 0


def test_intervals_need_an_index(golden):
    d = open(os.path.join(golden, "HiSeq.10000.vcf.bgz"), "rb").read()
    with _lib.Context(split_size=128 * 1024) as c:
        c.text_open_bytes(d)
        c.text_set_intervals([("chr1", 1, 10)])
        with pytest.raises(_lib.DqError, match="no index"):
            c.text_run()


def test_variants_storage_mirror(golden, tmp_path):
    """HtsjdkVariantsRddStorage.read as T/HtsjdkVariantsRddTest.java:124-149 uses it."""
    import shutil
    from disq_amd.storage import HtsjdkVariantsRddStorage, Interval
    p = str(tmp_path / "HiSeq.10000.vcf.bgz")
    shutil.copy(os.path.join(golden, "HiSeq.10000.vcf.bgz"), p)
    st = HtsjdkVariantsRddStorage.makeDefault().splitSize(128 * 1024)
    v = st.read(p).getVariants()
    assert v.getNumPartitions() == 4 and v.count() == 9965
    shutil.copy(os.path.join(golden, "HiSeq.10000.vcf.bgz.tbi"), p + ".tbi")
    v = st.read(p, [Interval("chr1", 2700000, 2800000)]).getVariants()
    assert v.getNumPartitions() == 1 and v.count() == 243
