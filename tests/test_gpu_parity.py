"""GPU parity: libdisq_gpu.so (HIP, gfx950) against the oracle on the same inputs.

Bar: bit-exact.  Decompressed stream, per-partition record lists (count, order, voffset),
fixed fields and per-record raw-byte hashes must equal the oracle's.
"""
import os

import numpy as np
import pytest

from disq_amd import _lib, synth
from disq_amd.storage import (HtsjdkReadsRddStorage, HtsjdkReadsTraversalParameters, Interval)
from oracle import oracle as O

pytestmark = pytest.mark.gpu

FIELDS = ("voffset", "block_size", "ref_id", "pos", "l_seq", "next_ref_id", "next_pos", "tlen",
          "flag", "bin", "n_cigar", "mapq", "l_read_name", "hash")


def gpu_read(data, split=0, nio=False, traversal=None, bai=None, verify_crc=True):
    with _lib.Context(split_size=split, use_nio=nio, verify_crc=verify_crc) as c:
        c.open_bytes(data)
        if bai is not None:
            c.set_index(bai)
        return c.read(with_raw=True, traversal=traversal), c.plan(), c.inflated()


def assert_parity(data, split=0, nio=False, traversal=None, bai=None):
    ob = O.OracleBam(data)
    parts = ob.read_partitions(split, nio=nio, traversal=traversal, bai=bai)
    b, plan, u = gpu_read(data, split, nio, traversal, bai)
    assert np.array_equal(u, ob.inflate_all())
    # plan: same chunks as getPathChunks
    oplan = ob.plan(split, nio)
    assert [(s, e, ch) for s, e, ch in plan] == oplan
    po = b["part_offset"]
    assert len(po) - 1 == len(parts)
    for i, p in enumerate(parts):
        lo, hi = int(po[i]), int(po[i + 1])
        assert hi - lo == len(p), f"partition {i}"
        for f in FIELDS:
            assert np.array_equal(b[f][lo:hi], p[f]), (i, f)
        assert int(b["part_digest"][i]) == O.stream_digest(p["hash"])
    # raw bytes reproduce the hashes
    for k in np.linspace(0, len(b["voffset"]) - 1, num=min(50, len(b["voffset"])), dtype=int):
        o = int(b["raw_offset"][k])
        n = 4 + int(b["block_size"][k])
        assert O.record_hash(bytes(b["raw"][o:o + n])) == int(b["hash"][k])
    return b


@pytest.fixture(scope="module")
def bam1(golden):
    return open(os.path.join(golden, "1.bam"), "rb").read()


@pytest.mark.parametrize("split,nio", [(0, False), (128 * 1024, False), (128 * 1024, True),
                                       (40000, False), (14146, False), (19687, False),
                                       (65536, True), (1000, False)])
def test_1bam_partitions(bam1, split, nio):
    assert_parity(bam1, split, nio)


def test_1bam_golden_hashes(bam1, golden):
    ref = np.load(os.path.join(golden, "1.bam.records.npz"))
    b, _, _ = gpu_read(bam1, 0)
    assert np.array_equal(b["voffset"], ref["voffset"])
    assert np.array_equal(b["hash"], ref["hash"])


def test_hiseq_part_no_eof_block(golden):
    d = open(os.path.join(golden, "hiseq_part-r-00000.bam"), "rb").read()
    for split in (0, 40000, 10000):
        b = assert_parity(d, split)
    assert len(b["voffset"]) >= 837


@pytest.mark.parametrize("seed,n,split", [(1, 30000, 0), (2, 30000, 300000), (3, 8000, 65536),
                                          (4, 8000, 40000)])
def test_synth_wgs(seed, n, split):
    s = synth.generate(n, seed=seed, records_per_chunk=3000)
    assert_parity(s.bam, split)


def test_synth_level1_and_level9():
    for lvl in (1, 9, 0):
        s = synth.generate(3000, seed=11, level=lvl)
        assert_parity(s.bam, 65536)


def test_long_reads():
    s = synth.generate(80, seed=5, shape=synth.LONGREAD, records_per_chunk=40)
    for split in (0, 200000, 65536):
        assert_parity(s.bam, split)


def test_long_reads_2000_records():
    """configs[4] shape at >= 2,000 records (BamSource.java:110-153: the guesser walks up to
    MAX_READ_SIZE positions; BamRecordGuesser.java:34-52): ONT-like 10-100 kb reads and 1 % of
    0.5-2 Mb whose records span up to ~46 BGZF blocks; every partition field by field, the
    decompressed stream and the plan equal the oracle's, at split sizes down to 1 MiB (many splits
    start inside a record)."""
    s = synth.generate(2000, seed=41, shape=synth.LONGREAD, records_per_chunk=250, nthreads=8)
    assert s.n_records == 2000
    big = np.frombuffer(s.bam, np.uint8)
    assert len(big) > 40 << 20
    for split in (1 << 20, 8 << 20):
        b = assert_parity(s.bam, split)
        assert len(b["voffset"]) >= 2000
        assert int(b["block_size"].max()) > 4 * 65536  # records spanning many blocks


@pytest.fixture(scope="module")
def anysam():
    return synth.generate(1000, shape=synth.ANYSAM, bai=True)


@pytest.mark.parametrize("ivs,unplaced,expected", [
    ([("chr21", 5000, 9999), ("chr21", 20000, 22999)], False, 16),
    ([("chr21", 1, 1000135)], False, 2000),
    ([("chr21", 5000, 9999), ("chr21", 20000, 22999)], True, 18),
    (None, True, 2),
    ([], True, 2),
])
@pytest.mark.parametrize("split", [40000, 8000, 3000])
def test_interval_traversal(anysam, ivs, unplaced, expected, split):
    ob = O.OracleBam(anysam.bam)
    conv = None if ivs is None else [(ob.ref_index(c), s, e) for c, s, e in ivs]
    b = assert_parity(anysam.bam, split, traversal=(conv, unplaced), bai=anysam.bai)
    assert len(b["voffset"]) == expected


@pytest.mark.parametrize("ivs,expected", [
    ([("chr21", 5000, 9999), ("chr21", 20000, 22999)], 16),
    ([("chr21", 1, 1000135)], 2000),
    ([("chr21", 20000, 22999), ("chr21", 5000, 9999), ("chr21", 9000, 9500)], 16),
])
def test_resident_interval_filter(anysam, ivs, expected):
    """dq_run_resident with intervals, both ways: the .bai span run (default) and kernel 4 over
    the whole resident stream (full_traversal) keep exactly the records the per-partition
    createIndexIterator path returns (one partition, no unplaced)."""
    ob = O.OracleBam(anysam.bam)
    conv = [(ob.ref_index(c), s, e) for c, s, e in ivs]
    with _lib.Context(split_size=0, verify_crc=True, full_traversal=True) as c:
        c.open_bytes(anysam.bam)
        c.set_index(anysam.bai)
        st = c.run_resident((conv, False))
        assert st.n_filtered == expected
        assert st.ms_filter > 0
        assert c.run_resident().n_filtered == -1
        assert c.run_resident((conv, False)).n_filtered == expected
        assert len(c.read(traversal=(conv, False))["voffset"]) == expected
        assert c.run_resident((conv, False)).n_filtered == expected
    with _lib.Context(split_size=0, verify_crc=True) as c:
        c.open_bytes(anysam.bam)
        c.set_index(anysam.bai)
        st = c.run_resident((conv, False))
        assert st.n_filtered == expected
        assert 0 < st.blocks_inflated <= st.n_blocks
        assert len(c.read(traversal=(conv, False))["voffset"]) == expected
        assert c.run_resident((conv, False)).n_filtered == expected


def test_resident_interval_filter_needs_index(anysam):
    with _lib.Context(split_size=0) as c:
        c.open_bytes(anysam.bam)
        with pytest.raises(_lib.DqError, match="index"):
            c.run_resident(([(0, 1, 100)], False))


def test_storage_api_mirror(tmp_path, anysam, golden):
    p = str(tmp_path / "anysam.bam")
    anysam.write(p)
    st = HtsjdkReadsRddStorage.makeDefault().splitSize(8000).useNio(False)
    rdd = st.read(p, HtsjdkReadsTraversalParameters(
        [Interval("chr21", 5000, 9999), Interval("chr21", 20000, 22999)], True))
    assert rdd.getReads().count() == 18
    rdd = st.read(os.path.join(golden, "1.bam"))
    assert rdd.getReads().count() == 4917
    assert rdd.getHeader().getSequenceDictionary()[0][0]
    # a directory of parts reads every non-hidden file
    d = tmp_path / "parts"
    d.mkdir()
    hi = open(os.path.join(golden, "hiseq_part-r-00000.bam"), "rb").read()
    (d / "part-r-00000.bam").write_bytes(hi)
    (d / "part-r-00001.bam").write_bytes(hi)
    (d / "_SUCCESS").write_bytes(b"")
    assert st.read(str(d)).getReads().count() >= 2 * 837


def test_crc_mismatch_detected(bam1):
    bad = bytearray(bam1)
    # flip one bit of block 0's stored CRC32 (bytes cSize-8 .. cSize-4 of the block)
    bad[14146 - 8] ^= 1
    with _lib.Context(verify_crc=True) as c:
        c.open_bytes(bytes(bad))
        with pytest.raises(_lib.DqError, match="CRC"):
            c.run_resident()
    with _lib.Context(verify_crc=False) as c:  # htsjdk's default does not check CRCs
        c.open_bytes(bytes(bad))
        c.run_resident()


def test_corrupt_deflate_detected(bam1):
    bad = bytearray(bam1)
    for i in range(200, 260):
        bad[i] ^= 0x5a
    with _lib.Context() as c:
        c.open_bytes(bytes(bad))
        with pytest.raises(_lib.DqError):
            c.run_resident()


def test_truncated_file(bam1):
    with _lib.Context() as c:
        c.open_bytes(bam1[:300000])
        with pytest.raises(_lib.DqError):
            c.run_resident()


def test_resident_rerun_is_idempotent():
    s = synth.generate(20000, seed=21)
    with _lib.Context(split_size=1 << 20) as c:
        c.open_bytes(s.bam)
        a = c.run_resident()
        b = c.run_resident()
        assert a.digest == b.digest and a.n_records == b.n_records == 20000
        assert a.decompressed_bytes == b.decompressed_bytes


def test_large_properties():
    """Size-independent properties at a larger size (oracle used only on a sample)."""
    s = synth.generate(400000, seed=9)
    with _lib.Context(split_size=8 << 20) as c:
        c.open_bytes(s.bam)
        st = c.run_resident()
        assert st.n_records == 400000
        assert st.n_partitions == len(O.path_splits(len(s.bam), 8 << 20))
        b = c.read(with_raw=False)
    v = b["voffset"]
    assert len(v) == 400000
    assert np.all(np.diff(v.astype(np.int64)) > 0)
    # record lengths tile the decompressed stream after the header
    assert int((4 + b["block_size"].astype(np.int64)).sum()) == s.record_bytes
    ob = O.OracleBam(s.bam)
    recs = ob.read_all()
    assert np.array_equal(recs["hash"], b["hash"])


@pytest.mark.parametrize("split", [14146, 40000, 128 * 1024])
def test_compat_dedupe_partitions_tile_the_file(golden, split):
    """dq_opts.compat = DEDUPE: chunk ends at splitEnd << 16, so a block starting at a split end
    (1.bam @ 14146: Disq reads its records twice, 5123 for 4917) belongs to the next partition
    only; the partitions concatenate to the file's record list.  DISQ_EXACT keeps the oracle's
    (Disq's) partitions."""
    data = open(os.path.join(golden, "1.bam"), "rb").read()
    ob = O.OracleBam(data)
    allrec = ob.read_all()
    exact = ob.read_partitions(split)
    plan = [(s, e) for s, e, ch in ob.plan(split) if ch is not None]
    want = [p[p["voffset"] < (np.uint64(e) << np.uint64(16))] for p, (s, e) in zip(exact, plan)]
    assert np.array_equal(np.concatenate(want)["voffset"], allrec["voffset"])
    with _lib.Context(split_size=split, compat=_lib.COMPAT_DEDUPE) as c:
        c.open_bytes(data)
        b = c.read(with_raw=False)
        chunks = c.plan()
    po = b["part_offset"]
    assert len(po) - 1 == len(want)
    for i, w in enumerate(want):
        assert np.array_equal(b["voffset"][int(po[i]):int(po[i + 1])], w["voffset"])
    assert np.array_equal(b["voffset"], allrec["voffset"])
    assert all(ch is None or ch[1] == (e << 16) for s, e, ch in chunks)
    with _lib.Context(split_size=split) as c:
        c.open_bytes(data)
        n_exact = len(c.read(with_raw=False)["voffset"])
    assert n_exact == sum(len(p) for p in exact) == (5123 if split == 14146 else 4917)
