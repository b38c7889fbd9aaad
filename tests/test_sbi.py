"""Splitting index (.sbi), SURVEY.md section 8(f) row 1.

* Writing: BAMSBIIndexer.createIndex + SBIIndexWriter (M/htsjdk/samtools/BAMSBIIndexer.java:45-66,
  SBIIndexWriter.java:84-151) -> dq_write_sbi.  Pinned by the reference's own fixture
  1-with-splitting-index.bam.sbi (htsjdk output, granularity 1, zero MD5/UUID): the GPU's index of
  1.bam must equal it byte for byte.
* Planning: SBIIndex.getChunk (SBIIndex.java:244-277) per split -> dq_set_splitting_index(..., 1).
  Disq's own getPathChunks loads the .sbi and discards it (BamSource.java:69-87), so by default it
  is only validated and the guessed plan is unchanged.
"""
import os

import numpy as np
import pytest

from disq_amd import _lib, synth
from oracle import oracle as O

FIELDS = ("voffset", "block_size", "ref_id", "pos", "l_seq", "next_ref_id", "next_pos", "tlen",
          "flag", "bin", "n_cigar", "mapq", "l_read_name", "hash")


@pytest.fixture(scope="module")
def bam1(golden):
    return open(os.path.join(golden, "1.bam"), "rb").read()


@pytest.fixture(scope="module")
def sbi1(golden):
    return open(os.path.join(golden, "1-with-splitting-index.bam.sbi"), "rb").read()


# ---------------------------------------------------------------------------- oracle (CPU)
def test_oracle_sbi_writer_reproduces_htsjdk_fixture(bam1, sbi1):
    assert O.OracleBam(bam1).write_sbi(1) == sbi1


def test_oracle_get_chunk_tiles_the_records(bam1, sbi1):
    offs = O.sbi_offsets(sbi1)
    for split in (40000, 128 * 1024, 14146, 1000, 0):
        chunks = [ch for _, _, ch in O.OracleBam(bam1).plan_sbi(sbi1, split)]
        got = [c for c in chunks if c is not None]
        # contiguous, non-overlapping, from the first record to the final pointer
        assert got[0][0] == int(offs[0]) and got[-1][1] == int(offs[-1])
        for a, b in zip(got, got[1:]):
            assert a[1] == b[0]
    with pytest.raises(ValueError):
        O.sbi_get_chunk(offs, 10, 10)


def test_oracle_sbi_partitions_cover_every_record_once(bam1, sbi1):
    ob = O.OracleBam(bam1)
    allr = ob.read_all()
    for split in (40000, 14146):
        parts = ob.read_partitions_sbi(sbi1, split)
        cat = np.concatenate([p["voffset"] for p in parts])
        assert np.array_equal(cat, allr["voffset"])   # no Disq duplicate-block quirk with .sbi


def test_oracle_sbi_granularity(bam1, sbi1):
    ob = O.OracleBam(bam1)
    offs = O.sbi_offsets(sbi1)
    for g in (2, 7, 4096):
        d = ob.write_sbi(g)
        o = O.sbi_offsets(d)
        assert np.array_equal(o[:-1], offs[:-1][::g]) and o[-1] == offs[-1]
        assert int.from_bytes(d[44:52], "little") == 4917
        assert int.from_bytes(d[52:60], "little") == g


# ---------------------------------------------------------------------------- GPU
def _ctx(data, split=0, **kw):
    c = _lib.Context(split_size=split, verify_crc=True, **kw)
    c.open_bytes(data)
    return c


@pytest.mark.gpu
def test_gpu_sbi_equals_htsjdk_fixture(bam1, sbi1):
    with _ctx(bam1) as c:
        assert c.write_sbi(1) == sbi1
        for g in (2, 7, 4096):
            assert c.write_sbi(g) == O.OracleBam(bam1).write_sbi(g)
        # the context still reads normally afterwards
        assert len(c.read(with_raw=False)["voffset"]) == 4917


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["wgs", "longread", "hiseq"])
def test_gpu_sbi_matches_oracle_and_generator(kind, golden):
    if kind == "wgs":
        s = synth.generate(20000, seed=3, sbi_granularity=1, records_per_chunk=3000)
        data, gen = s.bam, s.sbi
    elif kind == "longread":
        s = synth.generate(60, seed=5, shape=synth.LONGREAD, sbi_granularity=1)
        data, gen = s.bam, s.sbi
    else:  # no EOF block: the final pointer is the file length
        data = open(os.path.join(golden, "hiseq_part-r-00000.bam"), "rb").read()
        gen = None
    with _ctx(data) as c:
        got = c.write_sbi(1)
        got64 = c.write_sbi(64)
    ob = O.OracleBam(data)
    assert got == ob.write_sbi(1)
    assert got64 == ob.write_sbi(64)
    if gen is not None:   # the generator's own index (offsets recorded while writing)
        assert np.array_equal(O.sbi_offsets(got), O.sbi_offsets(gen))


@pytest.mark.gpu
@pytest.mark.parametrize("split", [40000, 128 * 1024, 14146, 1000])
def test_gpu_sbi_planning(bam1, sbi1, split):
    ob = O.OracleBam(bam1)
    oplan = ob.plan_sbi(sbi1, split)
    parts = ob.read_partitions_sbi(sbi1, split)
    with _ctx(bam1, split) as c:
        c.set_splitting_index(sbi1, use_for_planning=True)
        plan = c.plan()
        b = c.read(with_raw=True)
    assert plan == oplan
    po = b["part_offset"]
    assert len(po) - 1 == len(parts)
    for i, p in enumerate(parts):
        lo, hi = int(po[i]), int(po[i + 1])
        for f in FIELDS:
            assert np.array_equal(b[f][lo:hi], p[f]), (i, f)
        assert int(b["part_digest"][i]) == O.stream_digest(p["hash"])


@pytest.mark.gpu
def test_gpu_sbi_coarse_granularity_planning():
    s = synth.generate(20000, seed=9, sbi_granularity=1, records_per_chunk=3000)
    with _ctx(s.bam) as c:
        sbi = c.write_sbi(100)
    ob = O.OracleBam(s.bam)
    for split in (65536, 300000):
        parts = ob.read_partitions_sbi(sbi, split)
        with _ctx(s.bam, split) as c:
            c.set_splitting_index(sbi, use_for_planning=True)
            assert c.plan() == ob.plan_sbi(sbi, split)
            b = c.read(with_raw=False)
        assert np.array_equal(b["hash"], np.concatenate([p["hash"] for p in parts]))


@pytest.mark.gpu
def test_gpu_sbi_ignored_by_default_and_validated(bam1, sbi1):
    """Disq-exact: a valid .sbi does not change the guessed plan; an invalid one fails as
    SBIIndex.load does."""
    with _ctx(bam1, 40000) as c:
        want = c.plan()
        c.set_splitting_index(sbi1, use_for_planning=False)
        assert c.plan() == want
        with pytest.raises(_lib.DqError, match="Invalid file header in SBI"):
            c.set_splitting_index(b"XXXX" + sbi1[4:])
        bad = bytearray(sbi1)
        bad[68:76], bad[76:84] = sbi1[76:84], sbi1[68:76]   # first two offsets swapped
        with pytest.raises(_lib.DqError, match="not in order"):
            c.set_splitting_index(bytes(bad))


@pytest.mark.gpu
def test_gpu_sbi_storage_mirror(tmp_path, bam1, sbi1):
    from disq_amd.storage import BAMSBIIndexer, HtsjdkReadsRddStorage
    p = tmp_path / "1.bam"
    p.write_bytes(bam1)
    out = BAMSBIIndexer.createIndex(str(p), 1)
    assert open(out, "rb").read() == sbi1
    st = HtsjdkReadsRddStorage.makeDefault().splitSize(40000)
    guessed = st.read(str(p)).getReads()
    indexed = st.useSplittingIndex(True).read(str(p)).getReads()
    assert indexed.count() == 4917
    # guessing emits the split-boundary duplicate block of BamSource.java:140; the index does not
    assert guessed.count() >= indexed.count()
