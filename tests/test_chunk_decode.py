"""Task-side decode of one Chunk straight from a file (dq_decode_chunk), as a Spark task runs
BamSource.getIterator (D/impl/formats/bam/BamSource.java:172-175): only the chunk's compressed
bytes (plus the straddling record's blocks) are read and copied to the device.

Bar: every chunk of the plan decodes to exactly the oracle's records for that chunk (count, order,
every SoA field, hash, raw bytes), and the bytes copied host -> device stay close to the chunk's
compressed span instead of the whole file.
"""
import os
import threading

import numpy as np
import pytest

from disq_amd import _lib, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

FIELDS = ("voffset", "block_size", "ref_id", "pos", "l_seq", "next_ref_id", "next_pos", "tlen",
          "flag", "bin", "n_cigar", "mapq", "l_read_name", "hash")
WINDOW = 256 << 10  # dq_decode_chunk's first look-ahead past the chunk's last block


def check_chunks(path, split, max_extra=WINDOW + 65536):
    data = open(path, "rb").read()
    ob = O.OracleBam(data)
    plan = ob.plan(split)
    n = 0
    with _lib.Context(split_size=split, verify_crc=True) as c:
        for s, e, ch in plan:
            if ch is None:
                continue
            vs, ve = ch
            b = c.decode_chunk(path, vs, ve)
            ref = ob.read_chunk(vs, ve)
            assert len(b["voffset"]) == len(ref), (s, e)
            for f in FIELDS:
                assert np.array_equal(b[f], ref[f]), (s, f)
            raw = b["raw"] if b["raw"] is not None else np.zeros(0, np.uint8)
            assert len(raw) == int((4 + ref["block_size"].astype(np.int64)).sum())
            for k in range(0, len(ref), max(1, len(ref) // 7)):
                o = int(b["raw_offset"][k])
                assert O.record_hash(bytes(raw[o:o + 4 + int(ref["block_size"][k])])) == \
                    int(ref["hash"][k])
            h2d = c.stats().h2d_bytes
            span = (ve >> 16) - (vs >> 16)
            assert span <= h2d <= span + max_extra, (s, h2d, span)
            n += len(ref)
    return n


@pytest.mark.parametrize("split", [0, 128 * 1024, 40000, 14146])
def test_1bam_every_chunk(golden, split):
    n = check_chunks(os.path.join(golden, "1.bam"), split)
    assert n == (5123 if split == 14146 else 4917)


def test_hiseq_part_no_eof_block(golden):
    check_chunks(os.path.join(golden, "hiseq_part-r-00000.bam"), 40000)


def test_synthetic_chunks(tmp_path):
    p = str(tmp_path / "s.bam")
    synth.generate(120000, seed=13, nthreads=8).write(p)
    n = check_chunks(p, 1 << 20)
    assert n == 120000
    # a task reads about one split, not the file
    assert os.path.getsize(p) > 8 * (1 << 20)


def test_long_read_chunk_grows_the_window(tmp_path):
    """A record much longer than the first look-ahead forces the window to grow."""
    p = str(tmp_path / "l.bam")
    synth.generate(300, seed=5, shape=synth.LONGREAD, records_per_chunk=40, nthreads=8).write(p)
    check_chunks(p, 256 * 1024, max_extra=64 << 20)


def test_chunk_start_not_a_record(golden):
    path = os.path.join(golden, "1.bam")
    with _lib.Context() as c:
        with pytest.raises(_lib.DqError, match="record"):
            c.decode_chunk(path, (0 << 16) | 45847, (597482 << 16) | 0xffff)


def test_context_used_from_another_thread(golden):
    """A dq_ctx created on one thread decodes on another (one context per Spark task thread)."""
    path = os.path.join(golden, "1.bam")
    ob = O.OracleBam(open(path, "rb").read())
    (_, _, ch), = ob.plan(0)
    c = _lib.Context(verify_crc=True)
    out = {}

    def run():
        out["b"] = c.decode_chunk(path, *ch)

    t = threading.Thread(target=run)
    t.start()
    t.join(120)
    c.close()
    assert np.array_equal(out["b"]["hash"], ob.read_chunk(*ch)["hash"])


def check_filtered(path, bai, split, ivs, unplaced):
    data = open(path, "rb").read()
    ob = O.OracleBam(data)
    parts = iter(ob.read_partitions(split, traversal=(ivs, unplaced), bai=bai))
    n = 0
    with _lib.Context(split_size=split, verify_crc=True) as c:
        c.set_index(bai)
        for s, e, ch in ob.plan(split):
            if ch is None:
                continue
            b = c.decode_chunk(path, *ch, traversal=(ivs, unplaced))
            ref = next(parts)
            assert len(b["voffset"]) == len(ref), (s, e)
            for f in FIELDS:
                assert np.array_equal(b[f], ref[f]), (s, f)
            n += len(ref)
    return n


@pytest.mark.parametrize("split", [40000, 8000, 3000])
@pytest.mark.parametrize("ivs,unplaced,expected", [
    ([(20, 5000, 9999), (20, 20000, 22999)], False, 16),
    ([(20, 5000, 9999), (20, 20000, 22999)], True, 18),
    ([(20, 1, 1000135)], False, 2000),
    (None, True, 2),
    ([], True, 2),
])
def test_anysam_filtered_chunks(tmp_path, split, ivs, unplaced, expected):
    a = synth.generate(1000, shape=synth.ANYSAM, bai=True)
    p = str(tmp_path / "a.bam")
    a.write(p)
    assert check_filtered(p, a.bai, split, ivs, unplaced) == expected


def test_wgs_filtered_chunks(tmp_path):
    """Many intervals on a WGS-like file: each task reads only its chunk's .bai span."""
    w = synth.generate(60000, seed=41, bai=True, nthreads=8, unplaced_fraction=0.01)
    p = str(tmp_path / "w.bam")
    w.write(p)
    rng = np.random.default_rng(4)
    ivs = [(0, int(s), int(s + rng.integers(10, 600))) for s in rng.integers(1, 290000, size=200)]
    for unplaced in (False, True):
        assert check_filtered(p, w.bai, 1 << 20, ivs, unplaced) > 0
    with _lib.Context(split_size=1 << 20) as c:
        c.set_index(w.bai)
        c.decode_chunk(p, *O.OracleBam(w.bam).plan(1 << 20)[0][2], traversal=(ivs[:3], False))
        assert c.stats().h2d_bytes < len(w.bam) // 2
