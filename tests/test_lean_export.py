"""The lean export mode (DQ_EXPORT_LEAN, include/disq_gpu.h): a batch of voffsets and raw record
bytes only.  Every other SoA field is in each record's first 36 raw bytes, which is where htsjdk's
BAMRecordCodec.decode reads them (H/BAMFileReader2.java:929-931; SAMRecordFactory.createBAMRecord
takes the rest as restOfData), so a consumer that parses them there loses nothing: the fields parsed
from a lean batch equal a full batch's SoA and the oracle's records, and the batch's partition
digests are the full batch's."""
import os

import numpy as np
import pytest

from disq_amd import _lib, synth
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
FIELDS = ("block_size", "ref_id", "pos", "l_seq", "next_ref_id", "next_pos", "tlen", "flag",
          "bin", "n_cigar", "mapq", "l_read_name")


def test_lean_head_layout():
    """The 36-byte head the lean parser reads is SAMv1's fixed record layout."""
    assert _lib.LEAN_HEAD.itemsize == 36
    rec = (100).to_bytes(4, "little", signed=True) + (3).to_bytes(4, "little") + \
        (12345).to_bytes(4, "little") + bytes([9, 60]) + (4681).to_bytes(2, "little") + \
        (2).to_bytes(2, "little") + (99).to_bytes(2, "little") + (150).to_bytes(4, "little") + \
        (3).to_bytes(4, "little") + (12500).to_bytes(4, "little") + (-300).to_bytes(4, "little",
                                                                                   signed=True)
    raw = np.frombuffer(rec + bytes(100 - 32), np.uint8)
    off, f = _lib.parse_lean(raw, 1)
    assert off.tolist() == [0]
    assert (f["block_size"][0], f["ref_id"][0], f["pos"][0], f["l_read_name"][0], f["mapq"][0],
            f["bin"][0], f["n_cigar"][0], f["flag"][0], f["l_seq"][0], f["next_ref_id"][0],
            f["next_pos"][0], f["tlen"][0]) == (100, 3, 12345, 9, 60, 4681, 2, 99, 150, 3, 12500,
                                                -300)
    with pytest.raises(ValueError):
        _lib.parse_lean(raw[:-1], 1)


def test_export_mode_values():
    assert _lib.export_mode(True) == _lib.EXPORT_RAW
    assert _lib.export_mode(False) == _lib.EXPORT_FIELDS
    assert _lib.export_mode("lean") == _lib.EXPORT_LEAN
    with pytest.raises(ValueError):
        _lib.export_mode("thin")


def _check_lean(lean, full):
    n = len(full["voffset"])
    assert len(lean["voffset"]) == n
    assert np.array_equal(lean["voffset"], full["voffset"])
    assert np.array_equal(lean["raw"], full["raw"])
    for k in ("hash", "raw_offset", "block_size"):  # not exported
        assert len(lean[k]) == 0, k
    assert np.array_equal(lean["part_offset"], full["part_offset"])
    assert np.array_equal(lean["part_digest"], full["part_digest"])
    off, f = _lib.parse_lean(lean["raw"], n)
    assert np.array_equal(off, full["raw_offset"])
    for k in FIELDS:
        assert np.array_equal(f[k], full[k]), k
    return f


@pytest.mark.gpu
@pytest.mark.parametrize("name,split", [("1.bam", 14146), ("1.bam", 128 << 10), ("wgs", 1 << 20)])
def test_lean_batch_equals_full_batch_and_oracle(name, split):
    data = (open(os.path.join(GOLD, name), "rb").read() if name != "wgs"
            else synth.generate(30000, seed=5, nthreads=8).bam)
    ref = np.concatenate(O.OracleBam(data).read_partitions(split))
    with _lib.Context(split_size=split, verify_crc=True) as c:
        c.open_bytes(data)
        full = c.read(with_raw=True)
        lean = c.read(with_raw="lean")
        f = _check_lean(lean, full)
        assert np.array_equal(lean["voffset"], ref["voffset"])
        for k in FIELDS:
            assert np.array_equal(f[k], ref[k]), k
        # one chunk (dq_decode), in the pinned export arena as the streaming reader uses it
        c.set_export_arena(64 << 20)
        vs, ve = int(full["voffset"][0]), (len(data) << 16) | 0xffff
        lf = c.decode(vs, ve, with_raw="lean")
        assert lf["raw"] is not None and not lf["raw"].flags.writeable
        n = len(lf["voffset"])
        off, f2 = _lib.parse_lean(lf["raw"], n)
        got = {k: f2[k].copy() for k in FIELDS}
        del lf, f2
        ff = c.decode(vs, ve, with_raw=True)
        for k in FIELDS:
            assert np.array_equal(got[k], ff[k]), k
        del ff


@pytest.mark.gpu
def test_lean_filtered_chunk_from_file(tmp_path):
    """dq_decode_chunk_filtered (a task's interval traversal, several span windows concatenated)
    in lean mode: voffsets, raw bytes and the chunk's digest equal the full batch's."""
    w = synth.generate(30000, seed=41, bai=True, nthreads=8, unplaced_fraction=0.01)
    path = str(tmp_path / "w.bam")
    w.write(path)
    ob = O.OracleBam(w.bam)
    rng = np.random.default_rng(3)
    ivs = [(0, int(a), int(a + rng.integers(10, 2000))) for a in rng.integers(1, 140000, size=60)]
    checked = 0
    with _lib.Context(split_size=1 << 20, verify_crc=True) as c:
        c.set_index(w.bai)
        for s, e, ch in ob.plan(1 << 20):
            if ch is None:
                continue
            full = c.decode_chunk(path, *ch, traversal=(ivs, True))
            lean = c.decode_chunk(path, *ch, traversal=(ivs, True), with_raw="lean")
            _check_lean(lean, full)
            checked += len(full["voffset"])
    assert checked > 0


@pytest.mark.gpu
def test_unknown_export_mode_is_einval():
    with _lib.Context(split_size=0) as c:
        c.open_bytes(open(os.path.join(GOLD, "1.bam"), "rb").read())
        with pytest.raises(_lib.DqError) as e:
            c.read(with_raw=3)
        assert e.value.code == _lib.DQ_EINVAL
