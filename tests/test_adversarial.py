"""Adversarial fixtures for split planning.

1. A BGZF member header inside record payload at a split start.  Stored (level-0) blocks keep the
   payload bytes verbatim in the file, so BgzfBlockGuesser.guessNextBGZFPos
   (D/impl/formats/bgzf/BgzfBlockGuesser.java:76-149) sees them:
   - "eof": a complete empty member (the 28-byte EOF block) -- the guesser accepts it, the split's
     block iterator (BgzfBlockSource.java:63-84) yields it with uSize 0, then continues from
     its end (fake position + 28) to the next real block;
   - "broken": the magic with a bad 'BC' subfield -- the guesser rejects it and scans on from
     the magic + 4 (:138-144).
   In both cases getFirstReadInPartition (BamSource.java:110-153) ends on the same record start
   as without the fake bytes.
   - "data": a member with data (ISIZE > 0) -- the reference would inflate the fake member and
     run the record guesser over its bytes; the GPU planner does not reproduce that and must
     fail loudly instead of planning a different chunk.
2. A record longer than MAX_READ_SIZE (10,000,000 positions, BamSource.java:44,132-135): a split
   that starts inside it scans 10 M positions without a record start and gets no chunk (an empty
   partition), while later splits inside the record find the next record.
"""
import numpy as np
import pytest

from disq_amd import synth
from oracle import oracle as O

import bamutil as B

BROKEN = bytes.fromhex("1f8b08040000000000ff0600424402001b00")  # 'BD' instead of 'BC'


def fake_header_bam(kind, clean=False):
    """Level-0 BAM with `payload` in the qualities of record 400 (clean=True: zero bytes)."""
    r = synth.generate(800, seed=21, level=0, nthreads=4)
    u = bytearray(B.inflate_all(r.bam))
    off, ln = B.record_spans(u)[400]
    q = off + B.qual_offset(bytes(u[off:off + ln]))
    if kind == "eof":
        payload = B.EOF_BLOCK
    elif kind == "broken":
        payload = BROKEN
    else:
        payload = B.bgzf_member(b"hello, world", 6)
    u[q + 10:q + 10 + len(payload)] = bytes(len(payload)) if clean else payload
    bam = B.bgzf(bytes(u), level=0)
    if clean:
        return bam
    fake = bam.find(payload)
    assert 0 < fake < len(bam) - 28
    return bam, fake, payload


@pytest.mark.parametrize("kind", ["eof", "broken"])
def test_oracle_fake_header_at_split_start(kind):
    bam, fake, payload = fake_header_bam(kind)
    split = fake - 7  # split 1 starts 7 bytes before the fake member
    ob = O.OracleBam(bam)
    g = ob.guess_next_bgzf(split, 2 * split)
    if kind == "eof":
        assert g == (fake, 28, 0)  # the guesser takes the embedded member
    else:
        assert g[0] > fake  # rejected: the next real block
    parts = ob.read_partitions(split)
    allr = ob.read_all()
    got = np.concatenate([p["voffset"] for p in parts])
    assert np.array_equal(got, allr["voffset"])
    # the same chunks as the file without the fake bytes; split 1 starts in the first real block
    # after the fake member
    plan = ob.plan(split)
    assert plan == O.OracleBam(fake_header_bam(kind, clean=True)).plan(split)
    nxt = ob.guess_next_bgzf(fake + 4, 1 << 40)[0]
    assert plan[1][2][0] >> 16 == nxt


def stored_member(data: bytes) -> bytes:
    """A BGZF member holding `data` in ONE stored deflate block (payload bytes verbatim)."""
    import struct
    import zlib
    assert len(data) <= 65535
    body = bytes([1]) + struct.pack("<HH", len(data), len(data) ^ 0xffff) + data
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
    member = hdr + struct.pack("<H", 18 + len(body) + 8 - 1) + body
    return member + struct.pack("<II", zlib.crc32(data) & 0xffffffff, len(data))


N_FAKES = 65268 // 28  # 2331 empty members: a whole stored block's payload


def many_fakes_bam():
    """A real (stored) BGZF block whose payload is nothing but empty BGZF members (the 28-byte EOF
    block, 2331 times, in the qualities of a 70 kb record).  A split starting just before them makes
    BgzfBlockSource (BgzfBlockSource.java:63-84) hop over every one of them (uSize 0) before the
    next real block: the longest chain of guesses a BGZF file allows (real blocks are <= 64 KiB)."""
    import struct
    r = synth.generate(800, seed=23, level=0, nthreads=4)
    u = B.inflate_all(r.bam)
    off, _ = B.record_spans(u)[400]
    ref_id, pos = struct.unpack_from("<ii", u, off + 4)
    rec = B.make_record(ref_id, pos, b"fakes", 70000)
    u2 = bytearray(u[:off] + rec + u[off:])
    f0 = off + B.qual_offset(rec) + 100
    f1 = f0 + 28 * N_FAKES
    u2[f0:f1] = B.EOF_BLOCK * N_FAKES
    bounds = sorted(set(list(range(0, f0, B.BLOCK_U)) + [f0, f1] +
                        list(range(f1, len(u2), B.BLOCK_U))))
    bounds.append(len(u2))
    bam = b"".join(stored_member(bytes(u2[a:b])) for a, b in zip(bounds, bounds[1:])) + B.EOF_BLOCK
    first = bam.find(B.EOF_BLOCK * 4)
    assert first > 0 and bam[first + 28 * N_FAKES:first + 28 * N_FAKES + 4] != B.EOF_BLOCK[:4]
    return bam, first


def test_oracle_longest_guess_chain():
    bam, first = many_fakes_bam()
    ob = O.OracleBam(bam)
    assert ob.guess_next_bgzf(first - 7, 1 << 40) == (first, 28, 0)
    # the split's block list: every fake member (uSize 0), then the real blocks
    blocks = ob.split_blocks(first - 7, first - 7 + 200000)
    assert [b[2] for b in blocks[:N_FAKES]] == [0] * N_FAKES
    assert blocks[N_FAKES][2] > 0 and blocks[N_FAKES][0] == first + 28 * N_FAKES + 8
    parts = ob.read_partitions(first - 7)
    assert sum(len(p) for p in parts) >= 800


def giant_bam():
    r = synth.generate(300, seed=22, nthreads=4)
    u = B.inflate_all(r.bam)
    off, _ = B.record_spans(u)[250]
    giant = B.make_record(0, 1_000_000, b"giant", 7_000_000)
    assert len(giant) > 10_000_000
    u2 = u[:off] + giant + u[off:]
    return B.bgzf(u2, level=5), off, len(giant)


def dense_bam(n_tiny=6000):
    """6000 minimal records (44 bytes: a one-base read named "a") in a row inside a synthetic WGS
    BAM: a 64 KiB record-chain segment holds ~1490 starts there, more than the 512 the chain walk
    records (SEG_OFF_CAP), so those segments are walked a second time while their neighbours are
    copied from the recorded starts."""
    import struct
    r = synth.generate(900, seed=31, nthreads=4)
    u = B.inflate_all(r.bam)
    off, _ = B.record_spans(u)[450]
    ref_id, pos = struct.unpack_from("<ii", u, off + 4)
    tiny = B.make_record(ref_id, pos, b"a", 1)
    assert len(tiny) == 44
    return B.bgzf(u[:off] + tiny * n_tiny + u[off:], level=5), n_tiny


def test_oracle_dense_records():
    bam, n_tiny = dense_bam()
    allr = O.OracleBam(bam).read_all()
    assert len(allr) == 900 + n_tiny  # (synth's unplaced tail is part of the 900)
    assert (allr["block_size"] == 40).sum() == n_tiny


def test_oracle_max_read_size_empty_partition():
    """Split 1 starts two blocks into the giant record and its blocks reach past the record's
    end: the first 10 M positions hold no record start, so the split gets no chunk, and the
    records that start later in it are in no partition (BamSource.java:132-135 -- a reference
    quirk the GPU path reproduces)."""
    bam, off, glen = giant_bam()
    ob = O.OracleBam(bam)
    blocks = ob.split_blocks(0, len(bam))
    uo = np.cumsum([0] + [b[2] for b in blocks])
    j = int(np.searchsorted(uo, off, side="right")) - 1  # block holding the giant's first byte
    split = blocks[j + 2][0]
    assert off < uo[j + 2] < off + glen - 10_000_000
    r2 = int(np.searchsorted(uo, off + glen, side="right")) - 1  # block of the next record
    assert blocks[r2][0] < 2 * split  # ... which split 1 reaches
    plan = ob.plan(split)
    assert plan[1][2] is None
    allr = ob.read_all()
    assert (allr["block_size"] + 4 == glen).sum() == 1
    parts = ob.read_partitions(split)
    n_lost = len(allr) - sum(len(p) for p in parts)
    # the records after split 0's chunk end and before split 2's first record are in no partition
    v = allr["voffset"]
    lo = (split << 16) | 0xffff
    hi = plan[2][2][0] if len(plan) > 2 else 1 << 63
    assert n_lost == int(((v > lo) & (v < hi)).sum()) > 0


# ---- the GPU path on the same fixtures (bit-exact against the oracle)

@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["eof", "broken"])
def test_gpu_fake_header_at_split_start(kind):
    from test_gpu_parity import assert_parity
    bam, fake, _ = fake_header_bam(kind)
    for split in (fake - 7, fake, fake - 40000):
        assert_parity(bam, split)


@pytest.mark.gpu
def test_gpu_longest_guess_chain():
    """2331 guesser hops at one split start (round 3 stopped planning silently after 4096 hops;
    the hop bound is now the file's structure, as in the reference)."""
    from test_gpu_parity import assert_parity
    bam, first = many_fakes_bam()
    for split in (first - 7, first + 28 * 1000 - 3):
        assert_parity(bam, split)


@pytest.mark.gpu
def test_gpu_fake_member_with_data_fails_like_the_reference():
    """The reference fails on the bytes after a data-carrying fake member (htsjdk 'Invalid GZIP
    header' escapes getFirstReadInPartition); the GPU planner refuses the split loudly."""
    from disq_amd import _lib
    bam, fake, _ = fake_header_bam("data")
    with pytest.raises(O.OracleError):
        O.OracleBam(bam).plan(fake - 7)
    with _lib.Context(split_size=fake - 7) as c:
        with pytest.raises(_lib.DqError, match="BGZF"):
            c.open_bytes(bam)
            c.plan()


@pytest.mark.gpu
def test_gpu_max_read_size_empty_partition():
    from test_gpu_parity import assert_parity
    bam, off, glen = giant_bam()
    ob = O.OracleBam(bam)
    blocks = ob.split_blocks(0, len(bam))
    uo = np.cumsum([0] + [b[2] for b in blocks])
    j = int(np.searchsorted(uo, off, side="right")) - 1
    split = blocks[j + 2][0]
    b = assert_parity(bam, split)
    # getPathChunks drops the null chunk: split 1 contributes no partition
    assert len(b["part_offset"]) - 1 == 1


@pytest.mark.gpu
def test_gpu_dense_records_recorded_and_rewalked_segments():
    from test_gpu_parity import assert_parity
    bam, n_tiny = dense_bam()
    for split in (0, 70000, 150001):
        b = assert_parity(bam, split)
    assert (b["block_size"] == 40).sum() == n_tiny


def midsize_bam(n_mid=1500):
    """1500 records of 0.5-6 KB (reads of 300-4000 bases, names of 2-60 characters) in a row inside
    a synthetic WGS BAM: a 64 KiB chain segment's first record start often lies past the
    speculation's first 512-byte window (seg_spec_split_kernel searches several windows), and a
    group of 32 such records exceeds the decode's 12 KiB staging (the unstaged path, its block
    sizes read from U)."""
    import struct
    rng = np.random.default_rng(17)
    r = synth.generate(900, seed=33, nthreads=4)
    u = B.inflate_all(r.bam)
    off, _ = B.record_spans(u)[450]
    ref_id, pos = struct.unpack_from("<ii", u, off + 4)
    mids = []
    for k in range(n_mid):
        l_seq = int(rng.integers(300, 4001))
        name = (b"m%d_" % k) + b"x" * int(rng.integers(0, 50))
        mids.append(B.make_record(ref_id, pos, name, l_seq, qual=int(rng.integers(20, 41))))
    return B.bgzf(u[:off] + b"".join(mids) + u[off:], level=5), n_mid


def test_oracle_midsize_records():
    bam, n_mid = midsize_bam()
    assert len(O.OracleBam(bam).read_all()) == 900 + n_mid


@pytest.mark.gpu
def test_gpu_midsize_records():
    from test_gpu_parity import assert_parity
    bam, n_mid = midsize_bam()
    for split in (0, 70000, 150001, 1 << 20):
        b = assert_parity(bam, split)
    assert len(b["block_size"]) == 900 + n_mid
