"""Kernel 2 on DEFLATE shapes the synthetic generator does not produce.

htsjdk hands each BGZF member to java.util.zip.Inflater (zlib): any valid raw-DEFLATE stream must
inflate.  The records below keep their fields but carry quality strings drawn from a skewed byte
distribution (two frequent values, 254 rare ones), so zlib's literal/length code has dozens of
codes longer than the 10-bit root table under more distinct root prefixes (> 16) than round 2's
fixed second-level tables held: the variable-size second-level tables (one per prefix, sized by
its longest code) take all of them.  A hand-built block with more prefixes than the kernel keeps
tables for (MAXGRP = 64) reaches the canonical slow path, and one with long DISTANCE codes under 5
prefixes the distance tables.  The same stream is also compressed with fixed Huffman codes
(Z_FIXED) and stored (level 0).  Parity: the decompressed stream equals zlib's, every partition
equals the oracle's.  The CPU tests check the fixtures' shapes (a DEFLATE header parser counts the
prefixes), so the GPU tests cannot pass vacuously."""
import struct
import zlib

import numpy as np
import pytest

from disq_amd import synth
from oracle import oracle as O

import bamutil as B

LR, LSLOTS = 10, 16  # litlen root bits of dq_inflate3.hip; round 2's fixed second-level tables
MAXGRP = 64  # second-level litlen tables the kernel keeps (dq_inflate3.hip); more -> slow path


def skewed_stream(n=3000, seed=31, rare=0.03):
    r = synth.generate(n, seed=seed, nthreads=4)
    u = bytearray(B.inflate_all(r.bam))
    rng = np.random.default_rng(seed)
    p = np.full(256, rare / 254.0)
    p[65] = p[66] = (1 - rare) / 2
    for off, ln in B.record_spans(bytes(u)):
        q = off + B.qual_offset(bytes(u[off:off + ln]))
        u[q:off + ln] = rng.choice(256, size=off + ln - q, p=p).astype(np.uint8).tobytes()
    return bytes(u)


def member(data, level, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
    body = c.compress(data) + c.flush()
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
    m = hdr + struct.pack("<H", 18 + len(body) + 8 - 1) + body
    return m + struct.pack("<II", zlib.crc32(data) & 0xffffffff, len(data))


def bgzf(u, level, strategy=zlib.Z_DEFAULT_STRATEGY):
    return b"".join(member(u[a:a + B.BLOCK_U], level, strategy)
                    for a in range(0, len(u), B.BLOCK_U)) + B.EOF_BLOCK


CASES = [(1, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_DEFAULT_STRATEGY), (9, zlib.Z_DEFAULT_STRATEGY),
         (6, zlib.Z_FIXED), (0, zlib.Z_DEFAULT_STRATEGY)]


class _Bits:
    def __init__(self, b):
        self.b, self.p = b, 0

    def get(self, n):
        v = 0
        for i in range(n):
            v |= ((self.b[(self.p + i) >> 3] >> ((self.p + i) & 7)) & 1) << i
        self.p += n
        return v


def _canonical(lens):
    bl = [0] * 16
    for ln in lens:
        if ln:
            bl[ln] += 1
    nxt, code = [0] * 16, 0
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1 if b > 1 else 0
        nxt[b] = code
    out = []
    for ln in lens:
        out.append(nxt[ln] if ln else None)
        if ln:
            nxt[ln] += 1
    return out


def litlen_long_prefixes(body):
    """Distinct LR-bit prefixes of the litlen codes longer than LR bits in the first deflate block
    of a raw-DEFLATE body (0 for stored / fixed blocks)."""
    r = _Bits(body)
    r.get(1)
    if r.get(2) != 2:
        return 0
    hlit, hdist, hclen = r.get(5) + 257, r.get(5) + 1, r.get(4) + 4
    cl = [0] * 19
    for i in range(hclen):
        cl[[16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15][i]] = r.get(3)
    cc = _canonical(cl)
    tab = {(cc[s], cl[s]): s for s in range(19) if cl[s]}
    lens = []
    while len(lens) < hlit + hdist:
        code, n = 0, 0
        while (code, n) not in tab:
            code, n = (code << 1) | r.get(1), n + 1
        s = tab[(code, n)]
        if s < 16:
            lens.append(s)
        elif s == 16:
            lens += [lens[-1]] * (3 + r.get(2))
        else:
            lens += [0] * ((3 + r.get(3)) if s == 17 else (11 + r.get(7)))
    codes = _canonical(lens[:hlit])
    return len({codes[i] >> (ln - LR) for i, ln in enumerate(lens[:hlit]) if ln > LR})


@pytest.fixture(scope="module")
def stream():
    return skewed_stream()


def test_fixtures_need_many_second_level_tables(stream):
    """Every dynamic member of the level 1/6/9 files has long codes under more root prefixes than
    16 (the fixed tables of round 2, which sent the rest to the canonical slow path)."""
    for level in (1, 6, 9):
        bodies = [member(stream[a:a + B.BLOCK_U], level)[18:-8]
                  for a in range(0, len(stream), B.BLOCK_U)]
        counts = [litlen_long_prefixes(b) for b in bodies]
        assert min(counts) > LSLOTS, (level, counts)
    fixed = member(stream[:B.BLOCK_U], 6, zlib.Z_FIXED)[18:]
    assert (fixed[0] >> 1) & 3 == 1  # the first deflate block is fixed-Huffman


@pytest.mark.gpu
@pytest.mark.parametrize("level,strategy", CASES)
def test_gpu_inflate_long_codes_fixed_and_stored(stream, level, strategy):
    from disq_amd import _lib
    bam = bgzf(stream, level, strategy)
    split = 96 * 1024
    with _lib.Context(split_size=split, verify_crc=True, device=0) as c:
        c.open_bytes(bam)
        b = c.read(with_raw=False)
        u = c.inflated()
    assert np.array_equal(u, np.frombuffer(stream, np.uint8))
    parts = O.OracleBam(bam).read_partitions(split)
    ref = np.concatenate(parts)
    assert len(b["voffset"]) == len(ref)
    assert np.array_equal(b["voffset"], ref["voffset"])
    assert np.array_equal(b["hash"], ref["hash"])


# ---- a hand-built dynamic block with long DISTANCE codes: 10 nine-bit distance codes under 5
# distinct 8-bit prefixes (round 2 had 4 fixed second-level distance tables and a slow path).
DR, DSLOTS = 8, 4
LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
         131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537,
         2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]
# literal/length code: 256 literals of 9 bits, EOB and length 3 of 3 bits, lengths 4..42 of 6 bits
LL_LENS = [9] * 256 + [3, 3] + [6] * 16 + [0] * 12
# distance code: 3x2 + 3x4 + 5 + 7 + 8 + 10x9 bits (Kraft sum 1); symbols 9..18 are the long ones
D_LENS = [2, 2, 2, 4, 4, 4, 5, 7, 8] + [9] * 10 + [0] * 11


class _Writer:
    def __init__(self):
        self.v, self.n = 0, 0

    def bits(self, x, n):  # LSB first
        self.v |= (x & ((1 << n) - 1)) << self.n
        self.n += n

    def code(self, c, n):  # Huffman codes go MSB first
        self.bits(int(format(c, "0%db" % n)[::-1], 2), n)

    def bytes(self):
        return self.v.to_bytes((self.n + 7) // 8, "little")


def deflate_long_distances(data: bytes, stride: int, ll_lens=LL_LENS, d_lens=D_LENS) -> bytes:
    """One final dynamic block of `data`: matches at k * stride (k = 1..5, cycling) of <= 42
    bytes where the bytes repeat, literals elsewhere."""
    LL_LENS, D_LENS = ll_lens, d_lens
    llc, dc = _canonical(LL_LENS), _canonical(D_LENS)
    w = _Writer()
    w.bits(1, 1)
    w.bits(2, 2)
    w.bits(286 - 257, 5)
    w.bits(30 - 1, 5)
    w.bits(19 - 4, 4)
    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    cl = [4 if s < 16 else 0 for s in range(19)]  # code-length code: symbols 0..15, 4 bits each
    for s in order:
        w.bits(cl[s], 3)
    clc = _canonical(cl)
    for ln in LL_LENS + D_LENS:
        w.code(clc[ln], 4)
    i, k = 0, 0
    while i < len(data):
        k = k % 5 + 1
        d = k * stride
        n = 0
        while d <= i and n < 42 and i + n < len(data) and data[i + n] == data[i + n - d]:
            n += 1
        if n >= 3:
            ls = max(j for j in range(17) if LBASE[j] <= n)  # symbols 257..273
            w.code(llc[257 + ls], LL_LENS[257 + ls])
            w.bits(n - LBASE[ls], LEXT[ls])
            ds = max(j for j in range(30) if DBASE[j] <= d)
            assert D_LENS[ds], d
            w.code(dc[ds], D_LENS[ds])
            w.bits(d - DBASE[ds], DEXT[ds])
            i += n
        else:
            w.code(llc[data[i]], LL_LENS[data[i]])
            i += 1
    w.code(llc[256], LL_LENS[256])
    return w.bytes()


def long_distance_bam(ll_lens=LL_LENS):
    r = synth.generate(50, seed=33, nthreads=2)
    u = B.inflate_all(r.bam)
    head = u[:B.header_len(u)]
    rec = B.make_record(0, 5000, b"r", 58)
    stride = len(rec)
    assert stride == 129
    body = rec * 450  # 58,050 bytes: one member
    deflated = deflate_long_distances(body, stride, ll_lens)
    assert zlib.decompress(deflated, -15) == body
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
    m = hdr + struct.pack("<H", 18 + len(deflated) + 8 - 1) + deflated
    m += struct.pack("<II", zlib.crc32(body) & 0xffffffff, len(body))
    return member(head, 6) + m + member(rec * 40, 6) + B.EOF_BLOCK, head + body + rec * 40


def test_long_distance_fixture():
    dc = _canonical(D_LENS)
    prefixes = {dc[s] >> (ln - DR) for s, ln in enumerate(D_LENS) if ln > DR}
    assert len(prefixes) > DSLOTS
    bam, u = long_distance_bam()
    assert B.inflate_all(bam) == u
    used = set()  # the distances the stream uses reach the slow-path prefix group (255)
    for k in range(1, 6):
        d = k * 129
        used.add(max(j for j in range(30) if DBASE[j] <= d))
    assert {17, 18} <= used and dc[17] >> 1 == dc[18] >> 1 == 255


@pytest.mark.gpu
def test_gpu_inflate_distance_slow_path():
    from disq_amd import _lib
    bam, u = long_distance_bam()
    split = 8 * 1024
    with _lib.Context(split_size=split, verify_crc=True, device=0) as c:
        c.open_bytes(bam)
        b = c.read(with_raw=False)
        got = c.inflated()
    assert np.array_equal(got, np.frombuffer(u, np.uint8))
    ref = np.concatenate(O.OracleBam(bam).read_partitions(split))
    assert len(b["voffset"]) == len(ref) == 490
    assert np.array_equal(b["voffset"], ref["voffset"])
    assert np.array_equal(b["hash"], ref["hash"])


# ---- a hand-built literal/length code with 160 eleven-bit codes (literals 118..255, EOB and the
# lengths 257..277) under 80 distinct 10-bit prefixes: more than MAXGRP, so the codes of the last
# 16 prefixes take the canonical slow path; 118 seven-bit literals fill the rest (Kraft sum 1).
LL_MANY = [7] * 118 + [11] * 160 + [0] * 8


def test_many_prefix_fixture():
    assert sum(2.0 ** -n for n in LL_MANY if n) == 1.0
    cc = _canonical(LL_MANY)
    prefixes = {cc[s] >> (ln - LR) for s, ln in enumerate(LL_MANY) if ln > LR}
    assert len(prefixes) == 80 > MAXGRP
    bam, u = long_distance_bam(LL_MANY)
    assert B.inflate_all(bam) == u
    # the records' bytes use literals under the slow-path prefixes (the last 16 in code order)
    slow = {s for s, ln in enumerate(LL_MANY) if ln > LR and (cc[s] >> 1) >= 1024 - 16}
    assert slow & set(u)


@pytest.mark.gpu
def test_gpu_inflate_litlen_slow_path():
    from disq_amd import _lib
    bam, u = long_distance_bam(LL_MANY)
    split = 8 * 1024
    with _lib.Context(split_size=split, verify_crc=True, device=0) as c:
        c.open_bytes(bam)
        b = c.read(with_raw=False)
        got = c.inflated()
    assert np.array_equal(got, np.frombuffer(u, np.uint8))
    ref = np.concatenate(O.OracleBam(bam).read_partitions(split))
    assert len(b["voffset"]) == len(ref) == 490
    assert np.array_equal(b["voffset"], ref["voffset"])
    assert np.array_equal(b["hash"], ref["hash"])


# ---- an incomplete distance code: a single one-bit code (symbol 14: distances 129..192, 6 extra
# bits), which zlib's inflate accepts (inflate_table: an incomplete code is allowed only as one
# code of length 1).  Half of the 8-bit distance root indices have no code: the kernel's common
# path sends them to the invalid-code sentinel of the unused second-level area (dq_inflate3.hip
# build_tables), so a stream that uses one must fail like zlib ("invalid distance code").
D_ONE = [0] * 14 + [1] + [0] * 15


def deflate_one_distance(data: bytes, d: int, bad: bool = False) -> bytes:
    """One final dynamic block of `data` with LL_LENS and D_ONE: matches at distance d where the
    bytes repeat (<= 42 long), literals elsewhere.  bad: the first match's distance code is the
    code-less bit 1."""
    llc = _canonical(LL_LENS)
    w = _Writer()
    w.bits(1, 1)
    w.bits(2, 2)
    w.bits(286 - 257, 5)
    w.bits(30 - 1, 5)
    w.bits(19 - 4, 4)
    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    cl = [4 if s < 16 else 0 for s in range(19)]
    for s in order:
        w.bits(cl[s], 3)
    clc = _canonical(cl)
    for ln in LL_LENS + D_ONE:
        w.code(clc[ln], 4)
    assert DBASE[14] <= d < DBASE[15]
    i, first = 0, True
    while i < len(data):
        n = 0
        while d <= i and n < 42 and i + n < len(data) and data[i + n] == data[i + n - d]:
            n += 1
        if n >= 3:
            ls = max(j for j in range(17) if LBASE[j] <= n)
            w.code(llc[257 + ls], LL_LENS[257 + ls])
            w.bits(n - LBASE[ls], LEXT[ls])
            w.bits(1 if (bad and first) else 0, 1)  # the one distance code is the bit 0
            w.bits(d - DBASE[14], DEXT[14])
            first = False
            i += n
        else:
            w.code(llc[data[i]], LL_LENS[data[i]])
            i += 1
    w.code(llc[256], LL_LENS[256])
    return w.bytes()


def one_distance_bam(bad=False):
    r = synth.generate(50, seed=33, nthreads=2)
    u = B.inflate_all(r.bam)
    head = u[:B.header_len(u)]
    rec = B.make_record(0, 5000, b"r", 58)
    body = rec * 450
    deflated = deflate_one_distance(body, len(rec), bad)
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
    m = hdr + struct.pack("<H", 18 + len(deflated) + 8 - 1) + deflated
    m += struct.pack("<II", zlib.crc32(body) & 0xffffffff, len(body))
    return member(head, 6) + m + member(rec * 40, 6) + B.EOF_BLOCK, head + body + rec * 40, deflated


def test_one_distance_fixture():
    bam, u, deflated = one_distance_bam()
    assert zlib.decompress(deflated, -15) == u[B.header_len(u):][:58050]
    assert B.inflate_all(bam) == u
    _, _, bad = one_distance_bam(bad=True)
    with pytest.raises(zlib.error, match="invalid distance code"):
        zlib.decompress(bad, -15)


@pytest.mark.gpu
def test_gpu_inflate_incomplete_distance_code():
    from disq_amd import _lib
    bam, u, _ = one_distance_bam()
    split = 8 * 1024
    with _lib.Context(split_size=split, verify_crc=True, device=0) as c:
        c.open_bytes(bam)
        b = c.read(with_raw=False)
        got = c.inflated()
    assert np.array_equal(got, np.frombuffer(u, np.uint8))
    ref = np.concatenate(O.OracleBam(bam).read_partitions(split))
    assert len(b["voffset"]) == len(ref) == 490
    assert np.array_equal(b["hash"], ref["hash"])
    bad, _, _ = one_distance_bam(bad=True)
    with _lib.Context(split_size=split, verify_crc=True, device=0) as c:
        c.open_bytes(bad)
        with pytest.raises(_lib.DqError):
            c.run_resident()
