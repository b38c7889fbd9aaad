"""Directed tests of K2's tail hand-off.

inflate_block_kernel decodes a BGZF member's first deflate block and, when what follows is small
-- at most TOUT = 4096 output bytes and TAIL_MAX_BITS = 32768 compressed bits
(dq_inflate3.hip, the `tails && isize - produced <= TOUT && endbits - pos <= TAIL_MAX_BITS` gate)
-- leaves the rest to inflate_tail_kernel, which decodes it with one wave, resolves its matches
against the block kernel's output in U and finishes the member's CRC from the prefix's CRC
register.  htsjdk's level 5 makes such a tail in almost every block, so these members put the
boundary exactly where the gate decides: tails of 4096 / 4097 output bytes, of 32768 / 32769
bits, a tail after an empty first deflate block, tails of several deflate blocks (stored + fixed + dynamic), a match at distance 32768 into
the prefix, short-distance runs, and a flipped CRC, an invalid code and a too-far distance inside a
tail.  The members are written bit by bit (tests/deflate_writer.py) and checked against zlib here;
the GPU tests compare the decompressed stream with zlib's and expect the errors zlib raises (the
reference inflates with java.util.zip.Inflater, i.e. zlib; htsjdk BlockGunzipper)."""
import zlib

import numpy as np
import pytest

import bamutil as B
import deflate_writer as W
from disq_amd import synth

TOUT, TAIL_MAX_BITS = 4096, 32768  # dq_inflate3.hip


@pytest.fixture(scope="module")
def wgs():
    """A WGS-shaped BAM stream (the synthetic generator's records): realistic matches."""
    r = synth.generate(900, seed=41, nthreads=2)
    return B.inflate_all(r.bam)


def _first_block(D, toks, first):
    if first == "fixed":
        D.fixed(toks)
    else:
        D.dynamic(toks, lens=W.Deflater().dynamic_lengths(toks))


def build(prefix, tail, first="dynamic", mod8=None, pad_from=b"", isize_extra=0):
    """A member whose first deflate block holds `prefix` and whose later blocks are `tail`, a list
    of (kind, tokens or bytes, final) with kind fixed / dynamic / stored / fixed_bad (a fixed block
    with the invalid symbol 286 before its end).  mod8: pad the first block with literals (taken
    from pad_from) until its bit length is that residue mod 8.  Returns (member, data, gate) with
    gate = (tail output bytes, tail bits) as the block kernel computes them."""
    toks = W.lz77(prefix)
    lens = W.Deflater().dynamic_lengths(toks)
    if mod8 is not None:
        extra = []
        for b in pad_from:
            D = W.Deflater()
            t2 = toks + extra
            if first == "fixed":
                D.fixed(t2)
            else:
                D.dynamic(t2, lens=lens)
            if D.pos % 8 == mod8:
                break
            extra.append(b)
        else:
            raise AssertionError("no padding reaches the residue")
        toks = toks + extra
        prefix = prefix + bytes(extra)
    D = W.Deflater()
    if first == "fixed":
        D.fixed(toks)
    else:
        D.dynamic(toks, lens=lens)
    p = D.pos
    data = bytearray(prefix)
    for kind, payload, final in tail:
        if kind == "stored":
            D.stored(payload, final)
            data += payload
        else:
            if kind == "fixed":
                D.fixed(payload, final)
            elif kind == "fixed_bad":
                D.fixed(payload, final, extra=(286,))
            else:
                D.dynamic(payload, final)
            data += W.expand(payload, bytes(data))
    body = D.finish()
    return (W.member(body, bytes(data), isize=len(data) + isize_extra), bytes(data),
            (len(data) + isize_extra - len(prefix), 8 * len(body) - p))


def deferred(gate):
    return gate[0] <= TOUT and gate[1] <= TAIL_MAX_BITS


def literals_for_bits(T, rng):
    """Literal bytes whose fixed codes plus the block's 3 header and 7 EOB bits make T bits:
    a literal below 144 is 8 bits, one from 144 up 9."""
    n = (T - 10 + 8) // 9
    while 8 * n > T - 10 or 9 * n < T - 10:
        n += 1
    b = T - 10 - 8 * n
    assert 0 <= b <= n
    hi = rng.integers(144, 256, b)
    lo = rng.integers(0, 144, n - b)
    out = np.concatenate([hi, lo]).astype(np.uint8)
    rng.shuffle(out)
    return bytes(out)


def fixtures(u):
    """name -> (member bytes, decompressed bytes, gate, expected deferral, zlib error or None)."""
    rng = np.random.default_rng(7)
    f = {}
    # an empty, non-final first deflate block (only its EOB) and a small tail: the tail starts at
    # output byte 0 of the member (p0 = 0), so nothing of it lies in a prefix
    m, d, g = build(b"", [("fixed", W.lz77(u[:3000]), True)], first="fixed")
    f["empty_first"] = (m, d, g, True, None)
    pre = u[:60000]
    for n in (4096, 4097):
        data = u[:60000 + n]
        m, d, g = build(pre, [("fixed", W.lz77(data, 60000), True)])
        f["out%d" % n] = (m, d, g, n <= TOUT, None)
    # tails of exactly 32768 / 32769 bits (fixed literals), the first block padded so that the
    # member's last byte ends the tail exactly
    for bits, mod8 in ((32768, 0), (32769, 7)):
        T = bits if mod8 == 0 else bits
        lit = literals_for_bits(T, rng)
        m, d, g = build(pre, [("fixed", list(lit), True)], mod8=mod8, pad_from=u[60000:61000])
        f["bits%d" % bits] = (m, d, g, bits <= TAIL_MAX_BITS, None)
    # a tail of three deflate blocks: stored, fixed, dynamic
    a, b, c = 60000, 60600, 61800
    data = u[:63300]
    m, d, g = build(pre, [("stored", data[a:b], False), ("fixed", W.lz77(data, b, c), False),
                          ("dynamic", W.lz77(data, c, 63300), True)])
    f["stored_fixed_dynamic"] = (m, d, g, True, None)
    # a match at distance 32768 (and of length 258) reaching into the prefix, then more data
    p2 = bytearray(u[:60000])
    tail = bytes(p2[60000 - 32768:60000 - 32768 + 258]) + u[70000:72000]
    data = bytes(p2) + tail
    toks = [(258, 32768)] + W.lz77(data, 60258)
    m, d, g = build(bytes(p2), [("fixed", toks, True)])
    assert d == data
    f["dist32768"] = (m, d, g, True, None)
    # short-distance runs: distance 1 / 3 / 7 of the maximal length, inside the tail
    toks = [65, (258, 1), 66, 67, 68, (258, 3), 1, 2, 3, 4, 5, 6, 7, (200, 7), (10, 4000)]
    m, d, g = build(pre, [("dynamic", toks, True)])
    f["runs"] = (m, d, g, True, None)
    # errors inside a deferred tail: a flipped CRC byte, an invalid code (286), too far back.
    # The member's ISIZE claims bytes past the invalid code: java.util.zip.Inflater stops once
    # ISIZE bytes are out (BlockGunzipper inflates into an ISIZE-byte buffer), so a bad code after
    # them is never read -- by zlib or by the kernel
    m, d, g = f["out4096"][:3]
    bad = bytearray(m)
    bad[-8] ^= 0x40
    f["crc"] = (bytes(bad), d, g, True, "crc")
    m, d, g = build(pre, [("fixed_bad", W.lz77(u[:61000], 60000), True)], isize_extra=7)
    f["badcode"] = (m, d, g, True, "invalid literal/length code")
    small = u[:1000]
    m, d, g = build(small, [("fixed", [70, 71, 72, (5, 2000)], True)])
    f["toofar"] = (m, d, g, True, "invalid distance too far back")
    return f


@pytest.fixture(scope="module")
def fx(wgs):
    return fixtures(wgs)


def test_fixtures_hit_the_gate(fx):
    """Every member inflates with zlib to its data (or fails as intended), and the gate values sit
    on the boundary each name says."""
    for name, (m, d, g, dfr, err) in fx.items():
        body = m[18:-8]
        if err is None:
            assert zlib.decompress(body, -15) == d, name
            assert m[-4:] == len(d).to_bytes(4, "little")
        elif err != "crc":
            # an ISIZE-bounded inflate, as BlockGunzipper's, reaches the error
            isize = int.from_bytes(m[-4:], "little")
            with pytest.raises(zlib.error, match=err):
                zlib.decompressobj(-15).decompress(body, isize)
        assert deferred(g) == dfr, (name, g)
    assert fx["out4096"][2][0] == 4096 and fx["out4097"][2][0] == 4097
    assert fx["bits32768"][2][1] == 32768 and fx["bits32769"][2][1] == 32769
    assert fx["bits32768"][2][0] <= TOUT and fx["bits32769"][2][0] <= TOUT


def resolve_members(u):
    """zlib members of assorted sizes (the BGZF output offset mod 16 varies from member to member,
    so the resolve's image alignment does): 1 .. 65536 bytes at levels 1, 6, 9."""
    out, data = [], []
    sizes = [65536, 1, 65535, 17, 512, 513, 511, 4095, 65280, 3, 40000, 65498]
    for i, n in enumerate(sizes):
        s = (u * 2)[i * 3001:i * 3001 + n]
        lvl = (1, 6, 9)[i % 3]
        c = zlib.compressobj(lvl, zlib.DEFLATED, -15)
        body = c.compress(s) + c.flush()
        out.append(W.member(body, s))
        data.append(s)
    return out, data


def _gpu_inflate(bgzf_bytes):
    from disq_amd import _lib
    with _lib.Context(split_size=0, verify_crc=True, device=0) as c:
        c.text_open_bytes(bgzf_bytes)
        c.text_run(drop_header_lines=False)
        return c.inflated()


@pytest.mark.gpu
def test_gpu_tail_boundaries(fx):
    """The good members in one file: the decompressed stream equals zlib's byte for byte."""
    good = [(m, d) for m, d, g, dfr, err in fx.values() if err is None]
    got = _gpu_inflate(b"".join(m for m, _ in good) + B.EOF_BLOCK)
    want = b"".join(d for _, d in good)
    assert len(got) == len(want)
    assert np.array_equal(got, np.frombuffer(want, np.uint8))


@pytest.mark.gpu
def test_gpu_tail_after_empty_first_block(fx):
    """The empty-first-block member as the file's first block (its tail begins at U's first byte),
    then a deferred tail with a prefix: both equal zlib's output (advisor round 5: the tail resolve's
    dummy load must stay inside U when the prefix is empty; the checked build bounds it)."""
    a, b = fx["empty_first"], fx["out4096"]
    got = _gpu_inflate(a[0] + b[0] + B.EOF_BLOCK)
    want = a[1] + b[1]
    assert np.array_equal(got, np.frombuffer(want, np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["crc", "badcode", "toofar"])
def test_gpu_tail_errors(fx, wgs, name):
    """An error inside a deferred tail fails the read (DQ_EFORMAT), between two good members."""
    from disq_amd import _lib
    m = fx[name][0]
    ok = fx["out4096"][0]
    with pytest.raises(_lib.DqError):
        _gpu_inflate(ok + m + ok + B.EOF_BLOCK)


@pytest.mark.gpu
def test_gpu_resolve_alignments(wgs):
    """Members of 1 .. 65536 bytes back to back: every output alignment of the resolve's image."""
    ms, ds = resolve_members(wgs)
    got = _gpu_inflate(b"".join(ms) + B.EOF_BLOCK)
    want = b"".join(ds)
    assert np.array_equal(got, np.frombuffer(want, np.uint8))


def after_isize_member(u):
    """An invalid code (286) right after the ISIZE bytes of a deferred tail."""
    m, d, g = build(u[:60000], [("fixed_bad", W.lz77(u[:61000], 60000), True)])
    return m, d, g


def test_after_isize_fixture(wgs):
    """A documented difference (malformed input, out of scope per SURVEY.md section 7): zlib's
    inflate (java.util.zip.Inflater under BlockGunzipper) decodes the symbol after its output
    buffer is full -- its LEN state runs before the LIT state checks for room -- so an invalid code
    right after the ISIZE-th byte fails even an ISIZE-bounded inflate; the kernels stop at ISIZE
    and never read it."""
    m, d, g = after_isize_member(wgs)
    assert deferred(g)
    body = m[18:-8]
    with pytest.raises(zlib.error, match="invalid literal/length code"):
        zlib.decompressobj(-15).decompress(body, len(d))


@pytest.mark.gpu
def test_gpu_code_after_isize_is_not_read(wgs):
    m, d, _ = after_isize_member(wgs)
    got = _gpu_inflate(m + B.EOF_BLOCK)
    assert np.array_equal(got, np.frombuffer(d, np.uint8))
