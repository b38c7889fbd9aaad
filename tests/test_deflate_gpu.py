"""GPU BGZF compression, the write path: dq_bgzf_compress replaces
htsjdk BlockCompressedOutputStream under HeaderlessBamOutputFormat / BamSink.

Bar: the output is valid BGZF -- every member has the 'BC' field, BSIZE, a correct CRC32 and
ISIZE -- cut at htsjdk's 65280-byte block boundaries, and it inflates (zlib, independent of this
library) to exactly the input; a BAM assembled as BamSink.save does (header blocks, part blocks,
EOF block) reads back through the oracle to the same records.  Compressed bytes are not compared
with java.util.zip.Deflater's (a different encoder): parity is on the decompressed content."""
import os
import struct
import zlib

import numpy as np
import pytest

from disq_amd import _lib, synth
from oracle import oracle as O
import bamutil as B

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def members(bgzf):
    out, p = [], 0
    while p < len(bgzf):
        h = bgzf[p:p + 18]
        assert h[:4] == b"\x1f\x8b\x08\x04" and h[10:12] == b"\x06\x00" and h[12:14] == b"BC"
        cs = struct.unpack_from("<H", h, 16)[0] + 1
        body = bgzf[p + 18:p + cs - 8]
        crc, isize = struct.unpack_from("<II", bgzf, p + cs - 8)
        data = zlib.decompress(body, -15)
        assert len(data) == isize and zlib.crc32(data) & 0xffffffff == crc
        out.append(data)
        p += cs
    assert p == len(bgzf)
    return out


def check_roundtrip(c, data):
    z = c.bgzf_compress(data)
    blocks = members(z)
    assert b"".join(blocks) == data
    assert [len(x) for x in blocks] == [min(B.BLOCK_U, len(data) - i)
                                        for i in range(0, len(data), B.BLOCK_U)]
    return z


def test_edge_sizes():
    rng = np.random.default_rng(1)
    with _lib.Context() as c:
        assert c.bgzf_compress(b"") == b""
        # (32640: the parse kernel's chunk -- half a block -- whose matches end inside it)
        for n in (1, 2, 3, 257, 4096, 32639, 32640, 32641, 32642, 32643, 32700, B.BLOCK_U - 1,
                  B.BLOCK_U, B.BLOCK_U + 1, B.BLOCK_U + 32642, 3 * B.BLOCK_U + 17):
            check_roundtrip(c, rng.integers(0, 4, size=n, dtype=np.uint8).tobytes())


def test_incompressible_blocks_are_stored():
    data = np.random.default_rng(2).integers(0, 256, size=200000, dtype=np.uint8).tobytes()
    with _lib.Context() as c:
        z = len(check_roundtrip(c, data))
    assert z == len(data) + 4 * 26 + 4 * 5  # every block stored


def test_bam_stream_ratio_and_roundtrip():
    r = synth.generate(40000, seed=5, nthreads=8)
    u = B.inflate_all(r.bam)
    with _lib.Context() as c:
        z = check_roundtrip(c, u)
    assert len(z) < 0.6 * len(u)  # LZ77 + fixed Huffman on BAM records


def zlib5_bgzf_size(data):
    """htsjdk's BGZF size at its default level 5: a raw deflate member per 65280-byte block."""
    total = 0
    for i in range(0, len(data), B.BLOCK_U):
        z = zlib.compressobj(5, zlib.DEFLATED, -15)
        total += len(z.compress(data[i:i + B.BLOCK_U]) + z.flush()) + 26
    return total


@pytest.mark.parametrize("name", ["1.bam", "hiseq_part-r-00000.bam", "HiSeq.10000.vcf.bgz", "wgs"])
def test_ratio_at_zlib_level5(golden, name):
    """The chunked LDS parse (two 32640-byte chunks per block, 13600 bytes of reach before a chunk, a 4-byte bucket key) keeps
    htsjdk's level-5 ratio on the golden BAM / VCF streams and the synthetic WGS stream
    (tools/deflate_model.c, profiles/r4_deflate_chunk_model.txt): at most 0.5 % larger."""
    if name == "wgs":
        u = B.inflate_all(synth.generate(60000, seed=5, nthreads=8).bam)
    else:
        u = B.inflate_all(open(os.path.join(golden, name), "rb").read())
    with _lib.Context() as c:
        z = check_roundtrip(c, u)
    ref = zlib5_bgzf_size(u)
    assert len(z) <= 1.005 * ref, (len(z), ref, len(u) / len(z), len(u) / ref)


def test_bamsink_assembly_reads_back(tmp_path, golden):
    """BamSink.save: header file + headerless part files + terminator, merged in order."""
    from disq_amd.storage import HtsjdkReadsRddStorage
    src = os.path.join(golden, "1.bam")
    st = HtsjdkReadsRddStorage.makeDefault().splitSize(128 * 1024)
    rdd = st.read(src)
    out = str(tmp_path / "out.bam")
    st.write(rdd, out)
    ob = O.OracleBam.from_path(out, verify_crc=True)
    ref = O.OracleBam.from_path(src)
    a, b = ob.read_all(), ref.read_all()
    assert len(a) == len(b) == 4917
    assert np.array_equal(a["hash"], b["hash"])
    # and the GPU read path reads it back to the same records
    back = st.read(out)
    assert np.array_equal(back.getReads().hashes(), b["hash"])


def test_resident_stream_roundtrip(golden):
    with _lib.Context(verify_crc=True) as c:
        c.open_path(os.path.join(golden, "1.bam"))
        n, ms = c.bgzf_compress_resident()
        z = c.bgzf_fetch(n).tobytes()
    want = O.OracleBam.from_path(os.path.join(golden, "1.bam")).inflate_all().tobytes()
    assert b"".join(members(z)) == want


@pytest.mark.parametrize("period", [1, 3, 7, 100])
def test_repetitive_blocks_compress(period):
    """Long repetitive input: one repeated byte or a short pattern over whole 65280-byte
    blocks.  Round 3 stored such blocks (a lane's continuation of 258-byte matches never met
    another lane's symbol boundary); now the continuation is ended on a later lane's boundary and
    the block compresses like zlib's (a few hundred bytes per block)."""
    pat = np.random.default_rng(period).integers(0, 256, size=period, dtype=np.uint8).tobytes()
    data = (pat * (3 * B.BLOCK_U // period + 1))[:3 * B.BLOCK_U]
    with _lib.Context() as c:
        z = check_roundtrip(c, data)
    assert len(z) < 3 * 2048, len(z)  # zlib level 5: ~ 3 x 100-400 bytes


def test_randomized_length_roundtrip_sweep():
    """200 random lengths (0 .. 3 blocks), 2-bit and 8-bit alphabets, the default match search and
    the longest one (chain 128, nice 258, no `good` cut): every member inflates to its input."""
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 3 * B.BLOCK_U + 100, size=200)
    old = os.environ.get("DQ_DEFLATE")
    try:
        with _lib.Context() as c:
            for i, n in enumerate(lens):
                os.environ["DQ_DEFLATE"] = "96,32,96,8" if i % 2 else "128,32,258,0"
                hi = 4 if i % 4 < 2 else 256
                data = rng.integers(0, hi, size=int(n), dtype=np.uint8).tobytes()
                if i % 8 == 5:  # runs: long matches next to literals
                    data = bytes(np.repeat(np.frombuffer(data[: max(1, n // 50)], np.uint8),
                                           50)[:n]) if n else b""
                if n == 0:
                    assert c.bgzf_compress(data) == b""
                else:
                    check_roundtrip(c, data)
    finally:
        if old is None:
            os.environ.pop("DQ_DEFLATE", None)
        else:
            os.environ["DQ_DEFLATE"] = old


def test_output_is_deterministic():
    """Two compressions of the same bytes are byte-identical, as htsjdk's
    BlockCompressedOutputStream under HeaderlessBamOutputFormat.java:26-50 is: a WGS stream and the
    period-3 stream whose ratio moved between runs while round 4's lanes raced for odd segments
    (each segment's parse now starts at its own start, one lane per segment)."""
    r = synth.generate(20000, seed=5, nthreads=4)
    wgs = B.inflate_all(r.bam)
    per3 = (b"ACG" * 200000)[:500000]
    with _lib.Context() as c:
        for data in (wgs, per3):
            a = c.bgzf_compress(data)
            b = c.bgzf_compress(data)
            assert a == b
            assert b"".join(members(a)) == data
    with _lib.Context() as c2:  # and a fresh context
        assert c2.bgzf_compress(per3) == a


_BALLOT_SCRIPT = r"""
import sys
sys.path.insert(0, sys.argv[1])
from disq_amd import _lib
src = open(sys.argv[2], "rb").read()
with _lib.Context() as c:
    out = c.bgzf_compress(src)
open(sys.argv[3], "wb").write(out)
"""


@pytest.mark.gpu
def test_atomic_scatter_equals_ballot_build(tmp_path):
    """The product library ranks equal-hash positions of the bucket scatter by lane-ordered LDS
    atomics (observed on gfx950, not documented); the ballot build (DQ_SCAT_ATOMIC=0, `make
    ballot`) ranks them by ballots, deterministic by construction.  Both must write the same
    bytes: if the hardware ever returned the atomics out of lane order the parse would see other
    candidates and this comparison would fail (the output would still be valid DEFLATE)."""
    import subprocess
    import sys
    lib = os.path.join(ROOT, "disq_amd", "_build", "libdisq_gpu_ballot.so")
    if not os.path.exists(lib):
        pytest.fail("libdisq_gpu_ballot.so is not built (make -C disq_amd/csrc ballot)")
    r = synth.generate(20000, seed=9, nthreads=4)
    data = B.inflate_all(r.bam) + (b"ACG" * 100000)
    src, dst = tmp_path / "in.bin", tmp_path / "out.bgzf"
    src.write_bytes(data)
    env = dict(os.environ, DQ_GPU_LIB=lib)
    subprocess.run([sys.executable, "-c", _BALLOT_SCRIPT, ROOT, str(src), str(dst)], env=env,
                   check=True, timeout=300)
    with _lib.Context() as c:
        mine = c.bgzf_compress(data)
    assert dst.read_bytes() == mine
    assert b"".join(members(mine)) == data
