"""Test helpers: re-block a BAM's decompressed stream into BGZF at any deflate level, and build
records by hand -- to make adversarial fixtures the seeded generator does not produce (a BGZF
header inside record payload at a split start, a record longer than MAX_READ_SIZE).

Block layout follows htsjdk BlockCompressedOutputStream (gzip member with the 'BC' extra field,
BSIZE = member length - 1, CRC32 and ISIZE trailer) and ends with the 28-byte EOF block."""
import struct
import zlib

EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
BLOCK_U = 65280  # htsjdk BlockCompressedStreamConstants.DEFAULT_UNCOMPRESSED_BLOCK_SIZE


def inflate_all(bam: bytes) -> bytes:
    out, p = [], 0
    while p < len(bam):
        bsize = struct.unpack_from("<H", bam, p + 16)[0]
        cs = bsize + 1
        out.append(zlib.decompress(bam[p + 18:p + cs - 8], -15))
        p += cs
    return b"".join(out)


def bgzf_member(data: bytes, level: int) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    body = c.compress(data) + c.flush()
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
    member = hdr + struct.pack("<H", 18 + len(body) + 8 - 1) + body
    return member + struct.pack("<II", zlib.crc32(data) & 0xffffffff, len(data))


def bgzf(stream: bytes, level: int, block_u: int = BLOCK_U, cuts=()) -> bytes:
    """BGZF of `stream` in blocks of block_u bytes; `cuts` are extra block boundaries."""
    bounds = sorted(set(list(range(0, len(stream), block_u)) + [c for c in cuts if 0 < c < len(stream)]))
    bounds.append(len(stream))
    return b"".join(bgzf_member(stream[a:b], level) for a, b in zip(bounds, bounds[1:])) + EOF_BLOCK


def header_len(u: bytes) -> int:
    assert u[:4] == b"BAM\x01"
    l_text = struct.unpack_from("<i", u, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", u, p)[0]
    p += 4
    for _ in range(n_ref):
        l_name = struct.unpack_from("<i", u, p)[0]
        p += 4 + l_name + 4
    return p


def record_spans(u: bytes):
    """(offset, length incl. the block_size word) of every record."""
    p, out = header_len(u), []
    while p < len(u):
        bs = struct.unpack_from("<i", u, p)[0]
        out.append((p, 4 + bs))
        p += 4 + bs
    return out


def qual_offset(rec: bytes) -> int:
    """Offset of the quality string inside a record (including its block_size word)."""
    l_read_name = rec[12]
    n_cigar = struct.unpack_from("<H", rec, 16)[0]
    l_seq = struct.unpack_from("<i", rec, 20)[0]
    return 36 + l_read_name + 4 * n_cigar + (l_seq + 1) // 2


def make_record(ref_id, pos, name: bytes, l_seq, flag=0, mapq=60, base=0x11, qual=30,
                next_ref_id=-1, next_pos=-1, tlen=0) -> bytes:
    """A mapped record with one M cigar op over l_seq bases (all one base, constant quality)."""
    rn = name + b"\x00"
    cigar = struct.pack("<I", (l_seq << 4) | 0)
    seq = bytes([base]) * ((l_seq + 1) // 2)
    body = struct.pack("<iiBBHHHiiii", ref_id, pos, len(rn), mapq, 4680, 1, flag, l_seq,
                       next_ref_id, next_pos, tlen) + rn + cigar + seq + bytes([qual]) * l_seq
    return struct.pack("<i", len(body)) + body
