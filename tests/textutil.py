"""Synthetic BGZF text (VCF-like) files for the text-path tests: line lengths, terminators (LF,
CR LF, lone CR), a UTF-8 BOM, '#' lines and block boundaries placed where the reader's state
machine has its corners (a block ending right after a CR, between CR and LF, on a line start)."""
import numpy as np

import bamutil as B


def make_text(n_lines, seed=0, newline="lf", bom=False, header_lines=5, hash_every=0,
              min_len=0, max_len=300, long_every=0, long_len=200000):
    rng = np.random.default_rng(seed)
    nls = {"lf": [b"\n"], "crlf": [b"\r\n"], "cr": [b"\r"], "mixed": [b"\n", b"\r\n", b"\r"]}[newline]
    out = [b"\xef\xbb\xbf"] if bom else []
    for i in range(header_lines):
        out.append(b"##meta=%d" % i + nls[0])
    out.append(b"#CHROM\tPOS\tID\tREF\tALT" + nls[0])
    for i in range(n_lines):
        n = long_len if (long_every and i % long_every == long_every - 1) else int(rng.integers(min_len, max_len + 1))
        body = rng.integers(33, 127, size=n, dtype=np.uint8).tobytes().replace(b"#", b"x")
        if hash_every and i % hash_every == 0:
            body = b"#" + body
        nl = nls[int(rng.integers(0, len(nls)))]
        out.append(body + nl)
    return b"".join(out)


def corner_cuts(text, every=7):
    """Extra block boundaries: right after some CRs, between some CR LF pairs, after some LFs."""
    cuts = []
    for k, c in enumerate(text):
        if c in (10, 13) and k % every == 0:
            cuts.append(k + 1)
            if c == 13:
                cuts.append(k)
    return cuts


def bgzf_text(text, level=6, block_u=B.BLOCK_U, cuts=()):
    return B.bgzf(text, level, block_u=block_u, cuts=cuts)


def split_lines(text):
    """Lines as LineReader.readDefaultLine cuts them: LF, CR LF or a lone CR end a line; a last
    line without a terminator counts; no line after a final terminator."""
    out, a, i, n = [], 0, 0, len(text)
    while i < n:
        c = text[i]
        if c == 10:
            out.append(text[a:i]); i += 1; a = i
        elif c == 13:
            out.append(text[a:i]); i += 2 if i + 1 < n and text[i + 1] == 10 else 1; a = i
        else:
            i += 1
    if a < n:
        out.append(text[a:])
    return out


def make_vcf(n, seed=0, contigs=("chr1", "chr2", "chrX"), end_every=7):
    """A sorted VCF-like text: CHROM POS ID REF ALT QUAL FILTER INFO, some records with an INFO END
    (symbolic alleles) and multi-base REFs, a '#' header."""
    rng = np.random.default_rng(seed)
    out = [b"##fileformat=VCFv4.2", b"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO"]
    per = n // len(contigs)
    for c in contigs:
        pos = 1
        for i in range(per):
            pos += int(rng.integers(1, 400))
            ref = b"ACGT"[int(rng.integers(0, 4)):][:1] * int(rng.integers(1, 6))
            info = b"DP=%d" % int(rng.integers(1, 99))
            alt = b"T"
            if end_every and i % end_every == 0:
                info = b"SVTYPE=DEL;END=%d;DP=3" % (pos + int(rng.integers(50, 5000)))
                alt = b"<DEL>"
            out.append(b"\t".join([c.encode(), b"%d" % pos, b".", ref, alt, b"50", b"PASS", info]))
    return b"\n".join(out) + b"\n"


def whole_file_tabix(contigs, bgzf_len):
    """A decompressed tabix index whose only bin (0) holds one chunk over the whole file, for
    every contig: index pruning keeps every split, the line filter decides."""
    import struct
    names = b"".join(c.encode() + b"\x00" for c in contigs)
    d = b"TBI\x01" + struct.pack("<iiiiiiii", len(contigs), 2, 1, 2, 0, ord("#"), 0, len(names)) + names
    for _ in contigs:
        d += struct.pack("<i", 1) + struct.pack("<Ii", 0, 1) + struct.pack("<QQ", 0, bgzf_len << 16)
        d += struct.pack("<i", 0)
    return d
