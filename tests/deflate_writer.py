"""Test helper: a bit-exact raw-DEFLATE writer (RFC 1951) for hand-built BGZF members.

zlib decides its own block boundaries, bit counts and distances; the directed inflate tests need
them in exact places (a deflate block ending on a given bit, a tail of exactly 4096 output bytes, a
match at distance 32768).  This writer encodes explicit token lists -- a literal byte (int) or a
(length, distance) pair -- as stored, fixed-Huffman or dynamic-Huffman blocks and reports the bit
position of every block it wrote.  Test infrastructure only; every stream it makes is checked
against zlib.decompress by the tests that use it."""
import heapq
import struct
import zlib

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
         131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537,
         2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]
CL_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
FIXED_LL = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
FIXED_D = [5] * 30
BGZF_HDR = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"


def len_sym(n):
    s = max(i for i in range(29) if LBASE[i] <= n)
    if n == 258:
        s = 28
    return s, LEXT[s], n - LBASE[s]


def dist_sym(d):
    s = max(i for i in range(30) if DBASE[i] <= d)
    return s, DEXT[s], d - DBASE[s]


def canonical(lens):
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


def limited_lengths(freqs, limit):
    """Complete Huffman code lengths (Kraft sum exactly 1, at least two codes) of at most `limit`
    bits for the symbols with nonzero frequency."""
    freqs = list(freqs)
    used = [i for i, f in enumerate(freqs) if f > 0]
    for s in range(len(freqs)):
        if len(used) >= 2:
            break
        if freqs[s] == 0:
            freqs[s] = 1
            used.append(s)
    heap = [(freqs[s], i, [s]) for i, s in enumerate(used)]
    heapq.heapify(heap)
    depth = {s: 0 for s in used}
    k = len(heap)
    while len(heap) > 1:
        f1, _, a = heapq.heappop(heap)
        f2, _, b = heapq.heappop(heap)
        for s in a + b:
            depth[s] += 1
        heapq.heappush(heap, (f1 + f2, k, a + b))
        k += 1
    lens = [0] * len(freqs)
    for s in used:
        lens[s] = min(depth[s], limit)
    cap = 1 << limit
    kraft = sum(1 << (limit - lens[s]) for s in used)
    order = sorted(used, key=lambda s: (freqs[s], s))  # rarest first
    while kraft > cap:  # lengthen the rarest code that can still grow
        s = next(s for s in order if lens[s] < limit)
        kraft -= 1 << (limit - lens[s] - 1)
        lens[s] += 1
    while kraft < cap:  # shorten the longest code whose shortening still fits
        s = max((s for s in used if lens[s] > 1 and kraft + (1 << (limit - lens[s])) <= cap),
                key=lambda s: (lens[s], -freqs[s]))
        kraft += 1 << (limit - lens[s])
        lens[s] -= 1
    return lens


class BitWriter:
    def __init__(self):
        self.v, self.n = 0, 0

    def bits(self, x, n):  # LSB first
        self.v |= (x & ((1 << n) - 1)) << self.n
        self.n += n

    def code(self, c, n):  # Huffman codes go MSB first
        self.bits(int(format(c, "0%db" % n)[::-1], 2), n)

    def align(self):
        self.n = (self.n + 7) & ~7

    def bytes(self):
        return self.v.to_bytes((self.n + 7) // 8, "little")


def lz77(data, start=0, end=None, max_chain=16, max_len=258):
    """Greedy LZ77 tokens of data[start:end] with the 32 KiB window over all of data[:end]."""
    end = len(data) if end is None else end
    heads = {}
    for p in range(max(0, start - 32768), start):
        heads.setdefault(data[p:p + 3], []).append(p)
    toks, i = [], start
    while i < end:
        best, bd = 0, 0
        if i + 3 <= end:
            for p in reversed(heads.get(data[i:i + 3], [])[-max_chain:]):
                if i - p > 32768:
                    break
                n = 0
                while n < max_len and i + n < end and data[p + n] == data[i + n]:
                    n += 1
                if n > best:
                    best, bd = n, i - p
        step = best if best >= 3 else 1
        for q in range(i, i + step):
            if q + 3 <= end:
                heads.setdefault(data[q:q + 3], []).append(q)
        toks.append((best, bd) if best >= 3 else data[i])
        i += step
    return toks


def token_bytes(toks):
    return sum(t[0] if isinstance(t, tuple) else 1 for t in toks)


class Deflater:
    """Appends deflate blocks to one raw-DEFLATE stream; `starts` lists each block's bit offset."""

    def __init__(self):
        self.w = BitWriter()
        self.starts = []

    @property
    def pos(self):
        return self.w.n

    def stored(self, data, final=False):
        self.starts.append(self.w.n)
        self.w.bits(int(final), 1)
        self.w.bits(0, 2)
        self.w.align()
        self.w.bits(len(data), 16)
        self.w.bits(len(data) ^ 0xffff, 16)
        for b in data:
            self.w.bits(b, 8)

    def _symbols(self, toks, llc, ll_lens, dc, d_lens, extra=()):
        w = self.w
        for t in toks:
            if isinstance(t, tuple):
                n, d = t
                s, nb, v = len_sym(n)
                w.code(llc[257 + s], ll_lens[257 + s])
                w.bits(v, nb)
                s, nb, v = dist_sym(d)
                w.code(dc[s], d_lens[s])
                w.bits(v, nb)
            else:
                w.code(llc[t], ll_lens[t])
        for s in extra:  # raw symbols (e.g. an invalid 286 for a corrupt-code fixture)
            w.code(llc[s], ll_lens[s])
        w.code(llc[256], ll_lens[256])

    def fixed(self, toks, final=False, extra=()):
        self.starts.append(self.w.n)
        self.w.bits(int(final), 1)
        self.w.bits(1, 2)
        self._symbols(toks, canonical(FIXED_LL), FIXED_LL, canonical(FIXED_D), FIXED_D, extra)

    def dynamic_lengths(self, toks):
        """The (litlen, distance) code lengths dynamic() uses for `toks` (every literal gets a
        code, so padding literals can be appended with the same tables)."""
        lf, df = [1] * 256 + [1] + [0] * 29, [0] * 30
        for t in toks:
            if isinstance(t, tuple):
                lf[257 + len_sym(t[0])[0]] += 1
                df[dist_sym(t[1])[0]] += 1
            else:
                lf[t] += 1
        if not any(df):
            df[0] = 1
        return limited_lengths(lf, 15), limited_lengths(df, 15)

    def dynamic(self, toks, final=False, lens=None):
        ll, dl = lens if lens is not None else self.dynamic_lengths(toks)
        hlit = max(257, max(i for i, x in enumerate(ll) if x) + 1)
        hdist = max(1, max((i for i, x in enumerate(dl) if x), default=0) + 1)
        seq = ll[:hlit] + dl[:hdist]
        cf = [0] * 19
        for x in seq:
            cf[x] += 1
        cl = limited_lengths(cf, 7)
        hclen = max(4, max(i for i, s in enumerate(CL_ORDER) if cl[s]) + 1)
        self.starts.append(self.w.n)
        w = self.w
        w.bits(int(final), 1)
        w.bits(2, 2)
        w.bits(hlit - 257, 5)
        w.bits(hdist - 1, 5)
        w.bits(hclen - 4, 4)
        for s in CL_ORDER[:hclen]:
            w.bits(cl[s], 3)
        clc = canonical(cl)
        for x in seq:
            w.code(clc[x], cl[x])
        self._symbols(toks, canonical(ll + [0] * (288 - len(ll))), ll + [0] * (288 - len(ll)),
                      canonical(dl), dl)

    def finish(self):
        return self.w.bytes()


def expand(toks, history=b""):
    """The bytes `toks` produce after `history` (a check of the token lists themselves); a
    distance past the start (an invalid stream's) copies zeros."""
    out = bytearray(history)
    for t in toks:
        if isinstance(t, tuple):
            n, d = t
            for _ in range(n):
                out.append(out[-d] if d <= len(out) else 0)
        else:
            out.append(t)
    return bytes(out[len(history):])


def member(deflated, data, crc=None, isize=None):
    """A BGZF member (htsjdk layout: 'BC' extra field, BSIZE = length - 1) of a raw-DEFLATE body."""
    m = BGZF_HDR + struct.pack("<H", 18 + len(deflated) + 8 - 1) + deflated
    c = zlib.crc32(data) & 0xffffffff if crc is None else crc
    return m + struct.pack("<II", c, len(data) if isize is None else isize)
