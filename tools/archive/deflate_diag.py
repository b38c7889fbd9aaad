"""Dev tool: decode one GPU-compressed BGZF member symbol by symbol (a small Python inflater) and
report where its output departs from the input -- the symbols around the first wrong byte and the
parse lanes (255 bytes each) they fall in.  usage: DQ_DEFLATE=... python3 tools/deflate_diag.py"""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Bits:
    def __init__(self, b):
        self.b, self.p = b, 0

    def get(self, n):
        v = 0
        for i in range(n):
            v |= ((self.b[(self.p + i) >> 3] >> ((self.p + i) & 7)) & 1) << i
        self.p += n
        return v


def table(lens):
    bl = [0] * 16
    for l in lens:
        if l:
            bl[l] += 1
    code, nxt = 0, [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    t = {}
    for s, l in enumerate(lens):
        if l:
            t[(nxt[l], l)] = s
            nxt[l] += 1
    return t


def sym(r, t):
    c, n = 0, 0
    while (c, n) not in t:
        c, n = (c << 1) | r.get(1), n + 1
        if n > 15:
            raise ValueError("bad code at bit %d" % r.p)
    return t[(c, n)]


LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LE = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DB = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577]
DE = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]


def inflate_symbols(body):
    r = Bits(body)
    out, syms = bytearray(), []
    while True:
        final, bt = r.get(1), r.get(2)
        if bt == 0:
            raise NotImplementedError("stored")
        if bt == 1:
            ll = table([8] * 144 + [9] * 112 + [7] * 24 + [8] * 8)
            dd = table([5] * 32)
        else:
            hlit, hdist, hclen = r.get(5) + 257, r.get(5) + 1, r.get(4) + 4
            cl = [0] * 19
            for i in range(hclen):
                cl[[16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15][i]] = r.get(3)
            ct = table(cl)
            lens = []
            while len(lens) < hlit + hdist:
                s = sym(r, ct)
                if s < 16:
                    lens.append(s)
                elif s == 16:
                    lens += [lens[-1]] * (3 + r.get(2))
                elif s == 17:
                    lens += [0] * (3 + r.get(3))
                else:
                    lens += [0] * (11 + r.get(7))
            ll, dd = table(lens[:hlit]), table(lens[hlit:])
        while True:
            s = sym(r, ll)
            if s < 256:
                syms.append((len(out), "lit", 1, 0))
                out.append(s)
            elif s == 256:
                break
            else:
                k = s - 257
                ln = LB[k] + r.get(LE[k])
                ds = sym(r, dd)
                d = DB[ds] + r.get(DE[ds])
                syms.append((len(out), "match", ln, d))
                for _ in range(ln):
                    out.append(out[-d])
        if final:
            return bytes(out), syms


def main():
    from disq_amd import _lib
    rng = np.random.default_rng(1)
    for n in (1, 2, 3, 257):
        rng.integers(0, 4, size=n, dtype=np.uint8)
    data = rng.integers(0, 4, size=4096, dtype=np.uint8).tobytes()
    with _lib.Context() as c:
        z = c.bgzf_compress(data)
    cs = struct.unpack_from("<H", z, 16)[0] + 1
    out, syms = inflate_symbols(z[18:cs - 8])
    print("in", len(data), "out", len(out), "symbols", len(syms))
    bad = next((i for i in range(min(len(out), len(data))) if out[i] != data[i]), min(len(out), len(data)))
    print("first difference at", bad, "lane", bad // 255)
    for k, (p, kind, ln, d) in enumerate(syms):
        if bad - 300 <= p <= bad + 20:
            ok = out[p:p + ln] == data[p:p + ln]
            src_ok = data[p:p + ln] == bytes(data[p - d + (i % d)] for i in range(ln)) if kind == "match" else True
            print(k, p, "lane", p // 255, kind, ln, d, "ok" if ok else "BAD", "validmatch" if src_ok else "INVALID")


if __name__ == "__main__":
    main()
