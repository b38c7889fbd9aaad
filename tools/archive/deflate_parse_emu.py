"""Dev tool (CPU): a line-by-line Python emulation of bgzf_parse_kernel's chunk logic
(disq_amd/csrc/dq_deflate.hip) at reduced sizes -- hash buckets with the ordered scatter, the
16-way slot search, lazy parse steps, lane continuations with forced merges, pointer jumping over
the merges -- checking that the chunks' effective symbols rebuild the block exactly.

  python tools/deflate_parse_emu.py [--blocks 20] [--seed 1]

Sizes are scaled down (chunk 2040 bytes, 8-byte segments, 1024 bytes of reach) so the logic paths
(many segments, merges, overruns, forced merges) run in seconds; the kernel's are 32640 / 32 /
13600.  It models the merge rule (segments' own parses, continuations until a later segment's
symbol boundary, forced merges, pointer jumping); the kernel's staging (matches only, with literal
gaps; dense per-chunk areas) and its run-time segment claims are not modelled.
"""
import argparse
import random

MAXM, WIN, HBITS = 258, 32768, 11


def hash3(b, x):
    v = b[x] | b[x + 1] << 8 | b[x + 2] << 16
    return ((v * 2654435761) & 0xffffffff) >> (32 - HBITS)


class Chunk:
    def __init__(self, blk, cs, ch, xw, pseg, nlanes, chain, lazy, nice, good, own, cont, rng=None,
                 flow=0.0):
        self.rng, self.flow = rng, flow
        ce = min(len(blk), cs + ch)
        self.r0 = max(0, cs - xw)
        self.inb = bytes(blk[self.r0:ce]) + bytes(16)
        self.np = ce - self.r0
        self.xs = cs - self.r0
        self.pseg, self.nl = pseg, nlanes
        self.chain, self.lazy, self.nice, self.good = chain, lazy, nice, good
        self.own, self.cont = own, cont
        npos = max(0, self.np - 2)
        # counts, scan, ordered scatter (per-bucket ascending)
        head = [0] * (1 << HBITS)
        for x in range(npos):
            head[hash3(self.inb, x)] += 1
        cur, off = [0] * (1 << HBITS), 0
        for h in range(1 << HBITS):
            cur[h] = off
            off += head[h]
        self.bl = [0] * max(1, npos)
        for x in range(npos):  # the kernel's waves walk positions in order: the same result
            h = hash3(self.inb, x)
            self.bl[cur[h]] = x
            cur[h] += 1
        self.end = cur  # bucket ends

    def slot(self, lo, hi, x):
        a, b = lo, hi
        while b - a > 16:
            st = (b - a) >> 4
            m = sum(1 for k in range(1, 16) if self.bl[a + k * st] <= x)
            na = a + m * st
            b = b if m == 15 else na + st
            a = na
        return a + sum(1 for k in range(16) if a + k < b and self.bl[a + k] < x)

    def find(self, x, lim, ch):
        if lim < 3 or x + 3 > self.np:
            return 0, 0
        h = hash3(self.inb, x)
        blo = self.end[h - 1] if h else 0
        g = self.slot(blo, self.end[h], x)
        assert self.bl[g] == x
        lo = max(blo, g - ch)
        best, bd, cap = 0, 0, min(lim, self.nice)
        i = g - 1
        while i >= lo and best < cap:
            q = self.bl[i]
            if x - q > WIN:
                break
            l = 0
            while l < cap and self.inb[q + l] == self.inb[x + l]:
                l += 1
            if l > best:
                best, bd = l, x - q
            i -= 1
        if best >= cap and cap < lim:
            l = cap
            while l < lim and self.inb[x - bd + l] == self.inb[x + l]:
                l += 1
            best = l
        return (best, bd) if best >= 3 else (0, 0)

    def step(self, x, w, cap):
        n = self.np
        l, d = self.find(x, min(MAXM, n - x), self.chain)
        while l and l < self.lazy and x + 1 < n:
            ch = max(1, self.chain >> 2) if self.good > 0 and l >= self.good else self.chain
            l2, d2 = self.find(x + 1, min(MAXM, n - x - 1), ch)
            if l2 <= l:
                break
            assert len(w) < cap
            w.append(("L", self.inb[x]))
            x, l, d = x + 1, l2, d2
        assert len(w) < cap
        if l:
            w.append(("M", l, d))
            return x + l
        w.append(("L", self.inb[x]))
        return x + 1

    def run(self):
        np_, xs, P = self.np, self.xs, self.pseg
        nlc = (np_ - xs + P - 1) // P
        own, ex, begin = [], [], []
        for t in range(nlc):
            s0 = min(np_, xs + P * t)
            s1 = min(np_, s0 + P)
            # an odd segment is flowed into from its even predecessor's exit (the kernel's usual
            # case) or, when the predecessor's lane was late, started at its own start
            x = s0
            if t % 2 == 1 and self.rng.random() < self.flow:
                x = ex[t - 1]
            begin.append(x)
            w = []
            while x < s1:
                x = self.step(x, w, self.own)
            own.append(w)
            ex.append(x)
        # symbol starts of each lane's own parse (the kernel's sbits words)
        starts = []
        for t in range(nlc):
            s0, sb, x = xs + P * t, set(), begin[t]
            for sy in own[t]:
                if x < s0 + P:  # a deferred literal past the segment end is not recorded
                    sb.add(x)
                x += 1 if sy[0] == "L" else sy[1]
            assert x == ex[t]
            starts.append(sb)
        mrg, conts, forced = [], [], 0
        for t in range(nlc):
            E, u, k, cw, over = ex[t], t + 1, 0, [], False
            while True:
                if E >= np_:
                    u, k = None, 0
                    break
                if u >= nlc:
                    if len(cw) > self.cont - 40:
                        over = True
                        break
                    E = self.step(E, cw, self.cont)
                    continue
                su, eu = xs + P * u, ex[u]
                if E > eu:
                    u += 1
                    continue
                if E == eu:
                    k = len(own[u])
                    break
                if E < su + P and E in starts[u]:
                    k = sum(1 for q in starts[u] if q < E)
                    break
                if len(cw) > self.cont - 40:
                    forced += 1
                    nxt = [q for q in starts[u] if q > E] if E < su + P else []
                    pu = min(nxt) if nxt else eu
                    while E < pu and len(cw) < self.cont:
                        l, d = self.find(E, min(MAXM, pu - E), self.chain)
                        cw.append(("M", l, d) if l else ("L", self.inb[E]))
                        E += l if l else 1
                    if E != pu:
                        over = True
                        break
                    k = len(own[u]) if pu == eu else sum(1 for q in starts[u] if q < pu)
                    break
                E = self.step(E, cw, self.cont)
            mrg.append((None if over else u, k, over))
            conts.append(cw)
        # pointer jumping from lane 0 (the kernel's rounds), then first symbols
        jmp = [m[0] if m[0] is not None else None for m in mrg]
        mark = [t == 0 for t in range(nlc)]
        r = 0
        while (1 << r) < nlc:
            marks = list(mark)
            for t in range(nlc):
                if jmp[t] is not None and mark[t]:
                    marks[jmp[t]] = True
            mark = marks
            jmp = [jmp[jmp[t]] if jmp[t] is not None else None for t in range(nlc)]
            r += 1
        k0 = [0] * nlc
        for t in range(nlc):
            if mark[t] and mrg[t][0] is not None:
                k0[mrg[t][0]] = mrg[t][1]
            if mark[t]:
                assert not mrg[t][2], "overflow on the parse: the block would be stored"
        syms = []
        for t in range(nlc):
            if mark[t]:
                syms += own[t][k0[t]:] + conts[t]
        # the serial walk gives the same lanes
        cur, seen = 0, []
        while cur is not None:
            seen.append(cur)
            cur = mrg[cur][0]
        assert seen == [t for t in range(nlc) if mark[t]], (seen, mark)
        return syms, forced


def decode(syms, out):
    for s in syms:
        if s[0] == "L":
            out.append(s[1])
        else:
            _, l, d = s
            assert 1 <= d <= min(len(out), WIN) and 3 <= l <= MAXM
            for _ in range(l):
                out.append(out[-d])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cont", type=int, default=104, help="continuation staging (forced merges past cont - 40)")
    ap.add_argument("--flow", type=float, default=0.8, help="share of odd segments flowed into")
    a = ap.parse_args()
    rng = random.Random(a.seed)
    CH, NCH, XW, PSEG = 2040, 2, 1024, 8
    tot_forced = 0
    for i in range(a.blocks):
        n = rng.choice([1, 2, 3, 5, 100, CH - 1, CH, CH + 1, CH + 3, 2 * CH - 1, 2 * CH,
                        rng.randint(1, 2 * CH)])
        kind = i % 4
        if kind == 0:
            blk = bytes(rng.randrange(4) for _ in range(n))
        elif kind == 1:
            blk = bytes(rng.randrange(256) for _ in range(n))
        elif kind == 2:
            pat = bytes(rng.randrange(256) for _ in range(rng.randint(1, 9)))
            blk = (pat * (n // len(pat) + 1))[:n]
        else:
            words = [bytes(rng.randrange(97, 123) for _ in range(rng.randint(3, 12))) for _ in range(20)]
            blk = b"".join(rng.choice(words) for _ in range(n))[:n]
        cfg = rng.choice([(96, 32, 96, 8), (128, 32, 258, 0), (8, 4, 16, 2)])
        out = bytearray()
        for c in range(NCH):
            if c * CH >= n:
                continue
            ck = Chunk(blk, c * CH, CH, XW, PSEG, CH // PSEG, *cfg, own=8 + 33 + 3, cont=a.cont,
                       rng=rng, flow=a.flow)
            syms, forced = ck.run()
            tot_forced += forced
            decode(syms, out)
        assert bytes(out) == blk, (i, n, kind)
    print(f"{a.blocks} blocks: every chunk's parse rebuilds its bytes ({tot_forced} forced merges)")


if __name__ == "__main__":
    main()
