import struct, zlib, sys
import numpy as np
sys.path.insert(0, '/root/repo/tests')
import deflate_writer as W

class BR:
    def __init__(s, b): s.b, s.p = b, 0
    def get(s, n):
        v = 0
        for i in range(n):
            v |= ((s.b[(s.p + i) >> 3] >> ((s.p + i) & 7)) & 1) << i
        s.p += n
        return v

def build(lens):
    cnt = [0]*16
    for l in lens:
        if l: cnt[l] += 1
    code = 0; nxt = [0]*16
    for b in range(1, 16):
        code = (code + cnt[b-1]) << 1; nxt[b] = code
    tab = {}
    for s_, l in enumerate(lens):
        if l:
            tab[(nxt[l], l)] = s_; nxt[l] += 1
    return tab

def dec(r, tab):
    c = n = 0
    while True:
        c = (c << 1) | r.get(1); n += 1
        if (c, n) in tab: return tab[(c, n)]
        if n > 15: raise ValueError

def tokenize(body):
    r = BR(body); toks = []; blocks = []; pos = 0
    while True:
        start = r.p
        last = r.get(1); t = r.get(2)
        blocks.append((start, pos))
        if t == 0:
            r.p = (r.p + 7) & ~7; ln = r.get(16); r.get(16)
            for _ in range(ln): toks.append(r.get(8)); pos += 1
        else:
            if t == 1:
                ll = W.FIXED_LL; dl = [5]*30
            else:
                hl = r.get(5) + 257; hd = r.get(5) + 1; hc = r.get(4) + 4
                cl = [0]*19
                for i in range(hc): cl[W.CL_ORDER[i]] = r.get(3)
                ct = build(cl); lens = []
                while len(lens) < hl + hd:
                    s_ = dec(r, ct)
                    if s_ < 16: lens.append(s_)
                    elif s_ == 16: lens += [lens[-1]] * (3 + r.get(2))
                    elif s_ == 17: lens += [0] * (3 + r.get(3))
                    else: lens += [0] * (11 + r.get(7))
                ll = lens[:hl] + [0]*(288-hl); dl = lens[hl:]
            lt = build(ll); dt = build(dl)
            while True:
                s_ = dec(r, lt)
                if s_ < 256: toks.append(s_); pos += 1
                elif s_ == 256: break
                else:
                    s_ -= 257; L = W.LBASE[s_] + r.get(W.LEXT[s_]); d = dec(r, dt)
                    D = W.DBASE[d] + r.get(W.DEXT[d]); toks.append((L, D)); pos += L
        if last: break
    return toks, blocks, r.p

def members(bam):
    p = 0; out = []
    while p < len(bam):
        bs = struct.unpack_from('<H', bam, p + 16)[0]; cs = bs + 1
        isize = struct.unpack_from('<I', bam, p + cs - 4)[0]
        out.append((p, cs, isize, bam[p + 18:p + cs - 8])); p += cs
    return out

def emulate_tail(toks, p0, isize, ub, prefix_bytes):
    """The kernel's tail resolve on the tail tokens; returns the tail bytes."""
    sh = (ub + p0) & 15
    n = isize - p0
    out = bytearray(4096 + 32 + 512)
    bm = np.zeros(4096 // 32 + 1, np.uint32)
    k = 0
    for t in toks:
        if k >= n: break
        if isinstance(t, tuple):
            L, D = t
            desc = (D - 1) | ((L - 3) << 15)
            out[sh + k] = desc & 255; out[sh + k + 1] = (desc >> 8) & 255; out[sh + k + 2] = (desc >> 16) & 255
            bm[k >> 5] |= np.uint32(1 << (k & 31))
            k += L
        else:
            out[sh + k] = t; k += 1
    def load_desc(a):
        return out[a] | out[a+1] << 8 | out[a+2] << 16
    nrows = (sh + n + 255) >> 8
    carry = [-1, 0]
    def hops(row):
        cms, cdesc = carry
        res = []
        lsts = []
        b4s = []
        for lane in range(64):
            x0 = 256 * row + 4 * lane - sh
            nval = min(max(n - x0, 0), 4)
            b4 = 0
            if nval > 0:
                if x0 >= 0:
                    wi = x0 >> 5
                    lo = int(bm[wi]); hi = int(bm[min(wi + 1, 4096 // 32 - 1)])
                    b4 = ((hi << 32 | lo) >> (x0 & 31)) & 0xffffffff
                elif x0 > -4:
                    b4 = (int(bm[0]) << (-x0)) & 0xffffffff
                b4 &= (1 << nval) - 1
            b4s.append(b4)
            lsts.append(x0 + b4.bit_length() - 1 if b4 else -1)
        incl = np.maximum.accumulate(np.array(lsts))
        for lane in range(64):
            x0 = 256 * row + 4 * lane - sh
            nval = min(max(n - x0, 0), 4)
            b4 = b4s[lane]
            pre = -1 if lane == 0 else int(incl[lane - 1])
            o0 = x0 if (b4 & 1) else max(pre, cms)
            r1 = b4 & ~1
            p1 = x0 + ((r1 & -r1).bit_length() - 1) if r1 else -1
            d0 = 0 if o0 < 0 else (cdesc if o0 == cms else load_desc(sh + o0))
            d1 = 0 if p1 < 0 else load_desc(sh + p1)
            src = []; cpy = 0
            for i in range(4):
                x = x0 + i
                at1 = p1 >= 0 and x >= p1
                ms = p1 if at1 else o0
                ds = d1 if at1 else d0
                ln = (ds >> 15) + 3; D = (ds & 0x7fff) + 1
                copy = ms >= 0 and i < nval and x >= 0 and x < ms + ln
                jj = x - ms
                rm = jj % D if jj >= D else jj
                src.append(ms - D + rm)
                cpy |= (1 << i) if copy else 0
            res.append((src, cpy))
        last = max(int(incl[63]), cms)
        if last != cms:
            carry[1] = load_desc(sh + last); carry[0] = last
        return res
    TERM = 0x8000
    allh = [hops(r) for r in range(nrows)]  # in order (the carry)
    for row in range(nrows):
        H = allh[row]
        xr = 256 * row - sh
        nx = [0] * 256
        P = []; PEND = []
        for lane in range(64):
            Y = 256 * row + 4 * lane; x0 = Y - sh
            src, cpy = H[lane]
            live = Y < sh + n
            own = out[Y:Y+4]
            p = []; pend = 0
            for i in range(4):
                c = (cpy >> i) & 1; pre = c and src[i] < 0
                if pre:
                    own[i] = prefix_bytes[p0 + src[i]]
                p.append(((x0 + i) & 0xffffffff) | TERM if (not c or pre) else src[i])
                if c and not pre and src[i] >= xr: pend |= 1 << i
            if live: out[Y:Y+4] = own
            P.append(p); PEND.append(pend)
        def publish():
            for lane in range(64):
                for i in range(4): nx[4 * lane + i] = P[lane][i] & 0xffff
        publish()
        rnd = 0
        while any(PEND) and rnd < 10:
            Q = []
            for lane in range(64):
                q = []
                for i in range(4):
                    pd = (PEND[lane] >> i) & 1
                    q.append(nx[P[lane][i] - xr if pd else 4 * lane + i])
                Q.append(q)
            for lane in range(64):
                for i in range(4):
                    pd = (PEND[lane] >> i) & 1
                    if not pd: continue
                    q = Q[lane][i]
                    P[lane][i] = q
                    if (q & TERM) or q < xr: PEND[lane] &= ~(1 << i)
            publish(); rnd += 1
        if any(PEND): print("row", row, "unresolved after 10 rounds")
        V = []
        for lane in range(64):  # lock-step: every lane reads before any lane writes
            Y = 256 * row + 4 * lane
            src, cpy = H[lane]
            v = out[Y:Y+4]
            for i in range(4):
                c = (cpy >> i) & 1
                s_ = P[lane][i] & ~TERM
                if not (not c or src[i] < 0):
                    v[i] = out[sh + s_]
            V.append(v)
        for lane in range(64):
            Y = 256 * row + 4 * lane
            if Y < sh + n: out[Y:Y+4] = V[lane]
    return bytes(out[sh:sh + n])

def check(bam, verbose=True):
    ub = 0; bad = 0
    for (p, cs, isize, body) in members(bam):
        if isize == 0: continue
        data = zlib.decompress(body, -15)
        toks, blocks, endp = tokenize(body)
        if len(blocks) >= 2:
            pos = blocks[1][0]; produced = blocks[1][1]
            endbits = 8 * len(body)
            if isize - produced <= 4096 and endbits - pos <= 32768 and produced < isize:
                # tail tokens: from the token producing byte `produced`
                k = 0; ti = 0
                while k < produced:
                    t = toks[ti]; k += t[0] if isinstance(t, tuple) else 1; ti += 1
                got = emulate_tail(toks[ti:], produced, isize, ub, data)
                ok = got == data[produced:]
                if not ok:
                    bad += 1
                    first = next(i for i in range(len(got)) if got[i] != data[produced + i])
                    if verbose: print("member at", p, "tail", produced, isize, "MISMATCH at tail byte", first, "sh", (ub + produced) & 15)
        ub += isize
    return bad

if __name__ == "__main__":
    bam = open(sys.argv[1], 'rb').read()
    print("bad tails:", check(bam))
