import sys, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests'); sys.path.insert(0, '/root/repo/tools')
import numpy as np, zlib
import tail_emu as T
from disq_amd import _lib
bam = open('/root/repo/tests/golden/hiseq_part-r-00000.bam', 'rb').read()
with _lib.Context(split_size=0, verify_crc=False, device=0) as c:
    c.text_open_bytes(bam)
    c.text_run(drop_header_lines=False)
    got = c.inflated().tobytes()
ub = 0
for (p, cs, isize, body) in T.members(bam):
    if isize == 0: continue
    data = zlib.decompress(body, -15)
    g = got[ub:ub + isize]
    toks, blocks, _ = T.tokenize(body)
    prod = blocks[1][1] if len(blocks) > 1 else None
    if g != data:
        d = [i for i in range(isize) if g[i] != data[i]]
        print("member", p, "isize", isize, "tail start", prod, "sh", (ub + (prod or 0)) & 15, "ndiff", len(d), "first", d[:8], "last", d[-3:])
        if prod is not None:
            rel = [i - prod for i in d[:16]]
            print("   tail-relative", rel, "row/lane of first", [((i + ((ub + prod) & 15)) // 256, ((i + ((ub + prod) & 15)) % 256) // 4) for i in rel[:6]])
    ub += isize
print("done")
