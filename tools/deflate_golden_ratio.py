"""Dev tool: the write path's compressed size against zlib level 5 (htsjdk's BGZF) on the golden BAM
/ VCF streams and the synthetic WGS stream, at the DQ_DEFLATE setting of the environment.

  DQ_DEFLATE=16,16,32,4,1 python tools/deflate_golden_ratio.py
"""
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from disq_amd import _lib, synth  # noqa: E402
import bamutil as B  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def zlib5(data):
    t = 0
    for i in range(0, len(data), B.BLOCK_U):
        z = zlib.compressobj(5, zlib.DEFLATED, -15)
        t += len(z.compress(data[i:i + B.BLOCK_U]) + z.flush()) + 26
    return t


for name in ["1.bam", "hiseq_part-r-00000.bam", "HiSeq.10000.vcf.bgz", "wgs"]:
    if name == "wgs":
        u = B.inflate_all(synth.generate(60000, seed=5, nthreads=8).bam)
    else:
        u = B.inflate_all(open(os.path.join(GOLDEN, name), "rb").read())
    with _lib.Context() as c:
        z = c.bgzf_compress(u)
    ref = zlib5(u)
    print(f"{os.environ.get('DQ_DEFLATE', 'default'):14s} {name:26s} size/zlib5 {len(z) / ref:.4f}  ratio {len(u) / len(z):.3f}"
          f" (zlib5 {len(u) / ref:.3f})", flush=True)
