"""BGZF text (VCF) read path benchmark: a synthetic VCF compressed
htsjdk-style (zlib level 5, 65280-byte BGZF blocks), read by the GPU text path (dq_text_run: scan,
chain, inflate + CRC32, line terminators, Hadoop LineRecordReader split planning, per-line values,
hashes, '#' filter, partition digests) against the oracle's restatement of Disq's
VcfSource.getVariants (BGZFCodec + LineRecordReader per split, VcfSource.java:88-113).

  python tools/vcf_bench.py [--mb 4096] [--samples 0] [--split 33554432] [--steps 5] > out.json

Shapes: --samples 0 writes sites-only lines (8 columns, ~200 B); --samples N adds FORMAT and N
genotype columns (~20 B each).  Reports decompressed GB/s over the device time of dq_text_run
(HIP events), lines/s, the CPU baseline (the oracle's split reader over a bounded sample of the
same splits, one split per thread) and parity: every partition's line offsets and lengths equal
the oracle's.  Synthetic data: no network for real VCFs."""
import argparse
import json
import os
import struct
import sys
import time
import zlib
from concurrent.futures import ThreadPoolExecutor
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BLOCK_U = 65280  # htsjdk DEFAULT_UNCOMPRESSED_BLOCK_SIZE
EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
CONTIGS = [("chr%d" % i, 250_000_000 - 8_000_000 * i) for i in range(1, 23)] + [("chrX", 156_040_895)]


def _bgzf_member(chunk: bytes) -> bytes:
    c = zlib.compressobj(5, zlib.DEFLATED, -15, 8)
    body = c.compress(chunk) + c.flush()
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
    return (hdr + struct.pack("<H", 18 + len(body) + 8 - 1) + body +
            struct.pack("<II", zlib.crc32(chunk) & 0xffffffff, len(chunk)))


def _lines(seed: int, n: int, samples: int, chrom: str, pos0: int) -> bytes:
    rng = np.random.default_rng(seed)
    pos = pos0 + np.cumsum(rng.integers(1, 400, n))
    bases = np.array(list("ACGT"))
    ref = bases[rng.integers(0, 4, n)]
    alt = bases[(rng.integers(1, 4, n) + np.searchsorted(bases, ref)) % 4]
    qual = rng.integers(20, 5000, n) / 10.0
    ac = rng.integers(1, 2 * max(samples, 1) + 1, n)
    dp = rng.integers(10, 4000, n)
    rs = rng.integers(1, 900_000_000, n)
    has_rs = rng.random(n) < 0.6
    if samples:
        pool = ["%s:%d,%d:%d:%d" % (g, a, b, a + b, q) for g in ("0/0", "0/1", "1/1", "0|1", "1|0", "./.")
                for a in (0, 3, 11, 25) for b in (0, 2, 9, 30) for q in (3, 42, 99)]
        pick = rng.integers(0, len(pool), (n, samples))
    out = []
    for i in range(n):
        s = "%s\t%d\t%s\t%s\t%s\t%.1f\tPASS\tAC=%d;AF=%.4f;AN=%d;DP=%d;FS=%.3f;MQ=%.2f;QD=%.2f;SOR=%.3f" % (
            chrom, pos[i], ("rs%d" % rs[i]) if has_rs[i] else ".", ref[i], alt[i], qual[i], ac[i],
            ac[i] / (2.0 * max(samples, 1)), 2 * max(samples, 1), dp[i], (dp[i] % 97) / 7.0,
            60.0 - (dp[i] % 13) / 3.0, qual[i] / max(dp[i], 1), (dp[i] % 31) / 10.0)
        if samples:
            s += "\tGT:AD:DP:GQ\t" + "\t".join(pool[j] for j in pick[i])
        out.append(s)
    return ("\n".join(out) + "\n").encode()


def _chunk_job(args):
    seed, n, samples, chrom, pos0 = args
    return _lines(seed, n, samples, chrom, pos0)


_TEXT = b""  # the text being compressed: inherited by the forked workers, not pickled per task


def _compress_job(args):
    lo, hi = args
    return b"".join(_bgzf_member(_TEXT[a:min(a + BLOCK_U, hi)]) for a in range(lo, hi, BLOCK_U))


def make_vcf(mb: int, samples: int, procs: int):
    header = ["##fileformat=VCFv4.2", '##FILTER=<ID=PASS,Description="All filters passed">']
    header += ["##contig=<ID=%s,length=%d>" % c for c in CONTIGS]
    header += ['##INFO=<ID=%s,Number=1,Type=Float,Description="%s">' % (k, k)
               for k in ("AC", "AF", "AN", "DP", "FS", "MQ", "QD", "SOR")]
    cols = "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO"
    if samples:
        header.append('##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">')
        cols += "\tFORMAT\t" + "\t".join("S%04d" % i for i in range(samples))
    head = ("\n".join(header + [cols]) + "\n").encode()
    per_line = 103 + 14 * samples  # measured: 102.7 B sites-only, 2.94 KB at 200 samples
    n_lines = max(1, mb * 1_000_000 // per_line)
    per_job = 20000
    jobs = [(1000 + k, min(per_job, n_lines - k * per_job), samples,
             CONTIGS[(k * len(CONTIGS)) * per_job // n_lines][0], 10_000 + k * 7_000_000)
            for k in range((n_lines + per_job - 1) // per_job)]
    global _TEXT
    with Pool(procs) as p:
        text = head + b"".join(p.map(_chunk_job, jobs))
    _TEXT = text
    step = BLOCK_U * 64
    with Pool(procs) as p:
        parts = p.map(_compress_job, [(a, min(a + step, len(text))) for a in range(0, len(text), step)])
    _TEXT = b""
    return text, b"".join(parts) + EOF_BLOCK


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=4096, help="decompressed MB (approximately)")
    ap.add_argument("--samples", type=int, default=0)
    ap.add_argument("--split", type=int, default=32 << 20)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-splits", type=int, default=16)
    ap.add_argument("--procs", type=int, default=min(16, os.cpu_count() or 1))
    a = ap.parse_args()
    import torch  # noqa: F401 -- one HIP runtime
    from disq_amd import _lib
    from oracle import oracle as O

    t0 = time.time()
    text, data = make_vcf(a.mb, a.samples, a.procs)
    gen_s = time.time() - t0
    with _lib.Context(split_size=a.split, verify_crc=True) as c:
        c.text_open_bytes(data)
        c.text_run(True)  # warm-up: buffers grow to size
        ms = []
        for _ in range(a.steps):
            w0 = time.perf_counter()
            st = c.text_run(True)
            ms.append((st.ms_total, (time.perf_counter() - w0) * 1e3))
        b = c.text_read(True)
    dev = sorted(m[0] for m in ms)[len(ms) // 2]
    wall = sorted(m[1] for m in ms)[len(ms) // 2]
    ubytes = st.decompressed_bytes
    # parity: every partition's line offsets / lengths against the oracle (one split per thread)
    splits = O.path_splits(len(data), a.split)
    po = b["part_offset"]

    import queue
    handles = queue.Queue()  # one oracle handle per worker (a handle holds inflate state); opened
    for _ in range(a.procs):  # before the timed sample
        handles.put(O.OracleText(data))

    def oracle_split(se):
        ot = handles.get()
        try:
            return ot.split_lines(se[0], se[1], True)
        finally:
            handles.put(ot)

    with ThreadPoolExecutor(a.procs) as ex:
        t1 = time.perf_counter()
        sample = list(ex.map(oracle_split, splits[:a.cpu_splits]))
        cpu_s = time.perf_counter() - t1
        rest = list(ex.map(oracle_split, splits[a.cpu_splits:]))
    parts = sample + rest
    bad = 0
    for i, (vs, vl) in enumerate(parts):
        lo, hi = int(po[i]), int(po[i + 1])
        if hi - lo != len(vs) or not (np.array_equal(b["line_offset"][lo:hi], vs) and
                                      np.array_equal(b["line_len"][lo:hi], vl)):
            bad += 1
    sample_bytes = sum(int(vl.sum()) + len(vl) for vs, vl in sample)  # values + terminators
    out = {
        "metric": "decompressed VCF GB/s (BGZF text read path, row f4)",
        "value": round(ubytes / (dev / 1e3) / 1e9, 3), "unit": "GB/s",
        "device_ms": round(dev, 3), "wall_ms": round(wall, 3), "steps": a.steps,
        "lines": int(st.n_records), "lines_per_s": round(st.n_records / (dev / 1e3), 1),
        "config": {"samples": a.samples, "decompressed_gb": round(ubytes / 1e9, 4),
                   "compressed_gb": round(len(data) / 1e9, 4), "ratio": round(ubytes / len(data), 3),
                   "split_size": a.split, "partitions": len(splits), "mean_line_bytes":
                   round(ubytes / max(int(st.n_records), 1), 1), "generator_s": round(gen_s, 1),
                   "data": "synthetic VCF (seeded), zlib level 5 BGZF, htsjdk block size"},
        "cpu_baseline": {"value": round(sample_bytes / cpu_s / 1e9, 4), "unit": "GB/s",
                         "threads": a.procs, "kind": "port",
                         "sample": "first %d of %d splits, one split per thread: the oracle's "
                                   "BGZFCodec + LineRecordReader restatement (zlib inflate + line "
                                   "splitting); %.2f s" % (min(a.cpu_splits, len(splits)), len(splits), cpu_s)},
        "parity": {"status": "match" if bad == 0 else "MISMATCH", "partitions": len(parts),
                   "bad_partitions": bad,
                   "checked": "per-partition line offsets and lengths, GPU vs the oracle's split reader"},
    }
    print(json.dumps(out), flush=True)
    if bad:
        sys.exit(3)


if __name__ == "__main__":
    main()
