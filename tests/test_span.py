""".bai span traversal (AbstractBinarySamSource.java:86-112; BAMFileReader2.getFileSpan :1004-1019):
only the BGZF blocks of the intervals' index span, clipped to each partition chunk, are
inflated (dq_run_resident with intervals and a .bai).

Bar: per partition, the kept record count and the ordered digest of the kept records' raw-byte
hashes equal the oracle's Disq traversal (oracle.read_partitions with spans=True, which reads the
same spans; the CPU tests show it equals reading whole chunks), and equal the GPU's whole-file
filter (full_traversal).  The span computation itself restates htsjdk 2.16.0 (not vendored):
parity with htsjdk is unpinned; the record results are pinned by the overlap semantics.
"""
import numpy as np
import pytest

from disq_amd import _lib, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def intervals(n, lo, hi, ref=0, seed=3, min_len=20, max_len=5000):
    rng = np.random.default_rng(seed)
    ln = np.exp(rng.uniform(np.log(min_len), np.log(max_len), size=n)).astype(np.int64)
    st = rng.integers(lo, max(lo + 1, hi - 1), size=n)
    return [(ref, int(s), int(min(hi, s + l - 1))) for s, l in zip(st, ln)]


def gpu_span(data, bai, split, ivs, full=False, unplaced=False):
    with _lib.Context(split_size=split, verify_crc=True, full_traversal=full) as c:
        c.open_bytes(data)
        c.set_index(bai)
        st = c.run_resident((ivs, unplaced))
        cnt, dig = c.partition_digests()
    return st, cnt, dig


def oracle_parts(ob, split, ivs, bai):
    plan = ob.plan(split)
    parts = iter(ob.read_partitions(split, traversal=(ivs, False), bai=bai, spans=True))
    cnt, dig = [], []
    for _, _, ch in plan:
        if ch is None:
            cnt.append(0)
            dig.append(0)
            continue
        p = next(parts)
        cnt.append(len(p))
        dig.append(O.stream_digest(p["hash"]))
    return np.array(cnt), np.array(dig, np.uint64)


@pytest.mark.parametrize("split", [40000, 8000, 3000])
def test_anysam_spans(split):
    a = synth.generate(1000, shape=synth.ANYSAM, bai=True)
    ob = O.OracleBam(a.bam)
    for ivs in ([(20, 5000, 9999), (20, 20000, 22999)], [(20, 1, 1000135)], [(20, 1, 0)],
                [(20, 300000, 300500), (20, 700000, 900000), (3, 1, 100)]):
        st, cnt, dig = gpu_span(a.bam, a.bai, split, ivs)
        ocnt, odig = oracle_parts(ob, split, ivs, a.bai)
        assert np.array_equal(cnt, ocnt), ivs
        assert np.array_equal(dig, odig), ivs
        assert st.n_filtered == int(ocnt.sum())


@pytest.mark.parametrize("split,n_iv", [(1 << 20, 1000), (3 << 20, 3000)])
def test_wgs_spans_many_intervals(split, n_iv):
    """configs[3] shape: WGS-like file + .bai, thousands of intervals (sorted, overlapping ones
    merged by optimizeIntervals), several partitions; few blocks are inflated."""
    w = synth.generate(100000, seed=23, bai=True, nthreads=8, unplaced_fraction=0.005)
    ob = O.OracleBam(w.bam)
    ivs = intervals(n_iv, 1, 480000, seed=n_iv, max_len=400)
    st, cnt, dig = gpu_span(w.bam, w.bai, split, ivs)
    ocnt, odig = oracle_parts(ob, split, ivs, w.bai)
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(dig, odig)
    fst, fcnt, _ = gpu_span(w.bam, w.bai, split, ivs, full=True)
    assert fst.n_filtered == st.n_filtered == int(ocnt.sum())
    assert st.blocks_inflated < st.n_blocks


def test_long_read_spans_grow_windows():
    """Records spanning many blocks: a window's last record runs past its first extra blocks."""
    w = synth.generate(300, seed=5, shape=synth.LONGREAD, bai=True, records_per_chunk=40, nthreads=8)
    ob = O.OracleBam(w.bam)
    ivs = intervals(20, 1, 8_000_000, seed=9, min_len=100, max_len=20000)
    st, cnt, dig = gpu_span(w.bam, w.bai, 256 * 1024, ivs)
    ocnt, odig = oracle_parts(ob, 256 * 1024, ivs, w.bai)
    assert np.array_equal(cnt, ocnt) and np.array_equal(dig, odig)


@pytest.mark.parametrize("split", [1 << 20, 256 * 1024])
def test_wgs_spans_with_unplaced_tail(split):
    """traverseUnplacedUnmapped in a span run: the partition holding the start of the last linear
    bin appends the unplaced-unmapped tail after its interval records
    (AbstractBinarySamSource.java:116-129); every partition = the oracle's traversal."""
    w = synth.generate(60000, seed=29, bai=True, nthreads=8, unplaced_fraction=0.02)
    ivs = intervals(400, 1, 290000, seed=7, max_len=600)
    st, cnt, dig = gpu_span(w.bam, w.bai, split, ivs, unplaced=True)
    ocnt, odig = O.run_partitions_traversal(w.bam, O.path_splits(len(w.bam), split), 4, w.bai,
                                            ivs, True)
    c0, _ = O.run_partitions_traversal(w.bam, O.path_splits(len(w.bam), split), 4, w.bai, ivs,
                                       False)
    assert ocnt.sum() > c0.sum() + 500  # the tail is there
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(dig, odig)
    assert st.n_filtered == int(ocnt.sum())
