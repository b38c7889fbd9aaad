"""CPU checks of the .bai span restatement (oracle.bai_span, htsjdk 2.16.0 getFileSpan +
removeContentsBefore/After as Disq calls them, AbstractBinarySamSource.java:102-107): reading only
the clipped spans selects exactly the records that reading every partition chunk whole selects.
htsjdk is not vendored, so the span algorithm's parity with htsjdk itself is unpinned; these
tests pin that the spans lose no overlapping record on files whose .bai the generator wrote."""
import numpy as np
import pytest

from disq_amd import synth
from oracle import oracle as O


@pytest.mark.parametrize("ivs", [[(20, 5000, 9999), (20, 20000, 22999)], [(20, 1, 1000135)],
                                 [(20, 1, 0)], [(3, 5, 10)], [(20, 500000, 500000)]])
@pytest.mark.parametrize("split", [40000, 3000])
def test_anysam_spans_equal_whole_chunks(ivs, split):
    a = synth.generate(1000, shape=synth.ANYSAM, bai=True)
    ob = O.OracleBam(a.bam)
    x = ob.read_partitions(split, traversal=(ivs, False), bai=a.bai)
    y = ob.read_partitions(split, traversal=(ivs, False), bai=a.bai, spans=True)
    assert len(x) == len(y)
    assert all(np.array_equal(p["hash"], q["hash"]) for p, q in zip(x, y))


def test_wgs_spans_equal_whole_chunks():
    w = synth.generate(20000, seed=4, bai=True, unplaced_fraction=0.01, nthreads=4)
    ob = O.OracleBam(w.bam)
    rng = np.random.default_rng(1)
    ivs = [(0, int(s), int(s + rng.integers(10, 800))) for s in rng.integers(1, 99000, size=60)]
    x = ob.read_partitions(1 << 20, traversal=(ivs, False), bai=w.bai)
    y = ob.read_partitions(1 << 20, traversal=(ivs, False), bai=w.bai, spans=True)
    assert sum(len(p) for p in x) > 0
    assert all(np.array_equal(p["hash"], q["hash"]) for p, q in zip(x, y))


def test_span_is_clipped_to_the_chunk():
    a = synth.generate(1000, shape=synth.ANYSAM, bai=True)
    ob = O.OracleBam(a.bam)
    q = O.optimize_intervals([(20, 1, 0)])
    full = O.bai_span(a.bai, q, 0, (1 << 64) - 1)
    assert full and all(b < e for b, e in full)
    (s, e, ch), = [p for p in ob.plan(0)]
    vs, ve = ch
    mid = (full[0][0] + full[-1][1]) // 2
    left = O.bai_span(a.bai, q, vs, mid)
    right = O.bai_span(a.bai, q, mid, ve)
    assert all(vs <= b and e <= mid for b, e in left)
    assert all(mid <= b and e <= ve for b, e in right)


def _py_parts(ob, split, ivs, bai, unplaced, spans):
    parts = iter(ob.read_partitions(split, traversal=(ivs, unplaced), bai=bai, spans=spans))
    cnt, dig = [], []
    for _, _, ch in ob.plan(split):
        if ch is None:
            cnt.append(0)
            dig.append(0)
            continue
        p = next(parts)
        cnt.append(len(p))
        dig.append(O.stream_digest(p["hash"]))
    return np.array(cnt), np.array(dig, np.uint64)


@pytest.mark.parametrize("unplaced", [False, True])
@pytest.mark.parametrize("spans", [True, False])
def test_c_traversal_equals_the_restatement(unplaced, spans):
    """oracle.run_partitions_traversal (C, threaded, binary-search overlap test: the bench-scale
    interval-mode oracle) = read_partitions + stream_digest (the restatement the GPU tests use),
    with and without the unplaced-unmapped tail (AbstractBinarySamSource.java:116-129)."""
    w = synth.generate(20000, seed=4, bai=True, unplaced_fraction=0.01, nthreads=4)
    ob = O.OracleBam(w.bam)
    rng = np.random.default_rng(2)
    ivs = [(0, int(s), int(s + rng.integers(10, 3000))) for s in rng.integers(1, 99000, size=80)]
    ivs += [(1, 1, 0), (5, 100, 200)]  # an open-ended interval; a contig with no reads
    split = 256 * 1024
    splits = O.path_splits(len(w.bam), split)
    cnt, dig = O.run_partitions_traversal(w.bam, splits, 4, w.bai, ivs, unplaced, spans)
    pcnt, pdig = _py_parts(ob, split, ivs, w.bai, unplaced, spans)
    assert cnt.sum() > 0 and len(cnt) > 3
    assert np.array_equal(cnt, pcnt)
    assert np.array_equal(dig, pdig)
    if unplaced:
        c0, _ = O.run_partitions_traversal(w.bam, splits, 4, w.bai, ivs, False, spans)
        assert cnt.sum() > c0.sum()  # the tail is there
