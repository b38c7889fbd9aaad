"""Out-of-core streaming read (disq_amd/stream.py): windows of whole partitions decoded as shards
by several contexts at once equal the whole-file run (per-partition counts and digests, whole-file
digest), for window sizes that cut the file in many places."""
import numpy as np
import pytest

from disq_amd import _lib, stream, synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("window,depth,ramp", [(3 << 20, 2, False), (5 << 20, 3, False),
                                              (1 << 40, 1, False), (4 << 20, 3, True)])
def test_stream_equals_whole_file(window, depth, ramp):
    r = synth.generate(150000, seed=31, nthreads=8)
    data = r.bam
    with _lib.Context(split_size=1 << 20, verify_crc=True) as c:
        c.open_bytes(data)
        st = c.run_resident()
        cnt, dig = c.partition_digests()
        header = c.header()[1]
    out = stream.stream_read(lambda a, b: data[a:b], len(data), header, window=window, depth=depth,
                             split_size=1 << 20, halo=64 << 10, ramp=ramp)
    if ramp:  # quarter, half, whole ..., half, quarter windows
        assert out["windows"] >= 5
    assert np.array_equal(out["counts"], cnt)
    assert np.array_equal(out["digests"], dig)
    assert out["digest"] == st.digest and out["n_records"] == st.n_records == 150000
    assert out["owned_bytes"] == st.decompressed_bytes


def test_stream_long_reads_grow_halo():
    r = synth.generate(300, seed=5, shape=synth.LONGREAD, records_per_chunk=40, nthreads=8)
    data = r.bam
    with _lib.Context(split_size=256 << 10, verify_crc=True) as c:
        c.open_bytes(data)
        st = c.run_resident()
        header = c.header()[1]
    out = stream.stream_read(lambda a, b: data[a:b], len(data), header, window=1 << 20, depth=2,
                             split_size=256 << 10, halo=4096)
    assert out["digest"] == st.digest and out["n_records"] == st.n_records


def test_stream_from_path(tmp_path):
    r = synth.generate(60000, seed=37, nthreads=8)
    p = str(tmp_path / "s.bam")
    r.write(p)
    with _lib.Context(split_size=1 << 20, verify_crc=True) as c:
        c.open_path(p)
        st = c.run_resident()
    out = stream.stream_read_path(p, window=2 << 20, depth=2, split_size=1 << 20, halo=32 << 10)
    assert out["digest"] == st.digest and out["n_records"] == 60000
