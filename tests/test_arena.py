"""Export-arena batch lifetime: a batch exported into a context's pinned arena
(dq_set_export_arena) is a set of views of that memory, so the Python layer must never let the
library overwrite or free the arena while such views are alive."""
import gc

import numpy as np
import pytest

from disq_amd import _lib, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wgs():
    return synth.generate(20000, seed=41, nthreads=8).bam


def test_arena_batch_is_read_only_and_blocks_the_next_batch(wgs):
    with _lib.Context(split_size=1 << 20) as c:
        c.set_export_arena(64 << 20)
        c.open_bytes(wgs)
        b = c.read(with_raw=True)
        assert not b["voffset"].flags.writeable and not b["raw"].flags.writeable
        keep = {k: v.copy() for k, v in b.items() if v is not None}
        with pytest.raises(_lib.DqError, match="export arena"):
            c.read(with_raw=True)
        with pytest.raises(_lib.DqError, match="export arena"):
            c.set_export_arena(32 << 20)
        h = b["hash"]  # one view keeps the whole batch (and its arena) alive
        del b
        gc.collect()
        with pytest.raises(_lib.DqError):
            c.read(with_raw=True)
        assert np.array_equal(h, keep["hash"])
        del h
        gc.collect()
        b2 = c.read(with_raw=True)  # the arena is free again
        for k in ("voffset", "hash", "raw_offset", "part_digest"):
            assert np.array_equal(b2[k], keep[k]), k
        assert np.array_equal(b2["raw"], keep["raw"])


def test_arena_outlives_a_closed_context(wgs):
    c = _lib.Context(split_size=1 << 20)
    c.set_export_arena(64 << 20)
    c.open_bytes(wgs)
    b = c.read(with_raw=True)
    ref = {k: v.copy() for k, v in b.items() if v is not None}
    c.close()  # the arena is handed to the batch: its views stay valid
    del c
    gc.collect()
    for k, v in ref.items():
        assert np.array_equal(b[k], v), k
    del b
    gc.collect()  # the last view frees the batch, then the context and its arena


def test_c_abi_owns_the_arena(wgs):
    """The ownership rule lives in the C ABI itself (a JNI caller has no Python guard): with an
    arena batch alive, dq_read into the arena and dq_set_export_arena return DQ_EINVAL; after
    dq_batch_free the arena takes the next batch; dq_ctx_destroy with a live arena batch leaves the
    arena to it (its arrays stay readable) and dq_batch_free releases it."""
    import ctypes as C
    L = _lib.lib()
    c = _lib.Context(split_size=1 << 20)
    h = c._h
    assert L.dq_set_export_arena(h, 64 << 20) == 0
    buf = np.frombuffer(wgs, np.uint8)
    assert L.dq_open_memory(h, buf.ctypes.data, len(buf)) == 0
    b1 = C.POINTER(_lib.DqBatch)()
    assert L.dq_read(h, None, 1, C.byref(b1)) == 0
    assert b1.contents.in_arena == 1
    n = b1.contents.n_records
    first = np.ctypeslib.as_array(b1.contents.hash, shape=(n,)).copy()
    b2 = C.POINTER(_lib.DqBatch)()
    assert L.dq_read(h, None, 1, C.byref(b2)) == _lib.DQ_EINVAL
    assert b"export arena" in L.dq_last_error(h)
    assert L.dq_set_export_arena(h, 32 << 20) == _lib.DQ_EINVAL
    L.dq_batch_free(b1)
    assert L.dq_read(h, None, 1, C.byref(b2)) == 0  # the arena is free again
    assert np.array_equal(np.ctypeslib.as_array(b2.contents.hash, shape=(n,)), first)
    # destroy the context while b2 lives: its arrays stay valid until dq_batch_free
    c._h = None
    L.dq_ctx_destroy(h)
    assert np.array_equal(np.ctypeslib.as_array(b2.contents.hash, shape=(n,)), first)
    L.dq_batch_free(b2)
